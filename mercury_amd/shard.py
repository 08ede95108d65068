"""Sharding of packet batches across the GPUs of one node.

Packets are independent (reassembly off), so a batch splits into contiguous
shards, one per rank, with no data-path collective: rank r fingerprints and
classifies packets [lo_r, hi_r) on its own GPU and the shards concatenate in
rank order (packet order is preserved).  torch.distributed is used only for
control: the barrier and the max-over-ranks time of bench.py, and -- for
host pipelines that want one output stream -- gathering the per-shard records
to one rank.  The one cross-packet dependency, the classifier's unknown-TLS
prevalence set, is per context (per GPU); the reference itself is not
deterministic across threads there (analysis.h:390-394).
"""
import numpy as np

from .api import DESC_DTYPE, RECORD_DTYPE


def shard_bounds(n, rank, world):
    """Contiguous shard [lo, hi) of n packets for `rank` of `world` (sizes differ by at most one)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def shard_batch(arena, desc, rank, world):
    """The rank's packets as a compact host batch: (arena bytes, descriptors
    with offsets rebased into that arena, global index of its first packet).
    The arena keeps 16 bytes of slack after the last packet (the kernels read
    aligned 16-byte blocks, include/mfp.h)."""
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    lo, hi = shard_bounds(len(desc), rank, world)
    d = desc[lo:hi].copy()
    if len(d) == 0:
        return np.zeros(16, np.uint8), d, lo
    start = int(d["offset"].min())
    end = int((d["offset"] + d["caplen"].astype(np.uint64)).max())
    a = np.zeros(end - start + 16, np.uint8)
    a[:end - start] = arena[start:end]
    d["offset"] -= np.uint64(start)
    return a, d, lo


def merge_shards(parts):
    """[(records, fp arena bytes), ...] in rank order -> (records, fp arena bytes)
    of the whole batch, fingerprint offsets rebased into the concatenated arena."""
    recs, blobs, base = [], [], 0
    for rec, fp in parts:
        r = np.array(rec, dtype=RECORD_DTYPE, copy=True)
        r["fp_offset"] += np.uint64(base)
        recs.append(r)
        blobs.append(fp)
        base += len(fp)
    return (np.concatenate(recs) if recs else np.zeros(0, RECORD_DTYPE)), b"".join(blobs)


def gather_shards(rec, fp, group=None, dst=0):
    """Collect every rank's (records, fp arena) on rank `dst` (torch.distributed,
    any backend); returns the merged batch there and None elsewhere."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = [None] * world if dist.get_rank(group) == dst else None
    dist.gather_object((np.asarray(rec).tobytes(), bytes(fp)), out, dst=dst, group=group)
    if out is None:
        return None
    return merge_shards([(np.frombuffer(r, dtype=RECORD_DTYPE), f) for r, f in out])


def max_over_ranks(value, device=None, group=None):
    """The largest `value` (seconds) over all ranks -- bench.py's job time."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
