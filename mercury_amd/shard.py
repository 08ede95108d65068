"""Sharding of packet batches across the GPUs of one node.

Packets are independent (reassembly off), so a batch splits into contiguous
shards, one per rank, with no data-path collective: rank r fingerprints and
classifies packets [lo_r, hi_r) on its own GPU and the shards concatenate in
rank order (packet order is preserved).  torch.distributed is used only for
control: the barrier and the max-over-ranks time of bench.py, and -- for
host pipelines that want one output stream -- gathering the per-shard records
to one rank.

The one cross-packet dependency is the classifier's unknown-TLS prevalence
LRU (fingerprint_prevalence, analysis.h:362-421): a sighting's status depends
on every earlier sighting of the stream.  ordered_prevalence_merge is the
host-side ordered merge of SURVEY 8(e): every rank analyses its shard with the
decision deferred, the ranks exchange their batch's distinct unknown-TLS
fingerprints (a few hundred entries, fixed-size gloo all_gathers), and every rank applies
the same decisions, in shard order, to an identical copy of the LRU -- so the
sharded output equals one context over the concatenated stream.  When the
distinct form cannot be exact (more new fingerprints than the LRU holds), each
rank decides its own sightings from the set the earlier shards leave, known
from their summaries (at most the LRU's capacity each): every sighting is
decided once, by its own rank.
"""
import numpy as np

from .api import DESC_DTYPE, RECORD_DTYPE, SIGHTING_DTYPE


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


def _all_gather_rows(arr, group=None):
    """all_gather of one 1-D numpy array of fixed-size records per rank (any
    length), as fixed-size int64 tensors: the lengths first, then the rows
    padded to the longest.  Returns the ranks' arrays in rank order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    raw = np.ascontiguousarray(arr).view(np.uint8)
    words = (raw.nbytes + 7) // 8
    n = torch.tensor([words], dtype=torch.int64)
    ns = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    cap = max(1, max(int(x.item()) for x in ns))
    buf = np.zeros(cap * 8, np.uint8)
    buf[:raw.nbytes] = raw
    t = torch.from_numpy(buf.view(np.int64))
    outs = [torch.zeros(cap, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    return [o.numpy().view(np.uint8)[:int(k.item()) * 8].view(arr.dtype) for o, k in zip(outs, ns)]


last_merge_phases = {}   # seconds per phase of the last ordered_prevalence_merge (bench.py reports them)


def ordered_prevalence_merge(ctx, prev, shard_base, group=None):
    """Decide the unknown-TLS sightings of this rank's last analysed batch
    (ctx deferred, see Context.defer) in stream order across the ranks of
    `group`: rank order is stream order, `shard_base` is the stream position of
    this rank's first packet.  `prev` is this rank's copy of the LRU (every
    rank applies the same decisions to its own copy).  The exchange is two or
    three fixed-size int64 all_gathers (no pickling).  Returns the number of
    distinct fingerprints exchanged (or sightings, on the sequence path)."""
    import time
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    ph = last_merge_phases
    ph.clear()
    t0 = time.perf_counter()

    def lap(name):
        nonlocal t0
        t = time.perf_counter()
        ph[name] = ph.get(name, 0.0) + (t - t0)
        t0 = t
    nd = ctx.analysis_distinct_count()
    lap("distinct_count")
    # [distinct count or -1 (table overflow), this shard's stream base]
    hdr = torch.tensor([-1 if nd is None else nd, int(shard_base)], dtype=torch.int64)
    hdrs = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(hdrs, hdr, group=group)
    lap("header_gather")
    # the distinct form is exact only when no eviction can happen inside the
    # step; with more distinct fingerprints in the step than the LRU holds it
    # cannot be (every rank sees the same counts, so all take the same path)
    if all(int(h[0]) >= 0 for h in hdrs) and sum(int(h[0]) for h in hdrs) <= prev.capacity:
        dl = ctx.analysis_distinct()
        lap("distinct_export")
        lists = _all_gather_rows(dl if dl is not None else np.zeros(0, SIGHTING_DTYPE), group)
        for x, h in zip(lists, hdrs):
            x["first"] += np.uint64(int(h[1]))
            x["last"] += np.uint64(int(h[1]))
        allv = np.concatenate(lists) if lists else np.zeros(0, SIGHTING_DTYPE)
        lap("distinct_gather")
        if prev.resolve_distinct(allv):
            k = sum(len(x) for x in lists[:rank])
            ctx.analysis_resolve(allv[k:k + len(lists[rank])])
            lap("distinct_resolve")
            return len(allv)
        lap("distinct_resolve")
    # the sequence form, decided once: each rank decides its own sightings,
    # from the set that the earlier shards leave; a shard's effect on any later
    # one is its summary -- its distinct fingerprints by last sighting, at most
    # the LRU's capacity (what lru_at's walk back takes from it) -- so the ranks
    # exchange summaries, not sightings, and the work per rank does not grow
    # with the number of ranks
    seq = np.ascontiguousarray(ctx.analysis_sequence(), np.uint64)
    lap("sequence_export")
    mine = prev.summary(seq)
    lap("summary")
    summaries = _all_gather_rows(mine, group)
    lap("summary_gather")
    prior = np.concatenate(summaries[:rank][::-1]) if rank else np.zeros(0, np.uint64)
    seen = prev.resolve_shard(seq, prior)
    lap("resolve_shard")
    ctx.analysis_resolve_sequence(seen)
    lap("apply")
    prev.advance(np.concatenate(summaries[::-1]))
    lap("advance")
    return sum(len(x) for x in summaries)
