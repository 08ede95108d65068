"""Multi-GPU sharding logic (mercury_amd/shard.py) on the CPU: contiguous
shards, rebased host batches, and the world_size-2 gather / max-over-ranks
path over gloo.  Each rank fingerprints its shard with the C oracle (test
infrastructure standing in for the GPU) and rank 0 checks that the merged
shards equal the whole batch."""
import os
import socket

import numpy as np
import pytest

from mercury_amd import shard
from mercury_amd.api import RECORD_DTYPE
from oracle import oracle
from tests import synth


def test_shard_bounds_cover_exactly():
    for n in (0, 1, 7, 64, 1000, 1001):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_bounds(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.shard_bounds(10, 2, 2)


def oracle_records(arena, desc):
    """Records + fp arena of a host batch from the C oracle (test stand-in for the GPU)."""
    ft, fl, flags, strs = oracle.process_batch(arena, desc, oracle.config())
    rec = np.zeros(len(desc), RECORD_DTYPE)
    blob, off = [], 0
    for i, s in enumerate(strs):
        b = s.encode("latin-1")
        rec["fp_offset"][i] = off
        rec["fp_len"][i] = len(b)
        rec["fp_type"][i] = ft[i]
        rec["flags"][i] = flags[i]
        blob.append(b)
        off += len(b)
    return rec, b"".join(blob)


def test_shard_batch_rebased_equals_whole():
    arena, desc = synth.batch(3000, seed=0x5EED0003, workload="mixed", n_templates=256)
    want = oracle.process_batch(arena, desc, oracle.config())[3]
    parts = []
    for r in range(3):
        a, d, lo = shard.shard_batch(arena, desc, r, 3)
        assert lo == shard.shard_bounds(len(desc), r, 3)[0]
        parts.append(oracle_records(a, d))
    rec, fp = shard.merge_shards(parts)
    got = [fp[int(o):int(o) + int(n)].decode("latin-1") for o, n in zip(rec["fp_offset"], rec["fp_len"])]
    assert got == want


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        arena, desc = synth.batch(2000, seed=0x5EED0003, workload="mixed", n_templates=256)
        a, d, _ = shard.shard_batch(arena, desc, rank, world)
        rec, fp = oracle_records(a, d)
        t = shard.max_over_ranks(0.5 + rank)
        merged = shard.gather_shards(rec, fp)
        if rank == 0:
            want = oracle.process_batch(arena, desc, oracle.config())[3]
            got = [merged[1][int(o):int(o) + int(n)].decode("latin-1")
                   for o, n in zip(merged[0]["fp_offset"], merged[0]["fp_len"])]
            q.put((got == want, t, len(merged[0])))
        else:
            q.put((merged is None, t, 0))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_gather_and_max():
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for ok, _, _ in res)
    assert all(t == 1.5 for _, t, _ in res)          # max over ranks
    assert max(n for _, _, n in res) == 2000


class _ShardCtx:
    """Stands in for a deferred analysis context (CPU): one shard's unknown-TLS
    sightings as keys; records the decisions it is given."""

    def __init__(self, keys):
        from tests.test_prevalence import distinct_of, key_hash
        self.keys = keys
        self.dl = distinct_of(keys)
        self.seq = key_hash(keys)
        self.seen = None

    def analysis_distinct(self):
        return None if self.dl is None else self.dl.copy()

    def analysis_distinct_count(self):
        return None if self.dl is None else len(self.dl)

    def analysis_sequence(self):
        return self.seq

    def analysis_resolve(self, d):
        self.seen = np.ones(len(self.keys), np.uint8)
        for e in d:
            self.seen[int(e["first"]) - self.base] = e["first_seen"]

    def analysis_resolve_sequence(self, seen):
        self.seen = np.asarray(seen, np.uint8)


def _merge_worker(rank, world, port, q, cap, span, seed):
    import torch.distributed as dist
    import mercury_amd
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GLOO_SOCKET_IFNAME="lo")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(seed)
    prev = mercury_amd.Prevalence(cap)
    out = []
    for step in range(6):
        shards = [rng.integers(0, span, 50).tolist() for _ in range(world)]
        c = _ShardCtx(shards[rank])
        c.base = step * 50 * world + rank * 50
        shard.ordered_prevalence_merge(c, prev, c.base)
        out.append(c.seen.tolist())
    q.put((rank, out, prev.keys().tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("cap,span", [(400, 150), (60, 150)])
def test_ordered_prevalence_merge_world2(cap, span):
    """Two gloo ranks, each with its own shard of one stream: the ordered merge
    gives every sighting the status of one LRU over the concatenated stream
    (distinct form when exact, else the sequence form: cap 60 < the distinct
    fingerprints in flight), and both ranks end with the same LRU."""
    import multiprocessing as mp
    from tests.test_prevalence import key_hash, lru_model
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ps = [ctxm.Process(target=_merge_worker, args=(r, 2, port, q, cap, span, 11)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (o, k)) for r, o, k in [q.get(timeout=120) for _ in ps])
    for p in ps:
        p.join(timeout=60)
    rng = np.random.default_rng(11)
    stream = []
    for step in range(6):
        shards = [rng.integers(0, span, 50).tolist() for _ in range(2)]
        stream += shards[0] + shards[1]
    want, order = lru_model(stream, cap)
    got = []
    for step in range(6):
        got += res[0][0][step] + res[1][0][step]
    assert np.array_equal(np.array(got, np.uint8), want)
    assert res[0][1] == res[1][1] == key_hash(order).tolist()


def _gpu_merge_worker(rank, world, port, q):
    """One rank of bench.py's multi-GPU step, on cuda:0 (the one-GPU box): a
    deferred --analysis context over its shard of the LRU stream, then
    shard.ordered_prevalence_merge -- the function bench.py calls."""
    import torch.distributed as dist
    import mercury_amd
    from tests.test_prevalence import REF_ARCHIVE
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GLOO_SOCKET_IFNAME="lo")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, d = synth.lru_batch(synth.lru_keys())
        ctx = mercury_amd.Context(f"select=tls;resources={REF_ARCHIVE};analysis", device=0)
        prev = mercury_amd.Prevalence(100000)
        ctx.set_prevalence(prev)
        ctx.defer(True)
        step = 17000                      # 170 000 packets: 5 rounds of 2 shards
        got, exchanged = [], 0
        for lo in range(0, len(d), world * step):
            s_lo = lo + rank * step
            ctx.process_host_analysis(a, d[s_lo:s_lo + step])
            exchanged += shard.ordered_prevalence_merge(ctx, prev, s_lo)
            got.append(ctx.last_analysis()["status"].astype(np.uint8))
        q.put((rank, np.concatenate(got).tobytes(), prev.keys().tobytes(), exchanged))
        ctx.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_ordered_prevalence_merge_world2_hip():
    """bench.py's multi-rank step on the HIP path: two gloo ranks, each a
    process with its own deferred context on cuda:0, analyse alternate 17 000-
    packet shards of the 170 000-sighting LRU stream and decide them with
    shard.ordered_prevalence_merge; the statuses, in stream order, equal the
    reference's (tests/golden/lru_status.bin.gz), and both ranks end with the
    same LRU."""
    import multiprocessing as mp
    from tests.test_prevalence import golden_status
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ps = [ctxm.Process(target=_gpu_merge_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {r: (np.frombuffer(s, np.uint8), k, e) for r, s, k, e in [q.get(timeout=600) for _ in ps]}
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    step = 17000
    got = np.concatenate([res[r][0][k * step:(k + 1) * step] for k in range(5) for r in range(2)])
    want = golden_status()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} statuses differ, first at {bad[:5]}"
    assert res[0][1] == res[1][1] and res[0][2] > 0


def _gpu_pipe_worker(rank, world, port, q):
    """bench.py's pipelined multi-rank step on cuda:0: each step's kernels are
    launched (process_device + analyze_device_deferred_pipelined), then the
    previous step's sightings are decided across the ranks
    (shard.ordered_prevalence_merge) while the device runs this one."""
    import torch
    import torch.distributed as dist
    import mercury_amd
    from tests.test_prevalence import REF_ARCHIVE
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GLOO_SOCKET_IFNAME="lo")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, d = synth.lru_batch(synth.lru_keys())
        ctx = mercury_amd.Context(f"select=tls;resources={REF_ARCHIVE};analysis", device=0)
        prev = mercury_amd.Prevalence(100000)
        ctx.set_prevalence(prev)
        ctx.defer(True)
        step, cap = 17000, 48 * 1024 * 1024
        stream = torch.cuda.current_stream()
        d_arena = torch.from_numpy(np.ascontiguousarray(a)).cuda()
        sets = [dict(rec=torch.empty(step * 32, dtype=torch.uint8, device="cuda"),
                     fp=torch.empty(cap, dtype=torch.uint8, device="cuda"),
                     used=torch.zeros(4, dtype=torch.int64, device="cuda"),
                     an=torch.empty(step * mercury_amd.ANALYSIS_DTYPE.itemsize, dtype=torch.uint8, device="cuda"))
                for _ in range(2)]
        bases = list(range(0, len(d), world * step))
        got, descs = [], [None, None]

        def decide(k):
            shard.ordered_prevalence_merge(ctx, prev, bases[k] + rank * step)
            got.append(ctx.last_analysis()["status"].astype(np.uint8))

        for k, lo in enumerate(bases):
            s_lo = lo + rank * step
            dd = np.ascontiguousarray(d[s_lo:s_lo + step])
            b = sets[k % 2]
            descs[k % 2] = torch.from_numpy(dd.view(np.uint8)).cuda()
            ctx.process_device(d_arena.data_ptr(), descs[k % 2].data_ptr(), len(dd), b["rec"].data_ptr(),
                               b["fp"].data_ptr(), cap, b["used"].data_ptr(), stream.cuda_stream)
            ctx.analyze_device_deferred_pipelined(d_arena.data_ptr(), descs[k % 2].data_ptr(), len(dd),
                                                  b["rec"].data_ptr(), b["fp"].data_ptr(), b["an"].data_ptr(),
                                                  stream.cuda_stream)
            if k:
                decide(k - 1)     # step k-1's merge, with step k's kernels in flight
        ctx.analysis_defer_newest()
        decide(len(bases) - 1)
        torch.cuda.synchronize()
        q.put((rank, np.concatenate(got).tobytes(), prev.keys().tobytes()))
        ctx.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_ordered_prevalence_merge_pipelined_world2_hip():
    """The pipelined multi-rank step (bench.py --gpus N): two gloo ranks on
    cuda:0, step k's kernels launched before step k-1's ordered merge; the
    statuses, in stream order, equal the reference's
    (tests/golden/lru_status.bin.gz), and both ranks end with the same LRU."""
    import multiprocessing as mp
    from tests.test_prevalence import golden_status
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ps = [ctxm.Process(target=_gpu_pipe_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {r: (np.frombuffer(s, np.uint8), k) for r, s, k in [q.get(timeout=600) for _ in ps]}
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    step = 17000
    got = np.concatenate([res[r][0][k * step:(k + 1) * step] for k in range(5) for r in range(2)])
    want = golden_status()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} statuses differ, first at {bad[:5]}"
    assert res[0][1] == res[1][1]


def _scale_worker(rank, world, port, q, m, steps, threads=2):
    """One rank at the realistic-diversity leg's scale: m unknown-TLS sightings
    per step (mostly distinct fingerprints, cycling the 100 000-entry LRU),
    decided with shard.ordered_prevalence_merge; reports the merge's wall time
    per step.  `threads` LRU threads per rank (MFP_LRU_THREADS): world x
    threads stays within the host's cores."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GLOO_SOCKET_IFNAME="lo",
                      MFP_LRU_THREADS=str(threads))
    import time
    import torch.distributed as dist
    import mercury_amd
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        prev = mercury_amd.Prevalence(100000)
        ts, checks = [], []
        for step in range(steps):
            rng = np.random.default_rng(1000 * step + rank)
            # 2 % of the sightings repeat a small hot set, the rest are ~350 k
            # fingerprints per shard seen about 50 times each
            keys = rng.integers(0, 350_000, m, dtype=np.int64) + (rank + world * step) * 1_000_000
            hot = rng.random(m) < 0.02
            keys[hot] = rng.integers(0, 64, int(hot.sum()))
            c = _ShardCtx.__new__(_ShardCtx)
            c.seq = (keys.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)) ^ np.uint64(0x5EED)
            c.dl, c.seen = None, None
            # (dl None: the table overflowed: the sequence form)
            dist.barrier()
            t0 = time.perf_counter()
            shard.ordered_prevalence_merge(c, prev, rank * m)
            ts.append(time.perf_counter() - t0)
            checks.append(int(c.seen.sum()))
        q.put((rank, ts, checks, prev.keys()[-8:].tolist()))
    finally:
        dist.destroy_process_group()


def _run_scale(world, m, steps, threads=2):
    import multiprocessing as mp
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ps = [ctxm.Process(target=_scale_worker, args=(r, world, port, q, m, steps, threads)) for r in range(world)]
    for p in ps:
        p.start()
    res = {r: (t, c, k) for r, t, c, k in [q.get(timeout=600) for _ in ps]}
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def test_ordered_prevalence_merge_scale_world2_4_8():
    """SURVEY 8(e) at the diversity leg's scale: 17.5 M sightings per rank per
    step, world 2, 4 and 8 (one LRU thread per rank: 8 ranks fill this host's
    8 cores).  The sequence form decides every sighting once, on its own rank,
    so the merge's time per step does not grow with the number of ranks (the
    earlier form resolved all ranks' sightings on every rank: 8x the work at
    world 8).  Every rank ends each step with the same LRU.  The per-rank time
    at the GPU box's thread share: tools/merge_scale.py (profiles/)."""
    m, steps = 17_500_000, 2
    t = {}
    for world in (2, 4, 8):
        res = _run_scale(world, m, steps, threads=1)
        assert len({tuple(v[2]) for v in res.values()}) == 1      # same LRU on every rank
        t[world] = max(max(v[0][1:]) for v in res.values())      # steady state (the first step warms up)
    print("merge per step (1 LRU thread per rank): " + ", ".join(f"world {w} {x:.2f} s" for w, x in t.items()))
    assert t[4] < 1.6 * t[2] and t[8] < 1.8 * t[2], t
