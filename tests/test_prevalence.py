"""The unknown-TLS prevalence LRU (fingerprint_prevalence, analysis.h:362-421;
capacity 100000, analysis.h:433), decided on the host by mfp_prevalence
(mercury_amd/csrc/mfp_prevalence.cpp).

CPU: the LRU model of this file reproduces the REFERENCE's statuses on a
170 000-packet stream that crosses the capacity (tests/golden/lru_status.bin.gz
from oracle/_ref/merc_ref_drv, tests/golden/make_golden_lru.py); the C++ LRU
equals the model on that stream and on random small-capacity streams; the
distinct form equals the sequence form whenever it claims to be exact.
GPU: the device path (batch host API, pipelined path, device API, and two
shard contexts resolved in order against one shared LRU) reproduces the
reference's statuses on the same stream."""
import gzip
import os
from collections import OrderedDict

import numpy as np
import pytest

import mercury_amd
from mercury_amd.api import SIGHTING_DTYPE
from tests import synth

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
REF_ARCHIVE = os.path.join(GOLD, "resources-test.tgz")


def lru_model(keys, capacity):
    """fingerprint_prevalence::contains + update in stream order (analysis.h:366-408)."""
    lru, out = OrderedDict(), []
    for k in keys:
        if k in lru:
            out.append(1)
            lru.move_to_end(k)
        else:
            out.append(0)
            lru[k] = True
            if len(lru) > capacity:
                lru.popitem(last=False)
    return np.array(out, np.uint8), list(lru)


def golden_status():
    return np.frombuffer(gzip.open(os.path.join(GOLD, "lru_status.bin.gz")).read(), np.uint8)


def key_hash(keys):
    k = np.asarray(keys, np.uint64)
    return (k * np.uint64(0x9E3779B97F4A7C15)) ^ np.uint64(0x5EED)


def test_lru_model_pins_to_reference():
    keys = synth.lru_keys()
    seen, _ = lru_model(keys.tolist(), 100000)
    st = golden_status()
    assert len(st) == len(keys)
    assert np.array_equal(np.where(seen == 1, 3, 2).astype(np.uint8), st)
    assert (st == 2).sum() > 100000 and (st == 3).sum() > 10000


def test_prevalence_sequence_equals_model_on_reference_stream():
    keys = synth.lru_keys()
    p = mercury_amd.Prevalence(100000)
    seen = p.resolve_sequence(key_hash(keys))
    want, order = lru_model(keys.tolist(), 100000)
    assert np.array_equal(seen, want)
    assert len(p) == 100000
    assert np.array_equal(p.keys(), key_hash(order))


@pytest.mark.parametrize("cap,n,span,seed", [(1, 50, 3, 1), (5, 400, 9, 2), (64, 5000, 90, 3), (64, 5000, 60, 4),
                                             (1000, 20000, 1500, 5)])
def test_prevalence_sequence_random(cap, n, span, seed):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, span, n)
    p = mercury_amd.Prevalence(cap)
    assert np.array_equal(p.resolve_sequence(key_hash(keys)), lru_model(keys.tolist(), cap)[0])


@pytest.mark.parametrize("kind", ["few", "near_cap", "wide", "cycle", "bursts"])
def test_prevalence_sequence_parallel_chunks(kind):
    """Sequences long enough (>= 2 x 8 x capacity) to be decided in parallel
    chunks, each starting from the set rebuilt from the sightings before it:
    the same decisions and the same recency order as the one-pass model,
    across calls (the set carried over)."""
    rng = np.random.default_rng(["few", "near_cap", "wide", "cycle", "bursts"].index(kind) + 11)
    cap = 200
    p = mercury_amd.Prevalence(cap)
    allkeys = []
    for call in range(3):
        n = 60000 + 777 * call
        if kind == "few":
            keys = rng.integers(0, 150, n)             # fewer distinct keys than the capacity
        elif kind == "near_cap":
            keys = rng.integers(0, 260, n)
        elif kind == "wide":
            keys = rng.integers(0, 5000, n)
        elif kind == "cycle":
            keys = np.tile(np.arange(300), n // 300 + 1)[:n] + 1000 * call
        else:   # bursts of a small working set, now and then a new one
            keys = (rng.integers(0, 120, n) + 50 * (np.arange(n) // 9000)).astype(np.int64)
        allkeys += keys.tolist()
        want, order = lru_model(allkeys, cap)
        got = p.resolve_sequence(key_hash(keys))
        assert np.array_equal(got, want[len(allkeys) - n:]), (kind, call)
        assert np.array_equal(p.keys(), key_hash(order)), (kind, call)


def distinct_of(keys, base=0):
    """The batch's distinct list as the device exports it (insertion order)."""
    d, first = [], {}
    for j, k in enumerate(keys):
        if k not in first:
            first[k] = len(d)
            d.append([k, base + j, base + j, 0])
        e = d[first[k]]
        e[2] = base + j
        e[3] += 1
    out = np.zeros(len(d), SIGHTING_DTYPE)
    for i, (k, f, l, c) in enumerate(d):
        out[i] = (key_hash([k])[0], f, l, c, 0)
    return out


@pytest.mark.parametrize("seed", range(6))
def test_prevalence_distinct_equals_sequence_when_exact(seed):
    """Batches whose new fingerprints fit: the distinct form (first_seen per
    fingerprint, later sightings unlabeled) equals the sequence form, and the
    set afterwards is the same; a batch that could evict is refused."""
    rng = np.random.default_rng(seed)
    cap = 50
    pa, pb = mercury_amd.Prevalence(cap), mercury_amd.Prevalence(cap)
    refused = 0
    for b in range(40):
        keys = rng.integers(0, 70, int(rng.integers(1, 30))).tolist()
        seen = pb.resolve_sequence(key_hash(keys))
        d = distinct_of(keys)
        if pa.resolve_distinct(d):
            got = np.ones(len(keys), np.uint8)
            for e in d:
                got[int(e["first"])] = e["first_seen"]
            assert np.array_equal(got, seen), b
        else:
            refused += 1
            pa.resolve_sequence(key_hash(keys))
        assert np.array_equal(pa.keys(), pb.keys()), b
    assert refused > 0


def test_prevalence_distinct_across_shards():
    """Entries of several shards decided together (shard base + index order)
    equal the sequence form over the concatenated stream."""
    rng = np.random.default_rng(9)
    cap = 200
    pa, pb = mercury_amd.Prevalence(cap), mercury_amd.Prevalence(cap)
    for step in range(10):
        shards = [rng.integers(0, 120, 40).tolist() for _ in range(3)]
        seen = pb.resolve_sequence(key_hash(sum(shards, [])))
        base, parts = 0, []
        for sh in shards:
            parts.append(distinct_of(sh, base))
            base += len(sh)
        d = np.concatenate(parts)
        assert pa.resolve_distinct(d)
        got = np.ones(base, np.uint8)
        for e in d:
            got[int(e["first"])] = e["first_seen"]
        assert np.array_equal(got, seen), step
        assert np.array_equal(pa.keys(), pb.keys())


# ---------------------------------------------------------------------------
# the device path against the reference's statuses
# ---------------------------------------------------------------------------
def _statuses(an):
    return an["status"].astype(np.uint8)


@pytest.mark.gpu
def test_lru_stream_batches_vs_reference():
    """mfp_process_batch_host_ex batch after batch: the sighting sequence
    crosses 100 000 distinct fingerprints; statuses equal the reference's."""
    a, d = synth.lru_batch(synth.lru_keys())
    want = golden_status()
    ctx = mercury_amd.Context(f"select=tls;resources={REF_ARCHIVE};analysis", device=0)
    got = []
    for lo in range(0, len(d), 40000):
        _, _, an = ctx.process_host_analysis(a, d[lo:lo + 40000])
        got.append(_statuses(an))
    got = np.concatenate(got)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} statuses differ, first at {bad[:5]}: {got[bad[:5]]} vs {want[bad[:5]]}"
    assert ctx.analysis_stats()[3] == 100000
    ctx.close()


@pytest.mark.gpu
def test_lru_stream_small_batches_vs_reference():
    """Batches of at most MFP_SMALL_BATCH packets (the per-packet API's size)
    decide their sightings on the host from the returned copies
    (mfp_host.cpp resolve_on_host): the first 24 000 packets of the LRU stream
    in 200-packet batches give the reference's statuses."""
    a, d = synth.lru_batch(synth.lru_keys())
    want = golden_status()[:24000]
    ctx = mercury_amd.Context(f"select=tls;resources={REF_ARCHIVE};analysis", device=0)
    got = []
    for lo in range(0, 24000, 200):
        _, _, an = ctx.process_host_analysis(a, d[lo:lo + 200])
        got.append(_statuses(an))
    ctx.close()
    got = np.concatenate(got)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} statuses differ, first at {bad[:5]}"


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [25000, 170000])
def test_lru_stream_pipelined_vs_reference(chunk):
    a, d = synth.lru_batch(synth.lru_keys())
    ctx = mercury_amd.Context(f"select=tls;resources={REF_ARCHIVE};analysis", device=0)
    _, _, an = ctx.process_pipelined(a, d, chunk=chunk, analysis=True)
    assert np.array_equal(_statuses(an), golden_status())
    ctx.close()


@pytest.mark.gpu
def test_lru_stream_device_pipelined_vs_reference():
    """mfp_analyze_batch_device_pipelined over device batches (two sets of
    output buffers, alternating): batch k's kernels run while batch k-1 is
    decided; after the flush every batch's statuses equal the reference's."""
    import torch
    a, d = synth.lru_batch(synth.lru_keys())
    want = golden_status()
    ctx = mercury_amd.Context(f"select=tls;resources={REF_ARCHIVE};analysis", device=0)
    d_arena = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    chunk = 30000
    cap = 64 * 1024 * 1024
    bufs = [dict(rec=torch.empty(chunk * 32, dtype=torch.uint8, device="cuda"),
                 fp=torch.empty(cap, dtype=torch.uint8, device="cuda"),
                 used=torch.zeros(4, dtype=torch.int64, device="cuda"),
                 an=torch.empty(chunk * mercury_amd.ANALYSIS_DTYPE.itemsize, dtype=torch.uint8, device="cuda"))
            for _ in range(2)]
    stream = torch.cuda.current_stream()
    got, descs = [None] * ((len(d) + chunk - 1) // chunk), []
    for k, lo in enumerate(range(0, len(d), chunk)):
        dd = np.ascontiguousarray(d[lo:lo + chunk])
        descs.append(torch.from_numpy(dd.view(np.uint8)).cuda())
        b = bufs[k % 2]
        if k >= 2:                                    # batch k-2 was decided by the previous call
            got[k - 2] = _statuses(bufs[k % 2]["an"].cpu().numpy().view(mercury_amd.ANALYSIS_DTYPE))
        b["used"].zero_()
        ctx.process_device(d_arena.data_ptr(), descs[k].data_ptr(), len(dd), b["rec"].data_ptr(), b["fp"].data_ptr(),
                           cap, b["used"].data_ptr(), stream.cuda_stream)
        ctx.analyze_device_pipelined(d_arena.data_ptr(), descs[k].data_ptr(), len(dd), b["rec"].data_ptr(),
                                     b["fp"].data_ptr(), b["an"].data_ptr(), stream.cuda_stream)
    ctx.analysis_flush()
    torch.cuda.synchronize()
    nb = len(got)
    for k in range(max(0, nb - 2), nb):
        m = min(chunk, len(d) - k * chunk)
        got[k] = _statuses(bufs[k % 2]["an"].cpu().numpy().view(mercury_amd.ANALYSIS_DTYPE)[:m])
    got = np.concatenate(got)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} statuses differ, first at {bad[:5]}"
    assert ctx.analysis_stats()[3] == 100000
    ctx.close()


@pytest.mark.gpu
def test_lru_stream_pipelined_mixed_with_sync_calls():
    """Synchronous analysis calls (host batches, a synchronous device batch)
    interleaved with pipelined device batches: each synchronous call first
    decides the pipelined batches still pending, so the LRU sees the stream in
    order and the statuses of all of them equal the reference's."""
    import torch
    a, d = synth.lru_batch(synth.lru_keys())
    want = golden_status()
    ctx = mercury_amd.Context(f"select=tls;resources={REF_ARCHIVE};analysis", device=0)
    d_arena = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    chunk = 20000
    cap = 48 * 1024 * 1024
    stream = torch.cuda.current_stream()
    got = np.full(len(d), 255, np.uint8)
    pending = []                                         # (lo, m, buffers) of pipelined batches
    for k, lo in enumerate(range(0, len(d), chunk)):
        dd = np.ascontiguousarray(d[lo:lo + chunk])
        m = len(dd)
        if k % 3 == 2:                                   # a synchronous host batch
            _, _, an = ctx.process_host_analysis(a, dd)
            got[lo:lo + m] = _statuses(an)
        elif k % 6 == 4:                                 # a synchronous device batch
            b = dict(desc=torch.from_numpy(dd.view(np.uint8)).cuda(),
                     rec=torch.empty(m * 32, dtype=torch.uint8, device="cuda"),
                     fp=torch.empty(cap, dtype=torch.uint8, device="cuda"),
                     used=torch.zeros(4, dtype=torch.int64, device="cuda"),
                     an=torch.empty(m * mercury_amd.ANALYSIS_DTYPE.itemsize, dtype=torch.uint8, device="cuda"))
            ctx.process_device(d_arena.data_ptr(), b["desc"].data_ptr(), m, b["rec"].data_ptr(), b["fp"].data_ptr(),
                               cap, b["used"].data_ptr(), stream.cuda_stream)
            ctx.analyze_device(d_arena.data_ptr(), b["desc"].data_ptr(), m, b["rec"].data_ptr(), b["fp"].data_ptr(),
                               b["an"].data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize()
            got[lo:lo + m] = _statuses(b["an"].cpu().numpy().view(mercury_amd.ANALYSIS_DTYPE))
        else:                                            # pipelined (own buffers per batch: read at the end)
            b = dict(desc=torch.from_numpy(dd.view(np.uint8)).cuda(),
                     rec=torch.empty(m * 32, dtype=torch.uint8, device="cuda"),
                     fp=torch.empty(cap, dtype=torch.uint8, device="cuda"),
                     used=torch.zeros(4, dtype=torch.int64, device="cuda"),
                     an=torch.empty(m * mercury_amd.ANALYSIS_DTYPE.itemsize, dtype=torch.uint8, device="cuda"))
            ctx.process_device(d_arena.data_ptr(), b["desc"].data_ptr(), m, b["rec"].data_ptr(), b["fp"].data_ptr(),
                               cap, b["used"].data_ptr(), stream.cuda_stream)
            ctx.analyze_device_pipelined(d_arena.data_ptr(), b["desc"].data_ptr(), m, b["rec"].data_ptr(),
                                         b["fp"].data_ptr(), b["an"].data_ptr(), stream.cuda_stream)
            pending.append((lo, m, b))
    ctx.analysis_flush()
    torch.cuda.synchronize()
    for lo, m, b in pending:
        got[lo:lo + m] = _statuses(b["an"].cpu().numpy().view(mercury_amd.ANALYSIS_DTYPE))
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} statuses differ, first at {bad[:5]}"
    ctx.close()


@pytest.mark.gpu
def test_device_pipelined_refuses_deferred_context():
    import torch
    ctx = mercury_amd.Context(f"select=tls;resources={REF_ARCHIVE};analysis", device=0)
    ctx.defer(True)
    z = torch.zeros(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(mercury_amd.api.MercuryAmdError, match="defers"):
        ctx.analyze_device_pipelined(z.data_ptr(), z.data_ptr(), 0, z.data_ptr(), z.data_ptr(), z.data_ptr(), 0)
    ctx.close()


@pytest.mark.gpu
def test_lru_stream_two_shards_shared_prevalence():
    """Two contexts on cuda:0 as two shards of one stream: each analyses its
    half (deferred), then the shards are decided in shard order against one
    shared LRU; statuses equal one context over the whole stream (the
    reference's)."""
    a, d = synth.lru_batch(synth.lru_keys())
    want = golden_status()
    cfg = f"select=tls;resources={REF_ARCHIVE};analysis"
    ctxs = [mercury_amd.Context(cfg, device=0) for _ in range(2)]
    shared = mercury_amd.Prevalence(100000)
    for c in ctxs:
        c.set_prevalence(shared)
        c.defer(True)
    got = np.zeros(len(d), np.uint8)
    step = 20000
    for lo in range(0, len(d), 2 * step):
        parts = []
        for r, c in enumerate(ctxs):
            s_lo, s_hi = min(len(d), lo + r * step), min(len(d), lo + (r + 1) * step)
            if s_lo == s_hi:
                continue
            parts.append((c, s_lo, s_hi, c.process_host_analysis(a, d[s_lo:s_hi])))
        # the ordered host merge: every shard's distinct list, shard order
        lists = []
        for c, s_lo, s_hi, _ in parts:
            dl = c.analysis_distinct()
            dl["first"] += np.uint64(s_lo)
            dl["last"] += np.uint64(s_lo)
            lists.append(dl)
        allv = np.concatenate(lists)
        if shared.resolve_distinct(allv):
            k = 0
            for (c, s_lo, s_hi, _), dl in zip(parts, lists):
                c.analysis_resolve(allv[k:k + len(dl)])
                k += len(dl)
        else:
            for c, s_lo, s_hi, _ in parts:
                c.analysis_resolve_sequence(shared.resolve_sequence(c.analysis_sequence()))
        for c, s_lo, s_hi, (rec, fp, an) in parts:
            # the host copies were taken before the decision: re-read the device result
            got[s_lo:s_hi] = _statuses(c.last_analysis())
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} differ, first {bad[:5]}"
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("kind", ["few", "wide", "bursts", "cycle"])
@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_prevalence_shards_decided_where_they_lie(kind, world):
    """mfp_prevalence_summary / resolve_shard / advance (shard.py's
    decide-once merge): every shard decided from its predecessors' summaries,
    then the set advanced, over three steps, equals one pass over the
    concatenated stream -- decisions and the recency order at the end."""
    rng = np.random.default_rng(["few", "wide", "bursts", "cycle"].index(kind) * 10 + world)
    cap = 200
    ranks = [mercury_amd.Prevalence(cap) for _ in range(world)]
    whole = mercury_amd.Prevalence(cap)
    for step in range(3):
        shards = []
        for r in range(world):
            n = int(rng.integers(0, 5000)) if r != 1 else 40      # short shards too
            if kind == "few":
                keys = rng.integers(0, 150, n)
            elif kind == "wide":
                keys = rng.integers(0, 5000, n)
            elif kind == "bursts":
                keys = rng.integers(0, 120, n) + 50 * (np.arange(n) // 900) + 1000 * step
            else:
                keys = np.tile(np.arange(300), n // 300 + 1)[:n] + 7 * r
            shards.append(key_hash(keys))
        want = whole.resolve_sequence(np.concatenate(shards))
        for p in ranks:                                   # every rank's copy, same inputs
            summ = [p.summary(s) for s in shards]
            assert all(len(x) <= cap for x in summ)
            got = [p.resolve_shard(shards[r], np.concatenate(summ[:r][::-1]) if r else np.zeros(0, np.uint64))
                   for r in range(world)]
            assert np.array_equal(np.concatenate(got), want), (kind, world, step)
        for p in ranks:
            p.advance(np.concatenate([p.summary(s) for s in shards][::-1]))
            assert np.array_equal(p.keys(), whole.keys()), (kind, world, step)
