"""Parity of the HIP path (libmercury_amd.so, called through the C-ABI) with
the REFERENCE: every expected value below is the reference's own output
(libmerc 2.18.0 compiled from /root/reference by oracle/Makefile.ref, run by
tests/golden/make_golden*.py; committed under tests/golden/):

* golden: packets from the reference's own test pcaps (fmt 0/1/2) and its
  top_100_fingerprints.fp file;
* cases (tests/cases.py, tests/golden/cases/): 40 000 fuzzed packets per
  format, truncation/oversize edge cases, synthetic mixed and ClientHello
  batches, the reference's own fuzzing seeds, the analysis_context path, and
  every assignment of bin kernels;
* large: a BASELINE-sized device-resident batch (config 2, 10 M TLS
  ClientHellos): a seeded sample against the reference, plus size-independent
  properties (arena accounting, replica consistency).
Bar: byte-identical fingerprint strings, identical fp types, emit and
truncation flags.  (The C oracle, oracle/mfp_oracle.c, is a debugging twin,
pinned to the same reference outputs by tests/test_oracle.py.)
"""
import gzip
import os

import numpy as np
import pytest

import mercury_amd
from tests import cases, synth

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CONTRACT = "tls,dtls,ssh,http,tcp,tcp.syn_ack"


_M64 = (1 << 64) - 1


def _mix64(x):
    x ^= x >> 33
    x = (x * 0xff51afd7ed558ccd) & _M64
    x ^= x >> 33
    x = (x * 0xc4ceb9fe1a85ec53) & _M64
    return x ^ (x >> 33)


def str_hash(s):
    """mfpc::str_hash (mercury_amd/csrc/mfp_common.hpp)."""
    acc = 0
    for j in range(0, len(s), 8):
        w = int.from_bytes(s[j:j + 8].ljust(8, b"\0"), "little")
        acc ^= _mix64((w + (j // 8 + 1) * 0x9e3779b97f4a7c15) & _M64)
    return _mix64(acc ^ ((len(s) * 0x2545f4914f6cdd1d) & _M64))


def cfg_string(fmt):
    return CONTRACT if fmt == 0 else f"select={CONTRACT};format=tls/{fmt}"


def load_golden():
    z = np.load(os.path.join(GOLD, "ref_packets.npz"))
    return z["arena"], z["desc"], z["sources"]


def load_ref(fmt):
    rows = []
    with gzip.open(os.path.join(GOLD, f"ref_fp_fmt{fmt}.tsv.gz"), "rt", encoding="latin-1") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            rows.append((int(p[1]), int(p[2]), int(p[3]), p[4] if len(p) > 4 else ""))
    return rows


def run_gpu(arena, desc, fmt):
    ctx = mercury_amd.Context(cfg_string(fmt), device=0)
    try:
        rec, fp = ctx.process_host(arena, desc)
    finally:
        ctx.close()
    return rec, mercury_amd.fingerprints(rec, fp)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_golden_reference_pcaps(fmt):
    arena, desc, sources = load_golden()
    ref = load_ref(fmt)
    rec, fps = run_gpu(arena, desc, fmt)
    bad = []
    for i, (emit, t, trunc, s) in enumerate(ref):
        g_emit = int(rec["flags"][i] & 1)
        g_trunc = int((rec["flags"][i] >> 1) & 1) & g_emit
        if (g_emit, int(rec["fp_type"][i]), g_trunc, fps[i]) != (emit, t, trunc, s):
            bad.append((i, str(sources[i])))
    assert not bad, f"{len(bad)} mismatches, first: {bad[:5]}"
    assert sum(1 for r in ref if r[1]) > 1000


@pytest.mark.gpu
def test_golden_top100_file():
    """test/data/top_100_fingerprints.{pcap,fp}: the reference's own golden file."""
    arena, desc, sources = load_golden()
    sel = [i for i, s in enumerate(sources) if str(s).startswith("top_100_fingerprints.pcap:")]
    rec, fps = run_gpu(arena, desc[sel], 0)
    tls = [fps[k] for k in range(len(sel)) if rec["fp_type"][k] == 1]
    with open(os.path.join(GOLD, "top_100_fingerprints.fp")) as f:
        want = [line.strip().strip('"') for line in f if line.strip()]
    assert tls == want


def _vs_reference(name, fmt, mode="fp"):
    """The HIP path on case `name` against the reference's output."""
    pk = cases.CASES[name][0]()
    arena, desc = cases.batch(pk)
    want = cases.load_golden(name, fmt, mode)
    ctx = mercury_amd.Context(cfg_string(fmt), device=0, mode=0 if mode == "fp" else 1)
    try:
        rec, fp = ctx.process_host(arena, desc)
    finally:
        ctx.close()
    got = mercury_amd.fingerprints(rec, fp)
    bad = []
    for i, (emit, t, trunc, s) in enumerate(want):
        if mode == "fp":
            g_emit = int(rec["flags"][i] & 1)
            g = (g_emit, int(rec["fp_type"][i]), int((rec["flags"][i] >> 1) & 1) & g_emit, got[i])
            if g != (emit, t, trunc, s):
                bad.append(i)
        elif (int(rec["fp_type"][i]), got[i]) != (t, s):
            bad.append(i)
    return bad, rec


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [0, 1, 2])
@pytest.mark.parametrize("workload", ["mixed", "tls_ch"])
def test_synthetic_vs_reference(fmt, workload):
    bad, rec = _vs_reference(f"synth_{workload}{fmt}", fmt)
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"
    assert (rec["fp_type"] > 0).sum() > 10000


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_fuzzed_vs_reference(fmt):
    bad, _ = _vs_reference(f"fuzz{fmt}", fmt)
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_reference_fuzz_corpus(fmt):
    """The reference's own fuzzing seeds (test/fuzz/*/corpus) in frames, and all their prefixes."""
    bad, _ = _vs_reference("corpus", fmt)
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"


@pytest.mark.gpu
@pytest.mark.parametrize("seg_mask,lds_mask", [
    ("0x0", "0x0"), ("0xa", "0x0"), ("0xff", "0x0"), ("0xa", "0xff"), ("0x0", "0xff"), ("0xff", "0xff"),
    ("0xa", "0x5a")])
def test_bin_kernel_choices_vs_reference(seg_mask, lds_mask, monkeypatch):
    """Every bin kernel (HBM lane walker, lane walk + wave expansion, and the
    LDS-staged walker in both emission modes, each carrying only its bin's
    parser family) takes any packet (what it cannot fingerprint goes to the
    fallback lane): one batch of synthetic + fuzzed packets under each
    assignment of kernels to bins equals the reference."""
    monkeypatch.setenv("MFP_BIN_SEG_MASK", seg_mask)
    monkeypatch.setenv("MFP_BIN_LDS_MASK", lds_mask)
    for fmt in (0, 2):
        bad, rec = _vs_reference("binmix", fmt)
        assert not bad, f"fmt {fmt}: {len(bad)} mismatches, first {bad[:5]}"
    assert (rec["fp_type"] == 3).sum() > 100 and (rec["fp_type"] == 4).sum() > 100


@pytest.mark.gpu
def test_lane_strategy_vs_reference(monkeypatch):
    """MFP_STRATEGY=lane: one lane walker over the whole batch (no binning)."""
    monkeypatch.setenv("MFP_STRATEGY", "lane")
    bad, _ = _vs_reference("binmix", 0)
    assert not bad


@pytest.mark.gpu
def test_small_batch_strategy_vs_reference(monkeypatch):
    """MFP_STRATEGY_SMALL (batches up to MFP_SMALL_BATCH packets, the
    per-packet API): the all-family LDS-staged walker over the whole batch,
    then the fallback lane -- here forced for every batch size."""
    monkeypatch.setenv("MFP_SMALL_BATCH", str(1 << 40))
    for fmt in (0, 2):
        bad, _ = _vs_reference("binmix", fmt)
        assert not bad, f"fmt {fmt}: {len(bad)} mismatches, first {bad[:5]}"


@pytest.mark.gpu
def test_analysis_mode_vs_reference():
    """get_analysis_context semantics: no TCP SYN fingerprints (pkt_proc.cc:1624-1651)."""
    bad, rec = _vs_reference("analysis_mode", 1, "an")
    assert not bad
    assert int((rec["fp_type"] == 7).sum()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_edge_cases(fmt):
    """empty packets, 1-byte frames, truncation at every header boundary,
    65 535-byte frames and giant trailing data (the fallback lane)."""
    bad, _ = _vs_reference("edge", fmt)
    assert not bad


@pytest.mark.gpu
def test_large_device_batch_properties():
    """BASELINE-size batch (config 2 shape, 10 M TLS ClientHellos) device-resident;
    a seeded 20 000-packet sample must equal the reference byte for byte and the
    arena accounting must be exact."""
    import torch
    n = 10_000_000
    ua, ud = synth.batch(200_000, seed=0x5EED0001, workload="tls_ch", n_templates=4096)
    reps = n // len(ud)
    span = int(ud["offset"][-1] + ud["caplen"][-1])
    d_arena = torch.from_numpy(ua[:span + 64]).cuda()
    d_arena = d_arena.repeat(reps)
    desc = np.tile(ud, reps)
    desc["offset"] += (np.arange(reps, dtype=np.uint64) * np.uint64(span + 64)).repeat(len(ud))
    d_desc = torch.from_numpy(desc.view(np.uint8)).cuda()
    ctx = mercury_amd.Context(CONTRACT, device=0)
    cap = ctx.fp_arena_bound(desc)
    d_rec = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    d_fp = torch.empty(cap, dtype=torch.uint8, device="cuda")
    d_used = torch.zeros(4, dtype=torch.int64, device="cuda")
    ctx.process_device(d_arena.data_ptr(), d_desc.data_ptr(), n, d_rec.data_ptr(), d_fp.data_ptr(), cap,
                       d_used.data_ptr(), 0)
    torch.cuda.synchronize()
    reserved, overflow, exact, n_fallback = [int(x) for x in d_used.cpu()]
    assert overflow == 0
    rec = d_rec.cpu().numpy().view(mercury_amd.RECORD_DTYPE)
    assert int(rec["fp_len"].astype(np.int64).sum()) == exact
    # every string lies inside the reserved part of the arena
    assert int((rec["fp_offset"] + rec["fp_len"]).max()) <= reserved
    used = reserved
    # a seeded sample of packets whose unique original is in the reference's
    # golden head (the first 20 000 unique packets)
    rng = np.random.default_rng(1)
    sample = rng.choice(reps, 20000) * len(ud) + rng.integers(0, 20000, 20000)
    fp_host = d_fp[:used].cpu().numpy().tobytes()
    got = mercury_amd.fingerprints(rec[sample], fp_host)
    want = cases.load_golden("tls_ch_head", 0, "fp")
    assert got == [want[int(i) % len(ud)][3] for i in sample]
    assert [int(t) for t in rec["fp_type"][sample]] == [want[int(i) % len(ud)][1] for i in sample]
    # replicas are identical: per-position fp_len pattern repeats
    assert np.array_equal(rec["fp_len"][:len(ud)], rec["fp_len"][-len(ud):])
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seg_mask,lds_mask", [("0xa", "0xff"), ("0xa", "0x0"), ("0x0", "0x0")])
def test_device_hash_keys(seg_mask, lds_mask, monkeypatch):
    """Every fingerprint kernel stores its string's classifier key
    (mfpc::str_hash) right after the string (MFP_FLAG_HASHED), so k_analyze
    never re-reads the string to hash it."""
    import torch
    monkeypatch.setenv("MFP_BIN_SEG_MASK", seg_mask)
    monkeypatch.setenv("MFP_BIN_LDS_MASK", lds_mask)
    a, d = synth.batch(30000, seed=0x5EED0077, workload="mixed", n_templates=3000)
    n = len(d)
    ctx = mercury_amd.Context(CONTRACT, device=0)
    cap = ctx.fp_arena_bound(d)
    d_arena = torch.from_numpy(a).cuda()
    d_desc = torch.from_numpy(d.view(np.uint8)).cuda()
    d_rec = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    d_fp = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    d_used = torch.zeros(4, dtype=torch.int64, device="cuda")
    ctx.process_device(d_arena.data_ptr(), d_desc.data_ptr(), n, d_rec.data_ptr(), d_fp.data_ptr(), cap,
                       d_used.data_ptr(), 0)
    torch.cuda.synchronize()
    rec = d_rec.cpu().numpy().view(mercury_amd.RECORD_DTYPE)
    fp_host = d_fp[:int(d_used[0])].cpu().numpy().tobytes()
    ctx.close()
    checked = 0
    for r in rec:
        o, ln = int(r["fp_offset"]), int(r["fp_len"])
        if ln == 0 or not r["flags"] & 4:
            continue
        ho = o + ((ln + 7) & ~7)
        assert int.from_bytes(fp_host[ho:ho + 8], "little") == str_hash(fp_host[o:o + ln])
        checked += 1
    http = int(np.isin(rec["fp_type"], [3, 4]).sum())
    assert checked >= http > 1000
    assert checked == int(((rec["fp_len"] > 0) & (rec["fp_type"] > 0)).sum())   # every string hashed
