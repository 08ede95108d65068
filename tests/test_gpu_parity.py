"""Parity of the HIP path (libmercury_amd.so, called through the C-ABI) with
the reference.

* golden: packets from the reference's own test pcaps, compared with the
  reference's output committed under tests/golden/ (fmt 0/1/2);
* oracle: seeded synthetic and fuzzed batches, compared with the C oracle;
* large: BASELINE-sized device-resident batches checked through
  size-independent properties (every fingerprint string of a sample equals the
  oracle's; arena accounting; record/type consistency).
Bar: byte-identical fingerprint strings, identical fp types, emit and
truncation flags.
"""
import gzip
import os

import numpy as np
import pytest

import mercury_amd
from oracle import oracle
from tests import synth

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


def _compare(arena, desc, fmt, mode=0):
    cfg = oracle.config(tls_format=fmt, mode=mode)
    ft, fl, flags, want = oracle.process_batch(arena, desc, cfg)
    ctx = mercury_amd.Context(cfg_string(fmt), device=0, mode=mode)
    try:
        rec, fp = ctx.process_host(arena, desc)
    finally:
        ctx.close()
    got = mercury_amd.fingerprints(rec, fp)
    bad = [i for i in range(len(desc))
           if got[i] != want[i] or int(rec["fp_type"][i]) != int(ft[i])
           or int(rec["flags"][i] & 3) != int(flags[i] & 3) and (flags[i] & 1)]
    return bad, rec


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [0, 1, 2])
@pytest.mark.parametrize("workload", ["mixed", "tls_ch"])
def test_synthetic_vs_oracle(fmt, workload):
    arena, desc = synth.batch(30000, seed=0x5EED0003 + fmt, workload=workload, n_templates=3000)
    bad, rec = _compare(arena, desc, fmt)
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"
    assert (rec["fp_type"] > 0).sum() > 10000


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_fuzzed_vs_oracle(fmt):
    arena, desc, _ = load_golden()
    pk = [(int(d["linktype"]), arena[int(d["offset"]):int(d["offset"]) + int(d["caplen"])].tobytes()) for d in desc]
    a2, d2 = synth.batch(3000, seed=99, workload="mixed", n_templates=1000)
    pk += [(1, a2[int(d["offset"]):int(d["offset"]) + int(d["caplen"])].tobytes()) for d in d2]
    from tests import pcaplib
    fz = synth.fuzz(pk, 40000, seed=1000 + fmt)
    fa, fd = pcaplib.make_batch(fz)
    bad, _ = _compare(fa, fd, fmt)
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"


@pytest.mark.gpu
@pytest.mark.parametrize("seg_mask,lds_mask", [
    ("0x0", "0x0"), ("0xa", "0x0"), ("0xff", "0x0"), ("0xa", "0xff"), ("0x0", "0xff"), ("0xff", "0xff"),
    ("0xa", "0x5a")])
def test_bin_kernel_choices_vs_oracle(seg_mask, lds_mask, monkeypatch):
    """Every bin kernel (HBM lane walker, lane walk + wave expansion, and the
    LDS-staged walker in both emission modes, each carrying only its bin's
    parser family) takes any packet (what it cannot fingerprint goes to the
    fallback lane): one batch of synthetic + fuzzed packets under each
    assignment of kernels to bins equals the oracle."""
    from tests import pcaplib
    monkeypatch.setenv("MFP_BIN_SEG_MASK", seg_mask)
    monkeypatch.setenv("MFP_BIN_LDS_MASK", lds_mask)
    a2, d2 = synth.batch(6000, seed=0x5EED0042, workload="mixed", n_templates=1500)
    pk = [(1, a2[int(d["offset"]):int(d["offset"]) + int(d["caplen"])].tobytes()) for d in d2]
    pk += synth.fuzz(pk[:2000], 10000, seed=77)
    fa, fd = pcaplib.make_batch(pk)
    for fmt in (0, 2):
        bad, rec = _compare(fa, fd, fmt)
        assert not bad, f"fmt {fmt}: {len(bad)} mismatches, first {bad[:5]}"
    assert (rec["fp_type"] == 3).sum() > 100 and (rec["fp_type"] == 4).sum() > 100


@pytest.mark.gpu
def test_analysis_mode_vs_oracle():
    """get_analysis_context semantics: no TCP SYN fingerprints (pkt_proc.cc:1624-1651)."""
    arena, desc = synth.batch(20000, seed=5, workload="mixed", n_templates=2000)
    bad, rec = _compare(arena, desc, 1, mode=1)
    assert not bad
    assert int((rec["fp_type"] == 7).sum()) == 0


@pytest.mark.gpu
def test_edge_cases():
    """empty packets, zero-length batch members, ragged sizes, max-size frames."""
    from tests import pcaplib
    pk = [(1, b""), (1, b"\x00"), (101, b"\x45"), (1, bytes(14)), (1, bytes(65535))]
    a, d = synth.batch(200, seed=3, workload="mixed", n_templates=100)
    for x in d[:50]:
        b = a[int(x["offset"]):int(x["offset"]) + int(x["caplen"])].tobytes()
        pk.append((1, b + bytes(70000 - len(b))))   # giant trailing data
        for cut in (0, 13, 14, 33, 34, 53, 54, len(b) // 2, len(b) - 1):
            pk.append((1, b[:cut]))
    fa, fd = pcaplib.make_batch(pk)
    bad, _ = _compare(fa, fd, 0)
    assert not bad


@pytest.mark.gpu
def test_large_device_batch_properties():
    """BASELINE-size batch (config 2 shape, 10 M TLS ClientHellos) device-resident;
    a seeded 20 000-packet sample must equal the oracle byte for byte and the
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
    rng = np.random.default_rng(1)
    sample = rng.choice(n, 20000, replace=False)
    fp_host = d_fp[:used].cpu().numpy().tobytes()
    got = mercury_amd.fingerprints(rec[sample], fp_host)
    srec = desc[sample]
    ft, fl, flags, want = oracle.process_batch(ua, ud[sample % len(ud)], oracle.config())
    assert got == want
    # replicas are identical: per-position fp_len pattern repeats
    assert np.array_equal(rec["fp_len"][:len(ud)], rec["fp_len"][-len(ud):])
    ctx.close()
    del srec


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
