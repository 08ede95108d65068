"""QUIC Initial packets: decryption and fingerprinting on
the device (mercury_amd/csrc/mfp_quic.hip) against the REFERENCE.

Expected values are the reference's own outputs (libmerc 2.18.0 compiled by
oracle/Makefile.ref, run by tests/golden/make_golden_quic.py) on
* the packets of the reference's QUIC test pcaps (unit_tests/pcaps/quic*.pcap:
  v1, v2, draft-29, PPP-framed, reordered CRYPTO frames, fragmented
  ClientHellos, the crypto-packets capture);
* the synthetic Initials of tests/quic_synth.py (every version family, header
  field extremes, split / reordered / missing / overlapping CRYPTO frames,
  bad tags, reserved bits, non-Initial types, unprotected Initials, AAD over
  1 KiB, payloads past the 2 KiB plaintext buffer, 600 randomized Initials).
Bar: identical emit / fp type / truncation flags and byte-identical strings.

CPU tests: the device cryptography compiled for the host against RFC 9001
Appendix A and libcrypto (tests/c/quic_crypto_test.cc), and the config parser.
"""
import gzip
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import mercury_amd

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLD = os.path.join(HERE, "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "quic_manifest.json")))


def load():
    z = np.load(os.path.join(GOLD, "quic_packets.npz"))
    return z["arena"], z["desc"], z["sources"]


def load_ref(key):
    rows = []
    with gzip.open(os.path.join(GOLD, f"quic_fp_{key}.tsv.gz"), "rt", encoding="latin-1") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            rows.append((int(p[1]), int(p[2]), int(p[3]), p[4] if len(p) > 4 else ""))
    return rows


def test_quic_fixture_shape():
    arena, desc, sources = load()
    assert len(desc) == MANIFEST["packets"] == len(load_ref("q0"))
    assert MANIFEST["counts"]["q0"]["quic_fp"] > 700
    assert any(str(s).startswith("quic_v2.pcap") for s in sources)


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ and libcrypto headers")
def test_quic_crypto_host_build(tmp_path):
    """k_quic's SHA-256/HMAC/HKDF/AES/GHASH code (mfp_quic_crypto.hpp), built
    for the host: RFC 9001 A.1/A.2 answers and libcrypto on random vectors."""
    exe = tmp_path / "qct"
    src = os.path.join(HERE, "c", "quic_crypto_test.cc")
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-Wno-unknown-pragmas", "-Wno-deprecated-declarations",
                        "-I", os.path.join(ROOT, "mercury_amd", "csrc"), src, "-o", str(exe), "-lcrypto"],
                       capture_output=True, text=True)
    if r.returncode != 0 and "openssl" in r.stderr:
        pytest.skip("libcrypto headers unavailable")
    assert r.returncode == 0, r.stderr[-2000:]
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr[-2000:]


def test_quic_config_parse():
    lib = mercury_amd.load_library()
    import ctypes
    sel, fmt = ctypes.c_uint32(), ctypes.c_uint32()
    assert lib.mfp_parse_filter(b"quic", ctypes.byref(sel), ctypes.byref(fmt)) == 0
    assert sel.value == 1 << 10 and fmt.value == 0
    assert lib.mfp_parse_filter(b"select=tls,quic;format=tls/2,quic/1", ctypes.byref(sel), ctypes.byref(fmt)) == 0
    assert sel.value == (1 << 10) | 7 and fmt.value == 2 | (1 << 8)
    assert lib.mfp_parse_filter(b"select=quic;format=quic/2", ctypes.byref(sel), ctypes.byref(fmt)) != 0


def run_gpu(arena, desc, cfg, monkeypatch=None):
    ctx = mercury_amd.Context(cfg, device=0)
    try:
        rec, fp = ctx.process_host(arena, desc)
    finally:
        ctx.close()
    return rec, mercury_amd.fingerprints(rec, fp)


def compare(rec, fps, ref, sources):
    bad = []
    for i, (emit, t, trunc, s) in enumerate(ref):
        g_emit = int(rec["flags"][i] & 1)
        g = (g_emit, int(rec["fp_type"][i]), int((rec["flags"][i] >> 1) & 1) & g_emit, fps[i])
        if g != (emit, t, trunc, s):
            bad.append((i, str(sources[i]), g[:3], (emit, t, trunc)))
    return bad


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["q0", "q1", "mix"])
def test_quic_vs_reference(key):
    arena, desc, sources = load()
    rec, fps = run_gpu(arena, desc, MANIFEST["configs"][key])
    bad = compare(rec, fps, load_ref(key), sources)
    assert not bad, f"{len(bad)} mismatches, first: {bad[:5]}"
    q = rec["msg"] == 13
    assert int((rec["fp_type"][q] == 12).sum()) == MANIFEST["counts"][key]["quic_fp"]


@pytest.mark.gpu
def test_quic_lane_strategy_and_misbinning(monkeypatch):
    """Without the classify pass (MFP_STRATEGY=lane) every QUIC packet reaches
    k_quic through the walker's hand-over list; same output."""
    monkeypatch.setenv("MFP_STRATEGY", "lane")
    arena, desc, sources = load()
    rec, fps = run_gpu(arena, desc, MANIFEST["configs"]["mix"])
    bad = compare(rec, fps, load_ref("mix"), sources)
    assert not bad, f"{len(bad)} mismatches, first: {bad[:5]}"


@pytest.mark.gpu
def test_quic_replicated_batch():
    """A larger batch (the fixture replicated 40x, ~60 k packets, several k_quic
    tiles per workgroup): every replica equals the reference."""
    arena, desc, sources = load()
    reps = 40
    n = len(desc)
    big_desc = np.tile(desc, reps)
    big_desc["offset"] += np.repeat(np.arange(reps, dtype=np.uint64) * np.uint64(len(arena)), n)
    big_arena = np.tile(arena, reps)
    rec, fps = run_gpu(big_arena, big_desc, MANIFEST["configs"]["q0"])
    ref = load_ref("q0")
    for r in (0, reps // 2, reps - 1):
        sl = slice(r * n, (r + 1) * n)
        assert not compare(rec[sl], fps[sl], ref, sources), f"replica {r}"
    assert int((rec["fp_type"] == 12).sum()) == reps * MANIFEST["counts"]["q0"]["quic_fp"]


# ---------------------------------------------------------------------------
# --analysis on QUIC Initials (quic_init::do_analysis quic.h:1722-1752): the
# classifier reads the server name and the QUIC user agent from the sidecar
# k_quic writes behind the fingerprint; the archive's quic/1 entries force the
# QUIC format (pkt_proc.h:97-99)
# ---------------------------------------------------------------------------
def load_attr():
    return load_attr_file("quic_attr.tsv.gz")


def load_attr_file(name):
    rows = []
    with gzip.open(os.path.join(GOLD, name), "rt", encoding="latin-1") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            attrs = {}
            for kv in p[3].split(";"):
                if kv:
                    k, v = kv.split("=")
                    attrs[k] = v
            rows.append((int(p[1]), int(p[2]), attrs))
    return rows


@pytest.mark.gpu
def test_quic_analysis_vs_reference():
    from tests import test_analysis
    arena, desc, sources = load()
    cfg = f"select=quic;resources={os.path.join(GOLD, 'quic_resources.tgz')};analysis"
    ctx = mercury_amd.Context(cfg, device=0, mode=mercury_amd.api.MODE_ANALYSIS)
    try:
        assert ctx.analysis_enabled
        rec, fp, an, ap = ctx.process_host_analysis(arena, desc, attr_prob=True)
        names = [ctx.process_name(int(p)) for p in an["process"]]
        tag_names = {b: ctx.attribute_name(b) for b in range(16)}
    finally:
        ctx.close()
    ref = test_analysis.load_ref_an("quic_an.tsv.gz")
    bad = test_analysis.compare(ref, rec, an, names)
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"
    assert sum(r["valid"] for r in ref) > 700 and sum(r["status"] == 1 for r in ref) > 300
    # attributes: names and probabilities (%.17g of the same doubles)
    bad = []
    for i, (valid, status, want) in enumerate(load_attr()):
        got = {}
        for b in range(16):
            if not (int(an["attr"][i]) >> b) & 1:
                continue
            name = tag_names[b]
            if b >= mercury_amd.api.ATTR_DB_FIRST:
                p = float(ap[i][b - mercury_amd.api.ATTR_DB_FIRST])
            elif name == "encrypted_channel":
                p = float(an["malware_prob"][i])
            else:
                p = 1.0
            if p != 0:
                got[name] = "%.17g" % p
        if got != want:
            bad.append((i, got, want))
    assert not bad, f"{len(bad)} attribute mismatches, first {bad[:3]}"
    assert sum("encrypted_dns" in w for _, _, w in load_attr()) > 500


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["q0", "mix"])
def test_quic_json_vs_reference(key):
    """The write_json text of every packet: the "tls" object of the decrypted
    ClientHello (first server_name, quic_transport_parameters, google user
    agents) and the "quic" object (connection_info, version, dcid, scid,
    token, the last ack / ack_ecn / connection_close frame, salt_string,
    plaintext or raw_packet_data) rebuilt from k_quic's sidecar,
    byte-identical to the reference (quic.h:531-540, 1438-1452, 1662-1690)."""
    from tests import test_json
    arena, desc, sources = load()
    ctx = mercury_amd.Context(MANIFEST["configs"][key], device=0)
    try:
        rec, fp = ctx.process_host(arena, desc)
    finally:
        ctx.close()
    lines, skipped = mercury_amd.write_json(arena, desc, rec, fp, ts_ns=np.full(len(desc), test_json.TS, np.uint64),
                                            threads=2)
    test_json._check(lines, test_json._golden_lines(f"quic_json_{key}.txt.gz"), skipped)
    assert MANIFEST["counts"][key]["quic_objects"] == 833
