"""STUN and OpenVPN over TCP (beside QUIC): fingerprints
on the device against the REFERENCE.

* STUN (stun::message stun.h:783-1013) is parsed by the lane walker (the
  "other" bin, FAM_STUN); identification is udp4's length matcher
  (proto_identify.h:387-390, 868-870).  Requests give `stun/1/...`, responses
  a record without a fingerprint.  With --analysis the STUN request
  fingerprints are classified with SOFTWARE as the user agent
  (stun.h:1021-1036).
* OpenVPN over TCP (openvpn_tcp openvpn.h:353-500) on port 1194
  (proto_identify.h:1028-1030) is parsed by k_quic's lane (the ClientHello is
  gathered from several control records into an 800-byte buffer):
  `openvpn/(06)(records)(opcode key)(hmac length)` + the format-0 TLS
  ClientHello fingerprint.

Expected values: tests/golden/make_golden_stun_ovpn.py, the reference libmerc
(oracle/_ref) over the reference's stun/openvpn pcaps, the STUN/OpenVPN
packets of emix.pcap and surfshark.pcap, tests/stun_ovpn_synth.py scenarios
and 3000 mutations of them.  Bar: identical emit / fp type / truncation and
byte-identical strings; classifier status/process/malware exact, score and
p_malware within 1e-6.
"""
import ctypes
import gzip
import json
import os

import numpy as np
import pytest

import mercury_amd
from tests import test_analysis

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "stun_ovpn_manifest.json")))


def load():
    z = np.load(os.path.join(GOLD, "stun_ovpn_packets.npz"))
    return z["arena"], z["desc"], z["sources"]


def load_ref(key):
    rows = []
    with gzip.open(os.path.join(GOLD, f"stun_ovpn_fp_{key}.tsv.gz"), "rt", encoding="latin-1") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            rows.append((int(p[1]), int(p[2]), int(p[3]), p[4] if len(p) > 4 else ""))
    return rows


def test_fixture_shape():
    arena, desc, sources = load()
    assert len(desc) == MANIFEST["packets"] == len(load_ref("so"))
    c = MANIFEST["counts"]
    assert c["so"]["stun_fp"] > 500 and c["so"]["openvpn_fp"] > 100
    assert c["an"]["valid"] == c["stun"]["stun_fp"] and c["an"]["labeled"] > 300
    assert any(str(s).startswith("openvpn_tcp_multi.pcap") for s in sources)


def test_config_parse():
    lib = mercury_amd.load_library()
    sel, fmt = ctypes.c_uint32(), ctypes.c_uint32()
    assert lib.mfp_parse_filter(b"stun,openvpn_tcp", ctypes.byref(sel), ctypes.byref(fmt)) == 0
    assert sel.value == (1 << 14) | (1 << 15)
    assert lib.mfp_parse_filter(b"openvpn", ctypes.byref(sel), ctypes.byref(fmt)) != 0   # the reference's name is openvpn_tcp


def run_gpu(arena, desc, cfg):
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
            bad.append((i, str(sources[i]), g, (emit, t, trunc, s[:80])))
    return bad


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["so", "mix", "stun"])
def test_stun_ovpn_vs_reference(key):
    arena, desc, sources = load()
    rec, fps = run_gpu(arena, desc, MANIFEST["configs"][key])
    bad = compare(rec, fps, load_ref(key), sources)
    assert not bad, f"{len(bad)} mismatches, first: {bad[:4]}"
    assert int((rec["fp_type"] == 16).sum()) == MANIFEST["counts"][key]["stun_fp"]
    assert int((rec["fp_type"] == 14).sum()) == MANIFEST["counts"][key]["openvpn_fp"]


@pytest.mark.gpu
def test_stun_ovpn_lane_strategy(monkeypatch):
    """Without the classify pass every packet takes the all-protocol lane
    walker (STUN in place, OpenVPN handed to k_quic); same output."""
    monkeypatch.setenv("MFP_STRATEGY", "lane")
    arena, desc, sources = load()
    rec, fps = run_gpu(arena, desc, MANIFEST["configs"]["mix"])
    bad = compare(rec, fps, load_ref("mix"), sources)
    assert not bad, f"{len(bad)} mismatches, first: {bad[:4]}"


@pytest.mark.gpu
def test_stun_analysis_vs_reference():
    arena, desc, sources = load()
    cfg = f"select=stun;resources={os.path.join(GOLD, 'stun_resources.tgz')};analysis"
    ctx = mercury_amd.Context(cfg, device=0, mode=mercury_amd.api.MODE_ANALYSIS)
    try:
        assert ctx.analysis_enabled
        rec, fp, an = ctx.process_host_analysis(arena, desc)
        names = [ctx.process_name(int(p)) for p in an["process"]]
    finally:
        ctx.close()
    ref = test_analysis.load_ref_an("stun_ovpn_an.tsv.gz")
    bad = test_analysis.compare(ref, rec, an, names)
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"
    assert sum(r["status"] == 1 for r in ref) == MANIFEST["counts"]["an"]["labeled"]


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["so", "mix"])
def test_stun_ovpn_json_vs_reference(key):
    """The "stun" objects (attributes, addresses, usage) and "openvpn" objects
    (records, data length, the ClientHello's "tls" object) rebuilt by the host
    JSON writer from the records equal the reference's write_json text."""
    from tests import test_json
    arena, desc, sources = load()
    ctx = mercury_amd.Context(MANIFEST["configs"][key], device=0)
    try:
        rec, fp = ctx.process_host(arena, desc)
    finally:
        ctx.close()
    lines, skipped = mercury_amd.write_json(arena, desc, rec, fp, ts_ns=np.full(len(desc), test_json.TS, np.uint64),
                                            threads=4)
    gold = test_json._golden_lines(f"stun_ovpn_json_{key}.txt.gz")
    test_json._check(lines, gold, skipped)


@pytest.mark.gpu
def test_classifier_more_than_512_processes():
    """Fingerprints with 513..4096 processes (k_analyze_big: one wave per
    packet, 64 process chunks in LDS) equal the reference
    (tests/golden/make_golden_bigp.py)."""
    m = json.load(open(os.path.join(GOLD, "bigp_manifest.json")))
    arena, desc, sources = load()
    cfg = f"select=stun;resources={os.path.join(GOLD, 'bigp_resources.tgz')};analysis"
    ctx = mercury_amd.Context(cfg, device=0, mode=mercury_amd.api.MODE_ANALYSIS)
    try:
        rec, fp, an = ctx.process_host_analysis(arena, desc)
        names = [ctx.process_name(int(p)) for p in an["process"]]
        stats = ctx.analysis_stats()
    finally:
        ctx.close()
    ref = test_analysis.load_ref_an("bigp_an.tsv.gz")
    bad = test_analysis.compare(ref, rec, an, names)
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"
    assert m["valid_big_p"] > 50


@pytest.mark.gpu
def test_classifier_more_than_4096_processes():
    """Fingerprints with 4097..9000 processes (k_analyze_huge: one wave per
    packet, the score row in HBM scratch) equal the reference
    (tests/golden/make_golden_hugep.py); none is left unscored."""
    m = json.load(open(os.path.join(GOLD, "hugep_manifest.json")))
    arena, desc, sources = load()
    cfg = f"select=stun;resources={os.path.join(GOLD, 'hugep_resources.tgz')};analysis"
    ctx = mercury_amd.Context(cfg, device=0, mode=mercury_amd.api.MODE_ANALYSIS)
    try:
        rec, fp, an = ctx.process_host_analysis(arena, desc)
        names = [ctx.process_name(int(p)) for p in an["process"]]
        counters = ctx.analysis_counters()
    finally:
        ctx.close()
    ref = test_analysis.load_ref_an("hugep_an.tsv.gz")
    bad = test_analysis.compare(ref, rec, an, names)
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"
    assert m["valid_huge_p"] > 100
    assert counters["oversize"] >= m["valid_huge_p"]   # every one of them went through k_analyze_huge
