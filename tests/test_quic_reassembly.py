"""QUIC CRYPTO-frame reassembly (ClientHellos spanning several Initials:
process_udp_data pkt_proc.cc:933-939, process_quic_reassembly
reassembly.hpp:895-1033) against the reference.

Expected values: tests/golden/make_golden_quic_reasm.py, the reference libmerc
(oracle/_ref) with "reassembly" over one stream: the reference's own QUIC pcaps
(quic_fragmented, quic_reordered_frames, quic-crypto-packets,
quic_init.capture2), then tests/quic_reasm_synth.py (parts in order, permuted,
the first datagram last, several CRYPTO frames per datagram, gaps and a first
frame under 10 bytes, duplicates, overlaps, a lost datagram, two connection ids
on one 5-tuple, interleaved 5-tuples, IPv6, v2 and draft versions,
unprotected Initials, ClientHellos beyond the 8192-byte buffer) and a timed
stream whose connections stall past the 15 s timeout.  k_quic decrypts every
Initial and hands the host its plaintext; the host keeps the flow table in
stream order; completed ClientHellos are parsed by k_quic again from the
reassembled CRYPTO data in their completing packets' places
(MFP_DESC_QUIC_CRYPTO).
"""
import gzip
import json
import os

import numpy as np
import pytest

import mercury_amd
from mercury_amd import api
from tests import test_reassembly as tr

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "quic_reasm_manifest.json")))
TS = 1700000000 * 10**9


def load(name="quic_reasm_packets.npz"):
    z = np.load(os.path.join(GOLD, name))
    return z["arena"], z["desc"], (z["ts"].astype(np.uint64) * 10**9 if "ts" in z else None)


def load_ref(key):
    rows = []
    with gzip.open(os.path.join(GOLD, f"quic_reasm_fp_{key}.tsv.gz"), "rt", encoding="latin-1") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            rows.append((int(p[1]), int(p[2]), int(p[3]), p[4] if len(p) > 4 else ""))
    return rows


def test_fixture_shape():
    arena, desc, _ = load()
    assert len(desc) == MANIFEST["counts"]["packets"] == len(load_ref("q0"))
    c = MANIFEST["counts"]
    assert c["q0"]["reassembled"] > 40 and c["pcap_packets"] > 0
    assert c["timed"]["reassembled"] > 0 and c["an_path"]["more"] > 50


def run(cfg, arena, desc, ts_ns, chunk=None):
    ctx = mercury_amd.Context(cfg, device=0)
    try:
        n = len(desc)
        chunk = chunk or n
        recs, fps, props, lines = [], [], [], []
        for lo in range(0, n, chunk):
            d = desc[lo:lo + chunk]
            t = ts_ns[lo:lo + chunk]
            rec, fp, pr, a2, d2 = ctx.process_host_reassembly(arena, d, ts_ns=t)
            recs.append(rec)
            fps += mercury_amd.fingerprints(rec, fp)
            props.append(pr)
            ln, skipped = mercury_amd.write_json(a2, d2, rec, fp, ts_ns=t, threads=2, props=pr)
            assert skipped == 0
            lines += ln
        return np.concatenate(recs), fps, np.concatenate(props), lines
    finally:
        ctx.close()


def check(key, rec, fps, lines, json_name):
    from tests import test_json
    ref = load_ref(key)
    bad = []
    for i, (emit, t, trunc, s) in enumerate(ref):
        g = (int(rec["flags"][i] & 1), int(rec["fp_type"][i]) if rec["flags"][i] & 1 else 0, fps[i])
        if g != (emit, t, s):
            bad.append((i, g[:2], (emit, t)))
    assert not bad, f"{len(bad)} fingerprint mismatches, first: {bad[:4]}"
    test_json._check(lines, test_json._golden_lines(json_name), 0)


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["q0", "q1"])
def test_quic_reassembly_vs_reference(key):
    arena, desc, _ = load()
    rec, fps, props, lines = run(MANIFEST["configs"][key], arena, desc, np.full(len(desc), TS, np.uint64))
    check(key, rec, fps, lines, f"quic_reasm_json_{key}.txt.gz")
    assert int((props & 1).sum()) == MANIFEST["counts"][key]["reassembled"]


@pytest.mark.gpu
def test_quic_reassembly_across_batches():
    arena, desc, _ = load()
    rec, fps, props, lines = run(MANIFEST["configs"]["q0"], arena, desc, np.full(len(desc), TS, np.uint64), chunk=13)
    check("q0", rec, fps, lines, "quic_reasm_json_q0.txt.gz")


@pytest.mark.gpu
def test_quic_reassembly_timed_vs_reference():
    """Connections stalled past the 15 s timeout are reaped before their next
    Initial, which is then taken on its own."""
    from tests import test_json
    arena, desc, ts = load("quic_reasm_timed_packets.npz")
    ctx = mercury_amd.Context(MANIFEST["configs"]["q0"], device=0)
    try:
        rec, fp, props, a2, d2 = ctx.process_host_reassembly(arena, desc, ts_ns=ts)
    finally:
        ctx.close()
    lines, skipped = mercury_amd.write_json(a2, d2, rec, fp, ts_ns=ts, threads=2, props=props)
    test_json._check(lines, test_json._golden_lines("quic_reasm_timed_json.txt.gz"), skipped)


@pytest.mark.gpu
def test_quic_reassembly_analysis_path():
    """The analysis_context path: per packet the context's validity, status,
    process and more_pkts_needed equal the reference's (flow_state_pkts_needed
    while a ClientHello is in reassembly; the reassembled ClientHello classified
    in its completing packet's place)."""
    arena, desc, _ = load()
    ref = tr.load_ref_anr("quic_reasm_an.tsv.gz")
    cfg = MANIFEST["an_config"] + f";resources={os.path.join(GOLD, 'quic_resources.tgz')};analysis"
    ctx = mercury_amd.Context(cfg, device=0, mode=api.MODE_ANALYSIS)
    try:
        rec, fp, props, a2, d2, an, ap, more = ctx.analyze_host_reassembly(arena, desc,
                                                                         ts_ns=np.full(len(desc), TS, np.uint64))
    finally:
        ctx.close()
    bad = [(i, int(an["flags"][i] & 1), int(more[i]), r["valid"], r["more"]) for i, r in enumerate(ref)
           if (int(an["flags"][i] & 1), int(more[i])) != (r["valid"], r["more"])]
    assert not bad, f"{len(bad)} mismatches, first: {bad[:6]}"
    st = [(i, int(an["status"][i]), r["status"]) for i, r in enumerate(ref)
          if r["valid"] and int(an["status"][i]) != r["status"]]
    assert not st, f"{len(st)} status mismatches, first: {st[:6]}"
