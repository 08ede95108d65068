"""DTLS ClientHello fragment reassembly (UDP offset reassembly: process_udp_data
pkt_proc.cc:896-945, process_udp_offset_reassembly reassembly.hpp:1036-1100)
against the reference.

Expected values: tests/golden/make_golden_dtls_reasm.py, the reference libmerc
(oracle/_ref) with "reassembly" over one stream: the reference's own
fragmented-ClientHello pcaps (unit_tests/pcaps/dtls_fragmented_client_hello*,
dtls_interleaved_client_hello), then tests/dtls_reasm_synth.py (fragments in
order, permuted, duplicated, overlapping, missing, a later fragment first,
interleaved flows, a second message_seq on a 5-tuple in reassembly, IPv6, long
ClientHellos, messages beyond the 8192-byte buffer) and a timed stream whose
flows stall past the 15 s timeout.  The device walk records each fragment's
offset, length and additional bytes (MFP_SEG_DTLS); the host keeps the flow
table in stream order; completed messages are rebuilt as whole-message
datagrams and fingerprinted by the device in their completing packets' places.
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
MANIFEST = json.load(open(os.path.join(GOLD, "dtls_reasm_manifest.json")))
TS = 1700000000 * 10**9


def load(name="dtls_reasm_packets.npz"):
    z = np.load(os.path.join(GOLD, name))
    return z["arena"], z["desc"], (z["ts"].astype(np.uint64) * 10**9 if "ts" in z else None)


def load_ref(key):
    rows = []
    with gzip.open(os.path.join(GOLD, f"dtls_reasm_fp_{key}.tsv.gz"), "rt", encoding="latin-1") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            rows.append((int(p[1]), int(p[2]), int(p[3]), p[4] if len(p) > 4 else ""))
    return rows


def test_fixture_shape():
    arena, desc, _ = load()
    assert len(desc) == MANIFEST["counts"]["packets"] == len(load_ref("d0"))
    c = MANIFEST["counts"]
    assert c["d0"]["reassembled"] > 50 and c["pcap_packets"] > 0
    assert c["timed"]["reassembled"] > 0


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


def check(key, rec, fps, props, lines, json_name):
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
@pytest.mark.parametrize("key", ["d0", "d1"])
def test_dtls_reassembly_vs_reference(key):
    arena, desc, _ = load()
    rec, fps, props, lines = run(MANIFEST["configs"][key], arena, desc, np.full(len(desc), TS, np.uint64))
    check(key, rec, fps, props, lines, f"dtls_reasm_json_{key}.txt.gz")
    assert int((props & 1).sum()) == MANIFEST["counts"][key]["reassembled"]


@pytest.mark.gpu
def test_dtls_reassembly_across_batches():
    arena, desc, _ = load()
    rec, fps, props, lines = run(MANIFEST["configs"]["d0"], arena, desc, np.full(len(desc), TS, np.uint64), chunk=7)
    check("d0", rec, fps, props, lines, "dtls_reasm_json_d0.txt.gz")


@pytest.mark.gpu
def test_dtls_reassembly_timed_vs_reference():
    """Flows stalled past the 15 s timeout are reaped before their next
    fragment, which is then taken on its own."""
    from tests import test_json
    arena, desc, ts = load("dtls_reasm_timed_packets.npz")
    ctx = mercury_amd.Context(MANIFEST["configs"]["d0"], device=0)
    try:
        rec, fp, props, a2, d2 = ctx.process_host_reassembly(arena, desc, ts_ns=ts)
    finally:
        ctx.close()
    lines, skipped = mercury_amd.write_json(a2, d2, rec, fp, ts_ns=ts, threads=2, props=props)
    test_json._check(lines, test_json._golden_lines("dtls_reasm_timed_json.txt.gz"), skipped)


@pytest.mark.gpu
def test_dtls_reassembly_analysis_path_more_pkts_needed():
    """The analysis_context path: more_pkts_needed per packet equal to the
    reference's (flow_state_pkts_needed while a ClientHello is in reassembly)."""
    arena, desc, _ = load()
    ref = tr.load_ref_anr("dtls_reasm_an.tsv.gz")
    cfg = MANIFEST["an_config"] + f";resources={os.path.join(GOLD, 'resources-test.tgz')};analysis"
    ctx = mercury_amd.Context(cfg, device=0, mode=api.MODE_ANALYSIS)
    try:
        rec, fp, props, a2, d2, an, ap, more = ctx.analyze_host_reassembly(arena, desc,
                                                                         ts_ns=np.full(len(desc), TS, np.uint64))
    finally:
        ctx.close()
    bad = [(i, int(an["flags"][i] & 1), int(more[i]), r["valid"], r["more"]) for i, r in enumerate(ref)
           if (int(an["flags"][i] & 1), int(more[i])) != (r["valid"], r["more"])]
    assert not bad, f"{len(bad)} mismatches, first: {bad[:6]}"
    assert MANIFEST["counts"]["an_path"]["more"] > 50
