"""Reassembly reaping order against the reference: the flow table kept in the
reference's container with its hash (std::hash<key> flow_key.h:257-317) and
reaped from a persistent iterator as passive_reap / active_reap do
(reassembly.hpp:596-655).

Expected values: tests/golden/make_golden_reap.py, the reference libmerc
(oracle/_ref) over tests/reasm_synth.py reap_scenarios with per-packet capture
times: 10 150 flows opened (past the 10 000-entry table, so each new flow
drops two from the iterator), their second segments (152 flows were dropped,
which ones is the table's iteration order), then 64 flows stalled past the
15 s timeout and reaped two per lookup while new flows arrive -- 5 survive to
complete with "timeout".  Per packet: emit, fingerprint type, fingerprint and
"reassembly_properties" identical, as one batch and across batches.
"""
import gzip
import json
import os

import numpy as np
import pytest

import mercury_amd
from tests import test_reassembly as tr

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "reap_manifest.json")))


def load():
    z = np.load(os.path.join(GOLD, "reap_packets.npz"))
    return z["arena"], z["desc"], z["ts"].astype(np.uint64) * 10**9, z["phase"]


def load_ref():
    rows = []
    with gzip.open(os.path.join(GOLD, "reap_fp.tsv.gz"), "rt", encoding="latin-1") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            rows.append((int(p[1]), int(p[2]), int(p[3]), p[4] if len(p) > 4 else ""))
    with gzip.open(os.path.join(GOLD, "reap_props.txt.gz"), "rt", encoding="latin-1") as f:
        props = f.read().split("\n")[:len(rows)]
    return rows, props


def test_fixture_shape():
    arena, desc, ts, phase = load()
    c = MANIFEST["counts"]
    assert len(desc) == c["packets"] == len(load_ref()[0])
    assert 0 < c["finish"] < int((phase == "finish").sum())    # active reaping dropped some flows
    assert 0 < c["late"] < int((phase == "late").sum()) and c["timeout"] == c["late"]


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [None, 4096])
def test_reaping_order_vs_reference(chunk):
    arena, desc, ts, phase = load()
    ctx = mercury_amd.Context(MANIFEST["config"], device=0)
    try:
        n = len(desc)
        chunk = chunk or n
        recs, fps, props = [], [], []
        for lo in range(0, n, chunk):
            rec, fp, pr, _, _ = ctx.process_host_reassembly(arena, desc[lo:lo + chunk], ts_ns=ts[lo:lo + chunk])
            recs.append(rec)
            fps += mercury_amd.fingerprints(rec, fp)
            props.append(pr)
    finally:
        ctx.close()
    rec, props = np.concatenate(recs), np.concatenate(props)
    ref, ref_props = load_ref()
    bad = tr.compare(rec, fps, props, ref, ref_props)
    assert not bad, f"{len(bad)} mismatches, first: {[(i, str(phase[i]), g, w) for i, g, w in bad[:6]]}"
    assert int((props & 1).sum()) == MANIFEST["counts"]["reassembled"]
