"""Decapsulation (encapsulations::process_encapsulations pkt_proc.cc:959-1049):
GRE, VXLAN, Geneve and IP-in-IP on the device against the REFERENCE.

Expected values are the reference's own outputs (tests/golden/make_golden_tunnel.py
over the reference's gre / vxlan / geneve / ip_encapsulation pcaps and the
scenarios of tests/tunnel_synth.py: TLS, HTTP, SYN and QUIC payloads inside
every tunnel type, checksum and key bits, non-IP tunnel payloads, stacks of
two to six levels, headers cut at every byte), under four selections: every
tunnel, format tls/1, VXLAN only, and none (IP-in-IP is always walked).
Bar: identical emit / fp type / truncation flags and byte-identical strings.
"""
import gzip
import json
import os

import numpy as np
import pytest

import mercury_amd

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "tunnel_manifest.json")))


def load():
    z = np.load(os.path.join(GOLD, "tunnel_packets.npz"))
    return z["arena"], z["desc"], z["sources"]


def load_ref(key):
    rows = []
    with gzip.open(os.path.join(GOLD, f"tunnel_fp_{key}.tsv.gz"), "rt", encoding="latin-1") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            rows.append((int(p[1]), int(p[2]), int(p[3]), p[4] if len(p) > 4 else ""))
    return rows


def test_tunnel_fixture_shape():
    arena, desc, sources = load()
    assert len(desc) == MANIFEST["packets"] == len(load_ref("t0"))
    assert MANIFEST["counts"]["t0"]["fingerprints"] > 200
    assert MANIFEST["counts"]["none"]["fingerprints"] < MANIFEST["counts"]["t0"]["fingerprints"]


@pytest.mark.parametrize("cfg", ["gre", "vxlan", "geneve", "select=tls,gre;format=tls/1"])
def test_tunnel_selection_parses(cfg):
    sel, _ = mercury_amd.parse_filter(cfg)
    assert sel


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["t0", "t1", "vx", "none"])
def test_tunnels_vs_reference(key):
    arena, desc, sources = load()
    ctx = mercury_amd.Context(MANIFEST["configs"][key], device=0)
    try:
        rec, fp = ctx.process_host(arena, desc)
    finally:
        ctx.close()
    fps = mercury_amd.fingerprints(rec, fp)
    bad = []
    for i, (emit, t, trunc, s) in enumerate(load_ref(key)):
        g_emit = int(rec["flags"][i] & 1)
        g = (g_emit, int(rec["fp_type"][i]), int((rec["flags"][i] >> 1) & 1) & g_emit, fps[i])
        if g != (emit, t, trunc, s):
            bad.append((i, str(sources[i]), g[:3], (emit, t, trunc)))
    assert not bad, f"{len(bad)} mismatches, first: {bad[:5]}"
    # records reached through a tunnel carry MFP_FLAG_ENCAP, and only
    # IP-in-IP chains are regular (the JSON writer rebuilds their entries)
    enc = (rec["flags"] & 32) != 0
    assert enc.sum() >= (50 if key in ("t0", "t1") else 1)


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["t0", "vx", "none"])
def test_tunnel_json_vs_reference(key):
    """The whole write_json text of every packet of the tunnel stream:
    "encapsulations" arrays of GRE (over IP and UDP 4754), VXLAN, Geneve and
    IP-in-IP levels (outer IPv6 extension headers included), rebuilt by the
    host walk of mfp_encap.hpp, byte-identical to the reference; nothing is
    skipped."""
    from tests import test_json
    arena, desc, sources = load()
    ctx = mercury_amd.Context(MANIFEST["configs"][key], device=0)
    try:
        rec, fp = ctx.process_host(arena, desc)
    finally:
        ctx.close()
    lines, skipped = mercury_amd.write_json(arena, desc, rec, fp, ts_ns=np.full(len(desc), test_json.TS, np.uint64),
                                            threads=2)
    test_json._check(lines, test_json._golden_lines(f"tunnel_json_{key}.txt.gz"), skipped)
    assert skipped == 0
