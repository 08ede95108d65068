"""TCP reassembly: mfp_process_batch_reassembly
(mercury_amd/csrc/mfp_reassembly.cpp) -- the device walk, the flow table of
the reference's tcp_reassembler (reassembly.hpp:140-900) applied in stream
order on the host, and the reassembled messages fingerprinted by the device --
against the REFERENCE run with "reassembly" configured.

Expected values: tests/golden/make_golden_reasm.py, the reference libmerc
(oracle/_ref) over one stream: the 6 984 packets of the reference's unit-test
pcaps, then the synthetic streams of tests/reasm_synth.py (splits in order and
out of order, duplicates, the four overlap kinds, missing segments, more than
20 segments, sequence wrap, sequence 0, interleaved flows, IPv6, messages over
the 8 KiB buffer, SSH banner + KEXINIT, TLS ServerHello + Certificate).
Bar: per packet identical emit / fp type / truncation, byte-identical
fingerprints, and the same "reassembly_properties" object.  The stream runs
as one batch and as batches of 97 packets (flow state carries over).
"""
import ctypes
import gzip
import json
import os

import numpy as np
import pytest

import mercury_amd
from mercury_amd import api
from tests import pcaplib

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "reasm_manifest.json")))
TS = 1700000000 * 10**9


def load_stream():
    z = np.load(os.path.join(GOLD, "ref_packets.npz"))
    pk = [(int(d["linktype"]), bytes(z["arena"][int(d["offset"]):int(d["offset"]) + int(d["caplen"])]))
          for d in z["desc"]]
    s = np.load(os.path.join(GOLD, "reasm_packets.npz"))
    syn = [(1, bytes(s["arena"][int(d["offset"]):int(d["offset"]) + int(d["caplen"])])) for d in s["desc"]]
    return pcaplib.make_batch(pk + syn)


def load_ref(key):
    rows = []
    with gzip.open(os.path.join(GOLD, f"reasm_fp_{key}.tsv.gz"), "rt", encoding="latin-1") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            rows.append((int(p[1]), int(p[2]), int(p[3]), p[4] if len(p) > 4 else ""))
    with gzip.open(os.path.join(GOLD, f"reasm_props_{key}.txt.gz"), "rt", encoding="latin-1") as f:
        props = f.read().split("\n")[:len(rows)]
    return rows, props


def props_text(bits, truncated):
    """The record's reassembly_properties object (write_reassembly_properties
    reassembly.hpp:1231-1247, tcp_reassembler::write_json :860-880)."""
    if bits & 1:
        keys = ["reassembled"] + [n for k, n in enumerate(api.REASM_FLAGS) if bits >> (1 + k) & 1] + \
               [n for k, n in enumerate(api.REASM_OVERLAPS) if bits >> (8 + k) & 1]
        return "{" + ",".join(f'"{k}":true' for k in keys) + "}"
    return '{"truncated":true}' if truncated else ""


def test_fixture_shape():
    arena, desc = load_stream()
    assert len(desc) == MANIFEST["packets"]
    c = MANIFEST["counts"]["r0"]
    assert c["reassembled"] > 100 and c["overlaps"] > 5


def test_config():
    lib = mercury_amd.load_library()
    sel, fmt = ctypes.c_uint32(), ctypes.c_uint32()
    assert lib.mfp_parse_filter(b"select=tls;reassembly", ctypes.byref(sel), ctypes.byref(fmt)) == 0
    assert lib.mfp_parse_filter(b"select=tls;tcp-reassembly", ctypes.byref(sel), ctypes.byref(fmt)) == 0


def run(cfg, arena, desc, chunk=None):
    ctx = mercury_amd.Context(cfg, device=0)
    try:
        n = len(desc)
        chunk = chunk or n
        recs, fps, props = [], [], []
        for lo in range(0, n, chunk):
            d = desc[lo:lo + chunk]
            rec, fp, pr, _, _ = ctx.process_host_reassembly(arena, d, ts_ns=np.full(len(d), TS, np.uint64))
            recs.append(rec)
            fps += mercury_amd.fingerprints(rec, fp)
            props.append(pr)
        return np.concatenate(recs), fps, np.concatenate(props)
    finally:
        ctx.close()


def compare(rec, fps, props, ref, ref_props):
    bad = []
    for i, (emit, t, trunc, s) in enumerate(ref):
        g_emit = int(rec["flags"][i] & 1)
        g_trunc = int((rec["flags"][i] >> 1) & 1) & g_emit
        got = (g_emit, int(rec["fp_type"][i]), fps[i], props_text(int(props[i]), g_trunc) if g_emit else "")
        want = (emit, t, s, ref_props[i])
        if got != want:
            bad.append((i, got[:2] + (got[3],), want[:2] + (want[3],)))
    return bad


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["r0", "r1"])
def test_reassembly_vs_reference(key):
    arena, desc = load_stream()
    rec, fps, props = run(MANIFEST["configs"][key], arena, desc)
    ref, ref_props = load_ref(key)
    bad = compare(rec, fps, props, ref, ref_props)
    assert not bad, f"{len(bad)} mismatches, first: {bad[:4]}"
    assert int((props & 1).sum()) == MANIFEST["counts"][key]["reassembled"]


@pytest.mark.gpu
def test_reassembly_across_batches():
    arena, desc = load_stream()
    rec, fps, props = run(MANIFEST["configs"]["r0"], arena, desc, chunk=97)
    ref, ref_props = load_ref("r0")
    bad = compare(rec, fps, props, ref, ref_props)
    assert not bad, f"{len(bad)} mismatches, first: {bad[:4]}"


@pytest.mark.gpu
def test_reassembly_refusals():
    with pytest.raises(mercury_amd.MercuryAmdError):
        mercury_amd.Context("select=tls,quic;reassembly", device=0)
    with pytest.raises(mercury_amd.MercuryAmdError):
        mercury_amd.Context("select=tls;reassembly", device=0, mode=api.MODE_ANALYSIS)


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["r0", "r1"])
def test_reassembly_json_vs_reference(key):
    """The whole JSON line of every packet (mfp_write_json_batch_reassembly over
    the reassembled frames: server names, flow keys, the reassembler's
    properties) equals the reference's write_json text."""
    from tests import test_json
    arena, desc = load_stream()
    ctx = mercury_amd.Context(MANIFEST["configs"][key], device=0)
    try:
        rec, fp, props, arena2, desc2 = ctx.process_host_reassembly(arena, desc,
                                                                    ts_ns=np.full(len(desc), TS, np.uint64))
    finally:
        ctx.close()
    lines, skipped = mercury_amd.write_json(arena2, desc2, rec, fp, ts_ns=np.full(len(desc), TS, np.uint64),
                                            threads=4, props=props)
    test_json._check(lines, test_json._golden_lines(f"reasm_json_{key}.txt.gz"), skipped, allow_skip=True)


@pytest.mark.gpu
def test_libmerc_write_json_with_reassembly():
    """mercury_packet_processor_write_json_linktype with "reassembly" in the
    configuration: the processor's own reassembler, packet by packet, gives
    the reference's text for the synthetic streams."""
    from tests import test_json
    lib = mercury_amd.load_library()
    vp = ctypes.c_void_p

    class Timespec(ctypes.Structure):
        _fields_ = [("tv_sec", ctypes.c_long), ("tv_nsec", ctypes.c_long)]

    lib.mercury_init.restype = vp
    lib.mercury_init.argtypes = [ctypes.POINTER(test_json._LibmercConfig), ctypes.c_int]
    lib.mercury_packet_processor_construct.restype = vp
    lib.mercury_packet_processor_construct.argtypes = [vp]
    lib.mercury_packet_processor_destruct.argtypes = [vp]
    lib.mercury_finalize.argtypes = [vp]
    f = lib.mercury_packet_processor_write_json_linktype
    f.restype = ctypes.c_size_t
    f.argtypes = [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, ctypes.POINTER(Timespec), ctypes.c_uint16]
    cfg = test_json._LibmercConfig()
    cfg.packet_filter_cfg = MANIFEST["configs"]["r0"].encode()
    mc = lib.mercury_init(ctypes.byref(cfg), 0)
    assert mc
    p = lib.mercury_packet_processor_construct(mc)
    arena, desc = load_stream()
    gold = test_json._golden_lines("reasm_json_r0.txt.gz")
    buf = ctypes.create_string_buffer(1 << 16)
    first = MANIFEST["pcap_packets"]           # the synthetic streams follow the pcap packets
    bad = []
    for i in range(len(desc)):
        off, ln, lt = int(desc[i]["offset"]), int(desc[i]["caplen"]), int(desc[i]["linktype"])
        pkt = ctypes.create_string_buffer(arena[off:off + ln].tobytes() + bytes(16))
        ts = Timespec(1700000000, 0)
        n = f(p, buf, len(buf), pkt, ln, ctypes.byref(ts), lt)
        want = gold[i] + b"\n" if gold[i] else b""
        if i >= first and buf.raw[:n] != want:
            bad.append((i, buf.raw[:n][:200], want[:200]))
    lib.mercury_packet_processor_destruct(p)
    lib.mercury_finalize(mc)
    assert not bad, f"{len(bad)} mismatches, first {bad[:2]}"


@pytest.mark.gpu
def test_reassembly_with_analysis_json_vs_reference():
    """--analysis with reassembly: the reassembled ClientHellos classified in
    their completing packets' places (resources-test.tgz), the whole JSON text
    equal to the reference's."""
    from tests import test_json
    arena, desc = load_stream()
    cfg = MANIFEST["configs"]["r0"] + f";resources={os.path.join(GOLD, 'resources-test.tgz')};analysis"
    ctx = mercury_amd.Context(cfg, device=0)
    try:
        rec, fp, props, arena2, desc2, an, ap = ctx.process_host_reassembly(
            arena, desc, ts_ns=np.full(len(desc), TS, np.uint64), analysis=True)
        lines, skipped = mercury_amd.write_json(arena2, desc2, rec, fp, ts_ns=np.full(len(desc), TS, np.uint64),
                                                threads=4, ctx=ctx, analysis=an, attr_prob=ap, props=props)
    finally:
        ctx.close()
    test_json._check(lines, test_json._golden_lines("reasm_json_an.txt.gz"), skipped, allow_skip=True)
    assert MANIFEST["counts"]["an"]["analysis_objects"] > 50
