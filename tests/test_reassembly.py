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
    with gzip.open(os.path.join(GOLD, f"reasm_{key}_fp.tsv.gz" if key == "timed" else f"reasm_fp_{key}.tsv.gz"), "rt",
                   encoding="latin-1") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            rows.append((int(p[1]), int(p[2]), int(p[3]), p[4] if len(p) > 4 else ""))
    with gzip.open(os.path.join(GOLD, f"reasm_{key}_props.txt.gz" if key == "timed" else f"reasm_props_{key}.txt.gz"),
                   "rt", encoding="latin-1") as f:
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
    test_json._check(lines, test_json._golden_lines(f"reasm_json_{key}.txt.gz"), skipped)


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
    test_json._check(lines, test_json._golden_lines("reasm_json_an.txt.gz"), skipped)
    assert MANIFEST["counts"]["an"]["analysis_objects"] > 50


# ---------------------------------------------------------------------------
# the analysis_context path with reassembly (analyze_ip_packet
# pkt_proc.cc:1597-1662; mfp_process_batch_reassembly_context) and the
# per-packet flow_state_pkts_needed (mercury_packet_processor_more_pkts_needed)
# ---------------------------------------------------------------------------
def load_ref_anr(name):
    rows = []
    with gzip.open(os.path.join(GOLD, name), "rt", encoding="latin-1") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            rows.append(dict(valid=int(p[1]), fp_type=int(p[2]), status=int(p[3]), process=p[4], score=float(p[5]),
                             malware=int(p[6]), p_malware=float(p[7]), more=int(p[8]), fp=p[9] if len(p) > 9 else ""))
    return rows


def load_timed():
    z = np.load(os.path.join(GOLD, "reasm_timed_packets.npz"))
    return z["arena"], z["desc"], z["ts"].astype(np.uint64) * 10**9


def an_config():
    return MANIFEST["an_config"] + f";resources={os.path.join(GOLD, 'resources-test.tgz')};analysis"


def run_an_path(arena, desc, ts_ns, chunk=None):
    ctx = mercury_amd.Context(an_config(), device=0, mode=api.MODE_ANALYSIS)
    try:
        n = len(desc)
        chunk = chunk or max(n, 1)
        out = dict(rec=[], fps=[], an=[], more=[], names=[])
        for lo in range(0, n, chunk):
            rec, fp, props, a2, d2, an, ap, more = ctx.analyze_host_reassembly(arena, desc[lo:lo + chunk],
                                                                             ts_ns=ts_ns[lo:lo + chunk])
            out["rec"].append(rec)
            out["fps"] += mercury_amd.fingerprints(rec, fp)
            out["an"].append(an)
            out["more"].append(more)
            out["names"] += [ctx.process_name(int(p)) if an["flags"][k] & 1 else ""
                             for k, p in enumerate(an["process"])]
        return (np.concatenate(out["rec"]), out["fps"], np.concatenate(out["an"]), np.concatenate(out["more"]),
                out["names"])
    finally:
        ctx.close()


def compare_an_path(got, ref):
    rec, fps, an, more, names = got
    bad = []
    for i, r in enumerate(ref):
        valid = int(an["flags"][i] & 1)
        g = (valid, int(more[i]))
        w = (r["valid"], r["more"])
        if valid and r["valid"]:
            g += (int(rec["fp_type"][i]), fps[i], int(an["status"][i]), names[i], float(an["score"][i]),
                  int(bool(an["flags"][i] & 2)), float(an["malware_prob"][i]) if an["flags"][i] & 4 else 0.0)
            w += (r["fp_type"], r["fp"], r["status"], r["process"], r["score"], r["malware"], r["p_malware"])
        if g != w:
            bad.append((i, g[:6], w[:6]))
    return bad


def test_an_path_fixture_shape():
    ref = load_ref_anr("reasm_an_r0.tsv.gz")
    assert len(ref) == MANIFEST["packets"]
    c = MANIFEST["counts"]["an_path"]
    assert c["valid"] > 100 and c["more"] > 100
    a, d, ts = load_timed()
    assert len(d) == MANIFEST["counts"]["timed"]["packets"] == len(load_ref_anr("reasm_timed_an.tsv.gz"))
    assert len(set(ts.tolist())) > 50   # per-packet capture times, some going backwards
    assert (np.diff(ts.astype(np.int64)) < 0).any()


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [None, 97])
def test_analysis_path_reassembly_vs_reference(chunk):
    """valid / type / status / process / score / malware / more_pkts_needed per
    packet, equal to the reference's analysis_context path over the 7 538-packet
    stream (one batch, and batches of 97 with the state carried over)."""
    arena, desc = load_stream()
    got = run_an_path(arena, desc, np.full(len(desc), TS, np.uint64), chunk=chunk)
    bad = compare_an_path(got, load_ref_anr("reasm_an_r0.tsv.gz"))
    assert not bad, f"{len(bad)} mismatches, first: {bad[:4]}"


@pytest.mark.gpu
def test_timed_stream_vs_reference():
    """Per-packet capture times: flows stalled past the 15 s timeout, time going
    backwards, SYN/RST/FIN segments with data, other traffic between segments
    -- write_json records, reassembly_properties and the whole JSON text, then
    the analysis_context path with more_pkts_needed."""
    from tests import test_json
    arena, desc, ts = load_timed()
    ctx = mercury_amd.Context(MANIFEST["configs"]["r0"], device=0)
    try:
        rec, fp, props, arena2, desc2 = ctx.process_host_reassembly(arena, desc, ts_ns=ts)
    finally:
        ctx.close()
    ref, ref_props = load_ref("timed")
    bad = compare(rec, mercury_amd.fingerprints(rec, fp), props, ref, ref_props)
    assert not bad, f"{len(bad)} write_json mismatches, first: {bad[:4]}"
    lines, skipped = mercury_amd.write_json(arena2, desc2, rec, fp, ts_ns=ts, threads=2, props=props)
    test_json._check(lines, test_json._golden_lines("reasm_timed_json.txt.gz"), skipped)
    got = run_an_path(arena, desc, ts)
    bad = compare_an_path(got, load_ref_anr("reasm_timed_an.tsv.gz"))
    assert not bad, f"{len(bad)} analysis-path mismatches, first: {bad[:4]}"


@pytest.mark.gpu
def test_libmerc_more_pkts_needed():
    """mercury_packet_processor_get_analysis_context_linktype +
    mercury_packet_processor_more_pkts_needed, packet by packet through the
    libmerc shim (its processor's own reassembler), over the timed stream and
    the synthetic part of the main stream."""
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
    f = lib.mercury_packet_processor_get_analysis_context_linktype
    f.restype = vp
    f.argtypes = [vp, vp, ctypes.c_size_t, ctypes.POINTER(Timespec), ctypes.c_uint16]
    lib.mercury_packet_processor_more_pkts_needed.restype = ctypes.c_bool
    lib.mercury_packet_processor_more_pkts_needed.argtypes = [vp]
    lib.analysis_context_get_fingerprint_status.restype = ctypes.c_int
    lib.analysis_context_get_fingerprint_status.argtypes = [vp]
    lib.analysis_context_get_fingerprint_string.restype = ctypes.c_char_p
    lib.analysis_context_get_fingerprint_string.argtypes = [vp]
    res = os.path.join(GOLD, "resources-test.tgz").encode()
    for name, (arena, desc, ts), first in [
            ("reasm_timed_an.tsv.gz", load_timed(), 0),
            ("reasm_an_r0.tsv.gz", load_stream() + (np.full(MANIFEST["packets"], TS, np.uint64),),
             MANIFEST["pcap_packets"])]:
        cfg = test_json._LibmercConfig()
        cfg.packet_filter_cfg = MANIFEST["an_config"].encode()
        cfg.resources = res
        cfg.do_analysis = True
        mc = lib.mercury_init(ctypes.byref(cfg), 0)
        assert mc
        p = lib.mercury_packet_processor_construct(mc)
        ref = load_ref_anr(name)
        bad = []
        for i in range(first, len(desc)):
            off, ln, lt = int(desc[i]["offset"]), int(desc[i]["caplen"]), int(desc[i]["linktype"])
            pkt = ctypes.create_string_buffer(arena[off:off + ln].tobytes() + bytes(16))
            t = Timespec(int(ts[i]) // 10**9, 0)
            ac = f(p, pkt, ln, ctypes.byref(t), lt)
            g = (int(bool(ac)), int(lib.mercury_packet_processor_more_pkts_needed(p)))
            w = (ref[i]["valid"], ref[i]["more"])
            if ac and ref[i]["valid"]:
                g += (lib.analysis_context_get_fingerprint_status(ac),
                      lib.analysis_context_get_fingerprint_string(ac).decode("latin-1"))
                w += (ref[i]["status"], ref[i]["fp"])
            if g != w:
                bad.append((i, g[:3], w[:3]))
        lib.mercury_packet_processor_destruct(p)
        lib.mercury_finalize(mc)
        assert not bad, f"{name}: {len(bad)} mismatches, first {bad[:3]}"


@pytest.mark.gpu
def test_tunnelled_reassembly_json_vs_reference():
    """ClientHellos split inside IP-in-IP, GRE, VXLAN and Geneve: the
    reassembled message's frame keeps the completing packet's outer headers,
    so its record carries the reference's "encapsulations" (pkt_proc.cc:1231-1233)."""
    from tests import test_json
    z = np.load(os.path.join(GOLD, "reasm_tunnel_packets.npz"))
    arena, desc = z["arena"], z["desc"]
    ts = np.full(len(desc), TS, np.uint64)
    ctx = mercury_amd.Context(MANIFEST["tunnel_config"], device=0)
    try:
        rec, fp, props, arena2, desc2 = ctx.process_host_reassembly(arena, desc, ts_ns=ts)
    finally:
        ctx.close()
    lines, skipped = mercury_amd.write_json(arena2, desc2, rec, fp, ts_ns=ts, threads=2, props=props)
    test_json._check(lines, test_json._golden_lines("reasm_tunnel_json.txt.gz"), skipped)
    assert int((props & 1).sum()) == MANIFEST["counts"]["tunnel"]["reassembled"] == 18
