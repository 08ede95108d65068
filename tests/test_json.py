"""JSON records (mfp_write_json_batch, mercury_amd/csrc/mfp_json.cpp) against
the reference's own write_json text (stateful_pkt_proc::write_json,
src/libmerc/pkt_proc.cc:1157-1253), committed by tests/golden/make_golden_json.py.

* CPU: the writer alone, driven by records built from the crafted packets'
  known fields (no GPU walk): UTF-8/JSON escaping, the IPv6 zero-run quirk,
  certificate lists and roles, truncation, IPv4 digit counts.
* GPU: records from the HIP walk -> writer, byte-identical to the reference
  on the crafted packets, the packets of the reference's own test pcaps and
  a synthetic mixed batch.  Bar: every emitted line byte-identical,
  "encapsulations" arrays included (IP-in-IP, GRE, VXLAN, Geneve; outer IPv6
  extension headers); nothing is skipped.
"""
import gzip
import json
import os
import struct

import numpy as np
import pytest

import mercury_amd
from mercury_amd.api import FP_TYPE_NAMES, RECORD_DTYPE
from tests import synth

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CONTRACT = "tls,dtls,ssh,http,tcp,tcp.syn_ack"
TS = 1700000000 * 10**9          # the reference driver's fixed timestamp
ENCAP = 32                       # MFP_FLAG_ENCAP


def _crafted():
    z = np.load(os.path.join(GOLD, "json_crafted.npz"))
    blob = z["json"].tobytes()
    ends = [0] + [int(e) for e in z["json_end"]]
    lines = [blob[ends[i]:ends[i + 1]] for i in range(len(ends) - 1)]
    return z["arena"], z["desc"], z["fields"], lines


def _golden_lines(name):
    with gzip.open(os.path.join(GOLD, name), "rb") as f:
        return f.read().split(b"\n")[:-1]


def _check(lines, gold, skipped):
    """Every line byte-identical; nothing skipped."""
    assert len(lines) == len(gold)
    for i, (got, want) in enumerate(zip(lines, gold)):
        exp = want + b"\n" if want else b""
        assert got == exp, (i, got[:300], exp[:300])
    assert skipped == 0


def test_writer_crafted_records():
    """CPU: records assembled from the crafted packets' construction fields."""
    arena, desc, fields, gold = _crafted()
    n = len(desc)
    rec = np.zeros(n, RECORD_DTYPE)
    fp_blob = b""
    for i in range(n):
        msg, flags, so, sl, uo, ul = (int(x) for x in fields[i])
        off = int(desc[i]["offset"])
        pkt = arena[off:off + int(desc[i]["caplen"])].tobytes()
        ip = 14 + (20 if flags & ENCAP else 0)
        ver = pkt[ip] >> 4
        l4 = ip + (20 if ver == 4 else 40)
        sport, dport = struct.unpack(">HH", pkt[l4:l4 + 4])
        obj = json.loads(gold[i])
        fps = obj.get("fingerprints", {})
        fp_type, fp = 0, b""
        if fps:
            (name, s), = fps.items()
            fp_type, fp = FP_TYPE_NAMES.index(name), s.encode()
        levels = 1 if flags & ENCAP else 0          # one IPv4 outer header
        rec[i] = (len(fp_blob), len(fp), fp_type, msg, flags, 0, so, sl, uo, ul, sport, dport,
                  ip | (ver << 16) | (levels << 20))
        fp_blob += fp
    lines, skipped = mercury_amd.write_json(arena, desc, rec, fp_blob, ts_ns=np.full(n, TS, np.uint64))
    _check(lines, gold, skipped)


def test_writer_threads_and_timestamps():
    """CPU: threaded output equals single-threaded; timestamps as sec.usec."""
    arena, desc, fields, gold = _crafted()
    n = len(desc)
    rec = np.zeros(n, RECORD_DTYPE)
    for i in range(n):
        msg, flags, so, sl, uo, ul = (int(x) for x in fields[i])
        rec[i] = (0, 0, 0, msg, flags & ~ENCAP, 0, so, sl, uo, ul, 1, 2, 14 | (4 << 16))
    # replicate to cross the writer's per-thread split
    reps = 400
    big_desc = np.tile(desc, reps)
    big_rec = np.tile(rec, reps)
    ts = (np.arange(n * reps, dtype=np.uint64) * np.uint64(1_234_567) + np.uint64(TS))
    one, s1 = mercury_amd.write_json(arena, big_desc, big_rec, b"", ts_ns=ts, threads=1)
    many, s8 = mercury_amd.write_json(arena, big_desc, big_rec, b"", ts_ns=ts, threads=8)
    assert one == many and s1 == s8 == 0
    for i in (0, 1, 777, n * reps - 1):
        t = int(ts[i])
        assert one[i].endswith(b'"event_start":%d.%06d}\n' % (t // 10**9, t % 10**9 // 1000))


@pytest.mark.gpu
def test_json_crafted_device():
    arena, desc, _, gold = _crafted()
    ctx = mercury_amd.Context(CONTRACT, device=0)
    rec, fp = ctx.process_host(arena, desc)
    lines, skipped = mercury_amd.write_json(arena, desc, rec, fp, ts_ns=np.full(len(desc), TS, np.uint64))
    _check(lines, gold, skipped)
    ctx.close()


@pytest.mark.gpu
def test_json_reference_pcaps_device():
    with np.load(os.path.join(GOLD, "ref_packets.npz")) as z:
        arena, desc = z["arena"], z["desc"]
    gold = _golden_lines("json_ref.txt.gz")
    ctx = mercury_amd.Context(CONTRACT, device=0)
    rec, fp = ctx.process_host(arena, desc)
    lines, skipped = mercury_amd.write_json(arena, desc, rec, fp, ts_ns=np.full(len(desc), TS, np.uint64),
                                            threads=4)
    _check(lines, gold, skipped)
    ctx.close()


@pytest.mark.gpu
def test_json_synthetic_device():
    arena, desc = synth.batch(4000, seed=0x5EED0003)
    gold = _golden_lines("json_synth.txt.gz")
    ctx = mercury_amd.Context(CONTRACT, device=0)
    rec, fp = ctx.process_host(arena, desc)
    lines, skipped = mercury_amd.write_json(arena, desc, rec, fp, ts_ns=np.full(len(desc), TS, np.uint64))
    _check(lines, gold, skipped)
    assert sum(1 for l in lines if l) > 3000
    ctx.close()


class _LibmercConfig(__import__("ctypes").Structure):
    """struct libmerc_config (include/mercury_amd_libmerc.h, libmerc.h:109-154)."""
    import ctypes as _c
    _fields_ = [("dns_json_output", _c.c_bool), ("certs_json_output", _c.c_bool), ("metadata_output", _c.c_bool),
                ("do_analysis", _c.c_bool), ("do_stats", _c.c_bool), ("report_os", _c.c_bool),
                ("output_tcp_initial_data", _c.c_bool), ("output_udp_initial_data", _c.c_bool),
                ("resources", _c.c_char_p), ("enc_key", _c.c_void_p), ("key_type", _c.c_int),
                ("packet_filter_cfg", _c.c_char_p), ("fp_proc_threshold", _c.c_float),
                ("proc_dst_threshold", _c.c_float), ("max_stats_entries", _c.c_size_t)]


@pytest.mark.gpu
def test_libmerc_write_json_linktype_device():
    """mercury_packet_processor_write_json_linktype per packet, as the
    reference's libmerc fixture calls it (unit_tests/libmerc_fixture.cc)."""
    import ctypes
    lib = mercury_amd.load_library()
    vp = ctypes.c_void_p

    class Timespec(ctypes.Structure):
        _fields_ = [("tv_sec", ctypes.c_long), ("tv_nsec", ctypes.c_long)]

    lib.mercury_init.restype = vp
    lib.mercury_init.argtypes = [ctypes.POINTER(_LibmercConfig), ctypes.c_int]
    lib.mercury_packet_processor_construct.restype = vp
    lib.mercury_packet_processor_construct.argtypes = [vp]
    lib.mercury_packet_processor_destruct.argtypes = [vp]
    lib.mercury_finalize.argtypes = [vp]
    f = lib.mercury_packet_processor_write_json_linktype
    f.restype = ctypes.c_size_t
    f.argtypes = [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, ctypes.POINTER(Timespec), ctypes.c_uint16]
    cfg = _LibmercConfig()
    cfg.packet_filter_cfg = CONTRACT.encode()
    mc = lib.mercury_init(ctypes.byref(cfg), 0)
    assert mc
    p = lib.mercury_packet_processor_construct(mc)
    arena, desc, _, gold = _crafted()
    buf = ctypes.create_string_buffer(1 << 16)
    for i in range(len(desc)):
        off, ln = int(desc[i]["offset"]), int(desc[i]["caplen"])
        pkt = ctypes.create_string_buffer(arena[off:off + ln].tobytes() + bytes(16))
        ts = Timespec(1700000000, 0)
        n = f(p, buf, len(buf), pkt, ln, ctypes.byref(ts), 1)
        want = gold[i] + b"\n" if gold[i] else b""
        assert buf.raw[:n] == want, i
        # a buffer one byte short of the record: nothing written (pkt_proc.cc:1249-1253)
        if want:
            assert f(p, buf, len(want), pkt, ln, ctypes.byref(ts), 1) == 0
    # a zero timestamp is filled in with tsc_clock's seconds since the counter
    # started (pkt_proc.cc:1086-1089; here CLOCK_MONOTONIC), tv_nsec untouched
    import time
    off, ln = int(desc[0]["offset"]), int(desc[0]["caplen"])
    pkt = ctypes.create_string_buffer(arena[off:off + ln].tobytes() + bytes(16))
    ts = Timespec(0, 123)
    f(p, buf, len(buf), pkt, ln, ctypes.byref(ts), 1)
    assert abs(ts.tv_sec - time.monotonic()) < 3 and ts.tv_nsec == 123
    lib.mercury_packet_processor_destruct(p)
    lib.mercury_finalize(mc)


def test_libmerc_init_filter_forms():
    """CPU: mercury_init accepts the bare protocol list and the key=value
    form (global_config.h:148-152), the reference's default selection (empty =
    "all", global_config.h:248: the records of protocols outside this path
    are not written) and, as the reference does, a list with an unknown
    protocol (set_protocols logs it and stops there, global_config.h:246-275;
    the constructor ignores its result, :151)."""
    import ctypes
    lib = mercury_amd.load_library()
    lib.mercury_init.restype = ctypes.c_void_p
    lib.mercury_init.argtypes = [ctypes.POINTER(_LibmercConfig), ctypes.c_int]
    lib.mercury_finalize.argtypes = [ctypes.c_void_p]
    for filt, ok in ((CONTRACT, True), ("select=tls,http;format=tls/1", True), ("", True), ("all", True),
                     ("nosuchproto", True)):
        cfg = _LibmercConfig()
        cfg.packet_filter_cfg = filt.encode()
        mc = lib.mercury_init(ctypes.byref(cfg), 0)
        assert bool(mc) == ok, filt
        if mc:
            lib.mercury_finalize(mc)
