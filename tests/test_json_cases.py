"""JSON text and destination-context strings on the parity CASES
(tests/cases.py) against the REFERENCE (oracle/_ref/merc_ref_drv modes
"json" and "meta", committed by tests/golden/make_golden_cases.py):

* the 40 000 fuzzed packets per format, the reference's fuzzing corpus, the
  edge cases (empty, truncated at every header, 65 535/70 000-byte frames) --
  so the JSON writer is pinned wherever the fingerprints are;
* hello_meta: crafted ClientHellos whose JSON and analysis context depend on
  which extension the reference reads -- duplicate / empty / malformed
  server_name extensions (write_json prints the FIRST, tls.h:1052-1080; the
  analysis context keeps the LAST, tls.h:1316-1345), QUIC transport
  parameters over TCP with user agents (tls.h:1264-1311; the destination
  context takes the user agent from the draft type only, tls.h:1346-1355),
  a DTLS version inside a TLS record (tls.h:1823-1844), a soft-failed
  extension list.

Bar: every line byte-identical (nothing skipped); the accessors'
strings identical, NULL where the reference returns NULL.
"""
import ctypes

import numpy as np
import pytest

import mercury_amd
from tests import cases
from tests.test_gpu_parity import cfg_string
from tests.test_json import TS, _LibmercConfig

JSON_RUNS = [(name, fmt) for name, (_, runs) in cases.CASES.items() for fmt, mode in runs if mode == "json"]


def test_json_runs_registered():
    """CPU: every JSON golden the generator lists is present and has one line per packet."""
    import json
    import os
    man = json.load(open(os.path.join(cases.GOLD, "cases", "manifest.json")))["cases"]
    assert {"fuzz0", "fuzz1", "fuzz2", "edge", "corpus", "hello_meta"} <= {n for n, _ in JSON_RUNS}
    for name, fmt in JSON_RUNS:
        assert f"json{fmt}" in man[name]["runs"]
        assert len(cases.load_json_golden(name, fmt)) == man[name]["packets"]
    meta = cases.load_meta_golden("hello_meta")
    assert len(meta) == man["hello_meta"]["packets"]
    # the golden shows the first/last split the test is about
    gold = cases.load_json_golden("hello_meta", 0)
    assert b'"server_name":"first.example"' in gold[0] and meta[0][1] == b"second.example"


@pytest.mark.gpu
@pytest.mark.parametrize("name,fmt", JSON_RUNS)
def test_json_vs_reference(name, fmt):
    arena, desc = cases.batch(cases.CASES[name][0]())
    want = cases.load_json_golden(name, fmt)
    ctx = mercury_amd.Context(cfg_string(fmt), device=0)
    try:
        rec, fp = ctx.process_host(arena, desc)
    finally:
        ctx.close()
    lines, skipped = mercury_amd.write_json(arena, desc, rec, fp, ts_ns=np.full(len(desc), TS, np.uint64), threads=4)
    bad = [i for i, (g, w) in enumerate(zip(lines, want)) if g != (w + b"\n" if w else b"")]
    assert len(lines) == len(want)
    assert not bad, (f"{len(bad)} of {len(want)} lines differ; first {bad[:8]}; packet {bad[0]}:\n"
                     f"got  {lines[bad[0]][:600]!r}\nwant {want[bad[0]][:600]!r}")
    assert skipped == 0
    assert sum(1 for w in want if w) > (10 if name != "fuzz0" else 10000)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_hello_meta_fingerprints(fmt):
    from tests.test_gpu_parity import _vs_reference
    bad, rec = _vs_reference("hello_meta", fmt)
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"


@pytest.mark.gpu
def test_hello_meta_analysis_context():
    """The libmerc shim's analysis_context_get_server_name / _user_agent per
    packet (libmerc.cc:276-288) equal the reference's."""
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
    get = lib.mercury_packet_processor_get_analysis_context_linktype
    get.restype = vp
    get.argtypes = [vp, vp, ctypes.c_size_t, ctypes.POINTER(Timespec), ctypes.c_uint16]
    for f in (lib.analysis_context_get_server_name, lib.analysis_context_get_user_agent):
        f.restype = ctypes.c_char_p
        f.argtypes = [vp]
    cfg = _LibmercConfig()
    cfg.packet_filter_cfg = cfg_string(1).encode()
    cfg.resources = cases.META_RESOURCES.encode()
    cfg.do_analysis = True
    mc = lib.mercury_init(ctypes.byref(cfg), 0)
    assert mc
    p = lib.mercury_packet_processor_construct(mc)
    want = cases.load_meta_golden("hello_meta")
    pk = cases.hello_meta_case()
    bad = []
    for i, (lt, b) in enumerate(pk):
        buf = ctypes.create_string_buffer(b + bytes(16))
        ts = Timespec(1700000000, 0)
        ac = get(p, buf, len(b), ctypes.byref(ts), lt)
        got = (0, None, None) if not ac else (1, lib.analysis_context_get_server_name(ac),
                                              lib.analysis_context_get_user_agent(ac))
        if got != want[i]:
            bad.append((i, got, want[i]))
    lib.mercury_packet_processor_destruct(p)
    lib.mercury_finalize(mc)
    assert not bad, f"{len(bad)} mismatches: {bad[:6]}"


@pytest.mark.gpu
@pytest.mark.parametrize("name,limit", [("edge", None), ("corpus", None), ("fuzz0", 3000)])
def test_shim_write_json_per_packet_vs_reference(name, limit):
    """mercury_packet_processor_write_json_linktype packet by packet from 8
    threads at once (one processor each: their calls are combined into
    concurrent small batches, mfp_process_small_pinned; frames past the
    walker's LDS stage -- the 65 535/70 000-byte edge cases -- are walked from
    memory by their own wave): every record equals the reference's write_json
    line for that packet."""
    from concurrent.futures import ThreadPoolExecutor
    arena, desc = cases.batch(cases.CASES[name][0]())
    want = cases.load_json_golden(name, 0)
    n = len(desc) if limit is None else min(limit, len(desc))
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
    cfg.packet_filter_cfg = cfg_string(0).encode()
    mc = lib.mercury_init(ctypes.byref(cfg), 0)
    assert mc
    threads = 8

    def work(t):
        p = lib.mercury_packet_processor_construct(mc)
        buf = ctypes.create_string_buffer(1 << 20)
        bad = []
        for i in range(t, n, threads):
            off, ln = int(desc[i]["offset"]), int(desc[i]["caplen"])
            pkt = ctypes.create_string_buffer(arena[off:off + ln].tobytes() + bytes(16))
            ts = Timespec(TS // 1_000_000_000, TS % 1_000_000_000)
            k = f(p, buf, len(buf), pkt, ln, ctypes.byref(ts), int(desc[i]["linktype"]))
            if buf.raw[:k] != (want[i] + b"\n" if want[i] else b""):
                bad.append(i)
        lib.mercury_packet_processor_destruct(p)
        return bad

    with ThreadPoolExecutor(threads) as ex:
        bad = sorted(sum(ex.map(work, range(threads)), []))
    lib.mercury_finalize(mc)
    assert not bad, f"{len(bad)} of {n} packets differ, first {bad[:8]}"
