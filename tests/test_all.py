"""Selections that name protocols outside the device path ("all", the reference
CLI's default, and a mixed list) against the REFERENCE
(tests/golden/all_*, made by tests/golden/make_golden_all.py).

Expected, per packet: the reference's record under the selection when it is
the record of one of this path's protocols, else nothing -- including the
packets another selected protocol claims first (the matchers and ports of
traffic_selector, proto_identify.h:620-895, 936-1075; the encapsulation
walk's port table, pkt_proc.cc:1000-1018), which the device marks
MFP_MSG_OTHER.  Bar: byte-identical JSON lines and fingerprint rows.
"""
import gzip
import json
import os

import numpy as np
import pytest

import mercury_amd

GOLD = os.path.join(os.path.dirname(__file__), "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "all_manifest.json")))
TS = 1700000000 * 10**9
CONFIGS = ["all", "mix", "all_fmt1"]
OTHER = mercury_amd.api.MSG_NAMES.index("other")


def load():
    z = np.load(os.path.join(GOLD, "all_packets.npz"))
    return z["arena"], z["desc"], z["sources"]


def test_all_golden_shape():
    assert MANIFEST["packets"] > 9000
    m = MANIFEST["all"]
    assert m["records"] > 4000 and m["other_protocol_records"] > 1000 and m["claimed_from_own"] >= 50
    assert MANIFEST["mix"]["claimed_from_own"] > 10


@pytest.mark.gpu
@pytest.mark.parametrize("key", CONFIGS)
def test_selection_with_other_protocols_vs_reference(key):
    arena, desc, sources = load()
    ctx = mercury_amd.Context(MANIFEST[key]["config"], device=0)
    try:
        rec, fp = ctx.process_host(arena, desc)
    finally:
        ctx.close()
    lines, skipped = mercury_amd.write_json(arena, desc, rec, fp, ts_ns=np.full(len(desc), TS, np.uint64))
    with gzip.open(os.path.join(GOLD, f"all_json_{key}.txt.gz"), "rb") as f:
        want = f.read().split(b"\n")[:len(desc)]
    bad = [(i, str(sources[i])) for i in range(len(desc)) if lines[i] != (want[i] + b"\n" if want[i] else b"")]
    assert not bad, f"{len(bad)} JSON mismatches, first {bad[:5]}"
    assert skipped == 0
    fps = mercury_amd.fingerprints(rec, fp)
    with gzip.open(os.path.join(GOLD, f"all_fp_{key}.tsv.gz"), "rt", encoding="latin-1") as f:
        rows = [line.rstrip("\n").split("\t") for line in f][:len(desc)]
    bad = []
    for i, r in enumerate(rows):
        emit = int(rec["flags"][i] & 1)
        trunc = int((rec["flags"][i] >> 1) & 1) & emit
        if (emit, int(rec["fp_type"][i]), trunc, fps[i]) != (int(r[1]), int(r[2]), int(r[3]), r[4] if len(r) > 4 else ""):
            bad.append((i, str(sources[i])))
    assert not bad, f"{len(bad)} fingerprint mismatches, first {bad[:5]}"
    # the packets claimed away from this path's protocols are marked
    claimed = [i for i, s in enumerate(sources) if str(s).startswith(("other:http.rdp", "other:udp.wg.50000.443"))]
    if key != "mix":
        assert all(int(rec["msg"][i]) == OTHER for i in claimed), [(i, int(rec["msg"][i])) for i in claimed]


@pytest.mark.gpu
def test_shim_counts_packets_claimed_by_other_protocols():
    """The libmerc shim under "all": per-packet write_json returns 0 for every
    packet the device marks MFP_MSG_OTHER, and mercury_amd_other_packets
    counts them (the records the reference writes and this library does not)."""
    import ctypes
    from tests.test_json import _LibmercConfig
    arena, desc, _ = load()
    ctx = mercury_amd.Context(MANIFEST["all"]["config"], device=0)
    try:
        rec, _ = ctx.process_host(arena, desc)
    finally:
        ctx.close()
    idx = [i for i in range(len(desc)) if int(rec["msg"][i]) == OTHER][:200]
    assert len(idx) >= 50
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
    lib.mercury_amd_other_packets.restype = ctypes.c_uint64
    lib.mercury_amd_other_packets.argtypes = [vp]
    f = lib.mercury_packet_processor_write_json_linktype
    f.restype = ctypes.c_size_t
    f.argtypes = [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, ctypes.POINTER(Timespec), ctypes.c_uint16]
    cfg = _LibmercConfig()
    cfg.packet_filter_cfg = MANIFEST["all"]["config"].encode()
    mc = lib.mercury_init(ctypes.byref(cfg), 0)
    assert mc and lib.mercury_amd_other_packets(mc) == 0
    p = lib.mercury_packet_processor_construct(mc)
    buf = ctypes.create_string_buffer(1 << 16)
    for i in idx:
        off, ln = int(desc[i]["offset"]), int(desc[i]["caplen"])
        pkt = ctypes.create_string_buffer(arena[off:off + ln].tobytes() + bytes(16))
        ts = Timespec(TS // 10**9, 0)
        assert f(p, buf, len(buf), pkt, ln, ctypes.byref(ts), int(desc[i]["linktype"])) == 0, i
    assert lib.mercury_amd_other_packets(mc) == len(idx)
    lib.mercury_packet_processor_destruct(p)
    lib.mercury_finalize(mc)
