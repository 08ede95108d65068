"""Pins the C oracle (oracle/mfp_oracle.c) before it is trusted as the
checker of the HIP path.  CPU only.

* every packet of tests/golden/ref_packets.npz (taken from the reference's own
  test pcaps) must give exactly the reference's output committed in
  ref_fp_fmt{0,1,2}.tsv.gz (made by tests/golden/make_golden.py from the
  reference libmerc compiled out of /root/reference);
* the reference's golden file test/data/top_100_fingerprints.fp;
* the known-answer strings of the reference's in-header unit test
  (tls.h:377-420) and of SURVEY.md Appendix A (#3, #9), which were confirmed
  against the reference binary.
"""
import gzip
import os
import struct

import numpy as np
import pytest

from oracle import oracle
from tests import pcaplib, synth

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load_golden():
    z = np.load(os.path.join(GOLD, "ref_packets.npz"))
    return z["arena"], z["desc"], z["sources"]


def load_ref(fmt):
    rows = []
    with gzip.open(os.path.join(GOLD, f"ref_fp_fmt{fmt}.tsv.gz"), "rt", encoding="latin-1") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            rows.append((int(p[1]), int(p[2]), int(p[3]), p[4] if len(p) > 4 else ""))
    return rows


@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_oracle_matches_reference_outputs(fmt):
    arena, desc, sources = load_golden()
    ref = load_ref(fmt)
    assert len(ref) == len(desc)
    ft, fl, flags, fps = oracle.process_batch(arena, desc, oracle.config(tls_format=fmt))
    bad = []
    for i, (emit, t, trunc, s) in enumerate(ref):
        e = int(flags[i] & 1)
        tr = int((flags[i] >> 1) & 1) & e
        if (e, int(ft[i]), tr, fps[i]) != (emit, t, trunc, s):
            bad.append(str(sources[i]))
    assert not bad, f"{len(bad)} mismatches: {bad[:8]}"
    # the fixture really exercises every fingerprint family of the path
    types = {r[1] for r in ref}
    assert {1, 2, 3, 4, 6, 7, 10, 11, 13, 17, 19, 20}.issubset(types), types


def test_oracle_top100_golden_file():
    arena, desc, sources = load_golden()
    sel = [i for i, s in enumerate(sources) if str(s).startswith("top_100_fingerprints.pcap:")]
    ft, _, _, fps = oracle.process_batch(arena, desc[sel])
    got = [fps[k] for k in range(len(sel)) if ft[k] == 1]
    with open(os.path.join(GOLD, "top_100_fingerprints.fp")) as f:
        want = [line.strip().strip('"') for line in f if line.strip()]
    assert len(want) == 100
    assert got == want


def client_hello(exts, ciphers=b"\x0a\x0a\x13\x01\x13\x02"):
    body = b"\x03\x03" + bytes(32) + b"\x00" + struct.pack(">H", len(ciphers)) + ciphers + b"\x01\x00"
    body += struct.pack(">H", len(exts)) + exts
    hs = b"\x01" + struct.pack(">I", len(body))[1:] + body
    return b"\x16\x03\x01" + struct.pack(">H", len(hs)) + hs


def tls_frame(payload, dport=443):
    return synth.frame(synth.tcp(payload, sport=50000, dport=dport), 6)


def fp_of(pkt, fmt=0, linktype=1):
    ft, _, _, fps = oracle.process_batch(*pcaplib.make_batch([(linktype, pkt)]), oracle.config(tls_format=fmt))
    return int(ft[0]), fps[0]


def test_reference_unit_test_extension_encodings():
    """tls.h:377-420: format 1 / format 2 encodings of unassigned, private and
    GREASE extensions."""
    exts = bytes([0x00, 0x3f, 0x00, 0x01, 0x01, 0xff, 0x2b, 0x00, 0x01, 0x01, 0x1a, 0x1a, 0x00, 0x00,
                  0x2a, 0x2a, 0x00, 0x00, 0xff, 0x2b, 0x00, 0x01, 0x02, 0xff, 0x2b, 0x00, 0x01, 0x02,
                  0xff, 0x2b, 0x00, 0x01, 0x02])
    pkt = tls_frame(client_hello(exts))
    t, s1 = fp_of(pkt, 1)
    assert t == 1 and s1.endswith("[(003f)(0a0a)(0a0a)(ff2b)(ff2b)(ff2b)(ff2b)]"), s1
    t, s2 = fp_of(pkt, 2)
    assert t == 1 and s2.endswith("[(003e)(0a0a)(0a0a)(ff00)(ff00)(ff00)]"), s2


def test_appendix_a_grease_rules():
    """the two GREASE tests (confirmed with the reference)."""
    def e(t, b):
        return struct.pack(">HH", t, len(b)) + b
    exts = (e(0x1a0a, b"") + e(0x0a0a, b"") + e(0x000a, bytes.fromhex("00060a0a001d0017"))
            + e(0x002b, bytes.fromhex("040a0a0304")) + e(0x0000, b"") + e(0xff2b, b"") + e(0x0017, b""))
    pkt = tls_frame(client_hello(exts))
    assert fp_of(pkt, 0)[1] == ("tls/(0303)(0a0a13011302)((1a0a)(0a0a)(000a000800060a0a001d0017)"
                                "(002b0005040a0a0304)(0000)(ff2b)(0017))")
    assert fp_of(pkt, 1)[1] == ("tls/1/(0303)(0a0a13011302)[(0000)(000a000800060a0a001d0017)(0017)"
                                "(002b0005040a0a0304)(0a0a)(0a0a)(ff2b)]")
    assert fp_of(pkt, 2)[1] == ("tls/2/(0303)(0a0a13011302)[(0000)(000a000800060a0a001d0017)(0017)"
                                "(002b0005040a0a0304)(0a0a)(0a0a)(ff00)]")


@pytest.mark.parametrize("banner,want", [
    (b"SSH-2.0-OpenSSH_8.9\n", "ssh_init/(5353482d322e302d4f70656e5353485f382e)"),
    (b"SSH-2.0-OpenSSH_8.9\r\n", "ssh_init/(5353482d322e302d4f70656e5353485f382e39)"),
    (b"SSH-2.0-OpenSSH_8.9 Ubuntu\n", "ssh_init/(5353482d322e302d4f70656e5353485f382e39205562756e74)"),
])
def test_appendix_a_ssh_trim(banner, want):
    """ssh.h:393,396 trim exactly one byte."""
    pkt = synth.frame(synth.tcp(banner, sport=50000, dport=22), 6)
    t, s = fp_of(pkt)
    assert t == 17   # fingerprint_type_ssh_init (libmerc.h:368)
    assert s == want


def test_appendix_a_ipv4_options_not_skipped():
    """ip.h:124-137 takes a fixed 20-byte header."""
    l4 = synth.tcp(b"SSH-2.0-OpenSSH_8.9\r\n", sport=50000, dport=22)
    ok = synth.frame(l4, 6)
    ip = bytearray(synth.ipv4(b"\x01\x01\x01\x01" + l4, 6))
    ip[0] = 0x46
    assert fp_of(ok)[0] == 17
    assert fp_of(synth.eth(bytes(ip)))[0] == 0


def test_config1_known_answer():
    """SURVEY.md 8(d) config 1 expected fingerprint (reference output)."""
    arena, desc, sources = load_golden()
    i = [k for k, s in enumerate(sources) if str(s).startswith("tls_client_hello_test_packet.pcap:")][0]
    ft, _, _, fps = oracle.process_batch(arena, desc[i:i + 1])
    assert fps[0] == (
        "tls/(0303)(130113021303c02cc02bc024c023c00ac009cca9c030c02fc028c027c014c013cca8009d009c003d003c0035002f"
        "c008c012000a)((ff01)(0000)(0017)(000d0018001604030804040105030203080508050501080606010201)"
        "(000500050100000000)(0012)(0010000e000c02683208687474702f312e31)(000b00020100)(0033)(002d00020101)"
        "(002b0009080304030303020301)(000a000a0008001d001700180019)(0015))")


def test_synthetic_generator_deterministic():
    a1, d1 = synth.batch(500, seed=7, workload="mixed", n_templates=64)
    a2, d2 = synth.batch(500, seed=7, workload="mixed", n_templates=64)
    assert np.array_equal(a1, a2) and np.array_equal(d1, d2)
    ft, _, flags, _ = oracle.process_batch(a1, d1)
    # every family of the contract mix shows up, and "no output" packets exist
    assert set(np.unique(ft)) >= {0, 1, 2, 3, 7}
    assert (flags & 1).sum() < len(d1)


@pytest.mark.parametrize("name,fmt,mode", [("fuzz0", 0, "fp"), ("fuzz2", 2, "fp"), ("edge", 1, "fp"),
                                           ("corpus", 0, "fp"), ("analysis_mode", 1, "an")])
def test_oracle_vs_reference_cases(name, fmt, mode):
    """The C oracle (the debugging twin) equals the reference on the GPU
    parity cases too (tests/golden/cases, from oracle/_ref)."""
    from tests import cases
    pk = cases.CASES[name][0]()
    a, d = cases.batch(pk)
    ref = cases.load_golden(name, fmt, mode)
    ft, fl, flags, strs = oracle.process_batch(a, d, oracle.config(tls_format=fmt, mode=0 if mode == "fp" else 1))
    bad = 0
    for i, (emit, t, tr, s) in enumerate(ref):
        if mode == "fp":
            o = (int(flags[i] & 1), int(ft[i]), int((flags[i] >> 1) & 1) & int(flags[i] & 1), strs[i])
            bad += o != (emit, t, tr, s)
        else:
            bad += (int(ft[i]), strs[i]) != (t, s)
    assert bad == 0
