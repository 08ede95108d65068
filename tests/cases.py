"""Deterministic parity inputs shared by the golden generator
(tests/golden/make_golden_cases.py, which runs the REFERENCE over them) and
the GPU parity tests (which compare the HIP path with those reference
outputs).  Every case is regenerated from seeds and the committed
ref_packets.npz; only the reference's outputs are committed."""
import os
import struct

import numpy as np

from tests import pcaplib, synth

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def ref_pkts():
    z = np.load(os.path.join(GOLD, "ref_packets.npz"))
    a, d = z["arena"], z["desc"]
    return [(int(x["linktype"]), a[int(x["offset"]):int(x["offset"]) + int(x["caplen"])].tobytes()) for x in d]


def _synth_pkts(n, seed, n_templates, workload="mixed"):
    a, d = synth.batch(n, seed=seed, workload=workload, n_templates=n_templates)
    return [(1, a[int(x["offset"]):int(x["offset"]) + int(x["caplen"])].tobytes()) for x in d]


def fuzz_case(fmt):
    """40 000 mutations of the reference's pcap packets plus synthetic ones."""
    pk = ref_pkts() + _synth_pkts(3000, 99, 1000)
    return synth.fuzz(pk, 40000, seed=1000 + fmt)


def edge_case():
    """empty packets, 1-byte frames, truncation at every header boundary,
    65 535-byte frames and giant trailing data."""
    pk = [(1, b""), (1, b"\x00"), (101, b"\x45"), (1, bytes(14)), (1, bytes(65535))]
    a, d = synth.batch(200, seed=3, workload="mixed", n_templates=100)
    for x in d[:50]:
        b = a[int(x["offset"]):int(x["offset"]) + int(x["caplen"])].tobytes()
        pk.append((1, b + bytes(70000 - len(b))))
        for cut in (0, 13, 14, 33, 34, 53, 54, len(b) // 2, len(b) - 1):
            pk.append((1, b[:cut]))
    return pk


def binmix_case():
    pk = _synth_pkts(6000, 0x5EED0042, 1500)
    return pk + synth.fuzz(pk[:2000], 10000, seed=77)


def synth_case(workload, fmt):
    return _synth_pkts(30000, 0x5EED0003 + fmt, 3000, workload)


def analysis_mode_case():
    return _synth_pkts(20000, 5, 2000)


def corpus_case():
    """The reference's fuzzing seeds (test/fuzz/{tls_client_hello,
    http_request,http_response}/corpus: L7 payloads) wrapped in Ethernet/IPv4/
    TCP frames, client side to 443 / 80, server side from 80, each also with
    every prefix length in steps of 7 bytes; the payloads are committed as
    tests/golden/fuzz_corpus.npz (data files of the reference's tests)."""
    z = np.load(os.path.join(GOLD, "fuzz_corpus.npz"))
    out = []
    for kind, blob, ln in zip(z["kind"], z["payload"], z["length"]):
        p = bytes(blob[:int(ln)])
        for cut in sorted(set(list(range(0, len(p), 7)) + [len(p)])):
            q = p[:cut]
            if kind == "tls_client_hello":
                f = synth.frame(synth.tcp(q, sport=50000, dport=443), 6)
            elif kind == "http_request":
                f = synth.frame(synth.tcp(q, sport=50000, dport=80), 6)
            else:
                f = synth.frame(synth.tcp(q, sport=80, dport=50000), 6)
            out.append((1, f))
    return out


def _qtp(t, params):
    """a quic_transport_parameters(_draft) extension: (id, value) pairs as
    variable-length integers (tls.h:1237-1262)"""
    def vli(v):
        if v < 64:
            return bytes([v])
        if v < 16384:
            return struct.pack(">H", 0x4000 | v)
        return struct.pack(">I", 0x80000000 | v)
    return synth.ext(t, b"".join(vli(i) + vli(len(v)) + v for i, v in params))


def _hello_body(exts, version=0x0303, cookie=None, ciphers=b"\x13\x01\x13\x02\xc0\x2b", ext_claim=None):
    body = struct.pack(">H", version) + bytes(range(32)) + b"\x00"
    if cookie is not None:
        body += bytes([len(cookie)]) + cookie
    e = b"".join(exts)
    body += struct.pack(">H", len(ciphers)) + ciphers + b"\x01\x00"
    return body + struct.pack(">H", len(e) if ext_claim is None else ext_claim) + e


def hello_meta_case():
    """Crafted ClientHellos whose JSON text and destination context depend on
    WHICH extension the reference reads: duplicate, empty and malformed
    server_name extensions (write_json prints the first, tls.h:1052-1080; the
    analysis context keeps the last, tls.h:1316-1345), ALPN twice, QUIC
    transport parameters (and the draft type) over TCP with Google user
    agents (tls.h:1264-1311), a DTLS version over TCP (tls.h:1823-1844: cookie
    and "dtls" label), a soft-failed extension list; each over TCP/IPv4,
    TCP/IPv6 and DTLS (UDP/443)."""
    sni = synth.sni_ext
    ext = synth.ext
    sets = [
        [sni("first.example"), sni("second.example")],
        [ext(0, b""), sni("after.example")],
        [sni("only.example"), ext(0, b"\x00\x01\x00")],
        [sni("a"), ext(0, struct.pack(">HBH", 3, 0, 0))],
        [sni("x1.example"), sni("x2.example"), sni("x3.example")],
        [sni("q.example"), _qtp(0x39, [(1, b"\x00\x10"), (0x3129, b"Chrome/99.0"), (4, b"")])],
        [_qtp(0xffa5, [(0x3129, b"UA-draft")]), _qtp(0x39, [(0x3129, b"UA-v1"), (0x3129, b"UA-v1b")]),
         sni("both.example")],
        [],
        [synth.alpn_ext(["h2"]), sni("alpn.example"), synth.alpn_ext(["http/1.1"])],
        [sni("ok.example"), ext(0, bytes(20)), ext(23, b"")],
        [sni("café.example"), ext(0, struct.pack(">HBH", 7, 0, 4) + b"\xff\xfeAB")],
        [sni("v.example"), ext(0x39, b"\x71\x29\x05UA"), ext(0x39, b"")],
        [sni("p.example"), ext(0x0a0a, b""), sni("g.example")],
    ]
    out = []
    for k, exts in enumerate(sets):
        bodies = [_hello_body(exts)]
        # the extension list claims more bytes than the packet holds (parse_soft_fail tls.h:1865)
        bodies.append(_hello_body(exts, ext_claim=len(b"".join(exts)) + 40))
        for b in bodies:
            hs = b"\x01" + struct.pack(">I", len(b))[1:] + b
            rec = struct.pack(">BHH", 0x16, 0x0301, len(hs)) + hs
            out.append((1, synth.frame(synth.tcp(rec, sport=40000 + k, dport=443), 6)))
            out.append((1, synth.frame(synth.tcp(rec, sport=41000 + k, dport=443), 6, v6=True)))
        db = _hello_body(exts, version=0xfefd, cookie=b"\xaa\xbb\xcc\xdd")
        dhs = b"\x01" + struct.pack(">I", len(db))[1:] + struct.pack(">H", 0) + b"\x00\x00\x00" + \
            struct.pack(">I", len(db))[1:] + db
        drec = struct.pack(">BHH", 0x16, 0xfefd, 0) + bytes(6) + struct.pack(">H", len(dhs)) + dhs
        out.append((1, synth.frame(synth.udp(drec, sport=42000 + k, dport=443), 17)))
        # a DTLS version in a ClientHello over TCP: the cookie is skipped, the object is "dtls"
        hs = b"\x01" + struct.pack(">I", len(db))[1:] + db
        out.append((1, synth.frame(synth.tcp(struct.pack(">BHH", 0x16, 0x0301, len(hs)) + hs, sport=43000 + k,
                                             dport=443), 6)))
    return out


def batch(pkts):
    return pcaplib.make_batch(pkts)


def tls_ch_unique_head(n=20000):
    """The first n of the 200 000 unique packets bench.py / the large-batch
    test replicate for config 2 (10 M TLS ClientHellos)."""
    a, d = synth.batch(200_000, seed=0x5EED0001, workload="tls_ch", n_templates=4096)
    return [(1, a[int(x["offset"]):int(x["offset"]) + int(x["caplen"])].tobytes()) for x in d[:n]]


# name -> (packets builder, [(fmt, mode)])
CASES = {
    "fuzz0": (lambda: fuzz_case(0), [(0, "fp"), (0, "json")]),
    "fuzz1": (lambda: fuzz_case(1), [(1, "fp"), (1, "json")]),
    "fuzz2": (lambda: fuzz_case(2), [(2, "fp"), (2, "json")]),
    "edge": (edge_case, [(0, "fp"), (1, "fp"), (2, "fp"), (0, "json"), (1, "json"), (2, "json")]),
    "binmix": (binmix_case, [(0, "fp"), (2, "fp")]),
    "synth_mixed0": (lambda: synth_case("mixed", 0), [(0, "fp")]),
    "synth_mixed1": (lambda: synth_case("mixed", 1), [(1, "fp")]),
    "synth_mixed2": (lambda: synth_case("mixed", 2), [(2, "fp")]),
    "synth_tls_ch0": (lambda: synth_case("tls_ch", 0), [(0, "fp")]),
    "synth_tls_ch1": (lambda: synth_case("tls_ch", 1), [(1, "fp")]),
    "synth_tls_ch2": (lambda: synth_case("tls_ch", 2), [(2, "fp")]),
    "analysis_mode": (analysis_mode_case, [(1, "an")]),
    "corpus": (corpus_case, [(0, "fp"), (1, "fp"), (2, "fp"), (0, "json"), (1, "json"), (2, "json")]),
    "hello_meta": (hello_meta_case, [(0, "fp"), (1, "fp"), (2, "fp"), (0, "json"), (1, "json"), (2, "json"),
                                     (1, "meta")]),
    "tls_ch_head": (tls_ch_unique_head, [(0, "fp")]),
}


# the "meta" runs read the analysis context, which needs a classifier
META_RESOURCES = os.path.join(GOLD, "resources-test.tgz")


def golden_path(name, fmt, mode):
    ext = "txt" if mode == "json" else "tsv"
    return os.path.join(GOLD, "cases", f"{name}.{mode}{fmt}.{ext}.gz")


def load_json_golden(name, fmt):
    """The reference's write_json text per packet (b"" when it writes none)."""
    import gzip
    with gzip.open(golden_path(name, fmt, "json"), "rb") as f:
        return f.read().split(b"\n")[:-1]


def load_meta_golden(name, fmt=1):
    """(valid, server_name, user_agent) per packet from the analysis context
    accessors; None for a NULL string."""
    import gzip
    rows = []
    with gzip.open(golden_path(name, fmt, "meta"), "rt") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            rows.append((int(p[1]), None if p[2] == "-" else bytes.fromhex(p[2]),
                         None if p[3] == "-" else bytes.fromhex(p[3])))
    return rows


def load_golden(name, fmt, mode):
    """Reference rows: (emit, fp_type, truncated, fingerprint) per packet
    ("an" mode: emit = the analysis_context is valid, truncated = 0)."""
    import gzip
    rows = []
    with gzip.open(golden_path(name, fmt, mode), "rt", encoding="latin-1") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            if mode == "fp":
                rows.append((int(p[1]), int(p[2]), int(p[3]), p[4] if len(p) > 4 else ""))
            else:
                rows.append((int(p[1]), int(p[2]), 0, p[8] if len(p) > 8 else ""))
    return rows
