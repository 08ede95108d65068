"""Deterministic parity inputs shared by the golden generator
(tests/golden/make_golden_cases.py, which runs the REFERENCE over them) and
the GPU parity tests (which compare the HIP path with those reference
outputs).  Every case is regenerated from seeds and the committed
ref_packets.npz; only the reference's outputs are committed."""
import os

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


def batch(pkts):
    return pcaplib.make_batch(pkts)


def tls_ch_unique_head(n=20000):
    """The first n of the 200 000 unique packets bench.py / the large-batch
    test replicate for config 2 (10 M TLS ClientHellos)."""
    a, d = synth.batch(200_000, seed=0x5EED0001, workload="tls_ch", n_templates=4096)
    return [(1, a[int(x["offset"]):int(x["offset"]) + int(x["caplen"])].tobytes()) for x in d[:n]]


# name -> (packets builder, [(fmt, mode)])
CASES = {
    "fuzz0": (lambda: fuzz_case(0), [(0, "fp")]),
    "fuzz1": (lambda: fuzz_case(1), [(1, "fp")]),
    "fuzz2": (lambda: fuzz_case(2), [(2, "fp")]),
    "edge": (edge_case, [(0, "fp"), (1, "fp"), (2, "fp")]),
    "binmix": (binmix_case, [(0, "fp"), (2, "fp")]),
    "synth_mixed0": (lambda: synth_case("mixed", 0), [(0, "fp")]),
    "synth_mixed1": (lambda: synth_case("mixed", 1), [(1, "fp")]),
    "synth_mixed2": (lambda: synth_case("mixed", 2), [(2, "fp")]),
    "synth_tls_ch0": (lambda: synth_case("tls_ch", 0), [(0, "fp")]),
    "synth_tls_ch1": (lambda: synth_case("tls_ch", 1), [(1, "fp")]),
    "synth_tls_ch2": (lambda: synth_case("tls_ch", 2), [(2, "fp")]),
    "analysis_mode": (analysis_mode_case, [(1, "an")]),
    "corpus": (corpus_case, [(0, "fp"), (1, "fp"), (2, "fp")]),
    "tls_ch_head": (tls_ch_unique_head, [(0, "fp")]),
}


def golden_path(name, fmt, mode):
    return os.path.join(GOLD, "cases", f"{name}.{mode}{fmt}.tsv.gz")


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
