"""Golden JSON records WITH --analysis from the REFERENCE (write_json path,
libmerc do_analysis + a resource archive), and the analysis-context accessors
(attributes, os_info, ALPN) the embedders read.  Dev container only (needs
oracle/_ref built by oracle/Makefile.ref):

    python tests/golden/make_golden_analysis.py        (the archives first)
    python tests/golden/make_golden_json_analysis.py

Outputs (committed), all with select "tls,dtls,ssh,http,tcp,tcp.syn_ack",
report_os on (MERC_REPORT_OS=1) and every timestamp 1700000000.000000:
  json_an_crafted.npz    crafted packets for the classifier-agnostic
                         attributes and the analysis object's branches
                         (encrypted_dns by name / IPv4 / IPv6, domain_faking
                         mapped / faked / "www." / exception / private / IPv6
                         / index >= 256, faketls, ALPN), with synth_resources.tgz:
                         arena, desc, json lines, attr lines
  json_an_synth.txt.gz   synth.batch(4000, seed=0x5EED0003) with synth_resources.tgz
  json_an_ref.txt.gz     ref_packets.npz with resources-test.tgz
  an_attr_synth.tsv.gz   merc_ref_drv "attr" lines for the same synthetic batch
One line per packet, empty when the reference writes nothing.
"""
import gzip
import io
import os
import struct
import subprocess
import sys
import tarfile
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
from tests import pcaplib, synth  # noqa: E402
from oracle.compare_ref import REF, CONTRACT_SELECT  # noqa: E402

SYNTH_RES = os.path.join(HERE, "synth_resources.tgz")
TEST_RES = os.path.join(HERE, "resources-test.tgz")


def ref_lines(mode, arena, desc, resources):
    env = dict(os.environ, MERC_REPORT_OS="1")
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "b.mfpb")
        pcaplib.write_mfpb(p, arena, desc)
        out = subprocess.run([REF, mode, p, CONTRACT_SELECT, resources], capture_output=True, check=True,
                             env=env).stdout
    lines = out.split(b"\n")[:-1]
    assert len(lines) == len(desc), (mode, len(lines), len(desc))
    return lines


def member(path, name):
    with tarfile.open(path, "r:gz") as tf:
        return tf.extractfile(name).read().decode()


def v6(words):
    return b"".join(struct.pack(">H", w) for w in words)


def ch(sni, ciphers=(0x1301, 0x1302, 0xc02b), alpn=("h2", "http/1.1"), extra=b""):
    """A TLS 1.2-record ClientHello with SNI, ALPN, supported_versions."""
    cs = b"".join(struct.pack(">H", c) for c in ciphers)
    exts = (synth.sni_ext(sni) if sni is not None else b"") + synth.ext(23, b"") + \
        (synth.alpn_ext(alpn) if alpn else b"") + synth.versions_ext([0x0304, 0x0303]) + extra
    body = struct.pack(">H", 0x0303) + bytes(32) + b"\x00" + struct.pack(">H", len(cs)) + cs + b"\x01\x00"
    body += struct.pack(">H", len(exts)) + exts
    hs = b"\x01" + struct.pack(">I", len(body))[1:] + body
    return struct.pack(">BHH", 0x16, 0x0301, len(hs)) + hs


def tcp4(payload, dst, dport=443, src=0x0a000001):
    return synth.eth(synth.ipv4(synth.tcp(payload, 50000, dport), 6, src=src, dst=dst))


def tcp6(payload, dst_words, dport=443):
    return synth.eth(synth.ipv6(synth.tcp(payload, 50000, dport), 6, src=v6([0x2001, 0xdb8, 0, 0, 0, 0, 0, 5]),
                                dst=v6(dst_words)), 0x86dd)


def ip4(a, b, c, d):
    return a << 24 | b << 16 | c << 8 | d


def crafted():
    doh = [x for x in member(SYNTH_RES, "doh-watchlist.txt").splitlines() if x and not x[0] in "#*" and " " not in x]
    doh_names = [x for x in doh if not x[0].isdigit() and ":" not in x]
    import json
    maps = [json.loads(x) for x in member(SYNTH_RES, "domain-mappings.db").splitlines() if x.startswith("{")]
    mapped_home = [m["tag"] for m in maps if m["type"] == "domain_mapping" and m["subnet"] == "13.89.0.0/16"]
    mapped_away = [m["tag"] for m in maps if m["type"] == "domain_mapping" and m["subnet"].startswith(("8.", "9.", "1"))
                   and not m["tag"].startswith("filler") and m["subnet"] != "13.89.0.0/16"]
    mapped_v6 = [m["tag"] for m in maps if m["subnet"] == "2607:f8b0::/40"]
    late = [m["tag"] for m in maps if m["tag"].startswith("late-") or m["tag"].endswith(".late")]
    out = []
    dst = ip4(13, 89, 178, 27)
    # encrypted_dns: by server name, by IPv4 / IPv6 destination, neither
    for nm in doh_names[:3]:
        out.append(tcp4(ch(nm), dst))
    out.append(tcp4(ch("nobody.example.org"), ip4(13, 89, 7, 9)))
    out.append(tcp6(ch("nobody.example.org"), [0x2607, 0xf8b0, 0, 0, 0, 0, 0, 0x11]))
    out.append(tcp4(ch("dns.example.net"), dst))
    out.append(tcp4(ch("nobody.example.org"), dst))
    # domain_faking: mapped to the destination's range (no), elsewhere (yes),
    # with "www.", exception ranges, private destination, IPv6, late index
    for nm in mapped_home[:2] + mapped_away[:3]:
        out.append(tcp4(ch(nm), dst))
        out.append(tcp4(ch("www." + nm), dst))
    for nm in mapped_away[:2]:
        out.append(tcp4(ch(nm), ip4(13, 89, 200, 9)))    # sinkhole exception
        out.append(tcp4(ch(nm), ip4(13, 89, 130, 1)))    # proxy exception
        out.append(tcp4(ch(nm), ip4(192, 168, 1, 1)))    # private destination
        out.append(tcp4(ch(nm), ip4(13, 90, 0, 1)))      # no prefix at all
    for nm in mapped_v6[:2]:
        out.append(tcp6(ch(nm), [0x2607, 0xf8b0, 0, 0, 0, 0, 0, 0x22]))       # mapped
        out.append(tcp6(ch(nm), [0x2607, 0xf8b1, 0, 0, 0, 0, 0, 0x22]))       # outside
        out.append(tcp6(ch(nm), [0x2607, 0xf8b1, 0, 0x11fc, 0, 0, 0, 0x22]))  # byte 7 = fc ("private")
        out.append(tcp6(ch(nm), [0x2607, 0xf8b0, 0x4000, 0, 0, 0, 0, 1]))    # v6 sinkhole
    for nm in late + ["twice.example", "proxy", "zero.example", "private.example"]:
        out.append(tcp4(ch(nm), dst))
        out.append(tcp4(ch(nm), ip4(100, 0, 5, 1)))
    # faketls (randomized ClientHellos only): all suites unknown, none at all,
    # one known among unknown ones, GREASE + unknown
    out.append(tcp4(ch("fake.example", ciphers=(0x1234, 0x5678, 0x9abc)), dst))
    out.append(tcp4(ch("fake2.example", ciphers=()), dst))
    out.append(tcp4(ch("fake3.example", ciphers=(0x1234, 0x1301)), dst))
    out.append(tcp4(ch("fake4.example", ciphers=(0x3a3a, 0x4444)), dst))
    out.append(tcp4(ch("fake.example", ciphers=(0x1234, 0x5678, 0x9abc)), dst))   # second sighting: unlabeled
    # ALPN shapes: none, empty list, truncated list, two ALPN extensions
    out.append(tcp4(ch("alpn0.example", alpn=()), dst))
    out.append(tcp4(ch("alpn1.example", alpn=(), extra=synth.ext(16, b"\x00\x00")), dst))
    out.append(tcp4(ch("alpn2.example", alpn=(), extra=synth.ext(16, b"\x00\x09\x02h2")), dst))
    out.append(tcp4(ch("alpn3.example", extra=synth.alpn_ext(("spdy/3",))), dst))
    # destination addresses whose text form drops pieces (append_ipv6_addr run quirk)
    for w in ([1, 0, 2, 0, 0, 3, 0, 4], [0, 5, 0, 0, 6, 0, 0, 0], [0x2607, 0, 1, 0, 0, 2, 0, 0]):
        out.append(tcp6(ch("v6quirk.example"), w))
    # an HTTP request (unlabeled), no server name
    out.append(tcp4(b"GET / HTTP/1.1\r\nHost: h.example\r\nUser-Agent: curl/8.4.0\r\n\r\n", dst, dport=80))
    out.append(tcp4(ch(None), dst))
    return out


def main():
    frames = crafted()
    arena, desc = pcaplib.make_batch([(1, f) for f in frames])
    js = ref_lines("json", arena, desc, SYNTH_RES)
    at = ref_lines("attr", arena, desc, SYNTH_RES)
    blob = b"".join(js)
    ends = np.cumsum([len(x) for x in js]).astype(np.uint64)
    ablob = b"".join(x + b"\n" for x in at)
    np.savez_compressed(os.path.join(HERE, "json_an_crafted.npz"), arena=arena, desc=desc,
                        json=np.frombuffer(blob, np.uint8), json_end=ends, attr=np.frombuffer(ablob, np.uint8))
    sa, sd = synth.batch(4000, seed=0x5EED0003)
    with gzip.open(os.path.join(HERE, "json_an_synth.txt.gz"), "wb") as f:
        f.write(b"".join(x + b"\n" for x in ref_lines("json", sa, sd, SYNTH_RES)))
    with gzip.open(os.path.join(HERE, "an_attr_synth.tsv.gz"), "wb") as f:
        f.write(b"".join(x + b"\n" for x in ref_lines("attr", sa, sd, SYNTH_RES)))
    with np.load(os.path.join(HERE, "ref_packets.npz")) as z:
        ra, rd = z["arena"], z["desc"]
    with gzip.open(os.path.join(HERE, "json_an_ref.txt.gz"), "wb") as f:
        f.write(b"".join(x + b"\n" for x in ref_lines("json", ra, rd, TEST_RES)))
    n_an = sum(b'"analysis"' in x for x in js)
    print("crafted", len(frames), "with analysis", n_an, "synth", len(sd), "ref", len(rd))


if __name__ == "__main__":
    main()
