"""Subnet lookups of the --analysis classifier (subnet_data, addr.cc) against the
REFERENCE: the ASN of a destination (get_asn_info addr.cc:172-208) and the
domain_faking attribute (is_domain_faking addr.cc:707-792), both answered by the
reference's level-compressed tries (lctrie/lctrie.hpp:347-386), whose lookup is
not a clean longest-prefix match on nested prefixes.  Run in the dev container
(needs oracle/_ref):

    python tests/golden/make_golden_lpm.py

Tables (seeded): pyasn.db with the synthetic archive's lines (2607:f8b0::/32
holding exactly one /48), IPv6 structures that reach each quirk of the
reference's construction (a prefix of >= 64 host bits with one child counts as
full, two or three children overflow the size sum, chains /40 > /48 > /56 > /64,
prefixes longer than 64 bits, tilings), random IPv4 and IPv6 prefixes nested or
not, repeated prefixes, invalid lines; a domain-mapping table with nested IPv4
and IPv6 mappings, proxy / sinkhole exceptions, a prefix given twice and one
re-given with another length.

Queries: the first, last and a middle address of every prefix, the addresses
just outside it, random addresses, with server names that are mapped (with
and without "www."), unmapped or absent.

Outputs (committed):
  lpm_resources.tgz   the tables as a resource archive (plus one labeled TLS
                      fingerprint whose processes carry the table's ASNs)
  lpm_queries.tsv.gz  dst_ip  server_name
  lpm_ref.tsv.gz      merc_ref_drv lpm: dst_ip  server_name  asn  domain_faking
  lpm_packets.npz     TLS ClientHellos to a sample of the query addresses, with
                      the queries' server names
  lpm_an.tsv.gz       merc_ref_drv an on lpm_packets (the ASN moves the score)
  lpm_attr.tsv.gz     merc_ref_drv attr on lpm_packets (domain_faking)
  lpm_manifest.json
"""
import gzip
import io
import ipaddress
import json
import os
import subprocess
import sys
import tarfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
from tests import pcaplib, synth, synth_db  # noqa: E402
from oracle.compare_ref import REF  # noqa: E402

SEED = 0x5EED0C7E
MAPPED = ["google.com", "example.net", "video.example", "cdn.test", "mail.corp", "v6only.example", "nested.example",
          "late.example", "twice.example"]


def v6s(a, ln):
    return f"{ipaddress.IPv6Address(a).compressed}/{ln}"


def v4s(a, ln):
    return f"{ipaddress.IPv4Address(a)}/{ln}"


def mask(a, ln, bits):
    return a & (((1 << bits) - 1) ^ ((1 << (bits - ln)) - 1))


def asn_table(rng):
    lines = list(synth_db.ASN_LINES)          # 2607:f8b0::/32 with exactly one /48 inside
    pref = []                                 # (bits, addr, len) of the valid prefixes, for queries
    asn = iter(range(70000, 200000))

    def add6(a, ln):
        a = mask(a, ln, 128)
        lines.append(f"{v6s(a, ln)}\t{next(asn)}")
        pref.append((128, a, ln))

    def add4(a, ln):
        a = mask(a, ln, 32)
        lines.append(f"{v4s(a, ln)}\t{next(asn)}")
        pref.append((32, a, ln))

    def r6(top=0x2000):
        return (top + int(rng.integers(0, 0x1000))) << 112 | int(rng.integers(0, 1 << 62)) << 48 | int(rng.integers(0, 1 << 48))

    for k in range(64):
        root = r6()
        kind = k % 8
        if kind == 0:      # /32 holding one /48: "full" (size capped at UINT64_MAX)
            add6(root, 32); add6(root | int(rng.integers(0, 1 << 16)) << 80, 48)
        elif kind == 1:    # two /48s: the capped sizes overflow, not full
            add6(root, 32); add6(root | 1 << 80, 48); add6(root | 7 << 80, 48)
        elif kind == 2:    # three /48s and a /40
            add6(root, 32); add6(root | 3 << 80, 48); add6(root | 5 << 80, 48); add6(root | 0x9 << 84, 40)
        elif kind == 3:    # chain /40 > /48 > /56 > /64
            for ln in (40, 48, 56, 64):
                add6(root, ln)
        elif kind == 4:    # prefixes longer than 64 bits under a /64
            add6(root, 64); add6(root | 1 << 40, 96); add6(root | 1 << 40 | 5 << 20, 112); add6(root | 0xabc, 128)
            add6(root | 3 << 62, 66)
        elif kind == 5:    # a /48 tiled by two /49s
            add6(root, 48); add6(root, 49); add6(root | 1 << 79, 49)
        elif kind == 6:    # a /96 tiled by two /97s (exact sizes: full)
            add6(root, 96); add6(root, 97); add6(root | 1 << 31, 97)
        else:              # siblings under a /36, one of them nested again
            add6(root, 36); add6(root | 1 << 88, 44); add6(root | 2 << 88, 44); add6(root | 2 << 88 | 1 << 70, 60)
    for _ in range(1500):  # random IPv6, nested or not
        ln = int(rng.integers(16, 65)) if rng.random() < 0.9 else int(rng.integers(65, 129))
        add6(r6(0x2000 + 0x100 * int(rng.integers(0, 4))), ln)
    for _ in range(3000):  # random IPv4 (synth_db.asn_filler's shapes)
        ln = int(rng.integers(8, 25))
        add4(int(rng.integers(1, 224)) << 24 | int(rng.integers(0, 1 << 24)), ln)
    for base in (0x4D010000, 0x4D020000):   # IPv4 tilings: a /23 by two /24s, and a chain
        add4(base, 23); add4(base, 24); add4(base | 0x100, 24)
    add4(0x4D030000, 16); add4(0x4D030000, 17); add4(0x4D038000, 18); add4(0x4D03C000, 18)
    # repeated prefixes (the first one stays), unmasked addresses
    lines += [synth_db.ASN_LINES[1].split("\t")[0] + "\t4242", "2607:f8b0::/32\t4343", "13.89.178.77/24\t4444",
              "2a03:2880:f00d::1/48\t4545"]
    pref += [(32, 0x0D59B200, 24), (128, 0x2A032880F00D00000000000000000000, 48)]
    # lines the reference rejects
    lines += ["2001:db8::/0\t1", "2001:db8::/129\t1", "zzzz::/32\t5", "2001:db8::/32", "1.2.3.0/0\t5", "1.2.3.4/33\t5",
              "bogus"]   # (an empty line would end the archive reader, archive.h:247-270)
    perm = rng.permutation(len(lines))
    return [lines[int(i)] for i in perm], pref


def domain_table(rng):
    d = []   # (subnet, type, tag)
    d += [("13.89.0.0/16", "domain_mapping", "example.net"), ("13.89.0.0/18", "domain_mapping", "video.example"),
          ("13.89.64.0/18", "domain_mapping", "cdn.test"), ("13.89.128.0/17", "proxy", "corp proxy"),
          ("13.89.200.0/24", "sinkhole", "filter"), ("13.89.0.0/20", "domain_mapping", "twice.example"),
          ("13.89.0.0/20", "domain_mapping", "twice.example"), ("13.89.0.0/21", "domain_mapping", "mail.corp"),
          ("10.0.0.0/8", "domain_mapping", "mail.corp"), ("8.8.0.0/16", "domain_mapping", "google.com"),
          ("8.8.8.0/24", "domain_mapping", "nested.example"),
          ("2607:f8b0::/32", "domain_mapping", "google.com"), ("2607:f8b0::/48", "domain_mapping", "nested.example"),
          ("2607:f8b0:4000::/36", "sinkhole", "v6 sinkhole"), ("2a00:1450::/32", "domain_mapping", "google.com"),
          ("2a00:1450::/32", "domain_mapping", "v6only.example"), ("2a00:1450:4000::/40", "domain_mapping", "cdn.test"),
          ("2a00:1450:4001::/48", "domain_mapping", "video.example"), ("2001:db8::/64", "domain_mapping", "late.example"),
          ("2001:db8::/96", "domain_mapping", "example.net"), ("2001:db8::1:0:0/96", "proxy", "p6"),
          ("fc00::/7", "domain_mapping", "mail.corp")]
    for k in range(200):   # random nested IPv4 / IPv6 mappings
        tag = MAPPED[int(rng.integers(0, len(MAPPED)))]
        if k % 2:
            ln = int(rng.integers(12, 25))
            a = mask(int(rng.integers(1, 224)) << 24 | int(rng.integers(0, 1 << 24)), ln, 32)
            d.append((v4s(a, ln), "domain_mapping", tag))
        else:
            ln = int(rng.integers(24, 65))
            a = mask(0x2600 << 112 | int(rng.integers(0, 1 << 16)) << 96 | int(rng.integers(0, 1 << 62)) << 32, ln, 128)
            d.append((v6s(a, ln), "domain_mapping", tag))
    return d


def archive(asn_lines, dom, fp):
    """A resource archive: one labeled fingerprint whose processes carry the
    table's ASNs (so the ASN moves the score), the tables."""
    rng = np.random.default_rng(SEED + 1)
    asns = sorted({int(l.split("\t")[1]) for l in asn_lines if "\t" in l and l.split("\t")[1].isdigit()})
    procs = []
    for k, name in enumerate(["chrome.exe", "firefox.exe", "curl", "python", "java", "outlook.exe", "teams.exe", "zoom"]):
        e = synth_db._proc_entry(rng, name, int(rng.integers(50, 500)), MAPPED, MAPPED, None, k == 3, {}, True)
        pick = rng.choice(len(asns), 40, replace=False)
        e["classes_ip_as"] = {str(asns[int(j)]): int(rng.integers(1, e["count"] + 1)) for j in pick}
        for a in (15169, 15170, 8075, 8068):
            if rng.random() < 0.6:
                e["classes_ip_as"][str(a)] = int(rng.integers(1, e["count"] + 1))
        procs.append(e)
    files = {
        "VERSION": "2026.01.01; 2.0.dual\n",
        "fingerprint_db.json": json.dumps({"str_repr": fp, "fp_type": "tls", "total_count": sum(p["count"] for p in procs),
                                           "process_info": procs}) + "\n",
        "fp_prevalence_tls.txt": "",
        "pyasn.db": "\n".join(asn_lines) + "\n",
        "doh-watchlist.txt": "",
        "domain-mappings.db": "".join(json.dumps({"subnet": s, "type": t, "tag": g}) + "\n" for s, t, g in dom),
    }
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tf:
        for name, text in files.items():
            data = text.encode()
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            ti.mtime = 1700000000
            tf.addfile(ti, io.BytesIO(data))
    return buf.getvalue()


def queries(rng, pref, dom):
    out = []
    names = MAPPED + ["www." + m for m in MAPPED[:4]] + ["unmapped.example", ""]

    def text(bits, a):
        return str(ipaddress.IPv6Address(a)) if bits == 128 else str(ipaddress.IPv4Address(a))

    def pick():
        return names[int(rng.integers(0, len(names)))]
    spans = list(pref)
    for s, _, _ in dom:
        a, ln = s.split("/")
        if ":" in a:
            spans.append((128, int(ipaddress.IPv6Address(a)), int(ln)))
        else:
            spans.append((32, int(ipaddress.IPv4Address(a)), int(ln)))
    for bits, a, ln in spans:
        a = mask(a, ln, bits)
        top = a + (1 << (bits - ln)) - 1
        for x in (a, top, a + int(rng.integers(0, 1 << min(62, bits - ln))) if bits - ln else a, a - 1, top + 1):
            if 0 <= x < (1 << bits):
                out.append((text(bits, x), pick()))
    # the /32 outside its /48, inside the /48, outside both
    for x in ("2607:f8b0::5", "2607:f8b0:0:1::5", "2607:f8b0:1::5", "2607:f8b0:ffff::1", "2607:f8b1::1", "2607:f8af::1"):
        for nm in ("google.com", "nested.example", ""):
            out.append((x, nm))
    for _ in range(4000):
        if rng.random() < 0.5:
            out.append((text(32, int(rng.integers(1, 1 << 32))), pick()))
        else:
            out.append((text(128, int(rng.integers(0x2000, 0x2800)) << 112 | int(rng.integers(0, 1 << 62)) << 50), pick()))
    return out


def packets(rng, qs, n=3000):
    """TLS ClientHellos (one client profile: one fingerprint) to a sample of the
    query destinations, carrying the queries' server names."""
    sel = rng.choice(len(qs), min(n, len(qs)), replace=False)
    pk = []
    for j in sel:
        ip, name = qs[int(j)]
        ch = synth.client_hello(np.random.default_rng(7), "openssl", name or "none.example")
        l4 = synth.tcp(ch, sport=40000 + int(j) % 20000)
        if ":" in ip:
            pk.append((1, synth.eth(synth.ipv6(l4, 6, dst=ipaddress.IPv6Address(ip).packed), 0x86dd)))
        else:
            pk.append((1, synth.eth(synth.ipv4(l4, 6, dst=int(ipaddress.IPv4Address(ip))))))
    return pk


def gz(path, data):
    with open(path, "wb") as f:
        f.write(gzip.compress(data, mtime=0))


def main():
    rng = np.random.default_rng(SEED)
    asn_lines, pref = asn_table(rng)
    dom = domain_table(rng)
    qs = queries(rng, pref, dom)
    tmp = "/tmp/mfp_lpm"
    os.makedirs(tmp, exist_ok=True)
    with open(f"{tmp}/asn.db", "w") as f:
        f.write("\n".join(asn_lines) + "\n")
    with open(f"{tmp}/dom.tsv", "w") as f:
        # the pairs process_domain_mapping_line makes (analysis.h:797-815)
        f.write("".join(f"{s}\t{g if t == 'domain_mapping' else t}\n" for s, t, g in dom))
    with open(f"{tmp}/q.tsv", "w") as f:
        f.write("".join(f"{ip}\t{nm}\n" for ip, nm in qs))
    ref = subprocess.run([REF, "lpm", f"{tmp}/asn.db", f"{tmp}/dom.tsv", f"{tmp}/q.tsv"], capture_output=True,
                         check=True).stdout
    gz(os.path.join(HERE, "lpm_queries.tsv.gz"), "".join(f"{ip}\t{nm}\n" for ip, nm in qs).encode())
    gz(os.path.join(HERE, "lpm_ref.tsv.gz"), ref)
    # end to end: packets through the analysis path
    pk = packets(rng, qs)
    arena, desc = pcaplib.make_batch(pk)
    pcaplib.write_mfpb(f"{tmp}/p.mfpb", arena, desc)
    fpo = subprocess.run([REF, "fp", f"{tmp}/p.mfpb", "select=tls;format=tls/1"], capture_output=True,
                         check=True).stdout.decode().splitlines()
    fp = fpo[0].split("\t")[4]
    assert all(l.split("\t")[4] == fp for l in fpo), "one client profile, one fingerprint"
    data = archive(asn_lines, dom, fp)
    arch = os.path.join(HERE, "lpm_resources.tgz")
    with open(arch, "wb") as f:
        f.write(data)
    np.savez_compressed(os.path.join(HERE, "lpm_packets.npz"), arena=arena, desc=desc)
    for mode, name in (("an", "lpm_an.tsv.gz"), ("attr", "lpm_attr.tsv.gz")):
        out = subprocess.run([REF, mode, f"{tmp}/p.mfpb", "tls", arch], capture_output=True, check=True).stdout
        gz(os.path.join(HERE, name), out)
    rows = [l.split("\t") for l in ref.decode().splitlines()]
    info = {"queries": len(qs), "asn_lines": len(asn_lines), "domain_lines": len(dom), "packets": len(pk),
            "asn_nonzero": sum(r[2] != "0" for r in rows), "faking": sum(r[3] == "1" for r in rows),
            "gap_2607_f8b0_1__5": [r[2] for r in rows if r[0] == "2607:f8b0:1::5"][0]}
    json.dump(info, open(os.path.join(HERE, "lpm_manifest.json"), "w"), indent=1)
    print(json.dumps(info))


if __name__ == "__main__":
    main()
