"""Synthetic resource archive in the reference's format (analysis.h:854-931,
python/build_mercury_resources.py): VERSION, fingerprint_db.json,
fp_prevalence_tls.txt, pyasn.db, doh-watchlist.txt, domain-mappings.db -- for
the synthetic traffic of tests/synth.py, so that the --analysis path is
exercised at benchmark scale (BASELINE config 4).

Two sizes:
  * build()            the test archive (tests/golden/synth_resources.tgz):
                       the traffic's fingerprints, P ~ Zipf(1.6) on 1..256,
                       os_info, attribute tags, an encrypted-DNS watchlist and
                       domain mappings (mapped, faked, exception, IPv6 and
                       more than 256 mapped domains);
  * build_survey()     the SURVEY 8(d) config-4 archive: ~20 000
                       fingerprints (the traffic's plus filler), P ~ Zipf on
                       1..256, ~100 000 pyasn prefixes; written on demand to a
                       git-ignored path (survey_path()).

The fingerprint strings, server names and user agents of the synthetic
templates come from the C oracle (test infrastructure), so a seeded batch has
a controlled fraction of labeled, randomized and unlabeled fingerprints.
"""
import io
import json
import os
import sys
import tarfile

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import oracle  # noqa: E402
from tests import synth  # noqa: E402

ATTRS = ["evasive_vpn", "external_proxy", "malware", "multi_hop_proxy", "remote_access_tool"]
PROC_NAMES = (["chrome.exe", "firefox.exe", "msedge.exe", "safari", "curl", "python", "java", "outlook.exe",
               "teams.exe", "slack", "zoom", "svchost.exe", "onedrive.exe", "dropbox", "spotify", "steam",
               "generic dmz process", "powershell.exe", "wget", "git"] + [f"proc{i:03d}" for i in range(700)])
OS_NAMES = ["cpe:/o:microsoft:windows_10", "cpe:/o:microsoft:windows_11", "cpe:/o:apple:mac_os_x", "cpe:/o:apple:iphone_os",
            "cpe:/o:google:android", "cpe:/o:canonical:ubuntu_linux", "cpe:/o:redhat:enterprise_linux", "cpe:/o:freebsd:freebsd"]

# dst addresses of tests/synth.py: 13.89.x.y (IPv4), 2607:f8b0::xx (IPv6)
ASN_LINES = ["13.0.0.0/8\t8075", "13.89.0.0/16\t8068", "13.89.178.0/24\t8069", "13.89.200.0/22\t14618",
             "13.89.64.0/18\t16509", "10.0.0.0/8\t64512", "2607:f8b0::/32\t15169", "2607:f8b0::/48\t15170"]


def template_info(seed, n_templates, workload="mixed"):
    """(fp_type, fp string, server name, user agent) per template, fmt 1, analysis mode."""
    tpl, _ = synth.templates(seed, n_templates, workload)
    from tests import pcaplib
    arena, desc = pcaplib.make_batch([(1, t) for t in tpl])
    cfg = oracle.config(tls_format=1, mode=1)
    out = []
    for i, t in enumerate(tpl):
        r = oracle.process(t, 1, cfg)
        fp = r.fp[:r.fp_len].decode("latin-1") if r.fp_type else ""
        sni = t[r.sni_off:r.sni_off + r.sni_len].decode("latin-1") if r.sni_len > 0 else ""
        ua = t[r.ua_off:r.ua_off + r.ua_len].decode("latin-1") if r.ua_len > 0 else ""
        out.append((int(r.fp_type), fp, sni, ua))
    del arena, desc
    return out


def _proc_entry(rng, name, total_share, snis, domains, uas, malware, attrs, is_tls):
    cnt = max(1, int(total_share))
    def spread(keys, k):
        keys = list(dict.fromkeys(keys))
        if not keys:
            return {}
        sel = rng.choice(len(keys), min(k, len(keys)), replace=False)
        return {keys[int(j)]: int(rng.integers(1, cnt + 1)) for j in sel}
    e = {
        "process": name,
        "count": cnt,
        "sha256": "00" * 32,
        "attributes": {a: bool(attrs.get(a, False)) for a in ATTRS},
        "malware": bool(malware),
        "os_info": {OS_NAMES[int(j)]: int(rng.integers(1, cnt + 1))
                    for j in rng.choice(len(OS_NAMES), int(rng.integers(0, 4)), replace=False)},
        "classes_port_applications": {"https": cnt} if is_tls else {"http": cnt},
        "classes_port_port": {"443": cnt} if is_tls else {"80": cnt, "8080": max(1, cnt // 3)},
        "classes_hostname_tld": {},
        "classes_hostname_domains": spread(domains, 6),
        "classes_hostname_sni": spread(snis, 6),
        "classes_ip_as": {str(a): int(rng.integers(1, cnt + 1)) for a in rng.choice([8075, 8068, 8069, 14618, 16509, 15169], 3, replace=False)},
        "classes_ip_ip": {f"13.89.{int(rng.integers(0, 256))}.{int(rng.integers(0, 256))}": int(rng.integers(1, cnt + 1))
                          for _ in range(4)},
    }
    if rng.random() < 0.5:
        e["classes_ip_as"]["unknown"] = 1
    if uas is not None:
        e["classes_user_agent"] = spread(uas, 4) if uas else {"None": cnt}
    return e


def tld_domain(name):
    parts = name.split(".")
    return ".".join(parts[-2:]) if len(parts) >= 2 else name


def doh_lines(rng, snis):
    """doh-watchlist.txt (watchlist::process_line watchlist.hpp:624-652): server
    names the traffic uses, destination addresses of the synthetic ranges, an
    IPv6 address, a comment, a blank line and lines the parser ignores."""
    pop = list(dict.fromkeys(snis))[:40]
    names_ = [pop[int(i)] for i in rng.choice(len(pop), min(12, len(pop)), replace=False)] if pop else []
    lines = ["# encrypted DNS resolvers"] + names_ + ["13.89.7.9", "13.89.200.1", "13.89.77.77", "2607:f8b0::11",
                                                       "", "dns.example.net", "not a host!", "*.wild.example.com"]
    return "".join(x + "\n" for x in lines)


def domain_lines(rng, snis):
    """domain-mappings.db (analysis.h:765-819): popular traffic domains mapped
    to the traffic's destination range (not faking), to other ranges (faking),
    with a "www." form, proxy/sinkhole exceptions inside the destination range,
    IPv6 mappings, a prefix given twice, malformed lines, and filler mappings so
    that more than 256 domains exist (domain indices are stored as uint8_t)."""
    pop = [s[4:] if s.startswith("www.") else s for s in dict.fromkeys(snis)][:60]
    out = []
    for k, d in enumerate(pop):
        if k % 3 == 0:
            out.append({"subnet": "13.89.0.0/16", "type": "domain_mapping", "tag": d})
        elif k % 3 == 1:
            out.append({"subnet": f"{8 + k % 40}.{k}.0.0/16", "type": "domain_mapping", "tag": d})
        else:
            out.append({"subnet": "13.89.0.0/18", "type": "domain_mapping", "tag": d})
            out.append({"subnet": "2607:f8b0::/40", "type": "domain_mapping", "tag": d})
    out += [{"subnet": "13.89.128.0/17", "type": "proxy", "tag": "corp proxy"},
            {"subnet": "13.89.200.0/24", "type": "sinkhole", "tag": "dns filter"},
            {"subnet": "13.89.0.0/16", "type": "domain_mapping", "tag": "proxy"},
            {"subnet": "13.89.0.0/20", "type": "domain_mapping", "tag": "twice.example"},
            {"subnet": "13.89.0.0/20", "type": "domain_mapping", "tag": "twice.example"},
            {"subnet": "2607:f8b0:4000::/36", "type": "sinkhole", "tag": "v6 sinkhole"},
            {"subnet": "10.0.0.0/8", "type": "domain_mapping", "tag": "private.example"}]
    for i in range(300):   # filler: domain indices past 255
        out.append({"subnet": f"100.{i // 256}.{i % 256}.0/24", "type": "domain_mapping", "tag": f"filler{i}.example"})
    if pop:   # a popular domain mapped only after the filler: its index is >= 256
        out.append({"subnet": "13.89.0.0/16", "type": "domain_mapping", "tag": "late-" + pop[0]})
        out.append({"subnet": "13.89.0.0/16", "type": "domain_mapping", "tag": pop[-1] + ".late"})
    lines = [json.dumps(x) for x in out] + ["not json", '{"subnet": "1.2.3.0/24", "type": "bogus", "tag": "x"}',
                                            '{"subnet": "1.2.3.0/0", "type": "domain_mapping", "tag": "zero.example"}']
    return "".join(x + "\n" for x in lines)


def build(seed=0x5EED00DB, n_templates=4096, labeled_frac=0.6, max_procs=256, workload="mixed", filler_fps=0,
          asn_prefixes=0, zipf=1.6):
    """Returns (archive bytes, info dict)."""
    rng = np.random.default_rng(seed)
    info = template_info(0x5EED0003, n_templates, workload)
    by_fp = {}
    for t, fp, sni, ua in info:
        if t not in (1, 3) or not fp:
            continue
        d = by_fp.setdefault(fp, {"type": t, "snis": [], "uas": []})
        d["snis"].append(sni)
        d["uas"].append(ua)
    fps = sorted(by_fp)
    rng.shuffle(fps)
    n_lab = int(len(fps) * labeled_frac)
    labeled, rest = fps[:n_lab], fps[n_lab:]
    known_unlabeled = rest[: len(rest) // 3]       # fp_prevalence_tls.txt
    lines = []
    first = True
    for fp in labeled:
        d = by_fp[fp]
        is_tls = d["type"] == 1
        P = int(min(max_procs, rng.zipf(zipf)))
        total = 0
        procs = []
        names = list(rng.choice(PROC_NAMES, P, replace=False))
        if P > 1 and rng.random() < 0.1:
            names[0] = "generic dmz process"
        for k in range(P):
            share = int(rng.integers(1, 500))
            mal = rng.random() < 0.1
            attrs = {a: rng.random() < 0.15 for a in ATTRS}
            if first:
                attrs = {a: False for a in ATTRS}
                first = False
            snis = d["snis"] + [synth.names(rng)[int(rng.integers(0, 10000))] for _ in range(3)]
            doms = [tld_domain(s) for s in snis]
            uas = [u for u in d["uas"] if u] if not is_tls else []
            procs.append(_proc_entry(rng, names[k], share, snis, doms, uas, mal, attrs, is_tls))
            total += procs[-1]["count"]
        line = {"str_repr": fp, "fp_type": "tls" if is_tls else "http", "total_count": total, "process_info": procs}
        if rng.random() < 0.05:
            line["feature_weights"] = {"as": 0.2, "domain": 0.1, "port": 0.01, "ip": 0.5, "sni": 0.9, "ua": 0.8}
        lines.append(json.dumps(line))
    # filler fingerprints (never in the traffic): table size of a production DB
    for k in range(filler_fps):
        cs = "".join(f"{int(x):04x}" for x in rng.integers(0, 0x10000, int(rng.integers(4, 30))))
        ex = "".join(f"({int(x):04x})" for x in np.sort(rng.integers(0, 0x100, int(rng.integers(3, 16)))))
        fp = f"tls/1/(0303)({cs})[{ex}]"
        P = int(min(max_procs, rng.zipf(zipf)))
        names = list(rng.choice(PROC_NAMES, P, replace=False))
        procs = []
        for j in range(P):
            sn = [synth.names(rng)[int(rng.integers(0, 10000))] for _ in range(2)]
            procs.append(_proc_entry(rng, names[j], int(rng.integers(1, 500)), sn, [tld_domain(x) for x in sn], None,
                                     rng.random() < 0.1, {a: rng.random() < 0.15 for a in ATTRS}, True))
        lines.append(json.dumps({"str_repr": fp, "fp_type": "tls", "total_count": sum(p["count"] for p in procs),
                                 "process_info": procs}))
    # the randomized-fingerprint entry (analysis.h:1062-1074)
    procs = [_proc_entry(rng, n, int(rng.integers(10, 200)), [synth.names(rng)[i] for i in range(8)],
                         [tld_domain(synth.names(rng)[i]) for i in range(8)], None, rng.random() < 0.3, {}, True)
             for n in ("chrome.exe", "firefox.exe", "curl")]
    lines.append(json.dumps({"str_repr": "tls/1/randomized", "fp_type": "tls", "total_count": sum(p["count"] for p in procs),
                             "process_info": procs}))
    files = {
        "VERSION": "2026.01.01; 2.0.dual\n",
        "fingerprint_db.json": "\n".join(lines) + "\n",
        "fp_prevalence_tls.txt": "".join(fp + "\n" for fp in known_unlabeled if fp.startswith("tls/")),
        "pyasn.db": "\n".join(ASN_LINES + asn_filler(rng, asn_prefixes)) + "\n",
        "doh-watchlist.txt": doh_lines(rng, [s for t, fp, s, u in info if t == 1]),
        "domain-mappings.db": domain_lines(rng, [s for t, fp, s, u in info if t == 1]),
    }
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tf:
        for name, text in files.items():
            data = text.encode()
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            ti.mtime = 1700000000
            tf.addfile(ti, io.BytesIO(data))
    return buf.getvalue(), {"fingerprints": len(fps), "labeled": n_lab, "known_unlabeled": len(known_unlabeled),
                            "filler": filler_fps, "asn_prefixes": len(ASN_LINES) + asn_prefixes}


def asn_filler(rng, n):
    """n random pyasn prefixes (/8../24) over public IPv4 space, nested or not."""
    out = []
    for _ in range(n):
        ln = int(rng.integers(8, 25))
        a = int(rng.integers(1, 224)) << 24 | int(rng.integers(0, 1 << 24))
        a &= (0xffffffff << (32 - ln)) & 0xffffffff
        out.append(f"{a >> 24}.{a >> 16 & 255}.{a >> 8 & 255}.{a & 255}/{ln}\t{int(rng.integers(1, 400000))}")
    return out


SURVEY = dict(seed=0x5EED5A7E, n_templates=4096, labeled_frac=0.6, filler_fps=19500, asn_prefixes=100000)


def survey_path():
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "_gen", "survey_resources.tgz")


def build_survey(path=None):
    """The config-4 archive (SURVEY 8(d) sizes), written to `path` (default
    survey_path()) unless it is already there; returns the path."""
    path = path or survey_path()
    if not os.path.exists(path):
        data, _ = build(**SURVEY)
        # gzip header without a timestamp: the same bytes wherever it is built
        import gzip
        data = gzip.compress(gzip.decompress(data), compresslevel=9, mtime=0)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path + ".tmp", "wb") as f:
            f.write(data)
        os.replace(path + ".tmp", path)
    return path


if __name__ == "__main__":
    import sys
    data, inf = build()
    with open(sys.argv[1] if len(sys.argv) > 1 else "/tmp/synth_resources.tgz", "wb") as f:
        f.write(data)
    print(inf, len(data))
