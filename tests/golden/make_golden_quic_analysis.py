"""--analysis on QUIC Initials: a resource archive in the reference's format
whose fingerprints are the quic/1 fingerprints the reference computes for
tests/golden/quic_packets.npz, and the reference's classifier results on those
packets.  Run in the dev container (needs oracle/_ref):

    python tests/golden/make_golden_quic_analysis.py

Outputs (committed):
  quic_resources.tgz     VERSION, fp_prevalence_tls.txt (empty),
                         fingerprint_db.json (fp_type "quic": 60 % of
                         the distinct fingerprints labeled, P ~ Zipf, server
                         names / QUIC user agents / ports / ASNs / addresses as
                         features), pyasn.db, doh-watchlist.txt,
                         domain-mappings.db
  quic_an.tsv.gz         merc_ref_drv an: idx valid fp_type status process score
                         malware p_malware fingerprint
  quic_attr.tsv.gz       merc_ref_drv attr: idx valid status attributes os_info alpn
The archive's quic entries are format 1, so the reference (and the device)
fingerprint QUIC with quic/1 (pkt_proc.h:97-99).
"""
import gzip
import io
import json
import os
import subprocess
import sys
import tarfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
from tests import pcaplib, synth_db  # noqa: E402
from oracle.compare_ref import REF  # noqa: E402

SELECT = "quic"
SNIS = ["www.example.com", "cdn.video.example.net", "api.service.test", "quic.tech", "a.b.c.d.e.example.org",
        "quic.inner.test"]
UAS = ["Chrome/120.0.6099.71 Windows NT 10.0", "quic-go/0.42"] + [f"agent/{k}" for k in range(0, 600, 7)]


def build(seed=0x5EED0A1C):
    rng = np.random.default_rng(seed)
    fps = []
    with gzip.open(os.path.join(HERE, "quic_fp_q1.tsv.gz"), "rt", encoding="latin-1") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            if len(p) > 4 and p[2] == "12" and p[4]:
                fps.append(p[4])
    fps = sorted(set(fps))
    rng.shuffle(fps)
    labeled = fps[: int(len(fps) * 0.6)]
    lines = []
    for fp in labeled:
        P = int(min(40, rng.zipf(1.5)))
        names = list(rng.choice(synth_db.PROC_NAMES, P, replace=False))
        procs = []
        for k in range(P):
            e = synth_db._proc_entry(rng, names[k], int(rng.integers(1, 500)), SNIS, [synth_db.tld_domain(s) for s in SNIS],
                                     UAS, rng.random() < 0.15, {a: rng.random() < 0.2 for a in synth_db.ATTRS}, True)
            procs.append(e)
        lines.append(json.dumps({"str_repr": fp, "fp_type": "quic", "total_count": sum(p["count"] for p in procs),
                                 "process_info": procs}))
    files = {
        "VERSION": "2026.01.01; 2.0.dual\n",
        "fingerprint_db.json": "\n".join(lines) + "\n",
        "fp_prevalence_tls.txt": "",
        # 2607:f8b0::/32 holds one /48: the reference's IPv6 LC-trie finds no
        # ASN in the /32 outside the /48 (tests/test_lpm.py), as the device does
        "pyasn.db": "\n".join(synth_db.ASN_LINES) + "\n",
        "doh-watchlist.txt": "quic.tech\nwww.example.com\n13.89.178.27\n",
        "domain-mappings.db": "".join(json.dumps(x) + "\n" for x in [
            {"subnet": "13.89.0.0/16", "type": "domain_mapping", "tag": "example.net"},
            {"subnet": "8.8.0.0/16", "type": "domain_mapping", "tag": "service.test"}]),
    }
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tf:
        for name, text in files.items():
            data = text.encode()
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            ti.mtime = 1700000000
            tf.addfile(ti, io.BytesIO(data))
    return buf.getvalue(), {"fingerprints": len(fps), "labeled": len(labeled)}


def main():
    data, info = build()
    arch = os.path.join(HERE, "quic_resources.tgz")
    with open(arch, "wb") as f:
        f.write(data)
    z = np.load(os.path.join(HERE, "quic_packets.npz"))
    tmp = "/tmp/quic_an.mfpb"
    pcaplib.write_mfpb(tmp, z["arena"], z["desc"])
    for mode, name in (("an", "quic_an.tsv.gz"), ("attr", "quic_attr.tsv.gz")):
        out = subprocess.run([REF, mode, tmp, SELECT, arch], capture_output=True, check=True).stdout
        with gzip.open(os.path.join(HERE, name), "wb") as f:
            f.write(out)
    os.unlink(tmp)
    rows = [l.split(b"\t") for l in gzip.open(os.path.join(HERE, "quic_an.tsv.gz")).read().splitlines()]
    st = {}
    for r in rows:
        if r[1] == b"1":
            st[int(r[3])] = st.get(int(r[3]), 0) + 1
    print(json.dumps({**info, "statuses": st}))


if __name__ == "__main__":
    main()
