"""Fingerprints with more than 4096 processes (k_analyze_huge): a resource
archive in the reference format whose STUN fingerprints have P = 4097..9000
processes, over the STUN packets of stun_ovpn_packets.npz; expected values
from the REFERENCE (oracle/_ref/merc_ref_drv an).  Run in the dev container:

    python tests/golden/make_golden_hugep.py

Outputs (committed): hugep_resources.tgz, hugep_an.tsv.gz, hugep_manifest.json
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

SIZES = [4097, 5000, 6144, 9000]


def main():
    rng = np.random.default_rng(0x5EED0013)
    z = np.load(os.path.join(HERE, "stun_ovpn_packets.npz"))
    tmp = "/tmp/hugep.mfpb"
    pcaplib.write_mfpb(tmp, z["arena"], z["desc"])
    out = subprocess.run([REF, "fp", tmp, "stun", "-"], capture_output=True, check=True).stdout.decode("latin-1")
    from collections import Counter
    freq = Counter(l.split("\t")[4] for l in out.splitlines() if l.split("\t")[2] == "16")
    fps = sorted(freq, key=lambda f: (-freq[f], f))   # the most frequent take the huge sizes
    uas = ["libjingle", "WebRTC", "first", "second", "Coturn-4.5.2 'dan Eider'"]
    lines, sizes = [], {}
    for k, fp in enumerate(fps):
        P = SIZES[k] if k < len(SIZES) else int(rng.integers(1, 40))
        sizes[fp] = P
        procs = []
        for j in range(P):
            e = synth_db._proc_entry(rng, f"hugeproc{k}.{j}", int(rng.integers(1, 300)), [], [], uas,
                                     rng.random() < 0.1, {a: rng.random() < 0.1 for a in synth_db.ATTRS}, False)
            e["classes_port_port"] = {"3478": e["count"], "19302": max(1, e["count"] // 4)}
            e["classes_ip_ip"] = {"3.132.228.249": int(rng.integers(1, e["count"] + 1))}
            procs.append(e)
        lines.append(json.dumps({"str_repr": fp, "fp_type": "stun", "total_count": sum(p["count"] for p in procs),
                                 "process_info": procs}))
    files = {"VERSION": "2026.01.01; 2.0.dual\n", "fingerprint_db.json": "\n".join(lines) + "\n",
             "fp_prevalence_tls.txt": "", "pyasn.db": "\n".join(synth_db.ASN_LINES + ["3.128.0.0/13\t16509"]) + "\n"}
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tf:
        for name, text in files.items():
            data = text.encode()
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            ti.mtime = 1700000000
            tf.addfile(ti, io.BytesIO(data))
    apath = os.path.join(HERE, "hugep_resources.tgz")
    with open(apath, "wb") as f:
        f.write(buf.getvalue())
    an = subprocess.run([REF, "an", tmp, "stun", apath], capture_output=True, check=True).stdout
    with gzip.open(os.path.join(HERE, "hugep_an.tsv.gz"), "wb") as f:
        f.write(an)
    rows = [l.split(b"\t") for l in an.splitlines()]
    huge = sum(1 for r in rows if r[1] == b"1" and sizes.get(r[8].decode("latin-1"), 0) > 4096)
    m = {"packets": len(rows), "fingerprints": len(fps), "sizes": SIZES, "valid": sum(r[1] == b"1" for r in rows),
         "valid_huge_p": huge, "archive_bytes": len(buf.getvalue())}
    json.dump(m, open(os.path.join(HERE, "hugep_manifest.json"), "w"), indent=1)
    print(m)
    os.unlink(tmp)


if __name__ == "__main__":
    main()
