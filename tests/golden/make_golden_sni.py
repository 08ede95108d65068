"""Golden server-name normalisations from the REFERENCE (server_identifier,
watchlist.hpp:326-390) via oracle/_ref/merc_ref_drv sni.  Dev container only.

    python tests/golden/make_golden_sni.py      -> tests/golden/sni_norm.tsv.gz
"""
import gzip
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
from tests import synth  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "merc_ref_drv")


def cases(seed=7, n=6000):
    rng = np.random.default_rng(seed)
    names = synth.names(rng)
    out = ["", "None", "localhost", "intranet", "example.com.", "*.example.com", "1.1.1.1:443", "10.1.2.3",
           "[::1]:443", "2001:db8::1", "::ffff:1.2.3.4", "[::ffff:10.0.0.1]:80", "fe80::1", "::", "1::",
           "a:b:c:d:e:f:1:2", "www.example.com:8443", ":443", "host:99999", "host:", "#comment", " lead.space.com",
           "1.2.3", "256.1.1.1", "1.2.3.4.5", "*.", "*", "-.-", "_a.b", "a.1", "1.a", "0.0.0.0", "192.168.1.1:8080",
           "172.20.1.1", "172.32.1.1", "fd00::5", "fc00::1", "2607:f8b0::2", "abc", "cafe", "cafe::", "cafe:babe",
           "x..y", "x.y..", "a.b.c.", "A.B.COM", "localhost:80", "None:1", "12345", "1.1.1.1.", "[2001:db8::1]",
           "[2001:db8::1]:443", "2001:0:0:1:0:0:0:1", "0:0:1:0:0:0:0:0", "1:0:0:2:0:0:0:3"]
    out += list(names[:800])
    alphabet = list("abcdefghijklmnopqrstuvwxyzABC0123456789.-_:[]* f")
    for _ in range(n):
        k = int(rng.integers(0, 4))
        if k == 0:
            out.append("".join(rng.choice(alphabet, int(rng.integers(1, 24)))))
        elif k == 1:
            b = list(names[int(rng.integers(0, len(names)))])
            for _ in range(int(rng.integers(1, 4))):
                b[int(rng.integers(0, len(b)))] = str(rng.choice(alphabet))
            out.append("".join(b))
        elif k == 2:
            out.append(".".join(str(int(x)) for x in rng.integers(0, 300, int(rng.integers(2, 6)))) +
                       (f":{int(rng.integers(0, 70000))}" if rng.random() < 0.5 else ""))
        else:
            parts = [format(int(x), "x") for x in rng.integers(0, 65536, int(rng.integers(1, 9)))]
            if rng.random() < 0.5 and len(parts) > 1:
                parts[int(rng.integers(0, len(parts)))] = ""
            s = ":".join(parts)
            out.append(f"[{s}]:{int(rng.integers(0, 70000))}" if rng.random() < 0.3 else s)
    return out


def main():
    items = cases()
    tmp = "/tmp/golden_sni.txt"
    with open(tmp, "w", encoding="latin-1") as f:
        for s in items:
            f.write(s + "\n")
    out = subprocess.run([REF, "sni", tmp], capture_output=True, check=True).stdout
    with gzip.open(os.path.join(HERE, "sni_norm.tsv.gz"), "wb") as f:
        f.write(out)
    os.unlink(tmp)
    print(len(items))


if __name__ == "__main__":
    main()
