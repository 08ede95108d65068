"""Compare the C oracle against the reference (oracle/_ref/merc_ref_drv) on a
set of pcaps / batch files.  Test infrastructure; run in the dev container.

    python oracle/compare_ref.py [--fmt N] [--mode fp|an] file.pcap ...
"""
import argparse
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import oracle  # noqa: E402
from tests import pcaplib  # noqa: E402

REF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref", "merc_ref_drv")
CONTRACT_SELECT = "tls,dtls,ssh,http,tcp,tcp.syn_ack"


def ref_config(fmt):
    if fmt == 0:
        return CONTRACT_SELECT
    return f"select={CONTRACT_SELECT};format=tls/{fmt}"


def run_ref(path, fmt=0, mode="fp", resources="-"):
    out = subprocess.run([REF, mode, path, ref_config(fmt), resources], capture_output=True, check=True)
    rows = []
    for line in out.stdout.decode("latin-1").splitlines():
        f = line.split("\t")
        rows.append(f)
    return rows


def compare_pkts(pkts, fmt=0, label="", verbose=True):
    arena, desc = pcaplib.make_batch(pkts)
    with tempfile.NamedTemporaryFile(suffix=".mfpb", delete=False) as t:
        path = t.name
    pcaplib.write_mfpb(path, arena, desc)
    try:
        ref = run_ref(path, fmt)
    finally:
        os.unlink(path)
    ft, fl, flags, strs = oracle.process_batch(arena, desc, oracle.config(tls_format=fmt))
    bad = 0
    for i, r in enumerate(ref):
        emit, t, trunc, s = int(r[1]), int(r[2]), int(r[3]), r[4] if len(r) > 4 else ""
        o_emit, o_trunc = int(flags[i] & 1), int((flags[i] >> 1) & 1) & int(flags[i] & 1)
        if (emit, t, trunc, s) != (o_emit, int(ft[i]), o_trunc, strs[i]):
            bad += 1
            if verbose and bad <= 5:
                print(f"MISMATCH {label} pkt {i}: ref emit={emit} type={t} trunc={trunc}\n  ref: {s[:300]}\n"
                      f"  ora: emit={o_emit} type={int(ft[i])} trunc={o_trunc}\n  ora: {strs[i][:300]}")
    return len(ref), bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fmt", type=int, default=None)
    ap.add_argument("files", nargs="+")
    a = ap.parse_args()
    fmts = [a.fmt] if a.fmt is not None else [0, 1, 2]
    tot_bad = 0
    for fn in a.files:
        pkts = pcaplib.read_pcap(fn)
        for fmt in fmts:
            n, bad = compare_pkts(pkts, fmt, label=f"{os.path.basename(fn)}/fmt{fmt}")
            tot_bad += bad
            print(f"{os.path.basename(fn)} fmt{fmt}: {n} pkts, {bad} mismatches")
    sys.exit(1 if tot_bad else 0)


if __name__ == "__main__":
    main()
