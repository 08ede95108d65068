"""Per-kernel PMC summary of rocprofv3 --pmc passes over bench.py.

    python tools/pmc_kernels.py <out.json> <counter_collection.csv> [more csv ...]

Every pass profiles the same command (`bench.py --steps K --warmup W ...`).
Dispatches are labelled by their place in a step: a step starts at a
k_classify dispatch; the fingerprint launches after it are the protocol bins
in mfp_kernels.hip's order (tls_ch, http_req, tcp_syn, http_resp, other,
tls_sh, ssh, dtls), then the fallback lane; then k_analyze, k_analyze_wave,
k_analyze_status; any other dispatch (k_compact, calibration kernels) keeps
its own name.  The first step (the host-side sizing call) and the warmup
steps are dropped (the later half of the steps is kept) and each counter is
the median over the kept steps.

Derived, per kernel: HBM bytes with the calibrated corrections of
profiles/*calib*.json when given (--calib), else the guide's 16-B streaming
rule (FETCH_SIZE x2, WRITE_SIZE x1); SQ time split (WAIT_ANY, WAIT_INST_ANY,
ACTIVE_INST_ANY as fractions of WAVE_CYCLES) and instruction mix per wave.
"""
import csv
import json
import re
import statistics
import sys
from collections import defaultdict

BINS = ["tls_ch", "http_req", "tcp_syn", "http_resp", "other", "tls_sh", "ssh", "dtls"]
FP = re.compile(r"k_fingerprint|k_fp_seg|k_wave_fp|k_fp_tls|k_fp_")


def short(name):
    m = re.search(r"(k_[A-Za-z0-9_]+|c_[A-Za-z0-9_]+)", name)
    return m.group(1) if m else name


def label_dispatches(rows):
    """rows sorted by dispatch id -> list of (step index, label, row)."""
    out, step, fp_seen = [], -1, 0
    for r in rows:
        k = short(r["Kernel_Name"])
        if k == "k_classify":
            step += 1
            fp_seen = 0
            out.append((step, "k_classify", r))
            continue
        if FP.search(k) and step >= 0:
            lab = f"{k}/{BINS[fp_seen]}" if fp_seen < len(BINS) else f"{k}/fallback"
            fp_seen += 1
            out.append((step, lab, r))
            continue
        out.append((step, k, r))
    return out


def load(paths):
    """{label: {counter: [per-step values]}} over the kept steps of every pass."""
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        rows = list(csv.DictReader(open(p)))
        # one row per (dispatch, counter)
        by_disp = defaultdict(dict)
        meta = {}
        for r in rows:
            d = int(r["Dispatch_Id"])
            by_disp[d][r["Counter_Name"]] = by_disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta[d] = r
        disp = sorted(by_disp)
        labelled = label_dispatches([dict(meta[d], _d=d) for d in disp])
        nsteps = max([s for s, _, _ in labelled] + [-1]) + 1
        keep_from = 1 + (nsteps - 1) // 2 if nsteps > 1 else 0
        per = defaultdict(lambda: defaultdict(float))
        for s, lab, r in labelled:
            if nsteps and s < keep_from and s >= 0:
                continue
            for c, v in by_disp[r["_d"]].items():
                per[(s, lab)][c] += v
        for (s, lab), cs in per.items():
            for c, v in cs.items():
                acc[lab][c].append(v)
    return {lab: {c: statistics.median(v) for c, v in cs.items()} for lab, cs in acc.items()}


def derive(stats, calib=None):
    fetch_k = (calib or {}).get("fetch_factor", 2.0)
    write_k = (calib or {}).get("write_factor", 1.0)
    out = {}
    for lab, c in stats.items():
        d = dict(c)
        if "FETCH_SIZE" in c:
            d["hbm_read_bytes"] = c["FETCH_SIZE"] * 1024.0 * fetch_k
        if "WRITE_SIZE" in c:
            d["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024.0 * write_k
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS"):
                if k in c:
                    d[k + "/WAVE_CYCLES"] = round(c[k] / wc, 4)
        w = c.get("SQ_WAVES")
        if w:
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS",
                      "SQ_INSTS_SMEM"):
                if k in c:
                    d[k + "/wave"] = round(c[k] / w, 1)
        out[lab] = d
    return out


def main():
    args = sys.argv[1:]
    calib = None
    if args and args[0] == "--calib":
        calib = json.load(open(args[1]))
        args = args[2:]
    out, paths = args[0], args[1:]
    res = derive(load(paths), calib)
    json.dump({"kernels": res, "sources": paths, "calibration": calib}, open(out, "w"), indent=1, sort_keys=True)
    for lab in sorted(res):
        d = res[lab]
        keys = [k for k in ("hbm_read_bytes", "hbm_write_bytes", "SQ_WAIT_ANY/WAVE_CYCLES",
                            "SQ_ACTIVE_INST_ANY/WAVE_CYCLES", "SQ_INSTS_VALU/wave", "SQ_INSTS_VMEM_RD/wave")
                if k in d]
        print(lab, {k: (round(d[k] / 1e9, 3) if "bytes" in k else d[k]) for k in keys})


if __name__ == "__main__":
    main()
