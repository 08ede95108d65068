"""HBM traffic per bench step from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_traffic.py <fetch csv> <write csv> <config key> <out.json>

The passes profile `bench.py --steps K --warmup W ...`.  A step's kernels
start at a k_classify dispatch and run to the next one; the first group
(the sizing call on the unique packet set) and the warmup groups are
dropped and the median of the remaining groups is reported.  Correction per
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE (KiB) is
half the bytes of wide (16 B/lane) streaming reads on gfx950, so it is
doubled; WRITE_SIZE (KiB) is taken as is.  Accesses narrower than 16 B per
lane are uncalibrated (the guide says so), so the raw sums are kept too.
"""
import csv
import json
import statistics
import sys

MFP = ("k_classify", "k_fingerprint", "k_wave_fp", "k_analyze")


def groups(path):
    out, cur = [], None
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    for r in rows:
        name = r["Kernel_Name"]
        if not any(k in name for k in MFP):
            continue
        if "k_classify" in name:
            cur = {}
            out.append(cur)
        if cur is None:
            continue
        short = next(k for k in MFP if k in name)
        if "k_analyze_status" in name:
            short = "k_analyze_status"
        cur[short] = cur.get(short, 0.0) + float(r["Counter_Value"]) * 1024.0
    return out


def main():
    fetch_csv, write_csv, key, out = sys.argv[1:5]
    f, w = groups(fetch_csv), groups(write_csv)
    f, w = f[1:], w[1:]                      # drop the sizing call
    steps = f[len(f) // 2:], w[len(w) // 2:]  # the timed steps (warmup < steps in the profiled command)
    fr = statistics.median(sum(g.values()) for g in steps[0])
    wr = statistics.median(sum(g.values()) for g in steps[1])
    per_kernel = {}
    for k in steps[0][-1]:
        per_kernel[k] = {"fetch_raw": statistics.median(g.get(k, 0.0) for g in steps[0]),
                         "write_raw": statistics.median(g.get(k, 0.0) for g in steps[1])}
    res = {"config": key, "hbm_bytes_per_step": 2 * fr + wr, "fetch_bytes_raw": fr, "write_bytes_raw": wr,
           "correction": "FETCH_SIZE x2 (gfx950, 16-B streaming reads), WRITE_SIZE x1; KiB -> bytes",
           "per_kernel_raw": per_kernel, "fetch_csv": fetch_csv, "write_csv": write_csv}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("config", "hbm_bytes_per_step", "fetch_bytes_raw", "write_bytes_raw")}))


if __name__ == "__main__":
    main()
