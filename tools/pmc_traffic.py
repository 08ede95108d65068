"""HBM traffic per bench step from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_traffic.py <fetch csv> <write csv> <config key> <out.json>

The passes profile `bench.py --steps K --warmup W ...`.  A step's kernels
start at a k_classify dispatch and run to the next one; the first group
(the sizing call on the unique packet set) and the warmup groups are
dropped and the median of the remaining groups is reported, per launch in
dispatch order (the order mfp_profile_read reports the step's kernels in,
so bench.py can attach each launch's bytes to its own name) and in total.
Correction per /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE (KiB) is half the bytes of wide (16 B/lane) streaming reads on
gfx950, so it is doubled; WRITE_SIZE (KiB) is taken as is.  Accesses narrower
than 16 B per lane are uncalibrated (the guide says so; profiles/
r02_fetch_write_calibration.json holds the dword-load calibration), so the raw
sums are kept too.
"""
import csv
import json
import statistics
import sys

PREFIX = "k_"


def kname(full):
    """mfp kernel name with its template arguments, without the parameter list."""
    s = full.split("(")[0].strip()
    for p in ("void ", "mfp::", "mfpa::", "mfpk::"):
        s = s.replace(p, "")
    return s


def groups(path):
    out, cur = [], None
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    for r in rows:
        name = kname(r["Kernel_Name"])
        if not name.startswith(PREFIX):
            continue
        if name.startswith("k_classify"):
            cur = []
            out.append(cur)
        if cur is None:
            continue
        cur.append((name, float(r["Counter_Value"]) * 1024.0))
    return out


def main():
    fetch_csv, write_csv, key, out = sys.argv[1:5]
    f, w = groups(fetch_csv)[1:], groups(write_csv)[1:]      # drop the sizing call
    f, w = f[len(f) // 2:], w[len(w) // 2:]                  # the timed steps (warmup < steps)
    n = min(len(g) for g in f + w)
    launches = []
    for j in range(n):
        fr = statistics.median(g[j][1] for g in f)
        wr = statistics.median(g[j][1] for g in w)
        launches.append({"kernel": f[0][j][0], "fetch_raw": fr, "write_raw": wr, "hbm_bytes": 2 * fr + wr})
    fr = statistics.median(sum(x[1] for x in g) for g in f)
    wr = statistics.median(sum(x[1] for x in g) for g in w)
    res = {"config": key, "hbm_bytes_per_step": 2 * fr + wr, "fetch_bytes_raw": fr, "write_bytes_raw": wr,
           "correction": "FETCH_SIZE x2 (gfx950, 16-B streaming reads), WRITE_SIZE x1; KiB -> bytes",
           "per_launch": launches, "fetch_csv": fetch_csv, "write_csv": write_csv}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("config", "hbm_bytes_per_step", "fetch_bytes_raw", "write_bytes_raw")}))
    for x in launches:
        print(f"  {x['kernel']:50s} {x['hbm_bytes'] / 1e9:8.3f} GB")


if __name__ == "__main__":
    main()
