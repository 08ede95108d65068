"""Summarise tools/calib_fetch under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
(one pass each) into the calibration JSON profiles/<tag>_fetch_write_calibration.json:
per pattern kernel, factor = known bytes (2 GiB) / (counter KiB x 1024).
    python tools/calib_summary.py <cal_f csv> <cal_w csv> <out.json>"""
import csv
import json
import sys

KNOWN = 2 << 30


def per_kernel(path, counter):
    out = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        name = row["Kernel_Name"].split("(")[0]
        if not name.startswith("c_"):
            continue
        out[name] = out.get(name, 0.0) + float(row["Counter_Value"]) * 1024
    return out


def main():
    f, w, dst = sys.argv[1:4]
    fb, wb = per_kernel(f, "FETCH_SIZE"), per_kernel(w, "WRITE_SIZE")
    pats = {}
    for k in sorted(set(fb) | set(wb)):
        p = {"FETCH_SIZE_raw_bytes": fb.get(k, 0.0)}
        if fb.get(k):
            p["FETCH_SIZE_factor"] = round(KNOWN / fb[k], 3)
        p["WRITE_SIZE_raw_bytes"] = wb.get(k, 0.0)
        if wb.get(k):
            p["WRITE_SIZE_factor"] = round(KNOWN / wb[k], 3)
        pats[k] = p
    json.dump({"what": "tools/calib_fetch under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE on MI355X (one pass each), "
                       "2 GiB per pattern; factor = known bytes / (counter KiB x 1024)", "patterns": pats},
              open(dst, "w"), indent=1)


if __name__ == "__main__":
    main()
