"""Summarise rocprofv3 csv output (kernel stats + --pmc passes) per kernel."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
for f in glob.glob(os.path.join(d, "kt", "*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:60]:60s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:9.3f}")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-30:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    if "k_" not in k:
        continue
    print(f"== {k}")
    for c, v in sorted(cs.items()):
        vv = v[1:] if len(v) > 1 else v
        print(f"  {c:24s} {sum(vv)/len(vv):.4g}   (n={len(v)})")
