"""Per-dispatch counter table from rocprofv3 --pmc CSVs (one row per kernel
dispatch of the LAST bench step), so that the launches of one kernel for
different bins can be told apart.  usage: pmc_dispatch.py <dir> [n_last]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 12
rows = collections.OrderedDict()
for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "mfp" not in r["Kernel_Name"]:
            continue
        key = (os.path.basename(os.path.dirname(f)), int(r["Dispatch_Id"]))
        e = rows.setdefault(key, {"name": r["Kernel_Name"].split("(")[0][-24:], "grid": r["Grid_Size"]})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
by_pass = collections.defaultdict(list)
for (p, did), e in rows.items():
    by_pass[p].append((did, e))
for p, lst in sorted(by_pass.items()):
    lst.sort()
    print(f"== {p}")
    for did, e in lst[-n_last:]:
        cs = " ".join(f"{k}={v:.3g}" for k, v in e.items() if k not in ("name", "grid"))
        print(f"  {did:5d} {e['name']:24s} {cs}")
