"""Per-dispatch durations and counters (rocprofv3 csv) of the last bench step."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
rows = []
for f in glob.glob(os.path.join(d, "kt", "*kernel_trace.csv")):
    rows = list(csv.DictReader(open(f)))
rows = [r for r in rows if "mfp" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 7
for r in rows[-n:]:
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(f"{r['Kernel_Name'][:40]:40s} grid={r.get('Grid_Size', r.get('Grid_Size_X','?')):>10s} ms={dur:8.3f}")
pc = collections.OrderedDict()
for f in glob.glob(os.path.join(d, "p1", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "mfp" not in r["Kernel_Name"]:
            continue
        key = (int(r["Dispatch_Id"]), r["Kernel_Name"][:30])
        pc.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
keys = list(pc.keys())[-n:]
for k in keys:
    c = pc[k]
    print(k[1], " ".join(f"{x.replace('SQ_INSTS_','')}={c.get(x,0):.3g}" for x in
                         ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES"]))
