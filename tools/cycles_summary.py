"""Per kernel: mean duration, mean GRBM_GUI_ACTIVE / 8 (cycles of one XCD) and their quotient (the effective clock)
from a rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace directory. Usage: python tools/cycles_summary.py <dir> [label]"""
import csv
import glob
import sys
from collections import defaultdict

root, label = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
cyc, name = defaultdict(float), {}
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            cyc[r["Dispatch_Id"]] += float(r["Counter_Value"])
            name[r["Dispatch_Id"]] = r["Kernel_Name"]
dur = {}
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
agg = defaultdict(list)
for k, c in cyc.items():
    if k in dur:
        agg[name[k]].append((dur[k], c / 8))
for n, v in sorted(agg.items(), key=lambda kv: -sum(d for d, _ in kv[1]))[:4]:
    d = sum(x for x, _ in v) / len(v)
    c = sum(y for _, y in v) / len(v)
    print(f"{label:>14s} {n.split('(')[0][:40]:40s} n={len(v):3d} {d:9.1f} us {c / 1e3:9.1f} kcycles  {c / d:6.0f} MHz")
