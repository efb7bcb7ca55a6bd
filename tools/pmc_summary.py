"""Per-dispatch PMC summary (rocprofv3 counter_collection CSVs under the given dirs)."""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        rows = list(csv.DictReader(open(f)))
        disp = defaultdict(dict)
        names = {}
        for r in rows:
            k = int(r["Dispatch_Id"])
            disp[k][r["Counter_Name"]] = disp[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[k] = r["Kernel_Name"][:40]
        print(f)
        for k in sorted(disp):
            c = disp[k]
            print(f"  {k:3d} {names[k]:40s} " + " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
