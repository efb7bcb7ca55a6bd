"""Summary of tools/l2_attrib.sh: per PMC pass, the edge layer kernel's counters per launch
(rocprofv3 counter_collection CSVs), and the bench timing of each A-operand redirection.

    python tools/l2_summary.py gpurun_out/<tag>"""
import collections
import csv
import glob
import json
import os
import sys

KEY = "k_edge16_layer"


def counters(path):
    """{counter: mean value per launch of the edge layer kernel} over every CSV under path."""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if KEY in r["Kernel_Name"]:
                    per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {c: sum(v.values()) / len(v) for c, v in per.items() if v}


def main(root):
    for f in sorted(glob.glob(os.path.join(root, "bench_d*.json"))):
        try:
            line = [x for x in open(f) if x.startswith("{")][-1]
            d = json.loads(line)
            print(f"{os.path.basename(f)}: {d['ms_per_step']:.2f} ms/step, edge layer {d['roofline']['avg_ms']:.3f} ms")
        except Exception as e:  # noqa: BLE001
            print(f"{f}: {e!r}")
    for p in sorted(glob.glob(os.path.join(root, "pmc*")), key=lambda s: int(''.join(c for c in s if c.isdigit()) or 0)):
        if not os.path.isdir(p):
            continue
        spec = open(os.path.join(p, "spec.txt")).read().strip() if os.path.exists(os.path.join(p, "spec.txt")) else "?"
        c = counters(p)
        print(f"{os.path.basename(p)} [{spec}]")
        for k, v in sorted(c.items()):
            extra = ""
            if "RDREQ" in k:
                extra = f"  (x128 B = {v * 128 / 1e9:.2f} GB, x64 B = {v * 64 / 1e9:.2f} GB)"
            if k == "FETCH_SIZE":
                extra = f"  ({v * 1024 / 1e9:.2f} GB, x2 = {2 * v * 1024 / 1e9:.2f} GB)"
            print(f"   {k:28s} {v:.4g}{extra}")
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            h, m = c["TCC_HIT_sum"], c["TCC_MISS_sum"]
            print(f"   L2 hit rate {h / (h + m):.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
