"""Per-kernel averages of rocprofv3 --pmc passes (tools/pmc_kernels.sh): for every kernel name, the mean
per dispatch of each counter over all passes, plus derived ratios (MFMA busy share, LDS-stall share,
VALU instructions per MFMA). Usage: python tools/pmc_kernel_summary.py gpurun_out/<tag> [name filter]"""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    disp = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        k = r["Dispatch_Id"]
        disp[k][r["Counter_Name"]] += float(r["Counter_Value"])
        names[k] = r["Kernel_Name"]
    for k, c in disp.items():
        for n, v in c.items():
            acc[names[k]][n].append(v)
for name, cs in sorted(acc.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    if filt not in name:
        continue
    m = {n: sum(v) / len(v) for n, v in cs.items()}
    launches = max(len(v) for v in cs.values())
    line = f"{name[:70]:70s} n={launches}"
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
        line += f" mfma_busy={m['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * m['GRBM_GUI_ACTIVE'] / 8):.3f}"
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if n in m:
                line += f" {n[3:].lower()}={m[n] / wc:.3f}"
    if m.get("SQ_INSTS_MFMA"):
        line += f" valu/mfma={m.get('SQ_INSTS_VALU', 0) / m['SQ_INSTS_MFMA']:.2f} lds/mfma={m.get('SQ_INSTS_LDS', 0) / m['SQ_INSTS_MFMA']:.2f}"
    if m.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in m:
        line += f" bank_conflict_cyc/lds_inst={m['SQ_LDS_BANK_CONFLICT'] / m['SQ_INSTS_LDS']:.2f}"
    print(line)
    print("    " + " ".join(f"{n}={v:.4g}" for n, v in sorted(m.items())))
