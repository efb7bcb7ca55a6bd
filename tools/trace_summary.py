"""Summarise an edge-GEMM block timeline (CHM_EDGE_TRACE dump: per block {hw, t0, t_main, t_end},
s_memrealtime ticks of 10 ns)."""
import sys
from collections import defaultdict

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 6)
a = a[a[:, 1] > 0]
hw, t0, tm, te = a[:, 0], a[:, 1].astype(np.int64), a[:, 2].astype(np.int64), a[:, 3].astype(np.int64)
base = t0.min()
t0, tm, te = t0 - base, tm - base, te - base
print(f"blocks {len(a)}  span {te.max() / 100:.1f} us  CUs {len(np.unique(hw))}")
main, epi = (tm - t0) / 100, (te - tm) / 100
t4, t5 = a[:, 4].astype(np.int64) - base, a[:, 5].astype(np.int64) - base
ok = a[:, 4] > 0
if ok.any() and "--clock" in sys.argv:  # CHM_EDGE_DBG=4096: slots 4, 5 = s_memtime at block start / end
    f = (a[:, 5].astype(np.int64) - a[:, 4].astype(np.int64))[ok] / ((te - t0)[ok] / 100)
    print(f"shader clock over each block: median {np.median(f):.0f} MHz (p10 {np.percentile(f, 10):.0f}, "
          f"p90 {np.percentile(f, 90):.0f})")
elif ok.any():
    print(f"epilogue split (markers 4, 5): tm->4 {np.median((t4 - tm)[ok]) / 100:.1f} us, "
          f"4->5 {np.median((t5 - t4)[ok]) / 100:.1f} us, 5->end {np.median((te - t5)[ok]) / 100:.1f} us "
          f"({ok.sum()} blocks)")
print(f"per block: main {np.median(main):.1f} us (p10 {np.percentile(main, 10):.1f}, p90 {np.percentile(main, 90):.1f}), "
      f"epilogue {np.median(epi):.1f} us (p10 {np.percentile(epi, 10):.1f}, p90 {np.percentile(epi, 90):.1f})")
# per CU: busy fraction, and how much of each epilogue overlaps another block's main loop on the same CU
cu = defaultdict(list)
for i in range(len(a)):
    cu[int(hw[i])].append(i)
ov, tot, gaps = 0.0, 0.0, []
for k, idx in cu.items():
    idx = sorted(idx, key=lambda i: t0[i])
    for i in idx:
        for j in idx:
            if j == i:
                continue
            lo, hi = max(tm[i], t0[j]), min(te[i], tm[j])
            if hi > lo:
                ov += hi - lo
        tot += te[i] - tm[i]
    ends = sorted(te[i] for i in idx)
    starts = sorted(t0[i] for i in idx)
    gaps.append((ends[-1] - starts[0]) / 100)
print(f"epilogue time overlapped by another block's main loop on the same CU: {100 * ov / max(tot, 1):.1f}%")
print(f"CU active span: median {np.median(gaps):.1f} us, min {min(gaps):.1f}, max {max(gaps):.1f}")
# gap between one block's end marker and the next block's start on the same CU (store drain,
# wave teardown and dispatch)
ig = []
for k, idx in cu.items():
    idx = sorted(idx, key=lambda i: t0[i])
    ig += [(t0[b] - te[a_]) / 100 for a_, b in zip(idx, idx[1:]) if t0[b] > te[a_]]
if ig:
    print(f"inter-block gap on a CU: median {np.median(ig):.1f} us, p10 {np.percentile(ig, 10):.1f}, "
          f"p90 {np.percentile(ig, 90):.1f} ({len(ig)} gaps)")
# first-round phase offset between co-resident blocks
k0 = sorted(cu)[0]
for k in sorted(cu)[:3]:
    idx = sorted(cu[k], key=lambda i: t0[i])
    print(f"CU {k:#x}: " + " ".join(f"[{t0[i] / 100:.0f} {tm[i] / 100:.0f} {te[i] / 100:.0f}]" for i in idx[:8]))
# concurrency: fraction of CUs in their epilogue over time (10 us bins)
span = int(te.max())
bins = np.zeros(span // 1000 + 1)
for i in range(len(a)):
    lo, hi = int(tm[i]) // 1000, int(te[i]) // 1000
    bins[lo:hi + 1] += 1
frac = bins / len(cu)
print("CUs in epilogue per 10 us bin (first 40):", " ".join(f"{f:.2f}" for f in frac[:40]))
print(f"epilogue concurrency: mean {frac.mean():.2f}, p10 {np.percentile(frac, 10):.2f}, p90 {np.percentile(frac, 90):.2f}")
