"""Block timelines of one k_edge16_pairs_grid launch (CHM_EDGE_TRACE=file CHM_EDGE_TRACE_LAYER=4 with a library
built with CHM_BUILD_DEFS=-DCHM_GRID_TRACE=1): how well the static job lists pack the CUs.

Record per block (6 x u64, slot = blockIdx): hw id (XCC << 16 | SE << 8 | SH << 4 | CU), t0 (start), t_wait
(layer-2 jobs: the pair-tile wait is over; pair jobs: = t0), t_end, kind (1 pair, 2 layer 2), tile.
Times are s_memrealtime ticks (100 MHz). Usage: python tools/grid_trace.py trace.bin [label]
"""
import sys

import numpy as np

TICK_US = 0.01


def main(path, label=""):
    r = np.fromfile(path, dtype=np.uint64).reshape(-1, 6)
    r = r[r[:, 4] > 0]
    hw, t0, tw, t3, kind = r[:, 0], r[:, 1].astype(np.int64), r[:, 2].astype(np.int64), r[:, 3].astype(np.int64), r[:, 4]
    start, end = t0.min(), t3.max()
    span = (end - start) * TICK_US
    cus = np.unique(hw)
    busy = (t3 - t0).sum() * TICK_US
    waits = ((tw - t0)[kind == 2]).sum() * TICK_US
    pair, l2 = kind == 1, kind == 2
    print(f"{label} blocks {len(r)} (pair {pair.sum()}, layer 2 {l2.sum()}) on {len(cus)} CUs, span {span:.1f} us")
    print(f"  CU occupancy (block resident) {busy / (len(cus) * span):.3f}; of the resident time, layer-2 waits "
          f"{waits / busy:.3f}; work (no waits) {(busy - waits) / (len(cus) * span):.3f}")
    print(f"  per job: pair {((t3 - t0)[pair]).mean() * TICK_US:.1f} us (min {((t3 - t0)[pair]).min() * TICK_US:.1f}, "
          f"max {((t3 - t0)[pair]).max() * TICK_US:.1f}); layer 2 after its wait {((t3 - tw)[l2]).mean() * TICK_US:.1f} us "
          f"(min {((t3 - tw)[l2]).min() * TICK_US:.1f}, max {((t3 - tw)[l2]).max() * TICK_US:.1f}); "
          f"layer-2 wait mean {((tw - t0)[l2]).mean() * TICK_US:.2f} us, {(tw - t0 > 50)[l2].mean():.3f} of them > 0.5 us")
    # per CU: idle at the start, gaps between blocks, idle at the end
    head = tail = gaps = 0.0
    for c in cus:
        m = hw == c
        a, b = np.sort(t0[m]), np.sort(t3[m])
        ordr = np.argsort(t0[m])
        s_, e_ = t0[m][ordr], t3[m][ordr]
        head += (s_[0] - start) * TICK_US
        tail += (end - e_.max()) * TICK_US
        gaps += np.clip(s_[1:] - np.maximum.accumulate(e_)[:-1], 0, None).sum() * TICK_US
    tot = len(cus) * span
    print(f"  CU idle: before its first block {head / tot:.3f}, between blocks {gaps / tot:.3f}, after its last {tail / tot:.3f}")
    xcc = (hw >> 16) & 0xF
    fin = [(t3[xcc == x].max() - start) * TICK_US for x in range(8) if (xcc == x).any()]
    print("  per-XCD finish (us):", " ".join(f"{f:.0f}" for f in fin))
    # concurrency profile: resident blocks over time (10 bins)
    edges = np.linspace(start, end, 11)
    prof = []
    for i in range(10):
        lo, hi = edges[i], edges[i + 1]
        ov = np.clip(np.minimum(t3, hi) - np.maximum(t0, lo), 0, None).sum() / (hi - lo)
        wv = np.clip(np.minimum(tw, hi) - np.maximum(t0, lo), 0, None)[l2].sum() / (hi - lo)
        prof.append(f"{ov:.0f}/{wv:.0f}")
    print("  resident blocks / of them waiting, per tenth of the span:", " ".join(prof))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
