"""Block timeline of one k_edge16_layer grid (CHM_EDGE_TRACE_LAYER=3 dump: per block {hw id, t0, t_main,
t_end, slot 4, slot 5}, s_memrealtime ticks of 10 ns; slot = blockIdx). Block kinds from the same
block -> job map as edge16.hip's layer_job. Usage: python tools/trace_layer.py dump.bin n_samples n_atoms [lag]"""
import sys
from collections import defaultdict

import numpy as np


def layer_job(b, R, P, D):
    x, k = b & 7, b >> 3
    lo, hi = R * x // 8, R * (x + 1) // 8
    n = hi - lo
    G, d = 2 + 2 * P, min(D, n)
    if k < 2 * d:
        i, s = k // 2, k % 2
    elif k - 2 * d < (n - d) * G:
        i, s = d + (k - 2 * d) // G, (k - 2 * d) % G
    else:
        k2 = k - 2 * d - (n - d) * G
        if k2 >= d * 2 * P:
            return 0
        i, s = n + k2 // (2 * P), 2 + k2 % (2 * P)
    return 1 if s < 2 else 2


def main():
    a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 6)
    B, n = int(sys.argv[2]), int(sys.argv[3])
    D = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    R = (B * n * n + 255) // 256
    nb = 8 * ((R + 7) // 8) * 6
    a = a[:nb]
    kind = np.array([layer_job(b, R, 2, D) for b in range(nb)])
    ok = a[:, 1] > 0
    hw = a[:, 0]
    t = a[:, 1:].astype(np.int64)
    base = t[ok, 0].min()
    t0, tm, te, t4 = (t[:, 0] - base) / 100, (t[:, 1] - base) / 100, (t[:, 2] - base) / 100, (t[:, 3] - base) / 100
    print(f"R {R} row tiles, {nb} blocks ({ok.sum()} traced), span {te[ok].max():.1f} us, CUs {len(np.unique(hw[ok]))}")
    for k, name in ((1, "layer 1"), (2, "layer 2")):
        m = ok & (kind == k)
        main = tm[m] - (t4[m] if k == 2 else t0[m])
        epi = te[m] - tm[m]
        print(f"{name}: {m.sum()} tiles  main {np.median(main):.1f} us (p10 {np.percentile(main, 10):.1f}, "
              f"p90 {np.percentile(main, 90):.1f})  epilogue {np.median(epi):.1f} us (p90 {np.percentile(epi, 90):.1f})"
              + (f"  wait {np.median(t4[m] - t0[m]):.2f} us (p90 {np.percentile(t4[m] - t0[m], 90):.2f}, "
                 f"max {np.max(t4[m] - t0[m]):.1f})" if k == 2 else
                 f"  epilogue to marker 4 {np.median(t4[m] - tm[m]):.1f} us"))
    cu = defaultdict(list)
    for i in np.nonzero(ok)[0]:
        cu[int(hw[i])].append(i)
    gaps = defaultdict(list)
    busy, span = [], []
    for idx in cu.values():
        idx = sorted(idx, key=lambda i: t0[i])
        for p, q in zip(idx, idx[1:]):
            gaps[(kind[p], kind[q])].append(t0[q] - te[p])
        busy.append(sum(te[i] - t0[i] for i in idx))
        span.append(te[idx[-1]] - t0[idx[0]])
    for kk, g in sorted(gaps.items()):
        print(f"gap after a layer-{kk[0]} tile before a layer-{kk[1]} tile on the same CU: median {np.median(g):.2f} us, "
              f"p90 {np.percentile(g, 90):.2f} ({len(g)})")
    print(f"per CU: busy {np.median(busy):.0f} us of span {np.median(span):.0f} us; last CU done at "
          f"{te[ok].max():.0f} us, first CU idle at {min(te[sorted(v, key=lambda i: te[i])[-1]] for v in cu.values()):.0f} us")
    tot = {1: 0.0, 2: 0.0}
    for k in (1, 2):
        m = ok & (kind == k)
        tot[k] = float((te[m] - t0[m]).sum())
    print(f"CU-time: layer 1 {tot[1] / 1e3:.0f} ms-CU ({tot[1] / max(1, len(cu)) / 1e3:.2f} ms per CU), layer 2 "
          f"{tot[2] / 1e3:.0f} ms-CU ({tot[2] / max(1, len(cu)) / 1e3:.2f} ms per CU)")


if __name__ == "__main__":
    main()
