"""The schedule of both edge layers in one grid on pairs (k_edge16_pairs_grid, edge16.hip pair_plan),
checked on the CPU through chm_debug_pair_plan: every layer-2 row tile runs exactly once, in one list; every S row
it reads comes from a pair tile inside its list's pair range and its [lo, hi] range; every pair tile it reads is
listed earlier in the same list (so its wait is for work already taken: no deadlock); every index the
kernel derives (pair flags, job entries) stays inside its buffer."""

import ctypes

import numpy as np
import pytest

from chemeleon_amd import _lib

PBM, BM = 128, 256


def plan(nat, P=2, lag=10):
    L = _lib.load()
    arr = (ctypes.c_int32 * len(nat))(*nat)
    E = sum(n * n for n in nat)
    R = (E + BM - 1) // BM
    rng = (ctypes.c_int32 * (2 * R))()
    pa, pb, nj = (ctypes.c_int32 * 8)(), (ctypes.c_int32 * 8)(), (ctypes.c_int32 * 8)()
    J = L.chm_debug_pair_plan(arr, len(nat), P, lag, rng, 2 * R, pa, pb, nj, None, 0)
    assert J >= 0, L.chm_last_error()
    jobs = (ctypes.c_int32 * (2 * 8 * max(J, 1)))()
    assert L.chm_debug_pair_plan(arr, len(nat), P, lag, rng, 2 * R, pa, pb, nj, jobs, 2 * 8 * max(J, 1)) == J
    return (np.array(rng).reshape(R, 2), np.array(pa), np.array(pb), np.array(nj),
            np.array(jobs).reshape(8, max(J, 1), 2), R)


def pair_index(nat):
    """(crystal, i, j) -> global pair index, crystal-major, row-major i <= j (the batch's pair table)."""
    idx, p = {}, 0
    for g, n in enumerate(nat):
        for i in range(n):
            for j in range(i, n):
                idx[(g, i, j)] = p
                p += 1
    return idx, p


@pytest.mark.parametrize("nat", [[40] * 64, [23, 7, 40, 1, 80] * 23, [1] * 300 + [2] * 70 + [3] * 9, [5, 9, 3],
                                 [80] * 9, [40] * 512, list(np.random.default_rng(7).integers(1, 81, 256))])
def test_pair_plan_covers_every_row_tile_with_its_pairs(nat):
    nat = [int(n) for n in nat]
    P = 2
    rng, pa, pb, nj, jobs, R = plan(nat, P)
    E = sum(n * n for n in nat)
    pidx, Ep = pair_index(nat)
    NP = (Ep + PBM - 1) // PBM
    # the pair tiles each directed edge row comes from
    src = np.empty(E, dtype=np.int64)
    r = 0
    for g, n in enumerate(nat):
        for i in range(n):
            for j in range(n):
                src[r] = pidx[(g, min(i, j), max(i, j))] // PBM
                r += 1
    owner = -np.ones(R, dtype=np.int64)
    for x in range(8):
        seen_pairs, npx = set(), pb[x] - pa[x]
        assert 0 <= pa[x] <= pb[x] <= NP
        for k in range(nj[x]):
            kind, tid = jobs[x, k]
            if kind == 1:
                p = tid // 2
                assert pa[x] <= p < pb[x] and 0 <= p - pa[x] < max(npx, 1)
                seen_pairs.add((p, tid % 2))
            else:
                assert kind == 2
                t, c = tid // (2 * P), (tid // 2) % P
                assert 0 <= t < R
                lo, hi = rng[t]
                rows = src[t * BM:min(E, t * BM + BM)]
                assert rows.min() >= lo and rows.max() <= hi, f"row tile {t} reads pair tiles outside [{lo}, {hi}]"
                assert pa[x] <= lo and hi < pb[x], f"row tile {t} on XCD {x} reads pair tiles outside its range"
                for p in range(lo, hi + 1):  # the waits are for jobs listed earlier on this XCD
                    assert (p, 0) in seen_pairs and (p, 1) in seen_pairs, f"row tile {t} waits for a later pair tile {p}"
                if c == 0 and tid % 2 == 0:
                    assert owner[t] == -1, f"row tile {t} scheduled twice"
                    owner[t] = x
    assert (owner >= 0).all(), "a row tile is never scheduled"
    # each row tile's 2 P jobs are all there
    counts = np.zeros(R, dtype=np.int64)
    for x in range(8):
        for k in range(nj[x]):
            if jobs[x, k, 0] == 2:
                counts[jobs[x, k, 1] // (2 * P)] += 1
    assert (counts == 2 * P).all()


@pytest.mark.parametrize("nat", [[40] * 64, [23, 7, 40, 1, 80] * 23, [1] * 300 + [2] * 70 + [3] * 9, [5, 9, 3],
                                 [80] * 9, [79, 78, 2, 80], list(np.random.default_rng(7).integers(1, 81, 256))])
def test_pair_tile_node_ranges_cover_their_pairs(nat):
    """The node range each pair tile's epilogue stages (chm_debug_pair_nodes, batch creation): every node i and j
    of the tile's pairs lies inside it, and it starts at the tile's first node (no row is staged below it)."""
    nat = [int(n) for n in nat]
    L = _lib.load()
    arr = (ctypes.c_int32 * len(nat))(*nat)
    NP = L.chm_debug_pair_nodes(arr, len(nat), None, 0)
    _, Ep = pair_index(nat)
    assert NP == (Ep + PBM - 1) // PBM
    out = (ctypes.c_int32 * (2 * NP))()
    assert L.chm_debug_pair_nodes(arr, len(nat), out, 2 * NP) == NP
    rng = np.array(out).reshape(NP, 2)
    # the pairs' nodes, crystal-major, row-major i <= j
    off = np.concatenate([[0], np.cumsum(nat)])
    pi, pj = [], []
    for g, n in enumerate(nat):
        for i in range(n):
            for j in range(i, n):
                pi.append(off[g] + i)
                pj.append(off[g] + j)
    pi, pj = np.array(pi), np.array(pj)
    for k in range(NP):
        a, b = k * PBM, min(Ep, k * PBM + PBM)
        lo, n = rng[k]
        nodes = np.concatenate([pi[a:b], pj[a:b]])
        assert lo == pi[a] and nodes.min() == lo and nodes.max() < lo + n, f"pair tile {k}: [{lo}, {lo + n})"
        assert n >= 1 and lo + n <= off[-1]
