"""Host logic of edge layer 2's row tiles (chm_debug_row_tiles, no GPU): for fc batches the tile
table must list, for every 256-row tile of the edge rows (grouped by source node, node v's n rows
from its crystal's offset + i n), the nodes that start in it, the node continued from the previous
tile and that node's offset in the continued-rows buffer. Checked against a direct Python
construction on uniform, ragged and degenerate batches."""

import ctypes

import numpy as np
import pytest

from chemeleon_amd import _lib


def reference_tiles(natoms):
    starts, ends = [], []
    e = 0
    for n in natoms:
        for _ in range(n):
            starts.append(e)
            ends.append(e + n)
            e += n
    E, N = e, len(starts)
    R = (E + 255) // 256
    rows, r2 = [], 0
    for t in range(R):
        s0 = 256 * t
        x = next((v for v in range(N) if starts[v] >= s0), N)
        y = next((v for v in range(N) if starts[v] >= s0 + 256), N)
        c = next((v for v in range(N) if starts[v] < s0 < ends[v]), -1)
        off = 0
        if c >= 0:
            off = r2
            r2 += ends[c] - s0
        rows.append((x, y, c, off))
    return rows, r2


def native_tiles(natoms):
    lib = _lib.load()
    nat = (ctypes.c_int32 * len(natoms))(*natoms)
    r2 = ctypes.c_int64()
    R = lib.chm_debug_row_tiles(nat, len(natoms), None, 0, ctypes.byref(r2))
    assert R > 0, _lib.load().chm_last_error()
    out = (ctypes.c_int32 * (4 * R))()
    assert lib.chm_debug_row_tiles(nat, len(natoms), out, 4 * R, ctypes.byref(r2)) == R
    return [tuple(out[4 * k:4 * k + 4]) for k in range(R)], r2.value


@pytest.mark.parametrize("natoms", [
    [40] * 64, [20] * 64, [6] * 4, [80] * 9, [1] * 600, [16] * 16, [256], [1, 255, 2, 80, 3],
    np.random.default_rng(7).integers(1, 81, 300).tolist(),
])
def test_row_tiles_match_direct_construction(natoms):
    got, r2 = native_tiles(natoms)
    want, r2_want = reference_tiles(natoms)
    assert got == want
    assert r2 == r2_want
    # every node is finished exactly once: its head tile lists it, and it is continued at most once
    N = sum(natoms)
    listed = sorted(v for x, y, _, _ in got for v in range(x, y))
    assert listed == list(range(N))
    conts = [c for _, _, c, _ in got if c >= 0]
    assert len(conts) == len(set(conts))


def test_row_tiles_reject_bad_batches():
    lib = _lib.load()
    nat = (ctypes.c_int32 * 2)(4, 0)
    assert lib.chm_debug_row_tiles(nat, 2, None, 0, None) < 0
    nat = (ctypes.c_int32 * 1)(300)
    assert lib.chm_debug_row_tiles(nat, 1, None, 0, None) < 0
