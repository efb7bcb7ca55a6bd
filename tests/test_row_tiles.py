"""Host logic of edge layer 2's row tiles (chm_debug_row_tiles, no GPU): for fc batches the tile
table must list, for every 256-row tile of the edge rows (grouped by source node, node v's n rows
from its crystal's offset + i n), the nodes that start in it, the node continued from the previous
tile and that node's offset in the continued-rows buffer. Checked against a direct Python
construction on uniform, ragged and degenerate batches."""

import collections
import ctypes

import numpy as np
import pytest

from chemeleon_amd import _lib


def tile_start(t, nbig):
    """Row tile t's first edge row: 256-row tiles, or on a mixed tiling (nbig >= 0) 256-row tiles before nbig and
    192-row tiles from there on."""
    return 256 * t if nbig < 0 or t <= nbig else 256 * nbig + 192 * (t - nbig)


def reference_tiles(natoms, nbig=-1):
    starts, ends = [], []
    e = 0
    for n in natoms:
        for _ in range(n):
            starts.append(e)
            ends.append(e + n)
            e += n
    E, N = e, len(starts)
    R = (E + 255) // 256 if nbig < 0 else nbig + (E - 256 * nbig + 191) // 192
    rows, r2 = [], 0
    for t in range(R):
        s0 = tile_start(t, nbig)
        x = next((v for v in range(N) if starts[v] >= s0), N)
        y = next((v for v in range(N) if starts[v] >= tile_start(t + 1, nbig)), N)
        c = next((v for v in range(N) if starts[v] < s0 < ends[v]), -1)
        off = 0
        if c >= 0:
            off = r2
            r2 += ends[c] - s0
        rows.append((x, y, c, off))
    return rows, r2


def native_tiles(natoms, nbig=-1):
    lib = _lib.load()
    nat = (ctypes.c_int32 * len(natoms))(*natoms)
    r2 = ctypes.c_int64()
    R = lib.chm_debug_row_tiles_ex(nat, len(natoms), nbig, None, 0, ctypes.byref(r2))
    assert R > 0, _lib.load().chm_last_error()
    out = (ctypes.c_int32 * (4 * R))()
    assert lib.chm_debug_row_tiles_ex(nat, len(natoms), nbig, out, 4 * R, ctypes.byref(r2)) == R
    if nbig < 0:  # (the uniform entry point agrees)
        out2 = (ctypes.c_int32 * (4 * R))()
        assert lib.chm_debug_row_tiles(nat, len(natoms), out2, 4 * R, None) == R and list(out2) == list(out)
    return [tuple(out[4 * k:4 * k + 4]) for k in range(R)], r2.value


# mixed tilings (r6): (crystals, 256-row tiles before the 192-row ones)
MIXED = [([20] * 64, 64), ([20] * 64, 0), ([20] * 64, 99), ([40] * 16, 10), ([6] * 4, 0), ([1] * 600, 1),
         ([192, 1, 192, 37], 2), (np.random.default_rng(11).integers(1, 193, 80).tolist(), 100),
         ([80] * 9, 0), ([3, 190, 2] * 30, 57)]


@pytest.mark.parametrize("natoms", [
    [40] * 64, [20] * 64, [6] * 4, [80] * 9, [1] * 600, [16] * 16, [256], [1, 255, 2, 80, 3],
    np.random.default_rng(7).integers(1, 81, 300).tolist(),
])
def test_row_tiles_match_direct_construction(natoms):
    check_tiles(natoms, -1)


@pytest.mark.parametrize("natoms,nbig", MIXED)
def test_mixed_row_tiles_match_direct_construction(natoms, nbig):
    """Mixed tilings (256-row tiles, then 192-row ones): the same table on the shifted tile starts."""
    check_tiles(natoms, nbig)


def check_tiles(natoms, nbig):
    got, r2 = native_tiles(natoms, nbig)
    want, r2_want = reference_tiles(natoms, nbig)
    assert got == want
    assert r2 == r2_want
    # every node is finished exactly once: its head tile lists it, and it is continued at most once
    N = sum(natoms)
    listed = sorted(v for x, y, _, _ in got for v in range(x, y))
    assert listed == list(range(N))
    conts = [c for _, _, c, _ in got if c >= 0]
    assert len(conts) == len(set(conts))


def reference_nodes(natoms, nbig=-1):
    """Each row tile's node list as edge16.hip's segment-mean epilogue derived it on the device before the
    host-built table (EdgeArgs::rinfo): {node, rows in the tile | first row << 10 | kind << 20}, kind 0 = a
    whole node, 1 = the head part of a node cut at the tile end (listed first), 2 = the rest of a node
    begun in the previous tile (listed last)."""
    tiles, _ = reference_tiles(natoms, nbig)
    starts, nn = [], []
    e = 0
    for n in natoms:
        for _ in range(n):
            starts.append(e)
            nn.append(n)
            e += n
    E = e
    out = []
    for t, (x, y, c, _) in enumerate(tiles):
        e0 = tile_start(t, nbig)
        e1 = min(E, tile_start(t + 1, nbig))
        nreg = y - x
        head = nreg > 0 and starts[y - 1] + nn[y - 1] > e1
        lst = []
        for i in range(nreg):
            v = x + ((nreg - 1 if i == 0 else i - 1) if head else i)
            es, end = starts[v], starts[v] + nn[v]
            lst.append((v, (min(end, e1) - es) | ((es - e0) << 10) | ((1 << 20) if head and i == 0 else 0)))
        if c >= 0:
            lst.append((c, (starts[c] + nn[c] - e0) | (2 << 20)))
        out.append(lst)
    return out


@pytest.mark.parametrize("natoms", [
    [40] * 64, [20] * 64, [6] * 4, [80] * 9, [1] * 600, [16] * 16, [256], [1, 255, 2, 80, 3],
    np.random.default_rng(7).integers(1, 81, 300).tolist(),
])
def test_row_tile_node_lists(natoms):
    """The host-built node lists (chm_debug_row_nodes, the table edge layer 2's epilogue reads) equal the
    device's former derivation, restated here from the tile table, node starts and degrees; every
    node's rows are covered exactly once across its head and continued parts."""
    check_nodes(natoms, -1)


@pytest.mark.parametrize("natoms,nbig", MIXED)
def test_mixed_row_tile_node_lists(natoms, nbig):
    check_nodes(natoms, nbig)


def check_nodes(natoms, nbig):
    lib = _lib.load()
    nat = (ctypes.c_int32 * len(natoms))(*natoms)
    R = lib.chm_debug_row_nodes_ex(nat, len(natoms), nbig, None, 0, None, 0)
    assert R > 0, lib.chm_last_error()
    K = 260
    out = (ctypes.c_int32 * (2 * K * R))()
    cnt = (ctypes.c_int32 * R)()
    assert lib.chm_debug_row_nodes_ex(nat, len(natoms), nbig, out, 2 * K * R, cnt, R) == R
    if nbig < 0:
        out2 = (ctypes.c_int32 * (2 * K * R))()
        assert lib.chm_debug_row_nodes(nat, len(natoms), out2, 2 * K * R, None, 0) == R and list(out2) == list(out)
    want = reference_nodes(natoms, nbig)
    assert len(want) == R
    rows = collections.Counter()
    for t in range(R):
        got = [(out[2 * (t * K + i)], out[2 * (t * K + i) + 1]) for i in range(cnt[t])]
        assert got == want[t], f"tile {t}"
        assert all(out[2 * (t * K + i)] == 0 and out[2 * (t * K + i) + 1] == 0 for i in range(cnt[t], K))
        for v, w in got:
            rows[v] += w & 1023
    assert all(rows[v] == n for v, n in enumerate(n for n in natoms for _ in range(n)))


def test_row_tiles_reject_bad_batches():
    lib = _lib.load()
    nat = (ctypes.c_int32 * 2)(4, 0)
    assert lib.chm_debug_row_tiles(nat, 2, None, 0, None) < 0
    nat = (ctypes.c_int32 * 1)(300)
    assert lib.chm_debug_row_tiles(nat, 1, None, 0, None) < 0
    nat = (ctypes.c_int32 * 2)(20, 20)  # 800 rows: 4 tiles of 256 leave no short tile
    assert lib.chm_debug_row_tiles_ex(nat, 2, 4, None, 0, None) < 0
    assert lib.chm_debug_row_tiles_ex(nat, 2, 3, None, 0, None) == 4


@pytest.mark.parametrize("natoms,P,ncu,lmin,want", [
    ([20] * 64, 2, 256, 256, 64),     # configs[1]: 400 jobs on 256 CUs -> 64 tiles of 256 rows + 48 of 192
    ([20] * 64, 1, 256, 256, -1),     # 200 jobs: one partial round of 256-row tiles, too full (78%) for short ones
    ([40] * 64, 2, 256, 256, -1),     # 400 row tiles: the pair grid's uniform tiles
    ([40] * 64, 2, 256, 1000, 384),   # (below a raised edge_layer_min: 1600 jobs -> 6 full rounds + 22 short tiles)
    ([6] * 4, 2, 256, 256, 0),        # one partial round: all short tiles
    ([20] * 30, 2, 256, 256, 0),      # 188 jobs (73% of a round): 63 short tiles = 252 jobs
    ([20] * 32, 2, 256, 256, -1),     # 200 jobs (78%): 67 short tiles = 268 jobs
    ([20] * 40, 2, 256, 256, -1),     # 252 jobs (98%): the short tiles would need 268 jobs
    ([193] + [20] * 63, 2, 256, 256, -1),  # a crystal above 192 atoms
    ([20] * 64, 2, 0, 256, -1),       # no CU count
])
def test_short_row_tiles_choice(natoms, P, ncu, lmin, want):
    """The mixed tiling a batch takes (chm_debug_short_row_tiles, the rule batch creation applies): 256-row tiles
    for every full round of the CUs, the rest as 192-row tiles when they fit one round; else uniform."""
    lib = _lib.load()
    nat = (ctypes.c_int32 * len(natoms))(*natoms)
    got = lib.chm_debug_short_row_tiles(nat, len(natoms), P, ncu, lmin)
    assert got == want
    if got >= 0:
        E = sum(n * n for n in natoms)
        R = got + (E - 256 * got + 191) // 192
        assert (R - got) * 2 * P <= ncu and 256 * got < E


@pytest.mark.parametrize("R,P,lag", [(400, 2, 10), (3200, 2, 10), (1367, 1, 10), (256, 2, 1), (300, 2, 3),
                                     (7, 2, 10), (9, 1, 4), (17500, 2, 10)])
def test_layer_grid_schedule(R, P, lag):
    """The one-grid edge-layer kernel's block -> job map (chm_debug_layer_jobs, the same function the
    kernel runs): every layer-1 tile (row tile, column tile) and every layer-2 tile (row tile,
    conditioning, column tile) is run by exactly one block, and every layer-2 block comes after both
    layer-1 blocks of its rows in the same XCD's sequence (blockIdx = XCD + 8 k): the invariant that
    keeps the in-grid waits free of deadlock (a waiting block's producers were dispatched before it)."""
    lib = _lib.load()
    nb = lib.chm_debug_layer_jobs(R, P, lag, None, 0)
    assert nb > 0
    out = (ctypes.c_int64 * (2 * nb))()
    assert lib.chm_debug_layer_jobs(R, P, lag, out, 2 * nb) == nb
    jobs = np.frombuffer(out, dtype=np.int64).reshape(nb, 2)
    l1 = {}
    for b, (kind, bid) in enumerate(jobs):
        if kind == 1:
            assert bid not in l1
            l1[int(bid)] = b
    assert sorted(l1) == list(range(2 * R))
    seen = set()
    for b, (kind, bid) in enumerate(jobs):
        if kind != 2:
            continue
        assert bid not in seen
        seen.add(int(bid))
        r = int(bid) // 2 // P
        for c in (0, 1):
            p = l1[2 * r + c]
            assert p < b and p % 8 == b % 8, f"layer-2 block {b} (row tile {r}) before its producer {p}"
    assert sorted(seen) == list(range(2 * P * R))
    assert set(jobs[:, 0].tolist()) <= {0, 1, 2}


@pytest.mark.parametrize("P,lag", [(2, 10), (1, 10), (2, 1), (2, 3), (1, 4)])
def test_persistent_layer_sequence(P, lag):
    """The persistent one-grid kernel's per-XCD job sequence (chm_debug_layer_seq, the function the
    kernel runs): every local row gets its 2 layer-1 tiles and its 2 P layer-2 tiles exactly once, column tile 0 of a row
    (the job that claims a pool row) comes before its column tile 1, every layer-2 job of a row comes
    after both of that row's layer-1 jobs (a layer-2 job's waits always point to jobs taken earlier),
    and layer-2 rows never go back (the kernel's exit rule: once a layer-2 job's row is past the last
    valid row, so is every later job's)."""
    n = 6000
    out = (ctypes.c_int64 * (3 * n))()
    assert _lib.load().chm_debug_layer_seq(n, P, lag, out) == 0
    jobs = [tuple(out[3 * k:3 * k + 3]) for k in range(n)]
    seen = {}
    for k, (kind, row, sub) in enumerate(jobs):
        assert (kind, row, sub) not in seen
        seen[(kind, row, sub)] = k
        if kind == 1:
            assert sub in (0, 1)
            if sub == 1:
                assert seen[(1, row, 0)] < k
        else:
            assert kind == 2 and 0 <= sub < 2 * P and row >= 0
            assert seen[(1, row, 0)] < k and seen[(1, row, 1)] < k
    rows2 = [row for kind, row, _ in jobs if kind == 2]
    assert rows2 == sorted(rows2)
    for r in range(max(rows2)):
        assert all((2, r, s) in seen for s in range(2 * P)) and all((1, r, s) in seen for s in (0, 1))
