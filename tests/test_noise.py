"""Parity-mode noise for a shard (chemeleon_amd.noise): the rows a rank keeps of the reference's
global CPU draws (chemeleon.py:348-349, 400-404, 418, 435, 455) equal the same rows of the
single-process draws bit for bit, and the CPU generator ends in the same state. CPU only: the MT19937
continuation (chm_mt19937_uniform) is a host function of the C-ABI library."""

import ctypes

import pytest
import torch

from chemeleon_amd import _lib
from chemeleon_amd.noise import StepNoise, rand_rows


@pytest.mark.parametrize("seed,pre,shape,r0,r1", [
    (5, 0, (20480, 104), 2560, 5120),   # the 64x40 share of 512x40, fresh engine
    (7, 13, (100, 104), 0, 100),        # whole tensor, mid-block start
    (9, 623, (7, 3), 2, 5),             # starts one output before a twist
    (1, 1000, (1280, 104), 640, 1280),  # configs[1], second rank
    (3, 0, (1, 1), 0, 1),
    (3, 5, (624, 1), 0, 0),             # keeps nothing, still advances
])
def test_rand_rows_matches_torch_rand(seed, pre, shape, r0, r1):
    torch.manual_seed(seed)
    torch.rand(pre)
    ref = torch.rand(shape)
    after = torch.rand(50), torch.randn(40)
    torch.manual_seed(seed)
    torch.rand(pre)
    got = rand_rows(shape, r0, r1)
    assert torch.equal(got, ref[r0:r1])
    after2 = torch.rand(50), torch.randn(40)
    assert torch.equal(after[0], after2[0]) and torch.equal(after[1], after2[1])


def test_rand_rows_on_a_private_generator():
    g1 = torch.Generator().manual_seed(11)
    g2 = torch.Generator().manual_seed(11)
    ref = torch.rand((300, 104), generator=g1)
    got = rand_rows((300, 104), 17, 250, generator=g2)
    assert torch.equal(got, ref[17:250])
    assert torch.equal(g1.get_state(), g2.get_state())


@pytest.mark.parametrize("natoms,world", [([40] * 16, 2), ([3, 7, 1, 12, 5, 9, 2], 3)])
def test_shards_reassemble_the_global_step_noise(natoms, world):
    from chemeleon_amd.distributed import partition
    N, B, A = sum(natoms), len(natoms), 104
    torch.manual_seed(42)
    full = [StepNoise(N, B, A).draw() for _ in range(3)]  # three reverse steps
    state_full = torch.get_rng_state()
    parts = []
    for g0, g1 in partition(natoms, world):
        n0, n1 = sum(natoms[:g0]), sum(natoms[:g1])
        sn = StepNoise(N, B, A, n0, n1, g0, g1)
        torch.manual_seed(42)
        parts.append([sn.draw() for _ in range(3)])
        assert torch.equal(torch.get_rng_state(), state_full)
    for step in range(3):
        for k, rows in enumerate(("node", "graph", "node", "node")):
            got = torch.cat([p[step][k] for p in parts])
            assert torch.equal(got, full[step][k]), (step, k)


def test_engine_position_is_checked():
    st = (ctypes.c_uint32 * 624)()
    left, nxt = ctypes.c_int32(0), ctypes.c_int32(0)
    rc = _lib.load().chm_mt19937_uniform(st, ctypes.byref(left), ctypes.byref(nxt), 4, 0, 4,
                                         ctypes.c_void_p(torch.empty(4).data_ptr()))
    assert rc == -1 and b"engine position" in _lib.load().chm_last_error()
    with pytest.raises(ValueError):
        rand_rows((4, 3), 3, 5)
