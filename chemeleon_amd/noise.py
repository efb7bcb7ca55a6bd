"""Parity-mode noise: the reference's CPU RNG stream, drawn for one shard of a sample-parallel run.

The reference's reverse loop draws, for every t > 1 and in this order (chemeleon.py:400-404, 418,
435, 455), on the global CPU generator:

    rand(N, A)        atom-type uniforms (D3PM Gumbel noise)
    randn(B, 3, 3)    lattice noise
    randn(N, 3)       coordinate noise of the predictor
    randn(N, 3)       coordinate noise of the corrector

N and B are the WHOLE batch. A rank that samples crystals [g0, g1) (nodes [n0, n1)) must advance the
generator over all four global tensors, so that its own rows are the ones the single-process run
would draw, and so that every rank's generator ends in the same state as the single-process run.
`StepNoise.draw` does that: the three normal tensors are drawn by torch itself (61 K values at
512x40, 0.3 ms) and sliced; the uniform tensor (2.1 M values at 512x40, 9 ms through torch.rand on
one core) goes through `chm_mt19937_uniform`, which continues the generator's MT19937 state and
converts only this rank's rows.
"""

from typing import Optional, Sequence, Tuple

import ctypes

import numpy as np
import torch

from chemeleon_amd import _lib

# CPUGeneratorImplState (ATen CPUGeneratorImpl.cpp): legacy pod {uint64 the_initial_seed, int left,
# int seeded, uint64 next, uint64 state[624], double normal_x, normal_y, normal_rho, int
# normal_is_valid}, then float next_float_normal_sample, bool is_valid
_OFF_LEFT, _OFF_NEXT, _OFF_STATE, _MT_N = 8, 16, 24, 624
_STATE_BYTES = 5056


def rand_rows(shape: Sequence[int], row0: int, row1: int, out: Optional[torch.Tensor] = None,
              generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """Rows [row0, row1) of torch.rand(shape, generator=generator) (a CPU generator), advancing the
    generator exactly as that call would. Bit-identical to slicing torch.rand's result."""
    gen = generator if generator is not None else torch.default_generator
    shape = tuple(int(s) for s in shape)
    row = int(np.prod(shape[1:], dtype=np.int64)) if len(shape) > 1 else 1
    count = int(np.prod(shape, dtype=np.int64))
    lo, hi = row0 * row, row1 * row
    if not (0 <= row0 <= row1 <= shape[0]):
        raise ValueError(f"rows [{row0}, {row1}) outside a tensor of {shape[0]} rows")
    if out is None:
        out = torch.empty((row1 - row0,) + shape[1:], dtype=torch.float32)
    if out.dtype != torch.float32 or out.device.type != "cpu" or not out.is_contiguous() or out.numel() != hi - lo:
        raise ValueError("out must be a contiguous CPU float32 tensor of the slice's size")
    st = gen.get_state()
    if st.numel() != _STATE_BYTES:
        raise RuntimeError(f"unexpected CPU generator state size {st.numel()} (torch {torch.__version__})")
    raw = st.numpy().copy()
    words = raw[_OFF_STATE:_OFF_STATE + 8 * _MT_N].view(np.uint64)
    mt = np.ascontiguousarray(words.astype(np.uint32))
    left = ctypes.c_int32(int(raw[_OFF_LEFT:_OFF_LEFT + 4].view(np.int32)[0]))
    nxt = ctypes.c_int32(int(raw[_OFF_NEXT:_OFF_NEXT + 8].view(np.uint64)[0]))
    _lib.check(_lib.load().chm_mt19937_uniform(mt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(left),
                                               ctypes.byref(nxt), count, lo, hi,
                                               ctypes.c_void_p(out.data_ptr()) if hi > lo else None),
               "chm_mt19937_uniform")
    words[:] = mt.astype(np.uint64)
    raw[_OFF_LEFT:_OFF_LEFT + 4] = np.array([left.value], dtype=np.int32).view(np.uint8)
    raw[_OFF_NEXT:_OFF_NEXT + 8] = np.array([nxt.value], dtype=np.uint64).view(np.uint8)
    gen.set_state(torch.from_numpy(raw))
    return out


class StepNoise:
    """One rank's slice of the per-step draws of the reference's CPU path: atom rows [n0, n1) and
    crystal rows [g0, g1) of tensors whose global sizes are N nodes and B crystals."""

    def __init__(self, N: int, B: int, A: int, n0: int = 0, n1: Optional[int] = None, g0: int = 0,
                 g1: Optional[int] = None):
        self.N, self.B, self.A = int(N), int(B), int(A)
        self.n0, self.n1 = int(n0), int(N if n1 is None else n1)
        self.g0, self.g1 = int(g0), int(B if g1 is None else g1)
        self.full = (self.n0, self.n1, self.g0, self.g1) == (0, self.N, 0, self.B)
        self.local_shapes = ((self.n1 - self.n0, self.A), (self.g1 - self.g0, 3, 3), (self.n1 - self.n0, 3),
                             (self.n1 - self.n0, 3))

    def draw(self, out: Optional[Tuple[torch.Tensor, ...]] = None) -> Tuple[torch.Tensor, ...]:
        """(rand_a, rand_l, rand_x1, rand_x2) of this slice, drawn in the reference's order from the
        global CPU generator; into `out` (four CPU float32 tensors of local_shapes, e.g. pinned)."""
        if out is None:
            out = tuple(torch.empty(sh, dtype=torch.float32) for sh in self.local_shapes)
        if self.full:
            torch.rand((self.N, self.A), out=out[0])
            torch.randn((self.B, 3, 3), out=out[1])
            torch.randn((self.N, 3), out=out[2])
            torch.randn((self.N, 3), out=out[3])
            return out
        rand_rows((self.N, self.A), self.n0, self.n1, out=out[0])
        out[1].copy_(torch.randn(self.B, 3, 3)[self.g0:self.g1])
        out[2].copy_(torch.randn(self.N, 3)[self.n0:self.n1])
        out[3].copy_(torch.randn(self.N, 3)[self.n0:self.n1])
        return out
