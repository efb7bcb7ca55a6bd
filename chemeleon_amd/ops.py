"""torch.ops.chemeleon.* / torch.classes.chemeleon.* — the torch-op layer over the C ABI
(csrc/torch_ops.cpp).

    from chemeleon_amd import ops
    ops.load()
    model = ops.model(chemeleon.decoder)                   # torch.classes.chemeleon.Model
    batch = torch.classes.chemeleon.Batch(model, [40] * 64, 2, False, 20)
    sched = ops.schedule(chemeleon, step_lr=1e-5)          # torch.classes.chemeleon.Schedule
    torch.ops.chemeleon.sample_step(batch, sched, t, 2.0, a, x, lat, cond, null, None, None, None, None, 0, 0, 0)

The classes own the library's objects (reference-counted: a Batch holds its Model, a Schedule its
tables), so TorchScript and C++ callers build and drive the sampler with no ctypes object in sight.
The ops launch on the current HIP stream of the batch's device under a device guard for it, refuse
tensors on any other device, allocate outputs through the PyTorch caching allocator and raise
RuntimeError (TORCH_CHECK) with chm_last_error() on a failing call. They are registered for the CUDA
(= HIP) dispatch key only: CPU tensors raise NotImplementedError, there is no CPU fallback. The sampler
itself keeps the ctypes binding (chemeleon_amd._lib); both reach the same entry points.
"""

import os
import threading

import torch

from chemeleon_amd import _lib

OPS_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), "libchemeleon_torch_ops.so")
_lock = threading.Lock()
_loaded = False


def load(path: str = None):
    """Register torch.ops.chemeleon.* and torch.classes.chemeleon.* (once). Raises ImportError if the
    op library is missing."""
    global _loaded
    with _lock:
        if _loaded:
            return torch.ops.chemeleon
        p = path or OPS_PATH
        if not os.path.exists(p):
            raise ImportError(f"chemeleon_amd: torch-op library not found at {p}; build it with "
                              "`python -m chemeleon_amd.build`")
        _lib.load()  # (the op library links libchemeleon_hip.so, found next to it)
        torch.ops.load_library(p)
        _loaded = True
        return torch.ops.chemeleon


def model(decoder, math: str = None):
    """torch.classes.chemeleon.Model of a CSPNet's current weights (its state_dict order, the C ABI's)."""
    load()
    params = [p.detach().float().contiguous() for p in decoder.ordered_parameters()]
    m = torch.classes.chemeleon.Model(params, decoder.hidden_dim, decoder.time_dim, decoder.text_dim,
                                      decoder.num_layers, decoder.max_atoms, decoder.num_freqs)
    if math is not None:
        m.set_math(math)
    return m


def schedule(chemeleon, step_lr: float = 1e-5):
    """torch.classes.chemeleon.Schedule of a Chemeleon's per-timestep tables (schedule_tables)."""
    load()
    _, (coef, temb, q1, qm) = chemeleon.schedule_tables(step_lr)
    return torch.classes.chemeleon.Schedule(coef, temb, q1, qm)
