"""torch.ops.chemeleon.* — the torch-op layer over the C ABI (csrc/torch_ops.cpp).

    from chemeleon_amd import ops
    ops.load()
    types, lattice, coords, nodes = torch.ops.chemeleon.decoder_forward(ops.handle(batch), 2, ...)

The ops take the library's batch handle (`CSPNet.hip_batch(...).handle`) and schedule address
(`Chemeleon.schedule_tables(...)[0]`), launch on the caller's current HIP stream, allocate outputs
through the PyTorch caching allocator and raise RuntimeError (TORCH_CHECK) with chm_last_error() on a
failing call. They are registered for the CUDA (= HIP) dispatch key only: CPU tensors raise
NotImplementedError, there is no CPU fallback. The ctypes binding (chemeleon_amd._lib) reaches the same
entry points; the sampler uses that one and the ops serve torch-native callers.
"""

import ctypes
import os
import threading

import torch

from chemeleon_amd import _lib

OPS_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), "libchemeleon_torch_ops.so")
_lock = threading.Lock()
_loaded = False


def load(path: str = None):
    """Register torch.ops.chemeleon.* (once). Raises ImportError if the op library is missing."""
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


def handle(obj) -> int:
    """The int the ops take for a batch: a HipBatch, its ctypes handle or an int."""
    h = getattr(obj, "handle", obj)
    h = getattr(h, "value", h)
    if not h:
        raise ValueError("null batch handle")
    return int(h)


def schedule_address(sched) -> int:
    """The int the ops take for a chm_schedule (Chemeleon.schedule_tables(step_lr)[0])."""
    return ctypes.addressof(sched)
