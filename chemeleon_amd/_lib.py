"""ctypes binding of libchemeleon_hip.so (the C ABI in include/chemeleon_hip.h).

The HIP library is the only compute path of this package: if it is missing,
or a tensor is not on a HIP device, calls raise instead of falling back to a
CPU implementation.
"""

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CHM_LIB", os.path.join(_HERE, "lib", "libchemeleon_hip.so"))

_lock = threading.Lock()
_lib = None

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_float = ctypes.c_float


class chm_dims(ctypes.Structure):
    _fields_ = [("hidden_dim", c_int), ("time_dim", c_int), ("text_dim", c_int), ("num_layers", c_int),
                ("max_atoms", c_int), ("num_freqs", c_int)]


class chm_batch_options(ctypes.Structure):
    _fields_ = [("edge_style", ctypes.c_int32), ("max_neighbors", ctypes.c_int32),
                ("knn_edges_per_atom", ctypes.c_int32), ("reserved", ctypes.c_int32)]


EDGES_FC, EDGES_KNN = 0, 1


class chm_train_tables(ctypes.Structure):
    _fields_ = [("T", c_int), ("d_coef4", c_void_p), ("d_q_one_step", c_void_p), ("d_q_mats", c_void_p),
                ("hybrid_coeff", c_float), ("cost_atom_types", c_float), ("cost_lattice", c_float),
                ("cost_coords", c_float)]


class chm_schedule(ctypes.Structure):
    _fields_ = [("T", c_int), ("num_classes", c_int), ("time_dim", c_int), ("reserved", c_int),
                ("d_coef", c_void_p), ("d_time_emb", c_void_p), ("d_q_one_step", c_void_p), ("d_q_mats", c_void_p)]


class chm_step_io(ctypes.Structure):
    """The buffers of one reverse step with their element counts (include/chemeleon_hip.h)."""
    _fields_ = [("d_atom_types", c_void_p), ("n_atom_types", c_i64), ("d_frac", c_void_p), ("n_frac", c_i64),
                ("d_lattices", c_void_p), ("n_lattices", c_i64), ("d_cond", c_void_p), ("n_cond", c_i64),
                ("d_null", c_void_p), ("n_null", c_i64), ("d_rand_a", c_void_p), ("n_rand_a", c_i64),
                ("d_rand_l", c_void_p), ("n_rand_l", c_i64), ("d_rand_x1", c_void_p), ("n_rand_x1", c_i64),
                ("d_rand_x2", c_void_p), ("n_rand_x2", c_i64)]


def step_io(a, x, lat, cond=None, null=None, noise=None, node0: int = 0, graph0: int = 0, nodes: int = None,
            graphs: int = None):
    """chm_step_io over tensors: the state (a [N] int64, x [N,3], lat [B,3,3]), conditioning rows
    [B, text_dim] and the optional parity-mode noise (rand_a [N,A], rand_l [B,3,3], rand_x1, rand_x2 [N,3]).
    With nodes / graphs given, the buffers are the rows [node0, node0 + nodes) / [graph0, graph0 + graphs)
    of those tensors (one lane of a captured step); counts are element counts of those rows."""
    nodes = a.shape[0] - node0 if nodes is None else nodes
    graphs = lat.shape[0] - graph0 if graphs is None else graphs

    def rows(t, first, n):
        if t is None:
            return None, 0
        per = t[0].numel() if t.dim() > 1 else 1
        return t.data_ptr() + first * per * t.element_size(), n * per

    io = chm_step_io()
    io.d_atom_types, io.n_atom_types = rows(a, node0, nodes)
    io.d_frac, io.n_frac = rows(x, node0, nodes)
    io.d_lattices, io.n_lattices = rows(lat, graph0, graphs)
    io.d_cond, io.n_cond = rows(cond, graph0, graphs)
    io.d_null, io.n_null = rows(null, graph0, graphs)
    if noise is not None and noise[0] is not None:
        ra, rl, rx1, rx2 = noise
        io.d_rand_a, io.n_rand_a = rows(ra, node0, nodes)
        io.d_rand_l, io.n_rand_l = rows(rl, graph0, graphs)
        io.d_rand_x1, io.n_rand_x1 = rows(rx1, node0, nodes)
        io.d_rand_x2, io.n_rand_x2 = rows(rx2, node0, nodes)
    return io


# name -> (restype, argtypes); every symbol declared in include/chemeleon_hip.h
SIGNATURES = {
    "chm_last_error": (ctypes.c_char_p, []),
    "chm_version": (ctypes.c_char_p, []),
    "chm_num_params": (c_int, [ctypes.POINTER(chm_dims)]),
    "chm_model_create": (c_int, [ctypes.POINTER(chm_dims), ctypes.POINTER(c_void_p), c_int, c_void_p,
                                 ctypes.POINTER(c_void_p)]),
    "chm_model_destroy": (None, [c_void_p]),
    "chm_model_set_option": (c_int, [c_void_p, ctypes.c_char_p, c_i64]),
    "chm_model_set_math": (c_int, [c_void_p, c_int]),
    "chm_model_get_math": (c_int, [c_void_p]),
    "chm_batch_create": (c_int, [c_void_p, ctypes.POINTER(ctypes.c_int32), c_int, c_int, ctypes.POINTER(c_void_p)]),
    "chm_batch_destroy": (None, [c_void_p]),
    "chm_batch_workspace_bytes": (ctypes.c_size_t, [c_void_p, ctypes.POINTER(ctypes.c_int32), c_int, c_int]),
    "chm_batch_create_with_workspace": (c_int, [c_void_p, ctypes.POINTER(ctypes.c_int32), c_int, c_int, c_void_p,
                                                ctypes.c_size_t, c_void_p, ctypes.POINTER(c_void_p)]),
    "chm_batch_workspace_bytes_ex": (ctypes.c_size_t, [c_void_p, ctypes.POINTER(ctypes.c_int32), c_int, c_int,
                                                       ctypes.POINTER(chm_batch_options)]),
    "chm_batch_create_ex": (c_int, [c_void_p, ctypes.POINTER(ctypes.c_int32), c_int, c_int,
                                    ctypes.POINTER(chm_batch_options), c_void_p, ctypes.c_size_t, c_void_p,
                                    ctypes.POINTER(c_void_p)]),
    "chm_training_loss": (c_int, [c_void_p, ctypes.POINTER(chm_train_tables)] + [c_void_p] * 17),
    "chm_knn_edges": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_i64,
                              ctypes.POINTER(c_i64), c_void_p]),
    "chm_debug_philox": (c_int, [c_u64, c_int, c_int, c_i64, c_i64, c_int, c_void_p, c_void_p]),
    "chm_debug_d3pm_philox": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_u64,
                                      c_i64, c_void_p, c_void_p]),
    "chm_debug_layer_jobs": (c_i64, [c_i64, c_int, c_int, ctypes.POINTER(c_i64), c_i64]),
    "chm_debug_layer_seq": (c_int, [c_i64, c_int, c_int, ctypes.POINTER(c_i64)]),
    "chm_debug_pair_plan": (c_i64, [ctypes.POINTER(ctypes.c_int32), c_int, c_int, c_int, ctypes.POINTER(ctypes.c_int32),
                                    c_i64, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                    ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32), c_i64]),
    "chm_debug_pair_nodes": (c_i64, [ctypes.POINTER(ctypes.c_int32), c_int, ctypes.POINTER(ctypes.c_int32), c_i64]),
    "chm_debug_row_nodes": (c_int, [ctypes.POINTER(ctypes.c_int32), c_int, ctypes.POINTER(ctypes.c_int32), c_i64,
                                    ctypes.POINTER(ctypes.c_int32), c_i64]),
    "chm_debug_row_tiles": (c_int, [ctypes.POINTER(ctypes.c_int32), c_int, ctypes.POINTER(ctypes.c_int32), c_i64,
                                    ctypes.POINTER(c_i64)]),
    "chm_debug_row_nodes_ex": (c_int, [ctypes.POINTER(ctypes.c_int32), c_int, c_i64, ctypes.POINTER(ctypes.c_int32),
                                       c_i64, ctypes.POINTER(ctypes.c_int32), c_i64]),
    "chm_debug_row_tiles_ex": (c_int, [ctypes.POINTER(ctypes.c_int32), c_int, c_i64, ctypes.POINTER(ctypes.c_int32),
                                       c_i64, ctypes.POINTER(c_i64)]),
    "chm_debug_short_row_tiles": (c_i64, [ctypes.POINTER(ctypes.c_int32), c_int, c_int, c_int, c_i64]),
    "chm_batch_short_row_tiles": (c_i64, [c_void_p]),
    "chm_batch_device_bytes": (ctypes.c_size_t, [c_void_p]),
    "chm_batch_num_nodes": (c_i64, [c_void_p]),
    "chm_batch_num_edges": (c_i64, [c_void_p]),
    "chm_batch_device": (c_int, [c_void_p]),
    "chm_batch_info": (c_int, [c_void_p, ctypes.POINTER(chm_dims), ctypes.POINTER(c_i64), ctypes.POINTER(c_int),
                               ctypes.POINTER(c_int)]),
    "chm_decoder_forward": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "chm_sample_step": (c_int, [c_void_p, ctypes.POINTER(chm_schedule), c_int, c_float, ctypes.POINTER(chm_step_io),
                                c_u64, c_i64, c_i64, c_void_p]),
    "chm_sample_step_dt": (c_int, [c_void_p, ctypes.POINTER(chm_schedule), c_void_p, c_float,
                                   ctypes.POINTER(chm_step_io), c_u64, c_i64, c_i64, c_void_p]),
    "chm_sample_step_dt_noise": (c_int, [c_void_p, ctypes.POINTER(chm_schedule), c_void_p, c_float,
                                         ctypes.POINTER(chm_step_io), c_void_p]),
    "chm_segment_mean": (c_int, [c_void_p, c_int, c_void_p, c_i64, c_void_p, c_i64, c_void_p]),
    "chm_d3pm_sample": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p]),
    "chm_edge_features": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "chm_edge_features_split": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "chm_prof_enable": (c_int, [c_int]),
    "chm_prof_reset": (c_int, []),
    "chm_prof_read": (c_int, [c_int, ctypes.POINTER(c_i64), ctypes.POINTER(ctypes.c_double)]),
    "chm_prof_events": (c_int, [ctypes.POINTER(c_i64), c_int]),
    "chm_prof_events_reset": (c_int, []),
    "chm_mt19937_uniform": (c_int, [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int32),
                                    ctypes.POINTER(ctypes.c_int32), c_i64, c_i64, c_i64, c_void_p]),
}


def load(path: str = None):
    """Load (once) and return the ctypes library. Raises loudly if absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise ImportError(
                f"chemeleon_amd: HIP library not found at {p}. Build it with `python -m chemeleon_amd.build` "
                "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        lib = ctypes.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is None:
                # (A/B runs load an older build through CHM_LIB: test hooks it predates stay unbound)
                if os.environ.get("CHM_LIB") and name.startswith(("chm_debug_", "chm_batch_short")):
                    continue
                raise ImportError(f"chemeleon_amd: {p} does not export {name} (stale build?)")
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = load().chm_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def ptr(t, byte_offset: int = 0):
    """Device pointer of a tensor (or None), optionally byte_offset bytes into it."""
    if t is None:
        return None
    return c_void_p(t.data_ptr() + byte_offset)


def stream_handle(device=None):
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device(*tensors):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("chemeleon_amd runs on a HIP device only: got a CPU tensor (no CPU fallback)")
        if not t.is_contiguous():
            raise RuntimeError("chemeleon_amd expects contiguous tensors")


MATH_BF16X3, MATH_F32, MATH_SPLIT16 = 0, 1, 2
K_EDGE_FOURIER, K_EDGE_MESSAGE, K_SEGMENT_MEAN, K_DECODER, K_EDGE_LAYER = 0, 1, 2, 3, 4


def prof_read(kernel: int):
    """(launches, total_ms) recorded for `kernel` since the last reset."""
    n = c_i64()
    ms = ctypes.c_double()
    check(load().chm_prof_read(kernel, ctypes.byref(n), ctypes.byref(ms)), "chm_prof_read")
    return int(n.value), float(ms.value)


EVENT_NAMES = ("layer_wait_timeouts", "layer_other_xcd", "layer_repairs", "tail_wait_timeouts", "tail_repairs",
               "layer_incomplete")


def prof_events(reset: bool = False):
    """The edge kernels' device health counters (include/chemeleon_hip.h, CHM_EV_*): wait timeouts,
    cross-XCD reads and the repair launches that ran since the last reset. Synchronous."""
    v = (c_i64 * 8)()
    check(load().chm_prof_events(v, 8), "chm_prof_events")
    out = {name: int(v[k]) for k, name in enumerate(EVENT_NAMES)}
    if reset:
        check(load().chm_prof_events_reset(), "chm_prof_events_reset")
    return out
