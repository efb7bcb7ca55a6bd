"""Checks of the C-ABI library itself. On the CPU: it loads, exports every symbol the header declares,
and reports argument errors without touching a GPU. On the GPU (-m gpu): the entry points refuse
mis-sized buffers and out-of-range indices themselves (non-zero status + chm_last_error()), before
anything is enqueued, whatever the caller's binding checked or did not check."""

import ctypes
import os
import re

import pytest

from chemeleon_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "chemeleon_hip.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(chm_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/chemeleon_hip.h but not exported"
    # and the ctypes table covers the same set
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)


def test_version_and_param_count():
    lib = _lib.load()
    assert b"gfx950" in lib.chm_version()
    d = _lib.chm_dims(512, 128, 512, 6, 104, 128)
    assert lib.chm_num_params(ctypes.byref(d)) == 73


def test_unsupported_dims_fail_loudly_without_gpu():
    lib = _lib.load()
    d = _lib.chm_dims(256, 128, 512, 6, 104, 128)
    out = ctypes.c_void_p()
    arr = (ctypes.c_void_p * 73)()
    rc = lib.chm_model_create(ctypes.byref(d), arr, 73, None, ctypes.byref(out))
    assert rc == -3
    assert b"hidden_dim" in lib.chm_last_error()
    d = _lib.chm_dims(512, 128, 512, 6, 104, 128)
    rc = lib.chm_model_create(ctypes.byref(d), arr, 72, None, ctypes.byref(out))
    assert rc == -1 and b"number of parameter" in lib.chm_last_error()
    rc = lib.chm_model_create(ctypes.byref(d), arr, 73, None, ctypes.byref(out))
    assert rc == -1 and b"NULL" in lib.chm_last_error()


def test_null_handles_are_rejected():
    lib = _lib.load()
    assert lib.chm_decoder_forward(None, 1, None, None, None, None, 0, None, None, None, None, None, None) == -1
    assert lib.chm_segment_mean(None, 1, None, 0, None, 0, None) == -1
    assert lib.chm_batch_device(None) == -1
    io = _lib.chm_step_io()
    assert lib.chm_sample_step(None, None, 1, 2.0, ctypes.byref(io), 0, 0, 0, None) == -1
    assert lib.chm_sample_step_dt_noise(None, None, None, 2.0, ctypes.byref(io), None) == -1
    assert lib.chm_batch_info(None, None, None, None, None) == -1
    assert lib.chm_d3pm_sample(-1, 104, 100, *([None] * 8)) == -1
    assert lib.chm_batch_num_nodes(None) == -1


def test_cpu_tensors_are_refused():
    import torch
    with pytest.raises(RuntimeError, match="HIP device only"):
        _lib.require_device(torch.zeros(3))


# ---------------------------------------------------------------- the sized entry points (GPU)
gpu = [pytest.mark.gpu]


def _gpu_batch(nat, pairs):
    import torch
    from chemeleon_amd import Chemeleon
    from chemeleon_amd.config import default_config
    from chemeleon_amd.synthetic import synthetic_state_dict
    cfg = default_config()
    cfg["timesteps"] = 100
    torch.manual_seed(0)
    m = Chemeleon(cfg)
    m.decoder.load_state_dict(synthetic_state_dict(default_config()))
    m = m.to("cuda").eval()
    return m, m.decoder.hip_batch(nat, max_pairs=pairs, private=True)


@pytest.mark.gpu
def test_sample_step_refuses_mis_sized_buffers():
    """Every buffer of chm_sample_step / _dt / _dt_noise carries its element count; each mis-sized one is
    refused with CHM_E_ARG naming it, and a schedule of another class count is refused."""
    import torch
    nat = [3, 5, 8]
    N, B = sum(nat), len(nat)
    m, b = _gpu_batch(nat, 2)
    lib = _lib.load()
    sched, _keep = m.schedule_tables(1e-5)
    dev = "cuda"
    a = torch.zeros(N, dtype=torch.long, device=dev)
    x = torch.rand(N, 3, device=dev)
    lat = torch.eye(3, device=dev).repeat(B, 1, 1).contiguous()
    c = torch.zeros(B, 512, device=dev)
    nz = [torch.rand(N, 104, device=dev), torch.randn(B, 3, 3, device=dev), torch.randn(N, 3, device=dev),
          torch.randn(N, 3, device=dev)]
    st = _lib.stream_handle()
    d_t = torch.full((1,), 100, dtype=torch.int32, device=dev)

    def step(io, entry="step"):
        if entry == "step":
            return lib.chm_sample_step(b.handle, sched, 50, 2.0, ctypes.byref(io), 0, 0, 0, st)
        if entry == "dt":
            return lib.chm_sample_step_dt(b.handle, sched, _lib.ptr(d_t), 2.0, ctypes.byref(io), 0, 0, 0, st)
        return lib.chm_sample_step_dt_noise(b.handle, sched, _lib.ptr(d_t), 2.0, ctypes.byref(io), st)

    for field, n_bad, name in [("n_atom_types", N - 1, b"atom_types"), ("n_frac", 3 * N + 3, b"frac"),
                               ("n_lattices", 9, b"lattices"), ("n_cond", 512, b"cond"), ("n_null", 0, b"null"),
                               ("n_rand_a", N * 100, b"rand_a"), ("n_rand_l", 9 * B - 1, b"rand_l"),
                               ("n_rand_x1", 3 * N - 3, b"rand_x1"), ("n_rand_x2", 3, b"rand_x2")]:
        io = _lib.step_io(a, x, lat, c, c, nz)
        setattr(io, field, n_bad)
        assert step(io) == -1, field
        err = lib.chm_last_error()
        assert name in err and b"elements" in err, (field, err)
    io = _lib.step_io(a, x, lat, c, c, nz)
    io.d_rand_x2 = None
    assert step(io) == -1 and b"all four" in lib.chm_last_error()
    assert step(_lib.step_io(a, x, lat, c, c, nz), "dt") == -1 and b"must be NULL" in lib.chm_last_error()
    assert step(_lib.step_io(a, x, lat, c, c), "dt_noise") == -1 and b"required" in lib.chm_last_error()
    bad = _lib.chm_schedule(sched.T, 50, sched.time_dim, 0, sched.d_coef, sched.d_time_emb, sched.d_q_one_step,
                            sched.d_q_mats)
    rc = lib.chm_sample_step(b.handle, bad, 50, 2.0, ctypes.byref(_lib.step_io(a, x, lat, c, c)), 0, 0, 0, st)
    assert rc == -1 and b"num_classes" in lib.chm_last_error()
    torch.cuda.synchronize()
    assert torch.equal(x, x)  # (nothing ran: the refused calls enqueued no work)
    # the correctly sized call runs
    assert step(_lib.step_io(a, x, lat, c, c, nz)) == 0, lib.chm_last_error()
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_segment_mean_refuses_mis_sized_messages():
    import torch
    nat = [4, 6]
    m, b = _gpu_batch(nat, 2)
    lib = _lib.load()
    E, N = b.num_edges, b.num_nodes
    msg = torch.zeros(2, E, 64, device="cuda")  # (the round-4 fault: 64-wide messages into a 512-wide kernel)
    agg = torch.zeros(2, N, 512, device="cuda")
    st = _lib.stream_handle()
    assert lib.chm_segment_mean(b.handle, 2, _lib.ptr(msg), msg.numel(), _lib.ptr(agg), agg.numel(), st) == -1
    assert b"msg" in lib.chm_last_error()
    msg = torch.zeros(2, E, 512, device="cuda")
    assert lib.chm_segment_mean(b.handle, 2, _lib.ptr(msg), msg.numel(), _lib.ptr(agg), agg.numel() - 1, st) == -1
    assert b"agg" in lib.chm_last_error()
    assert lib.chm_segment_mean(b.handle, 2, _lib.ptr(msg), msg.numel(), _lib.ptr(agg), agg.numel(), st) == 0
    assert lib.chm_batch_device(b.handle) == torch.cuda.current_device()
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_d3pm_sample_refuses_out_of_range_indices(golden):
    """The round-4 k_d3pm clamped caller indices into a plausible wrong sample; now an out-of-range t or x_t
    is found on the device and the call returns CHM_E_ARG naming the first such node (its output -1)."""
    import numpy as np
    import torch
    g = golden("units.npz")
    lg, xt, t, u = [torch.from_numpy(g[k]).cuda().contiguous() for k in ("d3pm_logits", "d3pm_xt", "d3pm_t", "d3pm_u")]
    N, A = lg.shape
    lib = _lib.load()
    m, _b = _gpu_batch([2], 1)
    q1, qm = m.d3pm.q_one_step_mats.cuda().contiguous(), m.d3pm.q_mats.cuda().contiguous()
    T = qm.shape[0] - 1
    out = torch.empty(N, dtype=torch.long, device="cuda")
    st = _lib.stream_handle()
    for k, (bad_t, bad_x) in enumerate([(T + 1, None), (0, None), (-5, None), (None, A), (None, -1)]):
        tt, xx = t.clone(), xt.clone()
        i = 1 + k % (N - 1)
        if bad_t is not None:
            tt[i] = bad_t
        if bad_x is not None:
            xx[i] = bad_x
        rc = lib.chm_d3pm_sample(N, A, T, _lib.ptr(lg), _lib.ptr(xx), _lib.ptr(tt), _lib.ptr(u), _lib.ptr(q1),
                                 _lib.ptr(qm), _lib.ptr(out), st)
        assert rc == -1, (bad_t, bad_x)
        assert f"node {i} has t outside".encode() in lib.chm_last_error()
        assert int(out[i]) == -1
    rc = lib.chm_d3pm_sample(N, A, T, _lib.ptr(lg), _lib.ptr(xt), _lib.ptr(t), _lib.ptr(u), _lib.ptr(q1), _lib.ptr(qm),
                             _lib.ptr(out), st)
    assert rc == 0
    np.testing.assert_array_equal(out.cpu().numpy(), g["d3pm_out"])
