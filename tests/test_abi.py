"""CPU-side checks of the C-ABI library: it loads, exports every symbol the
header declares, and reports argument errors without touching a GPU."""

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
    assert lib.chm_segment_mean(None, 1, None, None, None) == -1
    assert lib.chm_batch_info(None, None, None, None, None) == -1
    assert lib.chm_d3pm_sample(-1, 104, 100, *([None] * 8)) == -1
    assert lib.chm_batch_num_nodes(None) == -1


def test_cpu_tensors_are_refused():
    import torch
    with pytest.raises(RuntimeError, match="HIP device only"):
        _lib.require_device(torch.zeros(3))
