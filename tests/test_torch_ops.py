"""The torch-op layer (torch.ops.chemeleon.*, csrc/torch_ops.cpp) on the CPU: the library loads next to
libchemeleon_hip.so, registers every op with the schema the GPU tests call, and refuses CPU tensors
(there is no CPU kernel, so no silent fallback)."""

import pytest
import torch

from chemeleon_amd import ops


def test_ops_register_with_their_schemas():
    chem = ops.load()
    schemas = {name: str(getattr(chem, name).default._schema) for name in
               ("decoder_forward", "sample_step", "segment_mean", "d3pm_sample")}
    assert "Tensor(a!) atom_types" in schemas["sample_step"] and "-> ()" in schemas["sample_step"]
    assert schemas["decoder_forward"].endswith("Tensor? text) -> (Tensor, Tensor, Tensor, Tensor)")
    assert "Tensor msg" in schemas["segment_mean"]
    assert "Tensor q_mats" in schemas["d3pm_sample"]


def test_cpu_tensors_are_refused():
    chem = ops.load()
    with pytest.raises(NotImplementedError):
        chem.segment_mean(0, 1, torch.zeros(1, 1, 1))
    with pytest.raises(NotImplementedError):
        chem.d3pm_sample(*[torch.zeros(2, 3)] * 2, torch.zeros(2, dtype=torch.long), torch.zeros(2, 3),
                         torch.zeros(4, 3, 3), torch.zeros(4, 3, 3))


def test_load_fails_loudly_without_the_library(tmp_path):
    import importlib
    fresh = importlib.reload(ops)  # (a module whose registry has not loaded anything yet)
    try:
        with pytest.raises(ImportError, match="torch-op library not found"):
            fresh.load(str(tmp_path / "missing.so"))
    finally:
        importlib.reload(ops)


def test_handle_accepts_batches_handles_and_ints():
    import ctypes

    class FakeBatch:
        handle = ctypes.c_void_p(1234)

    assert ops.handle(FakeBatch()) == 1234
    assert ops.handle(ctypes.c_void_p(99)) == 99
    assert ops.handle(7) == 7
    with pytest.raises(ValueError):
        ops.handle(ctypes.c_void_p())
