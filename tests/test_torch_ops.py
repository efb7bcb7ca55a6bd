"""The torch-op layer (torch.ops.chemeleon.* / torch.classes.chemeleon.*, csrc/torch_ops.cpp) on the CPU:
the library loads next to libchemeleon_hip.so, registers every op with the schema the GPU tests call
(objects, not raw addresses) and the three classes, and refuses CPU tensors (there is no CPU kernel, so
no silent fallback)."""

import pytest
import torch

from chemeleon_amd import ops


def test_ops_register_with_their_schemas():
    chem = ops.load()
    schemas = {name: str(getattr(chem, name).default._schema) for name in
               ("decoder_forward", "sample_step", "segment_mean", "d3pm_sample")}
    assert "Tensor(a!) atom_types" in schemas["sample_step"] and "-> ()" in schemas["sample_step"]
    assert "__torch__.torch.classes.chemeleon.Batch batch" in schemas["sample_step"]
    assert "__torch__.torch.classes.chemeleon.Schedule schedule" in schemas["sample_step"]
    assert "__torch__.torch.classes.chemeleon.Batch batch" in schemas["decoder_forward"]
    assert schemas["decoder_forward"].endswith("Tensor? text) -> (Tensor, Tensor, Tensor, Tensor)")
    assert "Tensor msg" in schemas["segment_mean"] and "chemeleon.Batch batch" in schemas["segment_mean"]
    assert "Tensor q_mats" in schemas["d3pm_sample"]
    for name in ("decoder_forward", "sample_step", "segment_mean"):  # no int handles / addresses left
        assert "int batch" not in schemas[name] and "int schedule" not in schemas[name]


def test_classes_are_registered():
    ops.load()
    for cls in ("Model", "Batch", "Schedule"):
        assert getattr(torch.classes.chemeleon, cls) is not None


def test_schedule_refuses_cpu_tables():
    """Construction checks its tensors on the host (a CPU table can never reach a kernel)."""
    ops.load()
    with pytest.raises(RuntimeError, match="HIP device only"):
        torch.classes.chemeleon.Schedule(torch.zeros(3, 8), torch.zeros(3, 128), torch.zeros(3, 4, 4),
                                         torch.zeros(3, 4, 4))


def test_model_refuses_cpu_parameters():
    ops.load()
    with pytest.raises(RuntimeError, match="HIP device only"):
        torch.classes.chemeleon.Model([torch.zeros(4)], 512, 128, 512, 6, 104, 128)


def test_cpu_tensors_are_refused():
    chem = ops.load()
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
