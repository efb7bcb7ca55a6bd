"""The drop-in boundary's ownership and threading contract, through the C ABI:
caller-owned workspaces from the PyTorch caching allocator, samplers on several streams at
once, and the arithmetic choice surviving a weight reload. Run on an MI355X: pytest -m gpu."""

import threading

import pytest
import torch

from chemeleon_amd import _lib
from chemeleon_amd.config import default_config
from chemeleon_amd.synthetic import synthetic_state_dict, synthetic_text_embeds

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")]

DEV = "cuda"


@pytest.fixture(scope="module")
def model():
    from chemeleon_amd import Chemeleon
    cfg = default_config()
    cfg["timesteps"] = 100
    torch.manual_seed(0)
    m = Chemeleon(cfg)
    m.decoder.load_state_dict(synthetic_state_dict(default_config()))
    return m.to(DEV).eval()


@pytest.fixture(scope="module")
def cn():
    return synthetic_text_embeds(512)


def test_workspace_comes_from_the_caching_allocator(model):
    nat = [7, 3, 12, 1]
    before = torch.cuda.memory_allocated()
    b = model.decoder.hip_batch(nat, 2, private=True)
    arr = (_lib.ctypes.c_int32 * len(nat))(*nat)
    need = int(_lib.load().chm_batch_workspace_bytes(model.decoder.hip_model().handle, arr, len(nat), 2))
    assert b.workspace.numel() == need == b.device_bytes
    assert torch.cuda.memory_allocated() - before >= need
    # too small a workspace is refused with a message, nothing is written
    small = torch.empty(need // 2, dtype=torch.uint8, device=DEV)
    h = _lib.c_void_p()
    rc = _lib.load().chm_batch_create_with_workspace(model.decoder.hip_model().handle, arr, len(nat), 2,
                                                     _lib.ptr(small), small.numel(), _lib.stream_handle(), h)
    assert rc == -1 and b"too small" in _lib.load().chm_last_error()


def _run(model, cn, nat, seed, stream=None):
    ctx = torch.cuda.stream(stream) if stream is not None else torch.cuda.stream(torch.cuda.current_stream())
    with ctx:
        last = None
        for last in model.sample_states(nat, None, 2.0, 1e-5, noise="philox", seed=seed, text_embeds=cn[0],
                                        null_text_embeds=cn[1], clone=True, t_stop=85, graph=False):
            pass
        torch.cuda.current_stream().synchronize()
    return last


def test_concurrent_samplers_on_two_streams(model, cn):
    """Two samplers of the SAME crystal list run at once from two host threads on two streams.
    Each gets its own workspace (the batch cache is keyed by stream), so both equal their serial
    results bit for bit."""
    nat = [20] * 48
    serial = [_run(model, cn, nat, seed) for seed in (3, 4)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    out = [None, None]
    errs = []

    def work(k):
        try:
            out[k] = _run(model, cn, nat, 3 + k, streams[k])
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=work, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs
    for k in range(2):
        for j in (1, 2, 3):
            assert torch.equal(out[k][j], serial[k][j]), f"sampler {k} state {j} differs from its serial run"
    assert not torch.equal(out[0][2], out[1][2])  # (different seeds really ran)


def test_lanes_with_identical_crystal_lists(model, cn):
    """A captured step split over stream lanes whose crystal lists are identical ([8] * 6 over 2
    and 3 lanes): every lane has its own workspace, and the states equal eager stepping."""
    nat = [8] * 6
    eager = list(model.sample_states(nat, None, 2.0, 1e-5, noise="philox", seed=5, text_embeds=cn[0],
                                     null_text_embeds=cn[1], clone=True, graph=False, t_stop=90))
    for lanes in (2, 3):
        graph = list(model.sample_states(nat, None, 2.0, 1e-5, noise="philox", seed=5, text_embeds=cn[0],
                                         null_text_embeds=cn[1], clone=True, graph=True, t_stop=90, lanes=lanes))
        for se, sg in zip(eager, graph):
            for k in (1, 2, 3):
                assert torch.equal(se[k], sg[k]), f"lanes={lanes} t={se[0]} state {k}"


def test_math_choice_survives_weight_reload(model):
    model.decoder.set_math("bf16x3")
    try:
        model.decoder.load_state_dict(synthetic_state_dict(default_config()))  # bumps the parameter versions
        assert model.decoder.get_math() == "bf16x3"
    finally:
        model.decoder.set_math("split16")
    assert model.decoder.get_math() == "split16"
