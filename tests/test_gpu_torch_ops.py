"""torch.ops.chemeleon.* / torch.classes.chemeleon.* (csrc/torch_ops.cpp) on the GPU: each op reaches the
same kernels as the ctypes binding and gives bit-identical results, also from TorchScript with objects
built there; shape / device errors raise before any launch.
Run on an MI355X: pytest -m gpu."""

import numpy as np
import pytest
import torch

from chemeleon_amd import ops
from chemeleon_amd.config import default_config
from chemeleon_amd.synthetic import synthetic_state_dict, synthetic_text_embeds

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")]

DEV = "cuda"
NAT = [3, 7, 1, 12, 40, 5]


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
def chem():
    return ops.load()


@pytest.fixture(scope="module")
def tmodel(model, chem):
    """The decoder's weights as a torch.classes.chemeleon.Model."""
    return ops.model(model.decoder)


def _batch(tmodel, natoms, pairs):
    return torch.classes.chemeleon.Batch(tmodel, list(natoms), pairs, False, 20)


def _state(seed=1):
    g = torch.Generator().manual_seed(seed)
    N, B = sum(NAT), len(NAT)
    a = torch.randint(0, 100, (N,), generator=g)
    x = torch.rand(N, 3, generator=g)
    lat = torch.randn(B, 3, 3, generator=g) + 4 * torch.eye(3)
    return a.to(DEV), x.to(DEV), lat.to(DEV)


def test_decoder_forward_op_matches_ctypes(model, chem, tmodel):
    dec = model.decoder
    a, x, lat = _state()
    B = len(NAT)
    te = model.time_embed(torch.full((B,), 37, dtype=torch.long)).to(DEV).contiguous()
    c, _ = synthetic_text_embeds(dec.text_dim)
    tx = c.expand(B, -1).to(DEV).contiguous()
    ref = dec._run(1, a, x, lat, NAT, te, tx)
    b = _batch(tmodel, NAT, 1)
    assert (b.num_nodes(), b.num_graphs()) == (sum(NAT), len(NAT))
    got = chem.decoder_forward(b, 1, a, x, lat, te, tx.unsqueeze(0))
    torch.cuda.synchronize()
    for r, o in zip(ref, got):
        assert torch.equal(r, o)


def _noise(model, explicit):
    N, B = sum(NAT), len(NAT)
    if not explicit:
        return None
    g = torch.Generator().manual_seed(5)
    nz = [torch.rand(N, model.decoder.max_atoms, generator=g), torch.randn(B, 3, 3, generator=g),
          torch.randn(N, 3, generator=g), torch.randn(N, 3, generator=g)]
    return [z.to(DEV) for z in nz]


def _cond(model):
    B = len(NAT)
    c, n = synthetic_text_embeds(model.decoder.text_dim)
    return c.expand(B, -1).to(DEV).contiguous(), n.expand(B, -1).to(DEV).contiguous()


@pytest.mark.parametrize("noise", ["philox", "explicit"])
def test_sample_step_op_matches_ctypes(model, chem, tmodel, noise):
    a, x, lat = _state(2)
    c, n = _cond(model)
    nz = _noise(model, noise == "explicit")
    ra, rx, rl = model.reverse_step(50, a, x, lat, NAT, cond_scale=2.0, text_embeds=c, null_text_embeds=n,
                                    noise=nz, seed=11)
    sched = ops.schedule(model, 1e-5)
    assert sched.num_timesteps() == model.num_timesteps
    b = _batch(tmodel, NAT, 2)
    ga, gx, gl = a.clone(), x.clone(), lat.clone()
    chem.sample_step(b, sched, 50, 2.0, ga, gx, gl, c, n, *(nz if nz is not None else [None] * 4), 11, 0, 0)
    torch.cuda.synchronize()
    assert torch.equal(ga, ra) and torch.equal(gx, rx) and torch.equal(gl, rl)
    assert not torch.equal(gx, x)  # the step ran, in place


def test_torchscript_builds_a_batch_and_steps(model, chem, tmodel):
    """A TorchScript function (no Python ctypes objects anywhere) builds a Batch from the Model and a
    Schedule, runs the CFG decoder pair and one reverse step: bit-identical to the ctypes path."""
    from typing import List, Tuple

    @torch.jit.script
    def run(m: torch.classes.chemeleon.Model, sched: torch.classes.chemeleon.Schedule, natoms: List[int],
            a: torch.Tensor, x: torch.Tensor, lat: torch.Tensor, te: torch.Tensor, cond: torch.Tensor,
            null: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
        b = torch.classes.chemeleon.Batch(m, natoms, 2, False, 20)
        types, latt, coords, nodes = torch.ops.chemeleon.decoder_forward(b, 2, a, x, lat, te,
                                                                         torch.stack([cond, null], 0))
        torch.ops.chemeleon.sample_step(b, sched, 50, 2.0, a, x, lat, cond, null, None, None, None, None, 11, 0, 0)
        return types, coords, x, lat

    a, x, lat = _state(3)
    c, n = _cond(model)
    B = len(NAT)
    te = model.time_embed(torch.full((B,), 50, dtype=torch.long)).to(DEV).contiguous()
    rtypes, _rl, rcoords, _ = model.decoder.forward_cfg(a, x, lat, NAT, te, c, n)
    ra, rx, rl = model.reverse_step(50, a, x, lat, NAT, cond_scale=2.0, text_embeds=c, null_text_embeds=n, seed=11)
    ga, gx, gl = a.clone(), x.clone(), lat.clone()
    types, coords, ox, ol = run(tmodel, ops.schedule(model, 1e-5), list(NAT), ga, gx, gl, te, c, n)
    torch.cuda.synchronize()
    assert torch.equal(types, rtypes) and torch.equal(coords, rcoords)
    assert torch.equal(ga, ra) and torch.equal(ox, rx) and torch.equal(ol, rl)


def test_objects_keep_what_they_use_alive(model, chem):
    """A Batch holds its Model and a Schedule its tables: dropping every Python reference to them keeps the
    step working (reference counting, not raw addresses)."""
    import gc
    b = _batch(ops.model(model.decoder), NAT, 2)
    sched = ops.schedule(model, 1e-5)
    gc.collect()
    a, x, lat = _state(4)
    c, n = _cond(model)
    ra, rx, rl = model.reverse_step(20, a, x, lat, NAT, cond_scale=2.0, text_embeds=c, null_text_embeds=n, seed=3)
    chem.sample_step(b, sched, 20, 2.0, a, x, lat, c, n, None, None, None, None, 3, 0, 0)
    torch.cuda.synchronize()
    assert torch.equal(a, ra) and torch.equal(x, rx) and torch.equal(lat, rl)


def test_segment_mean_op_matches_oracle(model, chem, tmodel):
    from oracle import chemeleon_oracle as O
    b = _batch(tmodel, NAT, 2)
    g = torch.Generator().manual_seed(3)
    msg = torch.randn(2, b.num_edges(), 512, generator=g)
    agg = chem.segment_mean(b, 2, msg.to(DEV))
    e = O.fc_edges(NAT)
    for k in range(2):
        ref = O.scatter_mean(msg[k], e[0], b.num_nodes())
        np.testing.assert_allclose(agg[k].cpu().numpy(), ref.numpy(), rtol=1e-6, atol=1e-6)


def test_d3pm_sample_op_bit_exact(model, chem, golden):
    g = golden("units.npz")
    dp = model.d3pm
    args = [torch.from_numpy(g[k]).to(DEV) for k in ("d3pm_logits", "d3pm_xt", "d3pm_t", "d3pm_u")]
    out = chem.d3pm_sample(*args, dp.q_one_step_mats.contiguous(), dp.q_mats.contiguous())
    np.testing.assert_array_equal(out.cpu().numpy(), g["d3pm_out"])


def test_d3pm_sample_op_refuses_out_of_range_indices(model, chem, golden):
    """t outside [1, T] or x_t outside [0, A) raise (device-side check), instead of a plausible wrong sample."""
    g = golden("units.npz")
    dp = model.d3pm
    lg, xt, t, u = [torch.from_numpy(g[k]).to(DEV) for k in ("d3pm_logits", "d3pm_xt", "d3pm_t", "d3pm_u")]
    q1, qm = dp.q_one_step_mats.contiguous(), dp.q_mats.contiguous()
    T, A = qm.shape[0] - 1, qm.shape[1]
    for bad_t, bad_x in [(T + 1, None), (0, None), (None, A), (None, -1)]:
        tt, xx = t.clone(), xt.clone()
        if bad_t is not None:
            tt[2] = bad_t
        if bad_x is not None:
            xx[2] = bad_x
        with pytest.raises(RuntimeError, match="node 2 has t outside"):
            chem.d3pm_sample(lg, xx, tt, u, q1, qm)


def test_batch_used_from_two_streams_is_ordered(model, chem, tmodel):
    """One Batch drives two independent samplers, one per stream, with no ordering between the streams from the
    caller: each op waits for the previous stream's work on the batch's scratch, so both trajectories
    equal the same steps run alone."""
    c, n = _cond(model)
    sched = ops.schedule(model, 1e-5)
    states = [_state(6), _state(7)]
    refs = []
    b0 = _batch(tmodel, NAT, 2)
    for a, x, lat in states:
        ra, rx, rl = a.clone(), x.clone(), lat.clone()
        for t in (60, 59, 58):
            chem.sample_step(b0, sched, t, 2.0, ra, rx, rl, c, n, None, None, None, None, 7, 0, 0)
        refs.append((ra, rx, rl))
    torch.cuda.synchronize()
    b = _batch(tmodel, NAT, 2)  # (built on the default stream)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    work = [tuple(v.clone() for v in st) for st in states]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())  # (the inputs are ready)
    for t in (60, 59, 58):
        for s, (ga, gx, gl) in zip(streams, work):
            with torch.cuda.stream(s):
                chem.sample_step(b, sched, t, 2.0, ga, gx, gl, c, n, None, None, None, None, 7, 0, 0)
    torch.cuda.synchronize()
    for (ga, gx, gl), (ra, rx, rl) in zip(work, refs):
        assert torch.equal(ga, ra) and torch.equal(gx, rx) and torch.equal(gl, rl)


def test_d3pm_sample_op_under_graph_capture(model, chem, golden):
    """chm_d3pm_sample captured into a graph: no host sync in the capture; the replay gives the
    eager result, and an out-of-range node is marked -1 in the output instead of raising."""
    g = golden("units.npz")
    dp = model.d3pm
    lg, xt, t, u = [torch.from_numpy(g[k]).to(DEV) for k in ("d3pm_logits", "d3pm_xt", "d3pm_t", "d3pm_u")]
    q1, qm = dp.q_one_step_mats.contiguous(), dp.q_mats.contiguous()
    chem.d3pm_sample(lg, xt, t, u, q1, qm)  # (the first call on this thread allocates the check's flag word)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            out = chem.d3pm_sample(lg, xt, t, u, q1, qm)
    graph.replay()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), g["d3pm_out"])
    t[2] = qm.shape[0]  # t = T + 1: out of range
    graph.replay()
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert got[2] == -1
    np.testing.assert_array_equal(np.delete(got, 2), np.delete(g["d3pm_out"], 2))


def test_ops_check_shapes_and_devices_before_launch(model, chem, tmodel):
    """Every tensor is checked against the batch's sizes, the model's dimensions and the batch's device on
    the host: a mis-sized tensor or one on another device raises RuntimeError and nothing is launched."""
    a, x, lat = _state()
    B = len(NAT)
    b = _batch(tmodel, NAT, 2)
    te = torch.zeros(B, 128, device=DEV)
    tx = torch.zeros(1, B, 512, device=DEV)
    with pytest.raises(RuntimeError, match="atom_types: expected shape"):
        chem.decoder_forward(b, 1, a[:-1], x, lat, te, tx)
    with pytest.raises(RuntimeError, match="time_emb"):
        chem.decoder_forward(b, 1, a, x, lat, te[:, :64], tx)
    with pytest.raises(RuntimeError, match="text: expected shape"):
        chem.decoder_forward(b, 2, a, x, lat, te, tx)
    with pytest.raises(RuntimeError, match="pairs must be in"):
        chem.decoder_forward(b, 3, a, x, lat, te, tx.expand(3, -1, -1).contiguous())
    with pytest.raises(RuntimeError, match="msg: expected shape"):
        chem.segment_mean(b, 2, torch.zeros(2, b.num_edges(), 64, device=DEV))
    sched = ops.schedule(model, 1e-5)
    c = torch.zeros(B, 512, device=DEV)
    with pytest.raises(RuntimeError, match="all four noise tensors"):
        chem.sample_step(b, sched, 10, 2.0, a, x, lat, c, c, torch.zeros(1, device=DEV), None, None, None, 0, 0, 0)
    with pytest.raises(RuntimeError, match="rand_a: expected shape"):
        chem.sample_step(b, sched, 10, 2.0, a, x, lat, c, c, torch.zeros(sum(NAT), 64, device=DEV),
                         torch.zeros(B, 3, 3, device=DEV), torch.zeros(sum(NAT), 3, device=DEV),
                         torch.zeros(sum(NAT), 3, device=DEV), 0, 0, 0)
    with pytest.raises(RuntimeError, match="cond: expected shape"):
        chem.sample_step(b, sched, 10, 2.0, a, x, lat, c[:1], c, None, None, None, None, 0, 0, 0)
    with pytest.raises(RuntimeError, match="t must be in"):
        chem.sample_step(b, sched, sched.num_timesteps() + 1, 2.0, a, x, lat, c, c, None, None, None, None, 0, 0, 0)
    # a tensor on another device than the batch's: a CPU tensor beside HIP ones (the op is dispatched to the
    # HIP kernel by the others and must refuse it) and, where a second GPU exists, a tensor on that GPU
    with pytest.raises(RuntimeError, match="cond: chemeleon ops run on a HIP device only"):
        chem.sample_step(b, sched, 10, 2.0, a, x, lat, c.cpu(), c, None, None, None, None, 0, 0, 0)
    with pytest.raises(RuntimeError, match="text: chemeleon ops run on a HIP device only"):
        chem.decoder_forward(b, 1, a, x, lat, te, tx.cpu())
    with pytest.raises(RuntimeError, match="frac: chemeleon ops run on a HIP device only"):
        chem.decoder_forward(b, 1, a, x.cpu(), lat, te, tx)
    if torch.cuda.device_count() > 1:
        with pytest.raises(RuntimeError, match="cond is on cuda:1, the batch on cuda:0"):
            chem.sample_step(b, sched, 10, 2.0, a, x, lat, c.to("cuda:1"), c, None, None, None, None, 0, 0, 0)
    # a schedule of another class count
    T1 = sched.num_timesteps() + 1
    other = torch.classes.chemeleon.Schedule(torch.zeros(T1, 8, device=DEV), torch.zeros(T1, 128, device=DEV),
                                             torch.zeros(T1, 50, 50, device=DEV), torch.zeros(T1, 50, 50, device=DEV))
    with pytest.raises(RuntimeError, match="do not match the model"):
        chem.sample_step(b, other, 10, 2.0, a, x, lat, c, c, None, None, None, None, 0, 0, 0)
    torch.cuda.synchronize()  # (nothing was launched: the stream is clean)
