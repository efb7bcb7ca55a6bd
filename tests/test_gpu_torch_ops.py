"""torch.ops.chemeleon.* (csrc/torch_ops.cpp) on the GPU: each op reaches the same kernels as the ctypes
binding and gives bit-identical results; shape / device errors raise before any launch.
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


def _state(seed=1):
    g = torch.Generator().manual_seed(seed)
    N, B = sum(NAT), len(NAT)
    a = torch.randint(0, 100, (N,), generator=g)
    x = torch.rand(N, 3, generator=g)
    lat = torch.randn(B, 3, 3, generator=g) + 4 * torch.eye(3)
    return a.to(DEV), x.to(DEV), lat.to(DEV)


def test_decoder_forward_op_matches_ctypes(model, chem):
    dec = model.decoder
    a, x, lat = _state()
    B = len(NAT)
    te = model.time_embed(torch.full((B,), 37, dtype=torch.long)).to(DEV).contiguous()
    c, _ = synthetic_text_embeds(dec.text_dim)
    tx = c.expand(B, -1).to(DEV).contiguous()
    ref = dec._run(1, a, x, lat, NAT, te, tx)
    b = dec.hip_batch(NAT, max_pairs=1)
    got = chem.decoder_forward(ops.handle(b), 1, a, x, lat, te, tx.unsqueeze(0))
    torch.cuda.synchronize()
    for r, o in zip(ref, got):
        assert torch.equal(r, o)


@pytest.mark.parametrize("noise", ["philox", "explicit"])
def test_sample_step_op_matches_ctypes(model, chem, noise):
    a, x, lat = _state(2)
    N, B = sum(NAT), len(NAT)
    c, n = synthetic_text_embeds(model.decoder.text_dim)
    c, n = c.expand(B, -1).to(DEV).contiguous(), n.expand(B, -1).to(DEV).contiguous()
    if noise == "explicit":
        g = torch.Generator().manual_seed(5)
        nz = [torch.rand(N, model.decoder.max_atoms, generator=g), torch.randn(B, 3, 3, generator=g), torch.randn(N, 3, generator=g),
              torch.randn(N, 3, generator=g)]
        nz = [z.to(DEV) for z in nz]
    else:
        nz = None
    ra, rx, rl = model.reverse_step(50, a, x, lat, NAT, cond_scale=2.0, text_embeds=c, null_text_embeds=n,
                                    noise=nz, seed=11)
    sched, _keep = model.schedule_tables(1e-5)
    b = model.decoder.hip_batch(NAT, max_pairs=2)
    ga, gx, gl = a.clone(), x.clone(), lat.clone()
    chem.sample_step(ops.handle(b), ops.schedule_address(sched), 50, 2.0, ga, gx, gl, c, n,
                     *(nz if nz is not None else [None] * 4), 11, 0, 0)
    torch.cuda.synchronize()
    assert torch.equal(ga, ra) and torch.equal(gx, rx) and torch.equal(gl, rl)
    assert not torch.equal(gx, x)  # the step ran, in place


def test_segment_mean_op_matches_oracle(model, chem):
    from oracle import chemeleon_oracle as O
    b = model.decoder.hip_batch(NAT, max_pairs=2)
    g = torch.Generator().manual_seed(3)
    msg = torch.randn(2, b.num_edges, 512, generator=g)
    agg = chem.segment_mean(ops.handle(b), 2, msg.to(DEV))
    e = O.fc_edges(NAT)
    for k in range(2):
        ref = O.scatter_mean(msg[k], e[0], b.num_nodes)
        np.testing.assert_allclose(agg[k].cpu().numpy(), ref.numpy(), rtol=1e-6, atol=1e-6)


def test_d3pm_sample_op_bit_exact(model, chem, golden):
    g = golden("units.npz")
    dp = model.d3pm
    args = [torch.from_numpy(g[k]).to(DEV) for k in ("d3pm_logits", "d3pm_xt", "d3pm_t", "d3pm_u")]
    out = chem.d3pm_sample(*args, dp.q_one_step_mats.contiguous(), dp.q_mats.contiguous())
    np.testing.assert_array_equal(out.cpu().numpy(), g["d3pm_out"])


def test_ops_check_shapes_before_launch(model, chem):
    """Every tensor is checked against the batch's sizes and the model's dimensions (chm_batch_info) on the
    host: a mis-sized tensor raises RuntimeError and nothing is launched."""
    a, x, lat = _state()
    B = len(NAT)
    b = model.decoder.hip_batch(NAT, max_pairs=2)
    h = ops.handle(b)
    te = torch.zeros(B, 128, device=DEV)
    tx = torch.zeros(1, B, 512, device=DEV)
    with pytest.raises(RuntimeError, match="atom_types: expected shape"):
        chem.decoder_forward(h, 1, a[:-1], x, lat, te, tx)
    with pytest.raises(RuntimeError, match="time_emb"):
        chem.decoder_forward(h, 1, a, x, lat, te[:, :64], tx)
    with pytest.raises(RuntimeError, match="text: expected shape"):
        chem.decoder_forward(h, 2, a, x, lat, te, tx)
    with pytest.raises(RuntimeError, match="pairs must be in"):
        chem.decoder_forward(h, 3, a, x, lat, te, tx.expand(3, -1, -1).contiguous())
    with pytest.raises(RuntimeError, match="msg: expected shape"):
        chem.segment_mean(h, 2, torch.zeros(2, b.num_edges, 64, device=DEV))
    sched, _keep = model.schedule_tables(1e-5)
    c = torch.zeros(B, 512, device=DEV)
    with pytest.raises(RuntimeError, match="all four noise tensors"):
        chem.sample_step(h, ops.schedule_address(sched), 10, 2.0, a, x, lat, c, c, torch.zeros(1, device=DEV), None,
                         None, None, 0, 0, 0)
    with pytest.raises(RuntimeError, match="rand_a: expected shape"):
        chem.sample_step(h, ops.schedule_address(sched), 10, 2.0, a, x, lat, c, c,
                         torch.zeros(sum(NAT), 64, device=DEV), torch.zeros(B, 3, 3, device=DEV),
                         torch.zeros(sum(NAT), 3, device=DEV), torch.zeros(sum(NAT), 3, device=DEV), 0, 0, 0)
    with pytest.raises(RuntimeError, match="cond: expected shape"):
        chem.sample_step(h, ops.schedule_address(sched), 10, 2.0, a, x, lat, c[:1], c, None, None, None, None, 0, 0, 0)
    torch.cuda.synchronize()  # (nothing was launched: the stream is clean)
