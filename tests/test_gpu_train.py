"""The training forward / validation loss on the HIP path (Chemeleon.forward -> chm_training_loss:
q_sample kernels, the decoder, the loss kernels) against the reference's own Chemeleon.forward
(tests/golden/train_forward.npz) on the same draws, and against the oracle for the noised atom types
(bit-exact, like the sampler's D3PM). Gates: losses and predictions within 1e-4 relative; the score
target near t = T, where sigma_norm ~ 1e-15 turns fp32 rounding into O(1) values, through its
numerator (1e-6 absolute)."""

import types

import numpy as np
import pytest
import torch

from chemeleon_amd.config import default_config
from chemeleon_amd.synthetic import synthetic_state_dict, synthetic_text_embeds
from oracle import chemeleon_oracle as O

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")]

DEV = "cuda"


class StubEncoder:
    """The fixture's text encoder: cond vectors (cond_drop_prob 0)."""

    def __init__(self, cond):
        self.cond = cond

    def get_text_embeds(self, texts, cond_drop_prob, device):
        assert cond_drop_prob == 0.0
        return self.cond.expand(len(texts), -1).to(device)


def test_training_forward_matches_reference(golden):
    from chemeleon_amd import Chemeleon
    g = golden("train_forward.npz")
    cfg = default_config()
    cfg["text_guide"] = True
    cond, _ = synthetic_text_embeds(512)
    torch.manual_seed(0)
    m = Chemeleon(cfg, text_encoder=StubEncoder(cond))
    m.decoder.load_state_dict(synthetic_state_dict(default_config()))
    m = m.to(DEV).eval()
    m.cond_drop_prob = 0.0
    nat = torch.from_numpy(g["natoms"])
    B, N = len(nat), int(nat.sum())
    torch.manual_seed(int(g["noise_seed"]))
    ra, nl, nx = torch.rand(N, 104), torch.randn(B, 3, 3), torch.randn(N, 3)
    batch = types.SimpleNamespace(atom_types=torch.from_numpy(g["atom_types"]), frac_coords=torch.from_numpy(g["frac"]),
                                  lattices=torch.from_numpy(g["lattices"]), natoms=nat,
                                  batch=torch.arange(B).repeat_interleave(nat), text=["x"] * B)
    out = m(batch, noise=(torch.from_numpy(g["t"]), ra, nl, nx))
    def scaled(got, ref):
        got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
        scale = max(float(np.sqrt(np.mean(ref ** 2))), 1e-12)
        return float((np.abs(got - ref) / np.maximum(np.abs(ref), scale)).max())

    o = {k: v.detach().cpu().numpy() for k, v in out.items()}
    for k in ("vb_loss_atom_types", "ce_loss_atom_types", "true_noise_lattice", "pred_noise_lattice",
              "pred_noise_coords"):
        assert scaled(o[k], g["out_" + k]) <= 1e-4, (k, scaled(o[k], g["out_" + k]))
    # score target d_log_p / sqrt(sigma_norm): near t = T sigma_norm is ~1e-15 (sqrt 4e-8), so the
    # reference's value there is its own fp32 rounding noise amplified 2.6e7 times. Well-conditioned
    # nodes are compared directly; for the others the numerator d_log_p must agree to 1e-6.
    t_node = torch.from_numpy(g["t"])[torch.arange(B).repeat_interleave(nat)]
    torch.manual_seed(0)
    orc = O.OracleModel(default_config(), synthetic_state_dict(default_config()))
    rs = orc.sigmas_norm[t_node].sqrt().numpy()[:, None].astype(np.float64)
    good = rs[:, 0] >= 1e-2
    tgt, ref_t = o["true_noise_coords"].astype(np.float64), g["out_true_noise_coords"].astype(np.float64)
    assert scaled(tgt[good], ref_t[good]) <= 1e-4
    assert np.abs((tgt - ref_t) * rs)[~good].max() <= 1e-6
    # the reductions: our loss is our components' weighted sum, and the coordinate MSE is ours
    lx = float(np.mean((o["pred_noise_coords"].astype(np.float64) - tgt) ** 2))
    assert abs(float(o["loss_coords"]) - lx) <= 1e-5 * max(lx, 1.0)
    total = float(o["vb_loss_atom_types"]) + float(o["ce_loss_atom_types"]) + float(o["loss_lattice"]) + lx
    assert abs(float(o["loss"]) - total) <= 1e-5 * total
    ll_ref = float(np.mean((g["out_pred_noise_lattice"] - g["out_true_noise_lattice"]) ** 2))
    assert abs(float(o["loss_lattice"]) - ll_ref) <= 1e-4 * ll_ref
    # the noised atom types: bit-exact against the oracle's q_sample on the same uniforms
    ref_at = O.d3pm_q_sample(torch.from_numpy(g["atom_types"]), t_node, ra, orc.q_mats)
    assert torch.equal(out["x_t_atom_types"].cpu(), ref_at)


def test_training_forward_draws_in_reference_order():
    """Without explicit noise the draws follow the reference (numpy t, then rand, randn, randn on the
    CPU generator): two calls from the same seeds give the same loss, a different seed another one."""
    from chemeleon_amd import Chemeleon
    cfg = default_config()
    cfg["text_guide"] = False
    torch.manual_seed(0)
    m = Chemeleon(cfg)
    c = dict(default_config())
    c["text_dim"] = 0
    m.decoder.load_state_dict(synthetic_state_dict(c))
    m = m.to(DEV).eval()
    nat = torch.tensor([5, 8, 3])
    gen = torch.Generator().manual_seed(4)
    batch = types.SimpleNamespace(atom_types=torch.randint(1, 104, (16,), generator=gen),
                                  frac_coords=torch.rand(16, 3, generator=gen),
                                  lattices=torch.diag_embed(4 + torch.rand(3, 3, generator=gen)), natoms=nat,
                                  batch=torch.arange(3).repeat_interleave(nat), text=None)
    losses = []
    for seed in (1, 1, 2):
        np.random.seed(seed)
        torch.manual_seed(seed)
        losses.append(float(m(batch)["loss"]))
    assert losses[0] == losses[1] and losses[0] != losses[2] and np.isfinite(losses).all()
