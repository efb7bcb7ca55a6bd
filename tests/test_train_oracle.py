"""Pin the oracle's training forward (chemeleon.py:137-244: q_sample, decoder, D3PM hybrid loss,
lattice / coordinate MSEs) against the reference's own Chemeleon.forward (make_golden.py gen_train).
CPU only."""

import numpy as np
import torch

from chemeleon_amd.config import default_config
from chemeleon_amd.synthetic import synthetic_state_dict, synthetic_text_embeds, weights_crc
from oracle import chemeleon_oracle as O


def train_noise(g):
    """The reference's draws after torch.manual_seed(noise_seed): rand(N, A), randn_like(l_0),
    randn_like(frac_coords) (chemeleon.py:162-175)."""
    N, B = int(g["natoms"].sum()), len(g["natoms"])
    torch.manual_seed(int(g["noise_seed"]))
    return torch.rand(N, 104), torch.randn(B, 3, 3), torch.randn(N, 3)


def test_training_forward_matches_reference(golden):
    g = golden("train_forward.npz")
    sd = synthetic_state_dict(default_config())
    assert weights_crc(sd) == int(g["weights_crc"])
    cfg = default_config()
    cfg["timesteps"] = 1000
    torch.manual_seed(0)
    orc = O.OracleModel(cfg, sd)
    ra, nl, nx = train_noise(g)
    B = len(g["natoms"])
    cond, _ = synthetic_text_embeds(512)
    out = orc.training_forward(torch.from_numpy(g["atom_types"]), torch.from_numpy(g["frac"]),
                               torch.from_numpy(g["lattices"]), g["natoms"].tolist(), torch.from_numpy(g["t"]),
                               ra, nl, nx, cond.expand(B, -1))
    for k in ("loss", "vb_loss_atom_types", "ce_loss_atom_types", "true_noise_lattice", "pred_noise_lattice",
              "true_noise_coords", "pred_noise_coords"):
        ref = g["out_" + k]
        np.testing.assert_allclose(out[k].numpy(), ref, rtol=2e-5, atol=2e-5 * max(1.0, float(np.abs(ref).max())),
                                   err_msg=k)
