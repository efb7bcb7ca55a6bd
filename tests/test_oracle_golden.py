"""Pin the CPU oracle against fixtures generated from the reference itself
(tests/golden/make_golden.py). CPU only."""

import numpy as np
import pytest
import torch

from chemeleon_amd.config import default_config
from chemeleon_amd.synthetic import synthetic_state_dict, synthetic_text_embeds, weights_crc
from oracle import chemeleon_oracle as O


def _cfg(T=1000):
    c = default_config()
    c["timesteps"] = T
    return c


@pytest.fixture(scope="module")
def sd():
    return synthetic_state_dict(default_config())


@pytest.mark.parametrize("T", [100, 1000])
def test_schedules(golden, T):
    g = golden(f"schedules_T{T}.npz")
    b = O.beta_schedule(T, "cosine")
    for k_ref, k in (("betas", "betas"), ("alphas", "alphas"), ("alphas_cumprod", "alphas_cumprod"),
                     ("beta_sigmas", "sigmas")):
        np.testing.assert_array_equal(b[k].numpy(), g[k_ref])
    torch.manual_seed(0)
    s, sn = O.sigma_schedule(T)
    np.testing.assert_array_equal(s.numpy(), g["sigmas"])
    np.testing.assert_allclose(sn.numpy(), g["sigmas_norm"], rtol=1e-6)
    one, cum = O.d3pm_tables(b["betas"], T, 104)
    ts = g["qmat_t"]
    np.testing.assert_array_equal(one[ts].numpy(), g["q_one_step"])
    np.testing.assert_allclose(cum[ts].numpy(), g["q_mats"], rtol=1e-6, atol=1e-7)


def test_units(golden):
    g = golden("units.npz")
    x = torch.from_numpy(g["mod_in"])
    np.testing.assert_array_equal((x % 1.0).numpy(), g["mod_out"])
    np.testing.assert_array_equal(O.fourier(torch.from_numpy(g["fourier_in"]), 128).numpy(), g["fourier_out"])
    np.testing.assert_array_equal(O.time_embedding(torch.from_numpy(g["temb_in"]), 128).numpy(), g["temb_out"])
    out = O.scatter_mean(torch.from_numpy(g["scatter_src"]), torch.from_numpy(g["scatter_idx"]), 6)
    np.testing.assert_allclose(out.numpy(), g["scatter_out"], rtol=1e-6)
    b = O.beta_schedule(100)
    one, cum = O.d3pm_tables(b["betas"], 100, 104)
    a = O.d3pm_p_sample(torch.from_numpy(g["d3pm_logits"]), torch.from_numpy(g["d3pm_xt"]),
                        torch.from_numpy(g["d3pm_t"]), torch.from_numpy(g["d3pm_u"]), one, cum)
    np.testing.assert_array_equal(a.numpy(), g["d3pm_out"])


@pytest.mark.parametrize("name", ["decoder_4x6.npz", "decoder_ragged.npz"])
def test_decoder(golden, sd, name):
    g = golden(name)
    assert int(g["weights_crc"]) == int(weights_crc(sd)), "synthetic weight recipe changed"
    nat = torch.from_numpy(g["natoms"])
    n2g = torch.arange(len(nat)).repeat_interleave(nat)
    te = O.time_embedding(torch.full((len(nat),), int(g["t"]), dtype=torch.long), 128)
    cond, null = synthetic_text_embeds(512)
    hid = []
    types, lat, coords, h = O.cspnet_forward(sd, _cfg(), torch.from_numpy(g["atom_types"]), torch.from_numpy(g["frac"]),
                                             torch.from_numpy(g["lattices"]), nat, n2g, te,
                                             cond.expand(len(nat), -1), hidden=hid)
    tol = dict(rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(torch.stack(hid).numpy(), g["hidden"], **tol)
    np.testing.assert_allclose(types.numpy(), g["types"], **tol)
    np.testing.assert_allclose(lat.numpy(), g["lattice_out"], **tol)
    np.testing.assert_allclose(coords.numpy(), g["coords"], **tol)
    np.testing.assert_allclose(h.numpy(), g["node_features"], **tol)


def test_trajectory_c0(golden, sd):
    """C0: 4 x 6, T = 100, seed 42 — the whole reference sampler."""
    g = golden("trajectory_4x6_T100.npz")
    torch.manual_seed(0)
    m = O.OracleModel(_cfg(100), sd)
    cond, null = synthetic_text_embeds(512)
    torch.manual_seed(42)
    states = list(m.sample([6] * 4, cond.expand(4, -1), null.expand(4, -1)))[1:]
    a = torch.stack([s[1] for s in states]).numpy()
    x = torch.stack([s[2] for s in states]).numpy()
    lat = torch.stack([s[3] for s in states]).numpy()
    np.testing.assert_array_equal(a, g["atom_types"])
    d = np.abs(x - g["frac"])
    d = np.minimum(d, 1 - d)
    assert d.max() < 1e-4
    np.testing.assert_allclose(lat, g["lattices"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("tag", ["64x20", "16x40"])
def test_single_steps(golden, sd, tag):
    """Teacher-forced single reverse steps (reference state at t + seeded
    noise -> state at t-1) at 64 x 20 and 16 x 40, T = 1000."""
    g = golden(f"step_{tag}.npz")
    torch.manual_seed(0)
    m = O.OracleModel(_cfg(1000), sd)
    cond, null = synthetic_text_embeds(512)
    nat = torch.from_numpy(g["natoms"])
    B, N = len(nat), int(nat.sum())
    n2g = torch.arange(B).repeat_interleave(nat)
    for t in g["ts"]:
        t = int(t)
        torch.manual_seed(5000 + t)
        nz = m.draw_noise(t, N, B)
        a, x, l, _ = m.step(t, torch.from_numpy(g[f"t{t}_a"]), torch.from_numpy(g[f"t{t}_x"]),
                            torch.from_numpy(g[f"t{t}_l"]), nat, n2g, cond.expand(B, -1), null.expand(B, -1), nz)
        np.testing.assert_array_equal(a.numpy(), g[f"t{t}_a_out"])
        np.testing.assert_allclose(x.numpy(), g[f"t{t}_x_out"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(l.numpy(), g[f"t{t}_l_out"], rtol=1e-5, atol=1e-5)
