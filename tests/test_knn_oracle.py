"""Pin the knn (radius-graph) oracle against fixtures the reference itself wrote with its
torch_scatter segment ops injected (tests/golden/make_golden.py gen_knn; the reference path raises
NameError as shipped, data_utils.py:7). CPU only."""

import numpy as np
import pytest
import torch

from chemeleon_amd.config import default_config
from chemeleon_amd.synthetic import synthetic_state_dict, synthetic_text_embeds, weights_crc
from oracle import chemeleon_oracle as O
from oracle import knn_oracle as K

CASES = ["small", "dense", "uncapped"]


@pytest.fixture(scope="module")
def g(golden):
    return golden("knn.npz")


def _case(g, tag):
    return (torch.from_numpy(g[f"{tag}_natoms"]), torch.from_numpy(g[f"{tag}_atom_types"]),
            torch.from_numpy(g[f"{tag}_frac"]), torch.from_numpy(g[f"{tag}_lattices"]))


@pytest.mark.parametrize("tag", CASES)
def test_radius_graph_matches_reference(g, tag):
    nat, _, x, lat = _case(g, tag)
    n2g = torch.arange(len(nat)).repeat_interleave(nat)
    cart = torch.einsum("bi,bij->bj", x, lat[n2g])
    ei, img, nb = K.radius_graph_pbc(cart, lat, nat, 20)
    np.testing.assert_array_equal(ei.numpy(), g[f"{tag}_radius_edges"])
    np.testing.assert_array_equal(img.numpy(), g[f"{tag}_radius_images"])
    np.testing.assert_array_equal(nb.numpy(), g[f"{tag}_radius_counts"])


def test_cases_cover_the_neighbour_cap(g):
    """'small' and 'dense' exceed 20 neighbours (the cap and its +0.01 tie band act), 'uncapped'
    does not (the early-return branch, data_utils.py:357-364)."""
    for tag, capped in (("small", True), ("dense", True), ("uncapped", False)):
        nat, _, x, lat = _case(g, tag)
        n2g = torch.arange(len(nat)).repeat_interleave(nat)
        cart = torch.einsum("bi,bij->bj", x, lat[n2g])
        ei, _, _ = K.radius_graph_pbc(cart, lat, nat, 10 ** 9)  # no cap: every pair within the radius
        assert (int(torch.bincount(ei[1]).max()) > 20) == capped, tag


@pytest.mark.parametrize("tag", CASES)
def test_knn_edges_match_reference(g, tag):
    nat, _, x, lat = _case(g, tag)
    e, fd = K.knn_edges(nat.tolist(), x, lat, 20)
    np.testing.assert_array_equal(e.numpy(), g[f"{tag}_edges"])
    np.testing.assert_array_equal(fd.numpy(), g[f"{tag}_frac_diff"])


@pytest.mark.parametrize("tag", ["small", "dense"])
def test_knn_decoder_matches_reference(g, tag):
    sd = synthetic_state_dict(default_config())
    assert weights_crc(sd) == int(g["weights_crc"])
    nat, a, x, lat = _case(g, tag)
    B = len(nat)
    cfg = default_config()
    cfg["edge_style"] = "knn"
    te = O.time_embedding(torch.full((B,), 500, dtype=torch.long), 128)
    cond, _ = synthetic_text_embeds(512)
    types, lo, co, h = O.cspnet_forward(sd, cfg, a, x, lat, nat, torch.arange(B).repeat_interleave(nat), te,
                                        cond.expand(B, -1))
    for got, key in ((types, "types"), (co, "coords"), (lo, "lattice_out"), (h, "node_features")):
        ref = g[f"{tag}_{key}"]
        np.testing.assert_allclose(got.numpy(), ref, rtol=1e-5, atol=1e-5 * float(np.abs(ref).max()))
