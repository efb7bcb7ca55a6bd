"""The radius-graph edge mode (CSPNet(edge_style="knn")) on the GPU, against the
reference's own outputs (tests/golden/knn.npz, written with torch_scatter's segment ops injected,
make_golden.py gen_knn) and the oracle (oracle/knn_oracle.py, pinned to the same fixtures).

* edges: the device-built graph (knn.hip) equals the reference's, grouped by source node in the
  reference's order within each node (the order the fused scatter_mean sums in), frac_diff bit-exact;
* decoder outputs: within 1e-4 scaled, as the fc decoder tests;
* one reverse step in knn mode (both decoder calls rebuild the graph) against the oracle step.
"""

import numpy as np
import pytest
import torch

from chemeleon_amd import _lib
from chemeleon_amd.config import default_config
from chemeleon_amd.synthetic import synthetic_state_dict, synthetic_text_embeds, weights_crc
from oracle import chemeleon_oracle as O
from oracle import knn_oracle as K

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")]

DEV = "cuda"
CASES = ["small", "dense", "uncapped"]


def _model():
    from chemeleon_amd import Chemeleon
    cfg = default_config()
    cfg["edge_style"] = "knn"
    torch.manual_seed(0)
    m = Chemeleon(cfg)
    m.decoder.load_state_dict(synthetic_state_dict(default_config()))
    return m.to(DEV).eval()


@pytest.fixture(scope="module")
def model():
    return _model()


@pytest.fixture(scope="module")
def g(golden):
    return golden("knn.npz")


def _case(g, tag):
    return (torch.from_numpy(g[f"{tag}_natoms"]), torch.from_numpy(g[f"{tag}_atom_types"]),
            torch.from_numpy(g[f"{tag}_frac"]), torch.from_numpy(g[f"{tag}_lattices"]))


def _device_edges(model, nat, x, lat):
    b = model.decoder.hip_batch(nat.tolist(), 1)
    cap = 64 * int(nat.sum()) + 64
    src = torch.empty(cap, dtype=torch.int32, device=DEV)
    dst = torch.empty(cap, dtype=torch.int32, device=DEV)
    fd = torch.empty(cap, 3, device=DEV)
    n = _lib.c_i64()
    xd, ld = x.to(DEV).contiguous(), lat.to(DEV).contiguous()
    _lib.check(_lib.load().chm_knn_edges(b.handle, _lib.ptr(xd), _lib.ptr(ld), _lib.ptr(src), _lib.ptr(dst),
                                         _lib.ptr(fd), cap, _lib.ctypes.byref(n), _lib.stream_handle()), "knn")
    E = n.value
    assert E <= cap
    return src[:E].cpu().long(), dst[:E].cpu().long(), fd[:E].cpu()


def _grouped(edges, fd):
    order = torch.sort(edges[0], stable=True).indices
    return edges[0][order], edges[1][order], fd[order]


@pytest.mark.parametrize("tag", CASES)
def test_knn_edges_match_reference(model, g, tag):
    nat, _, x, lat = _case(g, tag)
    src, dst, fd = _device_edges(model, nat, x, lat)
    ref = torch.from_numpy(g[f"{tag}_edges"])
    rs, rd, rf = _grouped(ref, torch.from_numpy(g[f"{tag}_frac_diff"]))
    assert len(src) == len(rs), f"{tag}: {len(src)} edges on the device, {len(rs)} in the reference"
    assert torch.equal(src, rs) and torch.equal(dst, rd), f"{tag}: edge lists differ"
    assert torch.equal(fd, rf), f"{tag}: frac_diff differs"


def test_knn_edges_random_batches_match_oracle(model):
    """Random batches (1-30 atoms, cells of 3-8 A with shear, coordinates slightly outside [0, 1))
    against the oracle: same edges in the same order, frac_diff bit-exact. (A pair whose d^2 fell
    within rounding of its cut could be decided differently by the CPU's ATen kernels and these fp32
    expressions; none of these seeded batches has one.)"""
    gen = torch.Generator().manual_seed(5)
    checked = 0
    for trial in range(12):
        nat = torch.randint(1, 31, (int(torch.randint(1, 9, (1,), generator=gen)),), generator=gen)
        B, N = len(nat), int(nat.sum())
        x = torch.rand(N, 3, generator=gen) * 1.2 - 0.1  # (unwrapped, as the corrector's x_{t-1/2})
        diag = 3.0 + 5.0 * torch.rand(B, 3, generator=gen)
        lat = torch.diag_embed(diag) + 0.4 * (torch.rand(B, 3, 3, generator=gen) - 0.5) * diag.mean(1).view(B, 1, 1)
        ref, rfd = K.knn_edges(nat.tolist(), x, lat, 20)
        src, dst, fd = _device_edges(model, nat, x, lat)
        rs, rd, rf = _grouped(ref, rfd)
        if len(src) != len(rs) or not (torch.equal(src, rs) and torch.equal(dst, rd)):
            pytest.fail(f"trial {trial} natoms {nat.tolist()}: device graph differs from the oracle "
                        f"({len(src)} vs {len(rs)} edges)")
        assert torch.equal(fd, rf)
        checked += 1
    assert checked == 12


def test_knn_without_neighbour_cap_matches_oracle(g):
    """max_neighbors <= 0 keeps every pair within the radius, the intent of the reference's
    get_max_neighbors_mask (data_utils.py:341-348) for max_num_neighbors_threshold <= 0 (the C ABI used
    to read 0 as 'unset' and cap at 20). Parity-unpinned: the reference also clamps its per-image
    counts to 0 there and its symmetric reorder then raises IndexError (cspnet.py:289-293); the oracle
    defines the uncapped graph with the true counts. On the reference's 'small' case (cells of 1-12
    atoms, where the cap of 20 removes pairs) the device graph equals that one and is larger than the
    capped graph."""
    from chemeleon_amd import Chemeleon
    cfg = default_config()
    cfg["edge_style"] = "knn"
    cfg["max_neighbors"] = 0
    torch.manual_seed(0)
    m = Chemeleon(cfg)
    m.decoder.load_state_dict(synthetic_state_dict(default_config()))
    m = m.to(DEV).eval()
    assert m.decoder.max_neighbors == 0
    nat, _, x, lat = _case(g, "small")
    src, dst, fd = _device_edges(m, nat, x, lat)
    ref, rfd = K.knn_edges(nat.tolist(), x, lat, 0)
    rs, rd, rf = _grouped(ref, rfd)
    assert len(src) == len(rs) and torch.equal(src, rs) and torch.equal(dst, rd) and torch.equal(fd, rf)
    assert len(src) > len(g["small_edges"][0]), "the uncapped graph should be larger than the capped one"
    del m
    torch.cuda.empty_cache()


@pytest.mark.parametrize("tag", ["small", "dense"])
def test_knn_decoder_matches_reference(model, g, tag):
    sd = model.decoder.state_dict()
    assert weights_crc({k: v.cpu() for k, v in sd.items()}) == int(g["weights_crc"])
    nat, a, x, lat = _case(g, tag)
    B = len(nat)
    te = model.time_embed(torch.full((B,), 500, dtype=torch.long)).to(DEV)
    cond, _ = synthetic_text_embeds(512)
    out = model.decoder(atom_types=a.to(DEV), frac_coords=x.to(DEV), lattices=lat.to(DEV), num_atoms=nat.to(DEV),
                        node2graph=torch.arange(B).repeat_interleave(nat).to(DEV), t=te,
                        text_embeds=cond.expand(B, -1).to(DEV))
    for got, key in ((out.node_features, "node_features"), (out.atom_types_out, "types"),
                     (out.coords_out, "coords"), (out.lattice_out, "lattice_out")):
        ref = g[f"{tag}_{key}"].astype(np.float64)
        gpu = got.detach().cpu().numpy().astype(np.float64)
        scale = max(np.sqrt(np.mean(ref ** 2)), 1e-12)
        err = np.abs(gpu - ref) / np.maximum(np.abs(ref), scale)
        assert err.max() <= 1e-4, f"{tag} {key}: max scaled error {err.max():.3e}"


def test_knn_reverse_step_matches_oracle(model):
    """One reverse step t = 500 in knn mode (predictor and corrector decoder pairs, the corrector's
    graph built from the unwrapped x_{t-1/2}) against the oracle's step on the same noise."""
    cfg = default_config()
    cfg["edge_style"] = "knn"
    torch.manual_seed(0)
    orc = O.OracleModel(cfg, synthetic_state_dict(default_config()))
    nat = [6, 9, 4, 12]
    B, N = len(nat), sum(nat)
    gen = torch.Generator().manual_seed(8)
    a = torch.randint(0, 104, (N,), generator=gen)
    x = torch.rand(N, 3, generator=gen)
    diag = 3.5 + 3.0 * torch.rand(B, 3, generator=gen)
    lat = (torch.diag_embed(diag) + 0.3 * (torch.rand(B, 3, 3, generator=gen) - 0.5)) * O.LATTICE_MASK
    nz = (torch.rand(N, 104, generator=gen), torch.randn(B, 3, 3, generator=gen), torch.randn(N, 3, generator=gen),
          torch.randn(N, 3, generator=gen))
    cond, null = synthetic_text_embeds(512)
    t = 500
    ra, xa, la, _ = orc.step(t, a, x, lat, torch.tensor(nat), torch.arange(B).repeat_interleave(torch.tensor(nat)),
                             cond.expand(B, -1), null.expand(B, -1), nz)
    ga, gx, gl = model.reverse_step(t, a, x, lat, nat, 2.0, 1e-5, cond, null, noise=nz)
    assert torch.equal(ga.cpu(), ra), "atom types differ"
    d = (gx.cpu() - xa).abs()
    assert torch.minimum(d, 1 - d).max() <= 1e-4
    scale = la.abs().max()
    assert ((gl.cpu() - la).abs() / torch.maximum(la.abs(), 1e-4 * scale)).max() <= 1e-4


def test_knn_sampler_runs_eagerly(model):
    """sample_states in knn mode: eager launches (graph capture is refused), a few Philox steps."""
    cond, null = synthetic_text_embeds(512)
    it = model.sample_states([5, 7], None, noise="philox", seed=3, t_stop=997, text_embeds=cond.to(DEV),
                             null_text_embeds=null.to(DEV))
    states = list(it)
    assert len(states) == 4
    t, a, x, lat = states[-1]
    assert torch.isfinite(x).all() and torch.isfinite(lat).all()
    with pytest.raises(ValueError):
        next(model.sample_states([5, 7], None, noise="philox", seed=3, graph=True, text_embeds=cond.to(DEV),
                                 null_text_embeds=null.to(DEV)))
