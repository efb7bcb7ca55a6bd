"""Statistics of the perf-mode noise (noise="philox"): the device Philox4x32-10 streams the step
kernels draw from, exposed through chm_debug_philox / chm_debug_d3pm_philox. The reference draws
the same quantities on its CPU generator (torch.rand / torch.randn, chemeleon.py:400-404, 418,
435, 455); these tests check that the device streams have the distributions those calls have:
uniform [0, 1) and standard normal (moments and Kolmogorov-Smirnov over 4 M draws per stream),
no correlation between the streams, and D3PM's Gumbel-argmax sampling (diff_utils.py:307-329)
reproducing the posterior's softmax category frequencies (chi-square on fixed logits).
Run on an MI355X: pytest -m gpu."""

import numpy as np
import pytest
import torch

from chemeleon_amd import _lib

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")]

stats = pytest.importorskip("scipy.stats")

N = 1 << 22


def draw(seed, t, kind, normal, n=N, base=0):
    out = torch.empty(n, device="cuda")
    _lib.check(_lib.load().chm_debug_philox(seed, t, kind, base, n, normal, _lib.ptr(out), _lib.stream_handle()),
               "chm_debug_philox")
    return out.cpu().numpy().astype(np.float64)


def test_uniform_stream():
    u = draw(7, 500, 0, 0)
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 5 * np.sqrt(1 / 12 / N)
    assert abs(u.var() - 1 / 12) < 5 * np.sqrt(1 / 180 / N)
    ks = stats.kstest(u, "uniform")
    print(f"uniform: mean {u.mean():.6f} var {u.var():.6f} KS D {ks.statistic:.2e} p {ks.pvalue:.3f}")
    assert ks.pvalue > 1e-3


@pytest.mark.parametrize("kind", [1, 2, 3])
def test_normal_streams(kind):
    z = draw(11, 321, kind, 1)
    assert np.isfinite(z).all()
    assert abs(z.mean()) < 5 / np.sqrt(N)
    assert abs(z.var() - 1.0) < 5 * np.sqrt(2 / N)
    skew, kurt = stats.skew(z), stats.kurtosis(z)
    assert abs(skew) < 5 * np.sqrt(6 / N) and abs(kurt) < 5 * np.sqrt(24 / N)
    ks = stats.kstest(z, "norm")
    print(f"normal kind {kind}: mean {z.mean():.2e} var {z.var():.6f} skew {skew:.2e} kurt {kurt:.2e} "
          f"KS D {ks.statistic:.2e} p {ks.pvalue:.3f}")
    assert ks.pvalue > 1e-3


def test_streams_are_uncorrelated():
    """Different kinds, timesteps and neighbouring indices are independent draws."""
    a = draw(11, 321, 2, 1, n=1 << 20)
    for other in (draw(11, 321, 3, 1, n=1 << 20), draw(11, 320, 2, 1, n=1 << 20), draw(12, 321, 2, 1, n=1 << 20),
                  draw(11, 321, 2, 1, n=1 << 20, base=1)):
        r = np.corrcoef(a, other)[0, 1]
        assert abs(r) < 5 / np.sqrt(1 << 20), r


def test_d3pm_gumbel_argmax_frequencies():
    """Perf-mode D3PM sampling of one node's fixed logits, repeated over 400 k node indices (so
    every draw uses fresh Philox uniforms): the category frequencies match the posterior's
    softmax, softmax(log(fact1 + eps) + log(fact2 + eps)) (diff_utils.py:258-286), chi-square."""
    from chemeleon_amd import Chemeleon
    from chemeleon_amd.config import default_config
    cfg = default_config()
    cfg["timesteps"] = 100
    torch.manual_seed(0)
    m = Chemeleon(cfg)
    A, T, t = 104, 100, 40
    g = torch.Generator().manual_seed(3)
    logits = torch.randn(A, generator=g) * 1.5
    xt = 0  # the absorbing class: fact1 is then nearly flat, the posterior follows the prediction
    q1, qm = m.d3pm.q_one_step_mats.float(), m.d3pm.q_mats.float()
    fact1 = q1.transpose(1, 2)[t - 1, xt, :]
    fact2 = torch.softmax(logits, -1) @ qm[t - 2]
    post = torch.log(fact1 + 1e-6) + torch.log(fact2 + 1e-6)
    p = torch.softmax(post.double(), -1).numpy()
    n = 400_000
    dev = "cuda"
    L = logits[None].expand(n, A).contiguous().to(dev)
    xts = torch.full((n,), xt, dtype=torch.long, device=dev)
    ts = torch.full((n,), t, dtype=torch.long, device=dev)
    out = torch.empty(n, dtype=torch.long, device=dev)
    q1d, qmd = q1.contiguous().to(dev), qm.contiguous().to(dev)
    _lib.check(_lib.load().chm_debug_d3pm_philox(n, A, T, _lib.ptr(L), _lib.ptr(xts), _lib.ptr(ts), _lib.ptr(q1d),
                                                 _lib.ptr(qmd), 9, 0, _lib.ptr(out), _lib.stream_handle()),
               "chm_debug_d3pm_philox")
    counts = np.bincount(out.cpu().numpy(), minlength=A).astype(np.float64)
    exp = p * n
    big = exp >= 20  # pool the rare classes into one cell
    obs_c = np.append(counts[big], counts[~big].sum())
    exp_c = np.append(exp[big], exp[~big].sum())
    chi = stats.chisquare(obs_c, exp_c)
    print(f"d3pm: {int(big.sum())} cells + 1 pooled, chi2 {chi.statistic:.1f} p {chi.pvalue:.3f}; "
          f"top class p {p.max():.3f} freq {counts.max() / n:.3f}")
    assert chi.pvalue > 1e-4
