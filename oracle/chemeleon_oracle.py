"""ORACLE — test infrastructure only. Never imported by the product path.

A CPU (PyTorch fp32, ATen CPU kernels) restatement of ryannduma/chemeleon's
reverse-diffusion sampling loop, written from the reference's behaviour, not
copied from it. Every function cites the reference file:line it restates
(paths relative to the reference repo root).

Who may use this module: `tests/`, `__graft_entry__.smoke()` (as the checker)
and `bench.py`'s `cpu_baseline` leg (timed as the "port" CPU baseline).
The HIP product path (`chemeleon_amd`) must never import it.

Pinning: `tests/golden/make_golden.py` imports the unmodified reference under
import shims in the development container and writes fixtures to
`tests/golden/`; `tests/test_oracle_golden.py` checks this oracle against
them (bit-exact or within 1e-6). So parity is pinned by the reference's own
outputs on the same inputs, not by reference unit tests (it has none).
"""

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

LATTICE_MASK = torch.tensor([[1, 0, 1], [1, 1, 1], [0, 0, 1]]).bool()  # chemeleon/modules/chemeleon.py:70-72
EPS = 1.0e-6  # chemeleon/utils/diff_utils.py:165


# ----------------------------------------------------------------------------
# schedules  (chemeleon/utils/diff_utils.py)
# ----------------------------------------------------------------------------
def cosine_betas(T: int, s: float = 0.008) -> torch.Tensor:
    """diff_utils.py:10-19 — Nichol & Dhariwal cosine schedule, clipped."""
    x = torch.linspace(0, T, T + 1)
    abar = torch.cos(((x / T) + s) / (1 + s) * math.pi * 0.5) ** 2
    abar = abar / abar[0]
    return torch.clip(1 - (abar[1:] / abar[:-1]), 0.0001, 0.9999)


def beta_schedule(T: int, mode: str = "cosine", beta_start=0.0001, beta_end=0.02) -> Dict[str, torch.Tensor]:
    """diff_utils.py:57-102 — BetaScheduler buffers, index 0 = no noise."""
    if mode == "cosine":
        b = cosine_betas(T)
    elif mode == "linear":
        b = torch.linspace(beta_start, beta_end, T)
    elif mode == "quadratic":
        b = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, T) ** 2
    elif mode == "sigmoid":
        b = torch.sigmoid(torch.linspace(-6, 6, T)) * (beta_end - beta_start) + beta_start
    else:
        raise ValueError(f"Invalid scheduler mode: {mode}")
    betas = torch.cat([torch.zeros([1]), b])
    alphas = 1.0 - betas
    abar = torch.cumprod(alphas, axis=0)
    sig = torch.zeros_like(betas)
    sig[1:] = betas[1:] * (1.0 - abar[:-1]) / (1.0 - abar[1:])
    return {"betas": betas, "alphas": alphas, "alphas_cumprod": abar, "sigmas": torch.sqrt(sig)}


def p_wrapped_normal(x, sigma, N=10, T=1.0):
    """diff_utils.py:35-39"""
    p = 0
    for i in range(-N, N + 1):
        p = p + torch.exp(-((x + T * i) ** 2) / 2 / sigma ** 2)
    return p


def d_log_p_wrapped_normal(x, sigma, N=10, T=1.0):
    """diff_utils.py:42-46"""
    p = 0
    for i in range(-N, N + 1):
        p = p + (x + T * i) / sigma ** 2 * torch.exp(-((x + T * i) ** 2) / 2 / sigma ** 2)
    return p / p_wrapped_normal(x, sigma, N, T)


def sigma_schedule(T: int, sigma_begin=0.01, sigma_end=1.0, sn=10000):
    """diff_utils.py:49-54,109-127 — VE sigmas (numpy geomspace, f64 -> f32)
    and the Monte-Carlo score norm. Draws sn*T normals from the global torch
    generator, exactly as the reference constructor does."""
    sig = torch.FloatTensor(np.exp(np.linspace(np.log(sigma_begin), np.log(sigma_end), T)))
    sigs = sig[None, :].repeat(sn, 1)
    xs = (sig * torch.randn_like(sigs)) % 1.0
    norm = (d_log_p_wrapped_normal(xs, sigs) ** 2).mean(dim=0)
    return torch.cat([torch.zeros([1]), sig]), torch.cat([torch.ones([1]), norm])


# ----------------------------------------------------------------------------
# D3PM absorbing-state discrete diffusion  (diff_utils.py:152-329)
# ----------------------------------------------------------------------------
def d3pm_tables(betas: torch.Tensor, T: int, A: int):
    """diff_utils.py:168-213 — one-step matrices Q_t = diag(1-b_t) with b_t
    added to column 0, and cumulative products Q_1..Q_t."""
    one = []
    for t in range(T + 1):
        m = torch.diag(torch.full((A,), 1 - betas[t]), 0)
        m[:, 0] += betas[t]
        one.append(m)
    one = torch.stack(one, 0)
    q = one[0]
    cum = [q]
    for t in range(1, T + 1):
        q = q @ one[t]
        cum.append(q)
    return one, torch.stack(cum, 0)


def d3pm_p_sample(pred_logits, x_t, t_per_node, noise, q_one_step, q_mats):
    """diff_utils.py:258-286 (q_posterior_logits, x0 given as logits) and
    :307-329 (p_logits). Note the reference's indices: fact1 reads the one-step
    matrix at t-1 (`at`, :234), fact2 the cumulative matrix at t-2 (:280),
    which wraps to the last entry at t=1 where `where(t==1)` discards it."""
    fact1 = q_one_step.transpose(1, 2)[t_per_node - 1, x_t, :]
    sm = torch.softmax(pred_logits, dim=-1)
    fact2 = torch.einsum("bc,bcd->bd", sm, q_mats[t_per_node - 2])
    out = torch.log(fact1 + EPS) + torch.log(fact2 + EPS)
    post = torch.where((t_per_node == 1)[:, None], pred_logits, out)
    noise = torch.clamp(noise, min=EPS, max=1.0)
    nz = (t_per_node != 1).to(x_t.dtype)[:, None]
    g = -torch.log(-torch.log(noise))
    return torch.argmax(post + g * nz, dim=-1)


def d3pm_q_sample(x0, t_per_node, noise, q_mats):
    """diff_utils.py:236-256 — Categorical(x_0 Q_{1..t}) through the Gumbel argmax."""
    logits = torch.log(q_mats[t_per_node - 1, x0, :] + EPS)
    noise = torch.clip(noise, EPS, 1.0)
    return torch.argmax(logits + -torch.log(-torch.log(noise)), dim=-1)


def d3pm_q_posterior_logits(x0, x_t, t_per_node, q_one_step, q_mats, x0_is_logits: bool):
    """diff_utils.py:258-286 — logits of q(x_{t-1} | x_t, x_0); x_0 as indices (one-hot, + eps, log)
    or as logits (`is_x_0_one_hot=True` in the reference's naming)."""
    A = q_mats.shape[-1]
    x0_logits = x0.clone() if x0_is_logits else torch.log(F.one_hot(x0, A) + EPS)
    fact1 = q_one_step.transpose(1, 2)[t_per_node - 1, x_t, :]
    fact2 = torch.einsum("bc,bcd->bd", torch.softmax(x0_logits, dim=-1), q_mats[t_per_node - 2])
    out = torch.log(fact1 + EPS) + torch.log(fact2 + EPS)
    return torch.where((t_per_node == 1)[:, None], x0_logits, out)


def categorical_kl_logits(l1, l2, eps=1.0e-6):
    """diff_utils.py:288-305 — mean over rows of KL(C(l1) || C(l2)), logits shifted by eps."""
    out = torch.softmax(l1 + eps, dim=-1) * (torch.log_softmax(l1 + eps, dim=-1) - torch.log_softmax(l2 + eps, dim=-1))
    return out.sum(dim=-1).mean()


# ----------------------------------------------------------------------------
# score network  (chemeleon/modules/cspnet.py)
# ----------------------------------------------------------------------------
def time_embedding(t: torch.Tensor, dim: int) -> torch.Tensor:
    """cspnet.py:28-35 — sinusoidal, [sin | cos]."""
    half = dim // 2
    e = math.log(10000) / (half - 1)
    e = torch.exp(torch.arange(half) * -e)
    e = t[:, None] * e[None, :]
    return torch.cat((e.sin(), e.cos()), dim=-1)


def fourier_frequencies(num_freqs: int) -> torch.Tensor:
    """cspnet.py:45 — 2*pi*k rounded to fp32 after the int->float product."""
    return 2 * math.pi * torch.arange(num_freqs)


def fourier(frac_diff: torch.Tensor, num_freqs: int) -> torch.Tensor:
    """cspnet.py:48-52 — [E,3] -> [E, 3*K sin | 3*K cos], axis-major."""
    e = frac_diff.unsqueeze(-1) * fourier_frequencies(num_freqs)[None, None, :]
    e = e.reshape(-1, num_freqs * 3)
    return torch.cat((e.sin(), e.cos()), dim=-1)


def fc_edges(natoms: Sequence[int]) -> torch.Tensor:
    """cspnet.py:320-323 — block-diagonal all-ones adjacency through
    dense_to_sparse: row-major (i, j) pairs inside each crystal, self loops
    included. Built directly instead of through a dense N x N matrix."""
    rows, cols, off = [], [], 0
    for n in natoms:
        n = int(n)
        ii = torch.arange(n).repeat_interleave(n) + off
        jj = torch.arange(n).repeat(n) + off
        rows.append(ii)
        cols.append(jj)
        off += n
    return torch.stack([torch.cat(rows), torch.cat(cols)], 0)


def scatter_mean(src: torch.Tensor, index: torch.Tensor, dim_size: int) -> torch.Tensor:
    """chemeleon/utils/scatter.py:27-48,88-112 — scatter_add_ sum, count,
    count clamped to 1, true division."""
    out = torch.zeros((dim_size,) + tuple(src.shape[1:]), dtype=src.dtype)
    out.scatter_add_(0, index.view(-1, *([1] * (src.dim() - 1))).expand_as(src), src)
    cnt = torch.zeros(dim_size, dtype=src.dtype).scatter_add_(0, index, torch.ones(index.shape, dtype=src.dtype))
    cnt[cnt < 1] = 1
    return out / cnt.view(-1, *([1] * (src.dim() - 1)))


def _ln(x, sd, p):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], 1e-5)


def cspnet_forward(sd: Dict[str, torch.Tensor], cfg: Dict, atom_types, frac_coords, lattices,
                   num_atoms, node2graph, t_emb=None, text=None, hidden: Optional[List] = None):
    """cspnet.py:345-405 (ln, ip, smooth=False; cfg["edge_style"] "fc" (default) or "knn").

    Returns (type_logits [N,A], lattice_out [B,3,3], coords_out [N,3],
    node_features [N,H]). If `hidden` is a list, the node features after
    each layer are appended to it."""
    silu = F.silu
    natoms = [int(n) for n in num_atoms]
    if cfg.get("edge_style", "fc") == "knn":  # cspnet.py:325-343 (oracle/knn_oracle.py)
        from oracle.knn_oracle import knn_edges
        edges, frac_diff = knn_edges(natoms, frac_coords, lattices, cfg.get("max_neighbors", 20))
    else:
        edges = fc_edges(natoms)
        frac_diff = (frac_coords[edges[1]] - frac_coords[edges[0]]) % 1.0  # cspnet.py:324
    e2g = node2graph[edges[0]]  # :356
    h = F.embedding(atom_types, sd["node_embedding.weight"])  # :357
    t_atom = t_emb.repeat_interleave(num_atoms, dim=0) if t_emb is not None else None  # :360
    x_atom = text.repeat_interleave(num_atoms, dim=0) if text is not None else None  # :365
    if t_atom is not None and x_atom is not None:
        cond_in = torch.cat([t_atom, x_atom], dim=1)
    else:
        cond_in = t_atom if t_atom is not None else x_atom
    feats = fourier(frac_diff, cfg["num_freqs"])
    llt = (lattices @ lattices.transpose(-1, -2)).view(-1, 9) if cfg.get("ip", True) else lattices.view(-1, 9)
    for i in range(cfg["num_layers"]):
        if cond_in is not None:  # FilmLayer.forward, :78-97
            c = silu(F.linear(cond_in, sd["film_layer.mlp_cond.0.weight"], sd["film_layer.mlp_cond.0.bias"]))
            scale, shift = c.chunk(2, dim=1)
            x0 = h
            y = F.linear(h, sd["film_layer.proj.weight"], sd["film_layer.proj.bias"])
            y = _ln(y, sd, "film_layer.norm")
            h = silu(y * scale + shift) + x0
        p = f"csp_layer_{i}."
        hin = h  # CSPLayer.forward, :165-181
        hl = _ln(hin, sd, p + "layer_norm")
        ein = torch.cat([hl[edges[0]], hl[edges[1]], llt[e2g], feats], dim=1)  # :138-150
        m = silu(F.linear(ein, sd[p + "edge_mlp.0.weight"], sd[p + "edge_mlp.0.bias"]))
        m = silu(F.linear(m, sd[p + "edge_mlp.2.weight"], sd[p + "edge_mlp.2.bias"]))
        agg = scatter_mean(m, edges[0], hl.shape[0])  # :155-160
        nin = torch.cat([hl, agg], dim=1)
        o = silu(F.linear(nin, sd[p + "node_mlp.0.weight"], sd[p + "node_mlp.0.bias"]))
        o = silu(F.linear(o, sd[p + "node_mlp.2.weight"], sd[p + "node_mlp.2.bias"]))
        h = hin + o
        if hidden is not None:
            hidden.append(h)
    h = _ln(h, sd, "final_layer_norm")  # :385-386
    coords = F.linear(h, sd["coord_out.weight"])  # :388
    g = scatter_mean(h, node2graph, len(natoms))  # :390
    lat = F.linear(g, sd["lattice_out.weight"]).view(-1, 3, 3)
    if cfg.get("ip", True):
        lat = torch.einsum("bij,bjk->bik", lat, lattices)  # :394
    types = F.linear(h, sd["type_out.weight"], sd["type_out.bias"])  # :396
    return types, lat, coords, h


# ----------------------------------------------------------------------------
# sampler  (chemeleon/modules/chemeleon.py)
# ----------------------------------------------------------------------------
class OracleModel:
    """Holds what `Chemeleon.__init__` builds for sampling (chemeleon.py:32-91):
    schedules, D3PM tables, decoder weights."""

    def __init__(self, cfg: Dict, state_dict: Dict[str, torch.Tensor]):
        self.cfg = cfg
        self.T = cfg["timesteps"]
        self.A = cfg["max_atoms"]
        self.beta = beta_schedule(self.T, cfg["beta_schedule"])
        self.sigmas, self.sigmas_norm = sigma_schedule(self.T)  # consumes global RNG like the reference
        self.sigma_begin = 0.01
        self.q_one_step, self.q_mats = d3pm_tables(self.beta["betas"], self.T, self.A)
        self.sd = {k: v.detach().float().cpu() for k, v in state_dict.items()}

    def decoder(self, t_emb, a, x, l, natoms, n2g, text):
        return cspnet_forward(self.sd, self.cfg, a, x, l, natoms, n2g, t_emb, text)

    def model_predictions(self, t_emb, a, x, l, natoms, n2g, cond_scale, cond, null):
        """chemeleon.py:246-303 — classifier-free guidance over two decoder calls."""
        pc = self.decoder(t_emb, a, x, l, natoms, n2g, cond)
        pn = self.decoder(t_emb, a, x, l, natoms, n2g, null)
        mix = lambda n_, c_: (1 - cond_scale) * n_ + cond_scale * c_
        return mix(pn[0], pc[0]), mix(pn[1], pc[1]), mix(pn[2], pc[2])

    def step(self, t: int, a_t, x_t, l_t, natoms, n2g, cond, null, noise, cond_scale=2.0, step_lr=1e-5):
        """One reverse step, chemeleon.py:379-466. `noise` = (rand_a [N,A],
        rand_l [B,3,3], rand_x1 [N,3], rand_x2 [N,3]) or None at t == 1.
        Returns (a_{t-1}, x_{t-1} wrapped to [0,1), l_{t-1}, x_{t-1/2})."""
        B = l_t.shape[0]
        N = x_t.shape[0]
        bt = torch.full((B,), t, dtype=torch.long)
        te = time_embedding(bt, self.cfg["time_dim"])
        pa, pl, px = self.model_predictions(te, a_t, x_t, l_t, natoms, n2g, cond_scale, cond, null)
        if noise is None:
            ra, rl, rx1, rx2 = torch.zeros(N, self.A), torch.zeros(B, 3, 3), torch.zeros(N, 3), torch.zeros(N, 3)
        else:
            ra, rl, rx1, rx2 = noise
        a_prev = d3pm_p_sample(pa, a_t, bt[n2g], ra, self.q_one_step, self.q_mats)
        al = self.beta["alphas"][t]
        ab = self.beta["alphas_cumprod"][t]
        sg = self.beta["sigmas"][t]
        c0 = 1.0 / torch.sqrt(al)
        c1 = (1 - al) / torch.sqrt(1 - ab)
        rl = rl * LATTICE_MASK
        l_prev = (c0 * (l_t - c1 * pl) + sg * rl) * LATTICE_MASK
        if t == self.T:
            l_prev = l_prev.clip(-6, 6)
        sx = self.sigmas[t]
        sn = self.sigmas_norm[t]
        sa = self.sigmas[t - 1]
        step = sx ** 2 - sa ** 2
        std = torch.sqrt((sa ** 2 * (sx ** 2 - sa ** 2)) / (sx ** 2))
        x_half = x_t - step * (px * torch.sqrt(sn)) + std * rx1
        _, _, px2 = self.model_predictions(te, a_prev, x_half, l_prev, natoms, n2g, cond_scale, cond, null)
        step2 = step_lr * (sx / self.sigma_begin) ** 2
        std2 = torch.sqrt(2 * step2)
        x_prev = x_half - step2 * (px2 * torch.sqrt(sn)) + std2 * rx2
        return a_prev, x_prev % 1.0, l_prev, x_half

    def training_forward(self, a0, x0, l0, natoms, t, rand_a, noise_l, noise_x, text):
        """chemeleon.py:137-244 with the draws given: t [B], rand_a [N,A], noise_l [B,3,3] (unmasked),
        noise_x [N,3]; `text` [B, text_dim] as get_text_embeds returned it. Returns the loss dict."""
        nat = torch.as_tensor([int(n) for n in natoms])
        B = len(nat)
        n2g = torch.arange(B).repeat_interleave(nat)
        te = time_embedding(t, self.cfg["time_dim"])
        ac = self.beta["alphas_cumprod"][t]
        c0, c1 = torch.sqrt(ac), torch.sqrt(1.0 - ac)
        sig, sn = self.sigmas[t], self.sigmas_norm[t]
        tn = t[n2g]
        a_t = d3pm_q_sample(a0, tn, rand_a, self.q_mats)
        nl = noise_l * LATTICE_MASK
        l_t = c0[:, None, None] * l0 + c1[:, None, None] * nl
        s_a, sn_a = sig[n2g][:, None], sn[n2g][:, None]
        target = d_log_p_wrapped_normal(s_a * noise_x, s_a) / torch.sqrt(sn_a)
        x_t = (x0 + s_a * noise_x) % 1.0
        types, lat, coords, _ = self.decoder(te, a_t, x_t, l_t, nat, n2g, text)
        true_post = d3pm_q_posterior_logits(a0, a_t, tn, self.q_one_step, self.q_mats, False)
        pred_post = d3pm_q_posterior_logits(types, a_t, tn, self.q_one_step, self.q_mats, True)
        vb = categorical_kl_logits(true_post, pred_post)
        ce = F.cross_entropy(types, a0)
        la = vb + ce * self.cfg.get("d3pm_hybrid_coeff", 1.0)
        ll = F.mse_loss(lat.masked_select(LATTICE_MASK), nl.masked_select(LATTICE_MASK))
        lx = F.mse_loss(coords, target)
        loss = (self.cfg.get("cost_atom_types", 1.0) * la + self.cfg.get("cost_lattice", 1.0) * ll
                + self.cfg.get("cost_coords", 1.0) * lx)
        return {"loss": loss, "vb_loss_atom_types": vb, "ce_loss_atom_types": ce,
                "true_noise_lattice": nl.masked_select(LATTICE_MASK), "pred_noise_lattice": lat.masked_select(LATTICE_MASK),
                "true_noise_coords": target, "pred_noise_coords": coords, "x_t_atom_types": a_t}

    def draw_noise(self, t: int, N: int, B: int):
        """RNG order of chemeleon.py:400-404,418,435,455 on the global CPU
        generator; nothing is drawn at t == 1."""
        if t <= 1:
            return None
        ra = torch.rand((N, self.A))
        rl = torch.randn(B, 3, 3)
        rx1 = torch.randn(N, 3)
        rx2 = torch.randn(N, 3)
        return ra, rl, rx1, rx2

    def sample(self, natoms: Sequence[int], cond, null, cond_scale=2.0, step_lr=1e-5, t_stop: int = 0):
        """chemeleon.py:305-467 as a generator of (t-1, a, x, l) states.
        `cond`/`null` are the [B, text_dim] conditioning vectors the text
        encoder would return. Draws from the global CPU generator."""
        natoms = [int(n) for n in natoms]
        B, N = len(natoms), sum(natoms)
        nat = torch.tensor(natoms)
        n2g = torch.arange(B).repeat_interleave(nat)
        a = torch.zeros(N, dtype=torch.long)  # :347
        l = torch.randn(B, 3, 3) * LATTICE_MASK  # :348
        x = torch.randn(N, 3)  # :349
        x = x % 1.0
        yield self.T, a, x, l
        for t in range(self.T, t_stop, -1):
            nz = self.draw_noise(t, N, B)
            a, x, l, _ = self.step(t, a, x, l, nat, n2g, cond, null, nz, cond_scale, step_lr)
            yield t - 1, a, x, l
