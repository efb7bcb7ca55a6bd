"""Noise schedules and D3PM tables of the sampling path.

Same module names, buffers and state_dict keys as the reference
(`chemeleon/utils/diff_utils.py`), so that a released checkpoint's
`beta_scheduler.*`, `sigma_scheduler.*` and `d3pm.*` buffers load unchanged.
These run once at construction (host, PyTorch), exactly like the
reference's; the per-step work on these tables happens in the HIP kernels
(`chm_sample_step`).
"""

import math

import numpy as np
import torch
import torch.nn as nn

DEFAULT_DTYPE = torch.get_default_dtype()


def cosine_beta_schedule(timesteps, s=0.008):
    """diff_utils.py:10-19"""
    x = torch.linspace(0, timesteps, timesteps + 1)
    ac = torch.cos(((x / timesteps) + s) / (1 + s) * math.pi * 0.5) ** 2
    ac = ac / ac[0]
    return torch.clip(1 - (ac[1:] / ac[:-1]), 0.0001, 0.9999)


def linear_beta_schedule(timesteps, beta_start, beta_end):
    return torch.linspace(beta_start, beta_end, timesteps)


def quadratic_beta_schedule(timesteps, beta_start, beta_end):
    return torch.linspace(beta_start ** 0.5, beta_end ** 0.5, timesteps) ** 2


def sigmoid_beta_schedule(timesteps, beta_start, beta_end):
    return torch.sigmoid(torch.linspace(-6, 6, timesteps)) * (beta_end - beta_start) + beta_start


def p_wrapped_normal(x, sigma, N=10, T=1.0):
    """diff_utils.py:35-39: 21-term periodic Gaussian."""
    p = 0
    for i in range(-N, N + 1):
        p = p + torch.exp(-((x + T * i) ** 2) / 2 / sigma ** 2)
    return p


def d_log_p_wrapped_normal(x, sigma, N=10, T=1.0):
    """diff_utils.py:42-46: score of the wrapped normal."""
    p = 0
    for i in range(-N, N + 1):
        p = p + (x + T * i) / sigma ** 2 * torch.exp(-((x + T * i) ** 2) / 2 / sigma ** 2)
    return p / p_wrapped_normal(x, sigma, N, T)


def sigma_norm(sigma, T=1.0, sn=10000):
    """diff_utils.py:49-54: Monte-Carlo E[score^2]; draws from the global RNG."""
    sigmas = sigma[None, :].repeat(sn, 1)
    xs = (sigma * torch.randn_like(sigmas)) % T
    return (d_log_p_wrapped_normal(xs, sigmas, T=T) ** 2).mean(dim=0)


class BetaScheduler(nn.Module):
    """VP schedule for lattices (diff_utils.py:57-106)."""

    def __init__(self, timesteps, scheduler_mode, beta_start=0.0001, beta_end=0.02):
        super().__init__()
        self.timesteps = timesteps
        if scheduler_mode == "cosine":
            b = cosine_beta_schedule(timesteps)
        elif scheduler_mode == "linear":
            b = linear_beta_schedule(timesteps, beta_start, beta_end)
        elif scheduler_mode == "quadratic":
            b = quadratic_beta_schedule(timesteps, beta_start, beta_end)
        elif scheduler_mode == "sigmoid":
            b = sigmoid_beta_schedule(timesteps, beta_start, beta_end)
        else:
            raise ValueError(f"Invalid scheduler mode: {scheduler_mode}")
        betas = torch.cat([torch.zeros([1]), b], dim=0)
        alphas = 1.0 - betas
        ac = torch.cumprod(alphas, axis=0)
        pm1 = torch.ones_like(betas)
        pm1[1:] = betas[1:] * torch.sqrt(ac[:-1]) / (1.0 - ac[1:])
        pm2 = torch.zeros_like(betas)
        pm2[1:] = (1.0 - ac[:-1]) * torch.sqrt(alphas[1:]) / (1.0 - ac[1:])
        sig = torch.zeros_like(betas)
        sig[1:] = betas[1:] * (1.0 - ac[:-1]) / (1.0 - ac[1:])
        for name, val in (("betas", betas), ("alphas", alphas), ("alphas_cumprod", ac), ("posterior_mean_coeff1", pm1),
                          ("posterior_mean_coeff2", pm2), ("sigmas", torch.sqrt(sig))):
            self.register_buffer(name, val.to(DEFAULT_DTYPE))

    def uniform_sample_t(self, batch_size, device):
        return torch.from_numpy(np.random.choice(np.arange(1, self.timesteps + 1), batch_size)).to(device)


class SigmaScheduler(nn.Module):
    """VE schedule for fractional coordinates (diff_utils.py:109-131)."""

    def __init__(self, timesteps, sigma_begin=0.01, sigma_end=1.0):
        super().__init__()
        self.timesteps = timesteps
        self.sigma_begin = sigma_begin
        self.sigma_end = sigma_end
        sig = torch.FloatTensor(np.exp(np.linspace(np.log(sigma_begin), np.log(sigma_end), timesteps)))
        sn = sigma_norm(sig)
        self.register_buffer("sigmas", torch.cat([torch.zeros([1]), sig], dim=0).to(DEFAULT_DTYPE))
        self.register_buffer("sigmas_norm", torch.cat([torch.ones([1]), sn], dim=0).to(DEFAULT_DTYPE))

    def uniform_sample_t(self, batch_size, device):
        return torch.from_numpy(np.random.choice(np.arange(1, self.timesteps + 1), batch_size)).to(device)


class D3PM(nn.Module):
    """Absorbing-state discrete diffusion tables for atom types
    (diff_utils.py:152-213). Sampling itself (`p_logits`) runs in the
    `k_d3pm` HIP kernel; `p_logits` here dispatches to it."""

    def __init__(self, beta_scheduler: nn.Module, num_timesteps: int, max_atoms: int, d3pm_hybrid_coeff: float):
        super().__init__()
        self.beta_scheduler = beta_scheduler
        self.num_timesteps = num_timesteps
        self.max_atoms = max_atoms
        self.hybrid_coeff = d3pm_hybrid_coeff
        self.eps = 1.0e-6
        one = []
        for t in range(num_timesteps + 1):
            bt = beta_scheduler.betas[t]
            m = torch.diag(torch.full((max_atoms,), 1 - bt), 0)
            m[:, 0] += bt  # every class may jump to the absorbing class 0
            one.append(m)
        one = torch.stack(one, 0)
        self.register_buffer("q_one_step_mats", one)
        q = one[0]
        cum = [q]
        for t in range(1, num_timesteps + 1):
            q = q @ one[t]
            cum.append(q)
        self.register_buffer("q_mats", torch.stack(cum, 0))

    def p_logits(self, pred_x_start_logits, x_t_atom_types, t_per_node, noise):
        """diff_utils.py:307-329 on the GPU (k_d3pm): Gumbel-argmax sample of
        q(x_{t-1} | x_t, x0 = softmax(logits)). Inputs on the HIP device."""
        from chemeleon_amd import _lib
        lg = pred_x_start_logits.float().contiguous()
        xt = x_t_atom_types.long().contiguous()
        tn = t_per_node.long().contiguous()
        nz = noise.float().contiguous()
        _lib.require_device(lg, xt, tn, nz, self.q_mats)
        out = torch.empty_like(xt)
        N, A = lg.shape
        L = _lib.load()
        _lib.check(L.chm_d3pm_sample(N, A, self.num_timesteps, _lib.ptr(lg), _lib.ptr(xt), _lib.ptr(tn), _lib.ptr(nz),
                                     _lib.ptr(self.q_one_step_mats.contiguous()), _lib.ptr(self.q_mats.contiguous()),
                                     _lib.ptr(out), _lib.stream_handle()), "chm_d3pm_sample")
        return out
