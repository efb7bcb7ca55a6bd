"""Chemeleon sampler — drop-in for `chemeleon.modules.chemeleon.Chemeleon`
on the sampling path (reference `chemeleon/modules/chemeleon.py:31-490`).

Same constructor (`_config` dict of hyper-parameters), same buffers and
state_dict keys (`beta_scheduler.*`, `sigma_scheduler.*`, `d3pm.*`,
`decoder.*`), same `sample()` / `_sample_generator()` / `model_predictions()`
signatures and return types. Each reverse step runs as one C-ABI call
(`chm_sample_step`): the predictor and corrector classifier-free-guidance
pairs, D3PM / DDPM / VE updates, all in HIP kernels on the caller's stream.

Noise
-----
* ``noise="torch"`` (default, parity mode): every random tensor is drawn
  from the global CPU torch generator in the order of the reference's CPU
  path (chemeleon.py:348-349, 400-404, 418, 435, 455) and uploaded, so a run
  seeded like the reference reproduces the reference CPU trajectory (the
  parity target). The reference run on a GPU would draw rand_l / rand_x
  (``randn_like`` of device tensors, :418, 435, 455) from the device
  generator instead; that stream is not reproduced.
* ``noise="philox"`` (throughput mode): noise is generated inside the step
  kernels from a counter-based Philox stream keyed by (seed, t, global
  node / graph index); results do not depend on how samples are sharded.

Text conditioning runs once per call on the host side of the boundary (north
star: "computed once on host and broadcast"). As in the reference
(chemeleon.py:37-52), a text_guide model builds its
`chemeleon_amd.text_encoder.TextEncoder` from the config (`text_encoder`,
`text_embed_dim`, `max_text_len`, `text_dim`, optional `path_ckpt_clip=`
CrystalCLIP checkpoint) — here only when a local copy of the language model is
available (`text_model_dir=` or $CHEMELEON_TEXT_MODEL_DIR; nothing is
downloaded). Alternatively pass any `text_encoder` object with the reference's
`get_text_embeds(texts, cond_drop_prob, device)` method, or pass
`text_embeds=` / `null_text_embeds=` tensors directly.
"""

import ctypes
import os
from typing import Any, Dict, Iterator, List, Optional, Tuple, Union

import torch
import torch.nn as nn

from chemeleon_amd import _lib
from chemeleon_amd.config import default_config
from chemeleon_amd.modules.cspnet import CSPNet, SinusoidalTimeEmbeddings
from chemeleon_amd.modules.schema import TrajectoryContainer, TrajectoryStep, step_to_atoms
from chemeleon_amd.noise import StepNoise
from chemeleon_amd.utils.diff_utils import D3PM, BetaScheduler, SigmaScheduler

CHECKPOINT_DIR = os.environ.get("CHEMELEON_CHECKPOINT_DIR",
                                os.path.join(os.path.dirname(os.path.dirname(__file__)), "checkpoints"))
# file names of the released checkpoints (reference chemeleon/constants.py:3-7)
PATH_CHEMELEON_GENERAL_TEXT = os.path.join(CHECKPOINT_DIR, "chemeleon-7fsg68c3.ckpt")
PATH_CHEMELEON_COMPOSITION = os.path.join(CHECKPOINT_DIR, "chemeleon-fksq6cgp.ckpt")


class Chemeleon(nn.Module):
    def __init__(self, _config: Dict[str, Any], text_encoder=None, **kwargs):
        super().__init__()
        cfg = default_config()
        cfg.update(_config)
        self.hparams = cfg
        self.time_embed = SinusoidalTimeEmbeddings(cfg["time_dim"])
        self.text_guide = cfg["text_guide"]
        self.cond_drop_prob = cfg.get("cond_drop_prob", 0.2)
        if text_encoder is None and self.text_guide:
            text_encoder = self._build_text_encoder(cfg, kwargs)
        self.text_encoder = text_encoder
        self.num_timesteps = cfg["timesteps"]
        self.beta_scheduler = BetaScheduler(timesteps=self.num_timesteps, scheduler_mode=cfg["beta_schedule"])
        self.sigma_scheduler = SigmaScheduler(timesteps=self.num_timesteps)
        self.max_atoms = cfg["max_atoms"]
        self.d3pm = D3PM(beta_scheduler=self.beta_scheduler, num_timesteps=cfg["timesteps"],
                         max_atoms=cfg["max_atoms"], d3pm_hybrid_coeff=cfg["d3pm_hybrid_coeff"])
        self.mask_lattice_matrix = torch.tensor([[1, 0, 1], [1, 1, 1], [0, 0, 1]]).bool()  # chemeleon.py:70-72
        self.decoder = CSPNet(hidden_dim=cfg["hidden_dim"], time_dim=cfg["time_dim"],
                              text_dim=cfg["text_dim"] if self.text_guide else 0, num_layers=cfg["num_layers"],
                              max_atoms=cfg["max_atoms"], act_fn=cfg["act_fn"], dis_emb=cfg["dis_emb"],
                              num_freqs=cfg["num_freqs"], edge_style=cfg["edge_style"], cutoff=cfg["cutoff"],
                              max_neighbors=cfg["max_neighbors"], ln=cfg["ln"], ip=cfg["ip"], smooth=cfg["smooth"],
                              pred_atom_types=cfg["pred_atom_types"])
        self._tables: Dict[Tuple, Tuple] = {}

    # ------------------------------------------------------------------ training forward
    def forward(self, batch, noise=None) -> Dict[str, Any]:
        """Training forward / validation loss (chemeleon.py:137-244) on the HIP path: per-graph t from
        `beta_scheduler.uniform_sample_t` (numpy's global generator, as the reference), q_sample of
        atom types (D3PM), lattices (variance preserving) and fractional coordinates (variance
        exploding, score target d_log_p_wrapped_normal / sqrt(sigma_norm)), one decoder call, the D3PM
        hybrid loss (KL of the posteriors + hybrid_coeff * cross entropy), lattice and coordinate MSEs.

        `batch` has atom_types [N], frac_coords [N,3], lattices [B,3,3], natoms [B], batch [N] and,
        for text-guided models, text (List[str]) (what Batch.from_data_list builds); `noise` =
        (t [B], rand_a [N,A], noise_lattice [B,3,3] (unmasked), noise_coords [N,3]) or None to draw
        them in the order of the reference's CPU path (t from numpy, the rest from the CPU torch
        generator; the reference on a GPU would take the randn_like draws of :174, 179 from the device
        generator, which is not reproduced).
        Returns the reference's dict (loss, vb_loss_atom_types, ce_loss_atom_types, true / pred noise
        lattice (masked entries), true / pred noise coords). No autograd: the HIP decoder has no
        backward pass."""
        dev = self.device
        if dev.type != "cuda":
            raise RuntimeError("Chemeleon (chemeleon_amd) runs on a HIP device only; call .to('cuda') first")
        natoms = [int(n) for n in (batch.natoms.tolist() if torch.is_tensor(batch.natoms) else batch.natoms)]
        B, N, A, T = len(natoms), sum(natoms), self.max_atoms, self.num_timesteps
        mask = self.mask_lattice_matrix
        if noise is None:
            t = self.beta_scheduler.uniform_sample_t(B, "cpu")  # chemeleon.py:147
            rand_a = torch.rand(N, A)  # :162-164
            nl = torch.randn(B, 3, 3)  # :170 (randn_like(l_0))
            nx = torch.randn(N, 3)  # :175 (randn_like(frac_coords))
        else:
            t, rand_a, nl, nx = noise
        nl = (nl.float().cpu() * mask).to(dev).contiguous()
        t = torch.as_tensor(t).long().to(dev).contiguous()
        rand_a = rand_a.float().to(dev).contiguous()
        nx = nx.float().to(dev).contiguous()
        a0 = batch.atom_types.long().to(dev).contiguous()
        x0 = batch.frac_coords.float().to(dev).contiguous()
        l0 = batch.lattices.float().to(dev).contiguous()
        te = self.time_embed(t).float().contiguous()  # :149
        text = None
        if self.text_guide:  # :186-191 (cond_drop_prob applies, as in training)
            if self.text_encoder is None:
                raise RuntimeError("text_guide model: pass text_encoder=... to compute the training loss")
            text = self.text_encoder.get_text_embeds(list(batch.text), self.cond_drop_prob, device=dev)
            text = text.float().to(dev).contiguous()
        tt, _keep = self._train_tables()
        out = torch.empty(6, device=dev)
        a_t = torch.empty(N, dtype=torch.long, device=dev)
        x_t = torch.empty(N, 3, device=dev)
        l_t = torch.empty(B, 3, 3, device=dev)
        target = torch.empty(N, 3, device=dev)
        pl = torch.empty(B, 3, 3, device=dev)
        pc = torch.empty(N, 3, device=dev)
        b = self.decoder.hip_batch(natoms, max_pairs=1)
        P = _lib.ptr
        _lib.require_device(t, a0, x0, l0, te, text, rand_a, nl, nx)
        _lib.check(_lib.load().chm_training_loss(b.handle, ctypes.byref(tt), P(t), P(a0), P(x0), P(l0), P(te), P(text),
                                                 P(rand_a), P(nl), P(nx), P(out), P(a_t), P(x_t), P(l_t), P(target),
                                                 P(pl), P(pc), _lib.stream_handle(dev)), "chm_training_loss")
        m = mask.to(dev)
        return {"loss": out[0], "vb_loss_atom_types": out[1], "ce_loss_atom_types": out[2],
                "true_noise_lattice": nl.masked_select(m), "pred_noise_lattice": pl.masked_select(m),
                "true_noise_coords": target, "pred_noise_coords": pc,
                "loss_atom_types": out[3], "loss_lattice": out[4], "loss_coords": out[5],
                "x_t_atom_types": a_t, "x_t_coords": x_t, "x_t_lattice": l_t}

    def _train_tables(self):
        """Device tables of the training forward: {sqrt(abar_t), sqrt(1 - abar_t), sigma_t,
        sigmas_norm_t} per t (the reference's fp32 expressions, chemeleon.py:151-157) and the D3PM
        matrices; cached per device."""
        dev = self.device
        bufs = (self.beta_scheduler.alphas_cumprod, self.sigma_scheduler.sigmas, self.sigma_scheduler.sigmas_norm,
                self.d3pm.q_one_step_mats, self.d3pm.q_mats)
        key = ("train", str(dev), tuple((b.data_ptr(), b._version) for b in bufs),
               tuple(float(self.hparams[k]) for k in ("cost_atom_types", "cost_lattice", "cost_coords")))
        if key not in self._tables:
            for k in [k for k in self._tables if k[0] == "train"]:  # (one training entry at a time)
                del self._tables[k]
            ac = self.beta_scheduler.alphas_cumprod.float().cpu()
            coef = torch.stack([torch.sqrt(ac), torch.sqrt(1.0 - ac), self.sigma_scheduler.sigmas.float().cpu(),
                                self.sigma_scheduler.sigmas_norm.float().cpu()], dim=1).contiguous().to(dev)
            q1 = self.d3pm.q_one_step_mats.float().contiguous().to(dev)
            qm = self.d3pm.q_mats.float().contiguous().to(dev)
            h = self.hparams
            tt = _lib.chm_train_tables(self.num_timesteps, _lib.ptr(coef), _lib.ptr(q1), _lib.ptr(qm),
                                       float(self.d3pm.hybrid_coeff), float(h["cost_atom_types"]),
                                       float(h["cost_lattice"]), float(h["cost_coords"]))
            self._tables[key] = (tt, (coef, q1, qm))
        return self._tables[key]

    @staticmethod
    def _build_text_encoder(cfg, kwargs):
        """reference chemeleon.py:37-52, from local files only; None when no
        local language model is configured (then texts need an injected encoder)."""
        tdir = kwargs.get("text_model_dir")
        if tdir is None and not os.environ.get("CHEMELEON_TEXT_MODEL_DIR"):
            return None
        from chemeleon_amd.text_encoder import CrystalClip, TextEncoder
        clip = None
        if kwargs.get("path_ckpt_clip"):
            clip = CrystalClip.load_from_checkpoint(kwargs["path_ckpt_clip"], text_model_dir=tdir, graph=False)
        return TextEncoder(text_encoder_name=cfg["text_encoder"], text_embed_dim=cfg["text_embed_dim"],
                           max_text_len=cfg["max_text_len"], text_dim=cfg["text_dim"],
                           trainable_text_encoder=cfg["trainable_text_encoder"], pretrained_clip_model=clip,
                           local_path=None if clip is not None else tdir)

    # ------------------------------------------------------------------ loading
    @property
    def device(self):
        return next(self.decoder.parameters()).device

    @classmethod
    def load_from_checkpoint(cls, path: str, text_encoder=None, map_location="cpu", strict: bool = True, **kwargs):
        """Lightning checkpoint -> model (reference chemeleon.py:113-115 via
        LightningModule.load_from_checkpoint). Loaded with weights_only=True.
        Buffers (schedules, sigmas_norm, D3PM tables) come from the file."""
        ck = torch.load(path, map_location=map_location, weights_only=True)
        hp = dict(ck.get("hyper_parameters", {}))
        extra = {k: kwargs.pop(k) for k in ("text_model_dir", "path_ckpt_clip") if k in kwargs}
        hp.update(kwargs)
        m = cls(hp, text_encoder=text_encoder, **extra)
        sd = ck["state_dict"]
        own = {k: v for k, v in sd.items() if not k.startswith("text_encoder.")}
        missing, unexpected = m.load_state_dict(own, strict=False)
        missing = [k for k in missing if not k.startswith("text_encoder.")]
        if strict and (missing or unexpected):
            raise RuntimeError(f"checkpoint mismatch: missing {missing}, unexpected {unexpected}")
        if m.text_encoder is not None and isinstance(m.text_encoder, nn.Module):
            te = {k[len("text_encoder."):]: v for k, v in sd.items() if k.startswith("text_encoder.")}
            te_missing, te_unexpected = m.text_encoder.load_state_dict(te, strict=False)
            # the frozen language model (and a CrystalCLIP's own copy of it) is sourced from the local
            # model directory, and the CrystalCLIP graph side is training / retrieval only; everything
            # trained with the sampler (text_emb.*, null_text_embeds, the CLIP projection) must come
            # from the checkpoint
            frozen = ("text_encoder.", "clip_model.text_encoder.", "clip_model.graph_encoder.",
                      "clip_model.graph_proj.")
            te_missing = [k for k in te_missing if not k.startswith(frozen)]
            te_unexpected = [k for k in te_unexpected if not k.startswith(frozen)]
            if strict and (te_missing or te_unexpected):
                raise RuntimeError(f"checkpoint text-encoder mismatch: missing {te_missing}, "
                                   f"unexpected {te_unexpected}")
        return m

    @classmethod
    def _load_released(cls, path, **kwargs):
        if not os.path.exists(path):
            raise FileNotFoundError(
                f"{path} not found. The released checkpoints are downloaded by the reference from figshare "
                "(chemeleon/constants.py:9-14); this build does not download. Place the file there or set "
                "CHEMELEON_CHECKPOINT_DIR.")
        return cls.load_from_checkpoint(path, **kwargs)

    @classmethod
    def load_general_text_model(cls, *args, **kwargs):
        return cls._load_released(PATH_CHEMELEON_GENERAL_TEXT, **kwargs)

    @classmethod
    def load_composition_model(cls, *args, **kwargs):
        return cls._load_released(PATH_CHEMELEON_COMPOSITION, **kwargs)

    # ------------------------------------------------------------------ tables
    def schedule_tables(self, step_lr: float):
        """Per-t scalar coefficients computed with the reference's own fp32
        expressions (chemeleon.py:413-457) on the host, once; plus the
        time-embedding table (cspnet.py:28-35). Returns (chm_schedule, keepalive)."""
        dev = self.device
        bufs = [b for mod in (self.beta_scheduler, self.sigma_scheduler, self.d3pm) for b in mod.buffers()]
        key = (str(dev), float(step_lr), tuple((b.data_ptr(), b._version) for b in bufs))
        if key in self._tables:
            return self._tables[key]
        if len(self._tables) >= 4:
            self._tables.pop(next(iter(self._tables)))
        T = self.num_timesteps
        bs, ss = self.beta_scheduler, self.sigma_scheduler
        al_, ac_, sg_ = bs.alphas.cpu(), bs.alphas_cumprod.cpu(), bs.sigmas.cpu()
        sx_, sn_ = ss.sigmas.cpu(), ss.sigmas_norm.cpu()
        coef = torch.zeros(T + 1, 8)
        for t in range(1, T + 1):
            alphas, alphas_cumprod, sigmas = al_[t], ac_[t], sg_[t]
            c0 = 1.0 / torch.sqrt(alphas)
            c1 = (1 - alphas) / torch.sqrt(1 - alphas_cumprod)
            sigma_x, sigma_norm, adj = sx_[t], sn_[t], sx_[t - 1]
            step_size = sigma_x ** 2 - adj ** 2
            std_x = torch.sqrt((adj ** 2 * (sigma_x ** 2 - adj ** 2)) / (sigma_x ** 2))
            step2 = step_lr * (sigma_x / ss.sigma_begin) ** 2
            std2 = torch.sqrt(2 * step2)
            coef[t] = torch.stack([c0, c1, sigmas, step_size, std_x, torch.sqrt(sigma_norm), step2, std2])
        temb = self.time_embed(torch.arange(T + 1))
        coef_d = coef.to(dev).contiguous()
        temb_d = temb.float().to(dev).contiguous()
        q1 = self.d3pm.q_one_step_mats.to(dev).float().contiguous()
        qm = self.d3pm.q_mats.to(dev).float().contiguous()
        sched = _lib.chm_schedule(T, int(q1.shape[1]), int(temb_d.shape[1]), 0, coef_d.data_ptr(), temb_d.data_ptr(),
                                  q1.data_ptr(), qm.data_ptr())
        self._tables[key] = (sched, (coef_d, temb_d, q1, qm))
        return self._tables[key]

    # ------------------------------------------------------------------ API
    def model_predictions(self, time_emb, atom_types, frac_coords, lattices, batch_natoms, batch_idx,
                          cond_scale: float, text_embeds=None, null_text_embeds=None):
        """chemeleon.py:246-303 (both CFG decoder calls run as one batched
        HIP call)."""
        if self.text_guide:
            types, lat, coords, _ = self.decoder.forward_cfg(atom_types, frac_coords, lattices, batch_natoms,
                                                             time_emb, text_embeds, null_text_embeds)
            mix = lambda p: (1 - cond_scale) * p[1] + cond_scale * p[0]  # noqa: E731
            return mix(types), mix(lat), mix(coords)
        out = self.decoder(t=time_emb, atom_types=atom_types, frac_coords=frac_coords, lattices=lattices,
                           num_atoms=batch_natoms, node2graph=batch_idx)
        return out.atom_types_out, out.lattice_out, out.coords_out

    def _conditioning(self, texts, B, text_embeds, null_text_embeds):
        dev = self.device
        if not self.text_guide:
            return None, None
        if text_embeds is None or null_text_embeds is None:
            if self.text_encoder is None:
                raise RuntimeError("text_guide model: pass text_encoder=... or text_embeds=/null_text_embeds=")
            if texts is None:
                raise ValueError("texts are required for a text-guided model")
            text_embeds = self.text_encoder.get_text_embeds(texts, cond_drop_prob=0.0, device=dev)
            null_text_embeds = self.text_encoder.get_text_embeds(texts, cond_drop_prob=1.0, device=dev)
        cond = text_embeds.float().to(dev).expand(B, -1).contiguous()
        null = null_text_embeds.float().to(dev).expand(B, -1).contiguous()
        return cond, null

    @torch.no_grad()
    def sample_states(self, natoms: Union[int, List[int]], texts: Optional[Union[str, List[str]]] = None,
                      cond_scale: float = 2.0, step_lr: float = 1e-5, *, noise: str = "torch", seed: int = 0,
                      text_embeds=None, null_text_embeds=None, clone: bool = True, t_stop: int = 0,
                      node_base: int = 0, graph_base: int = 0,
                      init: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                      graph: Optional[bool] = None, lanes: int = 1,
                      global_sizes: Optional[Tuple[int, int]] = None) -> Iterator[Tuple]:
        """Reverse loop of chemeleon.py:305-467 yielding device tensors
        (t, atom_types [N], frac_coords [N,3] in [0,1), lattices [B,3,3]),
        starting with the pure-noise state at t = T.

        graph=True (the default on fc batches): one reverse step is captured once
        as a HIP graph (chm_sample_step_dt reads t from device memory and
        decrements it) and replayed for every timestep. With noise="torch" the
        step reads its noise from fixed device buffers (chm_sample_step_dt_noise):
        every step's draws come from the CPU generator in the order of the reference's CPU path
        (rand(N, A), randn(B, 3, 3), randn(N, 3), randn(N, 3)), into pinned host
        buffers (two, alternating, so the next draw overlaps the running step)
        and are copied in stream order before the replay.

        Initial noise: from `init` = (l_T [B,3,3], x_T [N,3]) if given, else drawn
        on the CPU from the global generator (noise="torch", chemeleon.py:348-349)
        or from Generator(seed) (noise="philox") for THIS batch.

        global_sizes = (N_total, B_total) (noise="torch"): this batch is the shard
        of a larger run whose crystals start at node_base / graph_base. Every
        draw of the reference's stream (initial l_T, x_T; per step rand(N, A),
        randn(B, 3, 3), randn(N, 3) x2) is then made at the GLOBAL size on the
        CPU generator and this shard keeps its rows (chemeleon_amd.noise), so a
        sample-parallel run reproduces the single-process trajectory bit for bit
        and every rank's generator ends where the single-process one does. The per-step
        Philox noise is keyed by global node / graph index (node_base,
        graph_base), so a shard reproduces its crystals of a larger run exactly
        when it is also given that run's initial noise for them (init=, as
        sample_distributed does).

        lanes > 1 (graph mode): the crystals are split into that many contiguous
        groups of similar edge work, each stepped on its own stream inside the
        one captured graph. The groups' kernels then run concurrently, so one
        group's GEMM epilogues (store bursts, VALU) overlap the other's matrix
        work instead of every CU reaching its epilogue at the same moment.
        Results are bit-identical: Philox noise is keyed by global node / graph
        index and crystals never interact."""
        if isinstance(natoms, int):
            natoms = [natoms]
        natoms = [int(n) for n in natoms]
        if texts is not None and isinstance(texts, str):
            texts = [texts]
        if texts is not None and len(texts) != len(natoms):
            raise ValueError("natoms and texts must have the same number of elements.")
        if noise not in ("torch", "philox"):
            raise ValueError("noise must be 'torch' or 'philox'")
        knn = getattr(self.decoder, "edge_style", "fc") == "knn"
        if graph is None:  # knn edges are rebuilt from the coordinates with a host sync: eager only
            graph = not knn
        if graph and knn:
            raise ValueError("edge_style='knn' rebuilds its edges every decoder call and cannot run as a captured graph")
        dev = self.device
        if dev.type != "cuda":
            raise RuntimeError("Chemeleon (chemeleon_amd) samples on a HIP device only; call .to('cuda') first")
        B, N, A, T = len(natoms), sum(natoms), self.max_atoms, self.num_timesteps
        mask = self.mask_lattice_matrix
        if global_sizes is None:
            step_noise = StepNoise(N, B, A)
        else:
            if noise != "torch":
                raise ValueError("global_sizes shards the reference's CPU RNG stream: it needs noise='torch'")
            NG, BG = (int(v) for v in global_sizes)
            if not (0 <= node_base and node_base + N <= NG and 0 <= graph_base and graph_base + B <= BG):
                raise ValueError(f"shard nodes [{node_base}, {node_base + N}) / crystals [{graph_base}, "
                                 f"{graph_base + B}) outside the global batch ({NG} nodes, {BG} crystals)")
            step_noise = StepNoise(NG, BG, A, node_base, node_base + N, graph_base, graph_base + B)
        a = torch.zeros(N, dtype=torch.long, device=dev)  # chemeleon.py:347 (absorbing class 0)
        if init is not None:
            l0, x0 = init
        elif noise == "torch":
            l0 = torch.randn(step_noise.B, 3, 3)[step_noise.g0:step_noise.g1] * mask  # :348
            x0 = torch.randn(step_noise.N, 3)[step_noise.n0:step_noise.n1]  # :349
        else:
            g = torch.Generator().manual_seed(seed)
            l0 = torch.randn(B, 3, 3, generator=g) * mask
            x0 = torch.randn(N, 3, generator=g)
        lat = l0.float().to(dev).contiguous()
        x = (x0 % 1.0).float().to(dev).contiguous()  # :359
        cond, null = self._conditioning(texts, B, text_embeds, null_text_embeds)
        if not self.text_guide:
            cond_scale = 1.0  # one conditioning: the CFG mix degenerates to the plain prediction
        sched, _keep = self.schedule_tables(step_lr)
        batch = self.decoder.hip_batch(natoms, max_pairs=2)
        L = _lib.load()
        stream = _lib.stream_handle(dev)
        emit = (lambda *ts: tuple(t.clone() for t in ts)) if clone else (lambda *ts: ts)
        yield (T,) + emit(a, x, lat)
        if graph and noise == "torch":
            if lanes > 1:
                raise ValueError("lanes > 1 needs noise='philox'")
            yield from self._replay_torch_noise(batch, sched, a, x, lat, cond, null, cond_scale, step_noise, T, t_stop,
                                                emit)
            return
        if graph:
            from ..distributed import partition
            groups = partition(natoms, max(1, min(int(lanes), B)))
            d_t = torch.full((len(groups),), T, dtype=torch.int32, device=dev)
            noff = [0]
            for n in natoms:
                noff.append(noff[-1] + n)
            # per-lane workspaces are created before the capture (allocation is not capturable); each
            # lane runs concurrently with the others, so each gets its own (never the shared cache entry,
            # which two lanes of identical crystal lists would otherwise both receive)
            lane_batches = [batch] if len(groups) == 1 else [
                self.decoder.hip_batch(natoms[g0:g1], max_pairs=2, private=True) for g0, g1 in groups]
            hg = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream(device=dev)
            lane_streams = [torch.cuda.Stream(device=dev) for _ in groups[1:]]
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                with torch.cuda.graph(hg, stream=side):
                    for k, (g0, g1) in enumerate(groups):
                        st = side if k == 0 else lane_streams[k - 1]
                        if k > 0:
                            st.wait_stream(side)
                        n0 = noff[g0]
                        bk = lane_batches[k]
                        io = _lib.step_io(a, x, lat, cond, null, node0=n0, graph0=g0, nodes=noff[g1] - n0,
                                          graphs=g1 - g0)
                        with torch.cuda.stream(st):
                            _lib.check(L.chm_sample_step_dt(
                                bk.handle, sched, _lib.ptr(d_t, 4 * k), float(cond_scale), io, seed, node_base + n0,
                                graph_base + g0, _lib.stream_handle(dev)), "chm_sample_step_dt")
                    for st in lane_streams:
                        side.wait_stream(st)
            torch.cuda.current_stream(dev).wait_stream(side)
            d_t.fill_(T)
            for t in range(T, t_stop, -1):
                hg.replay()
                yield (t - 1,) + emit(a, x, lat)
            return
        for t in range(T, t_stop, -1):
            if noise == "torch" and t > 1:  # :400-404, 418, 435, 455
                nz = tuple(z.to(dev) for z in step_noise.draw())
            else:
                nz = (None, None, None, None)
            io = _lib.step_io(a, x, lat, cond, null, nz)
            _lib.check(L.chm_sample_step(batch.handle, sched, t, float(cond_scale), io, seed, node_base, graph_base,
                                         stream), "chm_sample_step")
            yield (t - 1,) + emit(a, x, lat)

    def _replay_torch_noise(self, batch, sched, a, x, lat, cond, null, cond_scale, step_noise, T, t_stop, emit):
        """Parity-mode noise (the reference's CPU RNG stream, this shard's rows of it) under a captured
        reverse step, with no copy on the device's critical path.

        Two pinned host noise sets and two captured graphs of the same step: graph k reads set k in place
        (pinned host memory is mapped into the device's address space; the step kernels read each value
        once, coalesced), and the graphs alternate over the timesteps. The host draws step t's noise into
        set t & 1 while step t+1 replays, after waiting for the replay that last read that set (two steps
        earlier), so the compute stream never waits for a copy and the draw hides under the replays.
        Bit-identical to eager stepping (test_torch_noise_graph_matches_eager): the same draws reach the
        same kernels."""
        dev = self.device
        L = _lib.load()
        d_t = torch.full((1,), T, dtype=torch.int32, device=dev)
        shapes = step_noise.local_shapes
        pin = [[torch.zeros(sh, dtype=torch.float32).pin_memory() for sh in shapes] for _ in range(2)]
        graphs = [torch.cuda.CUDAGraph() for _ in range(2)]
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for k in range(2):
                with torch.cuda.graph(graphs[k], stream=side):
                    _lib.check(L.chm_sample_step_dt_noise(
                        batch.handle, sched, _lib.ptr(d_t), float(cond_scale),
                        _lib.step_io(a, x, lat, cond, null, pin[k]), _lib.stream_handle(dev)),
                        "chm_sample_step_dt_noise")
        cur = torch.cuda.current_stream(dev)
        cur.wait_stream(side)
        replayed = [None, None]  # the replay that read set k done: the host may draw into it again
        d_t.fill_(T)
        for t in range(T, t_stop, -1):
            k = t & 1
            if t > 1:  # chemeleon.py:400-404, 418, 435, 455 (none at t = 1)
                if replayed[k] is not None:
                    replayed[k].synchronize()
                step_noise.draw(out=pin[k])
            graphs[k].replay()
            replayed[k] = torch.cuda.Event()
            replayed[k].record(cur)
            yield (t - 1,) + emit(a, x, lat)

    @torch.no_grad()
    def reverse_step(self, t: int, atom_types, frac_coords, lattices, natoms: List[int], cond_scale: float = 2.0,
                     step_lr: float = 1e-5, text_embeds=None, null_text_embeds=None, noise=None, seed: int = 0,
                     node_base: int = 0, graph_base: int = 0):
        """One step t -> t-1 (chemeleon.py:379-466) from an explicit state.
        `noise` = (rand_a, rand_l, rand_x1, rand_x2) tensors or None (Philox).
        Returns new (atom_types, frac_coords, lattices) device tensors."""
        dev = self.device
        natoms = [int(n) for n in natoms]
        a = atom_types.to(dev).long().clone().contiguous()
        x = frac_coords.to(dev).float().clone().contiguous()
        lat = lattices.to(dev).float().clone().contiguous()
        cond, null = self._conditioning(None, len(natoms), text_embeds, null_text_embeds)
        if not self.text_guide:
            cond_scale = 1.0
        sched, _keep = self.schedule_tables(step_lr)
        batch = self.decoder.hip_batch(natoms, max_pairs=2)
        nz = [None] * 4 if noise is None else [z.to(dev).float().contiguous() for z in noise]
        N, B, A = sum(natoms), len(natoms), self.decoder.max_atoms
        if a.shape != (N,) or x.shape != (N, 3) or lat.shape != (B, 3, 3):
            raise ValueError("state shapes do not match natoms")
        if noise is not None and [tuple(z.shape) for z in nz] != [(N, A), (B, 3, 3), (N, 3), (N, 3)]:
            raise ValueError(f"noise must be (rand_a [N,{A}], rand_l [B,3,3], rand_x1 [N,3], rand_x2 [N,3])")
        _lib.require_device(a, x, lat, cond, null, *nz)
        _lib.check(_lib.load().chm_sample_step(batch.handle, sched, int(t), float(cond_scale),
                                               _lib.step_io(a, x, lat, cond, null, nz), seed, node_base, graph_base,
                                               _lib.stream_handle(dev)),
                   "chm_sample_step")
        return a, x, lat

    @staticmethod
    def _distributed(distributed: Optional[bool], group) -> bool:
        """Whether sample() / _sample_generator() shard over the ranks of `group`: `distributed` if
        given, else whenever torch.distributed is initialised with more than one rank."""
        if distributed is not None:
            return bool(distributed)
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1

    @torch.no_grad()
    def _sample_generator(self, natoms: Union[int, List[int]], texts: Optional[Union[str, List[str]]] = None,
                          cond_scale: float = 2.0, step_lr: float = 1e-5, *, distributed: Optional[bool] = None,
                          group=None, **kw):
        """chemeleon.py:305-467: yields, for every step t -> t-1, the list of
        structures at t-1 (TrajectoryContainer.get_atoms, schema.py:57-83).
        Under torch.distributed (see sample) the crystals are sharded over
        the ranks and every step's whole batch is all-gathered to every rank."""
        if isinstance(natoms, int):
            natoms = [natoms]
        if texts is not None and isinstance(texts, str):
            texts = [texts]
        if self._distributed(distributed, group):
            from chemeleon_amd.distributed import sample_states_distributed
            it = sample_states_distributed(self, natoms, texts, cond_scale, step_lr, group=group, every_step=True,
                                           **kw)
        else:
            it = self.sample_states(natoms, texts, cond_scale, step_lr, clone=False, **kw)
        next(it)
        for t, a, x, lat in it:
            yield step_to_atoms(a, x, lat, natoms)

    def sample(self, text_input: str, n_atoms: int, n_samples: int, cond_scale: float = 2.0, step_lr: float = 1e-5,
               return_trajectory: bool = False, stream: bool = False, *, distributed: Optional[bool] = None,
               group=None, **kw):
        """chemeleon.py:469-490. Without return_trajectory / stream, only the
        final state is copied to the host (the reference converts every step).
        Keyword arguments go to sample_states: noise="philox" (device noise)
        or the default noise="torch" (the reference's CPU RNG stream); either
        way one captured HIP graph is replayed per timestep (fc edges).

        Multi-GPU: with torch.distributed initialised over more than one rank
        (one process per GPU; or distributed=True / group=...), every rank
        calls sample() with the same arguments and the same seeded generator;
        the crystals are split over the ranks (chemeleon_amd.distributed), the
        text conditioning is computed on rank 0 and broadcast, and every rank
        returns the whole batch. In the default noise="torch" mode the result
        is bit-identical to the single-process call. Only the final state is
        exchanged, unless stream / return_trajectory ask for every step.
        distributed=False keeps each rank's call local."""
        natoms = [n_atoms] * n_samples
        texts = [text_input] * n_samples if text_input is not None else None
        kw.update(distributed=distributed, group=group)
        if stream:
            return self._sample_generator(natoms, texts, cond_scale, step_lr, **kw)
        if return_trajectory:
            return list(self._sample_generator(natoms, texts, cond_scale, step_lr, **kw))
        kw.pop("distributed"), kw.pop("group")
        if self._distributed(distributed, group):
            from chemeleon_amd.distributed import sample_states_distributed
            it = sample_states_distributed(self, natoms, texts, cond_scale, step_lr, group=group, **kw)
        else:
            it = self.sample_states(natoms, texts, cond_scale, step_lr, clone=False, **kw)
        last = None
        for last in it:
            pass
        _, a, x, lat = last
        return step_to_atoms(a, x, lat, natoms)

    def trajectory_container(self, natoms, texts=None, cond_scale=2.0, step_lr=1e-5, **kw) -> TrajectoryContainer:
        """All states t = T..0 as the reference's TrajectoryContainer."""
        if isinstance(natoms, int):
            natoms = [natoms]
        tc = TrajectoryContainer(total_steps=self.num_timesteps)
        nat = torch.tensor(natoms)
        bidx = torch.arange(len(natoms)).repeat_interleave(nat)
        for t, a, x, lat in self.sample_states(natoms, texts, cond_scale, step_lr, clone=True, **kw):
            tc[t] = TrajectoryStep(num_atoms=nat, atom_types=a.cpu(), frac_coords=x.cpu(), lattices=lat.cpu(),
                                   batch_idx=bidx)
        return tc
