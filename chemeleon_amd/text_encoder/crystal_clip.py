"""`CrystalClip` — the reference's contrastive text / crystal model
(`chemeleon/text_encoder/crystal_clip.py:15-112`), inference side:

* text: a BERT text encoder + tokenizer and the `text_proj` head (Linear, LayerNorm, GELU, Linear
  to `clip_dim`); `get_text_embeds(text)` returns the projected [CLS] embedding (host PyTorch, once
  per call, as the conditioning front-end);
* graph: `graph_encoder`, a CSPNet without FilmLayer (time_dim = text_dim = 0, crystal_clip.py:34-52)
  running on the HIP decoder (libchemeleon_hip, fc or knn edges), mean / sum pooling of its node
  features per crystal and the `graph_proj` head; `get_graph_embeds(batch)` (crystal_clip.py:98-112).

`load_from_checkpoint(path, text_model_dir)` reads a Lightning checkpoint with
`torch.load(weights_only=True)`: `hyper_parameters` give the dimensions; the BERT architecture and
vocabulary come from the local directory (the reference fetches them from the hub by name); every
other tensor (`text_encoder.*`, `text_proj.*`, `graph_encoder.*`, `graph_proj.*`) comes from the
checkpoint. `text=False` builds the graph side only (no language model needed).
"""

from typing import Dict, List, Optional

import torch
import torch.nn as nn

from chemeleon_amd.text_encoder import resolve_local


GRAPH_KEYS = ("hidden_dim", "num_layers", "max_atoms", "act_fn", "dis_emb", "num_freqs", "edge_style", "cutoff",
              "max_neighbors", "ln", "ip", "smooth", "pred_atom_types")


class CrystalClip(nn.Module):
    def __init__(self, _config: Dict, text_model_dir: Optional[str] = None, text: bool = True, graph: bool = True):
        super().__init__()
        self.hparams = dict(_config)
        self.clip_dim = _config["clip_dim"]
        self.text_encoder_name = _config.get("text_encoder")
        self.max_text_len = _config.get("max_text_len")
        self.text_embed_dim = _config.get("text_embed_dim")
        if text:
            import transformers as tf
            d = resolve_local(self.text_encoder_name, text_model_dir)
            self.tokenizer = tf.BertTokenizer.from_pretrained(d, local_files_only=True)
            self.text_encoder = tf.BertModel.from_pretrained(d, local_files_only=True)
            e = self.text_embed_dim
            self.text_proj = nn.Sequential(nn.Linear(e, e), nn.LayerNorm(e), nn.GELU(), nn.Linear(e, self.clip_dim))
        # graph keys the config lacks (then no graph side is built; a checkpoint that carries one fails
        # loudly in load_from_checkpoint, and get_graph_embeds says why)
        self.missing_graph_keys = [k for k in GRAPH_KEYS + ("graph_pooling",) if k not in _config] if graph else []
        if graph and not self.missing_graph_keys:
            from chemeleon_amd.modules.cspnet import CSPNet
            # graph encoder: a time- and text-free CSPNet (crystal_clip.py:34-52)
            self.graph_encoder = CSPNet(time_dim=0, text_dim=0, **{k: _config[k] for k in GRAPH_KEYS})
            self.graph_pooling = _config["graph_pooling"]  # (required, as crystal_clip.py:53-58)
            if self.graph_pooling not in ("mean", "sum"):
                raise ValueError(f"graph_pooling must be 'mean' or 'sum', got {self.graph_pooling!r}")
            g = _config["hidden_dim"]
            self.graph_embed_dim = g
            self.graph_proj = nn.Sequential(nn.Linear(g, g), nn.LayerNorm(g), nn.GELU(), nn.Linear(g, self.clip_dim))
        self.ignored_keys: List[str] = []

    @property
    def device(self):
        return next(self.parameters()).device

    def get_graph_embeds(self, batch) -> torch.Tensor:
        """crystal_clip.py:98-112: node features of the film-less CSPNet (HIP decoder), pooled per
        crystal (scatter_mean / scatter_sum over `batch.batch`), projected. `batch` needs
        atom_types [N], frac_coords [N,3], lattices [B,3,3], natoms [B] and batch [N] (what
        Batch.from_data_list builds)."""
        if not hasattr(self, "graph_encoder"):
            raise RuntimeError("this CrystalClip has no graph encoder: its config lacks "
                               f"{self.missing_graph_keys or 'nothing (built with graph=False)'}")
        out = self.graph_encoder(t=None, atom_types=batch.atom_types, frac_coords=batch.frac_coords,
                                 lattices=batch.lattices, num_atoms=batch.natoms, node2graph=batch.batch)
        h = out.node_features
        B = len(batch.natoms)
        pooled = torch.zeros(B, h.shape[1], dtype=h.dtype, device=h.device).index_add_(0, batch.batch, h)
        if self.graph_pooling == "mean":  # scatter_mean: sum / max(count, 1) (chemeleon/utils/scatter.py:88-112)
            cnt = torch.zeros(B, dtype=h.dtype, device=h.device).index_add_(
                0, batch.batch, torch.ones_like(batch.batch, dtype=h.dtype))
            pooled = pooled / cnt.clamp(min=1).view(-1, 1)
        return self.graph_proj(pooled)

    def get_text_embeds(self, text: List[str]) -> torch.Tensor:
        enc = self.tokenizer(list(text), padding="longest", max_length=self.max_text_len, truncation=True,
                             return_tensors="pt")
        out = self.text_encoder(enc["input_ids"].to(self.device), attention_mask=enc["attention_mask"].to(self.device))
        return self.text_proj(out.last_hidden_state[:, 0, :])

    @classmethod
    def load_from_checkpoint(cls, path: str, text_model_dir: Optional[str] = None, map_location="cpu",
                             graph: bool = True):
        """graph=False: the text side only (the sampler's conditioning front-end); the checkpoint's
        graph_encoder.* / graph_proj.* tensors are then listed in `ignored_keys`. graph=True: a
        checkpoint with a graph side must carry the hyper_parameters to build it."""
        ck = torch.load(path, map_location=map_location, weights_only=True)
        m = cls(dict(ck.get("hyper_parameters", {})), text_model_dir=text_model_dir, graph=graph)
        sd = ck["state_dict"]
        if graph and m.missing_graph_keys and any(k.startswith(("graph_encoder.", "graph_proj.")) for k in sd):
            raise RuntimeError("the checkpoint carries a graph encoder (graph_encoder.* / graph_proj.*) but its "
                               f"hyper_parameters lack {m.missing_graph_keys}: cannot build it")
        own = set(m.state_dict())
        keep = {k: v for k, v in sd.items() if k in own}
        m.ignored_keys = sorted(k for k in sd if k not in keep)
        missing, unexpected = m.load_state_dict(keep, strict=False)
        missing = [k for k in missing if not k.endswith("position_ids")]
        if missing or unexpected:
            raise RuntimeError(f"CrystalClip checkpoint mismatch: missing {missing}, unexpected {unexpected}")
        return m
