"""`CrystalClip` (text side) — the part of the reference's contrastive model
that conditioning uses (reference `chemeleon/text_encoder/crystal_clip.py:15-96`):
a BERT text encoder + tokenizer and the `text_proj` head (Linear, LayerNorm,
GELU, Linear to `clip_dim`), with `get_text_embeds(text)` returning the
projected [CLS] embedding.

`load_from_checkpoint(path, text_model_dir)` reads a Lightning checkpoint with
`torch.load(weights_only=True)`: `hyper_parameters` give `text_embed_dim`,
`clip_dim`, `max_text_len`; the BERT architecture and vocabulary come from the
local directory (the reference fetches them from the hub by name); the
`text_encoder.*` and `text_proj.*` tensors come from the checkpoint. The graph
side (`graph_encoder.*`, a time- and text-free CSPNet, and `graph_proj.*`) is
training / retrieval only and is not rebuilt; its keys are reported in
`ignored_keys`.
"""

from typing import Dict, List, Optional

import torch
import torch.nn as nn

from chemeleon_amd.text_encoder import resolve_local


class CrystalClip(nn.Module):
    def __init__(self, _config: Dict, text_model_dir: Optional[str] = None):
        super().__init__()
        import transformers as tf
        self.hparams = dict(_config)
        self.clip_dim = _config["clip_dim"]
        self.text_encoder_name = _config["text_encoder"]
        self.max_text_len = _config["max_text_len"]
        self.text_embed_dim = _config["text_embed_dim"]
        d = resolve_local(self.text_encoder_name, text_model_dir)
        self.tokenizer = tf.BertTokenizer.from_pretrained(d, local_files_only=True)
        self.text_encoder = tf.BertModel.from_pretrained(d, local_files_only=True)
        e = self.text_embed_dim
        self.text_proj = nn.Sequential(nn.Linear(e, e), nn.LayerNorm(e), nn.GELU(), nn.Linear(e, self.clip_dim))
        self.ignored_keys: List[str] = []

    @property
    def device(self):
        return next(self.text_proj.parameters()).device

    def get_text_embeds(self, text: List[str]) -> torch.Tensor:
        enc = self.tokenizer(list(text), padding="longest", max_length=self.max_text_len, truncation=True,
                             return_tensors="pt")
        out = self.text_encoder(enc["input_ids"].to(self.device), attention_mask=enc["attention_mask"].to(self.device))
        return self.text_proj(out.last_hidden_state[:, 0, :])

    @classmethod
    def load_from_checkpoint(cls, path: str, text_model_dir: Optional[str] = None, map_location="cpu"):
        ck = torch.load(path, map_location=map_location, weights_only=True)
        m = cls(dict(ck.get("hyper_parameters", {})), text_model_dir=text_model_dir)
        sd = ck["state_dict"]
        keep = {k: v for k, v in sd.items() if k.startswith("text_encoder.") or k.startswith("text_proj.")}
        m.ignored_keys = sorted(k for k in sd if k not in keep)
        missing, unexpected = m.load_state_dict(keep, strict=False)
        missing = [k for k in missing if not k.endswith("position_ids")]
        if missing or unexpected:
            raise RuntimeError(f"CrystalClip checkpoint mismatch: missing {missing}, unexpected {unexpected}")
        return m
