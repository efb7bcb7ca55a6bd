"""Conditioning front-end: the text encoder that turns
prompts into the [B, text_dim] vectors the sampler consumes once per call.

Mirrors `chemeleon/text_encoder/__init__.py`, `text_encoder.py` and the text
side of `crystal_clip.py`. It runs in host-side PyTorch (on whatever device the
caller names); the hot path starts at its output. This image has no network, so
every language model is loaded from a LOCAL directory (`from_pretrained(dir,
local_files_only=True)`), never from the hub or wandb: pass `local_path=`, or
set `CHEMELEON_TEXT_MODEL_DIR` to a directory holding one sub-directory per
model name with "/" replaced by "__" (e.g. `lfoppiano__MatTPUSciBERT`).
"""

import os

# reference chemeleon/text_encoder/__init__.py:1-12 (same names, same order)
MODEL_NAMES = [
    "pranav-s/MaterialsBERT",
    "m3rg-iitd/matscibert",
    "lfoppiano/MatTPUSciBERT",
    "t5-3b",
    "meta-llama/Meta-Llama-3-8B-Instruct",
    "microsoft/Phi-3-mini-4k-instruct",
    "microsoft/phi-2",
    "chemeleon/clip-mp-composition",
    "chemeleon/clip-mp-composition_crystalsystem",
    "chemeleon/clip-mp-prompt",
]


def resolve_local(name: str, local_path=None) -> str:
    """Local directory for a model name: `local_path`, `name` itself if it is a
    directory, or $CHEMELEON_TEXT_MODEL_DIR/<name with / -> __>."""
    if local_path:
        if not os.path.isdir(local_path):
            raise FileNotFoundError(f"text model directory {local_path} not found")
        return local_path
    if os.path.isdir(name):
        return name
    root = os.environ.get("CHEMELEON_TEXT_MODEL_DIR")
    if root:
        d = os.path.join(root, name.replace("/", "__"))
        if os.path.isdir(d):
            return d
    raise FileNotFoundError(
        f"no local copy of text model '{name}': the reference downloads it from the Hugging Face hub; "
        "this build does not download. Pass local_path= or set CHEMELEON_TEXT_MODEL_DIR.")


from chemeleon_amd.text_encoder.crystal_clip import CrystalClip  # noqa: E402,F401
from chemeleon_amd.text_encoder.text_encoder import TextEncoder, prob_mask_like  # noqa: E402,F401

__all__ = ["MODEL_NAMES", "TextEncoder", "CrystalClip", "prob_mask_like", "resolve_local"]
