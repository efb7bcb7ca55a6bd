"""Seeded synthetic weights and conditioning vectors.

The released checkpoints (figshare URLs in `chemeleon/constants.py:9-14` of
the reference) are not reachable offline, so every parity fixture and every
benchmark uses this recipe instead. It is deterministic on any host:

* each parameter gets its own `torch.Generator` seeded with
  `crc32(key) ^ seed`, so a tensor does not depend on which other
  parameters exist or on their order;
* Linear weights are `randn * gain / sqrt(fan_in)`, biases `0.02 * randn`,
  LayerNorm weights `1 + 0.05 * randn`, LayerNorm biases `0.05 * randn`,
  the atom embedding `randn` (the `nn.Embedding` default);
* the lattice head gets a small gain so that an untrained reverse process
  keeps lattices finite over 1000 steps.

The recipe is generated on the CPU and copied to the device, so the weights
are bit-identical wherever they are used.
"""

import zlib
from collections import OrderedDict
from typing import Dict, Tuple

import torch


def cspnet_param_shapes(cfg: Dict) -> "OrderedDict[str, Tuple[int, ...]]":
    """Parameter names and shapes of the reference `CSPNet` state_dict
    (`chemeleon/modules/cspnet.py:184-234`) for `smooth=False`, `ln=True`."""
    H = cfg["hidden_dim"]
    A = cfg["max_atoms"]
    T = cfg["time_dim"]
    X = cfg["text_dim"]
    F = cfg["num_freqs"] * 2 * 3
    s = OrderedDict()
    if cfg.get("smooth", False):
        s["node_embedding.weight"] = (H, A)
        s["node_embedding.bias"] = (H,)
    else:
        s["node_embedding.weight"] = (A, H)
    if T > 0 or X > 0:
        s["film_layer.mlp_cond.0.weight"] = (2 * H, T + X)
        s["film_layer.mlp_cond.0.bias"] = (2 * H,)
        s["film_layer.proj.weight"] = (H, H)
        s["film_layer.proj.bias"] = (H,)
        s["film_layer.norm.weight"] = (H,)
        s["film_layer.norm.bias"] = (H,)
    for i in range(cfg["num_layers"]):
        p = f"csp_layer_{i}."
        s[p + "edge_mlp.0.weight"] = (H, 2 * H + 9 + F)
        s[p + "edge_mlp.0.bias"] = (H,)
        s[p + "edge_mlp.2.weight"] = (H, H)
        s[p + "edge_mlp.2.bias"] = (H,)
        s[p + "node_mlp.0.weight"] = (H, 2 * H)
        s[p + "node_mlp.0.bias"] = (H,)
        s[p + "node_mlp.2.weight"] = (H, H)
        s[p + "node_mlp.2.bias"] = (H,)
        if cfg.get("ln", True):
            s[p + "layer_norm.weight"] = (H,)
            s[p + "layer_norm.bias"] = (H,)
    s["coord_out.weight"] = (3, H)
    s["lattice_out.weight"] = (9, H)
    s["type_out.weight"] = (A, H)
    s["type_out.bias"] = (A,)
    if cfg.get("ln", True):
        s["final_layer_norm.weight"] = (H,)
        s["final_layer_norm.bias"] = (H,)
    return s


def _gen(key: str, seed: int) -> torch.Generator:
    return torch.Generator().manual_seed((zlib.crc32(key.encode()) ^ seed) & 0x7FFFFFFF)


LATTICE_GAIN = 0.05


def synthetic_tensor(key: str, shape, seed: int = 0) -> torch.Tensor:
    g = _gen(key, seed)
    x = torch.randn(shape, generator=g, dtype=torch.float32)
    leaf = key.rsplit(".", 1)[-1]
    is_norm = "norm" in key
    if key == "node_embedding.weight" and len(shape) == 2 and shape[0] != shape[1] and "smooth" not in key:
        return x
    if is_norm:
        return 1.0 + 0.05 * x if leaf == "weight" else 0.05 * x
    if leaf == "bias":
        return 0.02 * x
    gain = LATTICE_GAIN if key.startswith("lattice_out") else 1.0
    return x * (gain / float(shape[-1]) ** 0.5)


def synthetic_state_dict(cfg: Dict, seed: int = 0) -> "OrderedDict[str, torch.Tensor]":
    return OrderedDict(
        (k, synthetic_tensor(k, shape, seed)) for k, shape in cspnet_param_shapes(cfg).items()
    )


def synthetic_clip_graph_state_dict(cfg: Dict, clip_dim: int, seed: int = 0) -> "OrderedDict[str, torch.Tensor]":
    """Graph side of the reference CrystalClip (crystal_clip.py:34-73): `graph_encoder.*` (a CSPNet
    with time_dim = text_dim = 0, same recipe per key) and `graph_proj.{0,1,3}.*` (Linear, LayerNorm,
    GELU, Linear to clip_dim)."""
    c = dict(cfg)
    c["time_dim"] = 0
    c["text_dim"] = 0
    sd = OrderedDict(("graph_encoder." + k, synthetic_tensor(k, shape, seed)) for k, shape in cspnet_param_shapes(c).items())
    H = cfg["hidden_dim"]
    for k, shape in (("graph_proj.0.weight", (H, H)), ("graph_proj.0.bias", (H,)), ("graph_proj.1.weight", (H,)),
                     ("graph_proj.1.bias", (H,)), ("graph_proj.3.weight", (clip_dim, H)), ("graph_proj.3.bias", (clip_dim,))):
        kk = k.replace("graph_proj.1", "graph_proj.norm")  # (LayerNorm recipe for index 1)
        sd[k] = synthetic_tensor(kk, shape, seed)
    return sd


def weights_crc(sd) -> int:
    """CRC32 over the tensors of a state dict in key order; stored in every
    fixture so a changed recipe is detected instead of silently compared."""
    c = 0
    for k in sorted(sd):
        c = zlib.crc32(sd[k].detach().cpu().contiguous().numpy().tobytes(), c)
    return c


def synthetic_text_embeds(text_dim: int = 512):
    """Stand-ins for `TextEncoder.get_text_embeds` outputs
    (`chemeleon/text_encoder/text_encoder.py:186-205`): cond with
    `cond_drop_prob=0`, null with `cond_drop_prob=1`, each [1, text_dim]."""
    cond = torch.randn(1, text_dim, generator=torch.Generator().manual_seed(1))
    null = torch.randn(1, text_dim, generator=torch.Generator().manual_seed(2))
    return cond, null
