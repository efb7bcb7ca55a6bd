"""Model hyper-parameters for the sampling path.

Defaults follow the reference's Sacred defaults that shape the hot path
(`chemeleon/config.py:28-60` in ryannduma/chemeleon): hidden 512, time 128,
text 512, 104 atom classes (103 elements + dummy), 6 layers, 128 Fourier
frequencies, fully connected edges, LayerNorm on, lattice inner products on,
cosine beta schedule, 1000 timesteps.

A released checkpoint stores these in `hyper_parameters`
(`chemeleon/modules/chemeleon.py:34`); `default_config()` returns the same
keys so a dict loaded from a checkpoint can be passed straight to
`Chemeleon(_config)`.
"""

from typing import Any, Dict


def default_config() -> Dict[str, Any]:
    return {
        # decoder (config.py:28-43)
        "hidden_dim": 512,
        "time_dim": 128,
        "text_dim": 512,
        "max_atoms": 103 + 1,
        "num_layers": 6,
        "act_fn": "silu",
        "dis_emb": "sin",
        "num_freqs": 128,
        "edge_style": "fc",
        "max_neighbors": 20,
        "cutoff": 6.0,
        "ln": True,
        "ip": True,
        "smooth": False,
        "pred_atom_types": True,
        # diffusion (config.py:45-60)
        "text_guide": True,
        "text_encoder": "lfoppiano/MatTPUSciBERT",
        "text_embed_dim": 768,
        "max_text_len": 256,
        "trainable_text_encoder": False,
        "cond_drop_prob": 0.2,
        "beta_schedule": "cosine",
        "timesteps": 1000,
        "d3pm_hybrid_coeff": 1.0,
        "cost_atom_types": 1.0,
        "cost_lattice": 1.0,
        "cost_coords": 1.0,
        "cond_scale": 2.0,
        # training-only keys kept so checkpoint dicts round-trip
        "optimizer": "adam",
        "lr": 1e-3,
        "weight_decay": 0,
        "scheduler": "reduce_on_plateau",
        "patience": 200,
    }
