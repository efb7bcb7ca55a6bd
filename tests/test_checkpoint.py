"""Checkpoint layout and loader (reference chemeleon.py:97-135,
base_module.py:14). CPU only: no compute call is made.

The reference's state_dict names and shapes (tests/golden/state_keys.json) were captured from
the reference itself by tests/golden/make_golden.py ("keys"); a released checkpoint carries
them under "state_dict" next to "hyper_parameters". No released checkpoint is reachable
offline, so the loader is exercised on a Lightning-format file written here with that layout.
"""

import json
import os

import pytest
import torch

from chemeleon_amd import Chemeleon
from chemeleon_amd.config import default_config
from chemeleon_amd.synthetic import synthetic_state_dict

HERE = os.path.dirname(os.path.abspath(__file__))


def _model():
    cfg = default_config()
    torch.manual_seed(0)
    m = Chemeleon(cfg)
    m.decoder.load_state_dict(synthetic_state_dict(cfg))
    return m, cfg


def test_state_dict_matches_reference_layout():
    ref = json.load(open(os.path.join(HERE, "golden", "state_keys.json")))
    m, _ = _model()
    own = {k: list(v.shape) for k, v in m.state_dict().items()}
    assert sorted(own) == sorted(ref), (sorted(set(own) ^ set(ref)))[:10]
    for k, shape in ref.items():
        assert own[k] == shape, k


def test_lightning_checkpoint_round_trip(tmp_path):
    m, cfg = _model()
    sd = dict(m.state_dict())
    sd["text_encoder.text_proj.weight"] = torch.zeros(512, 768)  # text-encoder keys are routed aside
    path = tmp_path / "chemeleon-test.ckpt"
    torch.save({"state_dict": sd, "hyper_parameters": dict(cfg), "epoch": 1}, path)
    m2 = Chemeleon.load_from_checkpoint(str(path))
    s2 = m2.state_dict()
    for k, v in m.state_dict().items():
        assert torch.equal(v, s2[k]), k
    assert m2.num_timesteps == m.num_timesteps


def test_checkpoint_key_mismatch_raises(tmp_path):
    m, cfg = _model()
    sd = {k: v for k, v in m.state_dict().items() if not k.startswith("decoder.csp_layer_5.")}
    path = tmp_path / "broken.ckpt"
    torch.save({"state_dict": sd, "hyper_parameters": dict(cfg)}, path)
    with pytest.raises(RuntimeError, match="checkpoint mismatch"):
        Chemeleon.load_from_checkpoint(str(path))


def test_released_checkpoint_missing_is_explicit():
    import chemeleon_amd.modules.chemeleon as mod
    if os.path.exists(mod.PATH_CHEMELEON_GENERAL_TEXT):
        pytest.skip("a released checkpoint is present")
    with pytest.raises(FileNotFoundError, match="figshare"):
        Chemeleon.load_general_text_model()


def _tiny_text_encoder():
    pytest.importorskip("transformers")
    from chemeleon_amd.text_encoder import TextEncoder
    bert = os.path.join(HERE, "golden", "tiny_bert")
    torch.manual_seed(3)
    return TextEncoder(text_encoder_name=bert, text_embed_dim=32, max_text_len=12, text_dim=24, local_path=bert)


def test_checkpoint_text_encoder_weights_load_strictly(tmp_path):
    """The trained conditioning head (text_emb.*, null_text_embeds) must come from the checkpoint;
    only the frozen language model is sourced locally. A file without them is refused rather
    than sampling with randomly initialised conditioning."""
    m, cfg = _model()
    te_src = _tiny_text_encoder()
    with torch.no_grad():
        for p in te_src.text_emb.parameters():
            p.add_(1.0)
        te_src.null_text_embeds.fill_(0.25)
    sd = dict(m.state_dict())
    for k, v in te_src.state_dict().items():
        sd["text_encoder." + k] = v
    path = tmp_path / "with-text.ckpt"
    torch.save({"state_dict": sd, "hyper_parameters": dict(cfg)}, path)
    m2 = Chemeleon.load_from_checkpoint(str(path), text_encoder=_tiny_text_encoder())
    for k, v in te_src.state_dict().items():
        if not k.startswith("text_encoder."):
            assert torch.equal(m2.text_encoder.state_dict()[k], v), k
    sd_bad = {k: v for k, v in sd.items() if not k.startswith("text_encoder.text_emb.")}
    path2 = tmp_path / "without-head.ckpt"
    torch.save({"state_dict": sd_bad, "hyper_parameters": dict(cfg)}, path2)
    with pytest.raises(RuntimeError, match="text-encoder mismatch"):
        Chemeleon.load_from_checkpoint(str(path2), text_encoder=_tiny_text_encoder())
    m3 = Chemeleon.load_from_checkpoint(str(path2), text_encoder=_tiny_text_encoder(), strict=False)
    assert m3.text_encoder is not None

