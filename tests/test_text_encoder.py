"""Conditioning front-end against the reference's own
TextEncoder, run by tests/golden/make_golden.py ("text") on a tiny seeded BERT
saved in tests/golden/tiny_bert (36-word vocabulary, 2 layers, width 32; no
pretrained weights exist offline). CPU only: the encoder runs once per sample()
call on the host side of the boundary."""

import os

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
BERT_DIR = os.path.join(HERE, "golden", "tiny_bert")
FIX = os.path.join(HERE, "golden", "text_encoder.npz")

transformers = pytest.importorskip("transformers")


@pytest.fixture(scope="module")
def gold():
    return np.load(FIX, allow_pickle=False)


def _load_prefixed(module, g, prefix):
    sd = {k[len(prefix):]: torch.from_numpy(np.array(g[k])) for k in g.files if k.startswith(prefix)}
    module.load_state_dict(sd, strict=True)


def _clip(g):
    from chemeleon_amd.text_encoder import CrystalClip
    clip = CrystalClip({"clip_dim": 32, "text_encoder": BERT_DIR, "max_text_len": 12, "text_embed_dim": 32},
                       text_model_dir=BERT_DIR)
    _load_prefixed(clip.text_proj, g, "p:")
    return clip.eval()


def _encoder(g, clip=None):
    from chemeleon_amd.text_encoder import TextEncoder
    te = TextEncoder(text_encoder_name=BERT_DIR, text_embed_dim=32, max_text_len=12, text_dim=24,
                     pretrained_clip_model=clip, local_path=None if clip is not None else BERT_DIR)
    sd = {k[2:]: torch.from_numpy(np.array(g[k])) for k in g.files if k.startswith("w:")}
    missing, unexpected = te.load_state_dict(sd, strict=False)
    assert not unexpected and all(k.startswith(("text_encoder.", "clip_model.")) for k in missing)
    return te


def test_bert_branch_matches_reference(gold):
    te = _encoder(gold)
    texts = [str(t) for t in gold["texts"]]
    with torch.no_grad():
        enc = te.text_encode(texts, "cpu")
        cond = te.get_text_embeds(texts, 0.0, "cpu")
    np.testing.assert_allclose(enc.numpy(), gold["bert_encode"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(cond.numpy(), gold["bert_cond"], rtol=0, atol=1e-6)


def test_clip_branch_and_cfg_dropout_match_reference(gold):
    te = _encoder(gold, clip=_clip(gold))
    texts = [str(t) for t in gold["texts"]]
    with torch.no_grad():
        np.testing.assert_allclose(te.text_encode(texts, "cpu").numpy(), gold["clip_encode"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(te.get_text_embeds(texts, 0.0, "cpu").numpy(), gold["clip_cond"], rtol=0, atol=1e-6)
        null = te.get_text_embeds(texts, 1.0, "cpu").numpy()
        np.testing.assert_allclose(null, gold["clip_null"], rtol=0, atol=1e-6)
        assert np.allclose(null, null[:1])  # every row is the projected null embedding
        torch.manual_seed(5)  # prob_mask_like draws uniform_ from the global generator, as the reference
        np.testing.assert_allclose(te.get_text_embeds(texts, 0.5, "cpu").numpy(), gold["clip_drop05"], rtol=0,
                                   atol=1e-6)


def test_truncation_to_max_text_len(gold):
    te = _encoder(gold)
    long = " ".join(["crystal"] * 40)
    enc = te.tokenizer([long], padding="longest", max_length=te.max_text_len, truncation=True, return_tensors="pt")
    assert enc["input_ids"].shape[1] == 12


def test_crystal_clip_checkpoint_roundtrip(gold, tmp_path):
    from chemeleon_amd.text_encoder import CrystalClip
    clip = _clip(gold)
    sd = {f"text_encoder.{k}": v for k, v in clip.text_encoder.state_dict().items()}
    sd.update({f"text_proj.{k}": v for k, v in clip.text_proj.state_dict().items()})
    sd["graph_proj.0.weight"] = torch.zeros(2, 2)  # graph side: training / retrieval only
    hp = {"clip_dim": 32, "text_encoder": BERT_DIR, "max_text_len": 12, "text_embed_dim": 32}
    path = tmp_path / "clip.ckpt"
    torch.save({"hyper_parameters": hp, "state_dict": sd}, path)
    c2 = CrystalClip.load_from_checkpoint(str(path), text_model_dir=BERT_DIR, graph=False)  # (text side only)
    assert c2.ignored_keys == ["graph_proj.0.weight"]
    texts = [str(t) for t in gold["texts"]]
    with torch.no_grad():
        np.testing.assert_array_equal(c2.eval().get_text_embeds(texts).numpy(), clip.get_text_embeds(texts).numpy())


def test_chemeleon_builds_text_encoder_from_local_model():
    from chemeleon_amd import Chemeleon
    from chemeleon_amd.config import default_config
    from chemeleon_amd.text_encoder import TextEncoder
    cfg = default_config()
    cfg.update({"text_guide": True, "text_encoder": BERT_DIR, "text_embed_dim": 32, "max_text_len": 12,
                "timesteps": 10})
    m = Chemeleon(cfg, text_model_dir=BERT_DIR)
    assert isinstance(m.text_encoder, TextEncoder)
    with torch.no_grad():
        e = m.text_encoder.get_text_embeds(["Ti O2", "Li Fe P O4"], 0.0, "cpu")
    assert e.shape == (2, cfg["text_dim"])
    assert Chemeleon(cfg).text_encoder is None  # no local model configured: nothing is fetched


def test_hub_names_need_a_local_copy(monkeypatch):
    from chemeleon_amd.text_encoder import TextEncoder
    monkeypatch.delenv("CHEMELEON_TEXT_MODEL_DIR", raising=False)
    with pytest.raises(FileNotFoundError, match="does not download"):
        TextEncoder("lfoppiano/MatTPUSciBERT")
    with pytest.raises(FileNotFoundError, match="CrystalCLIP"):
        TextEncoder("chemeleon/clip-mp-prompt")
    with pytest.raises(ValueError, match="Invalid model name"):
        TextEncoder("not-a-model")


def test_clip_checkpoint_with_graph_side_but_no_graph_config_fails_loudly(tmp_path):
    """A CrystalClip checkpoint whose state_dict carries graph_encoder.* / graph_proj.* tensors but whose
    hyper_parameters lack the graph keys cannot build its graph side: loading raises and names the
    missing keys (it used to file those tensors under ignored_keys and fail later in get_graph_embeds)."""
    from chemeleon_amd.text_encoder import CrystalClip
    hp = {"clip_dim": 32, "text_encoder": BERT_DIR, "max_text_len": 12, "text_embed_dim": 32}
    clip = CrystalClip(hp, text_model_dir=BERT_DIR)
    assert "graph_pooling" in clip.missing_graph_keys and "hidden_dim" in clip.missing_graph_keys
    with pytest.raises(RuntimeError, match="no graph encoder"):
        clip.get_graph_embeds(None)
    sd = dict(clip.state_dict())
    sd["graph_proj.0.weight"] = torch.zeros(4, 4)
    path = tmp_path / "clip.ckpt"
    torch.save({"state_dict": sd, "hyper_parameters": hp}, path)
    with pytest.raises(RuntimeError, match="graph_pooling"):
        CrystalClip.load_from_checkpoint(str(path), text_model_dir=BERT_DIR)
    del sd["graph_proj.0.weight"]  # without graph tensors the text-only checkpoint loads
    torch.save({"state_dict": sd, "hyper_parameters": hp}, path)
    CrystalClip.load_from_checkpoint(str(path), text_model_dir=BERT_DIR)
