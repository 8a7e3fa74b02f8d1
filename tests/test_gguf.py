"""GGUF model files (gguf.py): the encoder's weights, config and WordPiece vocabulary read
from the file format Ollama serves `shaw/dmeta-embedding-zh` from (reference
src/medical_engine.py:43), and the model name resolved through Ollama's local store.
Files are written to llama.cpp's layout by tests/gguf_writer.py (no real blob offline:
parity with one is unpinned)."""
import dataclasses
import json
import os

import numpy as np
import pytest

from gguf_writer import GGML_BF16, GGML_F16, GGML_F32, GGML_Q8_0, phantom, write_bert_gguf
from mediquery_hip.config import GELU_TANH, POOL_CLS, POOL_MEAN, BertConfig
from mediquery_hip.gguf import GGUFError, bert_from_gguf, read_gguf, resolve_ollama_model, unphantom
from mediquery_hip.weights import hf_names, synthetic_state_dict

VOCAB = (["[PAD]"] + ["[unused%d]" % i for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
         + list("血糖高压心脏病头痛发热咳嗽") + ["high", "##er", "##s", "blood", "pressure", "[", "]", "#"])


def tiny_cfg(**kw):
    base = dict(vocab_size=len(VOCAB), hidden=256, layers=2, heads=4, ffn=512, max_positions=64,
                type_vocab=2, ln_eps=1e-12, gelu=GELU_TANH, pooling=POOL_CLS)
    base.update(kw)
    return BertConfig(**base)


@pytest.mark.parametrize("ttype", [GGML_F32, GGML_F16, GGML_BF16, GGML_Q8_0])
@pytest.mark.parametrize("fused", [False, True])
def test_bert_gguf_round_trip(tmp_path, ttype, fused):
    cfg = tiny_cfg()
    sd = synthetic_state_dict(cfg, 3)
    path = str(tmp_path / "m.gguf")
    stored = write_bert_gguf(path, sd, cfg, VOCAB, ttype=ttype, fused_qkv=fused)
    got, gcfg, vocab = bert_from_gguf(path)
    assert gcfg == dataclasses.replace(cfg, ln_eps=float(np.float32(cfg.ln_eps)))  # stored as f32
    assert vocab == VOCAB
    assert sorted(got) == sorted(n for n, _ in hf_names(cfg))
    H = cfg.hidden
    for l in range(cfg.layers):
        p, b = "encoder.layer.%d." % l, "blk.%d." % l
        for i, proj in enumerate(("query", "key", "value")):
            w = got[p + "attention.self.%s.weight" % proj]
            ref = stored[b + "attn_qkv.weight"][i * H:(i + 1) * H] if fused else stored[b + "attn_%s.weight" % proj[0]]
            np.testing.assert_array_equal(w, ref)
        np.testing.assert_array_equal(got[p + "output.dense.weight"], stored[b + "ffn_down.weight"])
        np.testing.assert_array_equal(got[p + "output.LayerNorm.bias"], sd[p + "output.LayerNorm.bias"])
    np.testing.assert_array_equal(got["embeddings.word_embeddings.weight"], stored["token_embd.weight"])
    for name, x in got.items():
        assert x.dtype == np.float32 and x.flags["C_CONTIGUOUS"], name
        tol = {GGML_F32: 0, GGML_F16: 1e-3, GGML_BF16: 4e-3, GGML_Q8_0: 1e-2}[ttype] * max(1.0, np.abs(sd[name]).max())
        np.testing.assert_allclose(x, sd[name], atol=tol, rtol=0)


def test_gguf_metadata_config_and_pooling(tmp_path):
    cfg = tiny_cfg(ln_eps=1e-5)
    path = str(tmp_path / "m.gguf")
    write_bert_gguf(path, synthetic_state_dict(cfg, 0), cfg, VOCAB, ttype=GGML_F32, pooling_type=1)
    meta, tensors = read_gguf(path)
    assert meta["general.architecture"] == "bert" and meta["bert.block_count"] == 2
    assert tensors["blk.1.ffn_up.weight"].shape == (512, 256)
    _, gcfg, _ = bert_from_gguf(path)
    assert gcfg.pooling == POOL_MEAN and gcfg.gelu == GELU_TANH
    assert abs(gcfg.ln_eps - 1e-5) < 1e-12


def test_phantom_vocab_spelling_inverts():
    for tok in VOCAB + ["##", "▁", "a", "##ab"]:
        assert unphantom(phantom(tok)) == tok, tok


def test_rejects_non_gguf(tmp_path):
    p = tmp_path / "x.gguf"
    p.write_bytes(b"NOPE" + b"\0" * 64)
    with pytest.raises(GGUFError):
        read_gguf(str(p))


def _fake_store(root, name="shaw/dmeta-embedding-zh", tag="latest", blob=b"GGUF", with_model=True):
    parts = name.split("/")
    d = os.path.join(root, "manifests", "registry.ollama.ai", *parts)
    os.makedirs(d, exist_ok=True)
    digest = "sha256:" + "ab" * 32
    layers = [{"mediaType": "application/vnd.ollama.image.params", "digest": "sha256:" + "cd" * 32}]
    if with_model:
        layers.insert(0, {"mediaType": "application/vnd.ollama.image.model", "digest": digest})
    with open(os.path.join(d, tag), "w") as f:
        json.dump({"schemaVersion": 2, "layers": layers}, f)
    os.makedirs(os.path.join(root, "blobs"), exist_ok=True)
    path = os.path.join(root, "blobs", digest.replace(":", "-"))
    with open(path, "wb") as f:
        f.write(blob)
    return path


def test_resolve_ollama_model(tmp_path):
    root = str(tmp_path / "models")
    blob = _fake_store(root)
    assert resolve_ollama_model("shaw/dmeta-embedding-zh", root) == blob
    assert resolve_ollama_model("shaw/dmeta-embedding-zh:latest", root) == blob
    assert resolve_ollama_model("shaw/dmeta-embedding-zh:v2", root) is None
    assert resolve_ollama_model("nomic-embed-text", root) is None
    _fake_store(root, name="library/bge", blob=b"GGUF")
    assert resolve_ollama_model("bge", root).endswith("sha256-" + "ab" * 32)
    _fake_store(root, name="x/nomodel", with_model=False)
    with pytest.raises(GGUFError):
        resolve_ollama_model("x/nomodel", root)
