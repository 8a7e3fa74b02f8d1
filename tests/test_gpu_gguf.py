"""The reference's constructor line, unchanged: `OllamaEmbeddings(model="shaw/dmeta-embedding-zh")`
(src/medical_engine.py:43) resolves the model through Ollama's local store to its GGUF blob
and runs it on the HIP encoder - weights, architecture (GELU tanh, pooling from the file)
and WordPiece vocab all from that one file.  The store and blob here are written to
llama.cpp's layout by tests/gguf_writer.py (no real blob offline)."""
import json
import os

import numpy as np
import pytest

from gguf_writer import GGML_F16, write_bert_gguf
from mediquery_hip import OllamaEmbeddings
from mediquery_hip.config import GELU_TANH, POOL_CLS, BertConfig
from mediquery_hip.tokenizer import WordPieceTokenizer
from mediquery_hip.weights import synthetic_state_dict
from oracle.encoder import OracleEncoder

pytestmark = pytest.mark.gpu

VOCAB = (["[PAD]"] + ["[unused%d]" % i for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
         + list("血糖高压心脏病头痛发热咳嗽如何治疗") + ["high", "##er", "blood", "pressure", "?"])


def test_ollama_model_name_runs_the_gguf_blob(require_gpu, tmp_path, monkeypatch):
    cfg = BertConfig(vocab_size=len(VOCAB), hidden=256, layers=2, heads=4, ffn=512, max_positions=64,
                     gelu=GELU_TANH, pooling=POOL_CLS)
    sd = synthetic_state_dict(cfg, 5)
    root = tmp_path / "models"
    blob_dir, man_dir = root / "blobs", root / "manifests" / "registry.ollama.ai" / "shaw" / "dmeta-embedding-zh"
    blob_dir.mkdir(parents=True)
    man_dir.mkdir(parents=True)
    digest = "sha256:" + "5e" * 32
    stored = write_bert_gguf(str(blob_dir / digest.replace(":", "-")), sd, cfg, VOCAB, ttype=GGML_F16)
    (man_dir / "latest").write_text(json.dumps(
        {"layers": [{"mediaType": "application/vnd.ollama.image.model", "digest": digest}]}))
    for v in ("MQ_WEIGHTS_PATH", "MQ_VOCAB_FILE", "MQ_GGUF_PATH"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("OLLAMA_MODELS", str(root))

    embeddings = OllamaEmbeddings(model="shaw/dmeta-embedding-zh")   # the unchanged line :43
    assert embeddings.config.hidden == 256 and embeddings.config.gelu == GELU_TANH
    texts = ["血糖高如何治疗?", "blood pressure higher", "头痛发热咳嗽", "心脏病"]
    got = np.asarray(embeddings.embed_documents(texts), np.float32)

    # the same file through the Python WordPiece twin + the fp32 oracle (stored = f16 round trip)
    vocab_txt = tmp_path / "vocab.txt"
    vocab_txt.write_text("\n".join(VOCAB) + "\n", encoding="utf-8")
    ids, mask = WordPieceTokenizer(str(vocab_txt))(texts)
    tok_ids, tok_mask = embeddings.tokenizer(texts)
    np.testing.assert_array_equal(tok_ids, ids)
    assert ids[0, 1] == VOCAB.index("血") and VOCAB[ids[1, 4]] == "##er"
    sd16 = dict(sd)
    names = {"embeddings.word_embeddings.weight": "token_embd.weight",
             "embeddings.position_embeddings.weight": "position_embd.weight",
             "embeddings.token_type_embeddings.weight": "token_types.weight"}
    for hf, g in names.items():
        sd16[hf] = stored[g]
    for l in range(cfg.layers):
        p, b = "encoder.layer.%d." % l, "blk.%d." % l
        for hf, g in (("attention.self.query", "attn_q"), ("attention.self.key", "attn_k"),
                      ("attention.self.value", "attn_v"), ("attention.output.dense", "attn_output"),
                      ("intermediate.dense", "ffn_up"), ("output.dense", "ffn_down")):
            sd16[p + hf + ".weight"] = stored[b + g + ".weight"]
    ref = OracleEncoder(cfg, sd16).embed(ids, mask)
    np.testing.assert_allclose(got, ref, atol=1e-4, rtol=0)
    assert np.allclose(np.linalg.norm(got, axis=1), 1.0, atol=1e-5)
