"""Generate encoder + end-to-end golden fixtures with `transformers.BertModel`
(5.15.0, fp32, eager attention) - the stand-in for the absent Ollama dmeta encoder
(SURVEY.md §8c).  Run in the build container; the outputs are committed and travel.

Writes tests/golden/encoder_golden.npz with, per case, the token ids/mask and the
expected unit-norm pooled embeddings:
  tiny_a      2 layers, erf GELU, CLS,  B=4, L=32  (all tokens valid)
  tiny_b      2 layers, erf GELU, CLS,  B=3, L=128 (ragged: 128 / 77 / 9 valid)
  tiny_b_mean same inputs, masked-mean pooling
  tiny_tanh   2 layers, tanh GELU, CLS, B=4, L=32
  base        12 layers (dmeta-base shape), erf GELU, CLS, B=2, L=32
and tests/golden/config1_golden.npz (BASELINE config 1): the 154 parsed documents and
32 hand-written queries through the char tokenizer and the 12-layer seeded encoder,
their embeddings and the float64 exact top-5 (ids, cosine) per query.

Weights: mediquery_hip.weights.synthetic_state_dict(cfg, seed=0).
Usage: python tests/golden/make_encoder_golden.py
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mediquery-rag_amd"))
sys.path.insert(0, ROOT)

from mediquery_hip.config import BertConfig, DMETA_BASE, GELU_TANH  # noqa: E402
from mediquery_hip.tokenizer import CharTokenizer  # noqa: E402
from mediquery_hip.weights import synthetic_state_dict  # noqa: E402
from oracle.flat import search  # noqa: E402

TINY = BertConfig(layers=2)
TINY_TANH = BertConfig(layers=2, gelu=GELU_TANH)


def hf_model(cfg):
    from transformers import BertConfig as HFConfig, BertModel
    hf = HFConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden,
                  num_hidden_layers=cfg.layers, num_attention_heads=cfg.heads,
                  intermediate_size=cfg.ffn, max_position_embeddings=cfg.max_positions,
                  type_vocab_size=cfg.type_vocab, layer_norm_eps=cfg.ln_eps,
                  hidden_act="gelu_pytorch_tanh" if cfg.gelu == GELU_TANH else "gelu",
                  attn_implementation="eager")
    m = BertModel(hf, add_pooling_layer=False).eval()
    sd = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(cfg, 0).items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all("position_ids" in k or "token_type_ids" in k for k in missing), missing
    return m


@torch.no_grad()
def hf_embed(model, ids, mask, pooling="cls", batch=16):
    outs = []
    for s in range(0, len(ids), batch):
        i = torch.as_tensor(ids[s:s + batch], dtype=torch.long)
        m = torch.as_tensor(mask[s:s + batch], dtype=torch.long)
        h = model(input_ids=i, attention_mask=m).last_hidden_state
        if pooling == "mean":
            mf = m.unsqueeze(-1).float()
            e = (h * mf).sum(1) / mf.sum(1).clamp_min(1.0)
        else:
            e = h[:, 0]
        outs.append(torch.nn.functional.normalize(e, dim=-1).numpy())
    return np.concatenate(outs).astype(np.float32)


def synth_ids(rng, B, L, lengths=None, vocab=21128):
    ids = np.zeros((B, L), np.int32)
    mask = np.zeros((B, L), np.int32)
    for b in range(B):
        n = L if lengths is None else lengths[b]
        ids[b, 0] = 101
        ids[b, 1:n - 1] = rng.integers(106, vocab, n - 2)
        ids[b, n - 1] = 102
        mask[b, :n] = 1
    return ids, mask


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    rng = np.random.default_rng(1)
    out = {}
    tiny = hf_model(TINY)
    ids, mask = synth_ids(rng, 4, 32)
    out.update(tiny_a_ids=ids, tiny_a_mask=mask, tiny_a_emb=hf_embed(tiny, ids, mask))
    ids, mask = synth_ids(rng, 3, 128, lengths=[128, 77, 9])
    out.update(tiny_b_ids=ids, tiny_b_mask=mask, tiny_b_emb=hf_embed(tiny, ids, mask),
               tiny_b_mean_emb=hf_embed(tiny, ids, mask, pooling="mean"))
    tanh = hf_model(TINY_TANH)
    ids, mask = synth_ids(rng, 4, 32)
    out.update(tiny_tanh_ids=ids, tiny_tanh_mask=mask, tiny_tanh_emb=hf_embed(tanh, ids, mask))
    base = hf_model(DMETA_BASE)
    ids, mask = synth_ids(rng, 2, 32)
    out.update(base_ids=ids, base_mask=mask, base_emb=hf_embed(base, ids, mask))
    np.savez_compressed(os.path.join(HERE, "encoder_golden.npz"), **out)

    # ---- config 1: real corpus text, char tokenizer, 12-layer seeded encoder ----------
    docs = json.load(open(os.path.join(HERE, "corpus_docs.json"), encoding="utf-8"))["docs"]
    queries = json.load(open(os.path.join(HERE, "config1_queries.json"), encoding="utf-8"))["queries"]
    tok = CharTokenizer(DMETA_BASE.vocab_size, max_length=512)

    def embed_texts(texts):
        res = np.zeros((len(texts), DMETA_BASE.hidden), np.float32)
        order = sorted(range(len(texts)), key=lambda i: len(texts[i]))
        for s in range(0, len(order), 16):
            idx = order[s:s + 16]
            ids, mask = tok([texts[i] for i in idx])
            res[idx] = hf_embed(base, ids, mask)
        return res

    d_emb = embed_texts([d["page_content"] for d in docs])
    q_emb = embed_texts(queries)
    scores, ids = search(q_emb, d_emb, 5)
    np.savez_compressed(os.path.join(HERE, "config1_golden.npz"), doc_emb=d_emb, query_emb=q_emb,
                        top5_ids=ids, top5_scores=scores)
    print("wrote encoder_golden.npz and config1_golden.npz; top-1 ids:", ids[:, 0].tolist())


if __name__ == "__main__":
    main()
