"""Encoder weights: HF-named state dicts <-> the flat fp32 blob the C-ABI consumes.

No dmeta-embedding-zh weights exist in this environment, so parity and
benchmarks run on *seeded synthetic* weights of the exact BERT-base architecture.  The
generator is part of the input definition (like the seeded corpus), shared verbatim by
the product, the oracle and the fixture scripts.  Real weights load from a local
safetensors file with HF BERT names via `load_safetensors`.

Blob layout (all fp32, row-major, PyTorch Linear convention W[out][in]) - the order
`mq_encoder_load_weights` (include/mq.h) expects:
    word[V,H] pos[P,H] type[T,H] emb_ln.g[H] emb_ln.b[H]
    per layer l:  Wqkv[3H,H] (q rows, k rows, v rows)  bqkv[3H]
                  Wo[H,H] bo[H] ln1.g[H] ln1.b[H]
                  W1[F,H] b1[F] W2[H,F] b2[H] ln2.g[H] ln2.b[H]
"""
import numpy as np

from .config import BertConfig

_P = "encoder.layer.%d."


def hf_names(cfg: BertConfig):
    """(name, shape) of every tensor, HF BertModel naming, blob order."""
    H, F = cfg.hidden, cfg.ffn
    out = [("embeddings.word_embeddings.weight", (cfg.vocab_size, H)),
           ("embeddings.position_embeddings.weight", (cfg.max_positions, H)),
           ("embeddings.token_type_embeddings.weight", (cfg.type_vocab, H)),
           ("embeddings.LayerNorm.weight", (H,)),
           ("embeddings.LayerNorm.bias", (H,))]
    for l in range(cfg.layers):
        p = _P % l
        for proj in ("query", "key", "value"):
            out.append((p + "attention.self.%s.weight" % proj, (H, H)))
            out.append((p + "attention.self.%s.bias" % proj, (H,)))
        out += [(p + "attention.output.dense.weight", (H, H)),
                (p + "attention.output.dense.bias", (H,)),
                (p + "attention.output.LayerNorm.weight", (H,)),
                (p + "attention.output.LayerNorm.bias", (H,)),
                (p + "intermediate.dense.weight", (F, H)),
                (p + "intermediate.dense.bias", (F,)),
                (p + "output.dense.weight", (H, F)),
                (p + "output.dense.bias", (H,)),
                (p + "output.LayerNorm.weight", (H,)),
                (p + "output.LayerNorm.bias", (H,))]
    return out


def synthetic_state_dict(cfg: BertConfig, seed: int = 0):
    """Seeded BERT weights: N(0, 0.02) matrices/embeddings/biases, LayerNorm gain
    1 + N(0, 0.05) and bias N(0, 0.05) (non-trivial so LN bugs cannot hide)."""
    sd = {}
    for idx, (name, shape) in enumerate(hf_names(cfg)):
        rng = np.random.default_rng([seed, idx])
        x = rng.standard_normal(shape, dtype=np.float32)
        if name.endswith("LayerNorm.weight"):
            x = 1.0 + 0.05 * x
        elif name.endswith("LayerNorm.bias"):
            x = 0.05 * x
        else:
            x = 0.02 * x
        sd[name] = x.astype(np.float32, copy=False)
    return sd


def blob_size(cfg: BertConfig):
    H, F = cfg.hidden, cfg.ffn
    per_layer = 3 * H * H + 3 * H + H * H + H + 2 * H + F * H + F + H * F + H + 2 * H
    return (cfg.vocab_size + cfg.max_positions + cfg.type_vocab) * H + 2 * H + cfg.layers * per_layer


def state_dict_to_blob(cfg: BertConfig, sd):
    """HF-named dict of arrays (numpy or torch) -> contiguous fp32 blob."""
    parts = []

    def put(name, shape):
        v = sd[name]
        v = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
        if tuple(v.shape) != tuple(shape):
            raise ValueError("%s: shape %s, expected %s" % (name, v.shape, shape))
        parts.append(np.ascontiguousarray(v, dtype=np.float32).reshape(-1))

    names = dict(hf_names(cfg))
    for n in list(names)[:5]:
        put(n, names[n])
    for l in range(cfg.layers):
        p = _P % l
        for suffix in ("weight", "bias"):   # fused QKV: q rows, then k rows, then v rows
            for proj in ("query", "key", "value"):
                n = p + "attention.self.%s.%s" % (proj, suffix)
                put(n, names[n])
        for n in ("attention.output.dense.weight", "attention.output.dense.bias",
                  "attention.output.LayerNorm.weight", "attention.output.LayerNorm.bias",
                  "intermediate.dense.weight", "intermediate.dense.bias",
                  "output.dense.weight", "output.dense.bias",
                  "output.LayerNorm.weight", "output.LayerNorm.bias"):
            put(p + n, names[p + n])
    blob = np.concatenate(parts)
    assert blob.size == blob_size(cfg), (blob.size, blob_size(cfg))
    return blob


def load_safetensors(path, cfg: BertConfig):
    """Real weights from a LOCAL safetensors file with HF BERT names (an optional
    "bert." prefix is stripped). Nothing is downloaded."""
    from safetensors.numpy import load_file
    raw = load_file(path)
    sd = {}
    for k, v in raw.items():
        sd[k[5:] if k.startswith("bert.") else k] = v
    return sd
