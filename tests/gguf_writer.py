"""Test helper: write a GGUF v3 file the way llama.cpp's converter lays out a BERT model
(tensor names, reversed dims, aligned data, "phantom space" vocab spelling), so the loader
in mediquery_hip/gguf.py can be round-tripped without a real Ollama blob (absent offline).
Only tests import this."""
import struct

import numpy as np

GGML_F32, GGML_F16, GGML_Q8_0, GGML_BF16 = 0, 1, 8, 30
_U32, _F32, _STR, _ARR, _I32 = 4, 6, 8, 9, 5


def phantom(tok):
    """llama.cpp's BERT vocab spelling (the inverse of gguf.unphantom)."""
    if tok.startswith("[") and tok.endswith("]"):
        return tok
    if tok.startswith("##"):
        return tok[2:]
    return "▁" + tok


def _s(x):
    b = x.encode("utf-8")
    return struct.pack("<Q", len(b)) + b


def _kv(key, vtype, val):
    out = _s(key) + struct.pack("<I", vtype)
    if vtype == _STR:
        return out + _s(val)
    if vtype == _U32:
        return out + struct.pack("<I", val)
    if vtype == _F32:
        return out + struct.pack("<f", val)
    if vtype == _ARR:
        etype, items = val
        out += struct.pack("<IQ", etype, len(items))
        if etype == _STR:
            return out + b"".join(_s(i) for i in items)
        return out + np.asarray(items, dtype="<i4" if etype == _I32 else "<u4").tobytes()
    raise ValueError(vtype)


def quantize_q8_0(x):
    """fp32 -> Q8_0 bytes (blocks of 32: f16 scale = max|x| / 127, int8 round(x / scale))."""
    x = np.asarray(x, np.float32).reshape(-1, 32)
    d = (np.abs(x).max(1) / 127.0).astype(np.float16)
    df = d.astype(np.float32)
    q = np.where(df[:, None] > 0, np.round(x / np.where(df > 0, df, 1)[:, None]), 0).astype(np.int8)
    blocks = np.concatenate([d.view(np.uint8).reshape(-1, 2), q.view(np.uint8)], axis=1)
    return blocks.tobytes(), (q.astype(np.float32) * df[:, None]).reshape(-1)


def encode_tensor(x, ttype):
    """-> (bytes, the fp32 values a reader recovers)."""
    x = np.ascontiguousarray(x, np.float32)
    if ttype == GGML_F32:
        return x.tobytes(), x.reshape(-1)
    if ttype == GGML_F16:
        h = x.astype(np.float16)
        return h.tobytes(), h.astype(np.float32).reshape(-1)
    if ttype == GGML_BF16:
        u = x.view(np.uint32)
        b = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
        return b.tobytes(), (b.astype(np.uint32) << 16).view(np.float32).reshape(-1)
    if ttype == GGML_Q8_0:
        return quantize_q8_0(x)
    raise ValueError(ttype)


def write_bert_gguf(path, sd, cfg, vocab, ttype=GGML_F16, fused_qkv=False, pooling_type=2,
                    alignment=32):
    """HF-named fp32 state dict -> GGUF file; returns {gguf tensor name: fp32 values as
    stored} (after the dtype round trip).  1-D tensors (biases, norms) stay F32, as
    llama.cpp's converter keeps them."""
    H = cfg.hidden
    named = [("token_embd.weight", sd["embeddings.word_embeddings.weight"]),
             ("position_embd.weight", sd["embeddings.position_embeddings.weight"]),
             ("token_types.weight", sd["embeddings.token_type_embeddings.weight"]),
             ("token_embd_norm.weight", sd["embeddings.LayerNorm.weight"]),
             ("token_embd_norm.bias", sd["embeddings.LayerNorm.bias"])]
    for l in range(cfg.layers):
        p, b = "encoder.layer.%d." % l, "blk.%d." % l
        q, k, v = (sd[p + "attention.self.%s.weight" % n] for n in ("query", "key", "value"))
        qb, kb, vb = (sd[p + "attention.self.%s.bias" % n] for n in ("query", "key", "value"))
        if fused_qkv:
            named += [(b + "attn_qkv.weight", np.concatenate([q, k, v])),
                      (b + "attn_qkv.bias", np.concatenate([qb, kb, vb]))]
        else:
            named += [(b + "attn_q.weight", q), (b + "attn_q.bias", qb), (b + "attn_k.weight", k),
                      (b + "attn_k.bias", kb), (b + "attn_v.weight", v), (b + "attn_v.bias", vb)]
        for g, hf in (("attn_output", "attention.output.dense"), ("attn_output_norm", "attention.output.LayerNorm"),
                      ("ffn_up", "intermediate.dense"), ("ffn_down", "output.dense"),
                      ("layer_output_norm", "output.LayerNorm")):
            named += [(b + g + ".weight", sd[p + hf + ".weight"]), (b + g + ".bias", sd[p + hf + ".bias"])]
    meta = [("general.architecture", _STR, "bert"), ("general.alignment", _U32, alignment),
            ("bert.context_length", _U32, cfg.max_positions), ("bert.embedding_length", _U32, H),
            ("bert.feed_forward_length", _U32, cfg.ffn), ("bert.block_count", _U32, cfg.layers),
            ("bert.attention.head_count", _U32, cfg.heads),
            ("bert.attention.layer_norm_epsilon", _F32, cfg.ln_eps),
            ("bert.pooling_type", _U32, pooling_type),
            ("tokenizer.ggml.model", _STR, "bert"),
            ("tokenizer.ggml.tokens", _ARR, (_STR, [phantom(t) for t in vocab])),
            ("tokenizer.ggml.token_type", _ARR, (_I32, [1] * len(vocab)))]
    blobs, infos, stored, off = [], [], {}, 0
    for name, x in named:
        x = np.asarray(x, np.float32)
        tt = ttype if x.ndim == 2 else GGML_F32
        data, back = encode_tensor(x, tt)
        stored[name] = back.reshape(x.shape)
        pad = (-off) % alignment
        blobs.append(b"\0" * pad + data)
        off += pad
        dims = list(reversed(x.shape))
        infos.append(_s(name) + struct.pack("<I", len(dims)) + b"".join(struct.pack("<Q", d) for d in dims)
                     + struct.pack("<IQ", tt, off))
        off += len(data)
    head = b"GGUF" + struct.pack("<IQQ", 3, len(infos), len(meta))
    head += b"".join(_kv(*m) for m in meta) + b"".join(infos)
    head += b"\0" * ((-len(head)) % alignment)
    with open(path, "wb") as f:
        f.write(head)
        f.write(b"".join(blobs))
    return stored
