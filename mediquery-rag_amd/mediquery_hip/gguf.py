"""Local GGUF model files -> encoder weights, config and WordPiece vocabulary.

The reference embeds with `OllamaEmbeddings(model="shaw/dmeta-embedding-zh")`
(src/medical_engine.py:43, src/ingest_medical.py:104): Ollama serves that model from a
GGUF blob in its local store and runs it with llama.cpp's BERT graph.  This module reads
such a file - nothing is downloaded - so the MI355X encoder can run the same weights:

* `resolve_ollama_model(name)`: Ollama's on-disk store ($OLLAMA_MODELS or ~/.ollama/models):
  manifests/<registry>/<namespace>/<model>/<tag> (JSON) names the model layer's blob
  (`application/vnd.ollama.image.model`, digest sha256:<hex>) -> blobs/sha256-<hex>.
* `read_gguf(path)`: GGUF v2/v3 container (header, typed metadata, tensor table, aligned
  data) with F32 / F16 / BF16 / Q8_0 tensors, memory-mapped.
* `bert_from_gguf(path)`: llama.cpp BERT tensor names (token_embd, position_embd,
  token_types, token_embd_norm, blk.N.{attn_q,attn_k,attn_v | attn_qkv, attn_output,
  attn_output_norm, ffn_up, ffn_down, layer_output_norm}) -> the HF-named state dict of
  weights.py (dequantised to fp32), a BertConfig from the `bert.*` metadata (pooling from
  bert.pooling_type, GELU = tanh: the ggml op llama.cpp's BERT graph uses), and the
  WordPiece vocabulary from tokenizer.ggml.tokens with llama.cpp's "phantom space" token
  spelling undone ("▁word" -> "word", "piece" -> "##piece", "[X]" kept).

The file layout, tensor names and vocab spelling are those of llama.cpp's GGUF / BERT
conversion (third-party, absent here): parity with a real Ollama blob is UNPINNED; the
tests round-trip files written to the same spec (tests/gguf_writer.py).
"""
import json
import os
import struct

import numpy as np

from .config import BertConfig, GELU_TANH, POOL_CLS, POOL_MEAN

GGUF_MAGIC = b"GGUF"
# metadata value types
_U8, _I8, _U16, _I16, _U32, _I32, _F32, _BOOL, _STR, _ARR, _U64, _I64, _F64 = range(13)
_SCALAR = {_U8: "<B", _I8: "<b", _U16: "<H", _I16: "<h", _U32: "<I", _I32: "<i", _F32: "<f",
           _BOOL: "<?", _U64: "<Q", _I64: "<q", _F64: "<d"}
# ggml tensor types handled
GGML_F32, GGML_F16, GGML_Q8_0, GGML_BF16 = 0, 1, 8, 30
Q8_0_BLOCK = 32  # Q8_0: blocks of 32 values = f16 scale + 32 int8

OLLAMA_MODEL_MEDIA = "application/vnd.ollama.image.model"
# llama.cpp pooling enum (LLAMA_POOLING_TYPE_*)
_POOLING = {1: POOL_MEAN, 2: POOL_CLS}


class GGUFError(ValueError):
    pass


class _Reader:
    def __init__(self, buf):
        self.buf = buf
        self.pos = 0

    def take(self, fmt):
        v = struct.unpack_from(fmt, self.buf, self.pos)[0]
        self.pos += struct.calcsize(fmt)
        return v

    def string(self):
        n = self.take("<Q")
        s = bytes(self.buf[self.pos:self.pos + n]).decode("utf-8", errors="surrogateescape")
        self.pos += n
        return s

    def value(self, vtype):
        if vtype in _SCALAR:
            return self.take(_SCALAR[vtype])
        if vtype == _STR:
            return self.string()
        if vtype == _ARR:
            etype, n = self.take("<I"), self.take("<Q")
            if etype in _SCALAR:  # numeric arrays in one read
                fmt = _SCALAR[etype]
                size = struct.calcsize(fmt)
                out = np.frombuffer(self.buf, dtype=np.dtype(fmt), count=n, offset=self.pos).tolist()
                self.pos += n * size
                return out
            return [self.value(etype) for _ in range(n)]
        raise GGUFError("unknown GGUF metadata type %d" % vtype)


def read_gguf(path):
    """-> (metadata dict, {tensor name: np.ndarray in ggml's dims reversed, i.e. row-major
    [..., ne1, ne0]}).  F32/F16/BF16 tensors are zero-copy views of the mapped file (BF16
    widened to fp32), Q8_0 tensors are dequantised to fp32."""
    buf = np.memmap(path, dtype=np.uint8, mode="r")
    r = _Reader(buf)
    if bytes(buf[:4]) != GGUF_MAGIC:
        raise GGUFError("%s is not a GGUF file" % path)
    r.pos = 4
    version = r.take("<I")
    if version not in (2, 3):
        raise GGUFError("GGUF version %d unsupported (2, 3)" % version)
    n_tensors, n_kv = r.take("<Q"), r.take("<Q")
    meta = {}
    for _ in range(n_kv):
        key = r.string()
        meta[key] = r.value(r.take("<I"))
    infos = []
    for _ in range(n_tensors):
        name = r.string()
        nd = r.take("<I")
        dims = [r.take("<Q") for _ in range(nd)]
        ttype, off = r.take("<I"), r.take("<Q")
        infos.append((name, dims, ttype, off))
    align = int(meta.get("general.alignment", 32))
    data0 = (r.pos + align - 1) // align * align
    tensors = {}
    for name, dims, ttype, off in infos:
        shape = tuple(reversed(dims))  # ne0 is the fastest-varying dimension
        n = int(np.prod(dims)) if dims else 1
        at = data0 + off
        if ttype == GGML_F32:
            t = np.frombuffer(buf, np.float32, n, at)
        elif ttype == GGML_F16:
            t = np.frombuffer(buf, np.float16, n, at)
        elif ttype == GGML_BF16:
            t = (np.frombuffer(buf, np.uint16, n, at).astype(np.uint32) << 16).view(np.float32)
        elif ttype == GGML_Q8_0:
            if n % Q8_0_BLOCK:
                raise GGUFError("%s: Q8_0 tensor of %d values" % (name, n))
            blocks = np.frombuffer(buf, np.uint8, n // Q8_0_BLOCK * 34, at).reshape(-1, 34)
            d = blocks[:, :2].copy().view(np.float16).astype(np.float32)
            q = blocks[:, 2:].view(np.int8).astype(np.float32)
            t = (q * d).reshape(-1)
        else:
            raise GGUFError("%s: ggml tensor type %d unsupported (F32, F16, BF16, Q8_0)" % (name, ttype))
        tensors[name] = t.reshape(shape)
    return meta, tensors


def unphantom(tok):
    """llama.cpp BERT vocab spelling -> WordPiece: the converter wrote "[X]" unchanged,
    "##piece" as "piece" and every other token with a leading U+2581."""
    if tok.startswith("[") and tok.endswith("]"):
        return tok
    if tok.startswith("▁"):
        return tok[1:]
    return "##" + tok


def bert_from_gguf(path, gelu=GELU_TANH):
    """-> (state dict with HF BertModel names (fp32), BertConfig, WordPiece tokens or None)."""
    meta, t = read_gguf(path)
    arch = meta.get("general.architecture", "bert")
    if arch != "bert":
        raise GGUFError("%s: architecture %r, expected 'bert'" % (path, arch))

    def m(key, default=None):
        v = meta.get("bert." + key, default)
        if v is None:
            raise GGUFError("%s: missing metadata bert.%s" % (path, key))
        return v

    word = t["token_embd.weight"]
    H = int(m("embedding_length", word.shape[1]))
    layers = int(m("block_count"))
    cfg = BertConfig(vocab_size=int(word.shape[0]), hidden=H, layers=layers,
                     heads=int(m("attention.head_count")), ffn=int(m("feed_forward_length")),
                     max_positions=int(t["position_embd.weight"].shape[0]),
                     type_vocab=int(t["token_types.weight"].shape[0]) if "token_types.weight" in t else 1,
                     ln_eps=float(m("attention.layer_norm_epsilon", 1e-12)), gelu=gelu,
                     pooling=_POOLING.get(int(m("pooling_type", 2)), POOL_CLS))

    def f32(x):
        return np.ascontiguousarray(x, dtype=np.float32)

    sd = {"embeddings.word_embeddings.weight": f32(word),
          "embeddings.position_embeddings.weight": f32(t["position_embd.weight"]),
          "embeddings.token_type_embeddings.weight":
              f32(t["token_types.weight"]) if "token_types.weight" in t else np.zeros((1, H), np.float32),
          "embeddings.LayerNorm.weight": f32(t["token_embd_norm.weight"]),
          "embeddings.LayerNorm.bias": f32(t["token_embd_norm.bias"])}
    for l in range(layers):
        b, p = "blk.%d." % l, "encoder.layer.%d." % l
        if b + "attn_qkv.weight" in t:  # fused projection: q rows, k rows, v rows
            w, bias = f32(t[b + "attn_qkv.weight"]), f32(t[b + "attn_qkv.bias"])
            for i, proj in enumerate(("query", "key", "value")):
                sd[p + "attention.self.%s.weight" % proj] = w[i * H:(i + 1) * H]
                sd[p + "attention.self.%s.bias" % proj] = bias[i * H:(i + 1) * H]
        else:
            for g, proj in (("attn_q", "query"), ("attn_k", "key"), ("attn_v", "value")):
                sd[p + "attention.self.%s.weight" % proj] = f32(t[b + g + ".weight"])
                sd[p + "attention.self.%s.bias" % proj] = f32(t[b + g + ".bias"])
        for g, hf in (("attn_output", "attention.output.dense"),
                      ("attn_output_norm", "attention.output.LayerNorm"),
                      ("ffn_up", "intermediate.dense"), ("ffn_down", "output.dense"),
                      ("layer_output_norm", "output.LayerNorm")):
            sd[p + hf + ".weight"] = f32(t[b + g + ".weight"])
            sd[p + hf + ".bias"] = f32(t[b + g + ".bias"])
    toks = meta.get("tokenizer.ggml.tokens")
    vocab = None
    if toks is not None and meta.get("tokenizer.ggml.model", "bert") == "bert":
        vocab = [unphantom(x) for x in toks]
    return sd, cfg, vocab


def ollama_models_dir():
    return os.environ.get("OLLAMA_MODELS") or os.path.join(os.path.expanduser("~"), ".ollama", "models")


def resolve_ollama_model(name, models_dir=None):
    """Ollama model name ("shaw/dmeta-embedding-zh", "[host/]ns/model[:tag]") -> path of its
    GGUF blob in the local store, or None if the model was never pulled there."""
    root = models_dir or ollama_models_dir()
    ref, tag = name, "latest"
    if ":" in name.rsplit("/", 1)[-1]:
        ref, tag = name.rsplit(":", 1)
    parts = ref.split("/")
    if len(parts) == 1:
        parts = ["registry.ollama.ai", "library"] + parts
    elif len(parts) == 2:
        parts = ["registry.ollama.ai"] + parts
    manifest = os.path.join(root, "manifests", *parts, tag)
    if not os.path.isfile(manifest):
        return None
    with open(manifest, "r", encoding="utf-8") as f:
        layers = json.load(f).get("layers", [])
    for layer in layers:
        if layer.get("mediaType") == OLLAMA_MODEL_MEDIA:
            blob = os.path.join(root, "blobs", layer["digest"].replace(":", "-"))
            if not os.path.isfile(blob):
                raise FileNotFoundError("manifest %s names blob %s, which is missing" % (manifest, blob))
            return blob
    raise GGUFError("manifest %s has no %s layer" % (manifest, OLLAMA_MODEL_MEDIA))
