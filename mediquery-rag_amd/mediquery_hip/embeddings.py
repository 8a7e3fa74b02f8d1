"""`HipBertEmbeddings` - drop-in for `langchain_ollama.OllamaEmbeddings` on MI355X.

Reference call sites (unchanged by the swap):
  * `OllamaEmbeddings(model="shaw/dmeta-embedding-zh")`  src/medical_engine.py:43,
    src/ingest_medical.py:104
  * `embed_documents(texts)` - reached through `Chroma.from_documents(...)`
    (src/ingest_medical.py:106-110)
  * `embed_query(text)` - reached through `vectorstore.similarity_search(q, k=5)`
    (src/agents/nodes.py:93)
Same contract as LangChain's Embeddings: lists of python floats, one unit-norm
768-vector per text.  The forward runs in libmqhip.so (HIP, gfx950); nothing here
computes embeddings on the CPU.

Weights and vocabulary are never downloaded.  They come, in this order, from:
  1. `weights_path` + `vocab_file` (or $MQ_WEIGHTS_PATH + $MQ_VOCAB_FILE): a local
     safetensors file with HF BERT names and its vocab.txt;
  2. `gguf_path` (or $MQ_GGUF_PATH, or a `weights_path` ending in .gguf): a local GGUF file -
     weights, architecture and WordPiece vocab in one (gguf.py);
  3. Ollama's local model store: `model` resolved through its manifest to the GGUF blob an
     earlier `ollama pull` left there ($OLLAMA_MODELS or ~/.ollama/models) - so the
     reference's unchanged `OllamaEmbeddings(model="shaw/dmeta-embedding-zh")` runs the
     same model file on the MI355X.
Otherwise the constructor raises.  Seeded random weights with the char tokenizer (tests,
benchmarks) must be asked for explicitly with `synthetic=True`: a silently random encoder
would hand the Retrieve node semantically random documents.

Arithmetic (`precision=`): "f32x6" (the default, so the
reference's unchanged `OllamaEmbeddings(model=...)` line at src/medical_engine.py:43 and
src/ingest_medical.py:104 gets the headline configuration) splits every fp32 operand of the
batched GEMMs exactly into three bf16 planes and sums six bf16 MFMA products in fp32 -
fp32-class results (error within 3x of exact fp32 against float64, same parity tolerances);
"f32" runs the exact fp32 MFMA.  Single queries and other few-row batches run exact fp32
either way (the split does not pay when the weights, not the MFMAs, bound the launch).
$MQ_ENCODER_PRECISION sets the default for constructors that do not pass it.
"""
import os

import numpy as np

from . import _lib
from .compat import EmbeddingsBase
from .config import BertConfig, DMETA_BASE
from .gguf import bert_from_gguf, resolve_ollama_model
from .native import Encoder
from .tokenizer import NativeTokenizer
from .weights import load_safetensors

ENV_WEIGHTS = "MQ_WEIGHTS_PATH"
ENV_VOCAB = "MQ_VOCAB_FILE"
ENV_GGUF = "MQ_GGUF_PATH"
ENV_PRECISION = "MQ_ENCODER_PRECISION"
PRECISIONS = {"f32": _lib.MQ_DTYPE_F32, "f32x6": _lib.MQ_DTYPE_F32X6}
DEFAULT_PRECISION = "f32x6"


class HipBertEmbeddings(EmbeddingsBase):
    """BERT-base CLS embeddings computed by the hand-written HIP encoder.

    model:        the Ollama model name; resolved in Ollama's local store when no weight
                  file is given (source 3 above).
    weights_path: local safetensors with HF BERT names (default: $MQ_WEIGHTS_PATH), or a
                  .gguf file.
    vocab_file:   local WordPiece vocab.txt (default: $MQ_VOCAB_FILE); required with
                  safetensors weights - the char tokenizer would feed them meaningless ids.
    gguf_path:    local GGUF model file (default: $MQ_GGUF_PATH): weights, config (GELU =
                  tanh, llama.cpp's) and vocab; `config` overrides the derived config.
    synthetic:    True = seeded random weights + the deterministic char tokenizer
                  (`seed`); the only way to get them.
    precision:    "f32x6" (default; $MQ_ENCODER_PRECISION) or "f32" - module doc.
    """

    def __init__(self, model="shaw/dmeta-embedding-zh", *, weights_path=None, vocab_file=None,
                 gguf_path=None, synthetic=False, config: BertConfig = None, seed=0, device=0,
                 batch_size=256, max_length=512, precision=None, **kwargs):
        precision = precision or os.environ.get(ENV_PRECISION) or DEFAULT_PRECISION
        if precision not in PRECISIONS:
            raise ValueError("precision must be one of %s, got %r" % (sorted(PRECISIONS), precision))
        self.precision = precision
        self.model = model
        self.device = device
        self.batch_size = int(batch_size)
        self.synthetic = bool(synthetic)
        vocab_tokens = None
        if self.synthetic:
            if weights_path or vocab_file or gguf_path:
                raise ValueError("synthetic=True takes no weights_path / vocab_file / gguf_path")
            config = config or DMETA_BASE
            weights = None
        else:
            weights_path = weights_path or os.environ.get(ENV_WEIGHTS)
            vocab_file = vocab_file or os.environ.get(ENV_VOCAB)
            if weights_path and str(weights_path).endswith(".gguf"):
                gguf_path, weights_path = weights_path, None
            gguf_path = gguf_path or (None if weights_path else os.environ.get(ENV_GGUF))
            if not weights_path and not gguf_path:
                gguf_path = resolve_ollama_model(model)
            if gguf_path:
                if not os.path.isfile(gguf_path):
                    raise FileNotFoundError("GGUF file %r does not exist" % gguf_path)
                weights, gcfg, vocab_tokens = bert_from_gguf(gguf_path)
                config = config or gcfg
                if vocab_tokens is None and not vocab_file:
                    raise ValueError("GGUF file %r embeds no BERT vocabulary; pass vocab_file" % gguf_path)
            else:
                if not weights_path or not vocab_file:
                    raise ValueError(
                        "HipBertEmbeddings(model=%r) needs the model's local files (nothing is "
                        "downloaded): weights_path= + vocab_file= (or $%s + $%s), gguf_path= (or $%s), "
                        "or the model pulled into Ollama's local store. Missing: %s. Pass "
                        "synthetic=True for seeded random weights (tests/benchmarks only)."
                        % (model, ENV_WEIGHTS, ENV_VOCAB, ENV_GGUF,
                           ", ".join(n for n, v in (("weights", weights_path), ("vocab", vocab_file))
                                     if not v)))
                for what, p in (("weights", weights_path), ("vocab", vocab_file)):
                    if not os.path.isfile(p):
                        raise FileNotFoundError("%s file %r does not exist" % (what, p))
                config = config or DMETA_BASE
                weights = load_safetensors(weights_path, config)
        self.config = config
        self.max_length = min(int(max_length), config.max_positions)
        self.weights_path, self.vocab_file, self.gguf_path = weights_path, vocab_file, gguf_path
        self.encoder = Encoder(config, weights=weights, seed=seed, device=device)
        self.encoder.set_precision(PRECISIONS[precision])
        if vocab_file:  # C++ tokenizers of libmqhip.so
            self.tokenizer = NativeTokenizer.wordpiece(vocab_file, max_length=self.max_length)
        elif vocab_tokens is not None:
            self.tokenizer = NativeTokenizer.wordpiece_tokens(vocab_tokens, max_length=self.max_length)
        else:
            self.tokenizer = NativeTokenizer.char(config.vocab_size, max_length=self.max_length)

    # ---- batched core -------------------------------------------------------------
    def embed_array(self, texts):
        """texts -> float32 [len(texts), hidden]; length-sorted batches cut padding."""
        texts = list(texts)
        out = np.empty((len(texts), self.config.hidden), dtype=np.float32)
        if not texts:
            return out
        all_ids, all_mask = self.tokenizer(texts)
        lens = all_mask.sum(1)
        order = np.argsort(lens, kind="stable")
        for s in range(0, len(order), self.batch_size):
            idx = order[s:s + self.batch_size]
            L = int(lens[idx].max())
            out[idx] = self.encoder.embed(np.ascontiguousarray(all_ids[idx, :L]),
                                          np.ascontiguousarray(all_mask[idx, :L]))
        return out

    # ---- LangChain Embeddings interface ---------------------------------------------
    def embed_documents(self, texts):
        return self.embed_array(texts).tolist()

    def embed_query(self, text):
        return self.embed_array([text])[0].tolist()
