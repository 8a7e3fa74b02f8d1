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

Weights and vocabulary are never downloaded.  A real model needs BOTH a local
safetensors file and its WordPiece vocab, given as arguments or through the
environment (so the reference's constructor line stays unchanged):
    MQ_WEIGHTS_PATH=/models/dmeta.safetensors MQ_VOCAB_FILE=/models/vocab.txt
Seeded random weights with the char tokenizer (tests, benchmarks) must be asked for
explicitly with `synthetic=True`: a silently random encoder would hand the Retrieve
node semantically random documents.
"""
import os

import numpy as np

from .compat import EmbeddingsBase
from .config import BertConfig, DMETA_BASE
from .native import Encoder
from .tokenizer import NativeTokenizer
from .weights import load_safetensors

ENV_WEIGHTS = "MQ_WEIGHTS_PATH"
ENV_VOCAB = "MQ_VOCAB_FILE"


class HipBertEmbeddings(EmbeddingsBase):
    """BERT-base CLS embeddings computed by the hand-written HIP encoder.

    model:        kept for signature parity with OllamaEmbeddings (informational).
    weights_path: local safetensors with HF BERT names (default: $MQ_WEIGHTS_PATH).
    vocab_file:   local WordPiece vocab.txt (default: $MQ_VOCAB_FILE); required with
                  real weights - the char tokenizer would feed them meaningless ids.
    synthetic:    True = seeded random weights + the deterministic char tokenizer
                  (`seed`); the only way to get them.
    """

    def __init__(self, model="shaw/dmeta-embedding-zh", *, weights_path=None, vocab_file=None,
                 synthetic=False, config: BertConfig = DMETA_BASE, seed=0, device=0,
                 batch_size=256, max_length=512, **kwargs):
        self.model = model
        self.config = config
        self.device = device
        self.batch_size = int(batch_size)
        self.max_length = min(int(max_length), config.max_positions)
        self.synthetic = bool(synthetic)
        if self.synthetic:
            if weights_path or vocab_file:
                raise ValueError("synthetic=True takes no weights_path / vocab_file")
            weights = None
        else:
            weights_path = weights_path or os.environ.get(ENV_WEIGHTS)
            vocab_file = vocab_file or os.environ.get(ENV_VOCAB)
            if not weights_path or not vocab_file:
                raise ValueError(
                    "HipBertEmbeddings(model=%r) needs the model's local weights AND vocab "
                    "(weights_path=/vocab_file= or $%s/$%s; nothing is downloaded). Missing: %s. "
                    "Pass synthetic=True for seeded random weights (tests/benchmarks only)."
                    % (model, ENV_WEIGHTS, ENV_VOCAB,
                       ", ".join(n for n, v in (("weights", weights_path), ("vocab", vocab_file))
                                 if not v)))
            for what, p in (("weights", weights_path), ("vocab", vocab_file)):
                if not os.path.isfile(p):
                    raise FileNotFoundError("%s file %r does not exist" % (what, p))
            weights = load_safetensors(weights_path, config)
        self.weights_path, self.vocab_file = weights_path, vocab_file
        self.encoder = Encoder(config, weights=weights, seed=seed, device=device)
        if vocab_file:  # C++ tokenizers of libmqhip.so
            self.tokenizer = NativeTokenizer.wordpiece(vocab_file, max_length=self.max_length)
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
