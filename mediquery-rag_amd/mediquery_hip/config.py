"""Encoder architecture description shared by the host side and the C-ABI.

The reference embeds with Ollama's `shaw/dmeta-embedding-zh` (reference
src/medical_engine.py:43, src/ingest_medical.py:104): a BERT-base Chinese encoder
(12 layers, hidden 768, 12 heads, FFN 3072, vocab 21128, LayerNorm eps 1e-12),
CLS-pooled and L2-normalised by Ollama's /api/embed.
"""
from dataclasses import dataclass, asdict

GELU_ERF = 0    # HF BERT "gelu"  (exact erf form)  - the pinned variant
GELU_TANH = 1   # ggml / llama.cpp gelu (tanh approximation)
POOL_CLS = 0
POOL_MEAN = 1


@dataclass(frozen=True)
class BertConfig:
    vocab_size: int = 21128
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    max_positions: int = 1024
    type_vocab: int = 2
    ln_eps: float = 1e-12
    gelu: int = GELU_ERF
    pooling: int = POOL_CLS

    @property
    def head_dim(self):
        return self.hidden // self.heads

    def to_dict(self):
        return asdict(self)

    def flops_per_sequence(self, seq_len):
        """Algorithmic FLOPs of one forward:
        layers * [2*L*(4*d^2 + 2*d*ffn) + 4*L^2*d]."""
        d, f, L = self.hidden, self.ffn, seq_len
        return self.layers * (2 * L * (4 * d * d + 2 * d * f) + 4 * L * L * d)


DMETA_BASE = BertConfig()
