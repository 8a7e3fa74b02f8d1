"""ORACLE (test infrastructure only) - CPU restatement of the query/document encoder.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.

What it restates: the embedding step of the reference's retrieval path,
`OllamaEmbeddings("shaw/dmeta-embedding-zh").embed_query/embed_documents`
(reference src/medical_engine.py:43, src/ingest_medical.py:104, used by
similarity_search at src/agents/nodes.py:93): BERT-base forward -> CLS pool -> L2
normalise.  The Ollama/ggml implementation is third-party and
absent, so this restatement follows the published BERT algorithm and is pinned against
`transformers.BertModel` (5.15.0, fp32, eager attention, erf GELU) on seeded weights by
tests/golden/encoder_golden.npz (script: tests/golden/make_encoder_golden.py).
Parity vs the real dmeta weights / Ollama output: UNPINNED (no weights offline).

Written as explicit torch-CPU fp32 ops (not a call into transformers) so it also serves
as the CPU baseline timed beside the GPU in bench.py.
"""
import math

import numpy as np
import torch

GELU_ERF, GELU_TANH = 0, 1
POOL_CLS, POOL_MEAN = 0, 1


class OracleEncoder:
    def __init__(self, cfg, state_dict):
        self.cfg = cfg
        t = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float32)
        sd = {k: t(v) for k, v in state_dict.items()}
        self.word = sd["embeddings.word_embeddings.weight"]
        self.pos = sd["embeddings.position_embeddings.weight"]
        self.typ = sd["embeddings.token_type_embeddings.weight"]
        self.eln = (sd["embeddings.LayerNorm.weight"], sd["embeddings.LayerNorm.bias"])
        self.layers = []
        for l in range(cfg.layers):
            p = "encoder.layer.%d." % l
            g = lambda n: sd[p + n]
            self.layers.append(dict(
                wq=g("attention.self.query.weight"), bq=g("attention.self.query.bias"),
                wk=g("attention.self.key.weight"), bk=g("attention.self.key.bias"),
                wv=g("attention.self.value.weight"), bv=g("attention.self.value.bias"),
                wo=g("attention.output.dense.weight"), bo=g("attention.output.dense.bias"),
                ln1=(g("attention.output.LayerNorm.weight"), g("attention.output.LayerNorm.bias")),
                w1=g("intermediate.dense.weight"), b1=g("intermediate.dense.bias"),
                w2=g("output.dense.weight"), b2=g("output.dense.bias"),
                ln2=(g("output.LayerNorm.weight"), g("output.LayerNorm.bias"))))

    def _ln(self, x, gb):
        mu = x.mean(-1, keepdim=True)
        var = ((x - mu) ** 2).mean(-1, keepdim=True)
        return (x - mu) / torch.sqrt(var + self.cfg.ln_eps) * gb[0] + gb[1]

    def _gelu(self, x):
        if self.cfg.gelu == GELU_TANH:
            return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x ** 3)))
        return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))

    @torch.no_grad()
    def hidden_states(self, ids, mask):
        """ids, mask: int arrays [B, L] -> last hidden state [B, L, H] (fp32)."""
        cfg = self.cfg
        ids = torch.as_tensor(np.asarray(ids), dtype=torch.long)
        keep = torch.as_tensor(np.asarray(mask), dtype=torch.bool)
        B, L = ids.shape
        H, nh = cfg.hidden, cfg.heads
        dh = H // nh
        x = self.word[ids] + self.pos[:L].unsqueeze(0) + self.typ[0]
        x = self._ln(x, self.eln)
        bias = torch.zeros(B, 1, 1, L)
        bias.masked_fill_(~keep[:, None, None, :], float("-inf"))
        for w in self.layers:
            heads = lambda y: y.view(B, L, nh, dh).transpose(1, 2)
            q = heads(x @ w["wq"].T + w["bq"])
            k = heads(x @ w["wk"].T + w["bk"])
            v = heads(x @ w["wv"].T + w["bv"])
            s = (q @ k.transpose(-1, -2)) / math.sqrt(dh) + bias
            p = torch.softmax(s, dim=-1)
            ctx = (p @ v).transpose(1, 2).reshape(B, L, H)
            x = self._ln(x + ctx @ w["wo"].T + w["bo"], w["ln1"])
            h = self._gelu(x @ w["w1"].T + w["b1"])
            x = self._ln(x + h @ w["w2"].T + w["b2"], w["ln2"])
        return x

    def embed(self, ids, mask):
        """-> unit-norm embeddings [B, H] as float32 numpy (CLS or mean pooling)."""
        h = self.hidden_states(ids, mask)
        if self.cfg.pooling == POOL_MEAN:
            m = torch.as_tensor(np.asarray(mask), dtype=torch.float32).unsqueeze(-1)
            e = (h * m).sum(1) / m.sum(1).clamp_min(1.0)
        else:
            e = h[:, 0]
        e = e / e.norm(dim=-1, keepdim=True).clamp_min(1e-12)
        return e.numpy().astype(np.float32)
