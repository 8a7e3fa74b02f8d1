"""GPU parity of the HIP BERT encoder (K1..K7) through the C ABI: against the
transformers golden vectors and against the torch-CPU oracle on ragged shapes.
Tolerance: |emb - ref| <= 1e-4 per element and cos >= 1 - 1e-5."""
import os

import numpy as np
import pytest

from mediquery_hip import _lib
from mediquery_hip.config import BertConfig, DMETA_BASE, GELU_TANH, POOL_MEAN
from mediquery_hip.native import Encoder
from mediquery_hip.weights import synthetic_state_dict
from oracle.encoder import OracleEncoder

pytestmark = pytest.mark.gpu
ATOL = 1e-4


def _close(got, ref):
    np.testing.assert_allclose(got, ref, atol=ATOL, rtol=0)
    cos = (got * ref).sum(1) / np.linalg.norm(got, axis=1) / np.linalg.norm(ref, axis=1)
    assert cos.min() >= 1 - 1e-5, cos.min()


@pytest.fixture(scope="module")
def g(golden):
    return np.load(os.path.join(golden, "encoder_golden.npz"))


@pytest.mark.parametrize("prec", [_lib.MQ_DTYPE_F32, _lib.MQ_DTYPE_F32X6])
@pytest.mark.parametrize("case,cfg", [
    ("tiny_a", BertConfig(layers=2)),
    ("tiny_b", BertConfig(layers=2)),
    ("tiny_b_mean", BertConfig(layers=2, pooling=POOL_MEAN)),
    ("tiny_tanh", BertConfig(layers=2, gelu=GELU_TANH)),
    ("base", DMETA_BASE),
])
def test_golden(require_gpu, g, case, cfg, prec):
    src = case.replace("_mean", "")
    enc = Encoder(cfg)
    enc.set_precision(prec)
    _close(enc.embed(g[src + "_ids"], g[src + "_mask"]), g[case + "_emb"])


@pytest.mark.parametrize("B,L,layers,pool,gelu", [
    (9, 33, 3, POOL_MEAN, None),    # 297 rows: ragged 128-row tiles, the last layer's LN2 on its own
    (9, 33, 3, None, GELU_TANH),    # CLS pooling: the cls-only last layer's K/V GEMM normalises on load
    (5, 200, 2, None, None),        # 1000 rows, long sequences
    (300, 3, 4, POOL_MEAN, None),   # many short sequences
])
def test_layernorm_on_load_vs_oracle(require_gpu, B, L, layers, pool, gelu):
    """LayerNorm deferred into the consuming GEMM (MQ_ENC_OPT_LN_ON_LOAD = 1; measured
    slower, off by default): out-proj / FFN-down leave per-row partials, FFN-up / the next
    QKV normalise A while staging and their column-0 tiles write the residual x.  Against
    the oracle, and against the LayerNorm-launch path of the same encoder within 1e-5 (two
    summation orders of the same statistics)."""
    kw = {"layers": layers}
    if pool is not None:
        kw["pooling"] = pool
    if gelu is not None:
        kw["gelu"] = gelu
    cfg = BertConfig(**kw)
    rng = np.random.default_rng(B * 7 + L)
    ids = rng.integers(0, cfg.vocab_size, (B, L)).astype(np.int32)
    mask = np.ones((B, L), np.int32)
    for b in range(0, B, 2):
        n = int(rng.integers(1, L + 1))
        mask[b, n:] = 0
    ref = OracleEncoder(cfg, synthetic_state_dict(cfg, 0)).embed(ids, mask)
    enc = Encoder(cfg)
    assert enc.get_option("ln_on_load") == 0
    base = enc.embed(ids, mask)
    enc.set_option("ln_on_load", 1)
    got = enc.embed(ids, mask)
    _close(got, ref)
    np.testing.assert_allclose(got, base, atol=1e-5, rtol=0)


@pytest.mark.parametrize("prec", [_lib.MQ_DTYPE_F32, _lib.MQ_DTYPE_F32X6])
def test_headline_shape_vs_oracle(require_gpu, prec):
    """The exact encoder shape bench.py times (BASELINE config 3; the query embedding of
    src/medical_engine.py:43): 12-layer dmeta-base, B = 256, L = 32, the bench's token ids -
    the batched tiled path (not the few-row one) at full depth, host and device entry
    points, against the oracle."""
    import torch
    from mediquery_hip import synth
    ids, mask = synth.token_batch(256, 32)
    ref = OracleEncoder(DMETA_BASE, synthetic_state_dict(DMETA_BASE, 0)).embed(ids, mask)
    enc = Encoder(DMETA_BASE)
    enc.set_precision(prec)
    _close(enc.embed(ids, mask), ref)
    dev = torch.device("cuda", 0)
    out = torch.empty((256, 768), dtype=torch.float32, device=dev)
    enc.embed_device(torch.from_numpy(ids).to(dev), torch.from_numpy(mask).to(dev), out)
    torch.cuda.synchronize()
    _close(out.cpu().numpy(), ref)


@pytest.mark.parametrize("B,L,ragged", [(1, 1, False), (1, 2, False), (3, 31, True), (5, 33, True),
                                        (2, 64, False), (4, 65, True), (9, 130, True),
                                        (2, 300, True), (1, 512, False), (70, 32, False)])
@pytest.mark.parametrize("prec", [_lib.MQ_DTYPE_F32, _lib.MQ_DTYPE_F32X6])
def test_shapes_vs_oracle(require_gpu, B, L, ragged, prec):
    cfg = BertConfig(layers=2)
    rng = np.random.default_rng(B * 1000 + L)
    ids = rng.integers(0, cfg.vocab_size, (B, L)).astype(np.int32)
    mask = np.ones((B, L), np.int32)
    if ragged:
        for b in range(B):
            n = int(rng.integers(1, L + 1))
            mask[b, n:] = 0
            ids[b, n:] = 0
    ref = OracleEncoder(cfg, synthetic_state_dict(cfg, 0)).embed(ids, mask)
    enc = Encoder(cfg)
    enc.set_precision(prec)
    _close(enc.embed(ids, mask), ref)


@pytest.mark.parametrize("B,L,lens,kw", [
    (1, 256, [256], {"pooling": POOL_MEAN}),          # 96 triples -> 8 waves per triple
    (3, 200, [200, 3, 97], {"pooling": POOL_MEAN}),   # 8-way, whole key tiles fully masked
    (6, 130, [130, 1, 64, 65, 100, 129], {}),         # 4 key tiles -> 4 waves per triple
    (16, 96, [96] * 16, {"pooling": POOL_MEAN}),      # 576 triples -> 2 waves per triple
    (1, 512, [300], {"gelu": GELU_TANH}),
])
def test_key_split_attention_vs_oracle(require_gpu, B, L, lens, kw):
    """Few (sequence, head, query tile) triples with many keys (long single queries, the
    CLS-only last layer) split the key tiles over 2 / 4 / 8 waves whose softmax partials
    are merged in LDS (attention_kernel<NS>): against the oracle, ragged lengths."""
    cfg = BertConfig(**{"layers": 2, **kw})
    rng = np.random.default_rng(B * 7 + L)
    ids = rng.integers(106, cfg.vocab_size, (B, L)).astype(np.int32)
    mask = np.zeros((B, L), np.int32)
    for b, n in enumerate(lens):
        mask[b, :n] = 1
    ref = OracleEncoder(cfg, synthetic_state_dict(cfg, 0)).embed(ids, mask)
    _close(Encoder(cfg).embed(ids, mask), ref)


@pytest.mark.parametrize("B,L,kw", [
    (1, 32, {}), (1, 64, {}), (2, 32, {}), (3, 7, {}), (1, 1, {"layers": 1}),
    (1, 5, {"pooling": POOL_MEAN}), (2, 16, {"pooling": POOL_MEAN}), (1, 32, {"gelu": GELU_TANH}),
    (4, 16, {"layers": 3}),
    (2, 20, {"hidden": 256, "heads": 4, "ffn": 512}), (1, 33, {"hidden": 512, "heads": 8, "ffn": 2048}),
    (1, 24, {"hidden": 1024, "heads": 16, "ffn": 4096}),
])
def test_few_row_path_vs_oracle(require_gpu, B, L, kw):
    """B * L <= 64 token rows take the few-row forward (K2r: one 16x16 output tile per
    1024-thread workgroup over the full depth, LayerNorm applied while loading the next
    GEMM's rows, ln_pool at the end); ragged masks on every sequence after the first."""
    cfg = BertConfig(**{"layers": 2, **kw})
    rng = np.random.default_rng(B * 100 + L)
    ids = rng.integers(106, cfg.vocab_size, (B, L)).astype(np.int32)
    mask = np.ones((B, L), np.int32)
    for b in range(1, B):
        mask[b, int(rng.integers(1, L + 1)):] = 0
    ref = OracleEncoder(cfg, synthetic_state_dict(cfg, 0)).embed(ids, mask)
    enc = Encoder(cfg)
    _close(enc.embed(ids, mask), ref)


def test_few_row_path_matches_tiled_path(require_gpu):
    """The same sequences alone (few-row forward) and inside a 96-sequence batch (tiled
    GEMMs): equal within fp32 reassociation."""
    cfg = BertConfig(layers=3)
    enc = Encoder(cfg)
    rng = np.random.default_rng(11)
    ids = rng.integers(106, cfg.vocab_size, (96, 32)).astype(np.int32)
    mask = np.ones_like(ids)
    mask[1::3, 20:] = 0
    batch = enc.embed(ids, mask)
    for b in (0, 1, 50, 95):
        np.testing.assert_allclose(enc.embed(ids[b:b + 1], mask[b:b + 1])[0], batch[b], atol=1e-6)
    np.testing.assert_allclose(enc.embed(ids[4:6], mask[4:6]), batch[4:6], atol=1e-6)


def test_device_path_and_batch_invariance(require_gpu):
    import torch
    cfg = BertConfig(layers=2)
    enc = Encoder(cfg)
    rng = np.random.default_rng(5)
    ids = rng.integers(106, cfg.vocab_size, (300, 32)).astype(np.int32)
    mask = np.ones_like(ids)
    host = enc.embed(ids, mask)
    dev = torch.device("cuda", 0)
    out = torch.empty((300, 768), dtype=torch.float32, device=dev)
    enc.embed_device(torch.from_numpy(ids).to(dev), torch.from_numpy(mask).to(dev), out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), host)
    # a sequence's embedding does not depend on what else is in the batch
    np.testing.assert_allclose(enc.embed(ids[7:8], mask[7:8])[0], host[7], atol=1e-6)


@pytest.mark.parametrize("prec", [_lib.MQ_DTYPE_F32, _lib.MQ_DTYPE_F32X6])
def test_graph_replay_bit_identical(require_gpu, prec):
    """Captured-hipGraph forwards equal eager forwards bit for bit, across shape
    changes (more shapes than the graph cache holds), buffer growth, precision
    switches, timing on/off, host and device paths."""
    import torch
    cfg = BertConfig(layers=2)
    enc = Encoder(cfg)
    enc.set_precision(prec)
    rng = np.random.default_rng(8)
    shapes = [(1, 32), (4, 17), (1, 32), (2, 8), (3, 5), (5, 9), (6, 3), (7, 2), (64, 32), (1, 32), (4, 17)]
    dev = torch.device("cuda", 0)
    for B, L in shapes:
        ids = rng.integers(106, cfg.vocab_size, (B, L)).astype(np.int32)
        mask = np.ones_like(ids)
        mask[0, L // 2 + 1:] = 0
        enc.set_graphs(False)
        eager = enc.embed(ids, mask)
        enc.set_graphs(True)
        np.testing.assert_array_equal(enc.embed(ids, mask), eager)
        np.testing.assert_array_equal(enc.embed(ids, mask), eager)   # replay
        out = torch.empty((B, 768), dtype=torch.float32, device=dev)
        enc.embed_device(torch.from_numpy(ids).to(dev), torch.from_numpy(mask).to(dev), out)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), eager)
    enc.set_timing(True)       # timing forces eager launches; same numbers
    ids = rng.integers(106, cfg.vocab_size, (2, 11)).astype(np.int32)
    a = enc.embed(ids, np.ones_like(ids))
    enc.set_timing(False)
    np.testing.assert_array_equal(enc.embed(ids, np.ones_like(ids)), a)


def test_errors(require_gpu):
    enc = Encoder(BertConfig(layers=1, max_positions=64))
    with pytest.raises(_lib.MQError, match="max_positions"):
        enc.embed(np.zeros((1, 65), np.int32), np.ones((1, 65), np.int32))
    assert enc.embed(np.zeros((0, 8), np.int32), np.zeros((0, 8), np.int32)).shape == (0, 768)


@pytest.mark.parametrize("name,value,B,L", [
    ("rows_max", 0, 1, 32),        # one query through the tiled / split-K path
    ("rows_max", 256, 2, 100),     # 200 token rows through the few-row forward
    ("rows_splits", 1, 1, 32), ("rows_splits", 3, 2, 20), ("rows_splits", 4, 1, 48),
    ("splitk_max", 4, 1, 32), ("splitk_max", 64, 1, 40),   # (with rows_max 0 below)
    ("ln_rows_per_wave", 1, 9, 33), ("ln_rows_per_wave", 2, 9, 33),
    ("fuse_attn_oproj", 0, 1, 32), ("fuse_attn_oproj", 0, 2, 17),
    ("fused_ln", 1, 70, 32), ("fused_ln", 1, 9, 130),
    ("splitk_tiles", 64, 1, 256), ("splitk_tiles", 4096, 1, 100), ("splitk_tiles", 16, 2, 48),
    ("ln_on_load", 1, 70, 32), ("ln_on_load", 1, 9, 130),
    ("resident_layers", 0, 1, 32), ("resident_layers", 1, 2, 20), ("resident_layers", 12, 1, 48),
])
def test_options_non_default_values_vs_oracle(require_gpu, name, value, B, L):
    """Every non-default value of the explicit tuning options (mq_encoder_set_option,
    which replaced the old environment knobs) keeps the forward within the parity
    tolerance of the oracle; the option reads back, bad values raise."""
    cfg = BertConfig(layers=2)
    rng = np.random.default_rng(L)
    ids = rng.integers(0, cfg.vocab_size, (B, L)).astype(np.int32)
    mask = np.ones((B, L), np.int32)
    mask[-1, L // 2:] = 0
    ref = OracleEncoder(cfg, synthetic_state_dict(cfg, 0)).embed(ids, mask)
    enc = Encoder(cfg)
    if name in ("splitk_max", "splitk_tiles"):
        enc.set_option("rows_max", 0)
    if name == "ln_rows_per_wave":  # (the LayerNorm kernel runs on the unfused path)
        enc.set_option("fused_ln", 0)
    enc.set_option(name, value)
    assert enc.get_option(name) == value
    _close(enc.embed(ids, mask), ref)
    for bad in (-1, 1 << 20):
        with pytest.raises(_lib.MQError):
            enc.set_option(name, bad)


def test_resident_layers_changes_only_the_cache_policy(require_gpu):
    """MQ_ENC_OPT_RESIDENT_LAYERS picks which few-row layers load their weights
    non-temporally: the forward is bit-identical for every value (fused and two-launch
    attention paths, the CLS-only last layer)."""
    cfg = BertConfig(layers=4, max_positions=128)
    rng = np.random.default_rng(11)
    enc = Encoder(cfg)
    for B, L, fuse in ((1, 32, 1), (2, 17, 0)):
        ids = rng.integers(0, cfg.vocab_size, (B, L)).astype(np.int32)
        mask = np.ones((B, L), np.int32)
        mask[-1, L // 2:] = 0
        enc.set_option("fuse_attn_oproj", fuse)
        outs = []
        for v in (0, 2, 8):
            enc.set_option("resident_layers", v)
            outs.append(enc.embed(ids, mask))
        assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])


@pytest.mark.parametrize("B,L,layers,pool", [
    (256, 32, 12, None),           # the bench shape: every batched GEMM on K2p
    (9, 33, 3, POOL_MEAN),         # 297 rows: under-fills the chip -> exact-f32 tiles in both modes
    (9, 33, 3, None),              # CLS-only last layer (K2p tiles are covered shape by shape
    (300, 3, 2, None),             # in test_gpu_gemm_x6p.py, ragged M / N included)
])
def test_x6_presplit_bit_identical(require_gpu, B, L, layers, pool):
    """Split-f32 precision: the batched GEMMs on the pre-split W3 weights (K2p, default)
    give the same bits as the split-f32 tiles that re-split both operands (x6_presplit =
    0) - same planes, same six products in the same order - and match the oracle."""
    kw = {"layers": layers}
    if pool is not None:
        kw["pooling"] = pool
    cfg = BertConfig(**kw) if layers != 12 else DMETA_BASE
    rng = np.random.default_rng(B * 5 + L)
    ids = rng.integers(0, cfg.vocab_size, (B, L)).astype(np.int32)
    mask = np.ones((B, L), np.int32)
    for b in range(0, B, 3):
        mask[b, int(rng.integers(1, L + 1)):] = 0
    enc = Encoder(cfg)
    enc.set_precision(_lib.MQ_DTYPE_F32X6)
    assert enc.get_option("x6_presplit") == 1
    got = enc.embed(ids, mask)
    enc.set_option("x6_presplit", 0)
    old = enc.embed(ids, mask)
    assert np.array_equal(got, old), float(np.abs(got - old).max())
    ref = OracleEncoder(cfg, synthetic_state_dict(cfg, 0)).embed(ids, mask)
    _close(got, ref)


@pytest.mark.parametrize("B,L,layers,pool,gelu", [
    (1, 32, 12, None, None),        # the single-query bench shape (frag16 Q/K/V^T, CLS-only last layer)
    (1, 20, 3, POOL_MEAN, None),    # L % 16 != 0: row-major QKV for the fused attention
    (2, 32, 2, None, GELU_TANH),    # two sequences, both 16-row aligned
    (3, 21, 2, POOL_MEAN, None),    # ragged rows (63): the last 16-row block partly past M
])
def test_few_row_plane_merge_bit_identical(require_gpu, B, L, layers, pool, gelu):
    """Few-row forward (r6): FFN-down's two K splits and the fused attention's two head
    groups add into ONE zeroed plane by atomic adds (rows_planes = 0, default) - two addends
    per element, so bitwise the p0 + p1 the consumer summed from two planes (rows_planes =
    1) - run to run and against the oracle."""
    kw = {"layers": layers}
    if pool is not None:
        kw["pooling"] = pool
    if gelu is not None:
        kw["gelu"] = gelu
    cfg = BertConfig(**kw) if layers != 12 else DMETA_BASE
    rng = np.random.default_rng(B * 13 + L)
    ids = rng.integers(0, cfg.vocab_size, (B, L)).astype(np.int32)
    mask = np.ones((B, L), np.int32)
    if B > 1:
        mask[0, int(rng.integers(1, L)):] = 0
    enc = Encoder(cfg)
    assert enc.get_option("rows_planes") == 0
    got = enc.embed(ids, mask)
    again = enc.embed(ids, mask)
    enc.set_option("rows_planes", 1)
    planes = enc.embed(ids, mask)
    assert np.array_equal(got, again)
    assert np.array_equal(got, planes), float(np.abs(got - planes).max())
    _close(got, OracleEncoder(cfg, synthetic_state_dict(cfg, 0)).embed(ids, mask))
