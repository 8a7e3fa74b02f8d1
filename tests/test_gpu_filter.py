"""Device-side filtered search (Chroma's `similarity_search(filter=...)` on the VectorStore
surface): the `where` mask is built on the device
from the store's metadata code columns (mq_mask_eval / mq_mask_combine) and the masked
search runs the int8 certified screen with masked rows absent, or gathers the allowed rows
on the device.  Every answer against a float64 torch reference over exactly the rows
`_match` admits (tie-group-aware check_topk), at 1M rows and at edge sizes."""
import numpy as np
import pytest

from mediquery_hip import _lib, synth
from mediquery_hip.native import FlatIndex, mask_combine, mask_eval, mask_eval_bits
from mediquery_hip.vectorstore import HipChroma, _match
from oracle.flat import check_topk

pytestmark = pytest.mark.gpu


def _check(store, rows64, q, k, where, metas):
    import torch
    dev = rows64.device
    allowed = np.array([r for r, m in enumerate(metas) if _match(m, where)], dtype=np.int64)
    got = store._search_rows(q, k, where)
    kk = min(k, len(allowed))
    assert len(got) == kk, (where, len(got), kk)
    if kk == 0:
        return
    al = torch.as_tensor(allowed, device=dev)
    ref = (rows64[al] @ torch.as_tensor(q, dtype=torch.float64, device=dev)).cpu().numpy()
    order = np.lexsort((allowed, -ref))
    ids = np.array([[r for r, _ in got]])
    sc = np.array([[c for _, c in got]], dtype=np.float32)
    pos = {int(r): j for j, r in enumerate(allowed)}
    fails = check_topk(ids, sc, None, kk,
                       ref_top=(ref[order][None, :kk + 1], allowed[order][None, :kk + 1]), n_rows=len(rows64),
                       ref_lookup=lambda b, rr: ref[[pos[int(x)] for x in rr]] if all(int(x) in pos for x in rr)
                       else np.full(len(rr), -np.inf))
    assert fails == [], (where, fails[:3])


def test_mask_kernels_match_numpy(require_gpu):
    """mq_mask_eval / mq_mask_combine against numpy, with ragged n (tail words)."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    for n in (1, 31, 33, 64, 1000, 4097):
        codes = rng.integers(-1, 5, n).astype(np.int32)
        lut = rng.integers(0, 2, 6).astype(np.uint8)
        lut2 = rng.integers(0, 2, 6).astype(np.uint8)
        want = lut[np.where(codes >= 0, codes, 5)].astype(bool)
        want2 = lut2[np.where(codes >= 0, codes, 5)].astype(bool)
        w = (n + 31) // 32
        bits = torch.empty(w, dtype=torch.int32, device=dev)
        tmp = torch.empty_like(bits)
        dc = torch.as_tensor(codes, device=dev)
        mask_combine(bits, None, _lib.MQ_MASK_SET)
        mask_eval(dc, torch.as_tensor(lut, device=dev), bits, _lib.MQ_MASK_AND)
        mask_eval(dc, torch.as_tensor(lut2, device=dev), tmp, _lib.MQ_MASK_SET)
        mask_combine(bits, tmp, _lib.MQ_MASK_OR)
        got = np.unpackbits(bits.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
        assert np.array_equal(got, want | want2), n
        mask_combine(bits, None, _lib.MQ_MASK_CLEAR)
        assert int(bits.abs().sum()) == 0
        # the by-value table (<= 256 entries) gives the same words
        mask_combine(bits, None, _lib.MQ_MASK_SET)
        mask_eval_bits(dc, lut, bits, _lib.MQ_MASK_AND)
        mask_eval(dc, torch.as_tensor(lut2, device=dev), tmp, _lib.MQ_MASK_SET)
        mask_combine(bits, tmp, _lib.MQ_MASK_OR)
        got = np.unpackbits(bits.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
        assert np.array_equal(got, want | want2), n


@pytest.fixture(scope="module")
def big_store(require_gpu):
    import torch
    dev = torch.device("cuda", 0)
    n = 1_000_000
    rows = synth.corpus_device(n, 768, dev)
    metas = [{"src": int(i % 7), "year": int((i * 7919) % 50)} for i in range(n)]
    metas[123456]["rare"] = "yes"
    metas[654321]["rare"] = "yes"
    store = HipChroma(dim=768, auto_persist=False)
    store.add_embeddings(rows.cpu().numpy(), ["d%d" % i for i in range(n)], metas, ["id%d" % i for i in range(n)])
    rows64 = torch.nn.functional.normalize(rows.double(), dim=1)
    del rows
    yield store, rows64, metas
    del rows64


@pytest.mark.parametrize("where,k", [
    ({"src": 3}, 5),
    ({"$or": [{"src": 1}, {"year": {"$gte": 40}}]}, 5),
    ({"year": {"$lt": 1}}, 16),
    ({"$and": [{"src": {"$in": [0, 2]}}, {"year": {"$ne": 7}}]}, 1),
    ({"src": 3}, 20),              # k > 16: the gather path
    ({"rare": "yes"}, 5),          # two rows: fewer than k, the gather path
    ({"src": 99}, 5),              # no row
    ({"missing_key": {"$ne": 1}}, 5),  # absent key: $ne admits every row
])
def test_filtered_search_1m_equals_fp64_over_allowed_rows(big_store, where, k):
    store, rows64, metas = big_store
    rng = np.random.default_rng(abs(hash(str(where))) % 2**31)
    for j in range(3):
        r = int(rng.integers(0, len(metas)))
        q = rows64[r].float().cpu().numpy() + 0.02 * rng.standard_normal(768).astype(np.float32)
        _check(store, rows64, q, k, where, metas)


def test_wide_filters_certify_on_the_int8_screen(big_store):
    """The masked int8 screen answers the wide filters itself (no gather)."""
    store, rows64, metas = big_store
    g0 = store._index.masked_gathers
    rng = np.random.default_rng(11)
    for j in range(20):
        q = rows64[int(rng.integers(0, len(metas)))].float().cpu().numpy()
        store._search_rows(q, 5, {"src": j % 7})
    assert store._index.masked_gathers - g0 <= 2


def test_batch_search_with_filter_matches_single(require_gpu, big_store):
    """similarity_search_batch(filter=) (one device mask, one batched masked search call)
    returns what the single-query path returns, query by query."""
    store, rows64, metas = big_store

    class _Emb:  # the batch path embeds through the store's function: vectors pass through
        def __init__(self, vecs):
            self.vecs = vecs

        def embed_documents(self, texts):
            return [self.vecs[int(t)] for t in texts]

    rng = np.random.default_rng(21)
    vecs = [rows64[int(rng.integers(0, len(metas)))].float().cpu().numpy() for _ in range(6)]
    store._embedding_function = _Emb(vecs)
    where = {"$or": [{"src": 2}, {"year": {"$lt": 5}}]}
    got = store.similarity_search_batch([str(j) for j in range(6)], k=5, filter=where)
    for j, docs in enumerate(got):
        want = [r for r, _ in store._search_rows(vecs[j], 5, where)]
        assert [int(d.id[2:]) for d in docs] == want
    store._embedding_function = None


def test_mask_by_value_table_past_64_entries(require_gpu):
    """Tables of 65..256 entries (keys with that many distinct values) by value: the words
    past the first select the right bits."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(9)
    for n_lut in (65, 130, 200, 256):
        n = 5000
        codes = rng.integers(-1, n_lut - 1, n).astype(np.int32)
        lut = rng.integers(0, 2, n_lut).astype(np.uint8)
        want = lut[np.where(codes >= 0, codes, n_lut - 1)].astype(bool)
        bits = torch.empty((n + 31) // 32, dtype=torch.int32, device=dev)
        mask_eval_bits(torch.as_tensor(codes, device=dev), lut, bits, _lib.MQ_MASK_SET)
        got = np.unpackbits(bits.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
        assert np.array_equal(got, want), n_lut



def _rows_fp64_topk(rows64, allowed, Q, k):
    import torch
    al = torch.as_tensor(allowed, device=rows64.device)
    ref = (torch.as_tensor(Q, dtype=torch.float64, device=rows64.device) @ rows64[al].T).cpu().numpy()
    return ref


@pytest.mark.parametrize("where,k", [
    ({"src": 3}, 5),                                   # 1/7 of the rows: masked K9t + certificate
    ({"$or": [{"src": 1}, {"year": {"$gte": 40}}]}, 16),
    ({"src": 3}, 20),                                  # k > 16: the masked streaming exact scan
    ({"rare": "yes"}, 5),                              # two rows: fewer than k, padded
])
def test_batched_filtered_search_256_equals_fp64(big_store, where, k):
    """256 queries with one filter in ONE masked call (the bf16 threshold
    scan with the row mask, fp32 re-rank, certificate; the masked streaming exact scan for
    what it does not certify and for k > 16): every query's answer against float64 over the
    allowed rows, tie-group aware."""
    import torch
    store, rows64, metas = big_store
    allowed = np.array([r for r, m in enumerate(metas) if _match(m, where)], dtype=np.int64)
    rng = np.random.default_rng(77)
    src = rng.integers(0, len(metas), 256)
    Q = rows64[torch.as_tensor(src, device=rows64.device)].float().cpu().numpy()
    Q += 0.02 * rng.standard_normal(Q.shape).astype(np.float32)
    bits = store._cols.dmask(where, store._device)
    s, i = store._index.search_masked(Q, k, bits)
    assert s.shape == (256, k) and i.shape == (256, k)
    kk = min(k, len(allowed))
    assert (i[:, kk:] == -1).all() and np.isneginf(s[:, kk:]).all()
    ref = _rows_fp64_topk(rows64, allowed, Q, k)
    pos = {int(r): j for j, r in enumerate(allowed)}
    for qi in range(256):
        order = np.lexsort((allowed, -ref[qi]))
        fails = check_topk(i[qi:qi + 1, :kk], s[qi:qi + 1, :kk], None, kk,
                           ref_top=(ref[qi][order][None, :kk + 1], allowed[order][None, :kk + 1]),
                           n_rows=len(rows64),
                           ref_lookup=lambda b, rr, qi=qi: ref[qi][[pos[int(x)] for x in rr]]
                           if all(int(x) in pos for x in rr) else np.full(len(rr), -np.inf))
        assert fails == [], (where, qi, fails[:3])


def test_batched_filtered_search_cost_vs_unfiltered(big_store):
    """The 256-query filtered batch costs about what the unfiltered batch costs (the mask is
    1/6144 of the scan's bytes): measured and printed; asserted within 3x (VERDICT r5 #9's
    target is 2x, reported by tools/filter_latency.py on a quiet box)."""
    import time
    import torch
    store, rows64, metas = big_store
    rng = np.random.default_rng(5)
    Q = rows64[torch.as_tensor(rng.integers(0, len(metas), 256), device=rows64.device)].float().cpu().numpy()
    where = {"src": {"$ne": 3}}
    bits = store._cols.dmask(where, store._device)
    ix = store._index
    for _ in range(2):
        ix.search(Q, 5)
        ix.search_masked(Q, 5, bits)
    t0 = time.perf_counter()
    for _ in range(5):
        ix.search(Q, 5)
    t_plain = (time.perf_counter() - t0) / 5
    g0 = ix.masked_gathers
    t0 = time.perf_counter()
    for _ in range(5):
        ix.search_masked(Q, 5, bits)
    t_mask = (time.perf_counter() - t0) / 5
    print("batch256_unfiltered_ms %.3f filtered_ms %.3f ratio %.2f uncertified %d"
          % (t_plain * 1e3, t_mask * 1e3, t_mask / t_plain, ix.masked_gathers - g0))
    assert t_mask <= 3.0 * t_plain, (t_mask, t_plain)


def test_selective_filter_fewer_than_k_rows_certifies(big_store):
    """a filter admitting fewer than k rows (n >= 65536) is answered by the int8
    screen itself (tau = -inf: every allowed row survived) - no uncertified fallback."""
    store, rows64, metas = big_store
    g0 = store._index.masked_gathers
    for r in (123456, 654321, 7):
        q = rows64[r].float().cpu().numpy()
        got = store._search_rows(q, 5, {"rare": "yes"})
        assert sorted(x for x, _ in got) == [123456, 654321]
    assert store._index.masked_gathers == g0


def test_mask_on_another_device_or_short_is_rejected(big_store):
    """The masked search checks the mask's device, width and length before any kernel runs."""
    import torch
    store, rows64, metas = big_store
    q = rows64[0].float().cpu().numpy()
    short = torch.zeros(10, dtype=torch.int32, device="cuda:0")
    with pytest.raises(ValueError, match="ceil"):
        store._index.search_masked(q, 5, short)
    with pytest.raises(ValueError):
        store._index.search_masked(q, 5, torch.zeros((len(metas) + 31) // 32, dtype=torch.int64, device="cuda:0"))
    with pytest.raises(ValueError):
        store._index.search_masked(q, 5, torch.zeros((len(metas) + 31) // 32, dtype=torch.int32))
