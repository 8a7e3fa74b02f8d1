"""GPU parity of K9t, the bf16 threshold scan (thresh.hip) that produces the candidates of
batched bf16 searches over >= 65536 rows: the certified screen's first tier
(MQ_DTYPE_F32_SCREEN) and BASELINE config 5's coarse scan (MQ_DTYPE_BF16).  Exact mode
must return the oracle's top-k (tie-group aware) whichever candidate scan ran; the
approximate mode must agree with the tiled candidate scan it replaces."""
import numpy as np
import pytest

from mediquery_hip import _lib, synth
from mediquery_hip.native import FlatIndex
from oracle.flat import check_topk, exact_scores

pytestmark = pytest.mark.gpu


def _index(rows, prec):
    ix = FlatIndex(dim=rows.shape[1])
    ix.add(rows)
    ix.set_precision(prec)
    return ix


@pytest.mark.parametrize("n,nq,k", [(70001, 65, 5), (70001, 256, 5), (100000, 300, 50),
                                    (65536, 512, 16), (131075, 257, 1)])
def test_screen_with_threshold_scan_is_exact(require_gpu, n, nq, k):
    """Ragged last block (70001, 131075 rows), one and several 256-query groups, ragged
    query groups (65, 257, 300): exact top-k = oracle; same ids with the tiled scan."""
    c = synth.corpus(n, 768, seed=n, clustered=True)
    q, planted = synth.queries(nq, c, seed=nq)
    ref = exact_scores(q, c)
    ix = _index(c, _lib.MQ_DTYPE_F32_SCREEN)
    s, i = ix.search(q, k)
    assert check_topk(i, s, ref, k) == []
    pl = planted >= 0
    assert (i[pl, 0] == planted[pl]).all()
    ix.set_threshold_scan(False)
    s2, i2 = ix.search(q, k)
    assert check_topk(i2, s2, ref, k) == []
    np.testing.assert_allclose(s, s2, atol=1e-6)


@pytest.mark.parametrize("dim", [256, 512])
def test_threshold_scan_other_widths(require_gpu, dim):
    c = synth.corpus(80000, dim, seed=dim, clustered=True)
    q, planted = synth.queries(200, c, seed=1)
    ref = exact_scores(q, c)
    ix = _index(c, _lib.MQ_DTYPE_F32_SCREEN)
    s, i = ix.search(q, 5)
    assert check_topk(i, s, ref, 5) == []
    ix.set_precision(_lib.MQ_DTYPE_BF16)
    s, i = ix.search(q, 10)
    assert check_topk(i, s, ref, 10) == []


def test_config5_coarse_candidates_match_tiled_scan(require_gpu):
    """MQ_DTYPE_BF16, k = 50 (64 coarse candidates): the threshold scan and the tiled
    scan pick the same bf16 top-64 up to bf16-score ties at the 64th place (the two
    kernels sum the k-dimension in different orders), so the re-ranked top-50 agree on
    nearly every query, and recall vs exact fp32 stays >= 0.98."""
    n, nq, k = 120000, 256, 50
    c = synth.corpus(n, 768, seed=7, clustered=True)
    q, planted = synth.queries(nq, c, seed=7)
    ix = _index(c, _lib.MQ_DTYPE_BF16)
    s, i = ix.search(q, k)
    ix.set_threshold_scan(False)
    s2, i2 = ix.search(q, k)
    same = sum(set(a.tolist()) == set(b.tolist()) for a, b in zip(i, i2))
    assert same >= 0.99 * nq, same
    ref = exact_scores(q, c)
    got = np.take_along_axis(ref, i, axis=1)
    np.testing.assert_allclose(s, got, rtol=0, atol=1e-5)
    exact = np.argsort(-ref, axis=1, kind="stable")[:, :k]
    hits = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(i, exact))
    assert hits / (nq * k) >= 0.98
    pl = planted >= 0
    assert (i[pl, 0] == planted[pl]).all()


def test_threshold_scan_survivor_overflow_passes_down(require_gpu):
    """5000 copies of one direction: query 0 has more survivors than the 4096 kept, so
    its candidate set is incomplete; the select marks the bound +inf, the certificate
    fails and the query is re-run one tier down.  Results stay exact for every query."""
    c = synth.corpus(90000, 768, seed=3, clustered=True)
    q, _ = synth.queries(128, c, seed=3)
    c[20000:25000] = q[0]  # exact duplicates: 5000 rows tie at the top for query 0
    ix = _index(c, _lib.MQ_DTYPE_F32_SCREEN)
    s, i = ix.search(q, 5)
    assert ix.screen_passdowns + ix.screen_fallbacks >= 1
    assert i[0].tolist() == [20000, 20001, 20002, 20003, 20004]
    assert check_topk(i, s, exact_scores(q, c), 5) == []


def test_threshold_scan_full_size_planted(require_gpu):
    """BASELINE config 3 size through the default screen (the bench's search): 1M x 768,
    B = 256, k = 5 - planted queries find their rows and nothing falls back."""
    import torch
    dev = torch.device("cuda", 0)
    rows = synth.corpus_device(1_000_000, 768, dev)
    q, planted = synth.queries_device(256, rows)
    ix = FlatIndex(dim=768, capacity=1_000_000)
    ix.add_device(rows)
    ix.set_precision(_lib.MQ_DTYPE_F32_SCREEN)
    s = torch.empty((256, 5), dtype=torch.float32, device=dev)
    i = torch.empty((256, 5), dtype=torch.int64, device=dev)
    ix.search_device(q, 5, s, i)
    torch.cuda.synchronize()
    pl = planted >= 0
    assert bool((i[pl, 0] == planted[pl]).all())
    ix.set_precision(_lib.MQ_DTYPE_F32)
    s2, i2 = torch.empty_like(s), torch.empty_like(i)
    ix.search_device(q, 5, s2, i2)
    torch.cuda.synchronize()
    assert bool((i == i2).all())
    assert ix.screen_fallbacks == 0


@pytest.mark.parametrize("clustered", [False, True])
def test_bf16_mode_random_queries_k50_never_pad(require_gpu, clustered):
    """MQ_DTYPE_BF16 has no certificate: its threshold scan keeps tau at the 24th sample
    list maximum (~384 survivors) and re-runs any query left with fewer than kc (64) on
    the tiled scan - random, non-planted queries at k = 50 never come back with -1 ids or
    -inf scores (with tau at the 8th maximum ~1% of such queries fell short of 64)."""
    c = synth.corpus(200000, 768, seed=11, clustered=clustered)
    rng = np.random.default_rng(5)
    q = rng.standard_normal((512, 768)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    ix = _index(c, _lib.MQ_DTYPE_BF16)
    s, i = ix.search(q, 50)
    assert (i >= 0).all() and np.isfinite(s).all()
    assert all(len(set(r.tolist())) == 50 for r in i)
    ref = exact_scores(q, c)
    np.testing.assert_allclose(s, np.take_along_axis(ref, i, axis=1), rtol=0, atol=1e-5)
    assert (np.diff(s, axis=1) <= 0).all()
    exact = np.argsort(-ref, axis=1, kind="stable")[:, :50]
    hits = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(i, exact))
    assert hits / (512 * 50) >= 0.98


def test_bf16_mode_survivor_overflow_reruns_on_tiled_scan(require_gpu):
    """5000 exact duplicates of query 0's direction: more survivors than kTsCap, so the
    threshold scan's kept set depends on arrival order; the query is listed by the select
    and re-run on the tiled scan - deterministic ids: the 50 lowest duplicate rows."""
    c = synth.corpus(90000, 768, seed=3, clustered=True)
    q, _ = synth.queries(128, c, seed=3)
    c[20000:25000] = q[0]
    ix = _index(c, _lib.MQ_DTYPE_BF16)
    r0 = ix.rescans
    s, i = ix.search(q, 50)
    assert ix.rescans >= r0 + 1  # the re-run (plus the tiled scan's own 64-list re-scan on 5000 ties)
    assert i[0].tolist() == list(range(20000, 20050))
    assert (i >= 0).all()
    s2, i2 = ix.search(q, 50)  # deterministic across calls
    np.testing.assert_array_equal(i, i2)


def test_config5_full_size_recall(require_gpu):
    """BASELINE config 5 at its size: 1M x 768 bf16 shadow, batch 256, k = 50 - bf16 MFMA
    coarse top-64 + exact fp32 re-rank: recall@50 >= 0.98 against the direct exact fp32
    scan, returned scores exact fp32 dots of the returned rows (within two dot orders)."""
    import torch
    dev = torch.device("cuda", 0)
    rows = synth.corpus_device(1_000_000, 768, dev)
    q, planted = synth.queries_device(256, rows)
    ix = FlatIndex(dim=768, capacity=1_000_000)
    ix.add_device(rows)
    k = 50
    s = torch.empty((256, k), dtype=torch.float32, device=dev)
    i = torch.empty((256, k), dtype=torch.int64, device=dev)
    s2, i2 = torch.empty_like(s), torch.empty_like(i)
    ix.set_precision(_lib.MQ_DTYPE_F32)
    ix.search_device(q, k, s2, i2)
    ix.set_precision(_lib.MQ_DTYPE_BF16)
    ix.search_device(q, k, s, i)
    torch.cuda.synchronize()
    pl = planted >= 0
    assert bool((i[pl, 0] == planted[pl]).all())
    got, exact = i.cpu().numpy(), i2.cpu().numpy()
    assert (got >= 0).all()
    hits = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(got, exact))
    assert hits / (256 * k) >= 0.98, hits / (256 * k)
    normed = torch.nn.functional.normalize(rows, dim=1)
    dots = (normed[i] * q[:, None, :]).sum(-1)  # fp32 dots of the returned rows
    assert float((dots - s).abs().max()) < 1e-5
    # against float64 (the full-size case compared only with the HIP exact
    # path): the exact path within tie groups, with its tie swaps counted, and the bf16
    # path's recall@50
    del normed
    normed64 = torch.nn.functional.normalize(rows.double(), dim=1)
    ref_full = q.double() @ normed64.T
    del normed64
    rv, ri = torch.topk(ref_full, k + 1, dim=1)
    fails = check_topk(exact, s2.cpu().numpy(), None, k, ref_top=(rv.cpu().numpy(), ri.cpu().numpy()),
                       n_rows=1_000_000,
                       ref_lookup=lambda b, ids: ref_full[b, torch.as_tensor(ids, device=dev)].cpu().numpy())
    assert fails == [], fails[:3]
    swaps = int((i2 != ri[:, :k]).sum())  # positions inside a tie group that differ from float64
    ref_ids = ri[:, :k].cpu().numpy()
    hits64 = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(got, ref_ids))
    print("config5: exact-path tie swaps vs float64 %d of %d, bf16 recall@50 vs float64 %.5f"
          % (swaps, 256 * k, hits64 / (256 * k)))
    assert swaps <= 256 * k // 500, swaps
    assert hits64 / (256 * k) >= 0.98, hits64 / (256 * k)
