"""GPU parity of the flat index (K8 add, K9 fused score + top-k, K10 merge) through the
C ABI against the float64 oracle (tie-group-aware: ids exact outside tie groups,
cosine within 1e-4)."""
import os

import numpy as np
import pytest

from mediquery_hip import _lib, synth
from mediquery_hip.native import FlatIndex, merge_topk_device, merge_topk_host
from oracle.flat import check_topk, exact_scores, search

pytestmark = pytest.mark.gpu


def _index(rows, prec=_lib.MQ_DTYPE_F32):
    ix = FlatIndex(dim=rows.shape[1])
    ix.add(rows)
    ix.set_precision(prec)
    return ix


PRECS = [_lib.MQ_DTYPE_F32, _lib.MQ_DTYPE_F32X6]


@pytest.mark.parametrize("prec", PRECS)
def test_flat_golden_fixture(require_gpu, golden, prec):
    f = np.load(os.path.join(golden, "flat_golden.npz"))
    c = synth.corpus(int(f["n"]), int(f["dim"]), clustered=True)
    q, planted = synth.queries(int(f["nq"]), c)
    ref = exact_scores(q, c)
    ix = _index(c, prec)
    for k in (5, 50):
        s, i = ix.search(q, k)
        assert check_topk(i, s, ref, k) == [], k
        pl = planted >= 0
        assert (i[pl, 0] == planted[pl]).all()


@pytest.mark.parametrize("n,nq,k", [
    (1, 1, 1), (5, 3, 8), (127, 7, 5), (128, 32, 5), (129, 33, 9), (1000, 64, 32),
    (1000, 65, 33), (4099, 128, 5), (4099, 200, 64), (3000, 256, 5), (700, 1, 64), (2500, 300, 17)])
@pytest.mark.parametrize("prec", PRECS)
def test_shapes_vs_oracle(require_gpu, n, nq, k, prec):
    c = synth.corpus(n, 768, seed=n)
    q, _ = synth.queries(nq, c, seed=nq)
    ix = _index(c, prec)
    s, i = ix.search(q, k)
    ref = exact_scores(q, c)
    kk = min(k, n)
    assert check_topk(i[:, :kk], s[:, :kk], ref, k) == []
    if k > n:  # k > N: N results, then (-inf, -1) padding
        assert (i[:, n:] == -1).all() and np.isneginf(s[:, n:]).all()


@pytest.mark.parametrize("dim", [768, 128, 1024])
@pytest.mark.parametrize("n", [777, 20000])
def test_small_batch_stream_and_mfma_paths(require_gpu, dim, n):
    """Small batches (nq <= threshold) run the streaming fp32 kernel (K9s); threshold 0
    sends the same batches to the narrow MFMA tiles.  Both must match the oracle, for
    every NQ specialisation (1, 2, 4, 8, 16) and list length (8, 16, 16+rescan)."""
    c = synth.corpus(n, dim, seed=dim + n, clustered=True)
    ref_q, _ = synth.queries(16, c, seed=5)
    ref = exact_scores(ref_q, c)
    ix = _index(c)
    for thr in (16, 0):
        ix.set_stream_threshold(thr)
        for nq in (1, 2, 3, 5, 8, 13, 16):
            for k in (1, 5, 17, 50):
                s, i = ix.search(ref_q[:nq], k)
                assert check_topk(i, s, ref[:nq], k) == [], (thr, nq, k)


def test_stream_kernel_overflow_rescan(require_gpu):
    """Streaming kernel (K9s) list overflow: lane group g scans rows g, g+G, g+2G, ...
    (G = 16 x blocks, blocks = min(2 x CUs, ceil(n/128))); 20 copies of one row placed
    G apart all land in one group, so k = 20 must fire the check and re-scan."""
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n = 24 * 16 * 2 * cus
    G = 16 * min(2 * cus, (n + 127) // 128)
    rng = np.random.default_rng(5)
    c = rng.standard_normal((n, 768), dtype=np.float32)
    ids = 7 + G * np.arange(20)
    c[ids] = c[7]
    ix = _index(c)
    q = c[7:8] / np.linalg.norm(c[7])
    before = ix.rescans
    s, i = ix.search(q, 20)
    assert ix.rescans == before + 1
    assert i[0].tolist() == ids.tolist()
    np.testing.assert_allclose(s[0], 1.0, atol=1e-5)


def test_merge_concentrated_top_k(require_gpu):
    """k > 16 merges by threshold (no per-thread lists).  At B = 100 (wide tiles, 2 lists
    per 128-row tile: list = 2*tile + half for the first G tiles) 15 copies in tile 3
    (list 6) and 9 in tile 131 (list 262) would have put 24 top-k members in one 16-entry
    thread list of the thread-list merge; no scan list is full of copies: the result is
    exact without a re-scan or re-merge."""
    nq, n = 100, 128 * 1024
    rng = np.random.default_rng(9)
    c = rng.standard_normal((n, 768), dtype=np.float32)
    blk_a = np.arange(15) + 128 * 3
    blk_b = np.arange(9) + 128 * 131
    c[blk_a] = c[blk_a[0]]
    c[blk_b] = c[blk_a[0]]
    q = np.repeat(c[blk_a[0]:blk_a[0] + 1], nq, axis=0) / np.linalg.norm(c[blk_a[0]])
    ix = _index(c)
    r0, m0 = ix.rescans, ix.remerges
    s, i = ix.search(q, 30)
    assert (i[:, :24] == np.concatenate([blk_a, blk_b])).all()
    assert ix.rescans == r0
    assert ix.remerges == m0
    ref = exact_scores(q[:2], c)
    assert check_topk(i[:2], s[:2], ref, 30) == []


@pytest.mark.parametrize("prec", [_lib.MQ_DTYPE_F32, _lib.MQ_DTYPE_F32_SCREEN])
def test_merge_massive_ties_fall_back_to_thread_lists(require_gpu, prec):
    """4000 copies of the query row: every list head ties at the top score, more than
    the threshold merge's 2048 survivor slots qualify, and the merge falls back to
    register thread lists (and their 64-entry re-merge): ids 0..63 in id order."""
    rng = np.random.default_rng(13)
    c = rng.standard_normal((40000, 768), dtype=np.float32)
    c[:4000] = c[0]
    q = np.repeat(c[:1] / np.linalg.norm(c[0]), 100, axis=0)
    ix = _index(c, prec)
    s, i = ix.search(q, 64)
    assert (i == np.arange(64)).all()
    assert (s[:, 0] == s[:, 63]).all()


def test_other_dims(require_gpu):
    for dim in (32, 256, 1024):
        c = synth.corpus(900, dim, seed=dim)
        q, _ = synth.queries(20, c)
        s, i = _index(c).search(q, 10)
        assert check_topk(i, s, exact_scores(q, c), 10) == []


def test_duplicates_and_exact_ties(require_gpu):
    c = synth.corpus(300, 768)
    c[200] = c[10]          # exact duplicate rows: ids must come out in row order
    c[201] = 3.0 * c[10]    # same direction, different norm -> same cosine up to rounding
    q = c[10:11] / np.linalg.norm(c[10])
    ix = _index(c)
    for thr in (16, 0):     # streaming kernel and MFMA tiles
        ix.set_stream_threshold(thr)
        s, i = ix.search(q, 3)
        got = i[0].tolist()
        assert sorted(got) == [10, 200, 201]
        assert got.index(10) < got.index(200)   # bit-identical rows tie -> row order
        assert s[0][got.index(10)] == s[0][got.index(200)]
        np.testing.assert_allclose(s[0], 1.0, atol=1e-5)


def test_empty_append_reset_get(require_gpu, tmp_path):
    ix = FlatIndex(dim=768)
    q, _ = synth.queries(4, synth.corpus(10, 768))
    s, i = ix.search(q, 5)
    assert (i == -1).all()
    c = synth.corpus(1000, 768)
    ix.add(c[:300])
    ix.add(c[300:])        # appended rows keep insertion-order ids
    assert len(ix) == 1000
    s, i = ix.search(q, 5)
    assert check_topk(i, s, exact_scores(q, c), 5) == []
    got = ix.get(295, 10)
    np.testing.assert_allclose(got, c[295:305] / np.linalg.norm(c[295:305], axis=1, keepdims=True), atol=1e-6)
    p = str(tmp_path / "ix.flat")
    ix.save(p)
    ix2 = FlatIndex(dim=768)
    ix2.load(p)
    s2, i2 = ix2.search(q, 5)
    np.testing.assert_array_equal(i2, i)
    np.testing.assert_array_equal(s2, s)
    ix.reset()
    assert len(ix) == 0 and (ix.search(q, 3)[1] == -1).all()


def test_device_pointer_path_and_device_merge(require_gpu):
    import torch
    dev = torch.device("cuda", 0)
    c = synth.corpus(5000, 768, clustered=True)
    q, _ = synth.queries(96, c)
    ix = FlatIndex(dim=768)
    ix.add_device(torch.from_numpy(c).to(dev))
    qd = torch.from_numpy(q).to(dev)
    s = torch.empty((96, 10), dtype=torch.float32, device=dev)
    i = torch.empty((96, 10), dtype=torch.int64, device=dev)
    ix.search_device(qd, 10, s, i)
    torch.cuda.synchronize()
    assert check_topk(i.cpu().numpy(), s.cpu().numpy(), exact_scores(q, c), 10) == []
    # device merge of 3 shards == host merge == single index
    shards = [(0, 1700), (1700, 3300), (3300, 5000)]
    ss, ii = [], []
    for a, b in shards:
        sub = FlatIndex(dim=768)
        sub.add(c[a:b])
        s_, i_ = sub.search(q, 10)
        ss.append(s_)
        ii.append(np.where(i_ >= 0, i_ + a, -1))
    hs, hi = merge_topk_host(np.stack(ss), np.stack(ii), 10)
    np.testing.assert_array_equal(hi, i.cpu().numpy())
    ds = torch.empty_like(s)
    di = torch.empty_like(i)
    merge_topk_device(torch.from_numpy(np.stack(ss)).to(dev), torch.from_numpy(np.stack(ii)).to(dev), 10, ds, di)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(di.cpu().numpy(), hi)


@pytest.mark.parametrize("prec", PRECS + [_lib.MQ_DTYPE_F32_SCREEN])
def test_full_size_1m_planted_and_fp64_reference(require_gpu, prec):
    """BASELINE config 3 size (1M x 768, B = 256, k = 5): planted queries hit their
    rows, and the ids equal a float64 torch reference of the same device corpus - for
    the headline's own search mode (MQ_DTYPE_F32_SCREEN: certified bf16 screen + fp32
    re-rank) directly, not only through its equality with the direct scan."""
    import torch
    dev = torch.device("cuda", 0)
    rows = synth.corpus_device(1_000_000, 768, dev)
    q, planted = synth.queries_device(256, rows)
    ix = FlatIndex(dim=768, capacity=1_000_000)
    ix.add_device(rows)
    ix.set_precision(prec)
    s = torch.empty((256, 5), dtype=torch.float32, device=dev)
    i = torch.empty((256, 5), dtype=torch.int64, device=dev)
    ix.search_device(q, 5, s, i)
    torch.cuda.synchronize()
    pl = planted >= 0
    assert bool((i[pl, 0] == planted[pl]).all())
    normed = torch.nn.functional.normalize(rows.double(), dim=1)
    ref_full = q.double() @ normed.T                         # [256, 1M] float64
    rv, ri = torch.topk(ref_full, 6, dim=1)
    del normed
    fails = check_topk(i.cpu().numpy(), s.cpu().numpy(), None, 5,
                       ref_top=(rv.cpu().numpy(), ri.cpu().numpy()), n_rows=1_000_000,
                       ref_lookup=lambda b, ids: ref_full[b, torch.as_tensor(ids, device=dev)].cpu().numpy())
    assert fails == []
    if prec in (_lib.MQ_DTYPE_F32, _lib.MQ_DTYPE_F32_SCREEN):
        # pins check_topk's tie tolerance at its 1e-6 floor on typical data: the
        # fp32 scores of the unplanted queries (|score| ~0.2) are within 3.3e-7 of float64,
        # so 3 e_b <= 1e-6 and every position outside a 1e-6 tie must match exactly
        err = (s.double() - torch.gather(ref_full, 1, i)).abs()[~pl]
        assert float(err.max()) <= 1e-6 / 3, float(err.max())


@pytest.mark.parametrize("nq,k", [(1, 5), (64, 5), (256, 5), (300, 16), (200, 50), (33, 64)])
def test_bf16_coarse_rerank_recall(require_gpu, nq, k):
    """BASELINE config 5 path: bf16 coarse scan (top max(2k, 50), capped at 64) + exact
    fp32 re-rank.  Approximate by design.  With a >= 2x coarse margin (k <= 32) the
    re-ranked top-k equals the exact top-k on this data; for k = 50/64 the margin is
    thin, so recall@k >= 0.98 is required.  Returned scores are always exact fp32 dots."""
    c = synth.corpus(20000, 768, clustered=True)
    q, planted = synth.queries(nq, c, seed=3)
    ix = _index(c, _lib.MQ_DTYPE_BF16)
    s, i = ix.search(q, k)
    ref = exact_scores(q, c)
    pl = planted >= 0
    assert (i[pl, 0] == planted[pl]).all()
    assert (i >= 0).all()
    got = np.take_along_axis(ref, i, axis=1)          # exact scores of the returned ids
    np.testing.assert_allclose(s, got, rtol=0, atol=1e-5)
    if k <= 32:
        assert check_topk(i, s, ref, k) == []
    else:
        exact = np.argsort(-ref, axis=1, kind="stable")[:, :k]
        hits = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(i, exact))
        assert hits / (nq * k) >= 0.98


@pytest.mark.parametrize("prec", PRECS + [_lib.MQ_DTYPE_BF16])
@pytest.mark.parametrize("nq", [1, 100])
def test_large_k_list_overflow_rescan(require_gpu, prec, nq):
    """k > 16 runs the scan with 16-entry lists and the merge's overflow check.  Plant 60
    identical rows in one contiguous block (one row tile -> one list) so a query equal
    to that row has its whole top-50 in a single list: the check must fire and the
    re-scan with 64-entry lists must return the 50 copies in id order."""
    rng = np.random.default_rng(11)
    c = rng.standard_normal((9000, 768)).astype(np.float32)
    c[4000:4060] = c[4000]
    q = np.repeat(c[4000:4001], nq, axis=0) / np.linalg.norm(c[4000])
    q[1:] = q[1:] + 0.001 * rng.standard_normal(q[1:].shape).astype(np.float32)
    ix = _index(c, prec)
    for k in (17, 50, 64):
        before = ix.rescans
        s, i = ix.search(q, k)
        if nq > 8:   # tiled scan: the block of copies is one row tile -> one list
            assert ix.rescans == before + 1
        assert (i[0, :min(k, 60)] == np.arange(4000, 4000 + min(k, 60))).all(), (k, i[0])
        if prec != _lib.MQ_DTYPE_BF16:
            ref = exact_scores(q, c)
            assert check_topk(i, s, ref, k) == []


def test_select_gathers_and_compacts(require_gpu):
    """mq_index_select: device gather of chosen rows (any order, repeats) into another
    index, and in-place compaction; rows come back bit-identical, search follows."""
    c = synth.corpus(3000, 768, clustered=True)
    ix = _index(c)
    stored = ix.get()
    sel = np.array([2999, 5, 5, 17, 0, 1234], np.int64)
    sub = ix.select(sel)
    assert len(sub) == len(sel)
    np.testing.assert_array_equal(sub.get(), stored[sel])
    s, i = sub.search(stored[[17]], 2)
    assert i[0, 0] == 3 and i[0, 1] != 3
    keep = np.arange(0, 3000, 3)
    ix.select(keep, out=ix)
    assert len(ix) == len(keep)
    np.testing.assert_array_equal(ix.get(), stored[keep])
    ix.add(c[:2])  # grows again after a compaction
    assert len(ix) == len(keep) + 2
    ix.select([], out=ix)
    assert len(ix) == 0
    with pytest.raises(_lib.MQError, match="out of range"):
        sub.select([6])


@pytest.mark.parametrize("nq", [1, 3, 40, 256])
@pytest.mark.parametrize("k", [1, 5, 50])
def test_screened_exact_matches_direct_exact(require_gpu, golden, k, nq):
    """MQ_DTYPE_F32_SCREEN returns the exact fp32 top-k through certified screens (bf16
    shadow stream for nq <= 4, bf16 MFMA scan for batches, split-f32 for the queries
    passed down, direct scan last): same ids as the direct exact scan outside tie groups,
    oracle parity, scores within two fp32 dot orders."""
    f = np.load(os.path.join(golden, "flat_golden.npz"))
    c = synth.corpus(int(f["n"]), int(f["dim"]), clustered=True)
    q, planted = synth.queries(nq, c)
    ref = exact_scores(q, c)
    ix = _index(c, _lib.MQ_DTYPE_F32_SCREEN)
    s, i = ix.search(q, k)
    assert check_topk(i, s, ref, k) == []
    pl = planted >= 0
    assert (i[pl, 0] == planted[pl]).all()
    ix.set_precision(_lib.MQ_DTYPE_F32)
    s2, i2 = ix.search(q, k)
    assert check_topk(i2, s2, ref, k) == []
    np.testing.assert_allclose(s, s2, atol=1e-5)  # two fp32 dot orders


def test_screened_falls_back_when_uncertified(require_gpu):
    """Twenty copies of the best row: the last candidate ties the k-th result, no
    certificate can hold, and the query is re-run on the direct exact scan (the bf16
    screen passes it to the direct scan, a lone failure; the others stay certified)."""
    c = synth.corpus(4000, 768, clustered=True)
    q, _ = synth.queries(128, c)
    c[1000:1070] = q[0]  # exact duplicates of query 0's direction (more than 64)
    ix = _index(c, _lib.MQ_DTYPE_F32_SCREEN)
    s, i = ix.search(q, 5)
    assert ix.screen_fallbacks >= 1
    assert i[0].tolist() == [1000, 1001, 1002, 1003, 1004]
    assert check_topk(i, s, exact_scores(q, c), 5) == []
    before = ix.screen_fallbacks
    s1, i1 = ix.search(q[:1], 5)  # single query: bf16 stream screen -> exact stream
    assert ix.screen_fallbacks == before + 1
    assert i1[0].tolist() == [1000, 1001, 1002, 1003, 1004]


def _dup_corpus(n_fail, n=6000, copies=70, seed=0):
    """Queries 0..n_fail-1 each get `copies` exact duplicate rows (ids 1000 + 80 j ..):
    their top scores tie beyond the 64 screen candidates, so no certificate can hold."""
    c = synth.corpus(n, 768, seed=seed, clustered=True)
    q, _ = synth.queries(128, c, seed=seed)
    for j in range(n_fail):
        c[1000 + 80 * j:1000 + 80 * j + copies] = q[j]
    return c, q


@pytest.mark.parametrize("n_fail,k", [(1, 5), (6, 5), (9, 50), (5, 16)])
def test_async_screen_fallback_exact(require_gpu, n_fail, k):
    """The default batched screen never reads its certificate back: uncertified queries
    are gathered and re-run on the device in one exact MFMA pass (fallback_search /
    fallback_merge, k <= 16) and written in place; k = 50 skips the bf16 tier and runs the
    split-f32 screen, whose failures go to the direct scan.  Results equal the oracle, the
    duplicates come out in id order, the count reaches screen_fallbacks, and after a
    failure has been observed the next batches take the synchronous tiered path (same
    results)."""
    c, q = _dup_corpus(n_fail)
    ref = exact_scores(q, c)
    ix = _index(c, _lib.MQ_DTYPE_F32_SCREEN)
    s, i = ix.search(q, k)
    assert check_topk(i, s, ref, k) == []
    for j in range(n_fail):
        assert i[j].tolist() == list(range(1000 + 80 * j, 1000 + 80 * j + k)), j
    # (at k = 50 over 6000 rows other queries' 50th and 64th scores crowd within the
    # bf16 bound too: they fail and are re-run the same way)
    assert ix.screen_fallbacks >= n_fail
    s2, i2 = ix.search(q, k)  # failure seen -> synchronous tiers for the cooldown
    assert check_topk(i2, s2, ref, k) == []
    assert (i2 == i).all()
    np.testing.assert_allclose(s2, s, atol=1e-6)
    assert ix.screen_fallbacks + ix.screen_passdowns >= 2 * n_fail


def test_async_screen_fallback_many_failures_threshold_scan(require_gpu):
    """130 of 256 queries uncertified on the threshold-scan path (>= 65536 rows): the device
    fallback re-runs them in one pass on the wide MFMA tile and every result equals the
    oracle; the synchronous cooldown path then passes them down to the split-f32 tier
    (> 64 failures) with the same ids."""
    rng = np.random.default_rng(9)
    c = synth.corpus(70000, 768, seed=9, clustered=True)
    q, _ = synth.queries(256, c, seed=9)
    fails = rng.choice(256, 130, replace=False)
    for n, j in enumerate(fails):
        c[200 * n:200 * n + 70] = q[j]
    ref = exact_scores(q, c)
    ix = _index(c, _lib.MQ_DTYPE_F32_SCREEN)
    s, i = ix.search(q, 5)
    assert check_topk(i, s, ref, 5) == []
    for n, j in enumerate(fails):
        assert i[j].tolist() == list(range(200 * n, 200 * n + 5)), j
    assert ix.screen_fallbacks >= 130
    s2, i2 = ix.search(q, 5)
    assert (i2 == i).all()
    assert ix.screen_passdowns >= 130


def test_async_screen_matches_sync_when_certified(require_gpu):
    """No failures: the asynchronous and synchronous batched screens return bitwise the
    same results (the fallback kernels exit at once)."""
    c = synth.corpus(70000, 768, seed=4, clustered=True)
    q, _ = synth.queries(200, c, seed=4)
    ix = _index(c, _lib.MQ_DTYPE_F32_SCREEN)
    s, i = ix.search(q, 5)
    ix.set_async_screen(False)
    s2, i2 = ix.search(q, 5)
    assert (i == i2).all() and (s == s2).all()
    assert ix.screen_fallbacks == 0
    assert check_topk(i, s, exact_scores(q, c), 5) == []


def _near_tie_rows(q, spacing, count, rng):
    """Rows at cosine 1 - m * spacing (m = 0..count-1) from unit query q."""
    out = []
    for m in range(count):
        u = rng.standard_normal(q.shape[0]).astype(np.float64)
        u -= (u @ q) * q
        u /= np.linalg.norm(u)
        cm = 1.0 - m * spacing
        out.append(cm * q + np.sqrt(1.0 - cm * cm) * u)
    return np.array(out, np.float32)


def test_screened_passes_near_ties_to_split_f32(require_gpu):
    """Top-70 scores 4e-5 apart: the 5th and 64th best are 2.4e-3 apart, inside the bf16
    screen's ~3.5e-3 bound (uncertified); the 5th and 8th 1.2e-4 apart, outside the
    split-f32 screen's 8e-5 (certified): the 100 queries go down one tier, none reaches
    the direct scan, and the results stay exact."""
    rng = np.random.default_rng(5)
    c = rng.standard_normal((30000, 768)).astype(np.float32)
    q = rng.standard_normal((128, 768))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    for j in range(100):
        c[j * 70:(j + 1) * 70] = _near_tie_rows(q[j], 4e-5, 70, rng)
    q = q.astype(np.float32)
    ix = _index(c, _lib.MQ_DTYPE_F32_SCREEN)
    ix.set_async_screen(False)  # the tiered (synchronous) re-run
    s, i = ix.search(q, 5)
    assert ix.screen_passdowns >= 100
    assert ix.screen_fallbacks == 0
    assert check_topk(i, s, exact_scores(q, c), 5) == []
    for j in range(100):
        assert i[j].tolist() == list(range(j * 70, j * 70 + 5))


def test_config2_end_to_end_encoder_and_screen_vs_fp64(require_gpu):
    """BASELINE config 2 end to end: 100k x 768 corpus, B = 256 queries
    of L = 32 token ids through the 12-layer encoder at the headline arithmetic (split-f32)
    and the certified screen (MQ_DTYPE_F32_SCREEN), k = 5.  The embeddings against the
    torch-CPU oracle (1e-4 / cos 1 - 1e-5), the top-5 against float64 over the same device
    corpus, and the planted rows (each query's own embedding planted in the corpus) found."""
    import torch
    from mediquery_hip.config import DMETA_BASE
    from mediquery_hip.native import Encoder
    from mediquery_hip.weights import synthetic_state_dict
    from oracle.encoder import OracleEncoder
    dev = torch.device("cuda", 0)
    ids, mask = synth.token_batch(256, 32)
    enc = Encoder(DMETA_BASE)
    enc.set_precision(_lib.MQ_DTYPE_F32X6)
    q = torch.empty((256, 768), dtype=torch.float32, device=dev)
    enc.embed_device(torch.from_numpy(ids).to(dev), torch.from_numpy(mask).to(dev), q)
    torch.cuda.synchronize()
    ref_e = OracleEncoder(DMETA_BASE, synthetic_state_dict(DMETA_BASE, 0)).embed(ids, mask)
    qe = q.cpu().numpy()
    np.testing.assert_allclose(qe, ref_e, atol=1e-4, rtol=0)
    rows = synth.corpus_device(100_000, 768, dev, seed=synth.CORPUS_SEED + 2)
    plant = torch.arange(0, 100_000, 1000, device=dev)[:64]
    rows[plant] = q[:64]  # queries 0..63 planted (unit rows already)
    ix = FlatIndex(dim=768, capacity=100_000)
    ix.add_device(rows)
    ix.set_precision(_lib.MQ_DTYPE_F32_SCREEN)
    s = torch.empty((256, 5), dtype=torch.float32, device=dev)
    i = torch.empty((256, 5), dtype=torch.int64, device=dev)
    ix.search_device(q, 5, s, i)
    torch.cuda.synchronize()
    assert bool((i[:64, 0] == plant).all())
    normed = torch.nn.functional.normalize(rows.double(), dim=1)
    ref_full = q.double() @ normed.T
    rv, ri = torch.topk(ref_full, 6, dim=1)
    fails = check_topk(i.cpu().numpy(), s.cpu().numpy(), None, 5,
                       ref_top=(rv.cpu().numpy(), ri.cpu().numpy()), n_rows=100_000,
                       ref_lookup=lambda b, ids_: ref_full[b, torch.as_tensor(ids_, device=dev)].cpu().numpy())
    assert fails == []
