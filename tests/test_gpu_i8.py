"""GPU parity of K9q, the int8-shadow threshold scan that screens single queries first in
the exact mode (MQ_DTYPE_F32_SCREEN, >= 65536 rows).  Whatever the screen decides, the
result must be the oracle's exact top-k (tie-group aware) and identical to the bf16
stream tier's; uncertified queries pass down, and a corpus that defeats the int8 bound
switches the tier off for a while."""
import numpy as np
import pytest

from mediquery_hip import _lib, synth
from mediquery_hip.native import FlatIndex
from oracle.flat import check_topk, exact_scores

pytestmark = pytest.mark.gpu


def _index(rows):
    ix = FlatIndex(dim=rows.shape[1])
    ix.add(rows)
    ix.set_precision(_lib.MQ_DTYPE_F32_SCREEN)
    return ix


def _singles(ix, q, k):
    out = [ix.search(q[j:j + 1], k) for j in range(q.shape[0])]
    return np.concatenate([o[0] for o in out]), np.concatenate([o[1] for o in out])


@pytest.mark.parametrize("n,clustered", [(70001, True), (131075, False)])
@pytest.mark.parametrize("k", [1, 5, 16, 64])
def test_int8_screen_single_queries_exact(require_gpu, n, clustered, k):
    """Ragged last 8-row unit (70001, 131075 rows), clustered (crowded top scores: many
    pass down) and Gaussian corpora: exact top-k = oracle, same ids and scores as the
    bf16 stream tier."""
    c = synth.corpus(n, 768, seed=n + k, clustered=clustered)
    q, planted = synth.queries(12, c, seed=k)
    ref = exact_scores(q, c)
    ix = _index(c)
    s, i = _singles(ix, q, k)
    assert check_topk(i, s, ref, k) == []
    pl = planted >= 0
    assert (i[pl, 0] == planted[pl]).all()
    ix.set_int8_screen(False)
    s2, i2 = _singles(ix, q, k)
    np.testing.assert_array_equal(i, i2)
    np.testing.assert_allclose(s, s2, rtol=0, atol=1e-6)


def _int8_emulation(rows):
    """The int8 shadow as i8_shadow_kernel builds it (fp32 arithmetic, round half even)."""
    x = rows / np.linalg.norm(rows, axis=1, keepdims=True)
    amax = np.abs(x).max(axis=1, keepdims=True).astype(np.float32)
    sc = (amax / np.float32(127)).astype(np.float32)
    inv = (np.float32(127) / amax).astype(np.float32)
    r8 = np.clip(np.rint((x * inv).astype(np.float32)), -127, 127).astype(np.float32)
    return x, sc[:, 0], r8


def test_int8_screen_candidates_match_emulation(require_gpu):
    """The screen alone (mq_debug_int8_screen): candidate scores = scale * (q . r8) of a
    numpy int8 shadow to fp32 rounding, the candidates are the emulated top-64 (up to
    near-ties), the shadow's error maximum matches, and every exact score lies within
    the certificate's bound of its screen score."""
    c = synth.corpus(70001, 768, seed=4, clustered=False)
    q, _ = synth.queries(3, c, seed=4)
    ix = _index(c)
    x, sc, r8 = _int8_emulation(c)
    dmax = np.linalg.norm(x - sc[:, None] * r8, axis=1).max()
    for j in range(3):
        cs = np.empty(64, np.float32)
        ci = np.empty(64, np.int64)
        st = np.empty(2, np.float32)
        _lib.call("mq_debug_int8_screen", ix._h, _lib.ptr(np.ascontiguousarray(q[j])), 64, _lib.ptr(cs),
                  _lib.ptr(ci), _lib.ptr(st))
        assert abs(st[0] - dmax) <= 1e-5 * dmax, (st, dmax)
        emu = sc.astype(np.float64) * (r8.astype(np.float64) @ q[j].astype(np.float64))
        ok = ci >= 0
        assert ok.sum() >= 5
        np.testing.assert_allclose(cs[ok], emu[ci[ok]], rtol=0, atol=2e-6)
        kth = np.sort(emu)[-64]
        assert (emu[ci[ok]] >= kth - 1e-5).all()
        exact = x.astype(np.float64) @ q[j].astype(np.float64)
        assert np.abs(exact - emu).max() <= st[0] * np.linalg.norm(q[j]) + 1e-6


def test_int8_screen_certifies_gaussian_corpus(require_gpu):
    """Unit Gaussian rows, random queries (the bench's single-query workload at 1/5 size):
    the int8 bound (~0.01) sits well inside the gap between the 5th and 64th best scores,
    so almost every query is answered by the int8 tier."""
    c = synth.corpus(200000, 768, seed=11, clustered=False)
    rng = np.random.default_rng(5)
    q = rng.standard_normal((32, 768)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    ix = _index(c)
    s, i = _singles(ix, q, 5)
    assert check_topk(i, s, exact_scores(q, c), 5) == []
    assert ix.screen_passdowns <= 1, ix.screen_passdowns  # (4 would trip the sit-out)
    assert ix.screen_fallbacks == 0


@pytest.mark.parametrize("dim", [256, 512, 1024])
def test_int8_screen_other_widths(require_gpu, dim):
    c = synth.corpus(70000, dim, seed=dim, clustered=False)
    q, planted = synth.queries(6, c, seed=dim)
    ix = _index(c)
    s, i = _singles(ix, q, 5)
    assert check_topk(i, s, exact_scores(q, c), 5) == []


def test_int8_screen_crowded_corpus_passes_down_then_sits_out(require_gpu):
    """70000 near-copies of one direction (spread 1e-4, far inside the int8 bound): every
    int8 certificate fails and the query is answered by the bf16 stream tier; after four
    failures (running failure share > 0.3) the int8 tier sits out, so later queries no
    longer pass down.  Results exact throughout."""
    rng = np.random.default_rng(9)
    base = rng.standard_normal(768).astype(np.float32)
    c = base + 1e-4 * rng.standard_normal((70000, 768)).astype(np.float32)
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    q = (base + 0.01 * rng.standard_normal((10, 768))).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    ix = _index(c)
    s, i = _singles(ix, q, 5)
    assert check_topk(i, s, exact_scores(q, c), 5) == []
    assert ix.screen_passdowns == 4, ix.screen_passdowns
    ix.set_int8_screen(True)  # re-arms the tier
    ix.search(q[:1], 5)
    assert ix.screen_passdowns == 5


def test_int8_screen_full_size_planted(require_gpu):
    """BASELINE config 3's corpus (1M x 768 on the device), single planted queries: the
    int8 tier's answers equal the direct exact scan's."""
    import torch
    dev = torch.device("cuda", 0)
    rows = synth.corpus_device(1_000_000, 768, dev)
    q, planted = synth.queries_device(8, rows)
    ix = FlatIndex(dim=768, capacity=1_000_000)
    ix.add_device(rows)
    s = torch.empty((1, 5), dtype=torch.float32, device=dev)
    i = torch.empty((1, 5), dtype=torch.int64, device=dev)
    got, want = [], []
    for prec, out in ((_lib.MQ_DTYPE_F32_SCREEN, got), (_lib.MQ_DTYPE_F32, want)):
        ix.set_precision(prec)
        for j in range(8):
            ix.search_device(q[j:j + 1].contiguous(), 5, s, i)
            torch.cuda.synchronize()
            out.append(i.cpu().numpy().copy())
    np.testing.assert_array_equal(np.concatenate(got), np.concatenate(want))
    pl = (planted >= 0).cpu().numpy()
    assert (np.concatenate(got)[pl, 0] == planted.cpu().numpy()[pl]).all()
    assert ix.screen_fallbacks == 0
