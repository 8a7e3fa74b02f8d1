"""Flat exact-search oracle: ordering contract, tie handling, planted queries, and the
tie-group-aware checker used by every GPU parity test."""
import numpy as np
import pytest

from oracle.flat import check_topk, exact_scores, search, topk_from_scores
from mediquery_hip import synth


def test_order_and_ties():
    s = np.array([[0.5, 0.9, 0.9, 0.1, 0.9]])
    v, i = topk_from_scores(s, 4)
    assert i.tolist() == [[1, 2, 4, 0]]          # equal scores -> lower row id first
    v, i = topk_from_scores(s, 10)               # k > N returns N
    assert i.shape == (1, 5)
    v, i = topk_from_scores(np.zeros((2, 0)), 5)  # empty index
    assert i.shape == (2, 0)


def test_planted_queries_find_their_rows():
    c = synth.corpus(3000, 64)
    q, planted = synth.queries(16, c)
    _, ids = search(q, c, 5)
    pl = planted >= 0
    assert (ids[pl, 0] == planted[pl]).all()


def test_argsort_and_partition_restatements_agree():
    c = synth.corpus(1000, 32, clustered=True)
    q, _ = synth.queries(8, c)
    s = exact_scores(q, c)
    v, i = topk_from_scores(s, 20)
    for b in range(len(q)):
        part = np.argpartition(-s[b], 20)[:20]
        assert set(part) == set(i[b])


def test_checker_accepts_tie_permutations_and_rejects_errors():
    s = np.array([[0.9, 0.8, 0.8, 0.7, 0.1]])
    assert check_topk([[0, 2, 1]], [[0.9, 0.8, 0.8]], s, 3) == []     # swap inside tie group
    assert check_topk([[0, 1, 3]], [[0.9, 0.8, 0.7]], s, 3) != []     # 3 is outside the group
    assert check_topk([[1, 0, 2]], [[0.8, 0.9, 0.8]], s, 3) != []     # unambiguous position wrong
    assert check_topk([[0, 1, 2]], [[0.9, 0.8, 0.81]], s, 3) != []    # score off by 1e-2


def test_checker_tie_tolerance_stays_at_the_floor_for_accurate_scores():
    """the tie group is max(1e-6, 3 e_b) with e_b the result's own score error;
    with accurate scores it stays at the 1e-6 floor - two rows 2e-6 apart may not swap -
    and a result whose scores are 1e-5 off widens it only to the 1e-5 cap."""
    s = np.array([[0.2, 0.199998, 0.199996, 0.1]])
    assert check_topk([[1, 0, 2]], [[0.199998, 0.2, 0.199996]], s, 3) != []
    assert check_topk([[0, 1, 2]], [[0.2, 0.199998, 0.199996]], s, 3) == []
    s2 = np.array([[0.2, 0.199995, 0.19997, 0.1]])  # 5e-6 / 2.5e-5 apart
    assert check_topk([[1, 0, 2]], [[0.199995 + 4e-6, 0.2 - 4e-6, 0.19997]], s2, 3) == []
    assert check_topk([[0, 2, 1]], [[0.2 + 4e-6, 0.19997, 0.199995]], s2, 3) != []


def test_flat_golden_fixture(golden):
    f = np.load(golden + "/flat_golden.npz")
    c = synth.corpus(int(f["n"]), int(f["dim"]), clustered=True)
    assert np.isclose(float(c[:64].astype(np.float64).sum()), float(f["corpus_head_sum"]))
    q, planted = synth.queries(int(f["nq"]), c)
    for k in (5, 50):
        v, i = search(q, c, k)
        np.testing.assert_array_equal(i, f["ids_k%d" % k])
        np.testing.assert_allclose(v, f["scores_k%d" % k], rtol=0, atol=1e-12)
