"""ORACLE (test infrastructure only) - CPU restatement of the vector-store k-NN step.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.

What it restates: the k-NN half of `vectorstore.similarity_search(query, k=5)`
(reference src/agents/nodes.py:93 on the Chroma store built at src/medical_engine.py:52
and src/ingest_medical.py:106-110).  Chroma's default space is squared L2 (no
collection_metadata is passed at either call site); on unit vectors that is 2 - 2cos, so
ranking by cosine descending is ranking by distance ascending.  Chroma's
HNSW is approximate; this oracle is the EXACT answer it approximates:

    score(q, r) = <q, r/||r||>   in float64, order: score desc, row id asc (ties),
    k > N returns N results, an empty index returns nothing.

Parity vs Chroma itself: UNPINNED (chromadb is absent offline and the reference has no
tests).  The exact-search restatement is pinned by construction plus tests/golden
fixtures (argsort vs argpartition restatements agree; planted queries find their row).
"""
import numpy as np


def normalize_rows(x, eps=1e-12):
    """Row L2 normalisation as the index's add step does it (F.normalize semantics)."""
    x = np.asarray(x, dtype=np.float64)
    n = np.sqrt((x * x).sum(-1, keepdims=True))
    return x / np.maximum(n, eps)


def exact_scores(queries, corpus, normalize_corpus=True):
    q = np.asarray(queries, dtype=np.float64)
    c = normalize_rows(corpus) if normalize_corpus else np.asarray(corpus, np.float64)
    return q @ c.T


def topk_from_scores(scores, k):
    """scores [B, N] float64 -> (top scores [B, k'], ids [B, k']) with k' = min(k, N),
    ordered by (score desc, id asc)."""
    scores = np.atleast_2d(scores)
    B, N = scores.shape
    kk = min(k, N)
    if kk == 0:
        return np.zeros((B, 0)), np.zeros((B, 0), dtype=np.int64)
    ids = np.empty((B, kk), dtype=np.int64)
    for b in range(B):
        # lexsort: last key primary -> (-score, id)
        order = np.lexsort((np.arange(N), -scores[b]))[:kk]
        ids[b] = order
    return np.take_along_axis(scores, ids, 1), ids


def search(queries, corpus, k):
    return topk_from_scores(exact_scores(queries, corpus), k)


def search_fp32_torch(queries, corpus_normed, k, threads=None):
    """fp32 mm + topk on the CPU - the timed CPU baseline leg."""
    import torch
    if threads:
        torch.set_num_threads(threads)
    q = torch.as_tensor(np.asarray(queries, dtype=np.float32))
    c = torch.as_tensor(np.asarray(corpus_normed, dtype=np.float32))
    s = q @ c.T
    v, i = torch.topk(s, min(k, c.shape[0]), dim=1)
    return v.numpy(), i.numpy()


def check_topk(got_ids, got_scores, full_ref_scores, k, tol=1e-6, score_tol=1e-4,
               ref_top=None, ref_lookup=None, n_rows=None, err_factor=3.0, tol_cap=1e-5):
    """Tie-group-aware comparison of a device top-k against the float64 oracle.

    Returns a list of failure strings (empty == parity).  Rules:
      * returned ids are distinct and within range; count == min(k, N);
      * each returned score is within `score_tol` of the oracle's score for that id;
      * position i must carry exactly the oracle's id wherever the oracle ranking is
        unambiguous there (neighbouring oracle scores differ by more than the query's
        tie tolerance); inside a tie group, the returned id's oracle score must be
        within that tolerance of the oracle's score at that position.
    Tie tolerance of query b: max(tol, err_factor * e_b) with tol = 1e-6
    and e_b = the largest |device score - float64 score| among b's returned ids.  Why
    the floor alone is not always attainable: a device score is fp32 arithmetic on fp32
    data - the row norm (a 768-term sum of squares: relative error <= 768 u worst case,
    ~sqrt(768) u / 2 ~ 8e-7 typical, u = 2^-24), the normalisation, and the 768-term
    dot (<= 384 u sum|q_i r_i| for the MFMA's 2-term steps, ~1e-7 typical at |score|
    ~0.2).  For scores near 1 (planted queries, duplicates) the norm term alone is ~1e-6,
    so two rows whose float64 scores differ by 1e-6 can legitimately swap in fp32.  Two
    scores swap only when their gap is below the sum of their errors; e_b measures those
    errors on the rows in question (the missed row's is of the same size), so 3 e_b
    covers the pair while the check stays at 1e-6 wherever the arithmetic is that
    accurate (measured e_b ~1e-7 .. 5e-7 at |score| ~0.2).  Capped at tol_cap = 1e-5 (the
    fixed tolerance of rounds 1-3): where scores carry encoder error (~1e-5 .. 1e-4 when
    the oracle embedded the texts itself) the groups are no wider than before.
    For full-size checks pass `ref_top=(scores[B, k+1], ids[B, k+1])` (sorted) and
    `ref_lookup(b, ids) -> oracle scores` instead of the dense [B, N] score matrix.
    """
    fails = []
    if ref_top is None:
        full_ref_scores = np.atleast_2d(full_ref_scores)
        B, N = full_ref_scores.shape
        ref_s, ref_i = topk_from_scores(full_ref_scores, min(k + 1, N))
        ref_lookup = lambda b, ids: full_ref_scores[b, ids]
    else:
        ref_s, ref_i = ref_top
        B = ref_s.shape[0]
        N = n_rows if n_rows is not None else np.iinfo(np.int64).max
    kk = min(k, N)
    got_ids = np.asarray(got_ids).reshape(B, -1)
    got_scores = np.asarray(got_scores).reshape(B, -1)
    if got_ids.shape[1] < kk:
        return ["returned %d columns, expected %d" % (got_ids.shape[1], kk)]
    for b in range(B):
        gi = got_ids[b, :kk].astype(np.int64)
        if np.any(gi < 0) or np.any(gi >= N):
            fails.append("q%d: id out of range %s" % (b, gi))
            continue
        if len(set(gi.tolist())) != kk:
            fails.append("q%d: duplicate ids %s" % (b, gi))
        gref = np.asarray(ref_lookup(b, gi), dtype=np.float64)
        err = np.abs(got_scores[b, :kk] - gref)
        if np.any(err > score_tol):
            fails.append("q%d: score error %.3g" % (b, err.max()))
        rs = ref_s[b]
        tb = min(max(tol, err_factor * float(err.max(initial=0.0))), tol_cap)
        for i in range(kk):
            prev_gap = np.inf if i == 0 else rs[i - 1] - rs[i]
            next_gap = np.inf if i + 1 >= len(rs) else rs[i] - rs[i + 1]
            if prev_gap > tb and next_gap > tb:
                if gi[i] != ref_i[b, i]:
                    fails.append("q%d pos%d: id %d != oracle %d" % (b, i, gi[i], ref_i[b, i]))
            elif abs(gref[i] - rs[i]) > tb:
                fails.append("q%d pos%d: id %d outside tie group" % (b, i, gi[i]))
    return fails
