"""Single-query exact search where the int8 screen's certificate is stressed: in-distribution
queries (a corpus row + noise) over the clustered corpus (4096 centroids, sigma 0.35, the
reference's duplicate-row pattern) - the retrieve path of
src/agents/nodes.py:93 on crowded data, where the query's cluster-mates fill the top scores
within the int8 bound.  Every answer against a float64 torch reference of the same device
corpus (tie-group-aware check_topk), and the screen counters: the int8 tier must certify
nearly every query (the r4 certificate, against the 64th-best survivor, failed the first
few and then sat out 96 of 100)."""
import numpy as np
import pytest

from mediquery_hip import _lib, synth
from mediquery_hip.native import FlatIndex
from oracle.flat import check_topk

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,k,nq", [(1_000_000, 5, 100), (200_000, 1, 40), (200_000, 16, 40)])
def test_clustered_single_queries_certified_and_exact(require_gpu, n, k, nq):
    import torch
    dev = torch.device("cuda", 0)
    rows, _ = synth.clustered_corpus_device(n, 768, dev)
    q, planted = synth.queries_device(nq, rows, seed=synth.QUERY_SEED + 11, planted_frac=1.0)
    ix = FlatIndex(dim=768, capacity=n)
    ix.add_device(rows)
    ix.set_precision(_lib.MQ_DTYPE_F32_SCREEN)
    s = torch.empty((nq, k), dtype=torch.float32, device=dev)
    i = torch.empty((nq, k), dtype=torch.int64, device=dev)
    ix.search_device(q[:1], k, s[:1], i[:1])  # builds the int8 shadow
    fb0, pd0, sk0 = ix.screen_fallbacks, ix.screen_passdowns, ix.int8_skips
    for j in range(nq):
        ix.search_device(q[j:j + 1], k, s[j:j + 1], i[j:j + 1])
    torch.cuda.synchronize()
    skips, passdowns, fallbacks = ix.int8_skips - sk0, ix.screen_passdowns - pd0, ix.screen_fallbacks - fb0
    assert skips <= nq // 10, (skips, passdowns, fallbacks)
    assert fallbacks <= max(1, nq // 50), (skips, passdowns, fallbacks)
    normed = torch.nn.functional.normalize(rows.double(), dim=1)
    del rows
    ref_full = q.double() @ normed.T
    del normed
    rv, ri = torch.topk(ref_full, k + 1, dim=1)
    fails = check_topk(i.cpu().numpy(), s.cpu().numpy(), None, k,
                       ref_top=(rv.cpu().numpy(), ri.cpu().numpy()), n_rows=n,
                       ref_lookup=lambda b, ids: ref_full[b, torch.as_tensor(ids, device=dev)].cpu().numpy())
    assert fails == [], fails[:3]
    ix.close()
