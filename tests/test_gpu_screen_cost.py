"""Exactness AND cost of the certified screen's escalation paths (MQ_DTYPE_F32_SCREEN) at
BASELINE config 3 size (1M x 768, batch 256), the search behind the reference's
`vectorstore.similarity_search` (src/agents/nodes.py:93) when it runs batched.

The screen is only worth having if a query it cannot certify costs no more than the
direct exact scan would have: large k skips the bf16 tier (its 64 candidates leave no
margin), the asynchronous device re-run covers every failed query in ONE MFMA pass over
the slab, and a corpus that keeps failing the bf16 certificate switches the tier off.
The oracle here is the direct exact fp32 scan (itself pinned to float64 elsewhere) plus a
float64 torch reference of the same device corpus."""
import statistics

import numpy as np
import pytest

from mediquery_hip import _lib, synth
from mediquery_hip.native import FlatIndex
from oracle.flat import check_topk, exact_scores

pytestmark = pytest.mark.gpu

N, B = 1_000_000, 256


def _median_ms(fn, reps=5, prep=None):
    import torch
    out = []
    for _ in range(reps):
        if prep:
            prep()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1))
    return statistics.median(out)


def _fp64_check(rows, q, s, i, k):
    """check_topk of a device result against float64 on the device corpus."""
    import torch
    normed = torch.nn.functional.normalize(rows.double(), dim=1)
    ref = q.double() @ normed.T
    del normed
    rv, ri = torch.topk(ref, k + 1, dim=1)
    dev = rows.device
    fails = check_topk(i.cpu().numpy(), s.cpu().numpy(), None, k,
                       ref_top=(rv.cpu().numpy(), ri.cpu().numpy()), n_rows=rows.shape[0],
                       ref_lookup=lambda b, ids: ref[b, torch.as_tensor(ids, device=dev)].cpu().numpy())
    del ref
    torch.cuda.empty_cache()
    return fails


def _out(k):
    import torch
    dev = torch.device("cuda", 0)
    return (torch.empty((B, k), dtype=torch.float32, device=dev),
            torch.empty((B, k), dtype=torch.int64, device=dev))


def test_screen_k50_full_size_equals_direct_in_time(require_gpu):
    """k = 50 over 1M rows: the screen takes the split-f32 tier (no bf16 attempt) and
    returns the direct exact scan's ids (float64-checked) in <= 1.2x its time; r3 sent
    this batch to the bf16 tier, failed most certificates and re-ran them on a VALU
    fallback at ~50x the direct scan's cost."""
    import torch
    dev = torch.device("cuda", 0)
    rows = synth.corpus_device(N, 768, dev)
    q, planted = synth.queries_device(B, rows)
    ix = FlatIndex(dim=768, capacity=N)
    ix.add_device(rows)
    k = 50
    s, i = _out(k)
    s2, i2 = _out(k)
    ix.set_precision(_lib.MQ_DTYPE_F32_SCREEN)
    ix.search_device(q, k, s, i)
    t_screen = _median_ms(lambda: ix.search_device(q, k, s, i))
    ix.set_precision(_lib.MQ_DTYPE_F32)
    ix.search_device(q, k, s2, i2)
    t_direct = _median_ms(lambda: ix.search_device(q, k, s2, i2))
    torch.cuda.synchronize()
    pl = planted >= 0
    assert bool((i[pl, 0] == planted[pl]).all())
    same = (i == i2).float().mean().item()
    assert same > 0.999, same
    assert _fp64_check(rows, q, s, i, k) == []
    assert ix.screen_skips == 0
    print("k=50 screen %.3f ms, direct %.3f ms, ratio %.3f" % (t_screen, t_direct, t_screen / t_direct))
    assert t_screen <= 1.2 * t_direct, (t_screen, t_direct)


def test_async_fallback_many_failures_is_one_pass(require_gpu):
    """130 of 256 queries made uncertifiable (70 exact copies of each at 1M rows): the
    asynchronous device re-run does all 130 in one MFMA pass - the whole screened search
    costs <= 1.35x the direct exact scan of the full batch - and returns the copies in id
    order, the direct scan's ids elsewhere."""
    import torch
    dev = torch.device("cuda", 0)
    rows = synth.corpus_device(N, 768, dev)
    q, _ = synth.queries_device(B, rows)
    rng = np.random.default_rng(9)
    fails = rng.choice(B, 130, replace=False)
    for n, j in enumerate(fails):
        rows[200 * n:200 * n + 70] = q[int(j)]
    ix = FlatIndex(dim=768, capacity=N)
    ix.add_device(rows)
    k = 5
    s, i = _out(k)
    s2, i2 = _out(k)
    ix.set_precision(_lib.MQ_DTYPE_F32)
    ix.search_device(q, k, s2, i2)
    t_direct = _median_ms(lambda: ix.search_device(q, k, s2, i2))
    ix.set_precision(_lib.MQ_DTYPE_F32_SCREEN)

    def rearm():
        # fold the last call's device count in, then reset the cooldown it starts: every
        # timed call takes the asynchronous path
        ix.screen_fallbacks
        ix.set_async_screen(True)

    rearm()
    ix.search_device(q, k, s, i)  # builds the bf16 shadow
    t_async = _median_ms(lambda: ix.search_device(q, k, s, i), prep=rearm)
    torch.cuda.synchronize()
    got = i.cpu().numpy()
    for n, j in enumerate(fails):
        assert got[j].tolist() == list(range(200 * n, 200 * n + 5)), j
    assert (i == i2).float().mean().item() > 0.999
    assert ix.screen_fallbacks >= 130 * 6
    print("130 failures: async %.3f ms, direct %.3f ms, ratio %.3f" % (t_async, t_direct, t_async / t_direct))
    assert t_async <= 1.35 * t_direct, (t_async, t_direct)
    # synchronous cooldown path: > 64 failures pass down to the split-f32 tier, same ids
    s3, i3 = _out(k)
    ix.search_device(q, k, s3, i3)
    torch.cuda.synchronize()
    assert bool((i3 == i).all())


@pytest.mark.parametrize("nf", [1, 33, 64, 65, 129, 256])
def test_async_fallback_tile_shapes(require_gpu, nf):
    """Failure counts on both sides of the narrow/wide switch (64) and a whole batch:
    the device picks the tile shape from the count; results equal the oracle."""
    c = synth.corpus(70000, 768, seed=nf, clustered=True)
    q, _ = synth.queries(B, c, seed=nf)
    rng = np.random.default_rng(nf)
    fails = rng.choice(B, nf, replace=False)
    for n, j in enumerate(fails):
        c[250 * n:250 * n + 66] = q[j]
    ix = FlatIndex(dim=768)
    ix.add(c)
    ix.set_precision(_lib.MQ_DTYPE_F32_SCREEN)
    s, i = ix.search(q, 8)
    assert check_topk(i, s, exact_scores(q, c), 8) == []
    for n, j in enumerate(fails):
        assert i[j].tolist() == list(range(250 * n, 250 * n + 8)), j
    assert ix.screen_fallbacks >= nf


def _near_tie_rows(q, spacing, count, rng):
    out = []
    for m in range(count):
        u = rng.standard_normal(q.shape[0]).astype(np.float64)
        u -= (u @ q) * q
        u /= np.linalg.norm(u)
        cm = 1.0 - m * spacing
        out.append(cm * q + np.sqrt(1.0 - cm * cm) * u)
    return np.array(out, np.float32)


def test_crowded_corpus_switches_bf16_tier_off(require_gpu):
    """200 of 256 queries have 70 rows 4e-5 apart (inside the bf16 bound, outside the
    split-f32 one): the first batch re-runs them on the device, the cooldown batches
    measure the failure share and switch the bf16 tier off, later batches go straight to
    the split-f32 screen - every batch exact."""
    rng = np.random.default_rng(5)
    c = rng.standard_normal((70000, 768)).astype(np.float32)
    q = rng.standard_normal((B, 768))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    for j in range(200):
        c[j * 70:(j + 1) * 70] = _near_tie_rows(q[j], 4e-5, 70, rng)
    q = q.astype(np.float32)
    ref = exact_scores(q, c)
    ix = FlatIndex(dim=768)
    ix.add(c)
    ix.set_precision(_lib.MQ_DTYPE_F32_SCREEN)
    for it in range(6):
        s, i = ix.search(q, 5)
        assert check_topk(i, s, ref, 5) == [], it
        for j in range(200):
            assert i[j].tolist() == list(range(j * 70, j * 70 + 5)), (it, j)
    assert ix.screen_skips >= 1
    assert ix.screen_passdowns >= 200
