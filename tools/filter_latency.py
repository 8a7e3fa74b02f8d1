"""Filtered vs unfiltered search latency at the VectorStore surface:
`HipChroma.similarity_search_by_vector(q, k=5, filter=...)` over N synthetic rows whose
metadata carries a 16-value `tag` and an integer `n`; the filter passes ~1/2 or ~1/16 of
the rows.  Reports p50 ms for: no filter, a repeated filter and a fresh filter every call
(r5: the where-mask built on the device from the metadata code columns, then the masked
int8 certified search; r3/r4 gathered the allowed rows through a host row list), and the
masked searches that fell back to the device gather.  r6: the 256-query batched filtered
search (`similarity_search_batch(filter=)`: ONE masked call - the bf16 threshold scan with
the row mask) against the unfiltered 256-query batch, and `delete` of 1k ids with the store
in memory (auto_persist off: the device compaction + the host lists, no slab rewrite).

  python tools/filter_latency.py [--rows 1000000] [--iters 50]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mediquery-rag_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mediquery_hip import synth  # noqa: E402
from mediquery_hip.vectorstore import HipChroma  # noqa: E402


def p50(fn, iters):
    lat = []
    for it in range(iters + 3):
        a = time.perf_counter()
        fn(it)
        if it >= 3:
            lat.append((time.perf_counter() - a) * 1e3)
    return round(statistics.median(lat), 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    n = args.rows
    dev = torch.device("cuda", 0)
    emb = torch.nn.functional.normalize(synth.corpus_device(n, 768, dev), dim=1).cpu().numpy()
    rng = np.random.default_rng(0)
    tags = rng.integers(0, 16, n)
    metas = [{"tag": "t%d" % t, "n": int(i % 100)} for i, t in enumerate(tags)]
    store = HipChroma(dim=768, auto_persist=False)
    t0 = time.perf_counter()
    store.add_embeddings(emb, ["doc %d" % i for i in range(n)], metas, ["id%d" % i for i in range(n)])
    t_add = time.perf_counter() - t0
    qs = emb[rng.integers(0, n, 64)] + 0.01 * rng.standard_normal((64, 768)).astype(np.float32)
    out = {"rows": n, "add_s": round(t_add, 2)}
    out["unfiltered_ms"] = p50(lambda i: store.similarity_search_by_vector(qs[i % 64], k=5), args.iters)
    out["repeated_filter_half_ms"] = p50(
        lambda i: store.similarity_search_by_vector(qs[i % 64], k=5, filter={"n": {"$lt": 50}}), args.iters)
    out["repeated_filter_16th_ms"] = p50(
        lambda i: store.similarity_search_by_vector(qs[i % 64], k=5, filter={"tag": "t3"}), args.iters)
    out["fresh_filter_16th_ms"] = p50(
        lambda i: store.similarity_search_by_vector(qs[i % 64], k=5, filter={"tag": "t%d" % (i % 16)}), args.iters)
    out["fresh_filter_half_ms"] = p50(
        lambda i: store.similarity_search_by_vector(qs[i % 64], k=5, filter={"n": {"$lt": 40 + i % 20}}), args.iters)
    out["masked_gathers"] = store._index.masked_gathers
    # batches of 256 query vectors: one device search / one masked call for all of them
    qb = emb[rng.integers(0, n, 256)] + 0.01 * rng.standard_normal((256, 768)).astype(np.float32)
    ix = store._index
    out["batch256_unfiltered_ms"] = p50(lambda i: ix.search(qb, 5), 10)
    for name, f in (("half", {"n": {"$lt": 50}}), ("16th", {"tag": "t3"})):
        g0 = ix.masked_gathers
        out["batch256_filter_%s_ms" % name] = p50(lambda i, f=f: ix.search_masked(qb, 5, store._cols.dmask(f, 0)), 10)
        out["batch256_filter_%s_uncertified" % name] = ix.masked_gathers - g0
        out["batch256_filter_%s_ratio" % name] = round(out["batch256_filter_%s_ms" % name] / out["batch256_unfiltered_ms"], 2)
    t0 = time.perf_counter()
    store.delete(["id%d" % i for i in range(0, n, 1000)])
    out["delete_1k_of_n_s"] = round(time.perf_counter() - t0, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
