"""User-level single-query latency of the drop-in: `HipChroma.similarity_search(text, k=5)`
(the call at reference src/agents/nodes.py:93) over a 1M-row store, broken into its parts -
tokenise, embed (host ids -> device -> host vector), search (host vector -> device ->
host ids / scores), Document assembly.  Store rows are seeded unit vectors added through
`add_embeddings` (embedding 1M texts first would only add ingest time); queries are
Chinese symptom questions through the seeded encoder (char tokenizer).

  python tools/langchain_latency.py [--rows 1000000] [--iters 100]
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mediquery-rag_amd"), ROOT]
import numpy as np  # noqa: E402
from mediquery_hip import synth  # noqa: E402
from mediquery_hip.embeddings import HipBertEmbeddings  # noqa: E402
from mediquery_hip.vectorstore import HipChroma  # noqa: E402

QUERIES = ["血糖高如何治疗?", "高血压患者饮食要注意什么", "头痛发热咳嗽是感冒吗", "心脏病的早期症状有哪些",
           "糖尿病能吃水果吗", "失眠怎么办", "胃痛应该吃什么药", "孩子发烧39度怎么处理"]


def p50(xs):
    return round(statistics.median(xs), 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=100)
    args = ap.parse_args()
    emb = HipBertEmbeddings(synthetic=True)
    store = HipChroma(embedding_function=emb, auto_persist=False)
    rows = synth.corpus(args.rows, 768, seed=1)
    store.add_embeddings(rows, ["doc %d" % i for i in range(args.rows)], [{} for _ in range(args.rows)],
                         ["id%d" % i for i in range(args.rows)])
    del rows
    for q in QUERIES:  # warm-up (shadows, first launches)
        store.similarity_search(q, k=5)
    tot, tok, enc, srch, docs = [], [], [], [], []
    for it in range(args.iters):
        q = QUERIES[it % len(QUERIES)]
        a = time.perf_counter()
        store.similarity_search(q, k=5)
        tot.append((time.perf_counter() - a) * 1e3)
        a = time.perf_counter()
        ids, mask = emb.tokenizer([q])
        b = time.perf_counter()
        v = emb.embed_query(q)
        c = time.perf_counter()
        rr = store._search_rows(np.asarray(v, np.float32), 5)
        d = time.perf_counter()
        [store._doc(r) for r, _ in rr]
        e = time.perf_counter()
        tok.append((b - a) * 1e3)
        enc.append((c - b) * 1e3)
        srch.append((d - c) * 1e3)
        docs.append((e - d) * 1e3)
    print({"rows": args.rows, "similarity_search_p50_ms": p50(tot), "tokenize_p50_ms": p50(tok),
           "embed_query_p50_ms (incl. tokenize)": p50(enc), "search_p50_ms": p50(srch),
           "documents_p50_ms": p50(docs)}, flush=True)


if __name__ == "__main__":
    main()
