"""Ingest throughput (reference `Chroma.from_documents` at
src/ingest_medical.py:106-110): documents/s through `HipChroma.from_texts`' path -
`HipBertEmbeddings.embed_array` (char tokenizer, length-sorted batches of 256, one HIP
encoder forward per batch) + `FlatIndex.add` - on synthetic chunks whose texts are drawn
from the reference corpus (the 154 parsed docs of data/medical_data.txt, 25-399 tokens).

  python tools/ingest_bench.py [--docs 20000]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mediquery-rag_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mediquery_hip.config import DMETA_BASE  # noqa: E402
from mediquery_hip.embeddings import HipBertEmbeddings  # noqa: E402
from mediquery_hip.native import FlatIndex  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=20000)
    ap.add_argument("--chunk", type=int, default=4096)
    args = ap.parse_args()
    with open(os.path.join(ROOT, "tests", "golden", "corpus_docs.json"), encoding="utf-8") as f:
        base = [d["page_content"] for d in json.load(f)["docs"]]
    rng = np.random.default_rng(0)
    texts = [base[i] for i in rng.integers(0, len(base), args.docs)]
    emb = HipBertEmbeddings(synthetic=True)
    ix = FlatIndex(dim=768, capacity=args.docs)
    emb.embed_array(texts[:512])  # warm-up (graph capture per shape happens in the run too)
    _, mask = emb.tokenizer(texts)
    lens = mask.sum(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for n, s in enumerate(range(0, len(texts), args.chunk)):
        ix.add(emb.embed_array(texts[s:s + args.chunk]))
        if n % 25 == 24:  # progress (a long run must keep writing)
            print("progress %d docs %.1f s" % (s + args.chunk, time.perf_counter() - t0), file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    flops = sum(DMETA_BASE.flops_per_sequence(int(L)) for L in lens)
    print(json.dumps({"docs": args.docs, "docs_per_s": round(args.docs / dt, 1),
                      "tokens_per_s": round(float(lens.sum()) / dt, 1),
                      "mean_tokens": round(float(lens.mean()), 1),
                      "encoder_tflops_effective": round(flops / dt / 1e12, 2),
                      "seconds": round(dt, 3), "rows_indexed": len(ix)}))


if __name__ == "__main__":
    main()
