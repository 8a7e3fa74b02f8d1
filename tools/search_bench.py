"""Time the fused scan per precision on a device-resident corpus (BASELINE configs 3/5):
exact f32, split f32 (x6) and the bf16 coarse + fp32 re-rank path; recall@k of each
against the exact path on the same queries."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mediquery-rag_amd"), ROOT]
import torch  # noqa: E402
from mediquery_hip import _lib, synth  # noqa: E402
from mediquery_hip.native import FlatIndex  # noqa: E402


def main(n=1_000_000, batches=(1, 256, 1024), ks=(5, 50)):
    dev = torch.device("cuda", 0)
    rows = synth.corpus_device(n, 768, dev)
    ix = FlatIndex(dim=768, capacity=n)
    ix.add_device(rows)
    res = {}
    for B in batches:
        q, planted = synth.queries_device(B, rows)
        for k in ks:
            ref_ids = None
            for name, prec in (("f32", _lib.MQ_DTYPE_F32), ("f32x6", _lib.MQ_DTYPE_F32X6),
                               ("bf16_rerank", _lib.MQ_DTYPE_BF16)):
                ix.set_precision(prec)
                s = torch.empty((B, k), device=dev)
                i = torch.empty((B, k), dtype=torch.int64, device=dev)
                for _ in range(2):
                    ix.search_device(q, k, s, i)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                reps = 5
                e0.record()
                for _ in range(reps):
                    ix.search_device(q, k, s, i)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                if ref_ids is None:
                    ref_ids = i.clone()
                recall = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(i, ref_ids)) / (B * k)
                res["B%d/k%d/%s" % (B, k, name)] = {"ms": round(ms, 3), "qps": round(B / ms * 1e3, 1),
                                                    "recall_vs_f32": round(recall, 5)}
                print("B=%5d k=%2d %-12s %8.3f ms  %10.1f q/s  recall %.5f" % (B, k, name, ms, B / ms * 1e3, recall),
                      flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
