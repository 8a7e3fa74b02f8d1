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


def small_batch_crossover(ix, rows, dev, batches=(1, 2, 4, 8, 16, 32), k=5):
    """Streaming kernel (threshold 16) vs narrow MFMA tiles (threshold 0) per batch."""
    out = {}
    ix.set_precision(_lib.MQ_DTYPE_F32)
    for B in batches:
        q, _ = synth.queries_device(B, rows)
        s = torch.empty((B, k), device=dev)
        i = torch.empty((B, k), dtype=torch.int64, device=dev)
        for thr in (16, 0):
            ix.set_stream_threshold(thr)
            for _ in range(3):
                ix.search_device(q, k, s, i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                ix.search_device(q, k, s, i)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            name = "stream" if thr else "mfma"
            out["B%d/%s" % (B, name)] = round(ms, 4)
            print("B=%3d %-6s %7.3f ms  (%.0f GB/s row stream)" % (B, name, ms, rows.numel() * 4 / ms / 1e6),
                  flush=True)
    ix.set_stream_threshold(8)
    # stage split (scan vs merge) and overflow re-scans at k = 5 / 50
    for B, prec in ((1, 0), (8, 0), (64, 0), (256, 0), (256, _lib.MQ_DTYPE_F32X6), (256, _lib.MQ_DTYPE_BF16),
                    (1024, _lib.MQ_DTYPE_BF16)):
        ix.set_precision(prec)
        q, _ = synth.queries_device(B, rows)
        for kk in (5, 50):
            s = torch.empty((B, kk), device=dev)
            i = torch.empty((B, kk), dtype=torch.int64, device=dev)
            ix.search_device(q, kk, s, i)
            torch.cuda.synchronize()
            r0 = ix.rescans
            ix.set_timing(True)
            for _ in range(5):
                ix.search_device(q, kk, s, i)
            t = ix.read_timing()
            ix.set_timing(False)
            print("B=%4d k=%2d prec %d stages %s rescans %d" % (B, kk, prec, {a: round(b / 5, 4) for a, b in t.items()},
                                                               ix.rescans - r0), flush=True)
    ix.set_precision(_lib.MQ_DTYPE_F32)
    return out


def main(n=1_000_000, batches=(1, 256, 1024), ks=(5, 50)):
    dev = torch.device("cuda", 0)
    rows = synth.corpus_device(n, 768, dev)
    ix = FlatIndex(dim=768, capacity=n)
    ix.add_device(rows)
    res = {"crossover": small_batch_crossover(ix, rows, dev)}
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
