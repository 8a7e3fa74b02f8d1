"""Time the batched bf16 screen (K9t threshold scan + tau + select + fp32 re-rank +
certificate) on a device-resident 1M x 768 corpus; stage split and the tiled-scan
comparison.  Run under rocprofv3 --kernel-trace --stats for per-kernel durations."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mediquery-rag_amd"), ROOT]
import torch  # noqa: E402
from mediquery_hip import _lib, synth  # noqa: E402
from mediquery_hip.native import FlatIndex  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=1_000_000)
ap.add_argument("--batches", default="256,1024")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--tiled", action="store_true", help="also time the tiled scan")
args = ap.parse_args()
dev = torch.device("cuda", 0)
rows = synth.corpus_device(args.rows, 768, dev)
ix = FlatIndex(dim=768, capacity=args.rows)
ix.add_device(rows)
for B in [int(b) for b in args.batches.split(",")]:
    q, planted = synth.queries_device(B, rows)
    for k, prec in ((5, _lib.MQ_DTYPE_F32_SCREEN), (50, _lib.MQ_DTYPE_BF16)):
        ix.set_precision(prec)
        s = torch.empty((B, k), device=dev)
        i = torch.empty((B, k), dtype=torch.int64, device=dev)
        for variant in ([True, False] if args.tiled else [True]):
            ix.set_threshold_scan(variant)
            ix.search_device(q, k, s, i)
            torch.cuda.synchronize()
            ix.set_timing(True)
            t0 = time.perf_counter()
            for _ in range(args.iters):
                ix.search_device(q, k, s, i)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / args.iters * 1e3
            st = {a: round(b / args.iters, 4) for a, b in ix.read_timing().items()}
            ix.set_timing(False)
            print("B=%4d k=%2d prec=%d %-6s %.3f ms/search stages %s gb/s(shadow) %.0f" % (
                B, k, prec, "thresh" if variant else "tiled", ms, st,
                args.rows * 768 * 2 / (st["flat_search_kernel"] * 1e-3) / 1e9), flush=True)
        ix.set_threshold_scan(True)
