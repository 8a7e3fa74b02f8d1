"""Time the encoder's batched GEMM shapes (M = 8192 = 256 queries x 32 tokens, BERT-base)
on the exact-f32 tiles, the split-f32 (x6) tiles of gemm_f32.hpp and the pre-split K2p
tiles (gemm_x6p.hip).  Prints one JSON line per (shape, kernel): us per launch and
fp32-equivalent TFLOP/s (2 M N K / t).  Run on the GPU box from the repo root."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mediquery-rag_amd"))

import torch  # noqa: E402

from mediquery_hip import _lib  # noqa: E402

SHAPES = {"qkv": (8192, 2304, 768, 0), "out_proj": (8192, 768, 768, 3), "ffn_up": (8192, 3072, 768, 1),
          "ffn_down": (8192, 768, 3072, 3), "kv_last": (8192, 1536, 768, 0)}


REPS = 3


def timed(fn, iters):
    """Median over REPS runs of `iters` back-to-back launches (us per launch)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    runs = []
    for _ in range(REPS):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        runs.append(e0.elapsed_time(e1) * 1000.0 / iters)
    return sorted(runs)[len(runs) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--f32-tiles", default="0,1,5,6,7")
    ap.add_argument("--x6p-tiles", default="-1,0,1,2,3")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    global REPS
    REPS = a.reps
    dev = torch.device("cuda", 0)
    st = _lib.stream_handle()
    for name in a.shapes.split(","):
        M, N, K, epi = SHAPES[name]
        g = torch.Generator(device=dev).manual_seed(1)
        A = torch.randn(M, K, device=dev, generator=g)
        W = torch.randn(N, K, device=dev, generator=g) * 0.05
        b = torch.randn(N, device=dev, generator=g)
        R = torch.randn(M, N, device=dev, generator=g)
        out = torch.empty(M, N, device=dev)
        w3 = torch.empty(_lib.lib().mq_debug_w3_bytes(N, K), dtype=torch.uint8, device=dev)
        _lib.call("mq_debug_split_w3", _lib.ptr(W), N, K, _lib.ptr(w3), st)
        flop = 2.0 * M * N * K
        ref = None
        for t in [int(x) for x in a.f32_tiles.split(",") if x]:
            us = timed(lambda: _lib.call("mq_debug_gemm_f32", _lib.ptr(A), _lib.ptr(W), _lib.ptr(b), _lib.ptr(R),
                                         _lib.ptr(out), M, N, K, epi, t, st), a.iters)
            if t == 5:
                ref = out.clone()
            print(json.dumps({"shape": name, "kernel": "f32_tile%d" % t, "us": round(us, 2),
                              "tflops": round(flop / us / 1e6, 2)}), flush=True)
        for t in [int(x) for x in a.x6p_tiles.split(",") if x]:
            us = timed(lambda: _lib.call("mq_debug_gemm_x6p", _lib.ptr(A), _lib.ptr(w3), _lib.ptr(b), _lib.ptr(R),
                                         _lib.ptr(out), M, N, K, epi, t, st), a.iters)
            same = None if ref is None else bool(torch.equal(out, ref))
            print(json.dumps({"shape": name, "kernel": "x6p_tile%d" % t, "us": round(us, 2),
                              "tflops": round(flop / us / 1e6, 2), "frac_417": round(flop / us / 1e6 / 416.7, 3),
                              "bit_identical_to_x6": same}), flush=True)


if __name__ == "__main__":
    main()
