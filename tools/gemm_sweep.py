"""Time the fp32 MFMA GEMM core per tile geometry on the encoder's shapes (B=256, L=32)
through the mq_debug_gemm_f32 hook.  Prints TFLOP/s per (shape, tile)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mediquery-rag_amd"), ROOT]
import torch  # noqa: E402
from mediquery_hip import _lib  # noqa: E402

SHAPES = {"qkv": (8192, 2304, 768), "out_proj": (8192, 768, 768), "ffn_up": (8192, 3072, 768),
          "ffn_down": (8192, 768, 3072)}
TILES = {0: "f32_128x128", 1: "f32_128x96", 2: "f32_128x64", 3: "f32_32x128", 5: "x6_128x128", 6: "x6_128x96", 7: "x6_128x64", 8: "f32w_128x192", 9: "x6w_128x192"}


def main():
    # optional filters: --shapes qkv,ffn_up --tiles 1,6 --iters 20
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--tiles", default=",".join(str(t) for t in TILES))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--epi", type=int, default=-1, help="override the epilogue (0 bias, 1 GELU erf, 2 GELU tanh, 3 residual)")
    args = ap.parse_args()
    shapes = {k: SHAPES[k] for k in args.shapes.split(",")}
    tiles = {int(t): TILES[int(t)] for t in args.tiles.split(",")}
    dev = torch.device("cuda", 0)
    res = {}
    for name, (M, N, K) in shapes.items():
        A = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev) * 0.05
        b = torch.randn(N, device=dev)
        R = torch.randn(M, N, device=dev)
        out = torch.empty(M, N, device=dev)
        epi = 1 if name == "ffn_up" else (3 if name in ("out_proj", "ffn_down") else 0)
        if args.epi >= 0:
            epi = args.epi
        for t, tname in tiles.items():
            def run():
                _lib.call("mq_debug_gemm_f32", _lib.ptr(A), _lib.ptr(W), _lib.ptr(b), _lib.ptr(R),
                          _lib.ptr(out), M, N, K, epi, t, _lib.stream_handle())
            for _ in range(3):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = args.iters
            e0.record()
            for _ in range(n):
                run()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / n
            res["%s/%s/epi%d" % (name, tname, epi)] = {"ms": round(ms, 4), "tflops": round(2 * M * N * K / ms / 1e9, 1)}
    print(json.dumps(res, indent=1))
    for k, v in res.items():
        print("%-32s %6.1f TF" % (k, v["tflops"]))


if __name__ == "__main__":
    main()
