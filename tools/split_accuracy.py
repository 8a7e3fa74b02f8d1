"""Accuracy of the GEMM arithmetics against float64 (mq_debug_gemm_f32): exact f32 MFMA
(tile 0) vs the 3-way bf16 split (tile 5) of the loaded library - max and RMS error on
the encoder's shapes with encoder-like operand scales.

  python tools/split_accuracy.py      (MQ_LIB_PATH selects a variant build)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mediquery-rag_amd"), ROOT]
import torch  # noqa: E402
from mediquery_hip import _lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    res = {}
    for M, N, K in ((1024, 768, 768), (1024, 3072, 768), (1024, 768, 3072)):
        A = torch.randn(M, K, device=dev, generator=g)
        W = torch.randn(N, K, device=dev, generator=g) * 0.02
        b = torch.zeros(N, device=dev)
        ref = A.double() @ W.double().T
        for tile in (0, 5):
            out = torch.empty(M, N, device=dev)
            _lib.call("mq_debug_gemm_f32", _lib.ptr(A), _lib.ptr(W), _lib.ptr(b), _lib.ptr(b), _lib.ptr(out),
                      M, N, K, 0, tile, _lib.stream_handle())
            torch.cuda.synchronize()
            e = out.double() - ref
            res["%dx%dx%d/tile%d" % (M, N, K, tile)] = (float(e.abs().max()), float(e.pow(2).mean().sqrt()))
    for k, (mx, rms) in res.items():
        print("%-22s max %.3e  rms %.3e" % (k, mx, rms))


if __name__ == "__main__":
    main()
