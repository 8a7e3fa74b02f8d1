"""Dump encoder / GEMM outputs of the library at MQ_LIB_PATH (or the in-tree one) for a
bitwise A/B between two builds: python tools/ab_outputs.py OUT.npz; then compare."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mediquery-rag_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mediquery_hip import _lib, synth  # noqa: E402
from mediquery_hip.config import DMETA_BASE  # noqa: E402
from mediquery_hip.native import Encoder  # noqa: E402

if sys.argv[1] == "compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    for k in a.files:
        same = np.array_equal(a[k], b[k])
        print("%-14s %s  max|d| %.3g" % (k, "bit-identical" if same else "DIFFERENT",
                                        float(np.abs(a[k] - b[k]).max())))
    sys.exit(0)
out = {}
enc = Encoder(DMETA_BASE, device=0)
for B, L in ((256, 32), (3, 128), (1, 32), (40, 17)):
    ids, mask = synth.token_batch(B, L)
    if B == 40:
        mask[5, 9:] = 0
    out["enc_%dx%d" % (B, L)] = enc.embed(ids, mask)
dev = torch.device("cuda", 0)
g = torch.Generator(device="cpu").manual_seed(0)
for M, N, K, epi in ((8192, 2304, 768, 0), (8192, 3072, 768, 1), (8192, 768, 3072, 3), (300, 768, 768, 3),
                     (33, 2304, 768, 0)):
    A = torch.randn(M, K, generator=g).to(dev)
    W = (torch.randn(N, K, generator=g) * 0.05).to(dev)
    bias = torch.randn(N, generator=g).to(dev)
    R = torch.randn(M, N, generator=g).to(dev)
    for tile in (0, 1, 2, 3, 8):
        o = torch.empty(M, N, device=dev)
        _lib.call("mq_debug_gemm_f32", _lib.ptr(A), _lib.ptr(W), _lib.ptr(bias), _lib.ptr(R), _lib.ptr(o),
                  M, N, K, epi, tile, _lib.stream_handle())
        torch.cuda.synchronize()
        out["gemm_%d_%d_%d_t%d" % (M, N, K, tile)] = o.cpu().numpy()
np.savez(sys.argv[1], **out)
print("saved", len(out))
