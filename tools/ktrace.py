"""Phase timeline of the few-row kernels from a -DMQ_KTRACE measurement build.

  MQ_LIB_PATH=variants/ktrace.so python tools/ktrace.py [--L 32]

Runs single-query forwards (mean pooling, so every layer has the same shapes), then
reads mq_ktrace: per kernel class, thread 0 of every workgroup stamped the 100 MHz wall
clock at its phase boundaries.  Prints, per class, the median over workgroups of each
phase (us, relative to that workgroup's first stamp) and the spread of workgroup start
times (dispatch skew) and end times.
Slots: rows_gemm_kernel 0 start, 1 LayerNorm rows ready (LN input), 2 after the LDS
barrier, 3 MFMA loop done, 4 partial tiles summed, 5 stored; K3o 0 start, 1 operands
landed, 2 attention done (wave 0), 3 after the ctx barrier, 4 projection MFMAs done,
5 partials summed, 6 stored.
"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mediquery-rag_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mediquery_hip import _lib, synth  # noqa: E402
from mediquery_hip.config import BertConfig, POOL_MEAN  # noqa: E402
from mediquery_hip.native import Encoder  # noqa: E402

NAMES = ["qkv (rows_gemm EPI_BIAS)", "ffn_up (rows_gemm GELU)", "ffn_down (rows_gemm RESID)", "attn+oproj (K3o)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=32)
    args = ap.parse_args()
    lib = _lib.lib()
    fn = lib.mq_debug_ktrace_read
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    n = 4 * 1024 * 8
    buf = np.zeros(n, np.int64)
    cfg = BertConfig(pooling=POOL_MEAN)
    enc = Encoder(cfg, device=0)
    dev = torch.device("cuda", 0)
    ids_np, mask_np = synth.token_batch(1, args.L)
    ids, mask = torch.from_numpy(ids_np).to(dev), torch.from_numpy(mask_np).to(dev)
    q = torch.empty((1, cfg.hidden), device=dev)
    for _ in range(20):
        enc.embed_device(ids, mask, q)
    torch.cuda.synchronize()
    res = {}
    for rep in range(5):
        fn(buf.ctypes.data, n)  # clear
        enc.embed_device(ids, mask, q)
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data, n) == 0
        t = buf.reshape(4, 1024, 8)
        for r in range(4):
            wgs = [w for w in range(1024) if t[r, w, 0] > 0]
            if not wgs:
                continue
            start = min(t[r, w, 0] for w in wgs)
            for slot in range(1, 8):
                d = [(t[r, w, slot] - t[r, w, 0]) / 100.0 for w in wgs if t[r, w, slot] > 0]
                if d:
                    res.setdefault((r, slot), []).append(statistics.median(d))
            res.setdefault((r, "skew"), []).append(statistics.median((t[r, w, 0] - start) / 100.0 for w in wgs))
            res.setdefault((r, "maxskew"), []).append(max((t[r, w, 0] - start) / 100.0 for w in wgs))
            last = max(max(t[r, w, s] for s in range(8)) for w in wgs)
            res.setdefault((r, "span"), []).append((last - start) / 100.0)
            res.setdefault((r, "wgs"), []).append(len(wgs))
    for r in range(4):
        keys = [k for k in res if k[0] == r]
        if not keys:
            continue
        print(NAMES[r])
        for k in sorted(keys, key=lambda k: str(k[1])):
            print("   %-8s %8.2f" % (k[1], statistics.median(res[k])))


if __name__ == "__main__":
    main()
