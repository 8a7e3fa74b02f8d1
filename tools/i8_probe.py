"""Single-query int8 screen (K9q) on the bench corpus: certification rate, timing, and
the numbers behind the certificate (the int8 shadow's error maximum vs the gap between
the k-th and 64-th best exact scores).

  python tools/i8_probe.py [--rows 1000000] [--queries 64]
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mediquery-rag_amd"), ROOT]
import torch  # noqa: E402
from mediquery_hip import _lib, synth  # noqa: E402
from mediquery_hip.config import DMETA_BASE  # noqa: E402
from mediquery_hip.native import Encoder, FlatIndex  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--queries", type=int, default=64)
    ap.add_argument("--k", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    rows = synth.corpus_device(args.rows, 768, dev)
    ix = FlatIndex(dim=768, capacity=args.rows, device=0)
    ix.add_device(rows)
    rows = torch.nn.functional.normalize(rows, dim=1)
    # the int8 shadow's error maximum, recomputed with the kernel's rounding
    dmax = 0.0
    for s in range(0, args.rows, 1 << 17):
        r = rows[s:s + (1 << 17)]
        amax = r.abs().amax(dim=1, keepdim=True)
        q8 = torch.clamp(torch.round(r * (127.0 / amax)), -127, 127)
        dmax = max(dmax, float((r - (amax / 127.0) * q8).norm(dim=1).max()))
    enc = Encoder(DMETA_BASE, device=0)
    ids_np, mask_np = synth.token_batch(1, 32)
    qe = torch.empty((1, 768), device=dev)
    enc.embed_device(torch.from_numpy(ids_np).to(dev), torch.from_numpy(mask_np).to(dev), qe)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    qs = torch.nn.functional.normalize(torch.randn((args.queries, 768), generator=g, device=dev), dim=1)
    qs = torch.cat([qe, qs])
    top = torch.topk(qs @ rows.T, 64, dim=1).values
    gaps = (top[:, args.k - 1] - top[:, 63]).tolist()
    ix.set_precision(_lib.MQ_DTYPE_F32_SCREEN)
    s = torch.empty((1, args.k), device=dev)
    i = torch.empty((1, args.k), dtype=torch.int64, device=dev)
    res = {"rows": args.rows, "dmax_int8": round(dmax, 6),
           "gap_k_to_64_encoder_query": round(gaps[0], 6),
           "gap_k_to_64_random_median": round(statistics.median(gaps[1:]), 6),
           "gap_k_to_64_random_min": round(min(gaps[1:]), 6)}
    for on in (True, False):
        ix.set_int8_screen(on)
        p0 = ix.screen_passdowns
        lat = []
        for j in range(qs.shape[0]):
            q1 = qs[j:j + 1].contiguous()
            torch.cuda.synchronize()
            a = time.perf_counter()
            ix.search_device(q1, args.k, s, i)
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - a) * 1e3)
        res["int8_on" if on else "int8_off"] = {"passdowns": ix.screen_passdowns - p0,
                                                "p50_ms": round(statistics.median(lat), 4)}
    ix.set_int8_screen(True)
    ix.set_timing(True)
    for _ in range(20):
        ix.search_device(qs[1:2].contiguous(), args.k, s, i)
    res["stage_ms_int8_random_query"] = {k: round(v / 20, 4) for k, v in ix.read_timing().items()}
    print(res, flush=True)


if __name__ == "__main__":
    main()
