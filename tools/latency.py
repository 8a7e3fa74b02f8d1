"""Single-query latency breakdown (BASELINE metric's "p50 single-query ms"): one query
(L=32 token ids) through the 12-layer encoder and the exact search over a 1M x 768
corpus, each part timed alone and together, device-resident inputs.

  python tools/latency.py [--rows 1000000] [--iters 200]
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mediquery-rag_amd"), ROOT]
import torch  # noqa: E402
from mediquery_hip import synth  # noqa: E402
from mediquery_hip.config import DMETA_BASE  # noqa: E402
from mediquery_hip.native import Encoder, FlatIndex  # noqa: E402


def p50(fn, iters):
    lat = []
    for it in range(iters + 10):
        torch.cuda.synchronize()
        a = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        if it >= 10:
            lat.append((time.perf_counter() - a) * 1e3)
    return round(statistics.median(lat), 4), round(min(lat), 4)


def stage_ms(obj, fn, n=20):
    obj.set_timing(True)
    fn()
    obj.read_timing()
    for _ in range(n):
        fn()
    out = {k: round(v / n, 4) for k, v in obj.read_timing().items()}
    obj.set_timing(False)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--exact-direct", action="store_true", help="search with MQ_DTYPE_F32 (default: the screen)")
    ap.add_argument("--encoder-seq-lens", default="",
                    help="comma list: only the single-query encoder p50 at these token counts")
    ap.add_argument("--rows-max", default="",
                    help="comma list of MQ_ENC_OPT_ROWS_MAX values to compare in --encoder-seq-lens mode")
    ap.add_argument("--opt", default="",
                    help="NAME=V1,V2,...: an encoder option (Encoder.OPTIONS) to sweep in --encoder-seq-lens mode")
    ap.add_argument("--e2e-opt", default="",
                    help="NAME=V1,V2,...: sweep an encoder option over encoder and end-to-end p50 (L=32, full corpus)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    if args.encoder_seq_lens:
        enc = Encoder(DMETA_BASE, device=0)
        q = torch.empty((1, 768), device=dev)
        res = {}
        name, vals = "rows_max", args.rows_max
        if args.opt:
            name, vals = args.opt.split("=")
        for rm in [int(x) for x in vals.split(",")] if vals else [None]:
            tag = ""
            if rm is not None:
                enc.set_option(name, rm)
                tag = "_%s%d" % (name.replace("_", ""), rm)
            for L in [int(x) for x in args.encoder_seq_lens.split(",")]:
                ids_np, mask_np = synth.token_batch(1, L)
                ids = torch.from_numpy(ids_np).to(dev)
                mask = torch.from_numpy(mask_np).to(dev)
                res["encoder_ms_L%d%s" % (L, tag)] = p50(lambda: enc.embed_device(ids, mask, q), args.iters)
        print(res, flush=True)
        return
    corpus = synth.corpus_device(args.rows, 768, dev)
    ix = FlatIndex(dim=768, capacity=args.rows, device=0)
    ix.add_device(corpus)
    del corpus
    from mediquery_hip import _lib
    ix.set_precision(_lib.MQ_DTYPE_F32 if args.exact_direct else _lib.MQ_DTYPE_F32_SCREEN)
    enc = Encoder(DMETA_BASE, device=0)
    ids_np, mask_np = synth.token_batch(1, 32)
    ids = torch.from_numpy(ids_np).to(dev)
    mask = torch.from_numpy(mask_np).to(dev)
    q = torch.empty((1, 768), device=dev)
    s = torch.empty((1, args.k), device=dev)
    i = torch.empty((1, args.k), dtype=torch.int64, device=dev)
    if args.e2e_opt:
        name, vals = args.e2e_opt.split("=")
        res = {}
        for v in [int(x) for x in vals.split(",")]:
            enc.set_option(name, v)
            res["%s=%d" % (name, v)] = {
                "encoder_ms": p50(lambda: enc.embed_device(ids, mask, q), args.iters),
                "end_to_end_ms": p50(lambda: (enc.embed_device(ids, mask, q), ix.search_device(q, args.k, s, i)),
                                     args.iters)}
        print(res, flush=True)
        return
    res = {"note": "(p50 ms, min ms) per call; *_stage_ms = device time per kernel class"}
    res["encoder_ms"] = p50(lambda: enc.embed_device(ids, mask, q), args.iters)
    res["search_ms"] = p50(lambda: ix.search_device(q, args.k, s, i), args.iters)
    res["end_to_end_ms"] = p50(lambda: (enc.embed_device(ids, mask, q), ix.search_device(q, args.k, s, i)),
                               args.iters)
    enc.set_graphs(True)
    res["encoder_graph_ms"] = p50(lambda: enc.embed_device(ids, mask, q), args.iters)
    enc.set_graphs(False)
    res["encoder_stage_ms"] = stage_ms(enc, lambda: enc.embed_device(ids, mask, q))
    res["search_stage_ms"] = stage_ms(ix, lambda: ix.search_device(q, args.k, s, i))
    print(res, flush=True)


if __name__ == "__main__":
    main()
