import os, sys, time
sys.path[:0] = ["/root/repo/mediquery-rag_amd", "/root/repo"]
import torch
from mediquery_hip import _lib, synth
from mediquery_hip.native import FlatIndex
dev = torch.device("cuda", 0)
rows = synth.corpus_device(1_000_000, 768, dev)
ix = FlatIndex(dim=768, capacity=1_000_000); ix.add_device(rows)
for B in (256, 1024):
    q, planted = synth.queries_device(B, rows)
    for k in (5, 50):
        res = {}
        for name, p in (("f32", 0), ("screen", 3), ("x6", 2)):
            ix.set_precision(p)
            s = torch.empty((B, k), device=dev); i = torch.empty((B, k), dtype=torch.int64, device=dev)
            ix.search_device(q, k, s, i); torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(10): ix.search_device(q, k, s, i)
            torch.cuda.synchronize()
            res[name] = ((time.perf_counter() - t) / 10 * 1e3, i.clone(), s.clone())
        same = (res["screen"][1] == res["f32"][1]).float().mean().item()
        print("B=%d k=%d f32 %.3f ms screen %.3f ms x6 %.3f ms  ids equal %.5f  max|ds| %.2e fallbacks %d" % (
            B, k, res["f32"][0], res["screen"][0], res["x6"][0], same,
            (res["screen"][2] - res["f32"][2]).abs().max().item(), ix.screen_fallbacks), flush=True)
