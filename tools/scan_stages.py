"""Per-stage device time of the screened / bf16 searches on a 1M x 768 device corpus:
scan (K9) and merge (K10) from the index's HIP-event timeline, plus the wall time of the
whole call (re-rank, certificate, read-back included).  MQ_LIB_PATH selects a library
variant (experiments)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mediquery-rag_amd"), ROOT]
import torch  # noqa: E402
from mediquery_hip import _lib, synth  # noqa: E402
from mediquery_hip.native import FlatIndex  # noqa: E402

dev = torch.device("cuda", 0)
rows = synth.corpus_device(1_000_000, 768, dev)
ix = FlatIndex(dim=768, capacity=1_000_000)
ix.add_device(rows)
print("lib", _lib.LIB_PATH, flush=True)
for name, prec, B, k in (("screen", 3, 256, 5), ("screen", 3, 1, 5), ("bf16_cfg5", 1, 256, 50),
                         ("x6", 2, 256, 5), ("f32", 0, 256, 5), ("f32", 0, 1, 5)):
    ix.set_precision(prec)
    q, _ = synth.queries_device(B, rows, seed=11)
    s = torch.empty((B, k), device=dev)
    i = torch.empty((B, k), dtype=torch.int64, device=dev)
    for _ in range(3):
        ix.search_device(q, k, s, i)
    torch.cuda.synchronize()
    ix.set_timing(True)
    n = 20
    t = time.perf_counter()
    for _ in range(n):
        ix.search_device(q, k, s, i)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / n * 1e3
    st = {a: round(b / n, 4) for a, b in ix.read_timing().items()}
    ix.set_timing(False)
    print("%-9s B=%3d k=%2d wall %.4f ms stages %s fallbacks %d passdowns %d" % (
        name, B, k, wall, st, ix.screen_fallbacks, ix.screen_passdowns), flush=True)
