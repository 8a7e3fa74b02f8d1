"""Data-parallel ingest through the HIP encoder: the reference's
`Chroma.from_documents(documents=docs, embedding=OllamaEmbeddings(...))`
(src/ingest_medical.py:104-110) embeds every chunk on one server; here each of two ranks
(gloo, both on cuda:0) runs `ingest_sharded(texts, HipBertEmbeddings(...).embed_array,
FlatIndex.add)` over its contiguous block, then `ShardedSearcher` answers the config-1
queries over the two shards with one packed candidate all-gather.  Ids and scores must
equal a single-process ingest + search, and the float64 oracle on the same embeddings."""
import json
import os
import socket

import numpy as np
import pytest

from oracle.flat import check_topk, exact_scores

pytestmark = pytest.mark.gpu

COPIES, K = 4, 5


def _texts(golden):
    docs = json.load(open(os.path.join(golden, "corpus_docs.json"), encoding="utf-8"))["docs"]
    qs = json.load(open(os.path.join(golden, "config1_queries.json"), encoding="utf-8"))["queries"]
    # the 154 reference chunks x COPIES, each copy tagged so rows differ (plus the corpus's
    # own exact duplicates, which stay tied)
    texts = [d["page_content"] + ("" if c == 0 else " 第%d版" % c) for c in range(COPIES) for d in docs]
    return texts, qs


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, golden, out_q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "mediquery-rag_amd"), root]
    import torch
    import torch.distributed as dist
    from mediquery_hip import HipBertEmbeddings
    from mediquery_hip.distributed import ShardedSearcher, ingest_sharded
    from mediquery_hip.native import FlatIndex
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        texts, qs = _texts(golden)
        emb = HipBertEmbeddings(synthetic=True, batch_size=64)
        ix = FlatIndex(dim=768, device=0)
        off, cnt = ingest_sharded(texts, emb.embed_array, ix.add, chunk=100)
        assert len(ix) == cnt
        q = torch.from_numpy(emb.embed_array(qs)).to(dev)
        s_loc = torch.empty((len(qs), K), dtype=torch.float32, device=dev)
        i_loc = torch.empty((len(qs), K), dtype=torch.int64, device=dev)

        def local(qq, k):
            ix.search_device(qq, k, s_loc[:qq.shape[0]], i_loc[:qq.shape[0]])
            return s_loc[:qq.shape[0]], i_loc[:qq.shape[0]]

        s, i = ShardedSearcher(local, off).search(q, K)
        torch.cuda.synchronize()
        out_q.put((rank, off, cnt, i.cpu().numpy(), s.cpu().numpy(), ix.get()))
    except Exception as e:  # report instead of leaving the parent waiting
        out_q.put((rank, repr(e), None, None, None, None))
        raise
    finally:
        dist.destroy_process_group()


def test_dp_ingest_two_ranks_equals_single_process(require_gpu, golden):
    import torch.multiprocessing as mp
    from mediquery_hip import HipBertEmbeddings
    from mediquery_hip.native import FlatIndex
    world = 2
    ctx = mp.get_context("spawn")
    q_out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, golden, q_out)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted([q_out.get(timeout=150) for _ in range(world)], key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=30)
    for r in res:
        assert not isinstance(r[1], str), r[1]
    assert all(p.exitcode == 0 for p in procs)
    # single process: the same texts through one embedder and one index
    texts, qs = _texts(golden)
    emb = HipBertEmbeddings(synthetic=True, batch_size=64)
    ix = FlatIndex(dim=768)
    ix.add(emb.embed_array(texts))
    qv = emb.embed_array(qs)
    s1, i1 = ix.search(qv, K)
    rows = ix.get()
    # the shards are the single index's row blocks, embedded the same (length-sorted
    # batches differ, so within the encoder's batch invariance)
    assert res[0][1] == 0 and res[0][2] + res[1][2] == len(texts) and res[1][1] == res[0][2]
    np.testing.assert_allclose(np.concatenate([res[0][5], res[1][5]]), rows, atol=1e-6, rtol=0)
    ref = exact_scores(qv, rows)
    for rank, off, cnt, ids, scores, _ in res:
        assert check_topk(ids, scores, ref, K) == [], rank
        np.testing.assert_array_equal(ids, i1)
        np.testing.assert_allclose(scores, s1, atol=1e-6, rtol=0)
    assert check_topk(i1, s1, ref, K) == []
