"""BASELINE config 4 (10M x 768 row-sharded into 8 shards, batch 1024, k = 5) and the
sharded exchange on the GPU (the store being scaled is the Chroma
collection of reference src/medical_engine.py:52, searched at src/agents/nodes.py:93).

* `LocalShards`: the 8-shard partition held on one MI355X - K9 per shard + device merge
  (K10) - against one 10M-row index (ids identical) and against a float64 reference on
  64 sampled queries.
* Two processes (gloo, both on cuda:0) each own one shard through the HIP kernels; the
  single packed all-gather + merge is compared with the oracle.
"""
import os
import socket

import numpy as np
import pytest

from mediquery_hip import _lib, synth
from mediquery_hip.distributed import LocalShards
from mediquery_hip.native import FlatIndex
from oracle.flat import check_topk, exact_scores

pytestmark = pytest.mark.gpu


def _f64_top(q, rows, k, chunk=1_250_000):
    """float64 top-(k+1) of q [nq, dim] over device rows [N, dim] (normalised in float64),
    chunked so the float64 copy stays ~8 GB, plus a lookup of exact scores by id."""
    import torch
    qd = q.double()
    best_s = best_i = None
    for a in range(0, rows.shape[0], chunk):
        c = torch.nn.functional.normalize(rows[a:a + chunk].double(), dim=1)
        s = qd @ c.T
        v, i = torch.topk(s, k + 1, dim=1)
        i = i + a
        if best_s is None:
            best_s, best_i = v, i
        else:
            vs, order = torch.sort(torch.cat([best_s, v], 1), dim=1, descending=True, stable=True)
            best_i = torch.gather(torch.cat([best_i, i], 1), 1, order)[:, :k + 1]
            best_s = vs[:, :k + 1]
        del c, s

    def lookup(b, ids):
        r = torch.nn.functional.normalize(rows[torch.as_tensor(ids, device=rows.device)].double(), dim=1)
        return (r @ qd[b]).cpu().numpy()
    return (best_s.cpu().numpy(), best_i.cpu().numpy()), lookup


@pytest.mark.parametrize("prec", [_lib.MQ_DTYPE_F32_SCREEN, _lib.MQ_DTYPE_F32])
def test_config4_eight_shards_equal_single_index_and_fp64(require_gpu, prec):
    import torch
    dev = torch.device("cuda", 0)
    N, B, K = 10_000_000, 1024, 5
    rows = synth.corpus_device(N, 768, dev)
    q, planted = synth.queries_device(B, rows)
    sh = LocalShards(8, 768, device=0)
    sh.add_device(rows)
    assert len(sh) == N and sh.offsets == [i * 1_250_000 for i in range(8)]
    sh.set_precision(prec)
    s = torch.empty((B, K), dtype=torch.float32, device=dev)
    i = torch.empty((B, K), dtype=torch.int64, device=dev)
    sh.search_device(q, K, s, i)
    torch.cuda.synchronize()
    pl = planted >= 0
    assert bool((i[pl, 0] == planted[pl]).all())
    got_s, got_i = s.cpu().numpy(), i.cpu().numpy()
    del sh
    torch.cuda.empty_cache()
    # one 10M-row index: the same ids and scores (scores are fp32 dots of the same rows)
    one = FlatIndex(dim=768, capacity=N)
    one.add_device(rows)
    one.set_precision(prec)
    s1 = torch.empty_like(s)
    i1 = torch.empty_like(i)
    one.search_device(q, K, s1, i1)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(i1.cpu().numpy(), got_i)
    np.testing.assert_allclose(s1.cpu().numpy(), got_s, rtol=0, atol=2e-6)
    del one
    torch.cuda.empty_cache()
    # float64 reference on 64 sampled queries (32 planted, 32 free)
    pick = np.r_[0:32, B - 32:B]
    ref_top, lookup = _f64_top(q[pick], rows, K)
    fails = check_topk(got_i[pick], got_s[pick], None, K, ref_top=ref_top, n_rows=N, ref_lookup=lookup)
    assert fails == []


@pytest.mark.parametrize("n_shards,N", [(3, 20000), (8, 50000), (5, 3)])
def test_local_shards_vs_oracle_small(require_gpu, n_shards, N):
    """Uneven and tiny shards (k larger than a shard: padding candidates) through the
    per-shard kernels + device merge, exact against the float64 oracle."""
    import torch
    dev = torch.device("cuda", 0)
    c = synth.corpus(N, 768, clustered=True)
    q, _ = synth.queries(40, c)
    sh = LocalShards(n_shards, 768, device=0, base=0)
    sh.add_device(torch.from_numpy(c).to(dev))
    for k in (5, 17):
        s = torch.empty((40, k), dtype=torch.float32, device=dev)
        i = torch.empty((40, k), dtype=torch.int64, device=dev)
        sh.search_device(torch.from_numpy(q).to(dev), k, s, i)
        torch.cuda.synchronize()
        kk = min(k, N)
        assert check_topk(i.cpu().numpy()[:, :kk], s.cpu().numpy()[:, :kk], exact_scores(q, c), k) == []
        if k > N:
            assert (i.cpu().numpy()[:, N:] == -1).all()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_q, N, K, NQ):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "mediquery-rag_amd"), root]
    import torch
    import torch.distributed as dist
    from mediquery_hip import synth as sy
    from mediquery_hip.distributed import LocalShards as LS, ShardedSearcher, shard_bounds
    from mediquery_hip.native import FlatIndex as FI
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        c = sy.corpus(N, 768, clustered=True)
        off, cnt = shard_bounds(N, world, rank)
        shard = torch.from_numpy(c[off:off + cnt]).to(dev)
        if rank == 0:  # rank 0 holds its block as two local shards, rank 1 as one index
            ix = LS(2, 768, device=0)
        else:
            ix = FI(dim=768, device=0)
        ix.add_device(shard)
        s_loc = torch.empty((NQ, K), dtype=torch.float32, device=dev)
        i_loc = torch.empty((NQ, K), dtype=torch.int64, device=dev)

        def local(qq, k):
            ix.search_device(qq, k, s_loc[:qq.shape[0]], i_loc[:qq.shape[0]])
            return s_loc[:qq.shape[0]], i_loc[:qq.shape[0]]

        ss = ShardedSearcher(local, off)
        q, _ = sy.queries(NQ, c)
        s, i = ss.search(torch.from_numpy(q).to(dev), K)
        half = NQ // world
        _, i2 = ss.search_local_batch(torch.from_numpy(q[rank * half:(rank + 1) * half]).to(dev), K,
                                      sizes=[half] * world)
        torch.cuda.synchronize()
        out_q.put((rank, i.cpu().numpy(), s.cpu().numpy(), i2.cpu().numpy()))
    except Exception as e:  # report instead of leaving the parent waiting
        out_q.put((rank, repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


def test_two_process_hip_shards_single_allgather(require_gpu):
    import torch.multiprocessing as mp
    world, N, K, NQ = 2, 30001, 5, 64
    ctx = mp.get_context("spawn")
    q_out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q_out, N, K, NQ)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted([q_out.get(timeout=100) for _ in range(world)], key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=30)
    for r in res:
        assert not isinstance(r[1], str), r[1]
    assert all(p.exitcode == 0 for p in procs)
    c = synth.corpus(N, 768, clustered=True)
    q, _ = synth.queries(NQ, c)
    ref = exact_scores(q, c)
    half = NQ // world
    for rank, ids, scores, ids_dp in res:
        assert check_topk(ids, scores, ref, K) == []
        np.testing.assert_array_equal(ids_dp, ids[rank * half:(rank + 1) * half])
    np.testing.assert_array_equal(res[0][1], res[1][1])


def _rccl_worker(port, out_q, N, K, NQ):
    """One rank on the RCCL backend: the exact calls bench.py makes at N > 1
    (init_process_group("nccl", device_id=...), the packed candidate all-gather, the query
    all-gather and the batch-size all-gather of device tensors), at world size 1 - RCCL
    needs one GPU per rank, so more ranks cannot share this box's single GPU."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "mediquery-rag_amd"), root]
    import torch
    import torch.distributed as dist
    from mediquery_hip import synth as sy
    from mediquery_hip.distributed import ShardedSearcher
    from mediquery_hip.native import FlatIndex as FI
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        c = sy.corpus(N, 768, clustered=True)
        ix = FI(dim=768, device=0)
        ix.add_device(torch.from_numpy(c).to(dev))
        s_loc = torch.empty((NQ, K), dtype=torch.float32, device=dev)
        i_loc = torch.empty((NQ, K), dtype=torch.int64, device=dev)

        def local(qq, k):
            ix.search_device(qq, k, s_loc[:qq.shape[0]], i_loc[:qq.shape[0]])
            return s_loc[:qq.shape[0]], i_loc[:qq.shape[0]]

        q, _ = sy.queries(NQ, c)
        qd = torch.from_numpy(q).to(dev)
        ss = ShardedSearcher(local, 0)
        s, i = ss.search(qd, K)
        g = ss.gather_queries(qd)
        _, i2 = ss.search_local_batch(qd[:NQ - 3], K)  # sizes=None: the size all-gather runs
        ix.search_device(qd, K, s_loc, i_loc)
        torch.cuda.synchronize()
        out_q.put((s.is_cuda, i.cpu().numpy(), s.cpu().numpy(), bool(torch.equal(g, qd)), i2.cpu().numpy(),
                   i_loc.cpu().numpy()))
    except Exception as e:  # report instead of leaving the parent waiting
        out_q.put((repr(e),))
        raise
    finally:
        dist.destroy_process_group()


def test_rccl_backend_exchange_world1(require_gpu):
    """The RCCL code path of the sharded search (device tensors through
    all_gather_into_tensor on the nccl backend), checked against the plain index."""
    import torch.multiprocessing as mp
    N, K, NQ = 20011, 5, 48
    ctx = mp.get_context("spawn")
    q_out = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q_out, N, K, NQ))
    p.start()
    try:
        r = q_out.get(timeout=100)
    finally:
        p.join(timeout=30)
    assert len(r) > 1, r[0]
    assert p.exitcode == 0
    on_device, ids, scores, gathered_ok, ids_b, ids_plain = r
    assert on_device and gathered_ok
    np.testing.assert_array_equal(ids, ids_plain)
    np.testing.assert_array_equal(ids_b, ids_plain[:NQ - 3])
    c = synth.corpus(N, 768, clustered=True)
    q, _ = synth.queries(NQ, c)
    assert check_topk(ids, scores, exact_scores(q, c), K) == []
