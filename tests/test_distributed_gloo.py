"""Row-sharded search across processes (world_size 2 and 3, gloo, CPU): the all-gather
of per-shard candidates plus the merge must equal the single-index exact answer,
including uneven shards and k larger than a shard (padding candidates).  The per-shard
local search here is the oracle; on GPUs it is the K9/K10 kernels."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

DIM, NQ = 64, 12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_q, N, K):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "mediquery-rag_amd"), root]
    from mediquery_hip import synth
    from mediquery_hip.distributed import ShardedSearcher, shard_bounds
    from oracle.flat import search
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = synth.corpus(N, DIM, clustered=True)
        off, cnt = shard_bounds(N, world, rank)
        shard = c[off:off + cnt]

        def local(q, k):
            # the device contract (mq_index_search): [nq, k], padded with (-inf, -1)
            s, i = search(q.numpy(), shard, k)
            ps = np.full((q.shape[0], k), -np.inf, np.float32)
            pi = np.full((q.shape[0], k), -1, np.int64)
            ps[:, :s.shape[1]], pi[:, :i.shape[1]] = s, i
            return torch.from_numpy(ps), torch.from_numpy(pi)

        ss = ShardedSearcher(local, off)
        q, _ = synth.queries(NQ, c)
        s, i = ss.search(torch.from_numpy(q), K)
        # DP query path: each rank contributes half the batch
        half = NQ // world
        s2, i2 = ss.search_local_batch(torch.from_numpy(q[rank * half:(rank + 1) * half]), K)
        # ragged DP batches (a short last batch): ranks hold different query counts
        qo, qc = shard_bounds(NQ - 1, world, world - 1 - rank)
        _, i3 = ss.search_local_batch(torch.from_numpy(q[qo:qo + qc]), K)
        out_q.put((rank, i.numpy(), s.numpy(), (i2.numpy(), i3.numpy(), qo, qc)))
    except Exception as e:  # report instead of leaving the parent waiting
        out_q.put((rank, repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N,K", [(2, 997, 7), (3, 1000, 5), (3, 10, 7)])
def test_sharded_search_equals_single_index(world, N, K):
    from mediquery_hip import synth
    from oracle.flat import exact_scores, check_topk
    ctx = mp.get_context("spawn")
    q_out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q_out, N, K)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q_out.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = synth.corpus(N, DIM, clustered=True)
    q, _ = synth.queries(NQ, c)
    ref = exact_scores(q, c)
    res.sort(key=lambda r: r[0])
    for r in res:
        assert not isinstance(r[1], str), r[1]
    offsets = [r[3][2] for r in res]
    assert offsets == sorted(offsets, reverse=True)  # rank r holds block world-1-r
    for rank, ids, scores, (ids_dp, ids_ragged, qo, qc) in res:
        assert check_topk(ids, scores, ref, K) == []
        half = NQ // world
        np.testing.assert_array_equal(ids_dp, ids[rank * half:(rank + 1) * half])
        assert ids_ragged.shape == (qc, K)
        np.testing.assert_array_equal(ids_ragged, ids[qo:qo + qc])
    for r in res[1:]:
        np.testing.assert_array_equal(res[0][1], r[1])


@pytest.mark.parametrize("world,N,chunk", [(2, 997, 64), (3, 10, 4), (4, 3, 8)])
def test_ingest_sharded_blocks_line_up_with_search_ids(world, N, chunk):
    """Each rank's `ingest_sharded` block, appended in order, must be exactly rows
    [offset, offset+count) of the single-process ingest, so local id + offset is the
    global row id `ShardedSearcher` reports."""
    from mediquery_hip.distributed import ingest_sharded
    texts = ["doc %d" % i for i in range(N)]

    def embed(ts):  # deterministic stand-in for the encoder: one row per text
        return np.array([[float(t.split()[1]), len(t)] for t in ts], np.float32).reshape(-1, 2)

    whole = embed(texts)
    seen = []
    for rank in range(world):
        rows = []
        off, cnt = ingest_sharded(texts, embed, rows.append, world=world, rank=rank, chunk=chunk)
        local = np.concatenate(rows) if rows else np.zeros((0, 2), np.float32)
        assert local.shape[0] == cnt
        assert all(r.shape[0] <= chunk for r in rows)
        np.testing.assert_array_equal(local, whole[off:off + cnt])
        seen.append((off, cnt))
    assert seen[0][0] == 0 and sum(c for _, c in seen) == N
    assert all(seen[r][0] + seen[r][1] == seen[r + 1][0] for r in range(world - 1))


def test_pack_candidates_roundtrip_is_bit_exact():
    """The single candidate all-gather carries (score, id) as one int32 [nq, k, 3]
    tensor: scores (incl. -inf padding, -0.0, subnormals) and ids (incl. -1 and ids past
    2^32) must come back bit-exactly."""
    from mediquery_hip.distributed import pack_candidates, unpack_candidates
    s = torch.tensor([[1.0, -0.0, float("-inf")], [1e-40, 0.5, -2.5]], dtype=torch.float32)
    i = torch.tensor([[0, 5_000_000_000, -1], [7, 2**31 + 3, 123]], dtype=torch.int64)
    p = pack_candidates(s, i)
    assert p.dtype == torch.int32 and p.shape == (2, 3, 3)
    g = torch.stack([p, p])  # what an all-gather of two ranks stacks
    s2, i2 = unpack_candidates(g)
    assert s2.shape == (2, 2, 3) and i2.shape == (2, 2, 3)
    assert torch.equal(s2[1].view(torch.int32), s.view(torch.int32))
    assert torch.equal(i2[0], i)


class _OracleShard:
    """CPU stand-in with FlatIndex's surface (add_device / search_device / __len__): the
    oracle's exact search padded to the device contract (-inf, -1)."""

    def __init__(self, capacity=0):
        self.rows = np.zeros((0, DIM), np.float32)

    def add_device(self, rows):
        self.rows = rows.numpy().copy()

    def search_device(self, q, k, out_s, out_i):
        from oracle.flat import search
        out_s.fill_(float("-inf"))
        out_i.fill_(-1)
        if len(self.rows):
            s, i = search(q.numpy(), self.rows, k)
            out_s[:, :s.shape[1]] = torch.from_numpy(np.ascontiguousarray(s, np.float32))
            out_i[:, :i.shape[1]] = torch.from_numpy(np.ascontiguousarray(i, np.int64))

    def set_precision(self, dtype):
        pass

    def close(self):
        pass

    def __len__(self):
        return self.rows.shape[0]


C4_SHARDS = 8


def _config4_worker(rank, world, port, out_q, per, K, B):
    """bench.py config4()'s partition: 8 row shards of `per` rows, rank r owns shards
    [r*8/world, (r+1)*8/world) as one LocalShards (global id = first*per + shard offset +
    local id), embeds B/world queries (DP), one query all-gather, one packed candidate
    all-gather, merge of its own queries."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "mediquery-rag_amd"), root]
    from mediquery_hip import synth
    from mediquery_hip.distributed import LocalShards, ShardedSearcher
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = synth.corpus(C4_SHARDS * per, DIM, clustered=True)
        spr = C4_SHARDS // world
        first = rank * spr
        shards = LocalShards(spr, DIM, device=None, index_factory=_OracleShard)
        shards.add_device(torch.from_numpy(c[first * per:(first + spr) * per]))
        assert len(shards) == spr * per
        q, _ = synth.queries(B, c)
        bq = B // world
        s_loc = torch.empty((B, K), dtype=torch.float32)
        i_loc = torch.empty((B, K), dtype=torch.int64)

        def local(qq, k):
            n = qq.shape[0]
            shards.search_device(qq, k, s_loc[:n], i_loc[:n])
            return s_loc[:n], i_loc[:n]

        ss = ShardedSearcher(local, first * per)
        ss.timings = []
        s, i = ss.search_local_batch(torch.from_numpy(q[rank * bq:(rank + 1) * bq]), K, sizes=[bq] * world)
        tags = [t[0] for t in ss.resolve_timings()]
        out_q.put((rank, i.numpy(), s.numpy(), tags))
    except Exception as e:
        out_q.put((rank, repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_config4_eight_shard_partition_over_ranks(world):
    """BASELINE config 4's 8-shard partition through LocalShards at world 2 and 4 (gloo):
    each rank's merged answer for its own DP queries equals the exact top-k over the whole
    corpus, and the collectives are timed (one query and one candidate all-gather)."""
    from mediquery_hip import synth
    from oracle.flat import check_topk, exact_scores
    per, K, B = 125, 5, 16
    ctx = mp.get_context("spawn")
    q_out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_config4_worker, args=(r, world, port, q_out, per, K, B)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q_out.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = synth.corpus(C4_SHARDS * per, DIM, clustered=True)
    q, _ = synth.queries(B, c)
    ref = exact_scores(q, c)
    bq = B // world
    for rank, ids, scores, tags in sorted(res, key=lambda r: r[0]):
        assert not isinstance(ids, str), ids
        assert check_topk(ids, scores, ref[rank * bq:(rank + 1) * bq], K) == []
        assert tags == ["queries", "candidates"]


def test_local_shards_host_merge_equals_exact():
    """LocalShards on one process with host candidates (merge_topk_host): 8 uneven shards."""
    from mediquery_hip import synth
    from mediquery_hip.distributed import LocalShards
    from oracle.flat import check_topk, exact_scores
    c = synth.corpus(1003, DIM, clustered=True)
    q, _ = synth.queries(9, c)
    sh = LocalShards(8, DIM, device=None, base=0, index_factory=_OracleShard)
    sh.add_device(torch.from_numpy(c))
    s = torch.empty((9, 7), dtype=torch.float32)
    i = torch.empty((9, 7), dtype=torch.int64)
    sh.search_device(torch.from_numpy(q), 7, s, i)
    assert check_topk(i.numpy(), s.numpy(), exact_scores(q, c), 7) == []
