"""Row-sharded search over the GPUs of one node (BASELINE config 4).

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  Rank r owns
a contiguous block of rows [offset_r, offset_r + n_r); global row id = offset_r + local
id.  A search is:
  1. (optional) all-gather of the ranks' query embeddings  -> every rank holds all queries
  2. local exact top-k on the rank's shard                  (K9/K10 on the device)
  3. ONE all-gather of the per-shard [nq, k] (score, id) candidates, packed into a single
     int32 [nq, k, 3] tensor (score bits, id low word, id high word)
  4. merge to the global top-k by (score desc, global id asc)  (device K10 or host merge)
Scoring needs no communication; the exchanged bytes are nq*k*12 per rank.

`LocalShards` is the same partition held as several shards on ONE device (BASELINE
config 4's 8 shards on fewer GPUs than shards): per-shard K9 searches, then the device
merge (K10) - the exchange step without the collective.
"""
import time

import numpy as np
import torch
import torch.distributed as dist

from .native import FlatIndex, merge_topk_device, merge_topk_host


def shard_bounds(n_rows, world, rank):
    """Contiguous near-equal row blocks: (offset, count) of `rank`."""
    base, extra = divmod(n_rows, world)
    off = rank * base + min(rank, extra)
    return off, base + (1 if rank < extra else 0)


def pack_candidates(scores, ids):
    """(scores [nq, k] f32, ids [nq, k] int64) -> one int32 [nq, k, 3] tensor, so the
    candidate exchange is a single collective: word 0 = the score's bits, words 1-2 =
    the id (little-endian halves)."""
    nq, k = scores.shape
    packed = torch.empty((nq, k, 3), dtype=torch.int32, device=scores.device)
    packed[..., 0] = scores.contiguous().view(torch.int32)
    packed[..., 1:] = ids.contiguous().view(torch.int32).view(nq, k, 2)
    return packed


def unpack_candidates(packed):
    """[..., k, 3] int32 -> (scores [..., k] f32, ids [..., k] int64)."""
    s = packed[..., 0].contiguous().view(torch.float32)
    i = packed[..., 1:].contiguous().view(torch.int64).squeeze(-1)
    return s, i


class LocalShards:
    """Row shards of one corpus held as separate `FlatIndex` handles on ONE device
    (BASELINE config 4's 8-shard partition when a rank owns several shards; the
    reference store being scaled is the Chroma collection of src/medical_engine.py:52).
    Shard s holds rows `shard_bounds(n, n_shards, s)` of what `add_device` receives
    (global id = `base` + shard offset + local id); a search runs K9 on every shard into
    one [n_shards, nq, k] candidate buffer and merges it on the device (K10).

    `index_factory(capacity) -> index` builds one shard (default: a `FlatIndex` on
    `device`); any object with FlatIndex's add_device / search_device / set_precision /
    close / __len__ serves, so the CPU tests drive this partition with an oracle shard.
    Candidates on the host are merged by `merge_topk_host` (the same merge, in C)."""

    def __init__(self, n_shards, dim=768, device=0, base=0, index_factory=None):
        self.n_shards, self.dim, self.device, self.base = int(n_shards), dim, device, int(base)
        self._factory = index_factory or (lambda cap: FlatIndex(dim=dim, capacity=cap, device=device))
        self.shards = [self._factory(0) for _ in range(self.n_shards)]
        self.offsets = [0] * self.n_shards
        self._cand = None

    def __len__(self):
        return sum(len(s) for s in self.shards)

    def add_device(self, rows):
        """Partition `rows` [n, dim] (torch, device) into the shards (empty shards only)."""
        if len(self):
            raise ValueError("LocalShards holds rows already: partition once")
        n = int(rows.shape[0])
        self._cand = None  # its cached id offsets belong to the old (empty) partition
        for s in range(self.n_shards):
            off, cnt = shard_bounds(n, self.n_shards, s)
            self.offsets[s] = off
            if cnt:  # sized to the shard up front: no re-allocation while adding
                self.shards[s].close()
                self.shards[s] = self._factory(cnt)
                self.shards[s].add_device(rows[off:off + cnt].contiguous())

    def set_precision(self, dtype):
        for ix in self.shards:
            ix.set_precision(dtype)

    def search_device(self, queries, k, out_scores, out_ids):
        """Global top-k of `queries` [nq, dim] over every shard into out_scores [nq, k] f32
        / out_ids [nq, k] int64 (ids global: base + shard offset + local row)."""
        nq = int(queries.shape[0])
        shape = (self.n_shards, nq, k)
        if self._cand is None or self._cand[0].shape != shape:
            dev = queries.device
            offs = torch.tensor([self.base + o for o in self.offsets], dtype=torch.int64, device=dev)
            self._cand = (torch.empty(shape, dtype=torch.float32, device=dev),
                          torch.empty(shape, dtype=torch.int64, device=dev), offs.view(-1, 1, 1))
        cs, ci, offs = self._cand
        for s, ix in enumerate(self.shards):
            ix.search_device(queries, k, cs[s], ci[s])
        gi = torch.where(ci >= 0, ci + offs, ci)
        if cs.is_cuda:
            merge_topk_device(cs, gi, k, out_scores, out_ids)
        else:
            ms, mi = merge_topk_host(cs.numpy(), gi.numpy(), k)
            out_scores.copy_(torch.from_numpy(ms))
            out_ids.copy_(torch.from_numpy(mi))
        return out_scores, out_ids


class ShardedSearcher:
    """`local_search(queries, k) -> (scores[nq,k] f32, local ids[nq,k] int64)` runs the
    rank's shard (FlatIndex.search_device on a GPU); this class adds the global ids, the
    candidate all-gather and the merge."""

    def __init__(self, local_search, offset, group=None):
        self.local_search = local_search
        self.offset = int(offset)
        self.group = group
        # set to a list to time every collective: entries (tag, bytes per rank, ms), where
        # ms is HIP-event time on the launching stream for RCCL on device tensors (the
        # collective's stream is joined to it both ways) and host wall time for gloo;
        # the RCCL events stay pending until `resolve_timings()`
        self.timings = None
        self._pending = []

    def _all_gather(self, t, tag="gather"):
        """[...] per rank -> [world, ...]: ONE all_gather_into_tensor into a concatenated
        [world * n, ...] buffer (the form both RCCL and gloo accept, so the CPU tests run
        the very call the RCCL path makes), viewed rank-major."""
        world = dist.get_world_size(self.group)
        t = t.contiguous()
        # RCCL gathers device tensors over xGMI; gloo (CPU tests, or several ranks sharing
        # one GPU in a rehearsal) gathers host copies
        rccl = dist.get_backend(self.group) == "nccl"
        src = t if rccl else t.cpu()
        flat = src.reshape((-1,) + tuple(src.shape[1:])) if src.dim() else src.reshape(1)
        out = torch.empty((world * flat.shape[0],) + tuple(flat.shape[1:]), dtype=src.dtype, device=src.device)
        timed = self.timings is not None
        nbytes = flat.numel() * flat.element_size()
        if timed and src.is_cuda:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        elif timed:
            h0 = time.perf_counter()
        dist.all_gather_into_tensor(out, flat, group=self.group)
        if timed and src.is_cuda:
            e1.record()
            self._pending.append((tag, nbytes, e0, e1))
        elif timed:
            self.timings.append((tag, nbytes, (time.perf_counter() - h0) * 1e3))
        return out.view((world,) + tuple(t.shape)).to(t.device)

    def resolve_timings(self):
        """Turn the recorded RCCL events into `timings` entries (synchronises on them)."""
        for tag, nbytes, e0, e1 in self._pending:
            e1.synchronize()
            self.timings.append((tag, nbytes, e0.elapsed_time(e1)))
        self._pending = []
        return self.timings

    def gather_queries(self, q_local):
        """[B, dim] per rank -> [world*B, dim] on every rank (rank-major)."""
        g = self._all_gather(q_local, "queries")
        return g.reshape(-1, q_local.shape[-1])

    def search(self, queries, k, keep=None):
        """Global top-k of `queries` (identical on every rank) over all shards; with
        keep=(start, stop) only those query rows are merged and returned."""
        s, i = self.local_search(queries, k)
        if self.offset:
            i = torch.where(i >= 0, i + self.offset, i)
        gs, gi = unpack_candidates(self._all_gather(pack_candidates(s, i), "candidates"))  # [world, nq, k]
        if keep is not None:
            gs, gi = gs[:, keep[0]:keep[1]].contiguous(), gi[:, keep[0]:keep[1]].contiguous()
        nq = gs.shape[1]
        if gs.is_cuda:
            os_ = torch.empty((nq, k), dtype=torch.float32, device=gs.device)
            oi = torch.empty((nq, k), dtype=torch.int64, device=gs.device)
            merge_topk_device(gs, gi, k, os_, oi)
            return os_, oi
        os_, oi = merge_topk_host(gs.numpy(), gi.numpy(), k)
        return torch.from_numpy(os_), torch.from_numpy(oi)

    def search_local_batch(self, q_local, k, sizes=None):
        """DP-encoded queries: gather every rank's batch, search all, keep own rows.
        Ranks may hold different batch sizes (a ragged last batch): the sizes are
        all-gathered first (skipped when the caller passes every rank's `sizes`), every
        batch is padded to the largest for the one query all-gather, and the padding is
        dropped before the scan."""
        rank = dist.get_rank(self.group)
        B = int(q_local.shape[0])
        if sizes is None:
            sizes = self._all_gather(torch.tensor([B], dtype=torch.int64, device=q_local.device), "sizes")
            sizes = [int(x) for x in sizes.reshape(-1).tolist()]
        elif len(sizes) != dist.get_world_size(self.group) or sizes[rank] != B:
            raise ValueError("sizes %s do not match world size / this rank's batch %d" % (sizes, B))
        Bmax = max(sizes)
        if Bmax != B:
            pad = torch.zeros((Bmax - B, q_local.shape[1]), dtype=q_local.dtype, device=q_local.device)
            q_local = torch.cat([q_local, pad])
        g = self._all_gather(q_local, "queries")  # [world, Bmax, dim]
        if any(b != Bmax for b in sizes):
            allq = torch.cat([g[r, :b] for r, b in enumerate(sizes)])
        else:
            allq = g.reshape(-1, q_local.shape[-1])
        start = sum(sizes[:rank])
        if allq.shape[0] == 0:
            e = torch.empty((0, k), device=q_local.device)
            return e, e.to(torch.int64)
        return self.search(allq, k, keep=(start, start + B))  # merge own rows only


def ingest_sharded(texts, embed_fn, index_add, world=None, rank=None, group=None, chunk=4096):
    """Data-parallel ingest (the reference's `Chroma.from_documents` at
    src/ingest_medical.py:106-110 embeds every chunk on one Ollama server).  Rank r
    embeds only its contiguous block `shard_bounds(len(texts), world, r)` with
    `embed_fn(texts) -> [n, dim]` and appends it to its local shard with
    `index_add(rows)`, `chunk` texts at a time.  No collective: the block layout is the
    one `ShardedSearcher` assumes (global id = offset + local id), so the returned
    offset is that searcher's `offset`.  -> (offset, count)."""
    world = dist.get_world_size(group) if world is None else world
    rank = dist.get_rank(group) if rank is None else rank
    off, cnt = shard_bounds(len(texts), world, rank)
    for s in range(off, off + cnt, chunk):
        index_add(embed_fn(texts[s:min(s + chunk, off + cnt)]))
    return off, cnt
