"""`HipChroma` - drop-in for `langchain_chroma.Chroma` on MI355X.

Reference call sites (unchanged by the swap):
  * `Chroma(persist_directory=DB_PATH, embedding_function=embeddings)`
    src/medical_engine.py:52
  * `Chroma.from_documents(documents=docs, embedding=embeddings,
    persist_directory=DB_PATH)`  src/ingest_medical.py:106-110
  * `vectorstore.similarity_search(search_query, k=5)`  src/agents/nodes.py:93
    (and k=3 in the dead helper src/medical_engine.py:70)

The rows live in an HBM-resident flat index (libmqhip.so); documents and metadata stay
on the host, keyed by row id = insertion order.  Semantics follow Chroma's default
"l2" space: `similarity_search_with_score` returns squared L2 distance, which for the
unit-norm embeddings is 2 - 2*cos; `similarity_search` returns documents by ascending
distance, ties broken by insertion order.  k > N returns N documents; an empty store
returns [].  The device top-k holds at most MQ_MAX_K (64) results: a search whose result
count min(k, candidates) exceeds it raises instead of truncating.  Errors raise (the
reference's retrieve_node does not catch either).

Persistence: `mq_<collection>.json` (ids, documents, metadatas, and the name of the slab
file) is the base commit point; a full write (the first write, `delete`, an upsert that
replaces rows, an explicit `persist()`) puts the rows in a fresh `mq_<collection>.<gen>.flat`
and then atomically replaces the JSON, so a crash leaves either the old or the new store,
never a slab/sidecar mismatch.  A plain append (`add_texts` of new ids) is append-only: the
new rows go to a segment `mq_<collection>@<gen>.seg.flat` (+ `.seg.json`, their ids,
documents and metadatas), committed by atomically replacing the small manifest
`mq_<collection>@tail.json` (the base slab it extends + the segment list), so one added
document costs a few KB of writes instead of the whole slab and sidecar ('@' cannot occur
in a collection name: no sibling collection's file can match).  Loading applies the
manifest's segments when it names the loaded base; a full write supersedes them, and after
MAX_SEGMENTS appends the next one compacts.  A directory that holds a stock Chroma database
(`chroma.sqlite3`, written by the reference's ingest) but no sidecar is refused: it must be
re-ingested with this store (`python src/ingest_medical.py` after the import swap).
"""
import json
import math
import os
import re
import uuid

import numpy as np

from . import _lib
from .compat import Document, VectorStoreBase
from .native import FlatIndex, mask_combine, mask_eval, mask_eval_bits

DEFAULT_K = 4  # LangChain VectorStore.similarity_search default; the reference passes k=5

# search arithmetic (`HipChroma(search_precision=...)`): "screen" (default) = exact fp32
# top-k through the certified screens (int8 / bf16 shadow scans for candidates, fp32
# re-rank, a proven bound per query, uncertified queries re-run exactly); "f32" = the
# direct exact fp32 scan; "f32x6" = the direct scan on the split-f32 MFMA (fp32-class);
# "bf16" = BASELINE config 5's bf16 coarse scan + fp32 re-rank (approximate: recall is
# measured, not guaranteed)
SEARCH_PRECISIONS = {"screen": _lib.MQ_DTYPE_F32_SCREEN, "f32": _lib.MQ_DTYPE_F32,
                     "f32x6": _lib.MQ_DTYPE_F32X6, "bf16": _lib.MQ_DTYPE_BF16}


def _match(meta, where):
    """Chroma-style metadata filter: {"k": v}, {"k": {"$op": v}}, {"$and"/"$or": [...]}."""
    for key, cond in where.items():
        if key == "$and":
            if not all(_match(meta, c) for c in cond):
                return False
        elif key == "$or":
            if not any(_match(meta, c) for c in cond):
                return False
        else:
            v = meta.get(key)
            if isinstance(cond, dict):
                for op, x in cond.items():
                    ok = {"$eq": lambda: v == x, "$ne": lambda: v != x,
                          "$gt": lambda: v is not None and v > x,
                          "$gte": lambda: v is not None and v >= x,
                          "$lt": lambda: v is not None and v < x,
                          "$lte": lambda: v is not None and v <= x,
                          "$in": lambda: v in x, "$nin": lambda: v not in x}.get(op)
                    if ok is None:
                        raise ValueError("unsupported filter operator %r" % op)
                    try:
                        hit = ok()
                    except TypeError:  # incomparable types: no match (see _pred)
                        hit = False
                    if not hit:
                        return False
            elif v != cond:
                return False
    return True


_MISSING = object()


def _pred(op, v, x):
    """One Chroma where-operator on one metadata value (v None = key absent), as _match."""
    if op == "$eq":
        return v == x
    if op == "$ne":
        return v != x
    if op in ("$gt", "$gte", "$lt", "$lte"):
        if v is None:
            return False
        try:
            return {"$gt": lambda: v > x, "$gte": lambda: v >= x, "$lt": lambda: v < x,
                    "$lte": lambda: v <= x}[op]()
        except TypeError:  # incomparable types (a str value vs a number): no match, as in
            return False   # Chroma, whose typed SQL comparison never matches across types
    if op == "$in":
        return v in x
    if op == "$nin":
        return v not in x
    raise ValueError("unsupported filter operator %r" % op)


class _MetaColumns:
    """Metadata held column-wise for vectorised Chroma `where` filters: per key, int32
    codes [n] (-1 = key absent in that row) into the key's distinct values.  A condition
    is evaluated once per DISTINCT value (Python) into a truth table; the rows are mapped
    through it on the device (`dmask`: mq_mask_eval over a device mirror of the codes,
    a row bitmask the masked search reads) or by numpy (`mask`, for get()); results equal
    `_match` row by row."""

    def __init__(self):
        self.n = 0
        self.cols = {}  # key -> [codes np.int32 (capacity >= n), values list, {hash key: code}]
        self.ver = 0    # bumped by append / compact (device mirrors are per version)
        self.dev = {}   # key -> (ver, device int32 codes [n])
        self._num_cache = {}  # id(values list) -> (len, float64 array or None: not all numeric)

    @staticmethod
    def _hkey(v):
        try:
            return (type(v).__name__, v, hash(v))
        except TypeError:  # unhashable (list) values: keyed by their repr
            return (type(v).__name__, repr(v), None)

    def append(self, metas):
        m = len(metas)
        need = self.n + m
        for col in self.cols.values():
            if col[0].shape[0] < need:
                grown = np.full(max(need, 2 * col[0].shape[0]), -1, np.int32)
                grown[:self.n] = col[0][:self.n]
                col[0] = grown
            col[0][self.n:need] = -1
        for r, meta in enumerate(metas):
            for key, v in meta.items():
                col = self.cols.get(key)
                if col is None:
                    col = self.cols[key] = [np.full(max(need, 1024), -1, np.int32), [], {}]
                hk = self._hkey(v)
                code = col[2].get(hk)
                if code is None:
                    code = col[2][hk] = len(col[1])
                    col[1].append(v)
                col[0][self.n + r] = code
        self.n = need
        self.ver += 1

    def compact(self, keep):
        """Keep rows `keep` (sorted int64 row ids), in order."""
        for col in self.cols.values():
            col[0] = np.ascontiguousarray(col[0][:self.n][keep])
        self.n = len(keep)
        self.ver += 1

    _NUM_OPS = {"$eq": np.equal, "$ne": np.not_equal, "$gt": np.greater, "$gte": np.greater_equal,
                "$lt": np.less, "$lte": np.less_equal}

    @staticmethod
    def _is_num(v):  # a number float64 holds exactly (ints past 2^53 take the exact path)
        return (isinstance(v, float) or (isinstance(v, int) and abs(v) < 2 ** 53)) and not isinstance(v, bool)

    def _lut(self, values, op, x):
        """Truth table of one condition over a column's distinct values (+ absent, last).
        A comparison of a number against an all-numeric column is one numpy op (the
        per-value Python predicate cost ~0.4 us a value); anything else goes value by value
        through _pred (Chroma's typed comparison: mixed types never match)."""
        lut = np.zeros(len(values) + 1, np.uint8)
        lut[-1] = _pred(op, None, x)
        if op in self._NUM_OPS and self._is_num(x) and len(values) > 8:
            nums = self._num_cache.get(id(values))
            if nums is None or nums[0] != len(values):
                ok = all(self._is_num(v) for v in values)
                nums = (len(values), np.array(values, dtype=np.float64) if ok else None)
                self._num_cache[id(values)] = nums
            if nums[1] is not None:
                lut[:-1] = self._NUM_OPS[op](nums[1], float(x))
                return lut
        for cv, v in enumerate(values):
            lut[cv] = _pred(op, v, x)
        return lut

    def dev_codes(self, key, dev):
        got = self.dev.get(key)
        if got is None or got[0] != self.ver:
            import torch
            got = self.dev[key] = (self.ver, torch.from_numpy(self.cols[key][0][:self.n]).to(dev))
        return got[1]

    def dmask(self, where, device):
        """Row bitmask of `where` on the device (int32 words, bit r % 32 of word r / 32),
        built on `device` with that device's current stream whatever torch's current
        device is."""
        import torch
        dev = torch.device("cuda", device)
        with _lib.device_scope(device):
            bits = torch.empty(max(1, (self.n + 31) // 32), dtype=torch.int32, device=dev)
            mask_combine(bits, None, _lib.MQ_MASK_SET)  # all rows
            self._dapply(where, bits, dev)
        return bits

    def _dapply(self, where, bits, dev):
        """bits &= where (the conditions of one dict are ANDed)."""
        import torch
        for key, cond in where.items():
            if key == "$and":
                for c in cond:
                    self._dapply(c, bits, dev)
            elif key == "$or":
                acc, tmp = torch.empty_like(bits), torch.empty_like(bits)
                mask_combine(acc, None, _lib.MQ_MASK_CLEAR)
                for c in cond:
                    mask_combine(tmp, None, _lib.MQ_MASK_SET)
                    self._dapply(c, tmp, dev)
                    mask_combine(acc, tmp, _lib.MQ_MASK_OR)
                mask_combine(bits, acc, _lib.MQ_MASK_AND)
            else:
                col = self.cols.get(key)
                ops = cond.items() if isinstance(cond, dict) else (("$eq", cond),)
                for op, x in ops:
                    if col is None:  # no row has the key
                        if not _pred(op, None, x):
                            mask_combine(bits, None, _lib.MQ_MASK_CLEAR)
                        continue
                    lut = self._lut(col[1], op, x)
                    if len(lut) <= 256:  # by value: no host-to-device copy
                        mask_eval_bits(self.dev_codes(key, dev), lut, bits, _lib.MQ_MASK_AND)
                    else:
                        mask_eval(self.dev_codes(key, dev), torch.from_numpy(lut).to(dev), bits, _lib.MQ_MASK_AND)

    def mask(self, where):
        out = np.ones(self.n, bool)
        for key, cond in where.items():
            if key == "$and":
                for c in cond:
                    out &= self.mask(c)
            elif key == "$or":
                any_ = np.zeros(self.n, bool)
                for c in cond:
                    any_ |= self.mask(c)
                out &= any_
            else:
                col = self.cols.get(key)
                codes = col[0][:self.n] if col is not None else np.full(self.n, -1, np.int32)
                values = col[1] if col is not None else []
                ops = cond.items() if isinstance(cond, dict) else (("$eq", cond),)
                for op, x in ops:
                    # admitted codes -> one table lookup per row; code -1 (key absent)
                    # indexes the table's last entry
                    out &= self._lut(values, op, x).astype(bool)[codes]
        return out


class _IdRows:
    """id -> current row in O(1), kept across deletes without rebuilding a dict of every id:
    each id gets a stable slot when it is added (`slot`, a dict), and two int64 arrays map
    slot -> current row (-1 = deleted) and row -> slot.  A delete drops its ids' dict
    entries and renumbers the surviving rows with one numpy gather / scatter (a dict
    rebuild of a 1M-row store cost ~0.4 s per delete).  Dead slots are reclaimed by a
    rebuild once they outnumber the live rows."""

    def __init__(self, ids=()):
        self.slot = {}
        self._slot_row = np.zeros(1024, np.int64)
        self._row_slot = np.zeros(1024, np.int64)
        self.n_slots = 0
        self.n = 0
        self.extend(list(ids))

    def __contains__(self, i):
        return i in self.slot

    def __len__(self):
        return self.n

    def row(self, i):
        return int(self._slot_row[self.slot[i]])

    @staticmethod
    def _grow(a, need):
        if a.shape[0] >= need:
            return a
        b = np.zeros(max(need, 2 * a.shape[0]), np.int64)
        b[:a.shape[0]] = a
        return b

    def extend(self, ids):
        """ids (new, distinct) appended as rows n .. n + len(ids)."""
        m = len(ids)
        if not m:
            return
        s0, r0 = self.n_slots, self.n
        self._slot_row = self._grow(self._slot_row, s0 + m)
        self._row_slot = self._grow(self._row_slot, r0 + m)
        self._slot_row[s0:s0 + m] = np.arange(r0, r0 + m)
        self._row_slot[r0:r0 + m] = np.arange(s0, s0 + m)
        self.slot.update(zip(ids, range(s0, s0 + m)))
        self.n_slots += m
        self.n += m

    def compact(self, keep, dropped_ids):
        """Rows `keep` (sorted int64) survive, renumbered 0..len(keep); dropped_ids leave."""
        for i in dropped_ids:
            del self.slot[i]
        rs = self._row_slot[:self.n]
        keepm = np.zeros(self.n, bool)
        keepm[keep] = True
        self._slot_row[rs[~keepm]] = -1
        kept = rs[keepm]
        self._row_slot[:kept.shape[0]] = kept
        self._slot_row[kept] = np.arange(kept.shape[0])
        self.n = int(kept.shape[0])
        if self.n_slots > 2 * self.n + 1024:  # reclaim the dead slots
            order = sorted(self.slot, key=self.slot.__getitem__)
            rows = self._slot_row[[self.slot[i] for i in order]] if order else np.zeros(0, np.int64)
            ids_by_row = [None] * self.n
            for i, r in zip(order, rows.tolist()):
                ids_by_row[r] = i
            self.__init__(ids_by_row)


def _drop_sorted(lst, drop):
    """lst without the positions `drop` (sorted, distinct): list slices, no per-item Python."""
    out, prev = [], 0
    for d in drop:
        out += lst[prev:d]
        prev = d + 1
    out += lst[prev:]
    return out


def _check_k(k, n_candidates):
    """Result count of a top-k over n_candidates rows; raises past the device limit."""
    kk = min(int(k), int(n_candidates))
    if kk > _lib.MQ_MAX_K:
        raise ValueError("a search returning %d results (k=%d over %d rows) exceeds the device "
                         "top-k limit MQ_MAX_K=%d" % (kk, k, n_candidates, _lib.MQ_MAX_K))
    return kk


class HipChroma(VectorStoreBase):
    _FILES = ("mq_%s.flat", "mq_%s.json", "mq_%s@tail.json")
    FOREIGN_DB = "chroma.sqlite3"  # what langchain_chroma / chromadb persist
    _GEN = re.compile(r"[0-9a-f]{12}\.flat")  # slab generation suffix (persist() writes it)
    STALE_SLAB_S = 3600  # an uncommitted slab this old is a crashed writer's leftover
    _SEG = re.compile(r"[0-9a-f]{12}\.seg\.(flat|json)")  # segment files (after 'mq_<name>@')
    MAX_SEGMENTS = 256  # appends between compactions

    def __init__(self, collection_name="langchain", embedding_function=None,
                 persist_directory=None, client_settings=None, collection_metadata=None,
                 client=None, relevance_score_fn=None, *, device=0, dim=None,
                 auto_persist=True, search_precision="screen", _ingest=False, **kwargs):
        """auto_persist=False: writes stay in memory until `persist()` (bulk ingest);
        search_precision: SEARCH_PRECISIONS (default "screen": exact fp32 top-k)."""
        if search_precision not in SEARCH_PRECISIONS:
            raise ValueError("search_precision must be one of %s, got %r"
                             % (sorted(SEARCH_PRECISIONS), search_precision))
        self._search_precision = search_precision
        self._collection_name = collection_name
        self._embedding_function = embedding_function
        self._persist_directory = persist_directory
        self._collection_metadata = dict(collection_metadata or {})
        self.override_relevance_score_fn = relevance_score_fn
        self._device = device
        self._auto_persist = bool(auto_persist)
        self._ids, self._texts, self._metas = [], [], []
        self._id_row = _IdRows()       # id -> row (upsert / delete / get by id in O(1))
        self._cols = _MetaColumns()    # metadata column-wise, for vectorised filters
        self._version = 0              # bumped by every write
        self._index = None
        self._dim = dim
        self._slab_name = None
        self._segments = []    # committed segments after the base: {"slab", "delta", "n_rows"}
        self._written = set()  # slabs this instance wrote that no commit of its own names now
        if persist_directory and os.path.exists(self._path(1)):
            self._load()
        elif (persist_directory and not _ingest
              and os.path.exists(os.path.join(persist_directory, self.FOREIGN_DB))):
            raise RuntimeError(
                "%r holds a ChromaDB database (%s) but no %s sidecar: the MI355X store cannot "
                "read Chroma's files. Re-run the ingest (src/ingest_medical.py) with the "
                "mediquery_hip import swap to build it." % (persist_directory, self.FOREIGN_DB,
                                                            self._FILES[1] % collection_name))

    # ---- helpers ---------------------------------------------------------------------
    @property
    def embeddings(self):
        return self._embedding_function

    def _path(self, i):
        return os.path.join(self._persist_directory, self._FILES[i] % self._collection_name)

    def _ensure_index(self, dim):
        if self._index is None:
            self._dim = dim
            self._index = FlatIndex(dim=dim, device=self._device)
            self._index.set_precision(SEARCH_PRECISIONS[self._search_precision])
        elif dim != self._dim:
            raise ValueError("embedding dim %d != collection dim %d" % (dim, self._dim))

    def _persist(self):
        if self._auto_persist:
            self.persist()

    @staticmethod
    def _write_json(path, obj):
        """Write + fsync `path` + ".tmp", then atomically rename it to `path`."""
        tmp = path + ".tmp"
        with open(tmp, "w", encoding="utf-8") as f:
            json.dump(obj, f, ensure_ascii=False)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)

    def persist(self):
        """Write the whole store under persist_directory (crash-safe, see the module doc);
        supersedes (and deletes) the append segments."""
        if not self._persist_directory or self._index is None:
            return
        d = self._persist_directory
        os.makedirs(d, exist_ok=True)
        slab = "mq_%s.%s.flat" % (self._collection_name, uuid.uuid4().hex[:12])
        self._index.save(os.path.join(d, slab))
        self._write_json(self._path(1), {  # the commit point
            "dim": self._dim, "slab": slab, "n_rows": len(self._ids), "ids": self._ids,
            "documents": self._texts, "metadatas": self._metas,
            "collection_metadata": self._collection_metadata})
        replaced, self._slab_name = self._slab_name, slab
        if replaced:
            self._written.add(replaced)
        for seg in self._segments:  # superseded: the manifest names the old base
            self._written.update((seg["slab"], seg["delta"]))
        self._segments = []
        try:
            os.remove(self._path(2))
        except OSError:
            pass
        self._remove_orphan_slabs()

    def _persist_append(self, row0, m):
        """Commit rows [row0, row0 + m), just appended, as one segment (module doc)."""
        if not (self._auto_persist and self._persist_directory and self._index is not None):
            return
        if self._slab_name is None or len(self._segments) >= self.MAX_SEGMENTS:
            return self.persist()
        d = self._persist_directory
        stem = "mq_%s@%s.seg" % (self._collection_name, uuid.uuid4().hex[:12])
        seg = {"slab": stem + ".flat", "delta": stem + ".json", "n_rows": m}
        self._index.save_rows(os.path.join(d, seg["slab"]), row0, m)
        self._write_json(os.path.join(d, seg["delta"]), {
            "ids": self._ids[row0:], "documents": self._texts[row0:], "metadatas": self._metas[row0:]})
        self._write_json(self._path(2), {"base_slab": self._slab_name,  # the commit point
                                         "segments": self._segments + [seg]})
        self._segments.append(seg)

    def _own_slab(self, f):
        """Is file name `f` a slab or segment file of THIS collection (not of 'name.x', whose
        slabs also start with 'mq_name.')?  Its generated names and the legacy single-slab name."""
        prefix, sprefix = "mq_%s." % self._collection_name, "mq_%s@" % self._collection_name
        return f == self._FILES[0] % self._collection_name or (
            f.startswith(prefix) and self._GEN.fullmatch(f[len(prefix):]) is not None) or (
            f.startswith(sprefix) and self._SEG.fullmatch(f[len(sprefix):]) is not None)

    def _remove_orphan_slabs(self):
        """After a commit: delete the slabs this instance replaced (the one it loaded or
        wrote before), and this collection's slabs older than the sidecar by more than
        STALE_SLAB_S (a crashed writer's leftovers).  A younger uncommitted slab may be
        another process's write in flight (ingest and app share the directory), so it is
        left alone; nothing is deleted on load."""
        d = self._persist_directory
        try:
            side_mtime = os.path.getmtime(self._path(1))
        except OSError:
            return
        live = {self._slab_name}
        for seg in self._segments:
            live.update((seg["slab"], seg["delta"]))
        for f in os.listdir(d):
            if f in live or not self._own_slab(f):
                continue
            p = os.path.join(d, f)
            try:
                if f in self._written or os.path.getmtime(p) < side_mtime - self.STALE_SLAB_S:
                    os.remove(p)
            except OSError:
                pass
        self._written.clear()

    def _reindex_host(self):
        self._id_row = _IdRows(self._ids)
        self._cols = _MetaColumns()
        self._cols.append(self._metas)
        self._version += 1

    def _load(self):
        with open(self._path(1), "r", encoding="utf-8") as f:
            side = json.load(f)
        self._ensure_index(side["dim"])
        self._slab_name = side.get("slab", self._FILES[0] % self._collection_name)
        self._written.add(self._slab_name)  # replaced (so deleted) by this instance's first commit
        self._index.load(os.path.join(self._persist_directory, self._slab_name))
        self._ids, self._texts, self._metas = side["ids"], side["documents"], side["metadatas"]
        self._collection_metadata = side.get("collection_metadata", {})
        if len(self._index) != len(self._ids):
            raise RuntimeError("persisted index (%d rows) and sidecar (%d ids) disagree"
                               % (len(self._index), len(self._ids)))
        tail = None
        if os.path.exists(self._path(2)):
            with open(self._path(2), "r", encoding="utf-8") as f:
                tail = json.load(f)
        if tail and tail.get("base_slab") == self._slab_name:  # else superseded by a full write
            d = self._persist_directory
            for seg in tail["segments"]:
                self._index.load_append(os.path.join(d, seg["slab"]))
                with open(os.path.join(d, seg["delta"]), "r", encoding="utf-8") as f:
                    delta = json.load(f)
                self._ids += delta["ids"]
                self._texts += delta["documents"]
                self._metas += delta["metadatas"]
                if len(self._index) != len(self._ids):
                    raise RuntimeError("segment %s (%d rows) and its delta disagree"
                                       % (seg["slab"], seg["n_rows"]))
                self._segments.append(seg)
                self._written.update((seg["slab"], seg["delta"]))  # superseded by the next full write
        self._reindex_host()

    def _embed_query(self, query):
        if self._embedding_function is None:
            raise ValueError("HipChroma needs an embedding_function to search by text")
        return np.asarray(self._embedding_function.embed_query(query), dtype=np.float32)

    def _doc(self, row):
        return Document(page_content=self._texts[row], metadata=dict(self._metas[row]),
                        id=self._ids[row])

    # ---- writes -------------------------------------------------------------------------
    def add_texts(self, texts, metadatas=None, ids=None, **kwargs):
        texts = list(texts)
        if not texts:
            return []
        if ids is None:
            ids = [str(uuid.uuid4()) for _ in texts]
        ids = [str(i) for i in ids]
        metadatas = [dict(m or {}) for m in (metadatas or [{}] * len(texts))]
        if len(metadatas) != len(texts) or len(ids) != len(texts):
            raise ValueError("texts, metadatas and ids must have the same length")
        if self._embedding_function is None:
            raise ValueError("HipChroma needs an embedding_function to add texts")
        if hasattr(self._embedding_function, "embed_array"):
            emb = self._embedding_function.embed_array(texts)
        else:
            emb = np.asarray(self._embedding_function.embed_documents(texts), dtype=np.float32)
        self.add_embeddings(emb, texts, metadatas, ids)
        return ids

    def add_embeddings(self, embeddings, texts, metadatas, ids):
        """Upsert semantics as in Chroma: an existing id is replaced (row rebuilt)."""
        emb = np.ascontiguousarray(embeddings, dtype=np.float32)
        self._ensure_index(emb.shape[1])
        if len(set(ids)) != len(ids):  # last write of a repeated id wins, as in an upsert
            last = {i: j for j, i in enumerate(ids)}
            pick = sorted(last.values())
            emb, texts = emb[pick], [texts[j] for j in pick]
            metadatas, ids = [metadatas[j] for j in pick], [ids[j] for j in pick]
        existing = [i for i in ids if i in self._id_row]
        if existing:
            self.delete(existing, _persist=False)
        self._index.add(emb)
        base = len(self._ids)
        self._ids += ids
        self._texts += texts
        self._metas += metadatas
        self._id_row.extend(ids)
        self._cols.append(metadatas)
        self._version += 1
        if existing:  # rows were replaced: a full write (compaction)
            self._persist()
        else:
            self._persist_append(base, len(ids))

    def delete(self, ids=None, _persist=True, **kwargs):
        if not ids or self._index is None:
            return None
        gone = [i for i in set(ids) if i in self._id_row]
        if not gone:
            return True
        drop = sorted(self._id_row.row(i) for i in gone)
        keepm = np.ones(len(self._ids), bool)
        keepm[drop] = False
        keep = np.flatnonzero(keepm)
        self._index.select(keep, out=self._index)  # device compaction, rows bit-identical
        for name in ("_ids", "_texts", "_metas"):
            setattr(self, name, _drop_sorted(getattr(self, name), drop))
        self._cols.compact(keep)
        self._id_row.compact(keep, gone)
        self._version += 1
        if _persist:
            self._persist()
        return True

    def get(self, ids=None, where=None, limit=None, offset=None, include=None, **kwargs):
        rows = np.arange(len(self._ids))
        if ids is not None:
            want = [ids] if isinstance(ids, str) else ids
            rows = np.array(sorted({self._id_row.row(i) for i in want if i in self._id_row}), np.int64)
        if where:
            rows = rows[self._cols.mask(where)[rows]]
        rows = rows.tolist()[offset or 0:]
        if limit is not None:
            rows = rows[:limit]
        return {"ids": [self._ids[r] for r in rows], "documents": [self._texts[r] for r in rows],
                "metadatas": [self._metas[r] for r in rows]}

    # ---- search -------------------------------------------------------------------------
    def _search_rows(self, vec, k, filter=None):
        """-> list of (row, cosine) for one query vector, best first."""
        n = 0 if self._index is None else len(self._index)
        if n == 0 or k <= 0:
            return []
        q = np.ascontiguousarray(vec, dtype=np.float32).reshape(1, -1)
        if not filter:
            kk = _check_k(k, n)
            s, i = self._index.search(q, kk)
            return [(int(r), float(c)) for r, c in zip(i[0], s[0]) if r >= 0]
        # exact filtered search on the device: the where-mask built from the device codes
        # (mq_mask_eval), then the masked search (int8 certified screen with the mask, or
        # the allowed rows gathered on the device); nothing row-sized crosses PCIe
        if k > _lib.MQ_MAX_K:  # the result count decides between raising and returning all
            k = _check_k(k, int(self._cols.mask(filter).sum()))
            if k == 0:
                return []
        bits = self._cols.dmask(filter, self._device)
        s, i = self._index.search_masked(q, int(k), bits)
        return [(int(r), float(c)) for r, c in zip(i[0], s[0]) if r >= 0]

    def similarity_search_by_vector_with_score(self, embedding, k=DEFAULT_K, filter=None, **kwargs):
        return [(self._doc(r), max(0.0, 2.0 - 2.0 * c)) for r, c in self._search_rows(embedding, k, filter)]

    def similarity_search_by_vector(self, embedding, k=DEFAULT_K, filter=None, **kwargs):
        return [d for d, _ in self.similarity_search_by_vector_with_score(embedding, k, filter)]

    def similarity_search_with_score(self, query, k=DEFAULT_K, filter=None, **kwargs):
        return self.similarity_search_by_vector_with_score(self._embed_query(query), k, filter)

    def similarity_search(self, query, k=DEFAULT_K, filter=None, **kwargs):
        return [d for d, _ in self.similarity_search_with_score(query, k, filter)]

    def similarity_search_with_cosine(self, query, k=DEFAULT_K, filter=None):
        """(Document, cosine similarity) pairs - the index's native score."""
        return [(self._doc(r), c) for r, c in self._search_rows(self._embed_query(query), k, filter)]

    def similarity_search_batch(self, queries, k=DEFAULT_K, filter=None):
        """Many queries in one encoder batch + one device search (the throughput path).
        With `filter`, the where-mask is built once on the device and ONE masked search
        call serves the whole batch (mq_index_search_masked_batch)."""
        n = 0 if self._index is None else len(self._index)
        if n == 0 or not queries or k <= 0:
            return [[] for _ in queries]
        if hasattr(self._embedding_function, "embed_array"):
            q = self._embedding_function.embed_array(list(queries))
        else:
            q = np.asarray(self._embedding_function.embed_documents(list(queries)), np.float32)
        if filter:
            kk = k if k <= _lib.MQ_MAX_K else _check_k(k, int(self._cols.mask(filter).sum()))
            if kk == 0:
                return [[] for _ in queries]
            bits = self._cols.dmask(filter, self._device)
            _, rows = self._index.search_masked(q, int(kk), bits)
            return [[self._doc(int(r)) for r in row if r >= 0] for row in rows]
        kk = _check_k(k, n)
        _, ids = self._index.search(q, kk)
        return [[self._doc(int(r)) for r in row if r >= 0] for row in ids]

    def _select_relevance_score_fn(self):
        if self.override_relevance_score_fn:
            return self.override_relevance_score_fn
        return lambda d: 1.0 - d / math.sqrt(2)  # LangChain's euclidean relevance

    def similarity_search_with_relevance_scores(self, query, k=DEFAULT_K, **kwargs):
        fn = self._select_relevance_score_fn()
        return [(d, fn(s)) for d, s in self.similarity_search_with_score(query, k, **kwargs)]

    # ---- constructors ------------------------------------------------------------------
    @classmethod
    def from_texts(cls, texts, embedding=None, metadatas=None, ids=None,
                   collection_name="langchain", persist_directory=None, **kwargs):
        store = cls(collection_name=collection_name, embedding_function=embedding,
                    persist_directory=persist_directory, _ingest=True, **kwargs)
        store.add_texts(texts, metadatas=metadatas, ids=ids)
        return store

    @classmethod
    def from_documents(cls, documents, embedding=None, ids=None, collection_name="langchain",
                       persist_directory=None, **kwargs):
        documents = list(documents)
        return cls.from_texts([d.page_content for d in documents], embedding,
                              metadatas=[d.metadata for d in documents], ids=ids,
                              collection_name=collection_name,
                              persist_directory=persist_directory, **kwargs)

    def __len__(self):
        return len(self._ids)
