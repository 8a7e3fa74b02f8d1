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
file) is the commit point; each write puts the rows in a fresh `mq_<collection>.<gen>.flat`
and then atomically replaces the JSON, so a crash leaves either the old or the new store,
never a slab/sidecar mismatch.  A directory that holds a stock Chroma database
(`chroma.sqlite3`, written by the reference's ingest) but no sidecar is refused: it must be
re-ingested with this store (`python src/ingest_medical.py` after the import swap).
"""
import json
import math
import os
import uuid

import numpy as np

from . import _lib
from .compat import Document, VectorStoreBase
from .native import FlatIndex

DEFAULT_K = 4  # LangChain VectorStore.similarity_search default; the reference passes k=5


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
                    if not ok():
                        return False
            elif v != cond:
                return False
    return True


def _check_k(k, n_candidates):
    """Result count of a top-k over n_candidates rows; raises past the device limit."""
    kk = min(int(k), int(n_candidates))
    if kk > _lib.MQ_MAX_K:
        raise ValueError("a search returning %d results (k=%d over %d rows) exceeds the device "
                         "top-k limit MQ_MAX_K=%d" % (kk, k, n_candidates, _lib.MQ_MAX_K))
    return kk


class HipChroma(VectorStoreBase):
    _FILES = ("mq_%s.flat", "mq_%s.json")
    FOREIGN_DB = "chroma.sqlite3"  # what langchain_chroma / chromadb persist

    def __init__(self, collection_name="langchain", embedding_function=None,
                 persist_directory=None, client_settings=None, collection_metadata=None,
                 client=None, relevance_score_fn=None, *, device=0, dim=None,
                 auto_persist=True, _ingest=False, **kwargs):
        """auto_persist=False: writes stay in memory until `persist()` (bulk ingest)."""
        self._collection_name = collection_name
        self._embedding_function = embedding_function
        self._persist_directory = persist_directory
        self._collection_metadata = dict(collection_metadata or {})
        self.override_relevance_score_fn = relevance_score_fn
        self._device = device
        self._auto_persist = bool(auto_persist)
        self._ids, self._texts, self._metas = [], [], []
        self._index = None
        self._dim = dim
        self._slab_name = None
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
            # exact fp32 top-k; batched searches run the certified split-f32 screen
            self._index.set_precision(_lib.MQ_DTYPE_F32_SCREEN)
        elif dim != self._dim:
            raise ValueError("embedding dim %d != collection dim %d" % (dim, self._dim))

    def _persist(self):
        if self._auto_persist:
            self.persist()

    def persist(self):
        """Write the store under persist_directory (crash-safe, see the module doc)."""
        if not self._persist_directory or self._index is None:
            return
        d = self._persist_directory
        os.makedirs(d, exist_ok=True)
        slab = "mq_%s.%s.flat" % (self._collection_name, uuid.uuid4().hex[:12])
        self._index.save(os.path.join(d, slab))
        side = self._path(1)
        tmp = side + ".tmp"
        with open(tmp, "w", encoding="utf-8") as f:
            json.dump({"dim": self._dim, "slab": slab, "n_rows": len(self._ids), "ids": self._ids,
                       "documents": self._texts, "metadatas": self._metas,
                       "collection_metadata": self._collection_metadata}, f, ensure_ascii=False)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, side)  # the commit point
        old, self._slab_name = self._slab_name, slab
        for stale in (old, self._FILES[0] % self._collection_name):
            if stale and stale != slab and os.path.exists(os.path.join(d, stale)):
                os.remove(os.path.join(d, stale))

    def _load(self):
        with open(self._path(1), "r", encoding="utf-8") as f:
            side = json.load(f)
        self._ensure_index(side["dim"])
        self._slab_name = side.get("slab", self._FILES[0] % self._collection_name)
        self._index.load(os.path.join(self._persist_directory, self._slab_name))
        self._ids, self._texts, self._metas = side["ids"], side["documents"], side["metadatas"]
        self._collection_metadata = side.get("collection_metadata", {})
        if len(self._index) != len(self._ids):
            raise RuntimeError("persisted index (%d rows) and sidecar (%d ids) disagree"
                               % (len(self._index), len(self._ids)))

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
        existing = set(self._ids).intersection(ids)
        if existing:
            self.delete(list(existing), _persist=False)
        self._index.add(emb)
        self._ids += ids
        self._texts += texts
        self._metas += metadatas
        self._persist()

    def delete(self, ids=None, _persist=True, **kwargs):
        if not ids or self._index is None:
            return None
        drop = set(ids)
        keep = [r for r, i in enumerate(self._ids) if i not in drop]
        self._index.select(keep, out=self._index)  # device compaction, rows bit-identical
        self._ids = [self._ids[r] for r in keep]
        self._texts = [self._texts[r] for r in keep]
        self._metas = [self._metas[r] for r in keep]
        if _persist:
            self._persist()
        return True

    def get(self, ids=None, where=None, limit=None, offset=None, include=None, **kwargs):
        rows = range(len(self._ids))
        if ids is not None:
            want = set([ids] if isinstance(ids, str) else ids)
            rows = [r for r in rows if self._ids[r] in want]
        if where:
            rows = [r for r in rows if _match(self._metas[r], where)]
        rows = list(rows)[offset or 0:]
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
        allowed = np.array([r for r in range(n) if _match(self._metas[r], filter)], dtype=np.int64)
        if len(allowed) == 0:
            return []
        # exact filtered search: score only the allowed rows, gathered on the device into
        # a scratch index (rows bit-identical to the store's)
        sub = self._index.select(allowed)
        kk = _check_k(k, len(allowed))
        s, i = sub.search(q, kk)
        sub.close()
        return [(int(allowed[r]), float(c)) for r, c in zip(i[0], s[0]) if r >= 0]

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

    def similarity_search_batch(self, queries, k=DEFAULT_K):
        """Many queries in one encoder batch + one device search (the throughput path)."""
        n = 0 if self._index is None else len(self._index)
        if n == 0 or not queries or k <= 0:
            return [[] for _ in queries]
        kk = _check_k(k, n)
        if hasattr(self._embedding_function, "embed_array"):
            q = self._embedding_function.embed_array(list(queries))
        else:
            q = np.asarray(self._embedding_function.embed_documents(list(queries)), np.float32)
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
