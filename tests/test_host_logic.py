"""Host-side logic of the boundary that needs no device: metadata filters, shard
bounds, WordPiece tokenisation, the Document stand-in."""
import numpy as np
import pytest

from mediquery_hip.compat import Document
from mediquery_hip.distributed import shard_bounds
from mediquery_hip.tokenizer import WordPieceTokenizer
from mediquery_hip.vectorstore import _match


def test_metadata_filter():
    m = {"title": "a", "n": 3, "tags": "x"}
    assert _match(m, {"title": "a"})
    assert not _match(m, {"title": "b"})
    assert _match(m, {"n": {"$gte": 3}}) and not _match(m, {"n": {"$lt": 3}})
    assert _match(m, {"$or": [{"title": "b"}, {"tags": {"$in": ["x", "y"]}}]})
    assert not _match(m, {"$and": [{"title": "a"}, {"n": {"$ne": 3}}]})


def test_shard_bounds_cover_rows_exactly():
    for n in (0, 1, 7, 1000, 10_000_001):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, w, r) for r in range(w)]
            assert spans[0][0] == 0
            assert sum(c for _, c in spans) == n
            for (o1, c1), (o2, _) in zip(spans, spans[1:]):
                assert o1 + c1 == o2


def test_wordpiece(tmp_path):
    vocab = ["[PAD]"] + ["[unused%d]" % i for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]",
                                                                "[MASK]", "x", "y", "血", "糖", "high", "##er"]
    p = tmp_path / "vocab.txt"
    p.write_text("\n".join(vocab) + "\n", encoding="utf-8")
    t = WordPieceTokenizer(str(p))
    v = {w: i for i, w in enumerate(vocab)}
    assert t.encode("血糖 Higher zz") == [v["[CLS]"], v["血"], v["糖"], v["high"], v["##er"],
                                          v["[UNK]"], v["[SEP]"]]


def test_document_stand_in():
    d = Document(page_content="问题：x", metadata={"title": "x"})
    assert d.page_content == "问题：x" and d.metadata["title"] == "x"


def test_k_limit_is_enforced_on_result_count():
    """the device top-k limit applies to min(k, candidates) in every path."""
    import pytest
    from mediquery_hip import MQ_MAX_K
    from mediquery_hip.vectorstore import _check_k
    assert _check_k(5, 154) == 5
    assert _check_k(50, 20) == 20                      # k > N returns N
    assert _check_k(1000, MQ_MAX_K) == MQ_MAX_K
    for k, n in ((MQ_MAX_K + 1, 1000), (1000, MQ_MAX_K + 1), (200, 100)):
        with pytest.raises(ValueError, match="MQ_MAX_K"):
            _check_k(k, n)


def test_foreign_chroma_db_is_refused(tmp_path):
    """a stock Chroma directory must not open as an empty store."""
    import pytest
    from mediquery_hip.vectorstore import HipChroma
    (tmp_path / "chroma.sqlite3").write_bytes(b"SQLite format 3\x00")
    with pytest.raises(RuntimeError, match="re-run the ingest|Re-run the ingest"):
        HipChroma(persist_directory=str(tmp_path), embedding_function=None)
    HipChroma(persist_directory=str(tmp_path / "fresh"))  # a new directory is fine


def test_embeddings_refuse_silent_synthetic(tmp_path, monkeypatch):
    """the real model name without local weights + vocab raises; synthetic
    weights need synthetic=True; weights without a vocab raise."""
    import pytest
    from mediquery_hip.embeddings import ENV_VOCAB, ENV_WEIGHTS, HipBertEmbeddings
    monkeypatch.delenv(ENV_WEIGHTS, raising=False)
    monkeypatch.delenv(ENV_VOCAB, raising=False)
    monkeypatch.delenv("MQ_GGUF_PATH", raising=False)
    monkeypatch.setenv("OLLAMA_MODELS", str(tmp_path / "no_ollama_store"))
    with pytest.raises(ValueError, match="synthetic=True"):
        HipBertEmbeddings(model="shaw/dmeta-embedding-zh")
    w = tmp_path / "w.safetensors"
    w.write_bytes(b"")
    with pytest.raises(ValueError, match="vocab"):
        HipBertEmbeddings(weights_path=str(w))
    monkeypatch.setenv(ENV_WEIGHTS, str(w))
    with pytest.raises(ValueError, match="vocab"):
        HipBertEmbeddings()
    monkeypatch.setenv(ENV_VOCAB, str(tmp_path / "missing.txt"))
    with pytest.raises(FileNotFoundError):
        HipBertEmbeddings()
    with pytest.raises(ValueError, match="synthetic"):
        HipBertEmbeddings(synthetic=True, weights_path=str(w))


def test_metadata_columns_equal_row_filter():
    """The vectorised column filter (filtered searches, get(where=)) equals the row-wise
    Chroma `where` semantics on random metadata: missing keys, mixed types, bool vs int,
    compaction after deletes."""
    from mediquery_hip.vectorstore import _MetaColumns
    rng = np.random.default_rng(0)
    titles = ["t%d" % i for i in range(7)]
    metas = []
    for r in range(3000):
        m = {}
        if rng.random() < 0.9:
            m["title"] = titles[rng.integers(7)]
        if rng.random() < 0.7:
            m["n"] = int(rng.integers(0, 10))
        if rng.random() < 0.3:
            m["flag"] = bool(rng.integers(2))
        if rng.random() < 0.2:
            m["x"] = float(rng.standard_normal())
        metas.append(m)
    cols = _MetaColumns()
    cols.append(metas[:1000])
    cols.append(metas[1000:])
    wheres = [{"title": "t3"}, {"n": {"$gte": 5}}, {"n": {"$lt": 2}, "title": {"$ne": "t1"}},
              {"$or": [{"flag": True}, {"n": {"$in": [1, 3, 7]}}]}, {"missing": {"$nin": ["a"]}},
              {"$and": [{"x": {"$gt": 0.5}}, {"title": {"$in": titles[:3]}}]}, {"flag": 1},
              {"n": {"$ne": 4}}, {"missing": "z"}]
    for w in wheres:
        np.testing.assert_array_equal(cols.mask(w), [_match(m, w) for m in metas], err_msg=str(w))
    keep = np.flatnonzero(rng.random(3000) < 0.6)
    cols.compact(keep)
    kept = [metas[r] for r in keep]
    cols.append([{"title": "new", "n": 5}])
    kept.append({"title": "new", "n": 5})
    for w in wheres + [{"title": "new"}]:
        np.testing.assert_array_equal(cols.mask(w), [_match(m, w) for m in kept], err_msg=str(w))


def test_metadata_mixed_types_compare_as_no_match():
    """A range operator on a key whose values mix strings and numbers matches only the
    comparable values (Chroma's typed comparison), in both the row and column filters,
    instead of raising TypeError."""
    from mediquery_hip.vectorstore import _MetaColumns
    metas = [{"n": 3}, {"n": "7"}, {"n": 9.5}, {}, {"n": None}]
    cols = _MetaColumns()
    cols.append(metas)
    for w in ({"n": {"$gt": 4}}, {"n": {"$lte": 3}}, {"n": {"$gt": "5"}}):
        want = [_match(m, w) for m in metas]
        np.testing.assert_array_equal(cols.mask(w), want, err_msg=str(w))
    assert [_match(m, {"n": {"$gt": 4}}) for m in metas] == [False, False, True, False, False]
    assert [_match(m, {"n": {"$gt": "5"}}) for m in metas] == [False, True, False, False, False]


def test_metadata_numeric_tables_equal_row_filter():
    """The numpy truth tables of numeric comparisons (columns of > 8 distinct numbers)
    equal the row-wise semantics: ints and floats mixed, a bool among ints (exact path),
    an int past 2^53 (exact path), NaN."""
    from mediquery_hip.vectorstore import _MetaColumns
    metas = [{"n": i % 100, "f": (i % 37) / 3.0} for i in range(2000)]
    metas[3]["n"] = 2.5
    metas[7]["f"] = float("nan")
    metas2 = [dict(m) for m in metas]
    metas2[11]["n"] = True
    metas2[12]["f"] = 2 ** 60 + 1
    for ms in (metas, metas2):
        cols = _MetaColumns()
        cols.append(ms)
        for w in ({"n": {"$lt": 50}}, {"n": {"$gte": 2.5}}, {"n": {"$eq": 1}}, {"n": {"$ne": 4}},
                  {"f": {"$gt": 3.5}}, {"f": {"$lte": 2 ** 60}}, {"n": {"$gt": True}}):
            np.testing.assert_array_equal(cols.mask(w), [_match(m, w) for m in ms], err_msg=str(w))


def test_orphan_slab_sweep_spares_sibling_collections_and_writes_in_flight(tmp_path):
    """persist()'s sweep deletes only THIS collection's slabs that this instance replaced
    or that are stale crash leftovers: never a sibling collection's ('docs' vs 'docs.v2'),
    never another writer's fresh uncommitted slab, and nothing at load time."""
    import os
    import time
    from mediquery_hip.vectorstore import HipChroma
    d = str(tmp_path)
    store = HipChroma(collection_name="docs")  # no index yet: host-only object
    store._persist_directory = d
    names = {"own_old": "mq_docs.0123456789ab.flat", "own_cur": "mq_docs.aaaaaaaaaaaa.flat",
             "legacy": "mq_docs.flat", "sibling": "mq_docs.v2.bbbbbbbbbbbb.flat",
             "sibling_legacy": "mq_docs.v2.flat", "inflight": "mq_docs.cccccccccccc.flat",
             "stale": "mq_docs.dddddddddddd.flat", "other": "notes.flat"}
    for n in names.values():
        open(os.path.join(d, n), "wb").close()
    open(os.path.join(d, "mq_docs.json"), "w").close()
    old = time.time() - 2 * HipChroma.STALE_SLAB_S
    os.utime(os.path.join(d, names["stale"]), (old, old))
    assert store._own_slab(names["own_old"]) and store._own_slab(names["legacy"])
    assert not store._own_slab(names["sibling"]) and not store._own_slab(names["sibling_legacy"])
    store._slab_name = names["own_cur"]
    store._written = {names["own_old"], names["legacy"]}
    store._remove_orphan_slabs()
    left = set(os.listdir(d))
    assert names["own_old"] not in left and names["legacy"] not in left
    assert names["stale"] not in left
    for keep in ("own_cur", "sibling", "sibling_legacy", "inflight", "other"):
        assert names[keep] in left, keep


def test_id_rows_map_tracks_deletes_like_a_dict():
    """_IdRows (id -> row across deletes, numpy renumbering; VERDICT r5 #9's vectorised
    delete) against a rebuilt dict, over random append / delete rounds incl. the dead-slot
    reclaim; _drop_sorted against a comprehension."""
    from mediquery_hip.vectorstore import _IdRows, _drop_sorted
    rng = np.random.default_rng(0)
    ids, m = [], _IdRows()
    nxt = 0
    for rnd in range(60):
        add = ["id%d" % (nxt + j) for j in range(int(rng.integers(0, 400)))]
        nxt += len(add)
        ids += add
        m.extend(add)
        if ids and rnd % 2:
            gone = set(rng.choice(ids, size=min(len(ids), int(rng.integers(1, 300))), replace=False).tolist())
            drop = sorted(m.row(i) for i in gone)
            keepm = np.ones(len(ids), bool)
            keepm[drop] = False
            new = _drop_sorted(ids, drop)
            assert new == [v for v, kp in zip(ids, keepm.tolist()) if kp]
            ids = new
            m.compact(np.flatnonzero(keepm), gone)
        assert len(m) == len(ids)
        assert all(m.row(i) == r for r, i in enumerate(ids))
        assert all(("id%d" % j in m) == ("id%d" % j in set(ids)) for j in range(0, nxt, 97))


def test_mask_word_checks_without_a_gpu():
    """the mask wrappers reject a host tensor, a wrong element width, too few
    words, and a mask on another device than the index (checked before any launch)."""
    import torch
    from mediquery_hip.native import check_mask_words
    with pytest.raises(ValueError):
        check_mask_words(torch.zeros(4, dtype=torch.int32), 100)  # host memory

    class FakeDev:  # duck-typed device tensor (no GPU here)
        is_cuda = True

        def __init__(self, n, width=4, index=1):
            self._n, self._w = n, width
            self.device = type("D", (), {"index": index})()

        def element_size(self):
            return self._w

        def is_contiguous(self):
            return True

        def numel(self):
            return self._n

    check_mask_words(FakeDev(4), 100, device=1)
    with pytest.raises(ValueError, match="ceil"):
        check_mask_words(FakeDev(3), 100)
    with pytest.raises(ValueError):
        check_mask_words(FakeDev(4, width=8), 100)
    with pytest.raises(ValueError, match="cuda:1"):
        check_mask_words(FakeDev(4, index=1), 100, device=0)


def test_precision_arguments_are_validated():
    """HipBertEmbeddings(precision=) / HipChroma(search_precision=) take the documented
    names only."""
    from mediquery_hip import HipBertEmbeddings, HipChroma
    from mediquery_hip.embeddings import DEFAULT_PRECISION, PRECISIONS
    from mediquery_hip.vectorstore import SEARCH_PRECISIONS
    assert DEFAULT_PRECISION == "f32x6" and set(PRECISIONS) == {"f32", "f32x6"}
    assert set(SEARCH_PRECISIONS) == {"screen", "f32", "f32x6", "bf16"}
    with pytest.raises(ValueError, match="precision"):
        HipBertEmbeddings(synthetic=True, precision="bf16")
    with pytest.raises(ValueError, match="search_precision"):
        HipChroma(search_precision="hnsw")
