"""The drop-in boundary driven exactly as the reference drives it (BASELINE config 1):
  ingest  - Chroma.from_documents(documents=docs, embedding=embeddings,
            persist_directory=DB_PATH)                       src/ingest_medical.py:106-110
  engine  - Chroma(persist_directory=DB_PATH, embedding_function=embeddings)
                                                              src/medical_engine.py:52
  node    - [d.page_content for d in vectorstore.similarity_search(q, k=5)]
                                                              src/agents/nodes.py:93-94
with HipBertEmbeddings / HipChroma swapped in.  Expected: the committed config-1 golden
(transformers encoder + float64 exact top-5) within tie groups."""
import json
import os
import time

import numpy as np
import pytest

from mediquery_hip import Document, HipBertEmbeddings, HipChroma
from oracle.flat import check_topk, exact_scores

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def embeddings(require_gpu):
    # seeded weights + char tokenizer: the config-1 golden was made with the same
    return HipBertEmbeddings(model="shaw/dmeta-embedding-zh", synthetic=True)


@pytest.fixture(scope="module")
def docs(corpus_docs):
    return [Document(page_content=d["page_content"], metadata=d["metadata"]) for d in corpus_docs["docs"]]


def test_ingest_then_engine_then_retrieve(embeddings, docs, golden, tmp_path_factory):
    db = str(tmp_path_factory.mktemp("medical_db"))
    Cls = HipChroma
    Cls.from_documents(documents=docs, embedding=embeddings, persist_directory=db)   # ingest
    vectorstore = Cls(persist_directory=db, embedding_function=embeddings)           # engine
    assert len(vectorstore) == 154
    g = np.load(os.path.join(golden, "config1_golden.npz"))
    queries = json.load(open(os.path.join(golden, "config1_queries.json"), encoding="utf-8"))["queries"]
    contents = [d.page_content for d in docs]
    # document embeddings from the GPU match the golden ones
    d_emb = embeddings.embed_array(contents)
    np.testing.assert_allclose(d_emb, g["doc_emb"], atol=1e-4)
    ref = exact_scores(g["query_emb"], g["doc_emb"])
    for qi, q in enumerate(queries):
        got = [d.page_content for d in vectorstore.similarity_search(q, k=5)]      # retrieve node
        assert len(got) == 5
        rows = [r for r, _ in vectorstore._search_rows(vectorstore._embed_query(q), 5)]
        assert [contents[r] for r in rows] == got
        scores = [c for _, c in vectorstore._search_rows(vectorstore._embed_query(q), 5)]
        assert check_topk([rows], [scores], ref[qi:qi + 1], 5) == [], q


@pytest.mark.parametrize("precision,search_precision", [
    ("f32", "screen"), ("f32x6", "screen"), ("f32", "f32"), ("f32x6", "f32x6")])
def test_drop_in_precisions_against_config1_golden(docs, golden, tmp_path, require_gpu, precision,
                                                  search_precision):
    """the arithmetic is selectable on the drop-in -
    HipBertEmbeddings(precision=) (the unchanged OllamaEmbeddings(model=...) line of
    src/medical_engine.py:43 gets the default, f32x6) and HipChroma(search_precision=) -
    and at each setting from_documents -> Chroma(persist_directory=) -> similarity_search
    (src/ingest_medical.py:106-110, src/medical_engine.py:52, src/agents/nodes.py:93)
    reproduces the config-1 golden."""
    from mediquery_hip import OllamaEmbeddings, _lib
    emb = HipBertEmbeddings(model="shaw/dmeta-embedding-zh", synthetic=True, precision=precision)
    assert emb.precision == precision
    default = OllamaEmbeddings(model="shaw/dmeta-embedding-zh", synthetic=True) if precision == "f32x6" else None
    assert default is None or default.precision == "f32x6"
    db = str(tmp_path / "db")
    HipChroma.from_documents(documents=docs, embedding=emb, persist_directory=db, search_precision=search_precision)
    store = HipChroma(persist_directory=db, embedding_function=emb, search_precision=search_precision)
    g = np.load(os.path.join(golden, "config1_golden.npz"))
    queries = json.load(open(os.path.join(golden, "config1_queries.json"), encoding="utf-8"))["queries"]
    contents = [d.page_content for d in docs]
    # a batch of > 64 texts runs the batched GEMMs (the precision applies there)
    np.testing.assert_allclose(emb.embed_array(contents), g["doc_emb"], atol=1e-4)
    ref = exact_scores(g["query_emb"], g["doc_emb"])
    for qi, q in enumerate(queries):
        got = [d.page_content for d in store.similarity_search(q, k=5)]
        rows = [r for r, _ in store._search_rows(store._embed_query(q), 5)]
        assert [contents[r] for r in rows] == got
        scores = [c for _, c in store._search_rows(store._embed_query(q), 5)]
        assert check_topk([rows], [scores], ref[qi:qi + 1], 5) == [], q


def test_scores_distance_semantics_and_edges(embeddings, docs):
    store = HipChroma.from_documents(documents=docs[:20], embedding=embeddings)
    res = store.similarity_search_with_score(docs[3].page_content, k=3)
    assert res[0][0].page_content == docs[3].page_content
    assert res[0][1] == pytest.approx(0.0, abs=1e-5)             # squared L2 of unit vectors
    assert all(a[1] <= b[1] for a, b in zip(res, res[1:]))      # ascending distance
    assert len(store.similarity_search("血糖", k=50)) == 20     # k > N returns N
    empty = HipChroma(embedding_function=embeddings)
    assert empty.similarity_search("血糖", k=5) == []
    ids = store.add_texts(["额外的文本"], metadatas=[{"title": "extra", "tags": "t"}])
    assert store.similarity_search("额外的文本", k=1)[0].metadata["title"] == "extra"
    store.delete(ids)
    assert len(store) == 20
    f = store.similarity_search(docs[5].page_content, k=3, filter={"title": docs[7].metadata["title"]})
    assert [d.metadata["title"] for d in f] == [docs[7].metadata["title"]]


def test_batch_search_matches_single(embeddings, docs):
    store = HipChroma.from_documents(documents=docs, embedding=embeddings)
    qs = [d.page_content[:12] for d in docs[:40]]
    batch = store.similarity_search_batch(qs, k=5)
    for q, b in zip(qs, batch):
        single = store.similarity_search(q, k=5)
        assert [d.page_content for d in b] == [d.page_content for d in single]


def test_k_limit_and_crash_safe_persist(embeddings, docs, tmp_path):
    """k past the device limit raises in every path (n = 154 > 64); every
    write commits through one atomic sidecar replace; bulk ingest can defer writes;
    ingest into a directory holding a stock Chroma database rebuilds it as ours."""
    db = str(tmp_path / "db")
    store = HipChroma.from_documents(documents=docs, embedding=embeddings, persist_directory=db)
    for call in (lambda: store.similarity_search("血糖", k=200),            # k >= n > 64
                 lambda: store.similarity_search("血糖", k=65),
                 lambda: store.similarity_search_batch(["血糖"], k=100),
                 lambda: store.similarity_search("血糖", k=100, filter={"source": "《超越百岁》"})):
        with pytest.raises(ValueError, match="MQ_MAX_K"):
            call()
    assert len(store.similarity_search("血糖", k=64)) == 64
    slabs = [f for f in os.listdir(db) if f.endswith(".flat")]
    assert len(slabs) == 1 and not any(f.endswith(".tmp") for f in os.listdir(db))
    store.add_texts(["额外的文本"], metadatas=[{"title": "extra"}])  # append: base + one segment
    assert sorted(f for f in os.listdir(db) if f.endswith(".flat") and ".seg." not in f) == slabs
    again = HipChroma(persist_directory=db, embedding_function=embeddings)
    assert len(again) == 155
    assert again.similarity_search("额外的文本", k=1)[0].metadata["title"] == "extra"
    store.persist()  # a full write: new generation, old slab and the segment removed
    slabs2 = [f for f in os.listdir(db) if f.endswith(".flat")]
    assert len(slabs2) == 1 and slabs2 != slabs and not any(f.endswith(".tmp") for f in os.listdir(db))
    assert len(HipChroma(persist_directory=db, embedding_function=embeddings)) == 155

    bulk_db = str(tmp_path / "bulk")
    bulk = HipChroma.from_documents(documents=docs[:10], embedding=embeddings,
                                    persist_directory=bulk_db, auto_persist=False)
    assert not os.path.exists(os.path.join(bulk_db, "mq_langchain.json"))
    bulk.persist()
    assert len(HipChroma(persist_directory=bulk_db, embedding_function=embeddings)) == 10

    old = tmp_path / "old_chroma"
    old.mkdir()
    (old / "chroma.sqlite3").write_bytes(b"SQLite format 3\x00")
    with pytest.raises(RuntimeError, match="ChromaDB"):
        HipChroma(persist_directory=str(old), embedding_function=embeddings)
    HipChroma.from_documents(documents=docs[:5], embedding=embeddings, persist_directory=str(old))
    assert len(HipChroma(persist_directory=str(old), embedding_function=embeddings)) == 5


def test_upsert_by_existing_id_replaces_row_and_persists(embeddings, docs, tmp_path):
    """Chroma upsert semantics (`add_texts` with an id that exists, reference ingest
    src/ingest_medical.py:106-110 runs through add_texts): the row is replaced - one row
    per id, searches return the new text and metadata, a persisted reload agrees, and
    slabs left uncommitted are never touched at load (one may be another process's write
    in flight: ingest and app share the directory) and are swept by a later commit once
    stale, as is the slab that commit replaced; a sibling collection's slab survives."""
    db = str(tmp_path / "db")
    ids = ["doc%03d" % i for i in range(30)]
    store = HipChroma.from_documents(documents=docs[:30], embedding=embeddings, ids=ids,
                                     persist_directory=db)
    new_text = "更新后的内容：每天步行八千步有益健康"
    store.add_texts([new_text, docs[40].page_content], metadatas=[{"title": "updated"}, {"title": "d40"}],
                    ids=["doc007", "doc100"])
    assert len(store) == 31
    got = store.get(ids=["doc007"])
    assert got["documents"] == [new_text] and got["metadatas"] == [{"title": "updated"}]
    top = store.similarity_search(new_text, k=1)[0]
    assert top.page_content == new_text and top.metadata["title"] == "updated"
    assert all(d.page_content != docs[7].page_content for d in store.similarity_search(docs[7].page_content, k=5))
    # repeated ids inside one call: the last one wins
    store.add_texts(["甲", "乙"], ids=["dupe", "dupe"])
    assert store.get(ids=["dupe"])["documents"] == ["乙"] and len(store) == 32
    # filtered search after writes sees the new rows (the filter cache is keyed on writes)
    assert [d.page_content for d in store.similarity_search(new_text, k=3, filter={"title": "updated"})] == [new_text]
    store.delete(["doc007"])
    assert store.similarity_search(new_text, k=3, filter={"title": "updated"}) == []
    young, stale = "mq_langchain.deadbeef0000.flat", "mq_langchain.0badc0ffee00.flat"
    sibling = "mq_langchain.v2.0123456789ab.flat"  # collection "langchain.v2"
    for f in (young, stale, sibling):
        open(os.path.join(db, f), "wb").write(b"orphan")
    t_old = time.time() - 2 * HipChroma.STALE_SLAB_S
    os.utime(os.path.join(db, stale), (t_old, t_old))
    committed = store._slab_name
    again = HipChroma(persist_directory=db, embedding_function=embeddings)
    assert len(again) == 31 and again.get(ids=["doc007"])["ids"] == []
    assert again.get(ids=["dupe"])["documents"] == ["乙"]
    assert sorted(f for f in os.listdir(db) if f.endswith(".flat")) == sorted([committed, young, stale, sibling])
    s1 = [d.page_content for d in store.similarity_search(docs[3].page_content, k=5)]
    s2 = [d.page_content for d in again.similarity_search(docs[3].page_content, k=5)]
    assert s1 == s2
    again.add_texts(["新增"], ids=["doc200"])  # an append: one segment, nothing swept
    assert len([f for f in os.listdir(db) if f.endswith(".seg.flat")]) == 1
    assert len(HipChroma(persist_directory=db, embedding_function=embeddings)) == 32
    again.persist()  # a full write: the replaced + stale slabs and the superseded segment go
    assert sorted(f for f in os.listdir(db) if f.endswith(".flat")) == sorted([again._slab_name, young, sibling])
    assert len(HipChroma(persist_directory=db, embedding_function=embeddings)) == 32


def test_filtered_search_equals_oracle_on_allowed_rows(embeddings, docs):
    """filter= scores only the allowed rows (the where-mask built on the device from the
    metadata code columns, then one masked search - the masked scan, or at this store size
    the masked row gather): the result equals the exact top-k over the rows _match admits,
    for several filters in a row and for a repeated one."""
    from mediquery_hip.vectorstore import _match
    store = HipChroma.from_documents(documents=docs, embedding=embeddings)
    emb = embeddings.embed_array([d.page_content for d in docs])
    titles = sorted({d.metadata["title"] for d in docs})
    filters = [{"source": "《超越百岁》"}, {"title": {"$in": titles[:40]}},
               {"$or": [{"title": titles[3]}, {"title": titles[9]}]}, {"title": {"$in": titles[:40]}}]
    q = docs[11].page_content
    qe = embeddings.embed_array([q])
    for f in filters:
        allowed = np.array([r for r, d in enumerate(docs) if _match(d.metadata, f)])
        got = store._search_rows(qe[0], 5, f)
        ref = exact_scores(qe, emb[allowed])[0]
        order = np.lexsort((allowed, -ref))[:5]
        assert [r for r, _ in got] == allowed[order].tolist(), f


def test_append_only_persistence(embeddings, docs, tmp_path):
    """add_texts of new ids writes one segment (rows + a delta of their documents) and
    commits it by replacing the small manifest; the base slab and sidecar are untouched.
    A reload applies the committed segments in order (rows bit-identical), ignores an
    uncommitted segment and a manifest that names a superseded base; delete compacts into
    a new base and drops the segments."""
    db = str(tmp_path / "db")
    ids = ["doc%03d" % i for i in range(30)]
    store = HipChroma.from_documents(documents=docs[:30], embedding=embeddings, ids=ids, persist_directory=db)
    side = os.path.join(db, "mq_langchain.json")
    base_slab, side_bytes = store._slab_name, open(side, "rb").read()
    store.add_texts([docs[40].page_content, docs[41].page_content], metadatas=[{"t": 40}, {"t": 41}],
                    ids=["doc040", "doc041"])
    store.add_texts([docs[42].page_content], metadatas=[{"t": 42}], ids=["doc042"])
    assert open(side, "rb").read() == side_bytes and store._slab_name == base_slab
    tail = json.load(open(os.path.join(db, "mq_langchain@tail.json")))
    assert tail["base_slab"] == base_slab and [g["n_rows"] for g in tail["segments"]] == [2, 1]
    # an uncommitted segment (a writer that crashed before the manifest) is not loaded
    open(os.path.join(db, "mq_langchain@0123456789ab.seg.flat"), "wb").write(b"partial")
    again = HipChroma(persist_directory=db, embedding_function=embeddings)
    assert len(again) == 33 and again.get(ids=["doc041"])["metadatas"] == [{"t": 41}]
    assert np.array_equal(again._index.get(), store._index.get())  # bit-identical rows
    q = docs[41].page_content
    assert [d.page_content for d in again.similarity_search(q, k=5)] == \
        [d.page_content for d in store.similarity_search(q, k=5)]
    assert again.similarity_search(q, k=1, filter={"t": 41})[0].page_content == q
    # upsert of an existing id and delete compact: a new base, no segments
    again.delete(["doc040"])
    assert not os.path.exists(os.path.join(db, "mq_langchain@tail.json"))
    assert [f for f in os.listdir(db) if f.endswith(".seg.flat")] == ["mq_langchain@0123456789ab.seg.flat"]
    third = HipChroma(persist_directory=db, embedding_function=embeddings)
    assert len(third) == 32 and third.get(ids=["doc040"])["ids"] == []
    # a manifest that names a superseded base (another writer's full write won) is ignored
    json.dump({"base_slab": base_slab, "segments": tail["segments"]},
              open(os.path.join(db, "mq_langchain@tail.json"), "w"))
    assert len(HipChroma(persist_directory=db, embedding_function=embeddings)) == 32


def test_append_one_doc_to_1m_store_persists_fast(embeddings, tmp_path):
    """adding one document to a 1M-row persisted store commits in
    <= 50 ms (append-only segment + manifest; the whole-slab rewrite it replaces wrote
    3 GB and a 1M-document sidecar)."""
    db = str(tmp_path / "db")
    rng = np.random.default_rng(5)
    n = 1_000_000
    emb = rng.standard_normal((n, 768), dtype=np.float32)
    store = HipChroma(persist_directory=db, embedding_function=embeddings, auto_persist=False, _ingest=True)
    store.add_embeddings(emb, ["d%d" % i for i in range(n)], [{} for _ in range(n)], ["id%d" % i for i in range(n)])
    del emb
    store.persist()
    store._auto_persist = True
    one = rng.standard_normal((1, 768), dtype=np.float32)
    times = []
    for j in range(5):
        t0 = time.perf_counter()
        store.add_embeddings(one, ["new%d" % j], [{"j": j}], ["new%d" % j])
        times.append((time.perf_counter() - t0) * 1e3)
    print("append_one_doc_ms_1m", [round(t, 2) for t in times])
    assert sorted(times)[2] <= 50.0, times
    again = HipChroma(persist_directory=db, embedding_function=embeddings)
    assert len(again) == n + 5 and again.get(ids=["new3"])["metadatas"] == [{"j": 3}]

