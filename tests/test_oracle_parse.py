"""Oracle parser vs the reference's own output (tests/golden/corpus_docs.json, made by
importing reference src/ingest_medical.py:11-87 - see make_corpus_golden.py)."""
import hashlib
import os

from oracle.parse import parse_custom_format, parse_records


def _digest(records):
    return hashlib.sha256("\x00".join(r["page_content"] for r in records).encode("utf-8")).hexdigest()


def test_parse_matches_reference_golden(golden, corpus_docs):
    recs = parse_custom_format(os.path.join(golden, "medical_data.txt"))
    assert len(recs) == corpus_docs["count"] == 154
    assert recs == corpus_docs["docs"]
    assert _digest(recs) == corpus_docs["sha256_page_content_nul_joined"]
    assert _digest(recs) == "5fca2631cc943500a9d63faa700693bb5f4877307827907b1d7ba3a1ae29790d"


def test_parse_known_corpus_facts(corpus_docs):
    docs = corpus_docs["docs"]
    assert docs[0]["metadata"]["title"] == "常见的慢性病有几种？"
    assert all(d["metadata"]["source"] == "《超越百岁》" for d in docs)
    for a, b in [(72, 74), (104, 105), (110, 111), (120, 121)]:  # duplicate page_content rows
        assert docs[a]["page_content"] == docs[b]["page_content"]


def test_parse_edge_cases(tmp_path):
    assert parse_custom_format(str(tmp_path / "missing.txt")) == []
    assert parse_records("") == []
    # no title -> 未命名; tags label before source cuts the content; no labels -> to end
    txt = ("chunk_id: 1\ncontent: alpha beta\ntags: x, y\nsource: s\n"
           "chunk_id: 2\ntitle: T2\ncontent: tail text")
    r = parse_records(txt)
    assert r[0]["page_content"] == "问题：未命名\n答案：alpha beta"
    assert r[0]["metadata"]["tags"] == "x, y"
    assert r[1]["page_content"] == "问题：T2\n答案：tail text"
    assert r[1]["metadata"]["tags"] == ""
