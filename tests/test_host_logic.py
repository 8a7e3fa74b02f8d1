"""Host-side logic of the boundary that needs no device: metadata filters, shard
bounds, WordPiece tokenisation, the Document stand-in."""
import numpy as np

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
