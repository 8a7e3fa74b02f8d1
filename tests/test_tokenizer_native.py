"""C++ tokenizers (mq_tokenizer_*, host code, no GPU) against their Python twins on the
real corpus, the config-1 queries and edge cases."""
import json
import os

import numpy as np
import pytest

from mediquery_hip.tokenizer import CharTokenizer, NativeTokenizer, WordPieceTokenizer

EDGE = ["", " ", "\t\n", "abc", "ABC Déjà vu ÆØÅ ß", "血糖,高!", "（括号）【标题】：问题？",
        "a​b­c", "emoji 😀 ok", "ＡＢＣ１２３", "x" * 700, "中" * 600, "Ωμέγα Привет Йод ёж", "ĀāĞğİıĲĳĸĹĺĿŀŁłŉŊŋŒœŦŧŸſ", "ÀÉÎÕÜÆÐØÞßàéîõüæðøþÿ×÷"]


def _texts(golden):
    docs = json.load(open(os.path.join(golden, "corpus_docs.json"), encoding="utf-8"))["docs"]
    qs = json.load(open(os.path.join(golden, "config1_queries.json"), encoding="utf-8"))["queries"]
    return [d["page_content"] for d in docs] + qs + EDGE


def test_char_tokenizer_native_matches_python(golden):
    texts = _texts(golden)
    py = CharTokenizer(21128, max_length=512)
    nat = NativeTokenizer.char(21128, max_length=512)
    for t in texts:
        assert nat.encode(t) == py.encode(t), t[:30]
    ids_p, mask_p = py(texts)
    ids_n, mask_n = nat(texts)
    np.testing.assert_array_equal(ids_n, ids_p)
    np.testing.assert_array_equal(mask_n, mask_p)
    ids_n, _ = nat(["ab"], pad_to=40)
    assert ids_n.shape == (1, 40)


def test_wordpiece_native_matches_python(golden, tmp_path):
    texts = _texts(golden)
    # vocab: specials, every character of the texts, and some multi-char pieces
    chars = sorted({c for t in texts for c in t.lower() if not c.isspace()})
    pieces = ["high", "##er", "##s", "abc", "##c", "vu", "dej", "##a", "ok", "emoji", "x", "##x"]
    vocab = ["[PAD]"] + ["[unused%d]" % i for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    vocab += [c for c in chars if c not in vocab] + pieces + ["##" + c for c in chars[:200]]
    p = tmp_path / "vocab.txt"
    p.write_text("\n".join(vocab) + "\n", encoding="utf-8")
    py = WordPieceTokenizer(str(p), max_length=512)
    nat = NativeTokenizer.wordpiece(str(p), max_length=512)
    bad = [t[:30] for t in texts if nat.encode(t) != py.encode(t)]
    assert not bad, bad[:5]


@pytest.mark.parametrize("case", ["lower", "cased"])
def test_wordpiece_matches_published_bert_tokenizer(golden, case):
    """Bit-exact ids of transformers.BertTokenizer (the tokenizers crate's BertNormalizer
    + BertPreTokenizer + WordPiece) on a local vocab: 154 docs, 32 queries, edge strings
    (controls, private use, unassigned, NFD accents, Hangul, CJK compatibility and
    extension ranges, final sigma, >100-char words, 512-token truncation).  Fixture made
    by tests/golden/make_wordpiece_golden.py; reference site src/medical_engine.py:43."""
    g = json.load(open(os.path.join(golden, "wordpiece_golden.json"), encoding="utf-8"))
    c = g["cases"][case]
    vocab = os.path.join(golden, g["vocab"])
    nat = NativeTokenizer.wordpiece(vocab, max_length=g["max_length"], lower_case=c["do_lower_case"])
    py = WordPieceTokenizer(vocab, max_length=g["max_length"], lower_case=c["do_lower_case"])
    bad_n = [j for j, (t, ids) in enumerate(zip(g["texts"], c["ids"])) if nat.encode(t) != ids]
    bad_p = [j for j, (t, ids) in enumerate(zip(g["texts"], c["ids"])) if py.encode(t) != ids]
    assert not bad_n, [g["texts"][j][:20] for j in bad_n[:5]]
    assert not bad_p, [g["texts"][j][:20] for j in bad_p[:5]]
    # the batched call pads to the longest sequence, as the encoder consumes it
    ids, mask = nat(g["texts"][:40])
    for j in range(40):
        n = int(mask[j].sum())
        assert ids[j, :n].tolist() == c["ids"][j] and not ids[j, n:].any()
