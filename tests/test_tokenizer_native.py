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


def _random_texts(rng, n):
    """Random strings over the code-point classes the normaliser branches on: ASCII,
    Latin-1 accents, combining marks, CJK (BMP + extension B), Hangul, fullwidth forms,
    controls / format characters, private use, emoji, whitespace."""
    ranges = [(0x20, 0x7e), (0xc0, 0x17f), (0x300, 0x36f), (0x4e00, 0x9fff), (0x20000, 0x2a6df),
              (0xac00, 0xd7a3), (0xff01, 0xff5e), (0x0, 0x1f), (0x200b, 0x200f), (0xe000, 0xf8ff),
              (0x1f600, 0x1f64f), (0x3000, 0x303f)]
    out = []
    for _ in range(n):
        cps = []
        for _ in range(int(rng.integers(0, 1500))):
            lo, hi = ranges[int(rng.integers(len(ranges)))]
            cp = int(rng.integers(lo, hi + 1))
            cps.append(cp if cp else 0x20)  # (no NUL: the C ABI takes NUL-terminated strings)
        out.append("".join(map(chr, cps)))
    return out


def test_native_tokenizers_on_random_text_and_raw_bytes(golden):
    """Host-code robustness (also run under ASan + UBSan by tools/sanitize_cpu_tests.sh):
    random strings over every character class give the Python twins' ids; raw byte
    strings that are not UTF-8 (stray continuation bytes, truncated sequences, overlong
    forms, surrogates, > U+10FFFF) go through the C ABI without a fault, with ids inside
    the vocabulary and a mask that is a prefix of ones."""
    import ctypes
    from mediquery_hip import _lib
    rng = np.random.default_rng(123)
    g = json.load(open(os.path.join(golden, "wordpiece_golden.json"), encoding="utf-8"))
    vocab = os.path.join(golden, g["vocab"])
    texts = _random_texts(rng, 60)
    for nat, py in ((NativeTokenizer.char(21128, max_length=512), CharTokenizer(21128, max_length=512)),
                    (NativeTokenizer.wordpiece(vocab, max_length=512), WordPieceTokenizer(vocab, max_length=512))):
        bad = [j for j, t in enumerate(texts) if nat.encode(t) != py.encode(t)]
        assert not bad, [texts[j][:20] for j in bad[:3]]
    raw = [bytes(rng.integers(1, 256, int(rng.integers(0, 3000)), dtype=np.uint8)) for _ in range(40)]
    raw += [b"\x80\x80\x80", b"\xe4\xb8", b"\xc0\xaf", b"\xed\xa0\x80x", b"\xf4\x90\x80\x80", b"\xff" * 600]
    n_vocab = sum(1 for _ in open(vocab, encoding="utf-8"))
    for nat, vsize in ((NativeTokenizer.char(21128, max_length=512), 21128),
                       (NativeTokenizer.wordpiece(vocab, max_length=512), n_vocab)):
        cap = 512
        ids = np.zeros(len(raw) * cap, np.int32)
        mask = np.zeros(len(raw) * cap, np.int32)
        arr = (ctypes.c_char_p * len(raw))(*raw)
        L = ctypes.c_int()
        _lib.call("mq_tokenizer_encode_batch", nat._h, arr, len(raw), 0, _lib.ptr(ids), _lib.ptr(mask),
                  ctypes.byref(L))
        ids, mask = ids[:len(raw) * L.value].reshape(len(raw), -1), mask[:len(raw) * L.value].reshape(len(raw), -1)
        assert ((ids >= 0) & (ids < vsize)).all()
        n = mask.sum(1)
        assert (n >= 2).all()  # [CLS] ... [SEP] at least
        for j in range(len(raw)):
            assert mask[j, :n[j]].all() and not mask[j, n[j]:].any()
