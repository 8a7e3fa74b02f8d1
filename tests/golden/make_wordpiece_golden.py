"""Build tests/golden/wordpiece_golden.json + wordpiece_vocab.txt: token ids of the
published BERT WordPiece algorithm (transformers.BertTokenizer 5.15 = the `tokenizers`
crate's BertNormalizer + BertPreTokenizer + WordPiece model, run offline on a local vocab)
for the 154 corpus documents, the 32 config-1 queries and edge strings, uncased and cased.
The tokenisation step it pins is the one Ollama runs inside `OllamaEmbeddings` before the
BERT forward (reference src/medical_engine.py:43); dmeta's own vocab is absent offline, so
the vocab here is a deterministic test vocab made from the texts' characters plus
multi-character pieces that exercise greedy longest-match and "##" continuations.

Also recorded, for information: where transformers' pure-Python BertTokenizerLegacy (NFC
before splitting, lower-case before accent stripping) gives different ids.

Run from the repo root:  python tests/golden/make_wordpiece_golden.py
"""
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))

EDGE = [
    "", " ", "\t\n", "abc", "ABC Déjà vu ÆØÅ ß", "血糖,高!", "（括号）【标题】：问题？",
    "a​b­c", "emoji 😀 ok", "ＡＢＣ１２３", "x" * 700, "中" * 600,
    "Ωμέγα Привет Йод ёж", "ĀāĞğİıĲĳĸĹĺĿŀŁłŉŊŋŒœŦŧŸſ", "ÀÉÎÕÜÆÐØÞßàéîõüæðøþÿ×÷",
    # control / format / private-use / unassigned / separators
    "a\x0bb\x0cc\x1cd\x85e", "pq", "r͸s", "t u v", "w x　y",
    "zero‍width﻿join", "\x7f\x9fdel",
    # combining sequences, compatibility ideographs, Hangul, accents that NFD exposes
    "école", "Café NAÏVE", "豈更⾀0", "한국어 텍스트", "a`b",
    "ΟΔΟΣ ΣΟΦΙΑ", "İstanbul ǅemal ǈ", "⮋8⮂0⮁f", "\U0002B820\U0002B8FFx\U0002B920y\U0002A700z",
    # punctuation outside ASCII, symbols that are not punctuation, digits and mixed text
    "«quote» ¿qué? ¡sí! — dash … ellipsis", "1+1=2 < 3 > 0 | ~ ^ $ € ¥ © ®", "血压140/90mmHg，BMI=24.5",
    "维生素D3和Omega-3", "WHO建议每天30分钟运动", "“引号”‘单引号’《书名》〈括号〉",
]


def texts():
    docs = json.load(open(os.path.join(HERE, "corpus_docs.json"), encoding="utf-8"))["docs"]
    qs = json.load(open(os.path.join(HERE, "config1_queries.json"), encoding="utf-8"))["queries"]
    return [d["page_content"] for d in docs] + qs + EDGE


def build_vocab(ts):
    from tokenizers import normalizers, pre_tokenizers
    words = set()
    for lower in (True, False):
        nrm = normalizers.BertNormalizer(clean_text=True, handle_chinese_chars=True, lowercase=lower)
        pre = pre_tokenizers.BertPreTokenizer()
        for t in ts:
            words.update(w for w, _ in pre.pre_tokenize_str(nrm.normalize_str(t)))
    chars = sorted({c for w in words for c in w})
    pieces = set()
    for w in sorted(words):
        if len(w) >= 3 and re.fullmatch(r"[A-Za-z0-9]+", w) and len(w) <= 12:
            pieces.add(w[: (len(w) + 1) // 2])        # greedy prefix ...
            pieces.add("##" + w[(len(w) + 1) // 2:])  # ... and its continuation
    pieces.update(["high", "##er", "##s", "abc", "##c", "vu", "dej", "##a", "ok", "emoji", "x", "##x",
                   "omega", "##-", "mm", "##hg", "cafe", "ecole", "##ole"])
    vocab = ["[PAD]"] + ["[unused%d]" % i for i in range(1, 100)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    seen = set(vocab)
    # every character except a few held out (-> [UNK] words) and every 7th one only as a
    # continuation piece (-> multi-piece / unmatched paths)
    held_out = set("ŋ€ǅ")
    for i, c in enumerate(chars):
        if c in held_out:
            continue
        if i % 7 != 3 and c not in seen:
            vocab.append(c)
            seen.add(c)
    for p in sorted(pieces) + ["##" + c for c in chars[:300]]:
        if p not in seen:
            vocab.append(p)
            seen.add(p)
    return vocab


def main():
    from transformers import BertTokenizer
    from transformers.models.bert.tokenization_bert_legacy import BertTokenizerLegacy
    ts = texts()
    vocab = build_vocab(ts)
    vpath = os.path.join(HERE, "wordpiece_vocab.txt")
    with open(vpath, "w", encoding="utf-8") as f:
        f.write("\n".join(vocab) + "\n")
    out = {"tokenizer": "transformers.BertTokenizer %s (tokenizers BertNormalizer + BertPreTokenizer + WordPiece)"
           % __import__("transformers").__version__, "vocab": "wordpiece_vocab.txt", "max_length": 512,
           "texts": ts, "cases": {}}
    for lower in (True, False):
        tok = BertTokenizer(vpath, do_lower_case=lower)
        leg = BertTokenizerLegacy(vpath, do_lower_case=lower)
        ids, diff = [], []
        for j, t in enumerate(ts):
            a = tok(t, truncation=True, max_length=512)["input_ids"]
            full = tok._tokenizer.encode(t).ids  # the backend alone, untruncated
            assert a == (full if len(full) <= 512 else full[:511] + [full[-1]]), j
            ids.append(a)
            if leg(t, truncation=True, max_length=512)["input_ids"] != a:
                diff.append(j)
        out["cases"]["lower" if lower else "cased"] = {"do_lower_case": lower, "ids": ids,
                                                        "legacy_python_differs_at": diff}
        print("lower=%s: %d texts, %d tokens, legacy differs at %s" % (lower, len(ts), sum(map(len, ids)), diff))
    with open(os.path.join(HERE, "wordpiece_golden.json"), "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False)


if __name__ == "__main__":
    main()
