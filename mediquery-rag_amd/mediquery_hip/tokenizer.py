"""Host tokenisers feeding the encoder's int32 id/mask buffers.

In the reference, WordPiece tokenisation happens inside the Ollama server before the
BERT forward (reference src/medical_engine.py:43).  The dmeta vocab is
not available offline, so two tokenisers are provided:

* `CharTokenizer` - the deterministic stand-in used for parity and benchmarks: one token
  per non-space character (Chinese BERT tokenises CJK text one character per token),
  id = 106 + crc32(char) mod (vocab - 106), framed by [CLS]=101 / [SEP]=102, [PAD]=0.
* `WordPieceTokenizer` - BERT basic + greedy longest-match WordPiece over a LOCAL
  vocab.txt, for use with real weights.
`NativeTokenizer` runs either scheme in C++ inside libmqhip.so (mq_tokenizer_*); the two
Python classes above are its parity twins (tests/test_tokenizer_native.py).
"""
import unicodedata
import zlib

import numpy as np

PAD, UNK, CLS, SEP = 0, 100, 101, 102
FIRST_FREE_ID = 106


def _pack(seqs, max_length, pad_to=None):
    """List of id lists -> (ids[B, L] int32, mask[B, L] int32), right padded."""
    L = min(max((len(s) for s in seqs), default=0), max_length)
    if pad_to is not None:
        L = max(L, pad_to)
    ids = np.zeros((len(seqs), L), dtype=np.int32)
    mask = np.zeros((len(seqs), L), dtype=np.int32)
    for i, s in enumerate(seqs):
        s = s[:L]
        ids[i, :len(s)] = s
        mask[i, :len(s)] = 1
    return ids, mask


class CharTokenizer:
    def __init__(self, vocab_size=21128, max_length=512):
        self.vocab_size = vocab_size
        self.max_length = max_length

    def token_id(self, ch):
        return FIRST_FREE_ID + zlib.crc32(ch.encode("utf-8")) % (self.vocab_size - FIRST_FREE_ID)

    def encode(self, text):
        body = [self.token_id(c) for c in text if not c.isspace()]
        body = body[: self.max_length - 2]
        return [CLS] + body + [SEP]

    def __call__(self, texts, pad_to=None):
        return _pack([self.encode(t) for t in texts], self.max_length, pad_to)


class WordPieceTokenizer:
    """BERT WordPiece over a local vocab file, as the published tokenizer computes it
    (`tokenizers` BertNormalizer + BertPreTokenizer + WordPiece, i.e.
    transformers.BertTokenizer; pinned by tests/golden/wordpiece_golden.json):
      1. clean: drop NUL, U+FFFD and category Cc/Cf/Co/Cs except \\t \\n \\r (unassigned
         code points are kept); whitespace -> word break;
      2. CJK ideographs (the crate's ranges) become words of their own;
      3. lower_case: NFD, drop Mn, then each character's full lower-case mapping
         (per character: no final-sigma context);
      4. split on whitespace and isolate punctuation (ASCII symbols or category P*), on the
         normalised characters;
      5. greedy longest-match-first WordPiece ("##" continuations; [UNK] for a word with
         no match or over 100 code points); [CLS] body [SEP], truncated to max_length."""

    def __init__(self, vocab_file, max_length=512, lower_case=True, max_chars_per_word=100):
        with open(vocab_file, "r", encoding="utf-8") as f:
            self.vocab = {line.rstrip("\n"): i for i, line in enumerate(f)}
        self.max_length = max_length
        self.lower_case = lower_case
        self.max_chars = max_chars_per_word
        self.unk = self.vocab.get("[UNK]", UNK)
        self.cls = self.vocab.get("[CLS]", CLS)
        self.sep = self.vocab.get("[SEP]", SEP)

    @staticmethod
    def _is_cjk(cp):
        # the tokenizers crate's table (its fourth extension range starts at 0x2B920)
        return (0x4E00 <= cp <= 0x9FFF or 0x3400 <= cp <= 0x4DBF or 0x20000 <= cp <= 0x2A6DF
                or 0x2A700 <= cp <= 0x2B73F or 0x2B740 <= cp <= 0x2B81F or 0x2B920 <= cp <= 0x2CEAF
                or 0xF900 <= cp <= 0xFAFF or 0x2F800 <= cp <= 0x2FA1F)

    @staticmethod
    def _is_punct(ch):
        cp = ord(ch)
        if 33 <= cp <= 47 or 58 <= cp <= 64 or 91 <= cp <= 96 or 123 <= cp <= 126:
            return True
        return unicodedata.category(ch).startswith("P")

    @staticmethod
    def _is_control(ch):
        return ch not in "\t\n\r" and unicodedata.category(ch) in ("Cc", "Cf", "Co", "Cs")

    def _normalise(self, ch):
        if not self.lower_case:
            return ch
        d = unicodedata.normalize("NFD", ch)
        return "".join(c.lower() for c in d if unicodedata.category(c) != "Mn")

    def _basic(self, text):
        words, cur = [], []

        def flush():
            if cur:
                words.append("".join(cur))
                cur.clear()
        for ch in text:
            cp = ord(ch)
            if cp == 0 or cp == 0xFFFD or self._is_control(ch):
                continue
            if ch.isspace():
                flush()
            elif self._is_cjk(cp):
                flush()
                words.append(self._normalise(ch))
            else:
                for c in self._normalise(ch):
                    if self._is_punct(c):
                        flush()
                        words.append(c)
                    else:
                        cur.append(c)
        flush()
        return [w for w in words if w]

    def _wordpiece(self, word):
        if len(word) > self.max_chars:
            return [self.unk]
        out, start = [], 0
        while start < len(word):
            end, hit = len(word), None
            while start < end:
                piece = word[start:end] if start == 0 else "##" + word[start:end]
                if piece in self.vocab:
                    hit = self.vocab[piece]
                    break
                end -= 1
            if hit is None:
                return [self.unk]
            out.append(hit)
            start = end
        return out

    def encode(self, text):
        body = []
        for w in self._basic(text):
            body.extend(self._wordpiece(w))
        return [self.cls] + body[: self.max_length - 2] + [self.sep]

    def __call__(self, texts, pad_to=None):
        return _pack([self.encode(t) for t in texts], self.max_length, pad_to)


class NativeTokenizer:
    """C++ tokenizer of libmqhip.so: `NativeTokenizer.char(vocab, max_length)` or
    `NativeTokenizer.wordpiece(vocab_file, max_length, lower_case)`; call like the Python
    tokenizers: tok(texts, pad_to=None) -> (ids, mask) int32 [n, L]."""

    def __init__(self, handle, max_length):
        self._h = handle
        self.max_length = max_length

    @classmethod
    def char(cls, vocab_size=21128, max_length=512):
        import ctypes
        from . import _lib
        h = ctypes.c_void_p()
        _lib.call("mq_tokenizer_create_char", vocab_size, max_length, ctypes.byref(h))
        return cls(h, max_length)

    @classmethod
    def wordpiece(cls, vocab_file, max_length=512, lower_case=True):
        import ctypes
        from . import _lib
        h = ctypes.c_void_p()
        _lib.call("mq_tokenizer_create_wordpiece", str(vocab_file).encode(), int(lower_case),
                  max_length, ctypes.byref(h))
        return cls(h, max_length)

    @classmethod
    def wordpiece_tokens(cls, tokens, max_length=512, lower_case=True):
        """WordPiece over an in-memory vocabulary (token of id i = tokens[i]), e.g. the
        vocab a GGUF model file embeds (gguf.read_gguf)."""
        import ctypes
        from . import _lib
        tokens = list(tokens)
        arr = (ctypes.c_char_p * len(tokens))(*[t.encode("utf-8") for t in tokens])
        h = ctypes.c_void_p()
        _lib.call("mq_tokenizer_create_wordpiece_tokens", arr, len(tokens), int(lower_case), max_length,
                  ctypes.byref(h))
        return cls(h, max_length)

    def close(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            try:
                from . import _lib
                _lib.lib().mq_tokenizer_destroy(h)
            except Exception:
                pass

    __del__ = close

    def __call__(self, texts, pad_to=None):
        import ctypes
        from . import _lib
        texts = list(texts)
        n = len(texts)
        cap = max(self.max_length, pad_to or 0)
        ids = np.zeros(max(1, n * cap), dtype=np.int32)
        mask = np.zeros(max(1, n * cap), dtype=np.int32)
        arr = (ctypes.c_char_p * max(1, n))(*[t.encode("utf-8") for t in texts])
        L = ctypes.c_int()
        _lib.call("mq_tokenizer_encode_batch", self._h, arr, n, int(pad_to or 0), _lib.ptr(ids),
                  _lib.ptr(mask), ctypes.byref(L))
        return ids[:n * L.value].reshape(n, L.value).copy(), mask[:n * L.value].reshape(n, L.value).copy()

    def encode(self, text):
        ids, mask = self([text])
        return ids[0, :int(mask[0].sum())].tolist()
