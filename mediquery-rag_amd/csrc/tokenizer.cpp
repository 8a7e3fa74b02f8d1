// tokenizer.cpp - host-side BERT tokenisation for the encoder's int32 id/mask buffers.
//
// In the reference the WordPiece step runs inside the Ollama server ahead of the BERT
// forward (reference src/medical_engine.py:43).  This is the
// native restatement of mediquery_hip/tokenizer.py (the Python twin is the parity
// oracle for it):
//   * WordPiece as the published BERT tokenizer computes it (the `tokenizers` crate's
//     BertNormalizer + BertPreTokenizer + WordPiece = transformers.BertTokenizer; pinned
//     by tests/golden/wordpiece_golden.json): drop NUL / U+FFFD / Cc Cf Co Cs except
//     \t \n \r, isolate CJK ideographs, uncased: NFD + drop Mn + per-character lower-case
//     mapping, then split on whitespace and isolate punctuation (ASCII symbols or P*), and
//     greedy longest-match-first WordPiece over the vocab ("##" continuations, [UNK] for
//     unmatched words and words over 100 code points).
//   * Char: one id per non-space code point, 106 + crc32(utf-8 bytes) % (vocab - 106).
// Both frame sequences as [CLS] ... [SEP], truncate to max_length and right-pad with 0.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "mq.h"

namespace mq {
void set_error(const char* fmt, ...);
void clear_error();
}  // namespace mq

namespace {

constexpr int kPad = 0, kUnk = 100, kCls = 101, kSep = 102, kFirstFree = 106;

// --------------------------------------------------------------- UTF-8 -------
std::vector<uint32_t> decode_utf8(const char* s) {
  std::vector<uint32_t> out;
  const unsigned char* p = reinterpret_cast<const unsigned char*>(s);
  while (*p) {
    uint32_t c = *p;
    int extra = 0;
    if (c < 0x80) {
      extra = 0;
    } else if ((c >> 5) == 0x6) {
      c &= 0x1F;
      extra = 1;
    } else if ((c >> 4) == 0xE) {
      c &= 0x0F;
      extra = 2;
    } else if ((c >> 3) == 0x1E) {
      c &= 0x07;
      extra = 3;
    } else {  // stray continuation byte: U+FFFD
      out.push_back(0xFFFD);
      ++p;
      continue;
    }
    ++p;
    bool ok = true;
    for (int i = 0; i < extra; ++i) {
      if ((*p >> 6) != 0x2) {
        ok = false;
        break;
      }
      c = (c << 6) | (*p & 0x3F);
      ++p;
    }
    out.push_back(ok ? c : 0xFFFD);
  }
  return out;
}

void encode_utf8(uint32_t c, std::string& out) {
  if (c < 0x80) {
    out += static_cast<char>(c);
  } else if (c < 0x800) {
    out += static_cast<char>(0xC0 | (c >> 6));
    out += static_cast<char>(0x80 | (c & 0x3F));
  } else if (c < 0x10000) {
    out += static_cast<char>(0xE0 | (c >> 12));
    out += static_cast<char>(0x80 | ((c >> 6) & 0x3F));
    out += static_cast<char>(0x80 | (c & 0x3F));
  } else {
    out += static_cast<char>(0xF0 | (c >> 18));
    out += static_cast<char>(0x80 | ((c >> 12) & 0x3F));
    out += static_cast<char>(0x80 | ((c >> 6) & 0x3F));
    out += static_cast<char>(0x80 | (c & 0x3F));
  }
}

// ----------------------------------------------------- character classes -----
// Unicode data generated from Python's unicodedata by tools/gen_unicode_tables.py.
struct CpRange {
  uint32_t lo, hi;
};
struct CpMap4 {
  uint32_t cp, to[4];
};
struct CpMap3 {
  uint32_t cp, to[3];
};
#include "unicode_tables.inc"

template <size_t N>
bool in_ranges(const CpRange (&t)[N], uint32_t c) {
  size_t lo = 0, hi = N;
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (t[mid].hi < c)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < N && t[lo].lo <= c;
}

template <class M, size_t N>
const M* find_map(const M (&t)[N], uint32_t c) {
  size_t lo = 0, hi = N;
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (t[mid].cp < c)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < N && t[lo].cp == c ? &t[lo] : nullptr;
}

// White_Space (Python str.isspace() adds U+001C..U+001F, which are controls and dropped
// before this test is reached).
bool is_space(uint32_t c) {
  return c == ' ' || (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x1F) || c == 0x85 ||
         c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 ||
         c == 0x202F || c == 0x205F || c == 0x3000;
}

// The tokenizers crate's CJK table (its fourth extension range starts at 0x2B920).
bool is_cjk(uint32_t c) {
  return (c >= 0x4E00 && c <= 0x9FFF) || (c >= 0x3400 && c <= 0x4DBF) ||
         (c >= 0x20000 && c <= 0x2A6DF) || (c >= 0x2A700 && c <= 0x2B73F) ||
         (c >= 0x2B740 && c <= 0x2B81F) || (c >= 0x2B920 && c <= 0x2CEAF) ||
         (c >= 0xF900 && c <= 0xFAFF) || (c >= 0x2F800 && c <= 0x2FA1F);
}

// BERT's punctuation test: ASCII symbol ranges, or general category P*.
bool is_punct(uint32_t c) {
  if ((c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126))
    return true;
  return in_ranges(kPunct, c);
}

// Dropped by the clean-up: categories Cc / Cf / Co / Cs except \t \n \r.
bool is_control(uint32_t c) {
  if (c == '\t' || c == '\n' || c == '\r') return false;
  return in_ranges(kOther, c);
}

// Uncased normalisation of one code point: NFD (Hangul syllables algorithmically), drop
// category Mn, then each remaining character's full lower-case mapping.
void lower_strip(uint32_t c, std::vector<uint32_t>& out) {
  uint32_t d[4] = {c, 0, 0, 0};
  int nd = 1;
  if (c >= 0xAC00 && c <= 0xD7A3) {  // Hangul syllable -> L V (T) jamo
    const uint32_t s = c - 0xAC00;
    d[0] = 0x1100 + s / 588;
    d[1] = 0x1161 + (s % 588) / 28;
    nd = 2;
    if (s % 28) d[nd++] = 0x11A7 + s % 28;
  } else if (const CpMap4* m = find_map(kNfd, c)) {
    nd = 0;
    for (int i = 0; i < 4 && m->to[i]; ++i) d[nd++] = m->to[i];
  }
  for (int i = 0; i < nd; ++i) {
    if (in_ranges(kMn, d[i])) continue;
    if (const CpMap3* l = find_map(kLower, d[i])) {
      for (int j = 0; j < 3 && l->to[j]; ++j) out.push_back(l->to[j]);
    } else {
      out.push_back(d[i]);
    }
  }
}

uint32_t crc32_bytes(const std::string& s) {
  uint32_t crc = 0xFFFFFFFFu;
  for (unsigned char ch : s) {
    crc ^= ch;
    for (int k = 0; k < 8; ++k) crc = (crc >> 1) ^ (0xEDB88320u & (0u - (crc & 1u)));
  }
  return ~crc;
}

}  // namespace

struct mq_tokenizer {
  bool wordpiece = false;
  bool lower = true;
  int max_length = 512;
  int vocab_size = 21128;
  int unk = kUnk, cls = kCls, sep = kSep;
  std::unordered_map<std::string, int> vocab;

  void char_ids(const std::vector<uint32_t>& cps, std::vector<int>& body) const {
    std::string u;
    for (uint32_t c : cps) {
      if (is_space(c)) continue;
      u.clear();
      encode_utf8(c, u);
      body.push_back(kFirstFree + static_cast<int>(crc32_bytes(u) % (uint32_t)(vocab_size - kFirstFree)));
    }
  }

  void wordpiece_ids(const std::vector<uint32_t>& cps, std::vector<int>& body) const {
    // basic tokenisation into words (vectors of normalised code points): clean-up, CJK
    // isolation, per-character normalisation, then whitespace / punctuation splits on the
    // normalised characters (the BertNormalizer -> BertPreTokenizer order)
    std::vector<std::vector<uint32_t>> words;
    std::vector<uint32_t> cur, norm;
    auto flush = [&]() {
      if (!cur.empty()) words.push_back(cur);
      cur.clear();
    };
    for (uint32_t c : cps) {
      if (c == 0 || c == 0xFFFD || is_control(c)) continue;
      if (is_space(c)) {
        flush();
        continue;
      }
      norm.clear();
      if (lower)
        lower_strip(c, norm);
      else
        norm.push_back(c);
      if (is_cjk(c)) {
        flush();
        words.push_back(norm);
        continue;
      }
      for (uint32_t n : norm) {
        if (is_punct(n)) {
          flush();
          words.push_back({n});
        } else {
          cur.push_back(n);
        }
      }
    }
    flush();
    std::string piece;
    for (auto& lw : words) {
      if (lw.empty()) continue;
      if (lw.size() > 100) {
        body.push_back(unk);
        continue;
      }
      std::vector<int> sub;
      size_t start = 0;
      bool bad = false;
      while (start < lw.size()) {
        size_t end = lw.size();
        int hit = -1;
        while (start < end) {
          piece.clear();
          if (start > 0) piece = "##";
          for (size_t i = start; i < end; ++i) encode_utf8(lw[i], piece);
          auto it = vocab.find(piece);
          if (it != vocab.end()) {
            hit = it->second;
            break;
          }
          --end;
        }
        if (hit < 0) {
          bad = true;
          break;
        }
        sub.push_back(hit);
        start = end;
      }
      if (bad)
        body.push_back(unk);
      else
        body.insert(body.end(), sub.begin(), sub.end());
    }
  }

  std::vector<int> encode(const char* text) const {
    const std::vector<uint32_t> cps = decode_utf8(text ? text : "");
    std::vector<int> body;
    if (wordpiece)
      wordpiece_ids(cps, body);
    else
      char_ids(cps, body);
    const size_t keep = std::min<size_t>(body.size(), (size_t)std::max(0, max_length - 2));
    std::vector<int> seq;
    seq.reserve(keep + 2);
    seq.push_back(cls);
    seq.insert(seq.end(), body.begin(), body.begin() + keep);
    seq.push_back(sep);
    return seq;
  }
};

extern "C" {

int mq_tokenizer_create_char(int vocab_size, int max_length, mq_tokenizer** out) {
  mq::clear_error();
  if (!out || vocab_size <= kFirstFree || max_length < 2) {
    mq::set_error("bad char tokenizer arguments");
    return MQ_EINVAL;
  }
  auto t = std::make_unique<mq_tokenizer>();
  t->vocab_size = vocab_size;
  t->max_length = max_length;
  *out = t.release();
  return MQ_OK;
}

}  // extern "C"

namespace {

// WordPiece tokenizer over `tokens` in id order (a repeated token keeps its last index,
// as HF load_vocab does).
std::unique_ptr<mq_tokenizer> make_wordpiece(std::vector<std::string>& tokens, int lower_case,
                                             int max_length) {
  auto t = std::make_unique<mq_tokenizer>();
  t->wordpiece = true;
  t->lower = lower_case != 0;
  t->max_length = max_length;
  int idx = 0;
  for (std::string& tok : tokens) t->vocab[std::move(tok)] = idx++;
  t->vocab_size = idx;
  auto get = [&](const char* k, int dflt) {
    auto it = t->vocab.find(k);
    return it == t->vocab.end() ? dflt : it->second;
  };
  t->unk = get("[UNK]", kUnk);
  t->cls = get("[CLS]", kCls);
  t->sep = get("[SEP]", kSep);
  return t;
}

}  // namespace

extern "C" {

int mq_tokenizer_create_wordpiece(const char* vocab_path, int lower_case, int max_length,
                                  mq_tokenizer** out) {
  mq::clear_error();
  if (!out || !vocab_path || max_length < 2) {
    mq::set_error("bad wordpiece tokenizer arguments");
    return MQ_EINVAL;
  }
  std::ifstream f(vocab_path);
  if (!f) {
    mq::set_error("cannot open vocab file %s", vocab_path);
    return MQ_EIO;
  }
  std::vector<std::string> tokens;
  std::string line;
  while (std::getline(f, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    tokens.push_back(line);
  }
  *out = make_wordpiece(tokens, lower_case, max_length).release();
  return MQ_OK;
}

int mq_tokenizer_create_wordpiece_tokens(const char* const* tokens, int n_tokens, int lower_case,
                                         int max_length, mq_tokenizer** out) {
  mq::clear_error();
  if (!out || !tokens || n_tokens <= 0 || max_length < 2) {
    mq::set_error("bad wordpiece tokenizer arguments");
    return MQ_EINVAL;
  }
  std::vector<std::string> v;
  v.reserve((size_t)n_tokens);
  for (int i = 0; i < n_tokens; ++i) {
    if (!tokens[i]) {
      mq::set_error("token %d is NULL", i);
      return MQ_EINVAL;
    }
    v.emplace_back(tokens[i]);
  }
  *out = make_wordpiece(v, lower_case, max_length).release();
  return MQ_OK;
}

int mq_tokenizer_destroy(mq_tokenizer* t) {
  delete t;
  return MQ_OK;
}

int mq_tokenizer_encode_batch(mq_tokenizer* t, const char* const* texts, int n, int pad_to,
                              int32_t* ids, int32_t* mask, int* out_len) {
  mq::clear_error();
  if (!t || n < 0 || !out_len || (n > 0 && (!texts || !ids || !mask))) {
    mq::set_error("bad encode_batch arguments");
    return MQ_EINVAL;
  }
  std::vector<std::vector<int>> seqs((size_t)n);
  int L = 0;
  for (int i = 0; i < n; ++i) {
    seqs[i] = t->encode(texts[i]);
    L = std::max<int>(L, (int)seqs[i].size());
  }
  L = std::max(L, std::min(pad_to, t->max_length));
  if (pad_to > t->max_length) L = std::max(L, pad_to);
  for (int i = 0; i < n; ++i) {
    int32_t* row = ids + (size_t)i * L;
    int32_t* mrow = mask + (size_t)i * L;
    const int len = (int)seqs[i].size();
    for (int j = 0; j < L; ++j) {
      row[j] = j < len ? seqs[i][j] : kPad;
      mrow[j] = j < len ? 1 : 0;
    }
  }
  *out_len = L;
  return MQ_OK;
}

}  // extern "C"
