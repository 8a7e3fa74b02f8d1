// tokenizer.cpp - host-side BERT tokenisation for the encoder's int32 id/mask buffers.
//
// In the reference the WordPiece step runs inside the Ollama server ahead of the BERT
// forward (reference src/medical_engine.py:43).  This is the
// native restatement of mediquery_hip/tokenizer.py (the Python twin is the parity
// oracle for it):
//   * WordPiece: BERT basic tokenisation (drop control chars, split on whitespace,
//     isolate CJK ideographs and punctuation, lower-case + strip combining marks) and
//     greedy longest-match-first WordPiece over a local vocab.txt ("##" continuations,
//     [UNK] for unmatched words and words over 100 code points).
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
// Python str.isspace(): Unicode White_Space plus the ASCII separators.
bool is_space(uint32_t c) {
  return c == ' ' || (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x1F) || c == 0x85 ||
         c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 ||
         c == 0x202F || c == 0x205F || c == 0x3000;
}

bool is_cjk(uint32_t c) {
  return (c >= 0x4E00 && c <= 0x9FFF) || (c >= 0x3400 && c <= 0x4DBF) ||
         (c >= 0x20000 && c <= 0x2A6DF) || (c >= 0x2A700 && c <= 0x2CEAF) ||
         (c >= 0xF900 && c <= 0xFAFF) || (c >= 0x2F800 && c <= 0x2FA1F);
}

// BERT's punctuation test: ASCII symbol ranges, or Unicode category P* (the ranges
// below cover the P* code points of the BMP blocks the corpus uses: Latin-1, General
// Punctuation, CJK Symbols, Fullwidth/Halfwidth Forms, CJK Compatibility Forms).
bool is_punct(uint32_t c) {
  if ((c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126))
    return true;
  if (c == 0xA1 || c == 0xA7 || c == 0xAB || c == 0xB6 || c == 0xB7 || c == 0xBB || c == 0xBF ||
      c == 0x37E || c == 0x387)
    return true;
  if (c >= 0x2010 && c <= 0x2027) return true;
  if (c >= 0x2030 && c <= 0x2043) return true;
  if (c >= 0x2045 && c <= 0x2051) return true;
  if (c >= 0x2053 && c <= 0x205E) return true;
  if (c == 0x207D || c == 0x207E || c == 0x208D || c == 0x208E) return true;
  if (c >= 0x2308 && c <= 0x230B) return true;
  if (c == 0x2329 || c == 0x232A) return true;
  if (c >= 0x2768 && c <= 0x2775) return true;
  if (c >= 0x27C5 && c <= 0x27C6) return true;
  if (c >= 0x27E6 && c <= 0x27EF) return true;
  if (c >= 0x2E00 && c <= 0x2E4F) return true;
  if (c >= 0x3001 && c <= 0x3003) return true;
  if (c >= 0x3008 && c <= 0x3011) return true;
  if (c >= 0x3014 && c <= 0x301F) return true;
  if (c == 0x3030 || c == 0x303D || c == 0x30A0 || c == 0x30FB) return true;
  if (c >= 0xFE10 && c <= 0xFE19) return true;
  if (c >= 0xFE30 && c <= 0xFE52) return true;
  if (c >= 0xFE54 && c <= 0xFE61) return true;
  if (c == 0xFE63 || c == 0xFE68 || c == 0xFE6A || c == 0xFE6B) return true;
  if ((c >= 0xFF01 && c <= 0xFF03) || (c >= 0xFF05 && c <= 0xFF0A) || (c >= 0xFF0C && c <= 0xFF0F))
    return true;
  if (c == 0xFF1A || c == 0xFF1B || c == 0xFF1F || c == 0xFF20) return true;
  if ((c >= 0xFF3B && c <= 0xFF3D) || c == 0xFF3F || c == 0xFF5B || c == 0xFF5D) return true;
  if (c >= 0xFF5F && c <= 0xFF65) return true;
  return false;
}

// category Cc / Cf (dropped by the basic tokeniser unless \t \n \r)
bool is_control(uint32_t c) {
  if (c == '\t' || c == '\n' || c == '\r') return false;
  if (c < 0x20 || (c >= 0x7F && c <= 0x9F)) return true;
  return c == 0xAD || (c >= 0x600 && c <= 0x605) || c == 0x61C || c == 0x6DD || c == 0x70F ||
         c == 0x180E || (c >= 0x200B && c <= 0x200F) || (c >= 0x202A && c <= 0x202E) ||
         (c >= 0x2060 && c <= 0x2064) || (c >= 0x2066 && c <= 0x206F) || c == 0xFEFF ||
         (c >= 0xFFF9 && c <= 0xFFFB);
}

bool is_combining_mark(uint32_t c) {  // category Mn in the ranges lower-casing can produce
  return (c >= 0x300 && c <= 0x36F) || (c >= 0x1AB0 && c <= 0x1AFF) ||
         (c >= 0x1DC0 && c <= 0x1DFF) || (c >= 0x20D0 && c <= 0x20FF) || (c >= 0xFE20 && c <= 0xFE2F);
}

// lower-case + NFD accent strip (Python: NFD(lower(c)) minus category Mn) for ASCII,
// Latin-1, Greek / Cyrillic capitals and fullwidth Latin; other code points unchanged.
void lower_strip(uint32_t c, std::vector<uint32_t>& out) {
  if (c >= 'A' && c <= 'Z') {
    out.push_back(c + 32);
    return;
  }
  if (c >= 0xC0 && c <= 0xFF) {
    // base letter of each Latin-1 letter after NFD; '.' = keep the (lower-cased) char
    static const char kBase[65] =
        "aaaaaa.ceeeeiiii.nooooo..uuuuy.."   // C0..DF
        "aaaaaa.ceeeeiiii.nooooo..uuuuy.y";  // E0..FF
    const char b = kBase[c - 0xC0];
    if (b != '.') {
      out.push_back((uint32_t)b);
    } else if (c == 0xD7 || c == 0xF7 || c == 0xDF) {
      out.push_back(c);  // × ÷ ß
    } else {
      out.push_back(c <= 0xDE ? c + 32 : c);  // Æ Ð Ø Þ -> æ ð ø þ
    }
    return;
  }
  if (c >= 0x100 && c <= 0x17F) {  // Latin Extended-A
    static const char kBaseA[129] =
        "aaaaaaccccccccdd"   // 100-10F
        "..eeeeeeeeeegggg"   // 110-11F
        "gggghh..iiiiiiii"   // 120-12F
        "!...jjkk.llllll."   // 130-13F
        "...nnnnnn...oooo"   // 140-14F
        "oo..rrrrrrssssss"   // 150-15F
        "sstttt..uuuuuuuu"   // 160-16F
        "uuuuwwyyyzzzzzz.";  // 170-17F
    const char b = kBaseA[c - 0x100];
    if (b == '!') {
      out.push_back('i');  // İ -> i + U+0307 -> i
    } else if (b != '.') {
      out.push_back((uint32_t)b);
    } else if (c == 0x138 || c == 0x149 || c == 0x17F) {
      out.push_back(c);  // ĸ ŉ ſ
    } else if (c >= 0x139 && c <= 0x148) {
      out.push_back((c & 1) ? c + 1 : c);  // odd capitals in this stretch
    } else {
      out.push_back((c & 1) ? c : c + 1);
    }
    return;
  }
  switch (c) {  // Greek with tonos / dialytika -> base letter
    case 0x386: case 0x3AC: out.push_back(0x3B1); return;
    case 0x388: case 0x3AD: out.push_back(0x3B5); return;
    case 0x389: case 0x3AE: out.push_back(0x3B7); return;
    case 0x38A: case 0x3AF: case 0x390: case 0x3AA: case 0x3CA: out.push_back(0x3B9); return;
    case 0x38C: case 0x3CC: out.push_back(0x3BF); return;
    case 0x38E: case 0x3CD: case 0x3B0: case 0x3AB: case 0x3CB: out.push_back(0x3C5); return;
    case 0x38F: case 0x3CE: out.push_back(0x3C9); return;
    // Cyrillic letters with a combining mark in NFD -> base letter
    case 0x400: case 0x401: case 0x450: case 0x451: out.push_back(0x435); return;
    case 0x403: case 0x453: out.push_back(0x433); return;
    case 0x407: case 0x457: out.push_back(0x456); return;
    case 0x40C: case 0x45C: out.push_back(0x43A); return;
    case 0x40D: case 0x45D: case 0x419: case 0x439: out.push_back(0x438); return;
    case 0x40E: case 0x45E: out.push_back(0x443); return;
    default: break;
  }
  if (c >= 0x400 && c <= 0x40F) {  // remaining Cyrillic capitals of the 0x450 row
    out.push_back(c + 80);
    return;
  }
  if ((c >= 0x391 && c <= 0x3A9 && c != 0x3A2) || (c >= 0x410 && c <= 0x42F) ||
      (c >= 0xFF21 && c <= 0xFF3A)) {
    out.push_back(c + 32);  // Greek / Cyrillic / fullwidth capitals
    return;
  }
  out.push_back(c);
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
    // basic tokenisation into words (vectors of code points)
    std::vector<std::vector<uint32_t>> words;
    std::vector<uint32_t> cur;
    auto flush = [&]() {
      if (!cur.empty()) words.push_back(cur);
      cur.clear();
    };
    for (uint32_t c : cps) {
      if (c == 0 || c == 0xFFFD || is_control(c)) continue;
      if (is_space(c)) {
        flush();
      } else if (is_cjk(c) || is_punct(c)) {
        flush();
        words.push_back({c});
      } else {
        cur.push_back(c);
      }
    }
    flush();
    std::string piece;
    for (auto& w : words) {
      std::vector<uint32_t> lw;
      if (lower) {
        for (uint32_t c : w) lower_strip(c, lw);
        std::vector<uint32_t> kept;
        for (uint32_t c : lw)
          if (!is_combining_mark(c)) kept.push_back(c);
        lw.swap(kept);
      } else {
        lw = w;
      }
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
