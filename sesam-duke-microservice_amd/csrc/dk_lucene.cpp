// dk_lucene.cpp — the text analysis of the Lucene-compatible candidate source (DK_CAND_LUCENE):
// what IncrementalLuceneDatabase feeds its StandardAnalyzer at index time (:505-575, values
// as stored) and at query time (parseTokens :295-321 over escapeLucene :329-342).  Host C++.
//
// [Lucene 4.x, recalled -- PARITY UNPINNED: Lucene is absent from /root/reference]
// StandardAnalyzer = StandardTokenizer (Unicode UAX#29 word boundaries, rules WB4-WB13b,
// restated for code units U+0000-U+00FF; anything above is declined with DK_E_UNSUPPORTED so
// that batch's pipeline stays on Lucene) -> LowerCaseFilter -> StopFilter(English stop
// words).  Tokens keep the segment text (apostrophes, dots, underscores, soft hyphens);
// segments without a letter or digit are not tokens; tokens over 255 units are skipped.
// oracle/lucene_ref.py restates the same rules in Python (the CPU test compares both).
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "dukehip.h"

extern "C" int dk_fail_ingest(int code, const char* msg);  // dk_api.cpp: sets dk_last_error

namespace dk {

namespace {

enum WB : uint8_t { OTHER, ALETTER, NUMERIC, MIDLETTER, MIDNUMLET, MIDNUM, EXTENDNUMLET, FORMAT, NL };

inline WB wb_class(uint32_t c) {
  if (c == 0x0A || c == 0x0B || c == 0x0C || c == 0x0D || c == 0x85) return NL;
  if (c >= 0x30 && c <= 0x39) return NUMERIC;
  if ((c >= 0x41 && c <= 0x5A) || (c >= 0x61 && c <= 0x7A) || c == 0xAA || c == 0xB5 || c == 0xBA ||
      (c >= 0xC0 && c <= 0xD6) || (c >= 0xD8 && c <= 0xF6) || (c >= 0xF8 && c <= 0xFF))
    return ALETTER;
  if (c == 0x3A || c == 0xB7) return MIDLETTER;
  if (c == 0x27 || c == 0x2E) return MIDNUMLET;
  if (c == 0x2C || c == 0x3B) return MIDNUM;
  if (c == 0x5F) return EXTENDNUMLET;
  if (c == 0xAD) return FORMAT;
  return OTHER;
}

inline char lower1(uint32_t c) {
  if ((c >= 0x41 && c <= 0x5A) || (c >= 0xC0 && c <= 0xD6) || (c >= 0xD8 && c <= 0xDE)) c += 0x20;
  return (char)(unsigned char)c;
}

const char* const kStop[] = {"a", "an", "and", "are", "as", "at", "be", "but", "by", "for", "if",
                             "in", "into", "is", "it", "no", "not", "of", "on", "or", "such",
                             "that", "the", "their", "then", "there", "these", "they", "this",
                             "to", "was", "will", "with"};

bool is_stop(const std::string& t) {
  if (t.size() > 5) return false;
  for (const char* s : kStop)
    if (t == s) return true;
  return false;
}

// nearest non-Format position from k in direction step (may leave [lo, n))
inline long base_pos(const std::vector<WB>& cls, long k, long step) {
  while (k >= 0 && k < (long)cls.size() && cls[k] == FORMAT) k += step;
  return k;
}

// no word break before position j of the segment that starts at `start`
bool joins(const std::vector<WB>& cls, long start, long j) {
  const long a = base_pos(cls, j - 1, -1);
  if (a < start) return false;
  const WB A = cls[a], B = cls[j];
  if (A == NL || B == NL) return false;
  const long nx = base_pos(cls, j + 1, 1);
  const int C = nx < (long)cls.size() ? (int)cls[nx] : -1;
  const long pv = a - 1 >= start ? base_pos(cls, a - 1, -1) : -1;
  const int P = pv >= start ? (int)cls[pv] : -1;
  const bool midl = B == MIDLETTER || B == MIDNUMLET, midA = A == MIDLETTER || A == MIDNUMLET;
  if (A == ALETTER && B == ALETTER) return true;                              // WB5
  if (A == ALETTER && midl && C == ALETTER) return true;                      // WB6
  if (P == ALETTER && midA && B == ALETTER) return true;                      // WB7
  if (A == NUMERIC && B == NUMERIC) return true;                              // WB8
  if (A == ALETTER && B == NUMERIC) return true;                              // WB9
  if (A == NUMERIC && B == ALETTER) return true;                              // WB10
  if (P == NUMERIC && (A == MIDNUM || A == MIDNUMLET) && B == NUMERIC) return true;  // WB11
  if (A == NUMERIC && (B == MIDNUM || B == MIDNUMLET) && C == NUMERIC) return true;  // WB12
  if ((A == ALETTER || A == NUMERIC || A == EXTENDNUMLET) && B == EXTENDNUMLET) return true;  // WB13a
  if (A == EXTENDNUMLET && (B == ALETTER || B == NUMERIC)) return true;       // WB13b
  return false;
}

inline bool special(uint32_t c) {
  switch (c) {
    case '*': case '?': case '!': case '&': case '(': case ')': case '-': case '+': case ':':
    case '"': case '[': case ']': case '~': case '{': case '}': case '^': case '|':
      return true;
    default:
      return false;
  }
}

}  // namespace

// StandardAnalyzer over code units u[0, n) (escape: escapeLucene first).  Returns false when a
// unit is above U+00FF.
bool lucene_analyze(const uint32_t* u, size_t n, bool escape, std::vector<std::string>& out) {
  out.clear();
  std::vector<uint32_t> s;
  s.reserve(escape ? 2 * n : n);
  for (size_t i = 0; i < n; ++i) {
    if (u[i] > 0xFF) return false;
    if (escape && special(u[i])) s.push_back('\\');
    s.push_back(u[i]);
  }
  if (escape) {  // String.trim(): code units <= U+0020 at both ends
    size_t a = 0, b = s.size();
    while (a < b && s[a] <= 0x20) ++a;
    while (b > a && s[b - 1] <= 0x20) --b;
    s = std::vector<uint32_t>(s.begin() + a, s.begin() + b);
  }
  std::vector<WB> cls(s.size());
  for (size_t i = 0; i < s.size(); ++i) cls[i] = wb_class(s[i]);
  const long N = (long)s.size();
  long i = 0;
  std::string tok;
  while (i < N) {
    long j = i + 1;
    if (cls[i] != NL)
      while (j < N && cls[j] == FORMAT) ++j;
    while (j < N && joins(cls, i, j)) {
      ++j;
      while (j < N && cls[j] == FORMAT) ++j;
    }
    bool word = false;
    for (long k = i; k < j; ++k) word = word || cls[k] == ALETTER || cls[k] == NUMERIC;
    if (word && j - i <= 255) {
      tok.clear();
      for (long k = i; k < j; ++k) tok.push_back(lower1(s[k]));
      if (!is_stop(tok)) out.push_back(tok);
    }
    i = j;
  }
  return true;
}

// SmallFloat.floatToByte315 of DefaultSimilarity.lengthNorm = (float)(1 / sqrt(ntokens))
uint8_t lucene_norm_byte(uint32_t ntokens) {
  float f = ntokens ? (float)(1.0 / __builtin_sqrt((double)ntokens)) : __builtin_inff();
  int32_t bits;
  std::memcpy(&bits, &f, 4);
  const int32_t small = bits >> (24 - 3);
  if (small <= ((63 - 15) << 3)) return bits <= 0 ? 0 : 1;
  if (small >= ((63 - 15) << 3) + 0x100) return 255;
  return (uint8_t)(small - ((63 - 15) << 3));
}

}  // namespace dk

extern "C" {

// Test hook: the analyzer's tokens of one value, '\n'-joined into out (NUL terminated).
int dk_lucene_analyze(const uint16_t* units, uint64_t n, int escape, char* out, uint64_t cap,
                      uint64_t* ntokens) {
  if ((n && !units) || !out || !ntokens) return dk_fail_ingest(DK_E_INVALID, "NULL argument");
  std::vector<uint32_t> u(units, units + n);
  std::vector<std::string> toks;
  if (!dk::lucene_analyze(u.data(), n, escape != 0, toks))
    return dk_fail_ingest(DK_E_UNSUPPORTED, "code unit above U+00FF");
  std::string joined;
  for (size_t i = 0; i < toks.size(); ++i) {
    if (i) joined.push_back('\n');
    joined += toks[i];
  }
  if (joined.size() + 1 > cap) return dk_fail_ingest(DK_E_INVALID, "output buffer too small");
  std::memcpy(out, joined.c_str(), joined.size() + 1);
  *ntokens = toks.size();
  return DK_OK;
}

}  // extern "C"
