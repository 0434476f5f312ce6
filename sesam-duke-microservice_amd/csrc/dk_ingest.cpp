// dk_ingest.cpp — native ingestion of a POSTed entity batch into the SoA columns dk_upsert
// takes: JSON text -> records -> packed columns, without materialising
// Duke Record objects.  Host C++ only.
//
// Semantics followed (reference file:line under src/main/java/io/sesam/dukemicroservice/):
//   * the body is an array of entities or one entity object (App.java:955-965, 1104-1114);
//   * IncrementalDataSource.DatasetDataSourceRecordIterator.next (IncrementalDataSource.java:
//     50-101): `_id` via JsonElement.getAsString, empty or missing -> "Got an entity with no
//     '_id' attribute!"; per data-source column, entity.get(name): absent -> no value, a JSON
//     array -> addValue(column, array.getAsString()) once per element (so [] adds nothing,
//     [x] adds x, longer arrays throw: Gson's JsonArray.getAsString), otherwise
//     getAsString (string content, number literal text as written -- Gson's
//     LazilyParsedNumber --, "true"/"false"; null and objects throw); the synthetic ID
//     "<group>__<dataset>__<id>" / "<dataset>__<id>" (:76-88), dukeDeleted when `_deleted`
//     .getAsBoolean() is true (:92-98, Boolean.parseBoolean for strings);
//   * [Duke 1.2, recalled] RecordBuilder.addValue: cleaner first, then empty values skipped;
//     the cleaners named by the reference config (testdukeconfig.xml:50,55,66) as restated
//     in dukehip/records.py (PARITY UNPINNED: Duke's cleaner sources are absent).
// Gson parses leniently; this reader takes strict RFC 8259 JSON in UTF-8 and reports
// anything else -- and any value a cleaner table does not cover -- as DK_E_UNSUPPORTED,
// so the caller packs that batch on its own (Java / Python) path instead.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include <immintrin.h>

#include "dk_clean_table.h"
#include "dk_interner.h"
#include "dukehip.h"

// columns a key function reads but no property scores (dk_source_column.prop >= nprops)
constexpr int kMaxKeyOnly = 16;


extern "C" int dk_fail_ingest(int code, const char* msg);  // dk_api.cpp: sets dk_last_error

namespace {

struct Fail {
  int code;
  std::string msg;
};

[[noreturn]] void fail(int code, const std::string& m) { throw Fail{code, m}; }

// ---- JSON value spans ----------------------------------------------------------------
enum Kind { J_NULL, J_BOOL, J_NUM, J_STR, J_ARR, J_OBJ };

struct Val {
  Kind kind = J_NULL;
  const char* a = nullptr;  // J_STR: content between the quotes (escapes undecoded);
  const char* b = nullptr;  // J_NUM: the literal; J_BOOL: "true"/"false"; J_ARR/J_OBJ: text
  uint32_t nelem = 0;       // J_ARR: element count
  int32_t first = -1;       // J_ARR with one element: that element's index in the side store
};

// a zero byte in x (the classic SWAR test)
inline uint64_t zero_byte(uint64_t x) { return (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull; }
// does the 8-byte word hold a '"', a '\\' or a byte below 0x20?
// per byte: 0x80 where it is one of those; the lowest flagged byte is always a true one (a
// borrow only propagates upwards, from a byte that is flagged itself)
inline uint64_t special_bytes(uint64_t w) {
  return zero_byte(w ^ 0x2222222222222222ull) | zero_byte(w ^ 0x5C5C5C5C5C5C5C5Cull) |
         ((w - 0x2020202020202020ull) & ~w & 0x8080808080808080ull);
}

struct Reader {
  const char* p;
  const char* e;
  std::vector<Val>* side;  // one-element-array payloads of the current entity

  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  char peek() {
    ws();
    if (p >= e) fail(DK_E_UNSUPPORTED, "JSON: unexpected end of input");
    return *p;
  }
  void expect(char c) {
    if (peek() != c) fail(DK_E_UNSUPPORTED, std::string("JSON: expected '") + c + "'");
    ++p;
  }
  void lit(const char* w) {
    const size_t n = strlen(w);
    if ((size_t)(e - p) < n || memcmp(p, w, n) != 0) fail(DK_E_UNSUPPORTED, "JSON: bad literal");
    p += n;
  }
  bool esc = false;  // the last str() held a '\\'
  // string starting at '"': returns [a, b) of the raw content
  void str(const char** a, const char** b) {
    ++p;  // '"'
    *a = p;
    esc = false;
    for (;;) {
      // 8 bytes at a time to the first '"', '\\' or control character (the lowest flagged
      // byte of the SWAR masks is exact)
      if (e - p >= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        const uint64_t m = special_bytes(w);
        if (!m) {
          p += 8;
          continue;
        }
        p += __builtin_ctzll(m) >> 3;
      } else if (p >= e) {
        fail(DK_E_UNSUPPORTED, "JSON: unterminated string");
      }
      const unsigned char c = (unsigned char)*p;
      if (c == '"') break;
      if (c < 0x20) fail(DK_E_UNSUPPORTED, "JSON: control character in a string");
      if (c == '\\') {
        esc = true;
        p += 2;  // the escaped character (validated when decoded)
        if (p > e) fail(DK_E_UNSUPPORTED, "JSON: unterminated string");
        continue;
      }
      ++p;  // an ordinary byte of the tail (< 8 bytes left)
    }
    *b = p;
    ++p;
  }
  void num(Val& v) {
    const char* a = p;
    if (p < e && *p == '-') ++p;
    if (p < e && *p == '0') {
      ++p;
    } else {
      if (p >= e || *p < '1' || *p > '9') fail(DK_E_UNSUPPORTED, "JSON: bad number");
      while (p < e && *p >= '0' && *p <= '9') ++p;
    }
    if (p < e && *p == '.') {
      ++p;
      if (p >= e || *p < '0' || *p > '9') fail(DK_E_UNSUPPORTED, "JSON: bad number");
      while (p < e && *p >= '0' && *p <= '9') ++p;
    }
    if (p < e && (*p == 'e' || *p == 'E')) {
      ++p;
      if (p < e && (*p == '+' || *p == '-')) ++p;
      if (p >= e || *p < '0' || *p > '9') fail(DK_E_UNSUPPORTED, "JSON: bad number");
      while (p < e && *p >= '0' && *p <= '9') ++p;
    }
    v.kind = J_NUM;
    v.a = a;
    v.b = p;
  }
  // any value; nested containers are skipped (only their span is kept)
  void value(Val& v, int depth) {
    if (depth > 512) fail(DK_E_UNSUPPORTED, "JSON: nesting too deep");
    const char c = peek();
    if (c == '"') {
      v.kind = J_STR;
      str(&v.a, &v.b);
    } else if (c == '{') {
      v.kind = J_OBJ;
      v.a = p;
      ++p;
      if (peek() == '}') {
        ++p;
      } else {
        for (;;) {
          if (peek() != '"') fail(DK_E_UNSUPPORTED, "JSON: expected a member name");
          const char *ka, *kb;
          str(&ka, &kb);
          expect(':');
          Val x;
          value(x, depth + 1);
          if (peek() == ',') { ++p; continue; }
          expect('}');
          break;
        }
      }
      v.b = p;
    } else if (c == '[') {
      v.kind = J_ARR;
      v.a = p;
      ++p;
      v.nelem = 0;
      if (peek() == ']') {
        ++p;
      } else {
        Val x;
        for (;;) {
          value(x, depth + 1);
          if (++v.nelem == 1) {
            v.first = (int32_t)side->size();
            side->push_back(x);
          }
          if (peek() == ',') { ++p; continue; }
          expect(']');
          break;
        }
      }
      v.b = p;
    } else if (c == 't') {
      v.kind = J_BOOL;
      v.a = p;
      lit("true");
      v.b = p;
    } else if (c == 'f') {
      v.kind = J_BOOL;
      v.a = p;
      lit("false");
      v.b = p;
    } else if (c == 'n') {
      v.kind = J_NULL;
      lit("null");
    } else {
      num(v);
    }
  }
};

// UTF-8 (strict) string content with JSON escapes -> UTF-16 units appended to out
void decode_string(const char* a, const char* b, std::u16string& out) {
  const unsigned char* p = reinterpret_cast<const unsigned char*>(a);
  const unsigned char* e = reinterpret_cast<const unsigned char*>(b);
  {  // the common case: an ASCII run without escapes, widened in one resize
    const unsigned char* q = p;
    while (q < e && *q != '\\' && *q < 0x80) ++q;
    if (q > p) {
      const size_t o = out.size(), n = (size_t)(q - p);
      out.resize(o + n);
      char16_t* d = &out[o];
      for (size_t i = 0; i < n; ++i) d[i] = (char16_t)p[i];
      p = q;
    }
  }
  auto hex4 = [&](const unsigned char* q) -> uint32_t {
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      const unsigned c = q[i];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail(DK_E_UNSUPPORTED, "JSON: bad \\u escape");
    }
    return v;
  };
  while (p < e) {
    const unsigned c = *p;
    if (c == '\\') {
      if (p + 1 >= e) fail(DK_E_UNSUPPORTED, "JSON: bad escape");
      const unsigned x = p[1];
      p += 2;
      switch (x) {
        case '"': out.push_back(u'"'); break;
        case '\\': out.push_back(u'\\'); break;
        case '/': out.push_back(u'/'); break;
        case 'b': out.push_back(u'\b'); break;
        case 'f': out.push_back(u'\f'); break;
        case 'n': out.push_back(u'\n'); break;
        case 'r': out.push_back(u'\r'); break;
        case 't': out.push_back(u'\t'); break;
        case 'u':
          if (e - p < 4) fail(DK_E_UNSUPPORTED, "JSON: bad \\u escape");
          out.push_back((char16_t)hex4(p));  // lone surrogates pass through, as in Java
          p += 4;
          break;
        default: fail(DK_E_UNSUPPORTED, "JSON: bad escape");
      }
    } else if (c < 0x80) {
      out.push_back((char16_t)c);
      ++p;
    } else {
      int n;
      uint32_t cp;
      if ((c & 0xE0) == 0xC0) { n = 1; cp = c & 0x1F; }
      else if ((c & 0xF0) == 0xE0) { n = 2; cp = c & 0x0F; }
      else if ((c & 0xF8) == 0xF0) { n = 3; cp = c & 0x07; }
      else fail(DK_E_UNSUPPORTED, "invalid UTF-8");
      if (e - p <= n) fail(DK_E_UNSUPPORTED, "invalid UTF-8");
      for (int i = 1; i <= n; ++i) {
        if ((p[i] & 0xC0) != 0x80) fail(DK_E_UNSUPPORTED, "invalid UTF-8");
        cp = (cp << 6) | (p[i] & 0x3F);
      }
      static const uint32_t kMin[4] = {0, 0x80, 0x800, 0x10000};
      if (cp < kMin[n] || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF))
        fail(DK_E_UNSUPPORTED, "invalid UTF-8");
      if (cp >= 0x10000) {
        cp -= 0x10000;
        out.push_back((char16_t)(0xD800 + (cp >> 10)));
        out.push_back((char16_t)(0xDC00 + (cp & 0x3FF)));
      } else {
        out.push_back((char16_t)cp);
      }
      p += n + 1;
    }
  }
}

// com.google.gson.JsonElement.getAsString for the element kinds the reference reads
void as_string(const Val& v, const std::vector<Val>& side, std::u16string& out, const char* what) {
  out.clear();
  switch (v.kind) {
    case J_STR: decode_string(v.a, v.b, out); return;
    case J_NUM:
    case J_BOOL:
      for (const char* q = v.a; q < v.b; ++q) out.push_back((char16_t)(unsigned char)*q);
      return;
    case J_ARR:  // JsonArray.getAsString: the single element's, else IllegalStateException
      if (v.nelem == 1) { as_string(side[v.first], side, out, what); return; }
      fail(DK_E_INVALID, std::string(what) + ": JsonArray.getAsString on an array of " +
                             std::to_string(v.nelem) + " elements");
    case J_NULL: fail(DK_E_INVALID, std::string(what) + ": JsonNull.getAsString is unsupported");
    case J_OBJ: fail(DK_E_INVALID, std::string(what) + ": JsonObject.getAsString is unsupported");
  }
}

// JsonElement.getAsBoolean
bool as_boolean(const Val& v, const std::vector<Val>& side) {
  if (v.kind == J_BOOL) return v.a[0] == 't';
  if (v.kind == J_ARR && v.nelem == 1) return as_boolean(side[v.first], side);
  if (v.kind == J_STR || v.kind == J_NUM) {  // Boolean.parseBoolean(getAsString())
    std::u16string s;
    as_string(v, side, s, "_deleted");
    if (s.size() != 4) return false;
    const char16_t t[4] = {u't', u'r', u'u', u'e'};
    for (int i = 0; i < 4; ++i) {
      char16_t c = s[i];
      if (c >= u'A' && c <= u'Z') c = (char16_t)(c + 32);
      if (c != t[i]) return false;
    }
    return true;
  }
  fail(DK_E_INVALID, "_deleted: getAsBoolean on a JSON null / object / array");
}

// ---- cleaners (dukehip/records.py restatement; PARITY UNPINNED) ----------------------
bool is_norm_ws(char16_t c) {  // the runs LowerCaseNormalizeCleaner collapses
  return c == u' ' || c == u'\t' || c == u'\n' || c == u'\r' || c == 0x00A0;
}

inline bool py_isspace(uint32_t c) {  // Python str.isspace (str.split() / strip())
  if (c < 0x80) return (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x20);
  return c == 0x85 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) || c == 0x2028 ||
         c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}

void lowercase_normalize(std::u16string& s) {  // in place: the output is never longer
  size_t o = 0;
  bool pending = false;
  for (size_t i = 0; i < s.size(); ++i) {
    const char16_t c = s[i];
    if (c >= 0x370) fail(DK_E_UNSUPPORTED, "cleaner: character outside the native table");
    const uint16_t m = kCleanTable[c];
    if (m == 0xFFFF) fail(DK_E_UNSUPPORTED, "cleaner: character outside the native table");
    if (m == 0xFFFE) continue;  // a combining mark: removed with the accents
    const char16_t x = (char16_t)m;
    if (is_norm_ws(x)) {
      pending = true;
      continue;
    }
    if (pending && o) s[o++] = u' ';
    pending = false;
    s[o++] = x;
  }
  s.resize(o);
}

void country_name_clean(std::u16string& s) {
  lowercase_normalize(s);
  const std::u16string the = u"the ", comma_the = u", the";
  if (s.size() >= 4 && s.compare(0, 4, the) == 0) s.erase(0, 4);
  if (s.size() >= 5 && s.compare(s.size() - 5, 5, comma_the) == 0) s.erase(s.size() - 5);
}

void capital_clean(std::u16string& s) {
  lowercase_normalize(s);
  for (char16_t sep : {u',', u'('}) {
    const size_t i = s.find(sep);
    if (i != std::u16string::npos) s.erase(i);
  }
  size_t a = 0, b = s.size();
  while (a < b && py_isspace(s[a])) ++a;
  while (b > a && py_isspace(s[b - 1])) --b;
  s.erase(b);
  s.erase(0, a);
}

// ---- key functions: dukehip.records.PartsKey (code-point slicing, Python semantics) ----
struct KeyScratch {  // per worker, reused across records (no allocation per value)
  std::vector<uint32_t> cp;
  std::vector<std::pair<size_t, size_t>> toks;
};

void code_points(const std::u16string& s, std::vector<uint32_t>& cp) {
  cp.clear();
  for (size_t i = 0; i < s.size(); ++i) {
    const char16_t c = s[i];
    if (c >= 0xD800 && c <= 0xDBFF && i + 1 < s.size() && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
      cp.push_back(0x10000 + (((uint32_t)c - 0xD800) << 10) + (s[i + 1] - 0xDC00));
      ++i;
    } else {
      cp.push_back(c);
    }
  }
}

void append_cp(std::u16string& out, uint32_t c) {
  if (c >= 0x10000) {
    c -= 0x10000;
    out.push_back((char16_t)(0xD800 + (c >> 10)));
    out.push_back((char16_t)(0xDC00 + (c & 0x3FF)));
  } else {
    out.push_back((char16_t)c);
  }
}

// Python slice [start:end] of a sequence of length n (INT32_MIN = None)
void py_slice(int64_t n, int32_t start, int32_t end, int64_t* a, int64_t* b) {
  auto norm = [n](int64_t v, int64_t dflt) {
    if (v == INT32_MIN) return dflt;
    if (v < 0) v += n;
    return v < 0 ? (int64_t)0 : (v > n ? n : v);
  };
  *a = norm(start, 0);
  *b = norm(end, n);
  if (*b < *a) *b = *a;
}

// key_part over a value without surrogates: code points are its units
void key_part_bmp(const std::u16string& v, const dk_key_part& kp, std::u16string& out) {
  size_t lo = 0, hi = v.size();
  if (kp.token != INT32_MIN) {  // str.split() then toks[token], without materialising toks
    // token t >= 0: the t-th from the front; t < 0: the (-t)-th from the back (absent: "")
    const size_t n = v.size();
    if (kp.token >= 0) {
      int64_t k = 0;
      size_t i = 0;
      for (;; ++k) {
        while (i < n && py_isspace(v[i])) ++i;
        if (i >= n) return;
        const size_t a = i;
        while (i < n && !py_isspace(v[i])) ++i;
        if (k == kp.token) {
          lo = a;
          hi = i;
          break;
        }
      }
    } else {
      int64_t k = -1;
      size_t i = n;
      for (;; --k) {
        while (i > 0 && py_isspace(v[i - 1])) --i;
        if (i == 0) return;
        const size_t b = i;
        while (i > 0 && !py_isspace(v[i - 1])) --i;
        if (k == kp.token) {
          lo = i;
          hi = b;
          break;
        }
      }
    }
  }
  int64_t a, b;
  py_slice((int64_t)(hi - lo), kp.start, kp.end, &a, &b);
  out.append(v, lo + (size_t)a, (size_t)(b - a));
}

void key_part(const std::u16string* value, const dk_key_part& kp, std::u16string& out, KeyScratch& ks) {
  if (!value) return;  // a missing value contributes ""
  bool surrogate = false;
  for (char16_t c : *value) surrogate |= (c >= 0xD800 && c <= 0xDFFF);
  if (!surrogate) return key_part_bmp(*value, kp, out);
  std::vector<uint32_t>& cp = ks.cp;
  code_points(*value, cp);
  size_t lo = 0, hi = cp.size();
  if (kp.token != INT32_MIN) {  // str.split() then toks[token]
    auto& toks = ks.toks;
    toks.clear();
    size_t i = 0;
    while (i < cp.size()) {
      while (i < cp.size() && py_isspace(cp[i])) ++i;
      if (i >= cp.size()) break;
      const size_t a = i;
      while (i < cp.size() && !py_isspace(cp[i])) ++i;
      toks.emplace_back(a, i);
    }
    const int64_t nt = (int64_t)toks.size();
    int64_t t = kp.token;
    if (t < -nt || t >= nt) return;
    if (t < 0) t += nt;
    lo = toks[t].first;
    hi = toks[t].second;
  }
  int64_t a, b;
  py_slice((int64_t)(hi - lo), kp.start, kp.end, &a, &b);
  for (int64_t i = a; i < b; ++i) append_cp(out, cp[lo + i]);
}

// ---- parallel packing ------------------------------------------------------------------
// A batch is packed in three steps: (1) the top-level array is split into entity spans by a
// chunk-parallel structural scan (quote parity per chunk, then bracket events outside
// strings, then one pass over the events); (2) workers parse contiguous runs of entities
// into slices of every column; (3) the slices are concatenated in parallel and the record
// IDs interned in batch order.  Strict JSON only: every span goes through the Reader and
// every gap between spans is checked, so exactly the sequential reader's inputs are taken,
// and a failure reports the first failing entity (its error, or the split's).

int pack_threads(uint64_t work, uint64_t per_thread) {
  int t = 16;  // the GPU box's CPU share per GPU; the container's own core count if lower
  const unsigned hw = std::thread::hardware_concurrency();
  if (hw && hw < (unsigned)t) t = (int)hw;
  if (const char* e = getenv("DK_INGEST_THREADS")) {
    const int v = atoi(e);
    if (v > 0) return std::min(v, 64);  // forced (tests exercise the merge on small batches)
  }
  const uint64_t by_work = work / per_thread;
  return (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)t, by_work));
}

template <typename F>
void parallel_for(int n, F&& f) {
  std::vector<std::thread> th;
  th.reserve(n > 1 ? n - 1 : 0);
  for (int i = 1; i < n; ++i) th.emplace_back([&f, i] { f(i); });
  f(0);
  for (auto& t : th) t.join();
}

inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

// 8 bytes at a time: does the word hold a '"' or a '\\'?
inline bool has_quote_or_bs(uint64_t w) {
  auto zero = [](uint64_t x) { return (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull; };
  return zero(w ^ 0x2222222222222222ull) | zero(w ^ 0x5C5C5C5C5C5C5C5Cull);
}

struct Split {
  PodVec<uint64_t> starts, ends;  // entity k: [starts[k] ('{'), ends[k] (one past '}'))
  uint64_t n = 0;                 // entities (the arrays may hold one more start)
  int code = DK_OK;               // a structural error after the spans
  std::string msg;
};

// the unescaped-quote parity of [c0, c1) (the escape state at c0 from the backslash run
// before it: valid JSON has backslashes only inside strings, where they pair up)
bool chunk_escaped_at(const char* J, uint64_t lo, uint64_t c0) {
  uint64_t k = 0;
  while (c0 > lo + k && J[c0 - 1 - k] == '\\') ++k;
  return k & 1;
}

uint32_t quote_parity(const char* J, uint64_t c0, uint64_t c1, bool esc) {
  uint32_t q = 0;
  uint64_t i = c0;
  while (i < c1) {
    if (!esc && i + 8 <= c1) {
      uint64_t w;
      memcpy(&w, J + i, 8);
      if (!has_quote_or_bs(w)) { i += 8; continue; }
    }
    const char ch = J[i++];
    if (esc) { esc = false; continue; }
    if (ch == '\\') esc = true;
    else if (ch == '"') q ^= 1;
  }
  return q;
}

// Brackets outside strings in [c0, c1): f(pos, ch) for each of '{' '[' '}' ']'; f returns
// false to stop the scan.
template <typename F>
void for_brackets(const char* J, uint64_t c0, uint64_t c1, bool esc, bool instr, F&& f) {
  uint64_t i = c0;
  while (i < c1) {
    if (instr && !esc && i + 8 <= c1) {
      uint64_t w;
      memcpy(&w, J + i, 8);
      if (!has_quote_or_bs(w)) { i += 8; continue; }
    }
    const char ch = J[i];
    if (esc) {
      esc = false;
    } else if (ch == '\\') {
      esc = true;
    } else if (ch == '"') {
      instr = !instr;
    } else if (!instr && (ch == '{' || ch == '[' || ch == '}' || ch == ']')) {
      if (!f(i, ch)) return;
    }
    ++i;
  }
}

// ---- 64-byte blocks (AVX2 + carry-less multiply), the split's fast path ----------------
// Per block: the masks of '"', '\\' and the four brackets (movemask of byte compares); the
// escaped characters from the backslash mask (a character is escaped when an odd-length
// run of backslashes precedes it: runs starting on odd bits carry through the run when
// added to their start bit), carried from block to block; the in-string mask as the
// prefix XOR of the unescaped quotes (one PCLMULQDQ by all-ones), carried as a sign mask.
// The same state machine as quote_parity / for_brackets, 64 bytes per step.
struct BlockMasks {
  uint64_t quote, bs, open, close, square;  // square: '[' or ']'
};

__attribute__((target("avx2"))) inline BlockMasks block_masks(const char* p) {
  const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p));
  const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + 32));
#define DK_EQ64(c)                                                                               \
  ((uint64_t)(uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(a, _mm256_set1_epi8(c))) |          \
   ((uint64_t)(uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(b, _mm256_set1_epi8(c))) << 32))
  const uint64_t sqo = DK_EQ64('['), sqc = DK_EQ64(']');
  const BlockMasks m{DK_EQ64('"'), DK_EQ64('\\'), DK_EQ64('{') | sqo, DK_EQ64('}') | sqc, sqo | sqc};
#undef DK_EQ64
  return m;
}

// characters escaped by a preceding backslash run; *carry: the next block's first
// character is escaped
inline uint64_t escaped_bits(uint64_t bs, uint64_t* carry) {
  constexpr uint64_t kEven = 0x5555555555555555ull;
  bs &= ~*carry;  // an escaped backslash starts no escape
  const uint64_t follows = (bs << 1) | *carry;
  const uint64_t odd_starts = bs & ~kEven & ~follows;
  uint64_t seq_even;
  *carry = __builtin_add_overflow(odd_starts, bs, &seq_even) ? 1u : 0u;
  return (kEven ^ (seq_even << 1)) & follows;
}

__attribute__((target("avx2,pclmul"))) inline uint64_t prefix_xor(uint64_t x) {  // VEX-encoded: no SSE/AVX transition in the AVX2 loop
  return (uint64_t)_mm_cvtsi128_si64(
      _mm_clmulepi64_si128(_mm_set_epi64x(0, (long long)x), _mm_set1_epi8((char)0xFF), 0));
}

// vzeroupper when the CPU has AVX: a caller that used 256/512-bit registers (numpy under
// Python, or this file's AVX2 split) leaves the upper halves dirty, and on Intel cores every
// legacy-SSE instruction of the (compiler-vectorised) parse then pays a merge dependency --
// measured 4x slower per entity in this container until cleared.  AMD cores do not care.
__attribute__((target("avx"))) void zero_upper_avx() { _mm256_zeroupper(); }
void clear_upper() {
  static const bool avx = [] {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx") != 0;
  }();
  if (avx) zero_upper_avx();
}

bool simd_split_ok() {
  static const bool cpu = [] {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx2") && __builtin_cpu_supports("pclmul");
  }();
  const char* e = getenv("DK_INGEST_SCALAR");  // A/B and the differential tests
  return cpu && !(e && e[0] == '1');
}

// f(block base, masks) over [c0, c1) in 64-byte blocks, the last one zero padded
template <typename F>
__attribute__((target("avx2"))) void for_blocks(const char* J, uint64_t c0, uint64_t c1, F&& f) {
  uint64_t i = c0;
  for (; i + 64 <= c1; i += 64) f(i, block_masks(J + i));
  if (i < c1) {
    alignas(32) char tail[64] = {};
    memcpy(tail, J + i, c1 - i);
    f(i, block_masks(tail));
  }
}

// quote_parity of [c0, c1), 64 bytes per step
__attribute__((target("avx2,pclmul"))) uint32_t quote_parity_simd(const char* J, uint64_t c0, uint64_t c1, bool esc) {
  uint64_t carry = esc ? 1u : 0u;
  uint32_t q = 0;
  for_blocks(J, c0, c1, [&](uint64_t, const BlockMasks& m) {
    const uint64_t e = escaped_bits(m.bs, &carry);
    q ^= (uint32_t)__builtin_popcountll(m.quote & ~e) & 1u;
  });
  return q;
}

// the brackets outside strings in [c0, c1), in order, as position | kCloser | kSquare (the
// depth walk then never re-reads the body), and their depth change
constexpr uint64_t kCloser = 1ull << 63, kSquare = 1ull << 62, kPosMask = kSquare - 1;
__attribute__((target("avx2,pclmul"))) int64_t brackets_simd(const char* J, uint64_t c0, uint64_t c1, bool esc,
                                                            bool instr, std::vector<uint64_t>& out) {
  uint64_t carry = esc ? 1u : 0u;
  uint64_t inmask = instr ? ~0ull : 0ull;  // in a string at the block's start: all ones
  int64_t d = 0;
  for_blocks(J, c0, c1, [&](uint64_t base, const BlockMasks& m) {
    const uint64_t e = escaped_bits(m.bs, &carry);
    const uint64_t s = prefix_xor(m.quote & ~e) ^ inmask;
    inmask = (uint64_t)((int64_t)s >> 63);
    const uint64_t op = m.open & ~s, cl = m.close & ~s;
    d += __builtin_popcountll(op) - __builtin_popcountll(cl);
    uint64_t br = op | cl;
    while (br) {
      const int b = __builtin_ctzll(br);
      out.push_back((base + (uint64_t)b) | ((cl >> b & 1) ? kCloser : 0) | ((m.square >> b & 1) ? kSquare : 0));
      br &= br - 1;
    }
  });
  return d;
}

// One chunk of the top-level array, its depth at the start known: entity starts ('{' at
// depth 1) and ends (one past the '}' back to depth 1), the array's closing ']', or the
// first bracket that cannot be there.
struct ChunkScan {
  std::vector<uint64_t> starts, ends;
  uint64_t close = UINT64_MAX;  // the top-level ']'
  uint64_t bad = UINT64_MAX;    // a non-object element's '[' or a stray closer
};

// the chunk's depth walk over its brackets (each visited once, in order, by `each`)
template <typename Each>
void walk_chunk(Each&& each, int64_t depth, ChunkScan& C) {
  each([&](uint64_t pos, char ch) {
    if (ch == '{' || ch == '[') {
      if (depth == 1) {
        if (ch != '{') { C.bad = pos; return false; }
        C.starts.push_back(pos);
      }
      ++depth;
      return true;
    }
    --depth;
    if (depth == 1) {
      C.ends.push_back(pos + 1);
    } else if (depth == 0) {
      if (ch == ']') C.close = pos;
      else C.bad = pos;
      return false;
    } else if (depth < 0) {
      C.bad = pos;
      return false;
    }
    return true;
  });
}

void scan_chunk(const char* J, uint64_t c0, uint64_t c1, bool esc, bool instr, int64_t depth, ChunkScan& C) {
  walk_chunk([&](auto&& f) { for_brackets(J, c0, c1, esc, instr, f); }, depth, C);
}

// the same over a chunk's brackets found by brackets_simd (their kinds in the flag bits)
void scan_chunk_list(const std::vector<uint64_t>& br, int64_t depth, ChunkScan& C) {
  walk_chunk(
      [&](auto&& f) {
        for (uint64_t x : br) {
          const char ch = (x & kCloser) ? ((x & kSquare) ? ']' : '}') : ((x & kSquare) ? '[' : '{');
          if (!f(x & kPosMask, ch)) return;
        }
      },
      depth, C);
}

// The text between two elements of the top-level array: whitespace only, one ',' in
// whitespace, a ',' followed by something else, or something else.
enum Gap { kEmpty, kComma, kCommaOther, kOther };

Gap classify_gap(const char* J, uint64_t from, uint64_t to) {
  uint64_t i = from;
  while (i < to && is_ws(J[i])) ++i;
  if (i == to) return kEmpty;
  if (J[i] != ',') return kOther;
  ++i;
  while (i < to && is_ws(J[i])) ++i;
  return i == to ? kComma : kCommaOther;
}

// What follows the gap before element r: an entity '{', the array's ']', a misplaced
// bracket, or the end of the body.  True when well formed; otherwise S gets the error the
// sequential reader raises there (Reader.peek / expect, "entity r is not a JSON object").
enum Next { kEntity, kClose, kBad, kEnd };

bool element_check(Gap g, uint64_t r, Next nx, Split& S) {
  auto invalid = [&] {
    S.code = DK_E_INVALID;
    S.msg = "entity " + std::to_string(r) + " is not a JSON object";
    return false;
  };
  auto unsup = [&](const char* m) {
    S.code = DK_E_UNSUPPORTED;
    S.msg = m;
    return false;
  };
  if (r == 0) {  // right after '['
    if (g != kEmpty) return invalid();
    if (nx == kEntity || nx == kClose) return true;
    return nx == kEnd ? unsup("JSON: unexpected end of input") : invalid();
  }
  switch (g) {  // after entity r - 1
    case kEmpty:
      if (nx == kClose) return true;
      return unsup(nx == kEnd ? "JSON: unexpected end of input" : "JSON: expected ']'");
    case kComma:
      if (nx == kEntity) return true;
      return nx == kEnd ? unsup("JSON: unexpected end of input") : invalid();
    case kCommaOther:
      return invalid();
    default:
      return unsup("JSON: expected ']'");
  }
}

// Entity spans of the body: an array of entities, or one entity (App.java:955-965).  Four
// passes over chunks of the array on pack_threads() threads: unescaped-quote parity (so
// each chunk knows whether it starts inside a string), bracket depth change, then the
// entity starts / ends at the chunk's now known depth; the gaps between entities last.
void split_entities(const char* J, uint64_t len, Split& S) {
  static const bool timing = getenv("DK_INGEST_TIMING") != nullptr;  // sub-phase times
  auto T0 = std::chrono::steady_clock::now();
  auto lap = [&](const char* w) {
    if (!timing) return;
    const auto t1 = std::chrono::steady_clock::now();
    fprintf(stderr, "  split %s %.2f ms\n", w, std::chrono::duration<double, std::milli>(t1 - T0).count());
    T0 = t1;
  };
  uint64_t p = 0;
  while (p < len && is_ws(J[p])) ++p;
  if (p >= len) {
    S.code = DK_E_UNSUPPORTED;
    S.msg = "JSON: unexpected end of input";
    return;
  }
  if (J[p] != '[') {  // one entity: the worker parses it to the end of the body
    if (J[p] != '{') {
      S.code = DK_E_INVALID;
      S.msg = "entity 0 is not a JSON object";
      return;
    }
    S.starts.push_back(p);
    S.ends.push_back(len);
    S.n = 1;
    return;
  }
  const uint64_t lo = p + 1;
  const uint64_t body = len - lo;
  const int T = pack_threads(body, 1u << 20);
  std::vector<uint64_t> cut(T + 1);
  for (int t = 0; t <= T; ++t) cut[t] = lo + body * (uint64_t)t / (uint64_t)T;
  std::vector<uint32_t> par(T);
  std::vector<char> esc0(T), instr(T);
  std::vector<int64_t> delta(T), d0(T);
  std::vector<ChunkScan> CS(T);
  const bool simd = simd_split_ok();
  std::vector<std::vector<uint64_t>> BR(simd ? T : 0);  // SIMD: each chunk's brackets
  parallel_for(T, [&](int t) {
    esc0[t] = chunk_escaped_at(J, lo, cut[t]);
    par[t] = simd ? quote_parity_simd(J, cut[t], cut[t + 1], esc0[t])
                  : quote_parity(J, cut[t], cut[t + 1], esc0[t]);
  });
  lap("parity");
  for (int t = 0, q = 0; t < T; ++t) {
    instr[t] = (char)q;
    q ^= (int)par[t];
  }
  parallel_for(T, [&](int t) {
    int64_t d = 0;
    if (simd) {  // one pass: the positions (the depth walk reads their characters later)
      BR[t].reserve((cut[t + 1] - cut[t]) / 32 + 16);
      d = brackets_simd(J, cut[t], cut[t + 1], esc0[t], instr[t], BR[t]);
    } else {
      for_brackets(J, cut[t], cut[t + 1], esc0[t], instr[t], [&](uint64_t, char ch) {
        d += (ch == '{' || ch == '[') ? 1 : -1;
        return true;
      });
    }
    delta[t] = d;
  });
  lap("brackets");
  for (int t = 0; t < T; ++t) d0[t] = t ? d0[t - 1] + delta[t - 1] : 1;
  parallel_for(T, [&](int t) {
    if (d0[t] <= 0) return;
    if (simd) scan_chunk_list(BR[t], d0[t], CS[t]);
    else scan_chunk(J, cut[t], cut[t + 1], esc0[t], instr[t], d0[t], CS[t]);
  });
  lap("walk");
  // the chunks up to the first that closes the array or holds a misplaced bracket
  uint64_t stop = len, close = UINT64_MAX, bad = UINT64_MAX;
  int tl = T - 1;
  for (int t = 0; t < T; ++t) {
    if (CS[t].bad != UINT64_MAX) { bad = stop = CS[t].bad; tl = t; break; }
    if (CS[t].close != UINT64_MAX) { close = stop = CS[t].close; tl = t; break; }
  }
  std::vector<uint64_t> so(tl + 2, 0), eo(tl + 2, 0);
  for (int t = 0; t <= tl; ++t) {
    so[t + 1] = so[t] + CS[t].starts.size();
    eo[t + 1] = eo[t] + CS[t].ends.size();
  }
  // uninitialised: each chunk's worker writes (and first-touches) its part
  PodVec<uint64_t>& starts = S.starts;
  PodVec<uint64_t>& ends = S.ends;
  starts.reset_uninit(so[tl + 1]);
  ends.reset_uninit(eo[tl + 1]);
  parallel_for(tl + 1, [&](int t) {
    if (!CS[t].starts.empty()) memcpy(starts.data() + so[t], CS[t].starts.data(), CS[t].starts.size() * 8);
    if (!CS[t].ends.empty()) memcpy(ends.data() + eo[t], CS[t].ends.data(), CS[t].ends.size() * 8);
  });
  lap("concat");
  const uint64_t ns = starts.size(), ne = ends.size();  // ne == ns or ns - 1
  // the first entity whose gap is malformed (gaps in parallel; the first one found wins)
  std::vector<uint64_t> first_bad(T, UINT64_MAX);
  parallel_for(T, [&](int t) {
    const uint64_t k0 = ns * (uint64_t)t / (uint64_t)T, k1 = ns * (uint64_t)(t + 1) / (uint64_t)T;
    for (uint64_t k = k0; k < k1; ++k) {
      const Gap g = classify_gap(J, k ? ends[k - 1] : lo, starts[k]);
      if (g != (k ? kComma : kEmpty)) { first_bad[t] = k; break; }
    }
  });
  lap("gaps");
  uint64_t kbad = UINT64_MAX;
  for (int t = 0; t < T && kbad == UINT64_MAX; ++t) kbad = first_bad[t];
  const uint64_t nspans = kbad != UINT64_MAX ? kbad : ne;
  S.n = nspans;
  if (kbad != UINT64_MAX) {  // entity kbad follows a malformed gap
    element_check(classify_gap(J, kbad ? ends[kbad - 1] : lo, starts[kbad]), kbad, kEntity, S);
    return;
  }
  if (ns > ne) {  // an entity still open where the scan stopped (its gap was fine)
    S.code = DK_E_UNSUPPORTED;
    S.msg = "JSON: unexpected end of input";
    return;
  }
  const uint64_t last = nspans ? ends[nspans - 1] : lo;
  const Next nx = bad != UINT64_MAX ? kBad : (close != UINT64_MAX ? kClose : kEnd);
  if (!element_check(classify_gap(J, last, stop), nspans, nx, S)) return;
  uint64_t i = close + 1;  // kClose: whitespace only after the array
  while (i < len && is_ws(J[i])) ++i;
  if (i != len) {
    S.code = DK_E_UNSUPPORTED;
    S.msg = "JSON: trailing characters";
  }
}

// One worker's slice of a column: values back to back, offsets relative to the slice.  The
// units are kept one byte wide while every unit so far is <= 0xFF (the common case: half the
// scratch, and the merge copies them as they are), two bytes from the first wider one on
// (or from the start: the record-ID column, which the interner reads as UTF-16).
struct ColPart {
  PodVec<uint32_t> off;
  PodVec<uint8_t> u8;
  PodVec<char16_t> u16;
  PodVec<uint8_t> present;
  bool missing = false, wide = false;
  char16_t orv = 0;  // the OR of every unit: <= 0xFF iff the slice is narrow
  void init(uint64_t n, uint64_t units, bool wide16) {
    wide = wide16;
    off.reserve(n + 1);
    off.push_back(0);
    present.reserve(n);
    if (wide) u16.reserve(units);
    else u8.reserve(units);
  }
  uint64_t units() const { return wide ? u16.size() : u8.size(); }
  void widen() {
    u16.reserve(std::max<uint64_t>(2 * u8.size(), 64));
    u16.resize_uninit(u8.size());
    for (uint64_t i = 0; i < u8.size(); ++i) u16[i] = u8[i];
    u8 = PodVec<uint8_t>();
    wide = true;
  }
  void add(const char16_t* v, size_t n) {
    char16_t o = 0;
    for (size_t i = 0; i < n; ++i) o |= v[i];
    orv |= o;
    if (!wide && o > 0xFF) widen();
    if (wide) {
      u16.append(v, n);
    } else {
      const uint64_t b = u8.size();
      u8.resize_uninit(b + n);
      uint8_t* d = u8.data() + b;
      for (size_t i = 0; i < n; ++i) d[i] = (uint8_t)v[i];
    }
    off.push_back((uint32_t)units());
    present.push_back(1);
  }
  void add(const std::u16string& v) { add(v.data(), v.size()); }
  void add_bytes(const char* v, size_t n) {  // ASCII: the units are the bytes
    if (wide) {
      const uint64_t b = u16.size();
      u16.resize_uninit(b + n);
      for (size_t i = 0; i < n; ++i) u16[b + i] = (unsigned char)v[i];
    } else {
      u8.append(reinterpret_cast<const uint8_t*>(v), n);
    }
    off.push_back((uint32_t)units());
    present.push_back(1);
  }
  // pre (UTF-16) then the ASCII bytes v, as two-byte units; returns where the value starts
  const char16_t* add_prefixed(const char16_t* pre, size_t np, const char* v, size_t n) {
    if (!wide) widen();
    char16_t o = 0;
    for (size_t i = 0; i < np; ++i) o |= pre[i];
    orv |= o;
    const uint64_t b = u16.size();
    u16.resize_uninit(b + np + n);
    char16_t* d = u16.data() + b;
    memcpy(d, pre, np * 2);
    for (size_t i = 0; i < n; ++i) d[np + i] = (unsigned char)v[i];
    off.push_back((uint32_t)units());
    present.push_back(1);
    return d;
  }
  void add_missing() {
    off.push_back((uint32_t)units());
    present.push_back(0);
    missing = true;
  }
};

struct Slice {
  uint64_t e0 = 0, e1 = 0;      // entity range
  std::vector<ColPart> cols;    // nprops, then nkeys, then the record ID, then the entity id
  std::vector<uint8_t> deleted;
  std::vector<uint64_t> hash;   // record-ID hashes (U16Table::hash)
  int code = DK_OK;
  uint64_t fail_at = 0;
  std::string msg;
};

struct SourceView {
  const dk_source* src;
  std::vector<std::string> names;  // data-source columns, then "_id", "_deleted"
  int i_id, i_del;
  std::u16string ds;
};

// ---- the ASCII fast path ---------------------------------------------------------------
// [a, b) holds no '\\' and no byte >= 0x80: its JSON string content is its UTF-16 units
inline bool plain_ascii(const char* a, const char* b) {
  uint64_t acc = 0, bs = 0, w;
  for (; b - a >= 8; a += 8) {
    memcpy(&w, a, 8);
    acc |= w;
    bs |= zero_byte(w ^ 0x5C5C5C5C5C5C5C5Cull);
  }
  for (; a < b; ++a) {
    acc |= (unsigned char)*a;
    bs |= *a == '\\';
  }
  return !((acc & 0x8080808080808080ull) | bs);
}

// key_part_bmp over an ASCII value (code points = bytes; the same token and slice rules)
void key_part_ascii(const char* v, size_t n, const dk_key_part& kp, std::string& out) {
  size_t lo = 0, hi = n;
  if (kp.token != INT32_MIN) {
    if (kp.token >= 0) {
      size_t i = 0;
      for (int64_t k = 0;; ++k) {
        while (i < n && py_isspace((unsigned char)v[i])) ++i;
        if (i >= n) return;
        const size_t a = i;
        while (i < n && !py_isspace((unsigned char)v[i])) ++i;
        if (k == kp.token) {
          lo = a;
          hi = i;
          break;
        }
      }
    } else {
      size_t i = n;
      for (int64_t k = -1;; --k) {
        while (i > 0 && py_isspace((unsigned char)v[i - 1])) --i;
        if (i == 0) return;
        const size_t b = i;
        while (i > 0 && !py_isspace((unsigned char)v[i - 1])) --i;
        if (k == kp.token) {
          lo = i;
          hi = b;
          break;
        }
      }
    }
  }
  int64_t a, b;
  py_slice((int64_t)(hi - lo), kp.start, kp.end, &a, &b);
  out.append(v + lo + a, (size_t)(b - a));
}

// Does the entity take the fast path?  Every member read is a string without escapes or
// non-ASCII bytes, a number or a boolean literal (getAsString: the text as written), `_id`
// is one of those and not empty, `_deleted` (if present) is a boolean literal, no column
// cleans (checked per source) and no property gets a second value; the property values are
// then the members' raw spans (pa, pl).  Anything else -- arrays, null, escapes, UTF-8,
// errors -- goes through the general path, which decodes, or reports, it.
bool ascii_record(const SourceView& V, const std::vector<Val>& got, const std::vector<char>& has,
                  std::vector<const char*>& pa, std::vector<uint32_t>& pl, std::vector<char>& pset) {
  auto plain = [](const Val& v) {
    return v.kind == J_NUM || v.kind == J_BOOL || (v.kind == J_STR && plain_ascii(v.a, v.b));
  };
  const Val& id = got[V.i_id];
  if (!has[V.i_id] || !plain(id) || id.a == id.b) return false;
  if (has[V.i_del] && got[V.i_del].kind != J_BOOL) return false;
  std::fill(pset.begin(), pset.end(), 0);
  const dk_source* src = V.src;
  for (int c = 0; c < src->ncolumns; ++c) {
    if (!has[c]) continue;
    const Val& v = got[c];
    if (!plain(v)) return false;
    const int p = src->columns[c].prop;
    if (v.a == v.b || p < 0) continue;  // RecordBuilder.addValue skips ""
    if (pset[p]) return false;
    pset[p] = 1;
    pa[p] = v.a;
    pl[p] = (uint32_t)(v.b - v.a);
  }
  return true;
}

// IncrementalDataSource.DatasetDataSourceRecordIterator.next for entities [e0, e1)
void parse_slice(const SourceView& V, const char* J, const Split& S, Slice& out) {
  clear_upper();  // the calling thread's (a worker's is clean)
  const dk_source* src = V.src;
  const int np = src->nprops, nk = src->nkeys;
  out.cols.clear();
  out.cols.resize(np + nk + 2);
  const uint64_t n = out.e1 - out.e0;
  // a value is at most as long as its JSON text: the slice's bytes bound every property
  // column's units, so those buffers never grow and copy (reserved, untouched pages cost
  // nothing); keys and IDs grow geometrically from a per-record guess
  const uint64_t bytes = n ? S.ends[out.e1 - 1] - S.starts[out.e0] : 0;
  for (int c = 0; c < np + nk + 2; ++c)
    out.cols[c].init(n, c < np ? bytes + 64 : 16 * n + 64, c == np + nk);
  out.deleted.reserve(n);
  out.hash.reserve(n);
  std::vector<Val> got(V.names.size()), side;
  std::vector<char> has(V.names.size());
  // the scored properties, then the key-only ones (columns with prop >= nprops)
  std::vector<std::u16string> pv(np + kMaxKeyOnly);
  std::vector<char> pset(np + kMaxKeyOnly);
  std::u16string s, key, mname, eid, rid;
  if (src->group_no) {  // "<group>__<dataset>__" / "<dataset>__", then the entity id
    rid.push_back((char16_t)(u'0' + src->group_no));
    rid += u"__";
  }
  rid += V.ds;
  rid += u"__";
  const size_t rid_prefix = rid.size();
  KeyScratch ks;
  // the ASCII fast path (ascii_record): no column cleans (a cleaner rewrites the value)
  bool fast_src = !getenv("DK_INGEST_NOFAST");
  for (int c = 0; c < src->ncolumns; ++c) fast_src = fast_src && src->columns[c].cleaner == DK_CLEAN_NONE;
  std::vector<const char*> pa(np + kMaxKeyOnly);
  std::vector<uint32_t> pl(np + kMaxKeyOnly);
  std::string kb;
  uint64_t r = out.e0;
  try {
    for (; r < out.e1; ++r) {
      Reader R{J + S.starts[r], J + S.ends[r], &side};
      // one entity: its members in one pass (a repeated name: the last wins, as Gson's
      // JsonObject keeps it); nested containers are skipped
      side.clear();
      std::fill(has.begin(), has.end(), 0);
      if (R.peek() != '{') fail(DK_E_INVALID, "entity " + std::to_string(r) + " is not a JSON object");
      ++R.p;
      if (R.peek() == '}') {
        ++R.p;
      } else {
        for (;;) {
          const char *ka, *kb2;
          if (R.peek() != '"') fail(DK_E_UNSUPPORTED, "JSON: expected a member name");
          R.str(&ka, &kb2);
          const bool name_esc = R.esc;
          R.expect(':');
          Val v;
          R.value(v, 2);
          // the member names read are ASCII; compared after unescaping only when escaped
          const char* na = ka;
          size_t nn = (size_t)(kb2 - ka);
          std::string esc_name;
          if (name_esc) {
            mname.clear();
            decode_string(ka, kb2, mname);
            for (char16_t c : mname) {
              if (c > 0x7F) { esc_name = "\x01"; break; }  // not one of the names read
              esc_name.push_back((char)c);
            }
            na = esc_name.data();
            nn = esc_name.size();
          }
          for (size_t i = 0; i < V.names.size(); ++i) {  // the first column of that name
            if (V.names[i].size() == nn && (nn == 0 || (V.names[i][0] == na[0] &&
                                                        memcmp(V.names[i].data(), na, nn) == 0))) {
              got[i] = v;
              has[i] = 1;
              break;
            }
          }
          if (R.peek() == ',') { ++R.p; continue; }
          R.expect('}');
          break;
        }
      }
      R.ws();
      if (R.p != R.e) fail(DK_E_UNSUPPORTED, "JSON: trailing characters");
      if (fast_src && ascii_record(V, got, has, pa, pl, pset)) {
        // every value read is ASCII text as written: its bytes are its UTF-16 units, the
        // same values the general path below produces, without decoding
        for (int p = 0; p < np; ++p) {
          if (pset[p]) out.cols[p].add_bytes(pa[p], pl[p]);
          else out.cols[p].add_missing();
        }
        for (int k = 0; k < nk; ++k) {
          kb.clear();
          const dk_key_function& kf = src->keys[k];
          for (int i = 0; i < kf.nparts; ++i) {
            const dk_key_part& kp = kf.parts[i];
            if (kp.prop < 0 || kp.prop >= np + kMaxKeyOnly) fail(DK_E_INVALID, "key part property out of range");
            if (pset[kp.prop]) key_part_ascii(pa[kp.prop], pl[kp.prop], kp, kb);
          }
          out.cols[np + k].add_bytes(kb.data(), kb.size());
        }
        const Val& id = got[V.i_id];
        const char16_t* rp = out.cols[np + nk].add_prefixed(rid.data(), rid_prefix, id.a, (size_t)(id.b - id.a));
        out.hash.push_back(U16Table::hash(rp, rid_prefix + (size_t)(id.b - id.a)));
        out.cols[np + nk + 1].add_bytes(id.a, (size_t)(id.b - id.a));
        out.deleted.push_back(has[V.i_del] && got[V.i_del].a[0] == 't' ? 1 : 0);
        continue;
      }
      // entity id (IncrementalDataSource.java:54-61)
      eid.clear();
      if (has[V.i_id]) as_string(got[V.i_id], side, eid, "_id");
      if (eid.empty()) fail(DK_E_INVALID, "Got an entity with no '_id' attribute!");
      // columns in data-source order, RecordBuilder.addValue: clean, skip empty
      std::fill(pset.begin(), pset.end(), 0);
      for (int c = 0; c < src->ncolumns; ++c) {
        if (!has[c]) continue;
        const dk_source_column& sc = src->columns[c];
        const Val& v = got[c];
        int reps = 1;
        if (v.kind == J_ARR) {
          if (v.nelem == 0) continue;
          reps = (int)v.nelem;  // getAsString on the array itself, once per element
        }
        for (int rep = 0; rep < reps; ++rep) {
          as_string(v, side, s, sc.name);
          if (sc.cleaner == DK_CLEAN_LOWERCASE_NORMALIZE) lowercase_normalize(s);
          else if (sc.cleaner == DK_CLEAN_COUNTRY_NAME) country_name_clean(s);
          else if (sc.cleaner == DK_CLEAN_CAPITAL) capital_clean(s);
          if (s.empty() || sc.prop < 0) continue;
          if (pset[sc.prop])
            fail(DK_E_UNSUPPORTED, std::string("column ") + sc.name +
                                       ": a second value for one property (the GPU path holds one)");
          pv[sc.prop].swap(s);  // s takes the old buffer (cleared by the next as_string)
          pset[sc.prop] = 1;
        }
      }
      for (int p = 0; p < np; ++p) {
        if (pset[p]) out.cols[p].add(pv[p]);
        else out.cols[p].add_missing();
      }
      // key functions over the cleaned values
      for (int k = 0; k < nk; ++k) {
        key.clear();
        const dk_key_function& kf = src->keys[k];
        for (int i = 0; i < kf.nparts; ++i) {
          const dk_key_part& kp = kf.parts[i];
          if (kp.prop < 0 || kp.prop >= np + kMaxKeyOnly) fail(DK_E_INVALID, "key part property out of range");
          key_part(pset[kp.prop] ? &pv[kp.prop] : nullptr, kp, key, ks);
        }
        out.cols[np + k].add(key);
      }
      // synthetic properties (IncrementalDataSource.java:76-98)
      rid.resize(rid_prefix);
      rid += eid;
      out.cols[np + nk].add(rid);
      out.cols[np + nk + 1].add(eid);
      out.hash.push_back(U16Table::hash(rid.data(), rid.size()));
      out.deleted.push_back(has[V.i_del] && as_boolean(got[V.i_del], side) ? 1 : 0);
    }
  } catch (const Fail& f) {
    out.code = f.code;
    out.msg = f.msg;
    out.fail_at = r;
  } catch (const std::bad_alloc&) {
    out.code = DK_E_NOMEM;
    out.msg = "out of host memory";
    out.fail_at = r;
  }
}

// A packed column (owned by Packed)
struct FinalCol {  // uninitialised storage: the merge workers first-touch their own slices
  PodVec<uint32_t> off;
  PodVec<uint8_t> u8;
  PodVec<uint16_t> u16;
  PodVec<uint8_t> present;
};

struct Packed {
  dk_packed pub{};
  std::vector<dk_column> cols, keys;
  std::vector<FinalCol> store;  // sized once: the dk_column pointers stay valid
  std::vector<uint8_t> deleted, group;
  std::vector<uint64_t> ident;
};

// slices -> packed columns: sizes and widths first, then one parallel pass in which each
// worker copies its slice of every column into place
struct ColPlan {
  std::vector<uint64_t> ubase;  // per slice: first unit
  bool missing = false, narrow = true;
};

void merge_columns(std::vector<Slice>& sl, uint64_t n, std::vector<FinalCol>& F, std::vector<dk_column*>& out) {
  const int T = (int)sl.size(), NC = (int)F.size();
  std::vector<ColPlan> plan(NC);
  for (int c = 0; c < NC; ++c) {
    ColPlan& L = plan[c];
    L.ubase.assign(T + 1, 0);
    char16_t orv = 0;
    for (int t = 0; t < T; ++t) {
      const ColPart& P = sl[t].cols[c];
      L.ubase[t + 1] = L.ubase[t] + P.units();
      L.missing = L.missing || P.missing;
      orv |= P.orv;
    }
    if (L.ubase[T] >= (1ull << 32)) fail(DK_E_UNSUPPORTED, "a column of over 4G units in one batch");
    L.narrow = orv <= 0xFF;
    F[c].off.reset_uninit(n + 1);
    F[c].off[0] = 0;
    if (L.narrow) F[c].u8.reset_uninit(L.ubase[T] + 1);
    else F[c].u16.reset_uninit(L.ubase[T] + 1);
    if (L.missing) F[c].present.reset_uninit(n);
  }
  parallel_for(T, [&](int t) {
    const uint64_t r0 = sl[t].e0, m = sl[t].e1 - sl[t].e0;
    for (int c = 0; c < NC; ++c) {
      const ColPart& P = sl[t].cols[c];
      const ColPlan& L = plan[c];
      const uint32_t b = (uint32_t)L.ubase[t];
      uint32_t* o = F[c].off.data() + r0 + 1;
      for (uint64_t i = 0; i < m; ++i) o[i] = P.off[i + 1] + b;
      const size_t nu = P.units();
      if (L.narrow) {  // every part's units are <= 0xFF
        uint8_t* d = F[c].u8.data() + L.ubase[t];
        if (!P.wide) {
          if (nu) memcpy(d, P.u8.data(), nu);
        } else {
          const char16_t* u = P.u16.data();
          for (size_t i = 0; i < nu; ++i) d[i] = (uint8_t)u[i];
        }
        if (t == T - 1) F[c].u8[L.ubase[T]] = 0;
      } else {
        uint16_t* d = F[c].u16.data() + L.ubase[t];
        if (P.wide) {
          if (nu) memcpy(d, P.u16.data(), nu * 2);
        } else {
          const uint8_t* u = P.u8.data();
          for (size_t i = 0; i < nu; ++i) d[i] = u[i];
        }
        if (t == T - 1) F[c].u16[L.ubase[T]] = 0;
      }
      if (L.missing && m) memcpy(F[c].present.data() + r0, P.present.data(), m);
    }
  });
  for (int c = 0; c < NC; ++c) {
    out[c]->offsets = F[c].off.data();
    out[c]->units = plan[c].narrow ? (const void*)F[c].u8.data() : (const void*)F[c].u16.data();
    out[c]->width = plan[c].narrow ? 1 : 2;
    out[c]->present = plan[c].missing ? F[c].present.data() : nullptr;
  }
}

}  // namespace

extern "C" {

int dk_interner_create(dk_interner** out) {
  if (!out) return dk_fail_ingest(DK_E_INVALID, "out is NULL");
  *out = new (std::nothrow) dk_interner();
  return *out ? DK_OK : dk_fail_ingest(DK_E_NOMEM, "out of host memory");
}

void dk_interner_destroy(dk_interner* it) { delete it; }

uint64_t dk_interner_size(const dk_interner* it) { return it ? it->size() : 0; }

int dk_interner_find(const dk_interner* it, const uint16_t* units, uint64_t n, uint64_t* id) {
  if (!it || !id || (n && !units)) return dk_fail_ingest(DK_E_INVALID, "NULL argument");
  if (!it->find(reinterpret_cast<const char16_t*>(units), n, id))
    return dk_fail_ingest(DK_E_INVALID, "ID not interned");
  return DK_OK;
}

int dk_interner_intern(dk_interner* it, const dk_column* col, uint64_t n, uint64_t* out) {
  if (!it || !col || (n && (!out || !col->offsets || !col->units)))
    return dk_fail_ingest(DK_E_INVALID, "NULL argument");
  if (col->width != 1 && col->width != 2) return dk_fail_ingest(DK_E_INVALID, "width 1 or 2");
  for (uint64_t i = 0; i < n; ++i) {
    if (col->present && !col->present[i]) return dk_fail_ingest(DK_E_INVALID, "missing ID");
    if (col->offsets[i + 1] < col->offsets[i]) return dk_fail_ingest(DK_E_INVALID, "offsets not monotone");
  }
  try {
    std::u16string k;
    for (uint64_t i = 0; i < n; ++i) {
      const uint32_t a = col->offsets[i], b = col->offsets[i + 1];
      k.resize(b - a);
      for (uint32_t j = a; j < b; ++j)
        k[j - a] = col->width == 1 ? ((const uint8_t*)col->units)[j] : ((const uint16_t*)col->units)[j];
      out[i] = it->find_or_add(k.data(), k.size());
    }
  } catch (const std::bad_alloc&) {
    return dk_fail_ingest(DK_E_NOMEM, "out of host memory");
  }
  return DK_OK;
}

extern "C" void dk_clear_upper_state(void) { clear_upper(); }

int dk_pack_json(const dk_source* src, const char* json, uint64_t len, dk_interner* ids,
                 dk_packed** out) {
  if (!src || !json || !ids || !out) return dk_fail_ingest(DK_E_INVALID, "NULL argument");
  *out = nullptr;
  if (src->nprops < 0 || src->nprops > 16 || src->nkeys < 0 || src->nkeys > 8 ||
      src->ncolumns < 0 || (src->ncolumns && !src->columns) || (src->nkeys && !src->keys) ||
      !src->dataset_id || src->group_no < 0 || src->group_no > 2)
    return dk_fail_ingest(DK_E_INVALID, "bad dk_source");
  for (int c = 0; c < src->ncolumns; ++c) {
    const dk_source_column& sc = src->columns[c];
    if (!sc.name || sc.prop < -1 || sc.prop >= src->nprops + kMaxKeyOnly || sc.cleaner < DK_CLEAN_NONE ||
        sc.cleaner > DK_CLEAN_CAPITAL)
      return dk_fail_ingest(DK_E_INVALID, "bad dk_source_column");
  }
  try {
    SourceView V;
    V.src = src;
    for (int c = 0; c < src->ncolumns; ++c) V.names.emplace_back(src->columns[c].name);
    V.i_id = (int)V.names.size();
    V.i_del = V.i_id + 1;
    V.names.emplace_back("_id");
    V.names.emplace_back("_deleted");
    decode_string(src->dataset_id, src->dataset_id + strlen(src->dataset_id), V.ds);

    clear_upper();
    auto T0 = std::chrono::steady_clock::now();
    static const bool timing = getenv("DK_INGEST_TIMING") != nullptr;  // phase times to stderr
    auto lap = [&](const char* w) {
      if (!timing) return;
      const auto t1 = std::chrono::steady_clock::now();
      fprintf(stderr, "dk_pack_json %s %.2f ms\n", w, std::chrono::duration<double, std::milli>(t1 - T0).count());
      T0 = t1;
    };
    // 1. entity spans
    Split S;
    split_entities(json, len, S);
    clear_upper();
    const uint64_t n = S.n;
    lap("split");
    // 2. entity slices, parsed in parallel
    const int T = pack_threads(n, 4096);
    std::vector<Slice> sl(T);
    for (int t = 0; t < T; ++t) {
      sl[t].e0 = n * (uint64_t)t / (uint64_t)T;
      sl[t].e1 = n * (uint64_t)(t + 1) / (uint64_t)T;
    }
    parallel_for(T, [&](int t) { parse_slice(V, json, S, sl[t]); });
    lap("parse");
    for (const Slice& x : sl)  // the first failing entity, else the split's own error
      if (x.code != DK_OK) return dk_fail_ingest(x.code, x.msg.c_str());
    if (S.code != DK_OK) return dk_fail_ingest(S.code, S.msg.c_str());
    // 3. concatenated columns, interned record IDs
    Packed* P = new Packed();
    std::unique_ptr<Packed> guard(P);
    const int np = src->nprops, nk = src->nkeys;
    P->store.resize(np + nk + 2);
    P->cols.resize(np);
    P->keys.resize(nk);
    std::vector<dk_column*> dst;
    for (int p = 0; p < np; ++p) dst.push_back(&P->cols[p]);
    for (int k = 0; k < nk; ++k) dst.push_back(&P->keys[k]);
    dst.push_back(&P->pub.id);
    dst.push_back(&P->pub.entity_id);
    merge_columns(sl, n, P->store, dst);
    P->deleted.resize(n);
    for (const Slice& x : sl)
      if (!x.deleted.empty()) memcpy(P->deleted.data() + x.e0, x.deleted.data(), x.deleted.size());
    if (src->group_no) P->group.assign(n, (uint8_t)src->group_no);
    lap("merge");
    // record IDs in batch order: new ids are dense in first-appearance order
    if (ids->size() + n >= (1ull << 31)) fail(DK_E_UNSUPPORTED, "over 2^31 record IDs");
    P->ident.resize(n);
    {
      PodVec<const char16_t*> ptr;  // filled by the slices' workers (first touch in parallel)
      PodVec<uint32_t> ln;
      PodVec<uint64_t> hs;
      ptr.reset_uninit(n);
      ln.reset_uninit(n);
      hs.reset_uninit(n);
      parallel_for((int)sl.size(), [&](int t) {
        const Slice& x = sl[t];
        const ColPart& C = x.cols[np + nk];
        for (uint64_t i = 0; i < x.e1 - x.e0; ++i) {
          ptr[x.e0 + i] = C.u16.data() + C.off[i];   // the ID column is always wide
          ln[x.e0 + i] = C.off[i + 1] - C.off[i];
          hs[x.e0 + i] = x.hash[i];
        }
      });
      ids->intern_batch(n, ptr.data(), ln.data(), hs.data(), P->ident.data(), pack_threads(n, 4096));
    }
    lap("intern");
    std::vector<Slice>().swap(sl);  // the scratch goes now (timed), not at the scope's end
    S = Split();
    lap("free");
    P->pub.n = n;
    P->pub.columns = P->cols.data();
    P->pub.key_columns = P->keys.data();
    P->pub.ident = P->ident.data();
    P->pub.deleted = P->deleted.data();
    P->pub.group = src->group_no ? P->group.data() : nullptr;
    *out = &guard.release()->pub;  // pub is the first member
    return DK_OK;
  } catch (const Fail& f) {
    return dk_fail_ingest(f.code, f.msg.c_str());
  } catch (const std::bad_alloc&) {
    return dk_fail_ingest(DK_E_NOMEM, "out of host memory");
  }
}

void dk_free_packed(dk_packed* p) {
  delete reinterpret_cast<Packed*>(p);  // dk_packed is Packed's first member
}

}  // extern "C"
