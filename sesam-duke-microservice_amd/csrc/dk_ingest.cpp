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
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "dk_clean_table.h"
#include "dk_interner.h"
#include "dukehip.h"

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
  // string starting at '"': returns [a, b) of the raw content
  void str(const char** a, const char** b) {
    ++p;  // '"'
    *a = p;
    while (p < e && *p != '"') {
      if ((unsigned char)*p < 0x20) fail(DK_E_UNSUPPORTED, "JSON: control character in a string");
      if (*p == '\\') {
        ++p;
        if (p >= e) break;
      }
      ++p;
    }
    if (p >= e) fail(DK_E_UNSUPPORTED, "JSON: unterminated string");
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

bool py_isspace(uint32_t c) {  // Python str.isspace (str.split() / strip())
  return (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x20) || c == 0x85 || c == 0xA0 ||
         c == 0x1680 || (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 ||
         c == 0x202F || c == 0x205F || c == 0x3000;
}

void lowercase_normalize(std::u16string& s) {
  std::u16string out;
  out.reserve(s.size());
  bool pending = false;
  for (char16_t c : s) {
    if (c >= 0x370) fail(DK_E_UNSUPPORTED, "cleaner: character outside the native table");
    const uint16_t m = kCleanTable[c];
    if (m == 0xFFFF) fail(DK_E_UNSUPPORTED, "cleaner: character outside the native table");
    if (m == 0xFFFE) continue;  // a combining mark: removed with the accents
    const char16_t x = (char16_t)m;
    if (is_norm_ws(x)) {
      pending = true;
      continue;
    }
    if (pending && !out.empty()) out.push_back(u' ');
    pending = false;
    out.push_back(x);
  }
  s.swap(out);
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
  s = s.substr(a, b - a);
}

// ---- key functions: dukehip.records.PartsKey (code-point slicing, Python semantics) ----
std::vector<uint32_t> code_points(const std::u16string& s) {
  std::vector<uint32_t> cp;
  cp.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    const char16_t c = s[i];
    if (c >= 0xD800 && c <= 0xDBFF && i + 1 < s.size() && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
      cp.push_back(0x10000 + (((uint32_t)c - 0xD800) << 10) + (s[i + 1] - 0xDC00));
      ++i;
    } else {
      cp.push_back(c);
    }
  }
  return cp;
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

void key_part(const std::u16string* value, const dk_key_part& kp, std::u16string& out) {
  if (!value) return;  // a missing value contributes ""
  std::vector<uint32_t> cp = code_points(*value);
  if (kp.token != INT32_MIN) {  // str.split() then toks[token]
    std::vector<std::pair<size_t, size_t>> toks;
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
    cp = std::vector<uint32_t>(cp.begin() + toks[t].first, cp.begin() + toks[t].second);
  }
  int64_t a, b;
  py_slice((int64_t)cp.size(), kp.start, kp.end, &a, &b);
  for (int64_t i = a; i < b; ++i) append_cp(out, cp[i]);
}

// ---- packed output ---------------------------------------------------------------------
struct ColBuild {
  std::vector<uint32_t> off{0};
  std::u16string units;
  std::vector<uint8_t> present;
  bool any_missing = false;
  void add(const std::u16string* v) {
    if (v) units.append(*v);
    present.push_back(v ? 1 : 0);
    any_missing = any_missing || !v;
    off.push_back((uint32_t)units.size());
  }
};

}  // namespace


namespace {

struct Packed {
  dk_packed pub{};
  std::vector<dk_column> cols, keys;
  std::vector<std::vector<uint32_t>> offs;
  std::vector<std::vector<uint8_t>> units8, present;
  std::vector<std::u16string> units16;
  std::vector<uint8_t> deleted, group;
  std::vector<uint64_t> ident;
};

void finish_column(Packed& P, ColBuild& cb, dk_column& out) {
  P.offs.push_back(std::move(cb.off));
  bool narrow = true;
  for (char16_t c : cb.units)
    if (c > 0xFF) { narrow = false; break; }
  if (narrow) {
    std::vector<uint8_t> u(cb.units.size() + 1, 0);
    for (size_t i = 0; i < cb.units.size(); ++i) u[i] = (uint8_t)cb.units[i];
    P.units8.push_back(std::move(u));
    out.units = P.units8.back().data();
    out.width = 1;
  } else {
    cb.units.push_back(0);
    P.units16.push_back(std::move(cb.units));
    out.units = P.units16.back().data();
    out.width = 2;
  }
  out.offsets = P.offs.back().data();
  if (cb.any_missing) {
    P.present.push_back(std::move(cb.present));
    out.present = P.present.back().data();
  } else {
    out.present = nullptr;
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

uint64_t dk_interner_size(const dk_interner* it) { return it ? it->ids.size() : 0; }

int dk_interner_find(const dk_interner* it, const uint16_t* units, uint64_t n, uint64_t* id) {
  if (!it || !id || (n && !units)) return dk_fail_ingest(DK_E_INVALID, "NULL argument");
  const auto f = it->ids.find(std::u16string(reinterpret_cast<const char16_t*>(units), n));
  if (f == it->ids.end()) return dk_fail_ingest(DK_E_INVALID, "ID not interned");
  *id = f->second;
  return DK_OK;
}

int dk_interner_intern(dk_interner* it, const dk_column* col, uint64_t n, uint64_t* out) {
  if (!it || !col || (n && (!out || !col->offsets || !col->units)))
    return dk_fail_ingest(DK_E_INVALID, "NULL argument");
  if (col->width != 1 && col->width != 2) return dk_fail_ingest(DK_E_INVALID, "width 1 or 2");
  try {
    std::u16string k;
    for (uint64_t i = 0; i < n; ++i) {
      if (col->present && !col->present[i]) return dk_fail_ingest(DK_E_INVALID, "missing ID");
      const uint32_t a = col->offsets[i], b = col->offsets[i + 1];
      k.resize(b - a);
      for (uint32_t j = a; j < b; ++j)
        k[j - a] = col->width == 1 ? ((const uint8_t*)col->units)[j] : ((const uint16_t*)col->units)[j];
      const auto f = it->ids.find(k);
      out[i] = f != it->ids.end() ? f->second : it->add(std::move(k));
    }
  } catch (const std::bad_alloc&) {
    return dk_fail_ingest(DK_E_NOMEM, "out of host memory");
  }
  return DK_OK;
}

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
    if (!sc.name || sc.prop < -1 || sc.prop >= src->nprops || sc.cleaner < DK_CLEAN_NONE ||
        sc.cleaner > DK_CLEAN_CAPITAL)
      return dk_fail_ingest(DK_E_INVALID, "bad dk_source_column");
  }
  try {
    // the member names the data source reads
    std::vector<std::string> names;
    for (int c = 0; c < src->ncolumns; ++c) names.emplace_back(src->columns[c].name);
    const int i_id = (int)names.size(), i_del = i_id + 1;
    names.emplace_back("_id");
    names.emplace_back("_deleted");
    std::unordered_map<std::string, int> slot;
    for (int i = (int)names.size() - 1; i >= 0; --i) slot[names[i]] = i;

    std::vector<ColBuild> cb(src->nprops), kb(src->nkeys);
    ColBuild idc, eidc;
    Packed* P = new Packed();
    std::unique_ptr<Packed> guard(P);
    std::u16string ds;
    decode_string(src->dataset_id, src->dataset_id + strlen(src->dataset_id), ds);
    std::vector<Val> got(names.size()), side;
    std::vector<char> has(names.size());
    std::vector<std::u16string> pv(src->nprops);
    std::vector<char> pset(src->nprops);
    std::u16string s, key, mname;
    Reader R{json, json + len, &side};
    // the batch: an array of entity objects, or one entity (App.java:955-965)
    const bool batch = R.peek() == '[';
    if (batch) ++R.p;
    bool more = !batch || R.peek() != ']';
    if (batch && !more) ++R.p;
    uint64_t r = 0;
    while (more) {
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
          R.expect(':');
          Val v;
          R.value(v, 2);
          // member names compared after unescaping only when they hold an escape
          std::string nm(ka, kb2);
          if (nm.find('\\') != std::string::npos) {
            mname.clear();
            decode_string(ka, kb2, mname);
            nm.clear();
            for (char16_t c : mname) {
              if (c > 0x7F) { nm = "\x01"; break; }  // not one of the (ASCII) names read
              nm.push_back((char)c);
            }
          }
          const auto f = slot.find(nm);
          if (f != slot.end()) {
            got[f->second] = v;
            has[f->second] = 1;
          }
          if (R.peek() == ',') { ++R.p; continue; }
          R.expect('}');
          break;
        }
      }
      // entity id (IncrementalDataSource.java:54-61)
      std::u16string eid;
      if (has[i_id]) as_string(got[i_id], side, eid, "_id");
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
          pv[sc.prop] = s;
          pset[sc.prop] = 1;
        }
      }
      for (int p = 0; p < src->nprops; ++p) cb[p].add(pset[p] ? &pv[p] : nullptr);
      // key functions over the cleaned values
      for (int k = 0; k < src->nkeys; ++k) {
        key.clear();
        const dk_key_function& kf = src->keys[k];
        for (int i = 0; i < kf.nparts; ++i) {
          const dk_key_part& kp = kf.parts[i];
          if (kp.prop < 0 || kp.prop >= src->nprops) fail(DK_E_INVALID, "key part property out of range");
          key_part(pset[kp.prop] ? &pv[kp.prop] : nullptr, kp, key);
        }
        kb[k].add(&key);
      }
      // synthetic properties (IncrementalDataSource.java:76-98)
      std::u16string rid;
      if (src->group_no) {
        rid.push_back((char16_t)(u'0' + src->group_no));
        rid += u"__";
      }
      rid += ds;
      rid += u"__";
      rid += eid;
      idc.add(&rid);
      eidc.add(&eid);
      P->deleted.push_back(has[i_del] && as_boolean(got[i_del], side) ? 1 : 0);
      if (src->group_no) P->group.push_back((uint8_t)src->group_no);
      const auto f = ids->ids.find(rid);
      P->ident.push_back(f != ids->ids.end() ? f->second : ids->add(std::move(rid)));
      ++r;
      if (!batch) break;
      if (R.peek() == ',') {
        ++R.p;
      } else {
        R.expect(']');
        more = false;
      }
    }
    R.ws();
    if (R.p != R.e) fail(DK_E_UNSUPPORTED, "JSON: trailing characters");
    const uint64_t n = r;
    P->cols.resize(src->nprops);
    P->keys.resize(src->nkeys);
    for (int p = 0; p < src->nprops; ++p) finish_column(*P, cb[p], P->cols[p]);
    for (int k = 0; k < src->nkeys; ++k) finish_column(*P, kb[k], P->keys[k]);
    finish_column(*P, idc, P->pub.id);
    finish_column(*P, eidc, P->pub.entity_id);
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
