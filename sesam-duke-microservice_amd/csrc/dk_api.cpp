// dk_api.cpp — the C-ABI of libdukehip.so (include/dukehip.h): the device-resident record
// index (Duke Database), the batch matcher (Processor.deduplicate's match loop) and the
// result hand-back (MatchListener replay order).  Host-side C++; all per-pair work runs in
// the gfx950 kernels of dk_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "dk_interner.h"
#include "dk_internal.h"

using namespace dk;

namespace dk {  // dk_lucene.cpp (host): the StandardAnalyzer restatement
bool lucene_analyze(const uint32_t* u, size_t n, bool escape, std::vector<std::string>& out);
uint8_t lucene_norm_byte(uint32_t ntokens);
}  // namespace dk

// ----------------------------------------------------------------------------------------
// errors
// ----------------------------------------------------------------------------------------
static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

// The exception barrier of every C-ABI entry and host task: nothing C++ crosses the boundary
// (an escaping exception would std::terminate the JVM / Python host).  Out of host memory is
// DK_E_NOMEM; RAII undo logs (dk_upsert's Rollback) have run by the time it is returned.
// vzeroupper on entry (dk_ingest.cpp, host-compiled): a caller that left 256/512-bit upper
// halves dirty (numpy under Python) makes every legacy-SSE instruction of the host staging
// pay a merge dependency on Intel cores (measured 4x on the packer); AMD cores do not care.
extern "C" void dk_clear_upper_state(void);
static void clear_upper() { dk_clear_upper_state(); }

template <typename F>
static int guarded(F&& f) {
  clear_upper();
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return fail(DK_E_NOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return fail(DK_E_DEVICE, "internal error: %s", e.what());
  } catch (...) {
    return fail(DK_E_DEVICE, "internal error");
  }
}

#define HIPCHK(expr)                                                                 \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess)                                                            \
      return fail(DK_E_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                  __FILE__, __LINE__);                                               \
  } while (0)

// ----------------------------------------------------------------------------------------
// host helpers
// ----------------------------------------------------------------------------------------
// Record identity -> the row of its newest version (IncrementalLuceneDatabase's ID term).
// Dense identities (interner ids, sequence numbers) index a vector; any other u64 lives in
// a hash map.  kNoRow = absent.
struct IdentMap {
  static constexpr uint32_t kNoRow = 0xFFFFFFFFu;
  std::vector<uint32_t> dense;
  std::unordered_map<uint64_t, uint32_t> sparse;
  uint64_t dense_limit = 1u << 20;

  // identities below the limit go dense: a table of at most 8 entries per row (+ 1M)
  void plan(uint64_t rows) { dense_limit = std::min<uint64_t>(1ull << 28, 8 * rows + (1u << 20)); }
  uint32_t get(uint64_t id) const {
    if (id < dense.size() && dense[id] != kNoRow) return dense[id];
    if (sparse.empty()) return kNoRow;
    const auto it = sparse.find(id);
    return it == sparse.end() ? kNoRow : it->second;
  }
  // the dense table grown once to cover identity id (a batch's largest), as set() would
  void reserve_dense(uint64_t id) {
    if (id >= dense.size() && id < dense_limit)
      dense.resize(std::min<uint64_t>(dense_limit, std::max<uint64_t>(id + 1, 2 * dense.size())), kNoRow);
  }
  void set(uint64_t id, uint32_t row) {
    if (id >= dense.size() && id < dense_limit && row != kNoRow)
      dense.resize(std::min<uint64_t>(dense_limit, std::max<uint64_t>(id + 1, 2 * dense.size())), kNoRow);
    if (id < dense.size()) {
      dense[id] = row;
      if (!sparse.empty()) sparse.erase(id);  // an entry made while the limit was lower
    } else if (row == kNoRow) {
      sparse.erase(id);
    } else {
      sparse[id] = row;
    }
  }
  void clear() {
    dense.clear();
    sparse.clear();
  }
};

// Runs task(i) for i < n on up to n threads (inline when `parallel` is false); returns the
// first failing task's code in task order, with its dk_last_error message.
template <typename F>
static int run_tasks(int n, bool parallel, F&& task) {
  std::vector<int> rc(n, DK_OK);
  std::vector<std::string> msg(n);
  auto one = [&](int i) {
    rc[i] = guarded([&] { return task(i); });
    if (rc[i] != DK_OK) msg[i] = g_err;
  };
  if (!parallel || n <= 1) {
    for (int i = 0; i < n; ++i) {
      one(i);
      if (rc[i] != DK_OK) return rc[i];
    }
    return DK_OK;
  }
  dk_run_parts(n, one);  // `one` does not throw
  for (int i = 0; i < n; ++i)
    if (rc[i] != DK_OK) {
      g_err = msg[i];
      return rc[i];
    }
  return DK_OK;
}

// DK_HOST_TIMING=1: host phase times of dk_upsert / dk_match on stderr (diagnostics; with a
// stream, each lap first waits for it, so device work lands in the lap that queued it)
struct HostLap {
  bool on;
  const char* who;
  hipStream_t s;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  explicit HostLap(const char* w = "dk_upsert", hipStream_t st = nullptr)
      : on(getenv("DK_HOST_TIMING") != nullptr), who(w), s(st) {}
  void operator()(const char* what) {
    if (!on) return;
    if (s) (void)hipStreamSynchronize(s);
    const auto t1 = std::chrono::steady_clock::now();
    fprintf(stderr, "%s %s %.2f ms\n", who, what, std::chrono::duration<double, std::milli>(t1 - t0).count());
    t0 = t1;
  }
};

// f(lo, hi) over [0, n) in `parts` contiguous ranges on their own threads
// (an exception of any range is rethrown on the caller once every thread has joined)
template <typename F>
static void parallel_ranges(uint64_t n, int parts, F&& f) {
  if (parts <= 1 || n < 2u * (uint64_t)parts) {
    f((uint64_t)0, n);
    return;
  }
  dk_run_parts(parts, [&](int t) { f(n * t / parts, n * (t + 1) / parts); });
}

// ----------------------------------------------------------------------------------------
// device buffers
// ----------------------------------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  // grow to >= nb bytes (x1.5 headroom), preserving the first `keep` bytes
  hipError_t reserve(size_t nb, size_t keep, hipStream_t s) {
    if (nb <= bytes) return hipSuccess;
    size_t cap = std::max(nb, bytes + bytes / 2);
    cap = (cap + 255) & ~(size_t)255;
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, cap);
    if (e != hipSuccess) return e;
    if (keep && p) {
      e = hipMemcpyAsync(q, p, keep, hipMemcpyDeviceToDevice, s);
      if (e != hipSuccess) return e;
      e = hipStreamSynchronize(s);
      if (e != hipSuccess) return e;
    }
    if (p) (void)hipFree(p);
    p = q;
    bytes = cap;
    return hipSuccess;
  }
  template <typename T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

struct PinnedBuf {
  void* p = nullptr;
  size_t bytes = 0;
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
  // grow to >= nb bytes (x2 headroom), preserving the first `keep` bytes
  hipError_t reserve(size_t nb, size_t keep = 0) {
    if (nb <= bytes) return hipSuccess;
    size_t cap = std::max(nb, bytes * 2);
    void* q = nullptr;
    // portable: a group list (dk_create_multi) is filled by copies from every member device
    hipError_t e = hipHostMalloc(&q, cap, hipHostMallocPortable);
    if (e != hipSuccess) return e;
    if (keep && p) memcpy(q, p, keep);
    if (p) (void)hipHostFree(p);
    p = q;
    bytes = cap;
    return hipSuccess;
  }
  template <typename T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// ----------------------------------------------------------------------------------------
// java.lang.Double.parseDouble for NumericComparator values (host side, at index time):
// String.trim, [+-] then NaN | Infinity | hex 0x..p.. | decimal, optional [fFdD] suffix on
// the numeric forms; correctly rounded through strtod.  Returns false on
// NumberFormatException.
// ----------------------------------------------------------------------------------------
static bool is_hex(char c) {
  return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
}

static bool java_parse_double(const uint16_t* u, size_t n, double* out) {
  size_t a = 0, b = n;
  while (a < b && u[a] <= 0x20) ++a;
  while (b > a && u[b - 1] <= 0x20) --b;
  if (a == b) return false;
  {
    // fast path: [sign] digits [. digits], at most 15 digits in all -- the significand is
    // exact in a double and so is 10^k (k <= 15), so one IEEE division (or none) is the
    // correctly rounded value strtod returns (Clinger's fast path); -0 stays -0.0
    size_t i = a;
    const bool neg = u[i] == '-';
    if (u[i] == '+' || u[i] == '-') ++i;
    int64_t m = 0;
    int nd = 0, frac = 0;
    bool dot = false, ok = i < b;
    for (; i < b && ok; ++i) {
      const uint16_t ch = u[i];
      if (ch >= '0' && ch <= '9') {
        m = m * 10 + (ch - '0');
        ++nd;
        if (dot) ++frac;
      } else if (ch == '.' && !dot) {
        dot = true;
      } else {
        ok = false;
      }
    }
    if (ok && nd > 0 && nd <= 15) {
      static const double kPow10[16] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7,
                                        1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15};
      double v = (double)m;
      if (frac) v = v / kPow10[frac];
      *out = neg ? -v : v;
      return true;
    }
  }
  std::string s;
  s.reserve(b - a);
  for (size_t i = a; i < b; ++i) {
    if (u[i] > 0x7F) return false;
    s.push_back((char)u[i]);
  }
  size_t i = 0;
  bool neg = false;
  if (s[i] == '+' || s[i] == '-') neg = s[i++] == '-';
  const std::string body = s.substr(i);
  if (body == "NaN") { *out = NAN; return true; }
  if (body == "Infinity") { *out = neg ? -INFINITY : INFINITY; return true; }
  std::string num = s;
  if (body.size() > 1 && body[0] == '0' && (body[1] == 'x' || body[1] == 'X')) {
    size_t j = i + 2, digits = 0;
    while (j < s.size() && is_hex(s[j])) ++j, ++digits;
    if (j < s.size() && s[j] == '.') {
      ++j;
      while (j < s.size() && is_hex(s[j])) ++j, ++digits;
    }
    if (!digits || j >= s.size() || (s[j] != 'p' && s[j] != 'P')) return false;
    ++j;
    if (j < s.size() && (s[j] == '+' || s[j] == '-')) ++j;
    size_t ed = 0;
    while (j < s.size() && s[j] >= '0' && s[j] <= '9') ++j, ++ed;
    if (!ed) return false;
    if (j < s.size() && strchr("fFdD", s[j])) num = s.substr(0, j++);
    if (j != s.size()) return false;
  } else {
    size_t j = i, digits = 0;
    while (j < s.size() && s[j] >= '0' && s[j] <= '9') ++j, ++digits;
    if (j < s.size() && s[j] == '.') {
      ++j;
      while (j < s.size() && s[j] >= '0' && s[j] <= '9') ++j, ++digits;
    }
    if (!digits) return false;
    if (j < s.size() && (s[j] == 'e' || s[j] == 'E')) {
      ++j;
      if (j < s.size() && (s[j] == '+' || s[j] == '-')) ++j;
      size_t ed = 0;
      while (j < s.size() && s[j] >= '0' && s[j] <= '9') ++j, ++ed;
      if (!ed) return false;
    }
    if (j < s.size() && strchr("fFdD", s[j])) num = s.substr(0, j++);
    if (j != s.size()) return false;
  }
  *out = strtod(num.c_str(), nullptr);
  return true;
}

// doubles per row a property keeps in num / rnum: NumericComparator's value, or
// GeopositionComparator's (latitude, longitude)
static int num_words(int op) { return op == DK_CMP_NUMERIC ? 1 : op == DK_CMP_GEOPOSITION ? 2 : 0; }

// [Duke 1.2, recalled] utils.Geoposition.parse: the value split at its first ',', each half
// through Double.parseDouble (latitude, longitude in degrees).  Returns 1 when both parse,
// 0 when either half is not a Java double (GeopositionComparator.compare -> 0.5), -1 when the
// value has no ',' (stock Duke raises when it compares such a value).
static int parse_geoposition(const uint16_t* u, size_t n, double* lat, double* lng) {
  size_t comma = 0;
  while (comma < n && u[comma] != ',') ++comma;
  if (comma == n) return -1;
  *lat = 0.0;
  *lng = 0.0;
  if (!java_parse_double(u, comma, lat) || !java_parse_double(u + comma + 1, n - comma - 1, lng)) {
    *lat = 0.0;
    *lng = 0.0;
    return 0;
  }
  return 1;
}

// q-gram set of one value: sorted unique 64-bit codes, 16 bits per code unit
// (QGramComparator's HashSet<String> of substrings; POSITIONAL adds the index; ENDS
// [recalled] adds the start gram "^" + s[0, q-1) and the end gram s[n-q+1, n) + "$",
// i.e. it takes the grams of "^" + s + "$").
static void qgram_codes(const uint16_t* u0, int n0, int q, int tokenizer, std::vector<uint64_t>& g) {
  g.clear();
  std::vector<uint16_t> ends;
  const uint16_t* u = u0;
  int n = n0;
  if (tokenizer == DK_QGRAM_ENDS) {
    ends.resize(n0 + 2);
    ends[0] = '^';
    std::copy(u0, u0 + n0, ends.begin() + 1);
    ends[n0 + 1] = '$';
    u = ends.data();
    n = n0 + 2;
  }
  for (int ix = 0; ix + q <= n; ++ix) {
    uint64_t c = 0;
    for (int k = 0; k < q; ++k) c = (c << 16) | u[ix + k];
    if (tokenizer == DK_QGRAM_POSITIONAL) c |= (uint64_t)ix << 48;
    g.push_back(c);
  }
  std::sort(g.begin(), g.end());
  g.erase(std::unique(g.begin(), g.end()), g.end());
}

// The same for q <= 2 without POSITIONAL (codes fit 32 bits: configs[2]'s bigrams), straight
// from the column's units into `out` (sorted unique codes appended; returns their count):
// a stack array of u32 codes instead of a vector of u64, no widening copy of the value.
template <typename UT>
static int qgram_codes32(const UT* u0, int n0, int q, int tokenizer, std::vector<uint64_t>& out) {
  uint32_t stackbuf[256];
  std::vector<uint32_t> heap;
  const int n = n0 + (tokenizer == DK_QGRAM_ENDS ? 2 : 0);
  const int m = n - q + 1;
  if (m <= 0) return 0;
  uint32_t* c = m <= 256 ? stackbuf : (heap.resize(m), heap.data());
  auto unit = [&](int i) -> uint32_t {  // unit i of "^" + s + "$" (ENDS) or of s
    if (tokenizer != DK_QGRAM_ENDS) return u0[i];
    return i == 0 ? (uint32_t)'^' : i == n0 + 1 ? (uint32_t)'$' : (uint32_t)u0[i - 1];
  };
  if (q == 2) {
    if (tokenizer == DK_QGRAM_ENDS) {
      for (int ix = 0; ix < m; ++ix) c[ix] = (unit(ix) << 16) | unit(ix + 1);
    } else {
      for (int ix = 0; ix < m; ++ix) c[ix] = ((uint32_t)u0[ix] << 16) | (uint32_t)u0[ix + 1];
    }
  } else {
    for (int ix = 0; ix < m; ++ix) c[ix] = unit(ix);
  }
  std::sort(c, c + m);
  const size_t at = out.size();
  out.resize(at + m);
  uint64_t* o = out.data() + at;
  int k = 0;
  for (int i = 0; i < m; ++i)
    if (i == 0 || c[i] != c[i - 1]) o[k++] = c[i];
  out.resize(at + k);
  return k;
}

// [Duke 1.2, recalled] utils.StringUtils.split — the maximal runs of non-' ' units — as
// exact token ids (interned per property across batches), sorted with duplicates kept:
// the token comparators count, per token of the shorter list, membership in the other.
static void token_codes(const uint16_t* u, int n, std::unordered_map<std::u16string, uint64_t>& tab,
                        std::vector<uint64_t>& g) {
  g.clear();
  int i = 0;
  while (i < n) {
    while (i < n && u[i] == ' ') ++i;
    if (i >= n) break;
    const int a = i;
    while (i < n && u[i] != ' ') ++i;
    std::u16string t(reinterpret_cast<const char16_t*>(u + a), (size_t)(i - a));
    auto it = tab.find(t);
    if (it == tab.end()) it = tab.emplace(std::move(t), (uint64_t)tab.size()).first;
    g.push_back(it->second);
  }
  std::sort(g.begin(), g.end());
}

// ----------------------------------------------------------------------------------------
// context
// ----------------------------------------------------------------------------------------
struct PropState {
  dk_property cfg{};
  std::unordered_map<std::u16string, uint64_t> tokens;  // token comparators: token -> id
  int width = 0;           // arena width; 0 until the first batch
  uint64_t units_used = 0; // code units
  uint64_t grams_used = 0;
  int maxlen = 0;
  int maxgrams = 0;        // longest code list of a value
  DevBuf off, len, units, num, numok, goff, gcnt, grams;
  DevBuf gseed;            // Latin-1 bigram sets: per-row perfect-hash seed (DevProp::g16)
};

// QGram q = 2 without positions: its codes are bigrams, which a width-1 (Latin-1) arena packs
// as 16-bit keys with a per-row perfect hash (DevProp::g16)
static bool bigram_prop(const dk_property& p) {
  return p.comparator == DK_CMP_QGRAM && p.qgram_q == 2 && p.qgram_tokenizer != DK_QGRAM_POSITIONAL;
}

// One property's candidate replica (see dk_internal.h): values in replica-position order.
// The blocking tables own one set (index state); dk_compare_rows builds its own one-position
// set, so a single-pair compare never disturbs the cached tables.
struct Replica {
  int rlmax = 0;
  int rgmax = 0;
  int g16 = 0, rgrows = 0;  // bigram-key replica: u64 word rows per position
  int width = 0;
  uint64_t npos = 0;  // positions the buffers are laid out for (the transposed stride)
  DevBuf rlen, runits, rnum, rnumok, rgoff, rgcnt, rgrams;
};

// Result memory (device list + pinned host copy), pooled per ctx and handed back by
// dk_free_result, so steady-state batches allocate nothing.
struct ResultBufs {
  DevBuf d_cand, d_kind, d_prob, d_qidx, d_first;
  PinnedBuf h_first, h_cand, h_prob, h_kind;
};

struct ResultPool {
  std::mutex m;
  std::vector<std::unique_ptr<ResultBufs>> free;
  std::unique_ptr<ResultBufs> take() {
    std::lock_guard<std::mutex> g(m);
    if (free.empty()) return std::unique_ptr<ResultBufs>(new ResultBufs());
    auto b = std::move(free.back());
    free.pop_back();
    return b;
  }
  void give(std::unique_ptr<ResultBufs> b) {
    std::lock_guard<std::mutex> g(m);
    if (free.size() < 4) free.push_back(std::move(b));
  }
};

struct ResultHolder {
  dk_result r{};  // first member: dk_result* <-> ResultHolder*
  std::shared_ptr<ResultPool> pool;
  std::unique_ptr<ResultBufs> bufs;
  int device = 0;
  hipStream_t stream = nullptr;
  bool host_only = false;  // a multi-device ctx's list: host arrays only
};

struct dk_ctx {
  // dk_create_multi: a ctx of per-device member ctxs (the index replicated on each); the
  // fields below are then unused apart from schema, device (the first member's), pool, prof
  std::vector<dk_ctx*> members;
  bool broken = false;     // a replicated update failed on some members only
  dk_schema schema{};
  std::vector<PropState> P;
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // device->host copies of finished chunks
  hipEvent_t chunk_done = nullptr;
  uint64_t nrows = 0, cap = 0;
  DevBuf ident, flags, group;
  DevBuf oclass;                 // per row: Processor.compare order class (dk_schema.orders)
  std::vector<int32_t> orders;   // norders x nprops (empty: one class, the props' order)
  DevBuf keys[kMaxKeys];
  IdentMap ident_row;
  std::vector<U16Table> intern;  // key strings per key function (key style 2)
  int key_style = 0;  // 0 unset, 1 u64 keys, 2 interned strings
  // transient rows (dk_upsert_transient): the newest rows from transient_row0 on; the
  // arena fills at that point, restored by dk_drop_transient
  bool transient = false;
  uint64_t transient_row0 = 0;
  struct ArenaMark { uint64_t units, grams; int maxlen, maxgrams; };
  std::vector<ArenaMark> transient_mark;
  bool overwrite = false;  // Database.setOverwrite(true): no delete-by-ID on upsert
  std::vector<Replica> rep;       // candidate replica of the blocking tables, per property
  std::vector<Replica> pair_rep;  // dk_compare_rows' one-position replica, per property
  DevBuf pair_buf;                // dk_compare_rows' query row / rowof / staging
  dk_ctx* pair_ctx = nullptr;     // dk_compare_values: a 2-row ALLPAIRS index of the schema
  // match scratch
  DevBuf d_queries, sel, pos, usable, gkeys, skeys[kMaxSegs], rowof, sgroup[kMaxSegs];
  // The blocking tables + candidate replica are index state: built by the first dk_match
  // after the index changed (Duke's blocking database keeps its sorted key maps at index
  // time; the reference's Lucene index is likewise maintained by index/commit, not by the
  // query, IncrementalLuceneDatabase.java:146-165,498-575) and reused until the next change.
  uint64_t index_gen = 1, tables_gen = 0, tables_m = 0;
  BlockTables tables{};
  // base + delta: the base segments hold the usable rows below base_rows as
  // of the last full sort (base_m of them, each key function's segment followed by dcap
  // reserved delta positions); later index changes re-sort only the rows from base_rows on
  // and retire superseded base rows in place (base_dead: rows killed since the tables were
  // last built).  A full sort again when the delta outgrows dcap, too many base entries
  // are retired, or the replica's layout no longer fits a new value.
  bool base_ok = false;
  uint64_t base_rows = 0, base_m = 0, dcap = 0, base_retired = 0;
  std::vector<uint32_t> base_dead;
  DevBuf d_dead;
  const uint32_t* rowof_p = nullptr;  // replica position -> row (rowof, or usable in ALLPAIRS)
  uint64_t rstride = 0;               // replica positions
  DevBuf ranges, counts, qoff, wq, rident, rkeys[kMaxKeys], tmp;
  // k_score_grouped's execution order: task sort keys / values (double-buffered), chunk starts
  DevBuf task_key, task_val, task_cb, gprops, gqargs;
  DevBuf gram_tmp, gram_scratch;  // dk_upsert's device q-gram sets (dk_grams.hip)
  // symmetric dedup schedule: owner slot counts / offsets / wave map,
  // per-(key, query) bucket positions, owner results, chunk boundaries
  DevBuf ocounts, oqoff, owq, obase, okind, ores, mcounts, mqoff, mbase, mkind, mres, ecount, eincl, bidx, bval;
  DevBuf ploc, ptot, pbase;  // k_opack: first slot within the tile, tile slots, their scan
  // k_count_sym's bucket lookup for large batches (SymIndex), built once per table build
  DevBuf sx_posof, sx_hflag, sx_bstart, sx_bend, sx_bse, sx_tmp;
  uint64_t sx_gen = 0;
  DevBuf raised;           // k_score_geo: a compared GeopositionComparator value without ','
  PinnedBuf h_raised;
  PinnedBuf h_bounds;
  PinnedBuf h_pbase;  // k_opack's tile offsets, read back with the schedule's totals
  DevBuf counters;
  struct StageBufs { DevBuf bcnt, bscored, bbytes, boff, prob, cand, qidx, bexact; };
  StageBufs stage[2];                          // double-buffered per-chunk staging
  StageBufs owner_stage;  // block counters of the owner phase (it emits no entries)
  hipEvent_t count_ready[2] = {nullptr, nullptr};  // a chunk's entry count reached hs[]
  hipEvent_t compact_done[2] = {nullptr, nullptr}; // a chunk's staging set was drained
  // deferred profiling spans (Timer), resolved after dk_match's final synchronisation
  struct Span { hipEvent_t a, b; double* acc; };
  std::vector<hipEvent_t> ev_pool;
  size_t ev_next = 0;
  std::vector<Span> spans;
  PinnedBuf h_small;
  std::shared_ptr<ResultPool> pool = std::make_shared<ResultPool>();
  // caller-owned host region for DK_MATCH_HOST entries (dk_set_result_region), registered
  // with the HIP runtime so the chunk copies DMA straight into it
  struct Region {
    uint8_t* base = nullptr;
    uint64_t bytes = 0, max_queries = 0, cap = 0;
    uint64_t* first = nullptr;
    double* prob = nullptr;
    uint32_t* cand = nullptr;
    uint8_t* kind = nullptr;
  } region;
  // profiling (Processor.setPerformanceProfiling)
  int profiling = 0;  // 0 off, 1 every phase, 2 the scoring kernels only
  dk_profile prof{};
  // Lucene-compatible candidate source (dk_schema.lucene): per lookup field a term
  // dictionary; per row its query clauses (host offsets + device copy) and length norms;
  // the postings of indexed rows, appended per upsert and sorted by the first match after
  // an index change (index state, like the blocking tables)
  struct Lucene {
    bool on = false;
    std::vector<int> fields;
    int max_hits = 10;
    float min_rel = 0.9f;
    std::vector<std::unordered_map<std::string, uint32_t>> dict;
    std::vector<uint64_t> qoff{0};
    uint64_t npost = 0, nsorted = 0, max_doc = 0;
    bool unmerged = false;  // dk_lucene_set_stats(DK_LUCENE_STATS_UNMERGED)
    DevBuf pkey, ptf, qoff_d, qterm, norm, skey, stf, tkey, hits, exact;
  } luc;
};

static hipError_t grow_rows(dk_ctx* c, uint64_t need) {
  if (need <= c->cap) return hipSuccess;
  uint64_t nc = std::max<uint64_t>(need, std::max<uint64_t>(1024, c->cap * 2));
  hipStream_t s = c->stream;
  hipError_t e;
  const uint64_t n = c->nrows;
#define GROW(buf, T)                                              \
  if ((e = (buf).reserve(nc * sizeof(T), n * sizeof(T), s)) != hipSuccess) return e;
  GROW(c->ident, uint64_t);
  GROW(c->flags, uint8_t);
  GROW(c->group, uint8_t);
  GROW(c->oclass, uint8_t);
  for (int k = 0; k < c->schema.nkeys; ++k) GROW(c->keys[k], uint64_t);
  if (c->luc.on) {
    const uint64_t nf = c->luc.fields.size();
    if ((e = c->luc.norm.reserve(nc * nf, n * nf, s)) != hipSuccess) return e;
    if ((e = c->luc.qoff_d.reserve((nc + 1) * 8, (n + 1) * 8, s)) != hipSuccess) return e;
  }
  for (auto& p : c->P) {
    GROW(p.off, uint32_t);
    GROW(p.len, uint16_t);
    if (const int nw = num_words(p.cfg.comparator)) {
      if ((e = p.num.reserve(nc * 8 * nw, n * 8 * nw, s)) != hipSuccess) return e;
      GROW(p.numok, uint8_t);
    }
    if (uses_codes(p.cfg.comparator)) {
      GROW(p.goff, uint32_t);
      GROW(p.gcnt, uint16_t);
    }
    if (bigram_prop(p.cfg)) GROW(p.gseed, uint16_t);
  }
#undef GROW
  c->cap = nc;
  return hipSuccess;
}

static int validate_schema(const dk_schema* s) {
  if (!s) return fail(DK_E_INVALID, "schema is NULL");
  if (s->nprops < 0 || s->nprops > kMaxProps)
    return fail(DK_E_INVALID, "nprops %d out of range [0, %d]", s->nprops, kMaxProps);
  if (s->nprops > 0 && !s->props) return fail(DK_E_INVALID, "props is NULL");
  if (s->mode < DK_MODE_DEDUP || s->mode > DK_MODE_ALLPAIRS)
    return fail(DK_E_INVALID, "unknown mode %d", s->mode);
  if (s->lucene) {
    const dk_lucene& L = *s->lucene;
    if (s->mode == DK_MODE_ALLPAIRS)
      return fail(DK_E_INVALID, "the Lucene candidate source needs DEDUP or LINKAGE mode");
    if (s->nkeys != 0) return fail(DK_E_INVALID, "the Lucene candidate source takes no key functions");
    if (L.nlookup < 1 || L.nlookup > s->nprops || !L.lookup_prop)
      return fail(DK_E_INVALID, "nlookup %d out of range [1, %d]", L.nlookup, s->nprops);
    for (int i = 0; i < L.nlookup; ++i) {
      if (L.lookup_prop[i] < 0 || L.lookup_prop[i] >= s->nprops)
        return fail(DK_E_INVALID, "lookup property %d out of range", L.lookup_prop[i]);
      for (int j = 0; j < i; ++j)
        if (L.lookup_prop[j] == L.lookup_prop[i]) return fail(DK_E_INVALID, "lookup property repeated");
    }
    // a GeopositionComparator as the only lookup property: the reference's database searches
    // geo-spatially and raises (IncrementalLuceneDatabase.java:433-441, 460-463)
    if (L.nlookup == 1 && s->props && L.lookup_prop[0] >= 0 && L.lookup_prop[0] < s->nprops &&
        s->props[L.lookup_prop[0]].comparator == DK_CMP_GEOPOSITION)
      return fail(DK_E_UNSUPPORTED, "a GeopositionComparator as the only lookup property "
                  "(the reference's geo search raises, IncrementalLuceneDatabase.java:460-463)");
    if (L.max_hits < 1 || L.max_hits > kLuceneMaxHits)
      return fail(DK_E_UNSUPPORTED, "max_hits %d (supported 1..%d: larger values grow the search "
                  "limit adaptively, EstimateResultTracker)", L.max_hits, kLuceneMaxHits);
  } else if (s->mode != DK_MODE_ALLPAIRS && (s->nkeys < 1 || s->nkeys > kMaxKeys)) {
    return fail(DK_E_INVALID, "nkeys %d out of range [1, %d]", s->nkeys, kMaxKeys);
  }
  if (s->norders < 0 || s->norders > kMaxOrders)
    return fail(DK_E_UNSUPPORTED, "norders %d out of range [0, %d]", s->norders, kMaxOrders);
  if (s->norders > 0 && !s->orders) return fail(DK_E_INVALID, "orders is NULL");
  for (int o = 0; o < s->norders; ++o) {
    uint32_t seen = 0;
    for (int k = 0; k < s->nprops; ++k) {
      const int32_t v = s->orders[o * s->nprops + k];
      if (v < 0 || v >= s->nprops || (seen >> v) & 1u)
        return fail(DK_E_INVALID, "orders[%d] is not a permutation of the properties", o);
      seen |= 1u << v;
    }
  }
  for (int i = 0; i < s->nprops; ++i) {
    const dk_property& p = s->props[i];
    switch (p.comparator) {
      case DK_CMP_NONE:
      case DK_CMP_LEVENSHTEIN:
      case DK_CMP_JAROWINKLER:
      case DK_CMP_EXACT:
      case DK_CMP_NUMERIC:
      case DK_CMP_WEIGHTED_LEVENSHTEIN:
      case DK_CMP_DICE_TOKENS:
      case DK_CMP_JACCARD_TOKENS:
      case DK_CMP_GEOPOSITION:
        break;
      case DK_CMP_QGRAM:
        if (p.qgram_q < 1 || p.qgram_q > 4)
          return fail(DK_E_UNSUPPORTED, "property %d: QGramComparator q=%d (supported 1..4)", i,
                      p.qgram_q);
        if (p.qgram_tokenizer == DK_QGRAM_POSITIONAL && p.qgram_q > 3)
          return fail(DK_E_UNSUPPORTED, "property %d: POSITIONAL tokenizer needs q <= 3", i);
        if (p.qgram_tokenizer != DK_QGRAM_BASIC && p.qgram_tokenizer != DK_QGRAM_POSITIONAL &&
            p.qgram_tokenizer != DK_QGRAM_ENDS)
          return fail(DK_E_UNSUPPORTED, "property %d: q-gram tokenizer %d", i, p.qgram_tokenizer);
        if (p.qgram_formula < DK_QGRAM_OVERLAP || p.qgram_formula > DK_QGRAM_DICE)
          return fail(DK_E_UNSUPPORTED, "property %d: q-gram formula %d", i, p.qgram_formula);
        break;
      default:
        return fail(DK_E_UNSUPPORTED, "property %d: comparator %d has no GPU kernel", i,
                    p.comparator);
    }
  }
  return DK_OK;
}

// Public entry points: C linkage comes from the declarations in dukehip.h.

const char* dk_last_error(void) { return g_err.c_str(); }

// error hook of the host-only ingestion (dk_ingest.cpp)
extern "C" int dk_fail_ingest(int code, const char* msg) { return fail(code, "%s", msg); }

int dk_abi_version(void) { return DK_ABI_VERSION; }

static int create_impl(const dk_schema* schema, int device, dk_ctx** out) {
  if (!out) return fail(DK_E_INVALID, "out is NULL");
  *out = nullptr;
  int rc = validate_schema(schema);
  if (rc) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(DK_E_DEVICE, "no HIP device visible");
  if (device < 0 || device >= ndev)
    return fail(DK_E_INVALID, "device %d out of range (%d visible)", device, ndev);
  HIPCHK(hipSetDevice(device));
  dk_ctx* c = new (std::nothrow) dk_ctx();
  if (!c) return fail(DK_E_NOMEM, "out of host memory");
  c->schema = *schema;
  c->schema.props = nullptr;
  c->schema.lucene = nullptr;
  c->schema.orders = nullptr;
  if (schema->norders > 0)
    c->orders.assign(schema->orders, schema->orders + (size_t)schema->norders * schema->nprops);
  if (schema->lucene) {
    c->luc.on = true;
    c->luc.fields.assign(schema->lucene->lookup_prop, schema->lucene->lookup_prop + schema->lucene->nlookup);
    c->luc.max_hits = schema->lucene->max_hits;
    c->luc.min_rel = schema->lucene->min_relevance;
    c->luc.dict.resize(schema->lucene->nlookup);
  }
  c->P.resize(schema->nprops);
  for (int i = 0; i < schema->nprops; ++i) c->P[i].cfg = schema->props[i];
  if (c->schema.mode == DK_MODE_ALLPAIRS) c->schema.nkeys = 0;
  c->intern.resize(c->schema.nkeys);
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking);
  for (int b = 0; b < 2 && e == hipSuccess; ++b)
    e = hipEventCreateWithFlags(&c->count_ready[b], hipEventDisableTiming);
  for (int b = 0; b < 2 && e == hipSuccess; ++b)
    e = hipEventCreateWithFlags(&c->compact_done[b], hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->chunk_done, hipEventDisableTiming);
  if (e != hipSuccess) {
    delete c;
    return fail(DK_E_DEVICE, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  if (c->counters.reserve(4 * sizeof(uint64_t), 0, c->stream) != hipSuccess ||
      c->h_small.reserve(64) != hipSuccess || c->raised.reserve(64, 0, c->stream) != hipSuccess ||
      c->h_raised.reserve(64) != hipSuccess) {
    delete c;
    return fail(DK_E_DEVICE, "counter allocation failed");
  }
  *out = c;
  return DK_OK;
}

int dk_create(const dk_schema* schema, int device, dk_ctx** out) {
  return guarded([&] { return create_impl(schema, device, out); });
}

void dk_destroy(dk_ctx* c) {
  if (!c) return;
  if (!c->members.empty()) {
    for (dk_ctx* m : c->members) dk_destroy(m);
    delete c;
    return;
  }
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  (void)hipStreamSynchronize(c->copy_stream);
  if (c->region.base) (void)hipHostUnregister(c->region.base);
  if (c->pair_ctx) dk_destroy(c->pair_ctx);
  hipStream_t s = c->stream, cs = c->copy_stream;
  hipEvent_t ev = c->chunk_done;
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->count_ready)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->compact_done)
    if (e) (void)hipEventDestroy(e);
  delete c;
  if (ev) (void)hipEventDestroy(ev);
  if (cs) (void)hipStreamDestroy(cs);
  (void)hipStreamDestroy(s);
}

uint64_t dk_num_rows(const dk_ctx* c) {
  return c ? (c->members.empty() ? c->nrows : c->members[0]->nrows) : 0;
}

int dk_num_devices(const dk_ctx* c) { return c ? (c->members.empty() ? 1 : (int)c->members.size()) : 0; }

// IncrementalLuceneDatabase.findRecordById (:170-180): the row of the live version
int dk_row_of_ident(const dk_ctx* c, uint64_t ident, uint32_t* row) {
  if (!c || !row) return fail(DK_E_INVALID, "NULL argument");
  if (!c->members.empty()) return dk_row_of_ident(c->members[0], ident, row);
  const uint32_t r = c->ident_row.get(ident);
  if (r == IdentMap::kNoRow) return fail(DK_E_INVALID, "no indexed record with that ID");
  *row = r;
  return DK_OK;
}

int dk_set_profiling(dk_ctx* c, int on) {
  if (!c) return fail(DK_E_INVALID, "ctx is NULL");
  const int lv = on == 2 ? 2 : (on != 0 ? 1 : 0);  // 2: the scoring kernels' spans only
  c->profiling = lv;
  for (dk_ctx* m : c->members) m->profiling = lv;
  return DK_OK;
}

int dk_get_profile(const dk_ctx* c, dk_profile* out) {
  if (!c || !out) return fail(DK_E_INVALID, "NULL argument");
  *out = c->prof;
  if (!c->members.empty()) {  // counters summed, times the largest member's (they overlap)
    dk_profile t{};
    for (const dk_ctx* m : c->members) {
      const dk_profile& p = m->prof;
      t.ms_index = std::max(t.ms_index, p.ms_index);
      t.ms_generate = std::max(t.ms_generate, p.ms_generate);
      t.ms_score = std::max(t.ms_score, p.ms_score);
      t.ms_gather = std::max(t.ms_gather, p.ms_gather);
      t.ms_copy = std::max(t.ms_copy, p.ms_copy);
      t.ms_emit = std::max(t.ms_emit, p.ms_emit);
      t.score_launches += p.score_launches;
      t.pairs_scored += p.pairs_scored;
      t.pairs_generated += p.pairs_generated;
      t.score_bytes += p.score_bytes;
      t.sym_matches += p.sym_matches;
      t.sym2_matches += p.sym2_matches;
      t.pairs_exact += p.pairs_exact;
      t.full_builds += p.full_builds;
      t.delta_builds += p.delta_builds;
      t.replica_positions = std::max(t.replica_positions, p.replica_positions);
      t.gram_row_bytes = std::max(t.gram_row_bytes, p.gram_row_bytes);
    }
    t.ms_total = c->prof.ms_total;  // the multi-device dk_match's own wall time
    *out = t;
  }
  return DK_OK;
}

int dk_reset_profile(dk_ctx* c) {
  if (!c) return fail(DK_E_INVALID, "ctx is NULL");
  c->prof = dk_profile{};
  for (dk_ctx* m : c->members) m->prof = dk_profile{};
  return DK_OK;
}

// ----------------------------------------------------------------------------------------
// dk_upsert: Database.index(Record) for each record of the batch + Database.commit()
//
// Failure atomicity: a batch is validated and packed on the host first (stage_column,
// stage_key), then the device buffers are grown, and only then is anything committed —
// the ID map, the tombstones of older versions and the arenas.  A rejected batch (bad
// offsets, a value the GPU path does not hold, a bad group) leaves the index exactly as
// it was, so a caller may hand that batch to stock Duke and keep using the ctx.  This is
// Lucene's per-record delete-then-add made batch-atomic (IncrementalLuceneDatabase.java:
// 516-517, 578-590: the deletes and adds become visible together at commit, :146-165).
// ----------------------------------------------------------------------------------------
struct ColStage {
  int width = 0;                    // arena width after this batch
  bool widen = false;               // the arena goes from u8 to u16 units
  int maxlen = 0, maxgrams = 0;
  std::vector<uint32_t> off;        // relative to the arena's current fill
  std::vector<uint16_t> len;
  PodVec<uint8_t> bytes;            // the batch's units at the arena width (uninitialised:
                                    // the fill writes every byte, padding included)
  std::vector<double> num;
  std::vector<uint8_t> numok;
  std::vector<uint32_t> goff;       // relative to the code list's current fill
  std::vector<uint16_t> gcnt;
  std::vector<uint64_t> grams;
  uint64_t units = 0;               // code units appended (padded)
  // QGram sets built on the device (dk_grams.hip): per batch row its scratch run (values of
  // more than 64 raw grams), the raw-gram total (the arena's growth bound), the runs' total
  bool dev_grams = false;
  std::vector<uint64_t> soff;
  uint64_t rawtot = 0, longtot = 0;
};

// DK_DEV_GRAMS=0: QGram sets built on the host (qgram_codes) instead of the device (A/B)
static bool dev_grams_enabled() {
  const char* e = getenv("DK_DEV_GRAMS");
  return !(e && e[0] == '0');
}

static int stage_column(dk_ctx* c, int pidx, const dk_column* col, uint64_t n, ColStage& S) {
  PropState& P = c->P[pidx];
  if (!col->offsets || (n && !col->units && col->offsets[n] != col->offsets[0]))
    return fail(DK_E_INVALID, "property %d: offsets/units missing", pidx);
  if (col->width != 1 && col->width != 2)
    return fail(DK_E_INVALID, "property %d: width %d (1 or 2)", pidx, col->width);
  const int W = std::max(P.width, col->width);
  S.width = W;
  S.widen = P.width == 1 && W == 2;
  const uint64_t align = 4 / W;  // units per 4 bytes
  S.off.resize(n);
  S.len.resize(n);
  S.maxlen = P.maxlen;
  S.maxgrams = P.maxgrams;
  // values on the DP comparators are bounded by the long-value DP (query rows <= 256)
  const bool is_dp = P.cfg.comparator == DK_CMP_LEVENSHTEIN ||
                     P.cfg.comparator == DK_CMP_WEIGHTED_LEVENSHTEIN;
  const int nw = num_words(P.cfg.comparator);
  const bool is_num = nw > 0;
  const bool is_qg = uses_codes(P.cfg.comparator);
  const bool is_tok = P.cfg.comparator != DK_CMP_QGRAM;
  // pass 1: validate, lay out (4-byte aligned values)
  uint64_t cur = 0;
  int maxlen = S.maxlen;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t a = col->offsets[i], b = col->offsets[i + 1];
    if (b < a) return fail(DK_E_INVALID, "property %d: offsets not monotone at %llu", pidx,
                           (unsigned long long)i);
    const bool present = !col->present || col->present[i];
    const uint64_t L = b - a;
    if (present && L >= kMissing)
      return fail(DK_E_UNSUPPORTED, "property %d: value of %llu units (max %u)", pidx,
                  (unsigned long long)L, (unsigned)kMissing - 1);
    if (present && is_dp && L > (uint64_t)kMaxLongUnits)
      return fail(DK_E_UNSUPPORTED,
                  "property %d: (Weighted)Levenshtein value of %llu units (GPU limit %d)", pidx,
                  (unsigned long long)L, kMaxLongUnits);
    S.off[i] = (uint32_t)cur;
    S.len[i] = present ? (uint16_t)L : kMissing;
    if (!present) continue;
    maxlen = std::max<int>(maxlen, (int)L);
    cur += (L + align - 1) / align * align;
  }
  S.maxlen = maxlen;
  if (P.units_used + cur >= (1ull << 32))
    return fail(DK_E_UNSUPPORTED, "property %d: arena over 4G units", pidx);
  S.units = cur;
  // pass 2: the units at the arena width (row ranges in parallel for large batches)
  S.bytes.reset_uninit(cur * W);
  const uint8_t* u8 = (const uint8_t*)col->units;
  const uint16_t* u16 = (const uint16_t*)col->units;
  parallel_ranges(n, n >= (1u << 16) ? 4 : 1, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; ++i) {
      if (S.len[i] == kMissing) continue;
      const uint64_t a = col->offsets[i], L = S.len[i];
      const uint64_t padded = (L + align - 1) / align * align;
      uint8_t* d = S.bytes.data() + (uint64_t)S.off[i] * W;
      if (col->width == W) memcpy(d, (const uint8_t*)col->units + a * W, L * W);
      else  // u8 input into a u16 arena
        for (uint64_t k = 0; k < L; ++k) reinterpret_cast<uint16_t*>(d)[k] = u8[a + k];
      memset(d + L * W, 0, (padded - L) * W);  // zero padding to the 4-byte boundary
    }
  });
  if (!is_num && !is_qg) return DK_OK;
  if (is_qg && !is_tok && dev_grams_enabled()) {
    // the sets are built on the device from the units (commit_column); here only their
    // bounds: raw grams per value (an upper bound of its set), scratch runs of long values
    const int q = P.cfg.qgram_q, ends = P.cfg.qgram_tokenizer == DK_QGRAM_ENDS ? 2 : 0;
    S.dev_grams = true;
    S.soff.assign(n, 0);
    for (uint64_t i = 0; i < n; ++i) {
      if (S.len[i] == kMissing) continue;
      const int64_t m = std::max<int64_t>(0, (int64_t)S.len[i] + ends - q + 1);
      if (m >= (int64_t)kMissing)
        return fail(DK_E_UNSUPPORTED, "property %d: row %llu has too many q-grams", pidx,
                    (unsigned long long)i);
      S.rawtot += (uint64_t)m;
      if (m > 64) {
        S.soff[i] = S.longtot;
        S.longtot += (uint64_t)m;
      }
    }
    if (P.grams_used + S.rawtot >= (1ull << 32))
      return fail(DK_E_UNSUPPORTED, "property %d: over 4G q-gram codes", pidx);
    return DK_OK;
  }
  // numeric values / q-gram and token codes (per value, in row order).  Numeric parses and
  // q-gram sets run over row ranges on their own threads (serial staging was
  // most of a 1M-row linkage upsert); each range fills a gram buffer of its own, merged in
  // range order, so the code lists are in row order as before.  Token ids come from one
  // interner per property and stay serial.
  if (is_num) { S.num.assign(n * nw, 0.0); S.numok.assign(n, 0); }
  if (is_qg) { S.goff.assign(n, 0); S.gcnt.assign(n, 0); }
  const int parts = is_tok || n < (1u << 15) ? 1 : 8;
  std::vector<std::vector<uint64_t>> pg(parts);
  std::vector<int> pmax(parts, 0);
  std::vector<uint64_t> pbad(parts, ~0ull);  // first row of a range with too many codes
  const bool fast32 = is_qg && !is_tok && P.cfg.qgram_q <= 2 && P.cfg.qgram_tokenizer != DK_QGRAM_POSITIONAL;
  dk_run_parts(parts, [&](int t) {
    const uint64_t lo = n * t / parts, hi = n * (t + 1) / parts;
    std::vector<uint16_t> v16;
    std::vector<uint64_t> g;
    std::vector<uint64_t>& out = pg[t];
    if (fast32) {  // at most L + 1 codes per value
      uint64_t cap = 0;
      for (uint64_t i = lo; i < hi; ++i)
        if (S.len[i] != kMissing) cap += S.len[i] + 2;
      out.reserve(cap);
    }
    for (uint64_t i = lo; i < hi; ++i) {
      if (S.len[i] == kMissing) continue;
      if (fast32 && !is_num) {
        const uint64_t a = col->offsets[i], L = S.len[i];
        const uint64_t at = out.size();
        const int k = col->width == 1 ? qgram_codes32(u8 + a, (int)L, P.cfg.qgram_q, P.cfg.qgram_tokenizer, out)
                                      : qgram_codes32(u16 + a, (int)L, P.cfg.qgram_q, P.cfg.qgram_tokenizer, out);
        if (k >= (int)kMissing) {
          pbad[t] = i;
          return;
        }
        S.goff[i] = (uint32_t)at;
        S.gcnt[i] = (uint16_t)k;
        pmax[t] = std::max(pmax[t], k);
        continue;
      }
      const uint64_t a = col->offsets[i], L = S.len[i];
      v16.resize(L);
      if (col->width == 1) for (uint64_t k = 0; k < L; ++k) v16[k] = u8[a + k];
      else memcpy(v16.data(), u16 + a, L * 2);
      if (nw == 2) {
        const int r = parse_geoposition(v16.data(), L, &S.num[2 * i], &S.num[2 * i + 1]);
        // no ',': stock Duke raises when it COMPARES such a value -- kept with numok 2, and a
        // dk_match / compare that scores it fails (k_score_geo sets P.raised)
        S.numok[i] = (uint8_t)(r < 0 ? 2 : r);
      } else if (is_num) {
        double v = 0.0;
        S.numok[i] = java_parse_double(v16.data(), L, &v) ? 1 : 0;
        S.num[i] = v;
      }
      if (is_qg) {
        // token ids are interned per property; an id handed out by a batch that is then
        // rejected is merely unused (ids only need to be equal <=> tokens equal)
        if (is_tok) token_codes(v16.data(), (int)L, P.tokens, g);
        else qgram_codes(v16.data(), (int)L, P.cfg.qgram_q, P.cfg.qgram_tokenizer, g);
        if (g.size() >= kMissing) {
          pbad[t] = i;
          return;
        }
        S.goff[i] = (uint32_t)out.size();  // relative to the range's buffer until the merge
        S.gcnt[i] = (uint16_t)g.size();
        pmax[t] = std::max<int>(pmax[t], (int)g.size());
        out.insert(out.end(), g.begin(), g.end());
      }
    }
  });
  for (int t = 0; t < parts; ++t) {
    if (pbad[t] == ~0ull) continue;
    if (pbad[t] >> 63)
      return fail(DK_E_UNSUPPORTED, "property %d: row %llu: GeopositionComparator value without ',' "
                  "(Geoposition.parse raises in stock Duke)", pidx,
                  (unsigned long long)(pbad[t] & ~(1ull << 63)));
    return fail(DK_E_UNSUPPORTED, "property %d: row %llu has too many q-grams / tokens", pidx,
                (unsigned long long)pbad[t]);
  }
  if (is_qg) {
    std::vector<uint64_t> base(parts + 1, 0);
    for (int t = 0; t < parts; ++t) {
      base[t + 1] = base[t] + pg[t].size();
      S.maxgrams = std::max(S.maxgrams, pmax[t]);
    }
    if (parts == 1) {
      S.grams.swap(pg[0]);
    } else {
      S.grams.resize(base[parts]);
      dk_run_parts(parts, [&](int t) {
        const uint64_t lo = n * t / parts, hi = n * (t + 1) / parts;
        if (!pg[t].empty()) memcpy(S.grams.data() + base[t], pg[t].data(), pg[t].size() * 8);
        for (uint64_t i = lo; i < hi; ++i) S.goff[i] += (uint32_t)base[t];
      });
    }
  }
  if (P.grams_used + S.grams.size() >= (1ull << 32))
    return fail(DK_E_UNSUPPORTED, "property %d: over 4G q-gram / token codes", pidx);
  return DK_OK;
}

// Grows the property's device buffers for the staged batch (contents preserved; a failed
// allocation leaves the arena as it was).
static int reserve_column(dk_ctx* c, int pidx, const ColStage& S) {
  PropState& P = c->P[pidx];
  hipStream_t s = c->stream;
  const size_t used_b = P.units_used * S.width;
  if (S.widen) {
    // widen the arena: strings keep their unit offsets (4-byte alignment holds)
    DevBuf wide;
    const uint64_t tot = P.units_used + 512;
    HIPCHK(wide.reserve(std::max<size_t>(P.units.bytes * 2 + 1024, used_b + S.bytes.size() + 512), 0, s));
    HIPCHK(launch_widen_u8(P.units.as<uint8_t>(), wide.as<uint16_t>(), std::min<uint64_t>(tot, P.units.bytes), s));
    HIPCHK(hipStreamSynchronize(s));
    std::swap(P.units.p, wide.p);
    std::swap(P.units.bytes, wide.bytes);
    P.width = 2;  // same strings, wider units: the index content is unchanged
  }
  HIPCHK(P.units.reserve(used_b + S.bytes.size() + 512, used_b, s));
  if (S.dev_grams) {
    HIPCHK(P.grams.reserve((P.grams_used + S.rawtot + 64) * 8, P.grams_used * 8, s));
    const uint64_t n = S.len.size();
    HIPCHK(c->gram_tmp.reserve(n * 16 + 64, 0, s));   // soff, gcnt32, gpos, maxg
    HIPCHK(c->gram_scratch.reserve(S.longtot * 8 + 8, 0, s));
  } else if (!S.grams.empty() || uses_codes(P.cfg.comparator)) {
    HIPCHK(P.grams.reserve((P.grams_used + S.grams.size() + 64) * 8, P.grams_used * 8, s));
  }
  return DK_OK;
}

template <typename F>
static hipError_t with_tmp(dk_ctx* c, F&& f);

static int commit_column(dk_ctx* c, int pidx, ColStage& S, uint64_t n, uint64_t row0) {
  PropState& P = c->P[pidx];
  hipStream_t s = c->stream;
  const int W = S.width;
  P.width = W;
  for (auto& o : S.off) o += (uint32_t)P.units_used;
  for (auto& o : S.goff) o += (uint32_t)P.grams_used;
  // units arena: keep 512 bytes of zeroed tail for the kernels' fixed-width over-reads
  const size_t used_b = P.units_used * W, add_b = S.bytes.size();
  if (add_b) HIPCHK(hipMemcpyAsync(P.units.as<uint8_t>() + used_b, S.bytes.data(), add_b, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(P.units.as<uint8_t>() + used_b + add_b, 0, 512, s));
  P.units_used += S.units;
  P.maxlen = S.maxlen;
  P.maxgrams = S.maxgrams;
  HIPCHK(hipMemcpyAsync(P.off.as<uint32_t>() + row0, S.off.data(), n * 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(P.len.as<uint16_t>() + row0, S.len.data(), n * 2, hipMemcpyHostToDevice, s));
  if (!S.num.empty()) {
    const int nw = num_words(P.cfg.comparator);
    HIPCHK(hipMemcpyAsync(P.num.as<double>() + row0 * nw, S.num.data(), n * 8 * nw, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(P.numok.as<uint8_t>() + row0, S.numok.data(), n, hipMemcpyHostToDevice, s));
  }
  if (!S.gcnt.empty()) {
    HIPCHK(hipMemcpyAsync(P.goff.as<uint32_t>() + row0, S.goff.data(), n * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(P.gcnt.as<uint16_t>() + row0, S.gcnt.data(), n * 2, hipMemcpyHostToDevice, s));
    if (!S.grams.empty())
      HIPCHK(hipMemcpyAsync(P.grams.as<uint64_t>() + P.grams_used, S.grams.data(), S.grams.size() * 8,
                            hipMemcpyHostToDevice, s));
    P.grams_used += S.grams.size();
  }
  if (S.dev_grams && n) {
    // the sets on the device: count pass, scan, write pass; then the arena's fill and the
    // longest set are read back (the host needs both before the next batch / match)
    uint64_t* d_soff = c->gram_tmp.as<uint64_t>();
    uint32_t* d_cnt = reinterpret_cast<uint32_t*>(d_soff + n);
    uint32_t* d_pos = d_cnt + n;
    uint32_t* d_max = d_pos + n;
    if (S.longtot) HIPCHK(hipMemcpyAsync(d_soff, S.soff.data(), n * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(d_max, 0, 4, s));
    GramJob J{};
    J.units = P.units.p;
    J.width = W;
    J.q = P.cfg.qgram_q;
    J.tokenizer = P.cfg.qgram_tokenizer;
    J.off = P.off.as<uint32_t>();
    J.len = P.len.as<uint16_t>();
    J.row0 = row0;
    J.n = n;
    J.soff = d_soff;
    J.scratch = c->gram_scratch.as<uint64_t>();
    J.gcnt = P.gcnt.as<uint16_t>();
    J.gcnt32 = d_cnt;
    J.maxg = d_max;
    J.gpos = d_pos;
    J.gbase = (uint32_t)P.grams_used;
    J.goff = P.goff.as<uint32_t>();
    J.grams = P.grams.as<uint64_t>();
    HIPCHK(launch_qgram_sets(J, false, s));
    HIPCHK(with_tmp(c, [&](void* t, size_t& b) { return exclusive_scan_u32_dev(t, b, d_cnt, d_pos, n, s); }));
    HIPCHK(launch_qgram_sets(J, true, s));
    uint32_t* hs = c->h_small.as<uint32_t>();
    HIPCHK(hipMemcpyAsync(hs, d_pos + n - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hs + 1, d_cnt + n - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hs + 2, d_max, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    P.grams_used += (uint64_t)hs[0] + hs[1];
    P.maxgrams = std::max<int>(P.maxgrams, (int)hs[2]);
  }
  return DK_OK;
}

// Key ids of the batch for key function k (u64 keys as given, or key strings interned
// exactly).  Interning a key of a batch that is later rejected only adds an unused id.
static int stage_key(dk_ctx* c, const dk_batch* b, int style, int k, uint64_t* kv) {
  const uint64_t n = b->n;
  uint64_t* dst = kv + (uint64_t)k * n;
  if (style == 1) {
    memcpy(dst, b->keys + (uint64_t)k * n, n * 8);
    return DK_OK;
  }
  const dk_column& kc = b->key_columns[k];
  if (!kc.offsets || (kc.width != 1 && kc.width != 2) ||
      (n && !kc.units && kc.offsets[n] != kc.offsets[0]))
    return fail(DK_E_INVALID, "key function %d: bad key column", k);
  const int parts = n >= (1u << 16) ? 8 : 1;
  {  // offsets monotone (row ranges in parallel; the first failing row is reported)
    std::vector<uint64_t> bad(parts, UINT64_MAX);
    dk_run_parts(parts, [&](int t) {
      for (uint64_t i = n * t / parts; i < n * (t + 1) / parts; ++i)
        if (kc.offsets[i + 1] < kc.offsets[i]) {
          bad[t] = i;
          break;
        }
    });
    for (uint64_t i : bad)
      if (i != UINT64_MAX)
        return fail(DK_E_INVALID, "key function %d: offsets not monotone at %llu", k, (unsigned long long)i);
  }
  auto& tab = c->intern[k];
  if (tab.size() + n >= (1ull << 31)) return fail(DK_E_UNSUPPORTED, "key function %d: over 2^31 keys", k);
  // the key strings as UTF-16, their hashes, pointers and lengths (row ranges in parallel),
  // then the ordered insert into the key function's table
  const uint64_t base = n ? kc.offsets[0] : 0, tot = n ? kc.offsets[n] - base : 0;
  PodVec<char16_t> wide;  // uninitialised: filled by the range workers
  const char16_t* units = reinterpret_cast<const char16_t*>(kc.units) + (kc.width == 2 ? base : 0);
  PodVec<uint64_t> h;
  PodVec<const char16_t*> ptr;
  PodVec<uint32_t> ln;
  h.reset_uninit(n);
  ptr.reset_uninit(n);
  ln.reset_uninit(n);
  if (kc.width == 1) wide.reset_uninit(tot);
  const uint8_t* u8 = (const uint8_t*)kc.units + base;
  dk_run_parts(parts, [&](int t) {
    for (uint64_t i = n * t / parts; i < n * (t + 1) / parts; ++i) {
      const uint64_t a = kc.offsets[i] - base, e = kc.offsets[i + 1] - base;
      const char16_t* v = units + a;
      if (kc.width == 1) {
        for (uint64_t j = a; j < e; ++j) wide[j] = u8[j];
        v = wide.data() + a;
      }
      h[i] = U16Table::hash(v, e - a);
      ptr[i] = v;
      ln[i] = (uint32_t)(e - a);
    }
  });
  tab.intern_batch(n, ptr.data(), ln.data(), h.data(), dst, parts);
  return DK_OK;
}

// The Lucene source's share of a batch (IncrementalLuceneDatabase.index :505-575 and the
// query side of findCandidateMatches :459-492): per lookup field, each value analyzed as
// stored (postings + length norm; rows that enter the index only) and escaped (the row's
// query clauses, in lookup-field order).  Host only; term ids are interned into the ctx's
// dictionaries (an entry of a failed batch is harmless).
struct LuceneStage {
  std::vector<uint64_t> pkey;
  std::vector<uint32_t> ptf, qterm;
  std::vector<uint64_t> qoff;   // absolute clause offsets of rows row0 + 1 .. row0 + n
  std::vector<uint8_t> norm;    // [i * nfields + f]
};

static int stage_lucene(dk_ctx* c, const dk_batch* b, uint64_t n, uint64_t row0, bool transient,
                        LuceneStage& S) {
  auto& L = c->luc;
  const int nf = (int)L.fields.size();
  S.norm.assign(n * nf, 0);
  S.qoff.resize(n);
  std::vector<uint32_t> u;
  std::vector<std::string> toks;
  std::unordered_map<uint32_t, uint32_t> tf;
  uint64_t at = L.qoff.back();
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t nclauses = 0;
    for (int f = 0; f < nf; ++f) {
      const dk_column& col = b->columns[L.fields[f]];
      if (col.present && !col.present[i]) continue;
      const uint32_t a = col.offsets[i], e = col.offsets[i + 1];
      u.resize(e - a);
      for (uint32_t j = a; j < e; ++j)
        u[j - a] = col.width == 1 ? ((const uint8_t*)col.units)[j] : ((const uint16_t*)col.units)[j];
      auto& dict = L.dict[f];
      auto term_id = [&](const std::string& t, uint32_t* id) {
        auto it = dict.find(t);
        if (it == dict.end()) {
          if (dict.size() >= (1u << 24)) return false;
          it = dict.emplace(t, (uint32_t)dict.size()).first;
        }
        *id = ((uint32_t)f << 24) | it->second;
        return true;
      };
      if (!transient && !u.empty()) {  // index side: the value as stored ("" is skipped, :558)
        if (!lucene_analyze(u.data(), u.size(), false, toks))
          return fail(DK_E_UNSUPPORTED, "record %llu: a lookup value outside U+0000-U+00FF "
                      "(the native StandardAnalyzer covers Latin-1)", (unsigned long long)i);
        S.norm[i * nf + f] = lucene_norm_byte((uint32_t)toks.size());
        tf.clear();
        for (const auto& t : toks) {
          uint32_t id;
          if (!term_id(t, &id)) return fail(DK_E_UNSUPPORTED, "more than 2^24 terms in a lookup field");
          tf[id] += 1;
        }
        for (const auto& kv : tf) {
          S.pkey.push_back(((uint64_t)kv.first << 32) | (row0 + i));
          S.ptf.push_back(kv.second);
        }
      }
      // query side: escapeLucene, then the same analyzer (parseTokens)
      if (!lucene_analyze(u.data(), u.size(), true, toks))
        return fail(DK_E_UNSUPPORTED, "record %llu: a lookup value outside U+0000-U+00FF",
                    (unsigned long long)i);
      for (const auto& t : toks) {
        uint32_t id;
        if (!term_id(t, &id)) return fail(DK_E_UNSUPPORTED, "more than 2^24 terms in a lookup field");
        S.qterm.push_back(id);
        ++nclauses;
      }
    }
    if (nclauses > (uint64_t)kLuceneMaxClauses)
      return fail(DK_E_UNSUPPORTED, "record %llu: %llu query clauses (the GPU path holds %d)",
                  (unsigned long long)i, (unsigned long long)nclauses, kLuceneMaxClauses);
    at += nclauses;
    S.qoff[i] = at;
  }
  return DK_OK;
}

static int group_upsert(dk_ctx* g, const dk_batch* b, uint32_t* rows_out, bool transient);

static int upsert_rows(dk_ctx* c, const dk_batch* b, uint32_t* rows_out, bool transient) {
  HostLap lap;
  if (!c || !b) return fail(DK_E_INVALID, "NULL argument");
  if (!c->members.empty()) return group_upsert(c, b, rows_out, transient);
  if (!transient && c->transient)
    return fail(DK_E_STATE, "transient rows present: dk_drop_transient before indexing");
  if (b->n == 0) return DK_OK;
  if (!b->ident) return fail(DK_E_INVALID, "batch.ident is NULL");
  if (c->schema.nprops > 0 && !b->columns) return fail(DK_E_INVALID, "batch.columns is NULL");
  const uint64_t n = b->n, row0 = c->nrows;
  if (c->schema.mode == DK_MODE_LINKAGE) {
    // dukeGroupNo is 1 or 2 (IncrementalDataSource.java:80-84); a record without it makes
    // findCandidateMatches throw (IncrementalLuceneDatabase.java:469-471)
    if (!b->group) return fail(DK_E_INVALID, "LINKAGE mode needs batch.group (dukeGroupNo)");
    for (uint64_t i = 0; i < n; ++i)
      if (b->group[i] != 1 && b->group[i] != 2)
        return fail(DK_E_INVALID, "record %llu: dukeGroupNo %u (1 or 2 in LINKAGE mode)",
                    (unsigned long long)i, (unsigned)b->group[i]);
  }
  if (b->order_class) {
    const uint32_t no = c->orders.empty() ? 1u : (uint32_t)(c->orders.size() / std::max(1, c->schema.nprops));
    for (uint64_t i = 0; i < n; ++i)
      if (b->order_class[i] >= no)
        return fail(DK_E_INVALID, "record %llu: order class %u (the schema has %u)",
                    (unsigned long long)i, (unsigned)b->order_class[i], no);
  }
  const int nk = c->schema.nkeys;
  int style = 0;
  if (nk > 0) {
    style = b->keys ? 1 : (b->key_columns ? 2 : 0);
    if (!style) return fail(DK_E_INVALID, "batch has neither keys nor key_columns");
    if (c->key_style && c->key_style != style)
      return fail(DK_E_STATE, "key style changed between batches (u64 keys vs key strings)");
  }
  // rows < 2^29: K (<= 8) sorted tables of replica positions stay below the u32 sentinel
  if (row0 + n >= (1ull << 29))
    return fail(DK_E_UNSUPPORTED, "index would exceed %u rows", 1u << 29);

  // 0. the columns' structure, before any task reads them: the staging tasks run
  // concurrently, and the Lucene task reads the lookup columns that a column task is still
  // validating (a NULL or non-monotone offsets array must be DK_E_INVALID, not a crash)
  for (int p = 0; p < c->schema.nprops; ++p) {
    const dk_column& col = b->columns[p];
    if (!col.offsets || (!col.units && col.offsets[n] != col.offsets[0]))
      return fail(DK_E_INVALID, "property %d: offsets/units missing", p);
    if (col.width != 1 && col.width != 2)
      return fail(DK_E_INVALID, "property %d: width %d (1 or 2)", p, col.width);
    for (uint64_t i = 0; i < n; ++i)
      if (col.offsets[i + 1] < col.offsets[i])
        return fail(DK_E_INVALID, "property %d: offsets not monotone at %llu", p, (unsigned long long)i);
  }
  // 1. validate + pack on the host (no index state changes): one task per property, key
  // function and the Lucene source, on their own threads for large batches
  std::vector<ColStage> cols(c->schema.nprops);
  PodVec<uint64_t> kv;  // every entry written by its key function's task
  kv.reset_uninit((uint64_t)nk * n);
  LuceneStage ls;
  const int np = c->schema.nprops, ntask = np + nk + (c->luc.on ? 1 : 0);
  {
    int rc = run_tasks(ntask, n >= 8192, [&](int t) {
      const auto t0 = std::chrono::steady_clock::now();
      const int r = t < np ? stage_column(c, t, &b->columns[t], n, cols[t])
                    : t < np + nk ? stage_key(c, b, style, t - np, kv.data())
                                  : stage_lucene(c, b, n, row0, transient, ls);
      if (lap.on)
        fprintf(stderr, "dk_upsert   task %s %d %.2f ms\n", t < np ? "column" : t < np + nk ? "key" : "lucene",
                t < np ? t : t - np,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
      return r;
    });
    if (rc) return rc;
  }
  lap("stage");
  // identity + tombstones: delete-by-ID then add (IncrementalLuceneDatabase.java:516-517;
  // skipped with overwrite, :515); transient rows are neither alive (never candidates) nor
  // entered in the ID map.  The ID map is updated here with an undo log, rolled back if
  // anything below fails before the commit.
  for (uint64_t i = 0; i < n; ++i)
    if (b->ident[i] == kDeadIdent)
      return fail(DK_E_INVALID, "record %llu: identity 0x%llx is reserved", (unsigned long long)i,
                  (unsigned long long)kDeadIdent);
  std::vector<uint8_t> flags(n, 0);
  std::vector<uint32_t> dead;
  std::vector<std::pair<uint64_t, uint32_t>> undo;
  if (!transient && !c->overwrite) undo.reserve(n);  // no regrowth copies (10M records: 160 MB)
  c->ident_row.plan(row0 + n);
  IdentMap& IM = c->ident_row;
  bool par = false;  // the batch's identities resolved on parallel ranges (below)
  if (!transient && !c->overwrite) {  // the dense ID table grown once, not doubled in the loop
    uint64_t mx = 0;
    for (uint64_t i = 0; i < n; ++i) mx = std::max(mx, b->ident[i]);
    IM.reserve_dense(mx);
    par = n >= (1u << 16) && IM.sparse.empty() && mx < IM.dense.size();
  }
  if (par) {
    // Every identity dense and the sparse map empty: (1) each identity's row before the
    // batch, (2) the batch's rows written, (3) a repeated identity (some copy's row lost) ->
    // phase 2 undone and the serial loop below; otherwise flags, tombstones and the undo
    // log exactly as the serial loop gives them (no copy supersedes another in the batch).
    constexpr int kParts = 8;
    PodVec<uint32_t> oldv;
    oldv.reset_uninit(n);
    uint32_t* dn = IM.dense.data();
    auto ranges = [&](auto&& f) {
      dk_run_parts(kParts, [&](int t) { f(t, n * (uint64_t)t / kParts, n * (uint64_t)(t + 1) / kParts); });
    };
    ranges([&](int, uint64_t lo, uint64_t hi) {
      for (uint64_t i = lo; i < hi; ++i) oldv[i] = dn[b->ident[i]];
    });
    // every allocation before the first write (a std::bad_alloc leaves the map as it was)
    std::vector<std::vector<uint32_t>> pdead(kParts);
    for (int t = 0; t < kParts; ++t) pdead[t].reserve(n * (uint64_t)(t + 1) / kParts - n * (uint64_t)t / kParts);
    dead.reserve(n);
    // phases 2-4 start threads (dk_run_parts may allocate): a throw there restores every
    // identity's old row serially (no allocation; copies of one identity read the same old
    // row) before it leaves, so the map is as it was
    try {
      ranges([&](int, uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi; ++i) __atomic_store_n(&dn[b->ident[i]], (uint32_t)(row0 + i), __ATOMIC_RELAXED);
      });
      std::atomic<bool> dup{false};
      ranges([&](int, uint64_t lo, uint64_t hi) {
        bool d = false;
        for (uint64_t i = lo; i < hi && !d; ++i) d = __atomic_load_n(&dn[b->ident[i]], __ATOMIC_RELAXED) != row0 + i;
        if (d) dup.store(true);
      });
      if (dup.load()) {
        for (uint64_t i = 0; i < n; ++i) dn[b->ident[i]] = oldv[i];  // every copy read the same old row
        par = false;
      } else {
        undo.resize(n);  // reserved above: no allocation
        ranges([&](int t, uint64_t lo, uint64_t hi) {
          for (uint64_t i = lo; i < hi; ++i) {
            flags[i] = kAlive | kIndexed | ((b->deleted && b->deleted[i]) ? kDeleted : 0);
            const uint32_t old = oldv[i];
            if (old != IdentMap::kNoRow) pdead[t].push_back(old);  // a row before the batch
            undo[i] = {b->ident[i], old};
          }
        });
        for (const auto& d : pdead) dead.insert(dead.end(), d.begin(), d.end());
      }
    } catch (...) {
      for (uint64_t i = 0; i < n; ++i) dn[b->ident[i]] = oldv[i];
      throw;
    }
  }
  for (uint64_t i = 0; i < n && !transient && !par; ++i) {
    flags[i] = kAlive | kIndexed | ((b->deleted && b->deleted[i]) ? kDeleted : 0);
    if (c->overwrite) continue;
    const uint32_t old = c->ident_row.get(b->ident[i]);
    if (old != IdentMap::kNoRow) {
      if (old >= row0) flags[old - row0] &= (uint8_t)~kAlive;  // an older copy in this batch
      else dead.push_back(old);
    }
    undo.emplace_back(b->ident[i], old);
    c->ident_row.set(b->ident[i], (uint32_t)(row0 + i));
  }
  struct Mark {
    uint64_t units, grams;
    int maxlen, maxgrams, width;
  };
  struct Rollback {
    dk_ctx* c;
    std::vector<std::pair<uint64_t, uint32_t>>* undo;
    std::vector<Mark> marks;  // per property, taken before the commit
    bool armed = true;
    ~Rollback() {
      if (!armed) return;
      for (auto it = undo->rbegin(); it != undo->rend(); ++it) c->ident_row.set(it->first, it->second);
      for (size_t p = 0; p < marks.size(); ++p) {
        c->P[p].units_used = marks[p].units;
        c->P[p].grams_used = marks[p].grams;
        c->P[p].maxlen = marks[p].maxlen;
        c->P[p].maxgrams = marks[p].maxgrams;
        c->P[p].width = marks[p].width;
      }
    }
  } rollback{c, &undo, {}};

  lap("ident");
  // 2. device space (contents preserved; nothing logical changes on failure)
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  HIPCHK(grow_rows(c, row0 + n));
  for (int p = 0; p < c->schema.nprops; ++p) {
    int rc = reserve_column(c, p, cols[p]);
    if (rc) return rc;
  }
  DevBuf d_dead;
  if (!dead.empty()) HIPCHK(d_dead.reserve(dead.size() * 4, 0, s));
  auto& L = c->luc;
  if (L.on) {
    const uint64_t np = L.npost + ls.pkey.size(), nqt = L.qoff.back();
    HIPCHK(L.pkey.reserve(np * 8 + 8, L.npost * 8, s));
    HIPCHK(L.ptf.reserve(np * 4 + 4, L.npost * 4, s));
    HIPCHK(L.qterm.reserve((nqt + ls.qterm.size()) * 4 + 4, nqt * 4, s));
  }

  lap("reserve");
  // 3. commit
  c->index_gen++;
  if (transient && !c->transient) {
    c->transient_row0 = row0;
    c->transient_mark.clear();
    for (auto& p : c->P) c->transient_mark.push_back({p.units_used, p.grams_used, p.maxlen, p.maxgrams});
  }
  HIPCHK(hipMemcpyAsync(c->ident.as<uint64_t>() + row0, b->ident, n * 8, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(c->flags.as<uint8_t>() + row0, flags.data(), n, hipMemcpyHostToDevice, s));
  if (b->group)
    HIPCHK(hipMemcpyAsync(c->group.as<uint8_t>() + row0, b->group, n, hipMemcpyHostToDevice, s));
  else
    HIPCHK(hipMemsetAsync(c->group.as<uint8_t>() + row0, 0, n, s));
  if (b->order_class)
    HIPCHK(hipMemcpyAsync(c->oclass.as<uint8_t>() + row0, b->order_class, n, hipMemcpyHostToDevice, s));
  else
    HIPCHK(hipMemsetAsync(c->oclass.as<uint8_t>() + row0, 0, n, s));
  // the arena fill marks are restored if a device step below fails (Rollback)
  for (auto& p : c->P) rollback.marks.push_back({p.units_used, p.grams_used, p.maxlen, p.maxgrams, p.width});
  for (int p = 0; p < c->schema.nprops; ++p) {
    int rc = commit_column(c, p, cols[p], n, row0);
    if (rc) return rc;
    // a Latin-1 bigram property: the new rows' perfect-hash seeds (once the arena is wide,
    // or a set outgrows the replica, bigram keys are never used again, and neither are
    // seeds: both only grow until a rollback, which drops these rows too)
    PropState& P = c->P[p];
    if (bigram_prop(P.cfg) && P.width == 1 && P.maxgrams <= kMaxReplicaGrams)
      HIPCHK(launch_gram_seed(P.grams.as<uint64_t>(), P.goff.as<uint32_t>(), P.gcnt.as<uint16_t>(),
                              P.len.as<uint16_t>(), row0, n, P.gseed.as<uint16_t>(), s));
  }
  for (int k = 0; k < nk; ++k)
    HIPCHK(hipMemcpyAsync(c->keys[k].as<uint64_t>() + row0, kv.data() + (uint64_t)k * n, n * 8,
                          hipMemcpyHostToDevice, s));
  if (L.on) {
    const uint64_t nf = L.fields.size(), nqt = L.qoff.back();
    if (!ls.pkey.empty()) {
      HIPCHK(hipMemcpyAsync(L.pkey.as<uint64_t>() + L.npost, ls.pkey.data(), ls.pkey.size() * 8,
                            hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(L.ptf.as<uint32_t>() + L.npost, ls.ptf.data(), ls.ptf.size() * 4,
                            hipMemcpyHostToDevice, s));
    }
    if (!ls.qterm.empty())
      HIPCHK(hipMemcpyAsync(L.qterm.as<uint32_t>() + nqt, ls.qterm.data(), ls.qterm.size() * 4,
                            hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(L.norm.as<uint8_t>() + row0 * nf, ls.norm.data(), n * nf,
                          hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(L.qoff_d.as<uint64_t>() + row0, &L.qoff[row0], 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(L.qoff_d.as<uint64_t>() + row0 + 1, ls.qoff.data(), n * 8,
                          hipMemcpyHostToDevice, s));
  }
  // last device step: the superseded versions stop being alive (their identities already
  // map to the new rows); nothing after it can fail but the synchronisation itself
  if (!dead.empty()) {
    HIPCHK(hipMemcpyAsync(d_dead.p, dead.data(), dead.size() * 4, hipMemcpyHostToDevice, s));
    HIPCHK(launch_clear_flag(c->flags.as<uint8_t>(), d_dead.as<uint32_t>(), dead.size(), kAlive, s));
  }
  HIPCHK(hipStreamSynchronize(s));  // host staging goes out of scope
  lap("copy");
  if (L.on) {
    L.npost += ls.pkey.size();
    L.qoff.insert(L.qoff.end(), ls.qoff.begin(), ls.qoff.end());
  }
  rollback.armed = false;
  for (uint32_t r : dead)
    if (c->base_ok && r < c->base_rows) c->base_dead.push_back(r);
  if (nk > 0) c->key_style = style;
  c->nrows += n;
  c->index_gen++;
  if (transient) c->transient = true;
  if (rows_out)
    for (uint64_t i = 0; i < n; ++i) rows_out[i] = (uint32_t)(row0 + i);
  return DK_OK;
}

int dk_upsert(dk_ctx* c, const dk_batch* b, uint32_t* rows_out) {
  return guarded([&] { return upsert_rows(c, b, rows_out, false); });
}

// IncrementalLuceneDatabase.setIndexingIsDisabled(true) (:95-96, :498-512) around the
// httptransform batch (App.java:1130-1132, 1174-1175): the batch is matched against the
// index without entering it.
int dk_upsert_transient(dk_ctx* c, const dk_batch* b, uint32_t* rows_out) {
  return guarded([&] { return upsert_rows(c, b, rows_out, true); });
}

static int group_each(dk_ctx* c, int (*f)(dk_ctx*, void*), void* arg);
static int drop_transient_impl(dk_ctx* c);
static int drop_transient_member(dk_ctx* m, void*) { return drop_transient_impl(m); }

static int drop_transient_impl(dk_ctx* c) {
  if (!c) return fail(DK_E_INVALID, "NULL argument");
  if (!c->members.empty()) return group_each(c, drop_transient_member, nullptr);
  if (!c->transient) return DK_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->nrows = c->transient_row0;
  c->index_gen++;
  if (c->luc.on) c->luc.qoff.resize(c->nrows + 1);  // transient rows add no postings
  for (size_t p = 0; p < c->P.size(); ++p) {
    const auto& m = c->transient_mark[p];
    c->P[p].units_used = m.units;
    c->P[p].grams_used = m.grams;
    c->P[p].maxlen = m.maxlen;
    c->P[p].maxgrams = m.maxgrams;
  }
  c->transient = false;
  return DK_OK;
}

int dk_drop_transient(dk_ctx* c) {
  return guarded([&] { return drop_transient_impl(c); });
}

// Collection statistics of the Lucene source (include/dukehip.h dk_lucene_set_stats): every
// upsert deletes the ID's older version and adds the new one (IncrementalLuceneDatabase.java:
// 516-517, 578-590); Lucene 4 keeps a deleted document in maxDoc and docFreq until a merge of
// its segment reclaims it, and the reference never forces one (commit, :146-165).
static int lucene_stats_member(dk_ctx* m, void* a) {
  if (!m->luc.on) return fail(DK_E_STATE, "the ctx has no Lucene candidate source");
  m->luc.unmerged = *static_cast<int*>(a) == DK_LUCENE_STATS_UNMERGED;
  m->index_gen++;  // the statistics are index state
  return DK_OK;
}

static int lucene_merge_member(dk_ctx* m, void*) {
  if (!m->luc.on) return fail(DK_E_STATE, "the ctx has no Lucene candidate source");
  HIPCHK(hipSetDevice(m->device));
  HIPCHK(launch_lucene_merge(m->flags.as<uint8_t>(), m->nrows, m->stream));
  HIPCHK(hipStreamSynchronize(m->stream));
  m->index_gen++;
  return DK_OK;
}

int dk_lucene_set_stats(dk_ctx* c, int mode) {
  return guarded([&] {
    if (!c) return fail(DK_E_INVALID, "ctx is NULL");
    if (mode != DK_LUCENE_STATS_MERGED && mode != DK_LUCENE_STATS_UNMERGED)
      return fail(DK_E_INVALID, "unknown statistics mode %d", mode);
    return c->members.empty() ? lucene_stats_member(c, &mode) : group_each(c, lucene_stats_member, &mode);
  });
}

int dk_lucene_merge(dk_ctx* c) {
  return guarded([&] {
    if (!c) return fail(DK_E_INVALID, "ctx is NULL");
    return c->members.empty() ? lucene_merge_member(c, nullptr) : group_each(c, lucene_merge_member, nullptr);
  });
}

// ----------------------------------------------------------------------------------------
// dk_match: Processor.deduplicate's match loop over the given query rows
// ----------------------------------------------------------------------------------------
namespace {
// Profiling spans (dk_set_profiling): events recorded around stream work and resolved
// after dk_match's final synchronisation, so profiling never stalls the host pipeline.
struct Timer {
  dk_ctx* c;
  double* acc;
  hipStream_t s;
  hipEvent_t a = nullptr;
  Timer(dk_ctx* ctx, double* target, hipStream_t st);
  void stop();
  ~Timer() { stop(); }
};

static hipEvent_t pooled_event(dk_ctx* c) {
  if (c->ev_next == c->ev_pool.size()) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    c->ev_pool.push_back(e);
  }
  return c->ev_pool[c->ev_next++];
}

Timer::Timer(dk_ctx* ctx, double* target, hipStream_t st) : c(ctx), acc(target), s(st) {
  // level 2: only the scoring kernels' launches (each span's two events cost the stream a
  // few microseconds between dependent kernels)
  if (!c->profiling || (c->profiling == 2 && target != &c->prof.ms_score)) return;
  a = pooled_event(c);
  if (a) (void)hipEventRecord(a, s);
}

void Timer::stop() {
  if (!a) return;
  hipEvent_t b = pooled_event(c);
  if (b && hipEventRecord(b, s) == hipSuccess) c->spans.push_back(dk_ctx::Span{a, b, acc});
  a = nullptr;
}

// every span's events have completed (called after the final stream synchronisation)
static void resolve_spans(dk_ctx* c) {
  for (const auto& sp : c->spans) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, sp.a, sp.b) == hipSuccess) *sp.acc += ms;
  }
  c->spans.clear();
  c->ev_next = 0;
}

uint64_t chunk_slots() {
  const char* e = getenv("DK_CHUNK_SLOTS");
  uint64_t v = e ? strtoull(e, nullptr, 10) : 0;
  return v ? v : (1ull << 26);
}
}  // namespace

// Score parameters over a candidate replica set (`rep`, one per property) whose position g
// holds row rowof[g], npos positions.
static ScoreParams make_params(const dk_ctx* c, const std::vector<Replica>& rep,
                               const uint32_t* rowof, uint64_t npos) {
  ScoreParams P{};
  P.nprops = c->schema.nprops;
  P.mode = c->schema.mode;
  P.threshold = c->schema.threshold;
  P.maybe = c->schema.maybe_threshold;
  P.ident = c->ident.as<uint64_t>();
  P.rowof = rowof;
  P.rstride = npos;
  P.lev_rows = 0;
  P.long_rows = 0;
  P.raw_prop = -1;
  P.has_dp = 0;
  P.has_geo = 0;
  P.norders = c->orders.empty() ? 1 : (int32_t)(c->orders.size() / std::max(1, P.nprops));
  for (int o = 0; o < kMaxOrders; ++o) {
    P.order[o] = 0;
    if (o >= P.norders) continue;
    for (int k = 0; k < P.nprops; ++k)
      P.order[o] |= (uint64_t)(c->orders.empty() ? k : c->orders[(size_t)o * P.nprops + k]) << (4 * k);
  }
  P.oclass = c->oclass.as<uint8_t>();
  P.raised = c->raised.as<uint32_t>();
  for (const auto& S : c->P) {
    const int op = S.cfg.comparator;
    if (op == DK_CMP_LEVENSHTEIN || op == DK_CMP_JAROWINKLER || op == DK_CMP_WEIGHTED_LEVENSHTEIN) P.has_dp = 1;
    if (op == DK_CMP_GEOPOSITION) P.has_geo = 1;
    if (op == DK_CMP_QGRAM || op == DK_CMP_DICE_TOKENS || op == DK_CMP_JACCARD_TOKENS) P.has_grams = 1;
    if (S.cfg.comparator == DK_CMP_LEVENSHTEIN) {
      P.lev_rows = std::max(P.lev_rows, std::min(S.maxlen, kMaxUnits));
      if (S.maxlen > kMaxUnits) P.long_rows = std::max(P.long_rows, S.maxlen);
    }
    if (S.cfg.comparator == DK_CMP_WEIGHTED_LEVENSHTEIN)
      P.long_rows = std::max(P.long_rows, std::max(S.maxlen, 1));
  }
  for (int i = 0; i < P.nprops; ++i) {
    const PropState& S = c->P[i];
    const Replica& R = rep[i];
    DevProp& D = P.props[i];
    D.op = S.cfg.comparator;
    D.width = S.width ? S.width : 1;
    D.q = S.cfg.qgram_q;
    D.formula = S.cfg.qgram_formula;
    D.tokenizer = S.cfg.qgram_tokenizer;
    D.low = S.cfg.low;
    D.high = S.cfg.high;
    D.min_ratio = S.cfg.min_ratio;
    D.off = S.off.as<uint32_t>();
    D.len = S.len.as<uint16_t>();
    D.units = S.units.p;
    D.num = S.num.as<double>();
    D.numok = S.numok.as<uint8_t>();
    D.goff = S.goff.as<uint32_t>();
    D.gcnt = S.gcnt.as<uint16_t>();
    D.grams = S.grams.as<uint64_t>();
    D.rlmax = R.rlmax;
    D.rlen = R.rlen.as<uint16_t>();
    D.runits = R.runits.p;
    D.rnum = R.rnum.as<double>();
    D.rnumok = R.rnumok.as<uint8_t>();
    D.rgoff = R.rgoff.as<uint32_t>();
    D.rgcnt = R.rgcnt.as<uint16_t>();
    D.rgrams = R.rgrams.p;
    D.rgmax = R.rgmax;
    D.rg32 = 16 * S.cfg.qgram_q + (S.cfg.qgram_tokenizer == DK_QGRAM_POSITIONAL ? 16 : 0) <= 32;
    D.g16 = R.g16;
    D.rgrows = R.rgrows;
    D.gseed = S.gseed.as<uint16_t>();
  }
  return P;
}

// Candidate replica: every property's candidate-side values in replica order, units
// transposed ([unit][position]) for values of at most kMaxReplicaUnits units.  The layout
// (units / codes per value, width) follows the index's current longest values.
struct ReplicaShape { int rlmax, rgmax, width, rgw, rgrows; };

static ReplicaShape replica_shape(const PropState& S) {
  const int op = S.cfg.comparator;
  const bool strcmp_ = op == DK_CMP_LEVENSHTEIN || op == DK_CMP_JAROWINKLER ||
                       op == DK_CMP_EXACT || uses_codes(op) || op == DK_CMP_WEIGHTED_LEVENSHTEIN;
  ReplicaShape sh{};
  sh.width = S.width ? S.width : 1;
  sh.rlmax = strcmp_ && S.maxlen <= kMaxReplicaUnits ? ((std::max(S.maxlen, 1) + 3) & ~3) : 0;
  sh.rgmax = op == DK_CMP_QGRAM && S.maxgrams <= kMaxReplicaGrams ? std::max(S.maxgrams, 1) : 0;
  // codes pack 16 bits per unit (+16 for the POSITIONAL index): q <= 2 fits in a u32
  const int gram_bits = 16 * S.cfg.qgram_q + (S.cfg.qgram_tokenizer == DK_QGRAM_POSITIONAL ? 16 : 0);
  sh.rgw = gram_bits <= 32 ? 4 : 8;
  // Latin-1 bigrams: 16-bit keys, four per u64 word, an even number of word rows (k_score
  // reads two word rows per step)
  if (sh.rgmax && bigram_prop(S.cfg) && sh.width == 1) {
    sh.rgw = 2;
    sh.rgrows = std::max(2, ((sh.rgmax + 3) / 4 + 1) & ~1);
  }
  return sh;
}

// the replica can take values of the current index (a delta build keeps its layout)
static bool replica_fits(const dk_ctx* c, const std::vector<Replica>& rep) {
  if (rep.size() != c->P.size()) return false;
  for (size_t i = 0; i < c->P.size(); ++i) {
    const ReplicaShape sh = replica_shape(c->P[i]);
    if (sh.rlmax != rep[i].rlmax || sh.rgmax != rep[i].rgmax || sh.width != rep[i].width ||
        sh.rgrows != rep[i].rgrows || (sh.rgw == 2) != (rep[i].g16 != 0))
      return false;
  }
  return true;
}

static int layout_replica(dk_ctx* c, std::vector<Replica>& rep, uint64_t npos) {
  hipStream_t s = c->stream;
  rep.resize(c->P.size());
  for (size_t i = 0; i < c->P.size(); ++i) {
    const PropState& S = c->P[i];
    Replica& R = rep[i];
    const int op = S.cfg.comparator;
    const ReplicaShape sh = replica_shape(S);
    R.rlmax = sh.rlmax;
    R.rgmax = sh.rgmax;
    R.width = sh.width;
    R.g16 = sh.rgw == 2;
    R.rgrows = sh.rgrows;
    R.npos = npos;
    HIPCHK(R.rlen.reserve(npos * 2 + 8, 0, s));
    if (R.rlmax) HIPCHK(R.runits.reserve(npos * (uint64_t)R.rlmax * sh.width + 64, 0, s));
    if (const int nw = num_words(op)) {
      HIPCHK(R.rnum.reserve(npos * 8 * nw + 16, 0, s));
      HIPCHK(R.rnumok.reserve(npos + 8, 0, s));
    }
    if (uses_codes(op)) {
      HIPCHK(R.rgoff.reserve(npos * 4 + 8, 0, s));
      HIPCHK(R.rgcnt.reserve(npos * 2 + 8, 0, s));
    }
    if (R.rgmax)
      HIPCHK(R.rgrams.reserve(npos * (R.g16 ? (uint64_t)R.rgrows * 8 : (uint64_t)R.rgmax * sh.rgw) + 64, 0, s));
  }
  return DK_OK;
}

// positions [pos0, pos0 + n) <- rows rowof[pos0 ...]
static int fill_replica(dk_ctx* c, std::vector<Replica>& rep, const uint32_t* rowof, uint64_t pos0,
                        uint64_t n) {
  hipStream_t s = c->stream;
  for (size_t i = 0; i < c->P.size(); ++i) {
    const PropState& S = c->P[i];
    Replica& R = rep[i];
    const int op = S.cfg.comparator;
    ReplicaJob J{};
    J.width = R.width;
    J.rlmax = R.rlmax;
    J.has_num = num_words(op);
    J.has_qgram = uses_codes(op);
    J.stride = R.npos;
    J.off = S.off.as<uint32_t>();
    J.len = S.len.as<uint16_t>();
    J.units = S.units.p;
    J.num = S.num.as<double>();
    J.numok = S.numok.as<uint8_t>();
    J.goff = S.goff.as<uint32_t>();
    J.gcnt = S.gcnt.as<uint16_t>();
    J.rlen = R.rlen.as<uint16_t>();
    J.runits = R.runits.p;
    J.rnum = R.rnum.as<double>();
    J.rnumok = R.rnumok.as<uint8_t>();
    J.rgoff = R.rgoff.as<uint32_t>();
    J.rgcnt = R.rgcnt.as<uint16_t>();
    J.rgmax = R.rgmax;
    J.rg32 = replica_shape(S).rgw == 4;
    J.g16 = R.g16;
    J.rgrows = R.rgrows;
    J.grams = S.grams.as<uint64_t>();
    J.rgrams = R.rgrams.p;
    HIPCHK(launch_replicate(J, rowof, pos0, n, s));
  }
  return DK_OK;
}

static int build_replica(dk_ctx* c, std::vector<Replica>& rep, const uint32_t* rowof, uint64_t npos) {
  int rc = layout_replica(c, rep, npos);
  return rc ? rc : fill_replica(c, rep, rowof, 0, npos);
}

template <typename F>
static hipError_t with_tmp(dk_ctx* c, F&& f) {
  size_t bytes = 0;
  hipError_t e = f(nullptr, bytes);
  if (e != hipSuccess) return e;
  e = c->tmp.reserve(bytes + 16, 0, c->stream);
  if (e != hipSuccess) return e;
  return f(c->tmp.p, bytes);
}

// usable rows among [row0, row1): alive && !deleted, ordered by (group, row) in LINKAGE,
// row otherwise, into c->usable
static int build_usable(dk_ctx* c, uint64_t row0, uint64_t row1, uint64_t* m_out) {
  hipStream_t s = c->stream;
  const uint64_t N = row1 - row0;
  HIPCHK(c->sel.reserve(N * 4 + 4, 0, s));
  HIPCHK(c->pos.reserve(N * 4 + 4, 0, s));
  HIPCHK(c->usable.reserve(N * 4 + 4, 0, s));
  const bool link = c->schema.mode == DK_MODE_LINKAGE;
  uint64_t m = 0;
  for (int pass = 0; pass < (link ? 2 : 1) && N; ++pass) {
    HIPCHK(launch_select_rows(c->flags.as<uint8_t>(), c->group.as<uint8_t>(), row0, N,
                              link ? pass + 1 : 0, c->sel.as<uint32_t>(), s));
    HIPCHK(with_tmp(c, [&](void* t, size_t& b) {
      return exclusive_scan_u32(t, b, c->sel.as<uint32_t>(), c->pos.as<uint32_t>(), N, s);
    }));
    HIPCHK(launch_scatter_rows(c->sel.as<uint32_t>(), c->pos.as<uint32_t>(), row0, N, (uint32_t)m,
                               c->usable.as<uint32_t>(), s));
    uint32_t last_pos = 0, last_sel = 0;
    HIPCHK(hipMemcpyAsync(&last_pos, c->pos.as<uint32_t>() + N - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&last_sel, c->sel.as<uint32_t>() + N - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    m += (uint64_t)last_pos + last_sel;
  }
  *m_out = m;
  return DK_OK;
}

// Sort the m usable rows (c->usable) of key function k by key -- stable, so a bucket keeps
// (group, row) order -- into segment seg at replica position pos0; its sorted keys / groups
// go to buffers skeys[buf] / sgroup[buf] (k: base, kMaxKeys + k: delta).
static int sort_segment(dk_ctx* c, BlockTables& T, int k, int buf, int seg, uint64_t pos0, uint64_t m) {
  hipStream_t s = c->stream;
  uint32_t* rows = c->rowof.as<uint32_t>() + pos0;
  HIPCHK(c->gkeys.reserve(m * 8 + 8, 0, s));
  HIPCHK(c->skeys[buf].reserve(m * 8 + 8, 0, s));
  if (m) {
    HIPCHK(launch_gather_keys(c->keys[k].as<uint64_t>(), c->usable.as<uint32_t>(), c->gkeys.as<uint64_t>(), m, s));
    HIPCHK(with_tmp(c, [&](void* t, size_t& b) {
      return sort_pairs_u64_u32(t, b, c->gkeys.as<uint64_t>(), c->skeys[buf].as<uint64_t>(),
                                c->usable.as<uint32_t>(), rows, m, s);
    }));
  }
  if (T.linkage) {
    HIPCHK(c->sgroup[buf].reserve(m + 8, 0, s));
    if (m) HIPCHK(launch_gather_u8(c->group.as<uint8_t>(), rows, c->sgroup[buf].as<uint8_t>(), m, s));
  }
  T.skeys[seg] = c->skeys[buf].as<uint64_t>();
  T.sgroup[seg] = c->sgroup[buf].as<uint8_t>();
  T.seg_len[seg] = m;
  T.seg_off[seg] = pos0;
  return DK_OK;
}

// replica-ordered identity / keys (the candidate filters) of positions [pos0, pos0 + n)
static int fill_rows(dk_ctx* c, const BlockTables& T, uint64_t pos0, uint64_t n) {
  uint64_t* rk[kMaxKeys] = {};
  for (int k = 0; k + 1 < c->schema.nkeys; ++k) rk[k] = c->rkeys[k].as<uint64_t>();
  HIPCHK(launch_replicate_rows(c->rowof.as<uint32_t>(), pos0, n, c->ident.as<uint64_t>(),
                               c->rident.as<uint64_t>(), T, rk, c->stream));
  return DK_OK;
}

static bool delta_enabled() {
  const char* e = getenv("DK_DELTA");
  return !(e && e[0] == '0');
}

// delta capacity per key function: an eighth of the base, at least DK_DELTA_MIN rows
static uint64_t delta_capacity(uint64_t m) {
  const char* e = getenv("DK_DELTA_MIN");
  const uint64_t lo = e ? strtoull(e, nullptr, 10) : (1ull << 16);
  return std::max<uint64_t>(lo, m / 8);
}

// Full sort: every usable row into the base segments (ALLPAIRS: the usable rows are the
// replica, no tables).
static int build_full(dk_ctx* c, BlockTables& T, uint64_t* Mout) {
  hipStream_t s = c->stream;
  HostLap lap("dk_match build", s);
  const int nk = c->schema.nkeys;
  const bool allpairs = c->schema.mode == DK_MODE_ALLPAIRS;
  uint64_t M = 0;
  int rc = build_usable(c, 0, c->nrows, &M);
  if (rc) return rc;
  lap("usable");
  c->base_ok = false;
  c->base_dead.clear();
  if (allpairs) {
    c->rowof_p = c->usable.as<uint32_t>();
    c->rstride = M;
    rc = build_replica(c, c->rep, c->rowof_p, M);
    if (rc) return rc;
    *Mout = M;
    return DK_OK;
  }
  // transient rows are never usable; the base covers the rows below them
  const uint64_t rb = c->transient ? c->transient_row0 : c->nrows;
  uint64_t dcap = delta_enabled() ? delta_capacity(M) : 0;
  // replica positions (K * (M + dcap)) stay below the u32 sentinel
  const uint64_t lim = (uint64_t)kSentinel / (uint64_t)nk;
  if (M + dcap >= lim) dcap = M < lim ? lim - 1 - M : 0;
  const uint64_t kstride = M + dcap;
  const uint64_t npos = (uint64_t)nk * kstride;
  HIPCHK(c->rowof.reserve(npos * 4 + 4, 0, s));
  T.nseg = nk;
  T.seg_shift = 0;
  for (int k = 0; k < nk; ++k) {
    rc = sort_segment(c, T, k, k, k, (uint64_t)k * kstride, M);
    if (rc) return rc;
  }
  lap("sort");
  T.rowof = c->rowof.as<uint32_t>();
  c->rowof_p = T.rowof;
  c->rstride = npos;
  rc = layout_replica(c, c->rep, npos);
  if (rc) return rc;
  HIPCHK(c->rident.reserve(npos * 8 + 8, 0, s));
  for (int k = 0; k + 1 < nk; ++k) HIPCHK(c->rkeys[k].reserve(npos * 8 + 8, 0, s));
  T.rident = c->rident.as<uint64_t>();
  lap("layout");
  for (int k = 0; k < nk; ++k) {
    rc = fill_replica(c, c->rep, T.rowof, T.seg_off[k], M);
    if (rc) return rc;
    rc = fill_rows(c, T, T.seg_off[k], M);
    if (rc) return rc;
  }
  lap("fill");
  c->base_ok = dcap > 0;
  c->base_rows = rb;
  c->base_m = M;
  c->dcap = dcap;
  c->base_retired = 0;
  *Mout = M;
  return DK_OK;
}

// Delta build: retire the base rows superseded since the last build, re-sort the usable
// rows from base_rows on into the delta segments and replicate only those.  Cost O(delta
// + retired rows), independent of the base size.  Returns 1 when a full sort is due.
static int build_delta(dk_ctx* c, BlockTables& T) {
  hipStream_t s = c->stream;
  const int nk = c->schema.nkeys;
  if (!c->base_ok || c->nrows < c->base_rows || !replica_fits(c, c->rep)) return 1;
  if (c->base_retired + c->base_dead.size() > c->base_m / 4 + 1024) return 1;
  uint64_t Md = 0;
  int rc = build_usable(c, c->base_rows, c->nrows, &Md);
  if (rc) return rc;
  if (Md > c->dcap) return 1;
  const uint64_t kstride = c->base_m + c->dcap;
  T.nseg = 2 * nk;
  T.seg_shift = 1;
  T.rowof = c->rowof.as<uint32_t>();
  T.rident = c->rident.as<uint64_t>();
  for (int k = 0; k < nk; ++k) {  // the base segments as sorted
    T.skeys[2 * k] = c->skeys[k].as<uint64_t>();
    T.sgroup[2 * k] = c->sgroup[k].as<uint8_t>();
    T.seg_len[2 * k] = c->base_m;
    T.seg_off[2 * k] = (uint64_t)k * kstride;
  }
  if (!c->base_dead.empty()) {
    const uint64_t nd = c->base_dead.size();
    HIPCHK(c->d_dead.reserve(nd * 4 + 4, 0, s));
    HIPCHK(hipMemcpyAsync(c->d_dead.p, c->base_dead.data(), nd * 4, hipMemcpyHostToDevice, s));
    HIPCHK(launch_mark_dead(T, c->d_dead.as<uint32_t>(), nd, c->rident.as<uint64_t>(), s));
    HIPCHK(hipStreamSynchronize(s));  // the host list is reused
    c->base_retired += nd;
    c->base_dead.clear();
  }
  for (int k = 0; k < nk; ++k) {
    // delta skeys / sgroup live in the upper half of the segment buffers
    rc = sort_segment(c, T, k, kMaxKeys + k, 2 * k + 1, (uint64_t)k * kstride + c->base_m, Md);
    if (rc) return rc;
    rc = fill_replica(c, c->rep, T.rowof, T.seg_off[2 * k + 1], Md);
    if (rc) return rc;
    rc = fill_rows(c, T, T.seg_off[2 * k + 1], Md);
    if (rc) return rc;
  }
  if (Md == 0) {  // nothing added since the base: one segment per key function
    BlockTables B = T;
    B.nseg = nk;
    B.seg_shift = 0;
    for (int k = 0; k < nk; ++k) {
      B.skeys[k] = T.skeys[2 * k];
      B.sgroup[k] = T.sgroup[2 * k];
      B.seg_len[k] = T.seg_len[2 * k];
      B.seg_off[k] = T.seg_off[2 * k];
    }
    for (int k = nk; k < kMaxSegs; ++k) {
      B.skeys[k] = nullptr;
      B.sgroup[k] = nullptr;
      B.seg_len[k] = B.seg_off[k] = 0;
    }
    T = B;
  }
  return DK_OK;
}

// Lucene source: the postings of the rows in the index (kAlive: superseded versions were
// deleted by ID, transient rows never entered; dukeDeleted rows stay, as in the reference's
// index; with unmerged statistics also the superseded versions, kIndexed, which k_lucene_topk
// never returns) sorted by (field, term, row), and maxDoc.  Index state, built like the blocking
// tables by the first match after an index change.
static int build_lucene(dk_ctx* c, BlockTables& T, uint64_t* Mout) {
  auto& L = c->luc;
  hipStream_t s = c->stream;
  const uint64_t np = L.npost;
  HIPCHK(L.tkey.reserve(np * 8 + 8, 0, s));
  HIPCHK(L.skey.reserve(np * 8 + 8, 0, s));
  HIPCHK(L.stf.reserve(np * 4 + 4, 0, s));
  uint64_t* cnt = c->counters.as<uint64_t>() + 2;
  HIPCHK(hipMemsetAsync(cnt, 0, 16, s));
  HIPCHK(launch_lucene_prep(L.pkey.as<uint64_t>(), np, c->flags.as<uint8_t>(), c->nrows,
                            L.unmerged ? kIndexed : kAlive, L.tkey.as<uint64_t>(), cnt, s));
  if (np) {
    HIPCHK(with_tmp(c, [&](void* t, size_t& b) {
      return sort_pairs_u64_u32(t, b, L.tkey.as<uint64_t>(), L.skey.as<uint64_t>(), L.ptf.as<uint32_t>(),
                                L.stf.as<uint32_t>(), np, s);
    }));
  }
  uint64_t h[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(h, cnt, 16, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  L.nsorted = h[0];
  L.max_doc = h[1];
  T.nseg = 1;
  T.seg_shift = 0;
  *Mout = L.max_doc;
  return DK_OK;
}

// The blocking tables and the candidate replica (index state): built by the first call
// after the index changed, reused until the next change.  An index that only grew (or lost
// rows to delete-by-ID) since the last full sort gets a delta build.
static int ensure_tables(dk_ctx* c, BlockTables* Tout, uint64_t* Mout) {
  if (c->tables_gen == c->index_gen) {
    *Tout = c->tables;
    *Mout = c->tables_m;
    return DK_OK;
  }
  if (c->luc.on) {
    BlockTables T{};
    T.group = c->group.as<uint8_t>();
    uint64_t M = 0;
    int rc = build_lucene(c, T, &M);
    if (rc) return rc;
    c->prof.full_builds += 1;
    c->tables = T;
    c->tables_m = M;
    c->tables_gen = c->index_gen;
    *Tout = T;
    *Mout = M;
    return DK_OK;
  }
  BlockTables T{};
  T.nkeys = c->schema.nkeys;
  T.linkage = c->schema.mode == DK_MODE_LINKAGE;
  T.group = c->group.as<uint8_t>();
  for (int k = 0; k < T.nkeys; ++k) T.keys[k] = c->keys[k].as<uint64_t>();
  uint64_t M = c->base_m;
  int rc = c->schema.mode == DK_MODE_ALLPAIRS ? 1 : build_delta(c, T);
  if (rc == 1) {
    BlockTables F{};
    F.nkeys = T.nkeys;
    F.linkage = T.linkage;
    F.group = T.group;
    for (int k = 0; k < T.nkeys; ++k) F.keys[k] = T.keys[k];
    T = F;
    rc = build_full(c, T, &M);
    if (rc == DK_OK) c->prof.full_builds += 1;
  } else if (rc == DK_OK) {
    c->prof.delta_builds += 1;
  }
  if (rc) {
    c->base_ok = false;  // a failed build leaves no trusted base
    return rc;
  }
  c->tables = T;
  c->tables_m = M;
  c->tables_gen = c->index_gen;
  *Tout = T;
  *Mout = M;
  return DK_OK;
}

// k_score_sym2 (two queries per wave, owner slots padded to 32): schemas whose Levenshtein /
// JaroWinkler / Exact columns are Latin-1 (the wave's two 256-entry Peq tables fill its LDS
// slice), with a DP comparator and no gram sets; DK_SYM2=0 keeps one query per wave (A/B)
static bool sym2_ok(const dk_ctx* c, const ScoreParams& P) {
  const char* e = getenv("DK_SYM2");
  if ((e && e[0] == '0') || !P.has_dp || P.has_grams || P.has_geo || P.norders > 1) return false;
  for (int p = 0; p < P.nprops; ++p) {
    const DevProp& D = P.props[p];
    if (D.op != DK_CMP_LEVENSHTEIN && D.op != DK_CMP_JAROWINKLER && D.op != DK_CMP_EXACT &&
        D.op != DK_CMP_NUMERIC && D.op != DK_CMP_NONE)
      return false;
    if ((D.op == DK_CMP_LEVENSHTEIN || D.op == DK_CMP_JAROWINKLER || D.op == DK_CMP_EXACT) && D.width != 1)
      return false;
  }
  return true;
}

// k_opack's order within a tile: the query's length on the schema's longest Levenshtein
// property (the DP whose row bucket costs most), or none (DK_SYM_ORDER=0: query order)
static const uint16_t* sym2_order_len(const dk_ctx* c, const ScoreParams& P) {
  const char* e = getenv("DK_SYM_ORDER");
  if (e && e[0] == '0') return nullptr;
  int best = -1, bl = 0;
  for (int p = 0; p < P.nprops; ++p)
    if (P.props[p].op == DK_CMP_LEVENSHTEIN && c->P[p].maxlen > bl) {
      best = p;
      bl = c->P[p].maxlen;
    }
  return best < 0 ? nullptr : P.props[best].len;
}

static bool sym_enabled() {
  const char* e = getenv("DK_SYM");
  return !(e && e[0] == '0');
}

// The symmetric schedule holds when every comparator gives compare(a, b) and compare(b, a)
// the same PropertyImpl probability, or (JaroWinkler) the kernel computes both directions:
// Levenshtein (the cutoff only moves a < 0.5 similarity), QGram, Exact, Numeric, none.
// WeightedLevenshtein's stride aliasing and the token comparators' "shorter list first"
// are orientation dependent; the long-value kernels are not instantiated for it.
static bool sym_schema_ok(const dk_ctx* c, const ScoreParams& P) {
  // several order classes: compare(candidate, query) would follow the candidate's order
  if (c->schema.mode != DK_MODE_DEDUP || P.long_rows > 0 || P.norders > 1) return false;
  for (const auto& S : c->P) {
    const int op = S.cfg.comparator;
    if (op == DK_CMP_WEIGHTED_LEVENSHTEIN || op == DK_CMP_DICE_TOKENS || op == DK_CMP_JACCARD_TOKENS ||
        op == DK_CMP_GEOPOSITION)
      return false;
  }
  return true;
}

// k_score_grouped (dk_score_grouped.hip) serves the direct schedule of schemas made of
// Numeric properties and at most kGroupedTabs Latin-1 bigram QGram properties with a key
// replica (configs[2]); DK_GROUPED=0 keeps them on k_score_nodp (A/B).
static bool grouped_schema_ok(const ScoreParams& P) {
  const char* e = getenv("DK_GROUPED");
  if ((e && e[0] == '0') || P.has_dp || P.raw_prop >= 0 || P.nprops < 1) return false;
  // every offset of the kernel's raw buffer loads below 2^31 (a tail row of w has its own
  // buffer resource, so the replica's rows do not add up), and the head rows (read for
  // every pair through one resource) under 4 GiB
  if (P.rstride * 8 >= (1ull << 31)) return false;
  if (P.rstride * 8 * kGroupedHeadRows >= (1ull << 32)) return false;
  int tabs = 0;
  for (int p = 0; p < P.nprops; ++p) {
    const DevProp& D = P.props[p];
    if (D.op == DK_CMP_QGRAM) {
      if (!D.g16 || D.rgrows < 1 || D.width != 1) return false;
      ++tabs;
    } else if (D.op != DK_CMP_NUMERIC && D.op != DK_CMP_NONE) {
      return false;
    }
  }
  return tabs <= kGroupedTabs;
}

// k_score_grouped's per-property operand sources (GroupedProp) for the current replica
static std::vector<GroupedProp> grouped_props(const ScoreParams& P) {
  std::vector<GroupedProp> gp(P.nprops);
  const uint64_t n = P.rstride;
  uint32_t ts = 0;
  for (int p = 0; p < P.nprops; ++p) {
    const DevProp& D = P.props[p];
    GroupedProp& G = gp[p];
    memset(&G, 0, sizeof G);
    if (D.op == DK_CMP_QGRAM) G.tslot = ts++;
    G.len = D.rlen;
    G.len_n = (uint32_t)(n * 2);
    G.x = G.w = D.rlen;  // size 0 below unless the comparator has them
    if (D.op == DK_CMP_QGRAM) {
      G.x = D.rgcnt;
      G.x_n = (uint32_t)(n * 2);
      G.xsh = 1;
      G.w = D.rgrams;
      G.w_rows = (uint32_t)D.rgrows;
      G.w_head = G.w_rows;
      G.rowb = (uint32_t)(n * 8);
    } else if (D.op == DK_CMP_NUMERIC) {
      G.x = D.rnumok;
      G.x_n = (uint32_t)n;
      G.w = D.rnum;
      G.w_rows = 1;
      G.w_head = 1;
      G.rowb = (uint32_t)(n * 8);
    }
  }
  return gp;
}

// k_score_gq (round 5) serves the grouped schemas without DK_CMP_NONE properties, of 1-2
// bigram QGram and at most kGQMaxNum Numeric properties, whose key-word rows fit the head
// and tail buffer resources; DK_GQ=0 keeps k_score_grouped (A/B).  Fills the roles: QGram
// roles by key-word rows (fewest first: role 0 holds fewer rows in registers), Numeric roles
// in property order, and each order class's visiting order as roles.
static bool gq_args(const ScoreParams& P, GQArgs* A, int* nq, int* nn) {
  const char* e = getenv("DK_GQ");
  if (e && e[0] == '0') return false;
  memset(A, 0, sizeof *A);
  int qp[kMaxProps], np[kMaxProps], a = 0, b = 0;
  for (int p = 0; p < P.nprops; ++p) {
    const int op = P.props[p].op;
    if (op == DK_CMP_QGRAM) qp[a++] = p;
    else if (op == DK_CMP_NUMERIC) np[b++] = p;
    else return false;
  }
  if (a < 1 || a > kGroupedTabs || b > kGQMaxNum) return false;
  if (a == 2 && P.props[qp[1]].rgrows < P.props[qp[0]].rgrows) std::swap(qp[0], qp[1]);
  const uint64_t n = P.rstride;
  if (n * 2 >= (1ull << 32) || n * 8 >= (1ull << 32)) return false;
  A->nq = a;
  A->nn = b;
  A->len_bytes = (uint32_t)(n * 2);
  A->pos_n = (uint32_t)n;
  uint32_t role[kMaxProps];
  for (int i = 0; i < a; ++i) {
    const DevProp& D = P.props[qp[i]];
    GQRoleQ& R = A->q[i];
    R.rlen = D.rlen;
    R.rgcnt = D.rgcnt;
    R.rows = static_cast<const uint64_t*>(D.rgrams);
    R.tail = R.rows + (uint64_t)kGroupedHeadRows * n;
    R.nrows = (uint32_t)D.rgrows;
    R.rowb = (uint32_t)(n * 8);
    const uint64_t head = (uint64_t)std::min(D.rgrows, kGroupedHeadRows) * n * 8;
    const uint64_t tail = D.rgrows > kGroupedHeadRows ? (uint64_t)(D.rgrows - kGroupedHeadRows) * n * 8 : 0;
    if (head >= (1ull << 32) || tail >= (1ull << 32)) return false;
    R.head_bytes = (uint32_t)head;
    R.tail_bytes = (uint32_t)tail;
    R.prop = qp[i];
    R.formula = D.formula;
    R.low = D.low;
    R.high = D.high;
    R.flow = (float)D.low;
    R.fhigh = (float)D.high;
    R.flow0 = (float)std::max(0.0, D.low);
    const double g5 = (D.high - 0.5) * 0.25 + 0.5;
    R.fub = (float)std::max(std::max(0.0, D.low), std::max(g5, D.high));
    role[qp[i]] = (uint32_t)i;
  }
  for (int i = 0; i < b; ++i) {
    const DevProp& D = P.props[np[i]];
    GQRoleN& R = A->n[i];
    R.rlen = D.rlen;
    R.rnumok = D.rnumok;
    R.rnum = D.rnum;
    R.prop = np[i];
    R.low = D.low;
    R.high = D.high;
    R.min_ratio = D.min_ratio;
    role[np[i]] = 8u + (uint32_t)i;
  }
  for (int c = 0; c < kMaxOrders; ++c) {
    uint64_t w = 0;
    for (int k = 0; k < P.nprops; ++k) w |= (uint64_t)role[(P.order[c] >> (4 * k)) & 15u] << (4 * k);
    A->rorder[c] = w;
  }
  // the screen (k_score_gq): kind != 0 iff prob > tm; the bound's odds must reach
  // tm / (1 - tm), less a 2e-3 margin for the single-precision bound
  const double tm = P.maybe != 0.0 ? std::min(P.threshold, P.maybe) : P.threshold;
  A->screen = tm >= kScreenLo && tm <= kScreenHi ? (float)(tm / (1.0 - tm) * (1.0 - 2e-3)) : 0.0f;
  const char* es = getenv("DK_GQ_SCREEN");  // 0: every valid pair to the exact pass (A/B)
  if (es && es[0] == '0') A->screen = 0.0f;
  // the deferred QGram role: DK_GQ_DEFER = -1 / 0 / 1 (default 0 with two QGram roles)
  A->defer = a == 2 ? 0 : -1;
  const char* ed = getenv("DK_GQ_DEFER");
  if (ed && a == 2) A->defer = atoi(ed) < 0 ? -1 : std::min(atoi(ed), 1);
  *nq = a;
  *nn = b;
  return true;
}

// Lucene source, per dk_match: every query's hits (k_lucene_topk) become its candidate
// range -- positions qi * max_hits + j of a per-call candidate replica, in hit order -- and
// the slot layout (counts, offsets, wave map) of the direct schedule.  d_queries holds the
// query rows.  exact (host, optional): the hits per query.
static int lucene_candidates(dk_ctx* c, uint64_t nq, uint64_t* total, uint64_t* generated,
                             uint64_t* exact) {
  auto& L = c->luc;
  hipStream_t s = c->stream;
  const uint64_t K = (uint64_t)L.max_hits, npos = std::max<uint64_t>(nq * K, 1);
  HIPCHK(L.hits.reserve(npos * 4 + 4, 0, s));
  HIPCHK(hipMemsetAsync(L.hits.p, 0, npos * 4, s));  // unused positions name row 0
  HIPCHK(c->ranges.reserve(nq * 8 + 8, 0, s));
  HIPCHK(c->counts.reserve((nq + 1) * 8, 0, s));
  HIPCHK(c->qoff.reserve((nq + 1) * 8, 0, s));
  if (exact) HIPCHK(L.exact.reserve(nq * 8 + 8, 0, s));
  HIPCHK(hipMemsetAsync(c->counters.as<uint64_t>() + 2, 0, 8, s));
  LuceneParams P{};
  P.queries = c->d_queries.as<uint32_t>();
  P.nq = nq;
  P.qoff = L.qoff_d.as<uint64_t>();
  P.qterm = L.qterm.as<uint32_t>();
  P.skey = L.skey.as<uint64_t>();
  P.stf = L.stf.as<uint32_t>();
  P.npost = L.nsorted;
  P.norm = L.norm.as<uint8_t>();
  P.nfields = (int32_t)L.fields.size();
  P.linkage = c->schema.mode == DK_MODE_LINKAGE;
  P.flags = c->flags.as<uint8_t>();
  P.group = c->group.as<uint8_t>();
  P.max_doc = L.max_doc;
  P.max_hits = L.max_hits;
  P.min_relevance = L.min_rel;
  P.hits = L.hits.as<uint32_t>();
  P.ranges = c->ranges.as<uint2>();
  P.counts = c->counts.as<uint64_t>();
  P.exact = exact ? L.exact.as<uint64_t>() : nullptr;
  P.real = c->counters.as<uint64_t>() + 2;
  HIPCHK(launch_lucene_topk(P, s));
  if (exact) {
    HIPCHK(hipMemcpyAsync(exact, L.exact.p, nq * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return DK_OK;
  }
  uint64_t* hs = c->h_small.as<uint64_t>();
  HIPCHK(hipMemsetAsync(c->counts.as<uint64_t>() + nq, 0, 8, s));
  HIPCHK(with_tmp(c, [&](void* t, size_t& b) {
    return exclusive_scan_u64(t, b, c->counts.as<uint64_t>(), c->qoff.as<uint64_t>(), nq + 1, s);
  }));
  HIPCHK(hipMemcpyAsync(&hs[3], c->qoff.as<uint64_t>() + nq, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(&hs[2], c->counters.as<uint64_t>() + 2, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  *total = hs[3];
  *generated = hs[2];
  HIPCHK(c->wq.reserve(*total / 64 * 4 + 4, 0, s));
  HIPCHK(launch_wavemap(c->qoff.as<uint64_t>(), nq, c->wq.as<uint32_t>(), s));
  // the hits' values in candidate-replica order, and their identities (isSameAs)
  c->rowof_p = L.hits.as<uint32_t>();
  c->rstride = npos;
  int rc = layout_replica(c, c->rep, npos);
  if (rc) return rc;
  rc = fill_replica(c, c->rep, c->rowof_p, 0, npos);
  if (rc) return rc;
  HIPCHK(c->rident.reserve(npos * 8 + 8, 0, s));
  BlockTables T{};
  uint64_t* rk[kMaxKeys] = {};
  HIPCHK(launch_replicate_rows(c->rowof_p, 0, npos, c->ident.as<uint64_t>(), c->rident.as<uint64_t>(),
                               T, rk, s));
  return DK_OK;
}

// GeopositionComparator values without ',' (numok 2): cleared before a geo schema's scoring,
// read after it; set -> the call fails as stock Duke's compare would raise
static int geo_raise_clear(dk_ctx* c, const ScoreParams& P) {
  if (P.has_geo) HIPCHK(hipMemsetAsync(c->raised.p, 0, 4, c->stream));
  return DK_OK;
}
static int geo_raise_check(dk_ctx* c, const ScoreParams& P) {
  if (!P.has_geo) return DK_OK;
  HIPCHK(hipMemcpyAsync(c->h_raised.p, c->raised.p, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (*c->h_raised.as<uint32_t>())
    return fail(DK_E_UNSUPPORTED, "GeopositionComparator compared a value without ',' "
                                  "(stock Duke raises: Geoposition.parse)");
  return DK_OK;
}

static int run_match(dk_ctx* c, const uint32_t* query_rows, uint64_t nq, int flags,
                     ResultHolder* R, bool contiguous) {
  hipStream_t s = c->stream;
  HostLap lap("dk_match", s);
  c->spans.clear();   // left over by a failed call
  HIPCHK(hipStreamSynchronize(c->copy_stream));
  lap("streams");
  c->ev_next = 0;
  const auto t0 = std::chrono::steady_clock::now();
  const int nk = c->schema.nkeys;
  const bool allpairs = c->schema.mode == DK_MODE_ALLPAIRS;

  HIPCHK(c->d_queries.reserve(nq * 4 + 4, 0, s));
  // a contiguous batch (Processor.deduplicate's) is written on the device: a pageable 4 MB
  // host copy took 0.2 ms or, on a fresh context, 16 ms (DK_HOST_TIMING)
  if (contiguous && nq) HIPCHK(launch_iota_u32(c->d_queries.as<uint32_t>(), nq, query_rows[0], s));
  else HIPCHK(hipMemcpyAsync(c->d_queries.p, query_rows, nq * 4, hipMemcpyHostToDevice, s));

  // ---- index: usable rows + per key function sort by (key, group, row) ----
  lap("queries");
  Timer t_index(c, &c->prof.ms_index, s);
  uint64_t M = 0;
  BlockTables T{};
  int rc = ensure_tables(c, &T, &M);
  if (rc) return rc;
  t_index.stop();
  lap("index");

  // ---- candidate counts per query -> slot offsets ----
  Timer t_gen(c, &c->prof.ms_generate, s);
  uint64_t total = 0, generated = 0, mpad = 0, otot = 0, mtot = 0;
  const bool lucene = c->luc.on;
  if (lucene) {
    rc = lucene_candidates(c, nq, &total, &generated, nullptr);
    if (rc) return rc;
  }
  const ScoreParams P = make_params(c, c->rep, c->rowof_p, c->rstride);
  {
    const int rg = geo_raise_clear(c, P);
    if (rg) return rg;
  }
  c->prof.replica_positions = P.rstride;
  c->prof.gram_row_bytes = 0;
  for (int p = 0; p < P.nprops; ++p)
    if (P.props[p].op == DK_CMP_QGRAM)
      c->prof.gram_row_bytes = std::max(c->prof.gram_row_bytes, (uint64_t)P.props[p].rgrows * P.rstride * 8);
  bool sym = !lucene && contiguous && nq > 0 && sym_enabled() && sym_schema_ok(c, P);
  const bool two = sym && sym2_ok(c, P);  // k_score_sym2: half-wave queries
  bool grouped = false;  // k_score_grouped: query slots padded to kScoreBlock
  const uint32_t r0 = nq ? query_rows[0] : 0;
  uint64_t* hs = c->h_small.as<uint64_t>();
  SymIndex sx{};
  // a large batch looks its queries' buckets up in SymIndex (built once per table build: one
  // pass over the replica positions); a small one (an incremental batch) searches the tables
  const char* sxe = getenv("DK_SYMIDX");  // 1: always, 0: never (tests, A/B)
  if (sym && (sxe ? sxe[0] == '1' : nq * 8 >= P.rstride)) {
    if (c->sx_gen != c->tables_gen) {
      uint64_t maxlen = 1;
      for (int k = 0; k < T.nseg; ++k) maxlen = std::max<uint64_t>(maxlen, T.seg_len[k]);
      size_t tb = 0;
      HIPCHK(symidx_scan_bytes(maxlen, &tb));
      HIPCHK(c->sx_posof.reserve((uint64_t)T.nseg * c->nrows * 4 + 4, 0, s));
      HIPCHK(c->sx_hflag.reserve(P.rstride * 4 + 4, 0, s));
      HIPCHK(c->sx_bstart.reserve(P.rstride * 4 + 4, 0, s));
      HIPCHK(c->sx_bend.reserve(P.rstride * 4 + 4, 0, s));
      HIPCHK(c->sx_tmp.reserve(tb + 16, 0, s));
      HIPCHK(hipMemsetAsync(c->sx_posof.p, 0xFF, (uint64_t)T.nseg * c->nrows * 4, s));
      HIPCHK(c->sx_bse.reserve(P.rstride * 8 + 8, 0, s));
      HIPCHK(launch_symidx(T, c->nrows, c->sx_posof.as<uint32_t>(), c->sx_hflag.as<uint32_t>(),
                           c->sx_bstart.as<uint32_t>(), c->sx_bend.as<uint32_t>(), c->sx_bse.as<uint2>(), c->sx_tmp.p,
                           tb, s));
      c->sx_gen = c->tables_gen;
    }
    sx = SymIndex{c->sx_posof.as<uint32_t>(), c->sx_bstart.as<uint32_t>(), c->sx_bend.as<uint32_t>(), c->nrows,
                  c->sx_bse.as<uint2>()};
  }
  if (sym) {
    HIPCHK(c->ranges.reserve((uint64_t)T.nseg * nq * 16 + 16, 0, s));
    HIPCHK(c->counts.reserve((nq + 1) * 8, 0, s));
    HIPCHK(c->ocounts.reserve((nq + 1) * 8, 0, s));
    HIPCHK(c->qoff.reserve((nq + 1) * 8, 0, s));
    HIPCHK(c->oqoff.reserve((nq + 1) * 8, 0, s));
    HIPCHK(c->mcounts.reserve((nq + 1) * 8, 0, s));
    HIPCHK(c->mqoff.reserve((nq + 1) * 8, 0, s));
    HIPCHK(hipMemsetAsync(c->counters.as<uint64_t>() + 2, 0, 8, s));
    HIPCHK(launch_count_sym(c->d_queries.as<uint32_t>(), nq, T, r0, c->ranges.as<uint4>(),
                            c->counts.as<uint64_t>(), c->ocounts.as<uint64_t>(),
                            c->mcounts.as<uint64_t>(), c->counters.as<uint64_t>() + 2, two ? 1u : 64u, sx, s));
    HIPCHK(hipMemsetAsync(c->counts.as<uint64_t>() + nq, 0, 8, s));
    HIPCHK(hipMemsetAsync(c->ocounts.as<uint64_t>() + nq, 0, 8, s));
    HIPCHK(hipMemsetAsync(c->mcounts.as<uint64_t>() + nq, 0, 8, s));
    HIPCHK(with_tmp(c, [&](void* t, size_t& b) {
      return exclusive_scan_u64(t, b, c->mcounts.as<uint64_t>(), c->mqoff.as<uint64_t>(), nq + 1, s);
    }));
    HIPCHK(with_tmp(c, [&](void* t, size_t& b) {
      return exclusive_scan_u64(t, b, c->counts.as<uint64_t>(), c->qoff.as<uint64_t>(), nq + 1, s);
    }));
    if (two) {
      // waves of at most two queries, per tile of kPackTile queries (in the order of their length
      // on the longest Levenshtein property; DK_SYM_ORDER=0: query order)
      const uint64_t nt = opack_tiles(nq);
      HIPCHK(c->ploc.reserve(nq * 4 + 4, 0, s));
      HIPCHK(c->ptot.reserve((nt + 1) * 8, 0, s));
      HIPCHK(c->pbase.reserve((nt + 1) * 8, 0, s));
      HIPCHK(launch_opack(c->ocounts.as<uint64_t>(), nq, c->d_queries.as<uint32_t>(), sym2_order_len(c, P),
                          c->ploc.as<uint32_t>(), c->ptot.as<uint64_t>(), s));
      HIPCHK(hipMemsetAsync(c->ptot.as<uint64_t>() + nt, 0, 8, s));
      HIPCHK(with_tmp(c, [&](void* t, size_t& b) {
        return exclusive_scan_u64(t, b, c->ptot.as<uint64_t>(), c->pbase.as<uint64_t>(), nt + 1, s);
      }));
      HIPCHK(launch_opack_fin(c->ploc.as<uint32_t>(), c->pbase.as<uint64_t>(), nq, c->oqoff.as<uint64_t>(), s));
      HIPCHK(c->h_pbase.reserve((nt + 1) * 8));  // the chunks' owner slots without a second round trip
      HIPCHK(hipMemcpyAsync(c->h_pbase.p, c->pbase.p, (nt + 1) * 8, hipMemcpyDeviceToHost, s));
    } else {
      HIPCHK(with_tmp(c, [&](void* t, size_t& b) {
        return exclusive_scan_u64(t, b, c->ocounts.as<uint64_t>(), c->oqoff.as<uint64_t>(), nq + 1, s);
      }));
    }
    HIPCHK(hipMemcpyAsync(&hs[3], c->qoff.as<uint64_t>() + nq, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&hs[2], c->counters.as<uint64_t>() + 2, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&hs[1], c->oqoff.as<uint64_t>() + nq, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&hs[0], c->mqoff.as<uint64_t>() + nq, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    total = hs[3];
    generated = hs[2];
    otot = hs[1];
    mtot = hs[0];
  }
  // at least kMinChunks chunks (down to CH0/16 slots each): the emission pass and the list's
  // copies of chunk i overlap the scoring of chunk i+1, so a small call (one GPU's tile of a
  // multi-GPU match) still pipelines
  constexpr uint64_t kMinChunks = 8;
  const uint64_t CH0 = chunk_slots();
  auto chunk_len = [&](uint64_t tot) {
    return std::max<uint64_t>(kScoreBlock, (std::max(CH0 / 16, std::min(CH0, (tot + kMinChunks - 1) / kMinChunks)) +
                                            kScoreBlock - 1) / kScoreBlock * kScoreBlock);
  };
  // SYM: chunks cut by queries (an emission chunk reads the owner results of its own queries
  // and the mirror results earlier queries pushed): qb = the chunks' query bounds, obounds =
  // their owner slots; ochunk = the largest chunk's owner slots
  std::vector<uint64_t> qb, obounds;
  uint64_t ochunk = 1;
  if (sym) {
    // k_score_sym2's chunks are whole tiles of k_opack (its queries are ordered per tile)
    const uint64_t qg = two ? (uint64_t)kPackTile : 1;
    auto qcut = [&](uint64_t x) { return std::min(nq, (x + qg / 2) / qg * qg); };
    qb.push_back(0);
    const uint64_t nch = std::max<uint64_t>(1, (total + chunk_len(total) - 1) / chunk_len(total));
    for (uint64_t i = 1; i < nch; ++i) qb.push_back(qcut(nq * i / nch));
    qb.push_back(nq);
    if (!(flags & DK_MATCH_DEVICE)) {  // halve the last chunk twice
      for (int h = 0; h < 2; ++h) {
        const uint64_t a = qb[qb.size() - 2], e = qb.back();
        if (e - a >= 2 * qg) qb.insert(qb.end() - 1, qcut(a + (e - a) / 2));
      }
    }
    // more chunks than queries (small slot chunks): no empty chunk -- its count read-back
    // would be the previous query's inclusive prefix
    qb.erase(std::unique(qb.begin(), qb.end()), qb.end());
    const uint64_t nb = qb.size();
    if (two) {  // tile offsets (read back above)
      const uint64_t* tb = c->h_pbase.as<uint64_t>();
      for (uint64_t i = 0; i < nb; ++i) obounds.push_back(tb[(qb[i] + qg - 1) / qg]);
    } else {
      HIPCHK(c->bidx.reserve(nb * 8 + 8, 0, s));
      HIPCHK(c->bval.reserve(nb * 8 + 8, 0, s));
      HIPCHK(c->h_bounds.reserve(nb * 8 + 8));
      uint64_t* hb = c->h_bounds.as<uint64_t>();
      memcpy(hb, qb.data(), nb * 8);
      HIPCHK(hipMemcpyAsync(c->bidx.p, hb, nb * 8, hipMemcpyHostToDevice, s));
      HIPCHK(launch_gather_u64(c->oqoff.as<uint64_t>(), c->bidx.as<uint64_t>(), nb, c->bval.as<uint64_t>(), s));
      HIPCHK(hipMemcpyAsync(hb, c->bval.p, nb * 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      obounds.assign(hb, hb + nb);
    }
    // a half holds the chunk's slots from the wave of its first one (k_score_sym2's chunks
    // start inside a wave), plus 64 B the count pass's 16-B reads may touch past the end:
    // slot s of chunk ci at half + s - (obounds[ci] & ~63), 16-B aligned like s
    for (size_t i = 0; i + 1 < obounds.size(); ++i)
      ochunk = std::max(ochunk, obounds[i + 1] - (obounds[i] & ~(uint64_t)63));
    ochunk = (ochunk + 127) & ~(uint64_t)63;
    // mirror results live for the whole call (a query's emission reads what earlier
    // queries pushed): a decision byte + 8 B per mirror slot; owner results for one chunk
    // (its emission reads only its own queries' owner slots): two chunk-sized halves of a
    // byte + 8 B per owner slot.  Within a third of the free HBM, else the direct schedule.
    size_t fr = 0, tot_mem = 0;
    HIPCHK(hipMemGetInfo(&fr, &tot_mem));
    auto grow_by = [](const DevBuf& d, uint64_t want) { return want > d.bytes ? want - d.bytes : 0; };
    const size_t need = grow_by(c->ores, 2 * ochunk * 8 + 64) + grow_by(c->okind, 2 * ochunk + 64) +
                        grow_by(c->mres, mtot * 8 + 64) + grow_by(c->mkind, mtot + 64) +
                        grow_by(c->ecount, nq * 4 + 4) + grow_by(c->eincl, nq * 8 + 8);
    if (need > fr / 3) sym = false;
  }
  if (sym) {
    HIPCHK(c->mres.reserve(mtot * 8 + 64, 0, s));
    HIPCHK(c->mkind.reserve(mtot + 64, 0, s));
    HIPCHK(c->ores.reserve(2 * ochunk * 8 + 64, 0, s));
    HIPCHK(c->okind.reserve(2 * ochunk + 64, 0, s));
    HIPCHK(c->ecount.reserve(nq * 4 + 4, 0, s));
    HIPCHK(c->eincl.reserve(nq * 8 + 8, 0, s));
    HIPCHK(c->mbase.reserve((uint64_t)T.nseg * nq * 8 + 8, 0, s));
    HIPCHK(hipMemsetAsync(c->mkind.p, 0, mtot, s));  // no entry unless an owner pushes one
    HIPCHK(c->owq.reserve(otot / 64 * 8 + 8, 0, s));
    HIPCHK(c->obase.reserve((uint64_t)T.nseg * nq * 8 + 8, 0, s));
    if (two) HIPCHK(launch_wavemap2(c->oqoff.as<uint64_t>(), c->ocounts.as<uint64_t>(), nq, c->owq.as<uint2>(), s));
    else HIPCHK(launch_wavemap(c->oqoff.as<uint64_t>(), nq, c->owq.as<uint32_t>(), s));
    HIPCHK(launch_obase(c->ranges.as<uint4>(), c->oqoff.as<uint64_t>(), c->mqoff.as<uint64_t>(),
                        nq, T.nseg, c->obase.as<uint64_t>(), c->mbase.as<uint64_t>(), s));
  } else if (!allpairs && !lucene) {
    grouped = grouped_schema_ok(P);
    HIPCHK(c->ranges.reserve((uint64_t)T.nseg * nq * 8 + 8, 0, s));
    HIPCHK(c->counts.reserve((nq + 1) * 8, 0, s));
    HIPCHK(c->qoff.reserve((nq + 1) * 8, 0, s));
    HIPCHK(hipMemsetAsync(c->counters.as<uint64_t>() + 2, 0, 8, s));
    HIPCHK(launch_count(c->d_queries.as<uint32_t>(), nq, T, c->ranges.as<uint2>(), c->counts.as<uint64_t>(),
                        c->counters.as<uint64_t>() + 2, grouped ? kScoreBlock : 64, s));
    HIPCHK(hipMemsetAsync(c->counts.as<uint64_t>() + nq, 0, 8, s));
    HIPCHK(with_tmp(c, [&](void* t, size_t& b) {
      return exclusive_scan_u64(t, b, c->counts.as<uint64_t>(), c->qoff.as<uint64_t>(), nq + 1, s);
    }));
    HIPCHK(hipMemcpyAsync(&hs[3], c->qoff.as<uint64_t>() + nq, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&hs[2], c->counters.as<uint64_t>() + 2, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    total = hs[3];
    generated = hs[2];
    // every wave of slots knows its query
    HIPCHK(c->wq.reserve(total / 64 * 4 + 4, 0, s));
    HIPCHK(launch_wavemap(c->qoff.as<uint64_t>(), nq, c->wq.as<uint32_t>(), s));
  } else if (allpairs) {
    mpad = (M + 63) & ~(uint64_t)63;
    total = nq * mpad;
    generated = nq * M;
  }
  // chunk boundaries: (direct schedules) in slots: full chunks, then (host modes) the last
  // two chunks' worth halved down to CH/16, so the copy of the final chunk's entries (not
  // overlapped with scoring) is short; (SYM) the query bounds qb
  std::vector<uint64_t> bounds{0};
  if (sym) {
    bounds = qb;
  } else {
    const uint64_t CH = chunk_len(total);
    const uint64_t min_chunk = std::max<uint64_t>(kScoreBlock, CH / 16 / kScoreBlock * kScoreBlock);
    uint64_t at = 0;
    while (at < total) {
      const uint64_t rem = total - at;
      uint64_t len = rem > CH ? CH : rem;
      if (rem <= 2 * CH && rem > min_chunk && !(flags & DK_MATCH_DEVICE))
        len = std::max(min_chunk, (rem / 2 + kScoreBlock - 1) / kScoreBlock * kScoreBlock);
      at = std::min(total, at + len);
      bounds.push_back(at);
    }
  }
  t_gen.stop();
  lap("generate");

  // two staging sets (direct schedules): chunk i+1 scores into one while chunk i's entries
  // are compacted out of the other, so the host never waits between score launches
  StageOut st[2];
  if (!sym) {
    uint64_t chunk = 1;
    for (size_t i = 0; i + 1 < bounds.size(); ++i) chunk = std::max(chunk, bounds[i + 1] - bounds[i]);
    const uint64_t nblk_max = (chunk + kScoreBlock - 1) / kScoreBlock;
    for (int b = 0; b < 2; ++b) {
      dk_ctx::StageBufs& G = c->stage[b];
      HIPCHK(G.bcnt.reserve(nblk_max * 4 + 4, 0, s));
      HIPCHK(G.bscored.reserve(nblk_max * 4 + 4, 0, s));
      HIPCHK(G.bbytes.reserve(nblk_max * 4 + 4, 0, s));
      HIPCHK(G.boff.reserve(nblk_max * 8 + 8, 0, s));
      HIPCHK(G.prob.reserve(nblk_max * kScoreBlock * 8, 0, s));
      HIPCHK(G.cand.reserve(nblk_max * kScoreBlock * 4, 0, s));
      HIPCHK(G.qidx.reserve(nblk_max * kScoreBlock * 4, 0, s));
      st[b] = StageOut{c->counters.as<uint64_t>(), G.bcnt.as<uint32_t>(), G.bscored.as<uint32_t>(),
                       G.bbytes.as<uint32_t>(), G.prob.as<double>(), G.cand.as<uint32_t>(),
                       G.qidx.as<uint32_t>()};
    }
  }
  StageOut so{};  // SYM: the owner phase's block counters (it stages no entries)
  if (sym) {
    const uint64_t onblk = (ochunk + kScoreBlock - 1) / kScoreBlock;
    dk_ctx::StageBufs& G = c->owner_stage;
    HIPCHK(G.bcnt.reserve(onblk * 4 + 4, 0, s));
    HIPCHK(G.bscored.reserve(onblk * 4 + 4, 0, s));
    HIPCHK(G.bbytes.reserve(onblk * 4 + 4, 0, s));
    so = StageOut{c->counters.as<uint64_t>(), G.bcnt.as<uint32_t>(), G.bscored.as<uint32_t>(),
                  G.bbytes.as<uint32_t>(), nullptr, nullptr, nullptr};
  }
  HIPCHK(hipMemsetAsync(c->counters.p, 0, 4 * sizeof(uint64_t), s));
  ResultBufs& B = *R->bufs;
  uint64_t nm = 0;  // entries so far
  PairSource src{};
  src.queries = c->d_queries.as<uint32_t>();
  src.m = M;
  if (allpairs) {
    src.allpairs = 1;
    src.mpad = mpad;
  } else {
    src.wq = c->wq.as<uint32_t>();
    src.qoff = c->qoff.as<uint64_t>();
    src.ranges = c->ranges.as<uint2>();
    src.nq = nq;
    src.nkeys = nk;
    src.nseg = T.nseg;
    src.seg_shift = T.seg_shift;
    for (int k = 0; k < T.nseg; ++k) src.segoff[k] = T.seg_off[k];  // Lucene: one segment at 0
    src.rident = c->rident.as<uint64_t>();
    for (int k = 0; k < nk; ++k) {
      src.qkeys[k] = c->keys[k].as<uint64_t>();
      src.rkeys[k] = c->rkeys[k].as<uint64_t>();
    }
  }
  EmitSource esrc{};
  if (sym) {
    // owner slots: phase 1 scores them (okind / ores), the emission pass walks the queries
    src.sym = 1;
    src.two = two ? 1 : 0;
    src.wq = c->owq.as<uint32_t>();
    src.wq2 = two ? c->owq.as<uint2>() : nullptr;
    src.qoff = c->oqoff.as<uint64_t>();
    src.sranges = c->ranges.as<uint4>();
    src.mkind = c->mkind.as<uint8_t>();
    src.mres = c->mres.as<double>();
    src.mbase = c->mbase.as<uint64_t>();
    src.r0 = r0;
    src.r1 = r0 + (uint32_t)nq;
    esrc.sranges = c->ranges.as<uint4>();
    esrc.obase = c->obase.as<uint64_t>();
    esrc.mbase = c->mbase.as<uint64_t>();
    esrc.mkind = c->mkind.as<uint8_t>();
    esrc.mres = c->mres.as<double>();
    esrc.rowof = c->rowof.as<uint32_t>();
    esrc.nq = nq;
    esrc.nseg = T.nseg;
    for (int k = 0; k < T.nseg; ++k) esrc.segoff[k] = T.seg_off[k];
    esrc.ecount = c->ecount.as<uint32_t>();
    esrc.eincl = c->eincl.as<uint64_t>();
    esrc.oqoff = c->oqoff.as<uint64_t>();
    esrc.mqoff = c->mqoff.as<uint64_t>();
    esrc.ocnt = two ? c->ocounts.as<uint64_t>() : nullptr;
    HIPCHK(B.d_first.reserve((nq + 1) * 8, 0, s));  // k_sym_emit writes first[] per chunk
  }
  // k_score_grouped: the tasks of each chunk in the order of their first candidate's replica
  // position (bucket by bucket), DK_TASK_SORT=0: slot order (A/B)
  const uint32_t* perm = nullptr;
  int gmode = 0;  // k_score_grouped<MODE>: how the key-word rows are addressed
  GQArgs gqa;
  int gq_nq = 0, gq_nn = 0;
  const bool gq = grouped && gq_args(P, &gqa, &gq_nq, &gq_nn);
  if (gq) {
    // per staging block: the pairs that reached the exact pass (dk_profile.pairs_exact)
    uint64_t nbx = 1;
    for (size_t i = 0; i + 1 < bounds.size(); ++i) nbx = std::max(nbx, (bounds[i + 1] - bounds[i] + kScoreBlock - 1) / kScoreBlock);
    for (int b = 0; b < 2; ++b) {
      HIPCHK(c->stage[b].bexact.reserve(nbx * 4 + 4, 0, s));
      st[b].bexact = c->stage[b].bexact.as<uint32_t>();
    }
    // one copy per staging set (the launch's output buffers are part of it)
    GQArgs two[2] = {gqa, gqa};
    for (int b = 0; b < 2; ++b) {
      two[b].rident = src.rident;
      two[b].rkey0 = nk > 1 ? src.rkeys[0] : src.rident;
      two[b].rowof = P.rowof;
      two[b].oprob = st[b].prob;
      two[b].ocand = st[b].cand;
      two[b].oqidx = st[b].qidx;
      two[b].threshold = P.threshold;
      two[b].maybe = P.maybe;
    }
    HIPCHK(c->gqargs.reserve(sizeof two, 0, s));
    HIPCHK(hipMemcpyAsync(c->gqargs.p, two, sizeof two, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));  // two is a temporary
  } else if (grouped) {
    std::vector<GroupedProp> gp = grouped_props(P);
    // one resource per property while its rows (and the tail rows read past them) stay
    // below 2^32 bytes of offset
    for (const GroupedProp& G : gp)
      if ((uint64_t)(G.w_rows + 8) * G.rowb >= (1ull << 32)) gmode = 1;
    const char* er = getenv("DK_GROUPED_ROW");  // 1 / 2: that form at any size (tests)
    if (er && (er[0] == '1' || er[0] == '2')) gmode = er[0] - '0';
    if (gmode) {
      for (GroupedProp& G : gp) {
        // the head rows' resource: the rows under 4 GiB (>= kGroupedHeadRows of them,
        // grouped_schema_ok); the tail rows' one, or a resource per tail row past 4 GiB
        const uint64_t fit = G.rowb ? ((1ull << 32) - 1) / G.rowb : 0;
        G.w_head = (uint32_t)std::min<uint64_t>(G.w_rows, fit);
        const uint64_t tail = G.w_rows > (uint32_t)kGroupedHeadRows ? (uint64_t)(G.w_rows - kGroupedHeadRows) * G.rowb : 0;
        if (tail >= (1ull << 32)) gmode = 2;
        G.w_tailb = (uint32_t)std::min<uint64_t>(tail, 0xFFFFFFFFull);
      }
    }
    HIPCHK(c->gprops.reserve(gp.size() * sizeof(GroupedProp), 0, s));
    HIPCHK(hipMemcpyAsync(c->gprops.p, gp.data(), gp.size() * sizeof(GroupedProp), hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));  // gp is a temporary
  }
  if (grouped && !(getenv("DK_TASK_SORT") && getenv("DK_TASK_SORT")[0] == '0')) {
    const uint64_t ntask = total / kScoreBlock;
    const int nch = (int)bounds.size() - 1;
    HIPCHK(c->task_key.reserve(ntask * 16 + 16, 0, s));
    HIPCHK(c->task_val.reserve(ntask * 8 + 8, 0, s));
    HIPCHK(c->task_cb.reserve((uint64_t)(nch + 1) * 8, 0, s));
    HIPCHK(c->h_bounds.reserve((uint64_t)(nch + 1) * 8));
    uint64_t* hb = c->h_bounds.as<uint64_t>();
    for (int i = 0; i <= nch; ++i) hb[i] = bounds[i] / kScoreBlock;
    HIPCHK(hipMemcpyAsync(c->task_cb.p, hb, (uint64_t)(nch + 1) * 8, hipMemcpyHostToDevice, s));
    uint64_t* k0 = c->task_key.as<uint64_t>();
    uint32_t* v0 = c->task_val.as<uint32_t>();
    HIPCHK(launch_task_keys(src, ntask, c->task_cb.as<uint64_t>(), nch, k0, v0, s));
    int bits = 32;
    while ((1ll << (bits - 32)) <= nch) ++bits;
    HIPCHK(with_tmp(c, [&](void* t, size_t& b) {
      return sort_pairs_u64_u32_bits(t, b, k0, k0 + ntask, v0, v0 + ntask, ntask, bits, s);
    }));
    perm = v0 + ntask;
    HIPCHK(hipStreamSynchronize(s));  // h_bounds is reused below
  }
  hipStream_t cs = c->copy_stream;
  // Chunk ci scores on the main stream; its block-ordered compaction onto the match list (SYM:
  // its emission's write pass) and (host modes) the copy of its entries run on the copy
  // stream, beside the next chunk's scoring.  Staging set ci&1 (SYM: owner-result half ci&1)
  // is reused by chunk ci+2 once compact_done[ci&1] fired.
  auto compact_chunk = [&](size_t ci) -> int {
    const int b = (int)(ci & 1);
    HIPCHK(hipEventSynchronize(c->count_ready[b]));  // entry count of chunk ci is in hs[]
    const uint64_t nblk = (bounds[ci + 1] - bounds[ci] + kScoreBlock - 1) / kScoreBlock;
    const uint64_t add = hs[4 + 2 * b] + (hs[5 + 2 * b] & 0xFFFFFFFFu);
    if (add || sym) {  // SYM: the write pass also sets the chunk's first[] entries
      const uint64_t need = nm + add;
      // a list that outgrows its buffers is given the whole call's extrapolated size (entries
      // per slot so far x 1.1, at most one per slot): every regrowth copies the list so far
      // and frees the old buffer, which waits for the device
      const uint64_t done = bounds[ci + 1], all = bounds.back();
      const uint64_t want = done < all ? std::max(need, std::min<uint64_t>(all, (uint64_t)((double)need * (double)all / (double)done * 1.1)))
                                       : need;
      auto grow = [&](DevBuf& d, uint64_t el) {
        return d.reserve(((need + 1) * el > d.bytes ? want + 1 : need + 1) * el, nm * el, cs);
      };
      HIPCHK(grow(B.d_cand, 4));
      HIPCHK(grow(B.d_kind, 1));
      HIPCHK(grow(B.d_prob, 8));
      if (!sym) HIPCHK(grow(B.d_qidx, 4));
      MatchList ml{B.d_cand.as<uint32_t>(), B.d_kind.as<uint8_t>(), B.d_prob.as<double>(),
                   B.d_qidx.as<uint32_t>()};
      if (sym) {
        // the write pass on the ctx stream, behind chunk ci+1's scoring (the host waited for
        // chunk ci's count above, which the device reached before that scoring started): the
        // latency-bound pass never shares the CUs with k_score, and the stream never idles
        Timer t_gather(c, &c->prof.ms_gather, s);
        EmitSource e = esrc;  // chunk ci's owner results: half b, indexed by absolute owner slot
        const uint64_t o0 = obounds[ci];
        e.okind = c->okind.as<uint8_t>() + (uint64_t)b * ochunk - (o0 & ~(uint64_t)63);
        e.ores = reinterpret_cast<const double*>(
            reinterpret_cast<uintptr_t>(c->ores.as<double>() + (uint64_t)b * ochunk) - (o0 & ~(uint64_t)63) * sizeof(double));
        HIPCHK(launch_sym_emit(e, bounds[ci], bounds[ci + 1] - bounds[ci], true, nm, ml,
                               B.d_first.as<uint64_t>(), s));
        t_gather.stop();
        HIPCHK(hipEventRecord(c->compact_done[b], s));
        HIPCHK(hipStreamWaitEvent(cs, c->compact_done[b], 0));  // the copies below
      } else {
        HIPCHK(hipStreamWaitEvent(cs, c->count_ready[b], 0));
        Timer t_gather(c, &c->prof.ms_gather, cs);
        HIPCHK(launch_compact(st[b], c->stage[b].boff.as<uint64_t>(), nblk, nm, ml, cs));
        t_gather.stop();
      }
      if (!(flags & DK_MATCH_DEVICE) && add) {
        uint32_t* hc;
        double* hp;
        uint8_t* hk;
        if (c->region.base) {  // caller region (dk_set_result_region)
          if (need > c->region.cap) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamSynchronize(cs);
            return fail(DK_E_NOMEM, "match list needs more than %llu entries; the result region "
                        "holds %llu", (unsigned long long)need, (unsigned long long)c->region.cap);
          }
          hc = c->region.cand;
          hp = c->region.prob;
          hk = c->region.kind;
        } else {  // the pooled pinned buffers
          if (need * 8 > B.h_prob.bytes || need * 4 > B.h_cand.bytes || need > B.h_kind.bytes) {
            HIPCHK(hipStreamSynchronize(cs));
            HIPCHK(B.h_cand.reserve(want * 4, nm * 4));
            HIPCHK(B.h_prob.reserve(want * 8, nm * 8));
            HIPCHK(B.h_kind.reserve(want, nm));
          }
          hc = B.h_cand.as<uint32_t>();
          hp = B.h_prob.as<double>();
          hk = B.h_kind.as<uint8_t>();
        }
        Timer t_copy(c, &c->prof.ms_copy, cs);
        HIPCHK(hipMemcpyAsync(hc + nm, B.d_cand.as<uint32_t>() + nm, add * 4, hipMemcpyDeviceToHost, cs));
        HIPCHK(hipMemcpyAsync(hp + nm, B.d_prob.as<double>() + nm, add * 8, hipMemcpyDeviceToHost, cs));
        HIPCHK(hipMemcpyAsync(hk + nm, B.d_kind.as<uint8_t>() + nm, add, hipMemcpyDeviceToHost, cs));
        t_copy.stop();
      }
      nm = need;
    }
    if (!sym) HIPCHK(hipEventRecord(c->compact_done[b], cs));
    return DK_OK;
  };
  const size_t nchunks = bounds.size() - 1;
  // SYM: chunk ci's owner scoring, its emission's count pass and the scan of the counts run
  // on the ctx stream; its write pass on the copy stream (compact_chunk) beside chunk ci+1's
  // scoring.  Emission of chunk ci reads owner results of chunk ci and mirror results of
  // chunks <= ci only: an owner pushes mirror results to candidates after it in bucket
  // order, i.e. to later queries.
  for (size_t ci = 0; ci < nchunks; ++ci) {
    const int b = (int)(ci & 1);
    const uint64_t s0 = bounds[ci], s1 = bounds[ci + 1];
    const uint64_t nblk = (s1 - s0 + kScoreBlock - 1) / kScoreBlock;
    if (ci >= 2) HIPCHK(hipStreamWaitEvent(s, c->compact_done[b], 0));  // staging / half b drained
    if (sym) {
      // phase 1: the chunk's owner slots, both directions of every owned pair -> okind / ores
      // (half b, indexed by the absolute owner slot o0..o1-1) and the mirror results
      const uint64_t o0 = obounds[ci], o1 = obounds[ci + 1];
      PairSource osrc = src;
      osrc.okind = c->okind.as<uint8_t>() + (uint64_t)b * ochunk - (o0 & ~(uint64_t)63);
      osrc.ores = reinterpret_cast<double*>(
          reinterpret_cast<uintptr_t>(c->ores.as<double>() + (uint64_t)b * ochunk) - (o0 & ~(uint64_t)63) * sizeof(double));
      // k_score_sym2's chunks start inside a wave (packed owner slots): its launch starts at
      // the wave, the slots before o0 are left to the previous chunk
      const uint64_t w0 = o0 & ~(uint64_t)63;
      osrc.olo = o0;
      {
        Timer t_score(c, &c->prof.ms_score, s);
        HIPCHK(launch_score(P, osrc, w0, o1 - w0, so, s));
        t_score.stop();
      }
      HIPCHK(launch_reduce_blocks(so, (o1 - w0 + kScoreBlock - 1) / kScoreBlock, s));
      // phase 2: entries per query of the chunk, their inclusive scan, the chunk's total
      EmitSource e = esrc;
      e.okind = osrc.okind;
      e.ores = osrc.ores;
      Timer t_emit(c, &c->prof.ms_emit, s);
      HIPCHK(launch_sym_emit(e, s0, s1 - s0, false, 0, MatchList{}, nullptr, s));
      HIPCHK(with_tmp(c, [&](void* t, size_t& bytes) {
        return inclusive_scan_u32_u64(t, bytes, c->ecount.as<uint32_t>() + s0, c->eincl.as<uint64_t>() + s0,
                                      s1 - s0, s);
      }));
      hs[5 + 2 * b] = 0;
      HIPCHK(hipMemcpyAsync(&hs[4 + 2 * b], c->eincl.as<uint64_t>() + (s1 - 1), 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipEventRecord(c->count_ready[b], s));
      t_emit.stop();
    } else {
      {
        Timer t_score(c, &c->prof.ms_score, s);
        if (gq)
          HIPCHK(launch_score_gq(P, src, s0, s1 - s0, perm, c->gqargs.as<GQArgs>() + b, gq_nq, gq_nn, gqa.defer, st[b], s));
        else if (grouped)
          HIPCHK(launch_score_grouped(P, src, s0, s1 - s0, perm, c->gprops.as<GroupedProp>(), gmode, st[b], s));
        else HIPCHK(launch_score(P, src, s0, s1 - s0, st[b], s));
        t_score.stop();
      }
      HIPCHK(launch_reduce_blocks(st[b], nblk, s));
      Timer t_gather(c, &c->prof.ms_gather, s);
      HIPCHK(with_tmp(c, [&](void* t, size_t& bytes) {
        return exclusive_scan_u32_u64(t, bytes, st[b].bcnt, c->stage[b].boff.as<uint64_t>(), nblk, s);
      }));
      hs[5 + 2 * b] = 0;
      HIPCHK(hipMemcpyAsync(&hs[4 + 2 * b], c->stage[b].boff.as<uint64_t>() + nblk - 1, 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(&hs[5 + 2 * b], st[b].bcnt + nblk - 1, 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipEventRecord(c->count_ready[b], s));
      t_gather.stop();
    }
    c->prof.score_launches += 1;
    // the previous chunk's count is ready once its scan ran (before this chunk's score
    // started): its compaction and copies are issued while this chunk scores
    if (ci > 0) {
      int rc2 = compact_chunk(ci - 1);
      if (rc2) return rc2;
    }
  }
  if (nchunks) {
    int rc2 = compact_chunk(nchunks - 1);
    if (rc2) return rc2;
    HIPCHK(hipStreamWaitEvent(s, c->compact_done[(nchunks - 1) & 1], 0));  // list complete
  }
  HIPCHK(hipMemcpyAsync(c->h_small.p, c->counters.p, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  {
    const int rg = geo_raise_check(c, P);
    if (rg) return rg;
  }
  lap("score+emit");
  const uint64_t scored = c->h_small.as<uint64_t>()[0];
  const uint64_t sbytes = c->h_small.as<uint64_t>()[1];
  c->prof.pairs_exact += c->h_small.as<uint64_t>()[3];
  if (sym) c->prof.sym_matches += 1;
  if (sym && two) c->prof.sym2_matches += 1;
  R->r.pairs_scored = scored;
  R->r.pairs_generated = generated;
  c->prof.pairs_scored += scored;
  c->prof.pairs_generated += generated;
  c->prof.score_bytes += sbytes;

  // ---- per-query entry offsets, then (DK_MATCH_HOST) the copy into pinned host memory ----
  Timer t_gather(c, &c->prof.ms_gather, s);
  HIPCHK(B.d_first.reserve((nq + 1) * 8, (sym ? nq + 1 : 0) * 8, s));
  if (!sym) HIPCHK(launch_first(B.d_qidx.as<uint32_t>(), nm, nq, B.d_first.as<uint64_t>(), s));
  R->r.nqueries = nq;
  R->r.n = nm;
  if (!(flags & DK_MATCH_DEVICE) && c->region.base) {
    HIPCHK(hipStreamSynchronize(c->copy_stream));  // chunk copies landed
    HIPCHK(hipMemcpyAsync(c->region.first, B.d_first.p, (nq + 1) * 8, hipMemcpyDeviceToHost, s));
    R->r.first = c->region.first;
    R->r.candidate = c->region.cand;
    R->r.prob = c->region.prob;
    R->r.kind = c->region.kind;
  } else if (!(flags & DK_MATCH_DEVICE)) {
    HIPCHK(hipStreamSynchronize(c->copy_stream));  // chunk copies landed
    HIPCHK(B.h_first.reserve((nq + 1) * 8));
    HIPCHK(B.h_cand.reserve(nm * 4 + 4, nm * 4));
    HIPCHK(B.h_prob.reserve(nm * 8 + 8, nm * 8));
    HIPCHK(B.h_kind.reserve(nm + 1, nm));
    HIPCHK(hipMemcpyAsync(B.h_first.p, B.d_first.p, (nq + 1) * 8, hipMemcpyDeviceToHost, s));
    R->r.first = B.h_first.as<uint64_t>();
    R->r.candidate = B.h_cand.as<uint32_t>();
    R->r.prob = B.h_prob.as<double>();
    R->r.kind = B.h_kind.as<uint8_t>();
  }
  HIPCHK(hipStreamSynchronize(s));
  t_gather.stop();
  resolve_spans(c);
  lap("first");
  c->prof.ms_total +=
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return DK_OK;
}

static int group_match(dk_ctx* g, const uint32_t* query_rows, uint64_t nq, int flags, dk_result** out);

static int match_impl(dk_ctx* c, const uint32_t* query_rows, uint64_t nq, int flags, dk_result** out) {
  if (!c || !out) return fail(DK_E_INVALID, "NULL argument");
  *out = nullptr;
  if (!c->members.empty()) return group_match(c, query_rows, nq, flags, out);
  if (nq && !query_rows) return fail(DK_E_INVALID, "query_rows is NULL");
  if (flags & ~DK_MATCH_DEVICE) return fail(DK_E_INVALID, "unknown flags 0x%x", flags);
  HostLap lap("dk_match call");
  bool contiguous = true;  // query rows r0, r0+1, ... (Processor.deduplicate's batch)
  for (uint64_t i = 0; i < nq; ++i) {
    if (query_rows[i] >= c->nrows)
      return fail(DK_E_INVALID, "query row %u not in the index (%llu rows)", query_rows[i],
                  (unsigned long long)c->nrows);
    contiguous = contiguous && query_rows[i] == query_rows[0] + i;
  }
  if (nq >= (1ull << 32)) return fail(DK_E_UNSUPPORTED, "too many queries");
  if (c->region.base && !(flags & DK_MATCH_DEVICE) && nq > c->region.max_queries)
    return fail(DK_E_INVALID, "%llu queries; the result region was laid out for %llu",
                (unsigned long long)nq, (unsigned long long)c->region.max_queries);
  HIPCHK(hipSetDevice(c->device));
  ResultHolder* R = new (std::nothrow) ResultHolder();
  if (!R) return fail(DK_E_NOMEM, "out of host memory");
  R->pool = c->pool;
  R->bufs = c->pool->take();
  R->device = c->device;
  R->stream = c->stream;
  lap("validate");
  int rc = run_match(c, query_rows, nq, flags, R, contiguous);
  lap("run");
  if (rc) {
    R->pool->give(std::move(R->bufs));
    delete R;
    return rc;
  }
  *out = &R->r;
  return DK_OK;
}

int dk_match(dk_ctx* c, const uint32_t* query_rows, uint64_t nq, int flags, dk_result** out) {
  return guarded([&] { return match_impl(c, query_rows, nq, flags, out); });
}

// Per-query candidate counts of the blocking contract (the sum of the query's bucket
// sizes over the key functions, before the isSameAs / duplicate filters): the cost model
// of the multi-GPU query tiles.  ALLPAIRS: every query gets the usable rows.
static int candidate_counts_impl(dk_ctx* c, const uint32_t* query_rows, uint64_t nq, uint64_t* counts) {
  if (!c || (nq && (!query_rows || !counts))) return fail(DK_E_INVALID, "NULL argument");
  if (!c->members.empty()) {
    if (c->broken) return fail(DK_E_STATE, "a replicated update failed on some devices only");
    return candidate_counts_impl(c->members[0], query_rows, nq, counts);
  }
  for (uint64_t i = 0; i < nq; ++i)
    if (query_rows[i] >= c->nrows)
      return fail(DK_E_INVALID, "query row %u not in the index (%llu rows)", query_rows[i],
                  (unsigned long long)c->nrows);
  if (nq == 0) return DK_OK;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  BlockTables T{};
  uint64_t M = 0;
  int rc = ensure_tables(c, &T, &M);
  if (rc) return rc;
  if (c->schema.mode == DK_MODE_ALLPAIRS) {
    for (uint64_t i = 0; i < nq; ++i) counts[i] = M;
    return DK_OK;
  }
  HIPCHK(c->d_queries.reserve(nq * 4 + 4, 0, s));
  HIPCHK(hipMemcpyAsync(c->d_queries.p, query_rows, nq * 4, hipMemcpyHostToDevice, s));
  if (c->luc.on) return lucene_candidates(c, nq, nullptr, nullptr, counts);  // the hits
  HIPCHK(c->ranges.reserve((uint64_t)T.nseg * nq * 8 + 8, 0, s));
  HIPCHK(c->counts.reserve((nq + 1) * 8, 0, s));
  HIPCHK(launch_count_exact(c->d_queries.as<uint32_t>(), nq, T, c->ranges.as<uint2>(),
                            c->counts.as<uint64_t>(), s));
  HIPCHK(hipMemcpyAsync(counts, c->counts.p, nq * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return DK_OK;
}

int dk_candidate_counts(dk_ctx* c, const uint32_t* query_rows, uint64_t nq, uint64_t* counts) {
  return guarded([&] { return candidate_counts_impl(c, query_rows, nq, counts); });
}

int dk_result_copy_to_device(const dk_result* r, uint64_t* first, uint32_t* candidate,
                             double* prob, uint8_t* kind) {
  if (!r) return fail(DK_E_INVALID, "result is NULL");
  const ResultHolder* R = reinterpret_cast<const ResultHolder*>(r);
  if (R->host_only) return fail(DK_E_UNSUPPORTED, "a multi-device ctx's list is in host memory only");
  HIPCHK(hipSetDevice(R->device));
  const ResultBufs& B = *R->bufs;
  hipStream_t s = R->stream;
  if (first) HIPCHK(hipMemcpyAsync(first, B.d_first.p, (r->nqueries + 1) * 8, hipMemcpyDeviceToDevice, s));
  if (r->n) {
    if (candidate) HIPCHK(hipMemcpyAsync(candidate, B.d_cand.p, r->n * 4, hipMemcpyDeviceToDevice, s));
    if (prob) HIPCHK(hipMemcpyAsync(prob, B.d_prob.p, r->n * 8, hipMemcpyDeviceToDevice, s));
    if (kind) HIPCHK(hipMemcpyAsync(kind, B.d_kind.p, r->n, hipMemcpyDeviceToDevice, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  return DK_OK;
}

int dk_result_region_layout(uint64_t bytes, uint64_t max_queries, dk_region_layout* out) {
  if (!out) return fail(DK_E_INVALID, "out is NULL");
  const uint64_t head = (max_queries + 1) * 8;
  if (bytes < head) return fail(DK_E_INVALID, "region of %llu bytes cannot hold %llu queries",
                                (unsigned long long)bytes, (unsigned long long)max_queries);
  const uint64_t cap = (bytes - head) / 13;  // 8 (prob) + 4 (candidate) + 1 (kind) per entry
  out->capacity = cap;
  out->first_offset = 0;
  out->prob_offset = head;
  out->candidate_offset = head + cap * 8;
  out->kind_offset = head + cap * 12;
  return DK_OK;
}

static int set_result_region_impl(dk_ctx* c, void* base, uint64_t bytes, uint64_t max_queries) {
  if (!c) return fail(DK_E_INVALID, "ctx is NULL");
  if (!c->members.empty())
    return fail(DK_E_UNSUPPORTED, "a multi-device ctx writes its list into its own host memory");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->copy_stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (c->region.base) {
    (void)hipHostUnregister(c->region.base);
    c->region = dk_ctx::Region{};
  }
  if (!base) return DK_OK;
  if (reinterpret_cast<uintptr_t>(base) & 7) return fail(DK_E_INVALID, "region base not 8-byte aligned");
  dk_region_layout L{};
  int rc = dk_result_region_layout(bytes, max_queries, &L);
  if (rc) return rc;
  HIPCHK(hipHostRegister(base, bytes, hipHostRegisterDefault));
  uint8_t* b = static_cast<uint8_t*>(base);
  c->region.base = b;
  c->region.bytes = bytes;
  c->region.max_queries = max_queries;
  c->region.cap = L.capacity;
  c->region.first = reinterpret_cast<uint64_t*>(b + L.first_offset);
  c->region.prob = reinterpret_cast<double*>(b + L.prob_offset);
  c->region.cand = reinterpret_cast<uint32_t*>(b + L.candidate_offset);
  c->region.kind = b + L.kind_offset;
  return DK_OK;
}

int dk_set_result_region(dk_ctx* c, void* base, uint64_t bytes, uint64_t max_queries) {
  return guarded([&] { return set_result_region_impl(c, base, bytes, max_queries); });
}

void dk_free_result(dk_result* r) {
  if (!r) return;
  ResultHolder* R = reinterpret_cast<ResultHolder*>(r);  // dk_result is the first member
  (void)hipSetDevice(R->device);
  R->pool->give(std::move(R->bufs));
  delete R;
}

// Processor.compare(r1, r2) of two indexed rows.  The candidate side is a private
// one-position replica (pair_rep) and staging (pair_buf): the blocking tables, their
// replica and the result pools are untouched, so dk_match after a compare reuses them.
static int compare_one(dk_ctx* c, uint32_t r1, uint32_t r2, int raw_prop, double* prob);

static int compare_rows_impl(dk_ctx* c, uint32_t r1, uint32_t r2, double* prob) {
  return compare_one(c, r1, r2, -1, prob);
}

int dk_compare_rows(dk_ctx* c, uint32_t r1, uint32_t r2, double* prob) {
  return guarded([&] { return compare_rows_impl(c, r1, r2, prob); });
}

// Comparator.compare(v1, v2) of property `prop` (the raw similarity PropertyImpl maps to a
// probability) for two indexed rows, through the production scoring kernel.
static int property_similarity_impl(dk_ctx* c, int prop, uint32_t r1, uint32_t r2, double* sim) {
  if (!c || !sim) return fail(DK_E_INVALID, "NULL argument");
  if (prop < 0 || prop >= c->schema.nprops)
    return fail(DK_E_INVALID, "property %d out of range [0, %d)", prop, c->schema.nprops);
  return compare_one(c, r1, r2, prop, sim);
}

int dk_property_similarity(dk_ctx* c, int prop, uint32_t r1, uint32_t r2, double* sim) {
  return guarded([&] { return property_similarity_impl(c, prop, r1, r2, sim); });
}

static int compare_one(dk_ctx* c, uint32_t r1, uint32_t r2, int raw_prop, double* prob) {
  if (!c || !prob) return fail(DK_E_INVALID, "NULL argument");
  if (!c->members.empty()) {
    if (c->broken) return fail(DK_E_STATE, "a replicated update failed on some devices only");
    return compare_one(c->members[0], r1, r2, raw_prop, prob);
  }
  if (r1 >= c->nrows || r2 >= c->nrows) return fail(DK_E_INVALID, "row out of range");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  // pair_buf: [0] query row, [3] rowof[0] (the one replica position); then staging
  HIPCHK(c->pair_buf.reserve(8192, 0, s));
  uint32_t host[4] = {r1, 0u, 0u, r2};
  HIPCHK(hipMemsetAsync(c->pair_buf.p, 0, 8192, s));
  HIPCHK(hipMemcpyAsync(c->pair_buf.p, host, sizeof host, hipMemcpyHostToDevice, s));
  uint8_t* base = c->pair_buf.as<uint8_t>();
  StageOut st{reinterpret_cast<uint64_t*>(base + 64), reinterpret_cast<uint32_t*>(base + 96),
              reinterpret_cast<uint32_t*>(base + 100), reinterpret_cast<uint32_t*>(base + 104),
              reinterpret_cast<double*>(base + 128), reinterpret_cast<uint32_t*>(base + 2176),
              reinterpret_cast<uint32_t*>(base + 3200)};
  const uint32_t* rowof = c->pair_buf.as<uint32_t>() + 3;
  int rc = build_replica(c, c->pair_rep, rowof, 1);
  if (rc) return rc;
  ScoreParams P = make_params(c, c->pair_rep, rowof, 1);
  P.raw_prop = raw_prop;
  P.threshold = -INFINITY;  // every non-NaN probability is emitted
  P.maybe = 0.0;
  PairSource src{};  // one all-pairs slot: query r1 against replica position 0 (row r2)
  src.queries = c->pair_buf.as<uint32_t>();
  src.allpairs = 1;
  src.m = 1;
  src.mpad = 64;
  src.same_ok = 1;  // Processor.compare scores a record against itself too
  rc = geo_raise_clear(c, P);
  if (rc) return rc;
  HIPCHK(launch_score(P, src, 0, 1, st, s));
  uint32_t n = 0;
  double p = NAN;
  HIPCHK(hipMemcpyAsync(&n, base + 96, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(&p, base + 128, 8, hipMemcpyDeviceToHost, s));
  // Levenshtein's raw similarity: Duke's own early-exit value (the fused kernel's cut-off
  // distance differs from it; the probability it feeds does not)
  double lev = NAN;
  if (raw_prop >= 0 && c->P[raw_prop].cfg.comparator == DK_CMP_LEVENSHTEIN) {
    const PropState& S = c->P[raw_prop];
    HIPCHK(launch_lev_exact(S.off.as<uint32_t>(), S.len.as<uint16_t>(), S.units.p, S.width, r1, r2,
                            reinterpret_cast<double*>(base + 120), s));
    HIPCHK(hipMemcpyAsync(&lev, base + 120, 8, hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  rc = geo_raise_check(c, P);
  if (rc) return rc;
  *prob = n ? (lev == lev ? lev : p) : NAN;
  return DK_OK;
}

// Processor.compare(Record, Record) for two records that need not be indexed (SURVEY §8b
// dk_compare_pair): the pair is packed into a private 2-row ALLPAIRS index with the same
// properties (created on first use, emptied per call) and scored there.
static void clear_index(dk_ctx* c) {
  c->nrows = 0;
  c->index_gen++;
  c->base_ok = false;
  c->base_dead.clear();
  if (c->luc.on) {
    c->luc.qoff.assign(1, 0);
    c->luc.npost = 0;
    for (auto& d : c->luc.dict) d.clear();
  }
  c->ident_row.clear();
  for (auto& t : c->intern) t.clear();
  c->key_style = 0;
  c->transient = false;
  for (auto& p : c->P) {
    p.units_used = p.grams_used = 0;
    p.maxlen = p.maxgrams = 0;
    p.tokens.clear();
  }
}

static int compare_values_impl(dk_ctx* c, const dk_batch* pair, double* prob) {
  if (!c || !pair || !prob) return fail(DK_E_INVALID, "NULL argument");
  if (!c->members.empty()) return compare_values_impl(c->members[0], pair, prob);
  if (pair->n != 2) return fail(DK_E_INVALID, "dk_compare_values takes a batch of 2 records (r1, r2)");
  if (!c->pair_ctx) {
    std::vector<dk_property> props(c->P.size());
    for (size_t i = 0; i < c->P.size(); ++i) props[i] = c->P[i].cfg;
    dk_schema sc = c->schema;
    sc.props = props.data();
    sc.orders = c->orders.empty() ? nullptr : c->orders.data();
    sc.mode = DK_MODE_ALLPAIRS;
    sc.nkeys = 0;
    int rc = dk_create(&sc, c->device, &c->pair_ctx);
    if (rc) return rc;
  }
  dk_ctx* pc = c->pair_ctx;
  clear_index(pc);
  dk_batch b = *pair;
  const uint64_t ident[2] = {0, 1};  // Processor.compare does not apply isSameAs
  b.ident = ident;
  b.group = nullptr;
  b.deleted = nullptr;
  b.keys = nullptr;
  b.key_columns = nullptr;
  int rc = upsert_rows(pc, &b, nullptr, false);
  if (rc) return rc;
  return dk_compare_rows(pc, 0, 1, prob);
}

int dk_compare_values(dk_ctx* c, const dk_batch* pair, double* prob) {
  return guarded([&] { return compare_values_impl(c, pair, prob); });
}

int dk_set_overwrite(dk_ctx* c, int on) {
  if (!c) return fail(DK_E_INVALID, "ctx is NULL");
  c->overwrite = on != 0;
  for (dk_ctx* m : c->members) m->overwrite = on != 0;
  return DK_OK;
}

// ----------------------------------------------------------------------------------------
// dk_create_multi: one handle over several devices (include/dukehip.h).  Members are plain
// ctxs; the group fans updates out on one host thread per member and splits dk_match into
// cost-balanced contiguous query tiles, then gathers the tiles' device lists into
// one pinned host list, each member copying its slice over its own host link.
// ----------------------------------------------------------------------------------------
static int create_multi_impl(const dk_schema* schema, const int* devices, int ndev, dk_ctx** out) {
  if (!out) return fail(DK_E_INVALID, "out is NULL");
  *out = nullptr;
  if (!devices || ndev < 1) return fail(DK_E_INVALID, "no devices");
  if (ndev == 1) return create_impl(schema, devices[0], out);
  std::unique_ptr<dk_ctx> g(new dk_ctx());
  for (int i = 0; i < ndev; ++i) {
    dk_ctx* m = nullptr;
    const int rc = create_impl(schema, devices[i], &m);
    if (rc) {
      for (dk_ctx* x : g->members) dk_destroy(x);
      g->members.clear();
      return rc;
    }
    g->members.push_back(m);
  }
  g->schema = g->members[0]->schema;
  g->device = devices[0];
  *out = g.release();
  return DK_OK;
}

int dk_create_multi(const dk_schema* schema, const int* devices, int ndev, dk_ctx** out) {
  return guarded([&] { return create_multi_impl(schema, devices, ndev, out); });
}

// f on every member, one host thread each.  The replicas stay identical when every member
// returns the same status (a batch is validated identically everywhere); otherwise the
// group is marked broken.
static int group_each(dk_ctx* g, int (*f)(dk_ctx*, void*), void* arg) {
  if (g->broken) return fail(DK_E_STATE, "a replicated update failed on some devices only");
  const int nd = (int)g->members.size();
  std::vector<int> rc(nd, DK_OK);
  std::vector<std::string> msg(nd);
  dk_run_parts(nd, [&](int i) {
    rc[i] = guarded([&] { return f(g->members[i], arg); });
    if (rc[i]) msg[i] = g_err;
  });
  for (int i = 1; i < nd; ++i)
    if (rc[i] != rc[0]) {
      g->broken = true;
      const int bad = rc[0] ? 0 : i;
      return fail(DK_E_STATE, "device %d of %d diverged (%d): %s", bad, nd, rc[bad], msg[bad].c_str());
    }
  if (rc[0]) g_err = msg[0];
  return rc[0];
}

struct GroupUpsert {
  const dk_batch* b;
  bool transient;
  const std::vector<dk_ctx*>* members;
  std::vector<std::vector<uint32_t>> rows;  // per member
};

static int upsert_member(dk_ctx* m, void* a) {
  GroupUpsert* u = static_cast<GroupUpsert*>(a);
  const size_t i = (size_t)(std::find(u->members->begin(), u->members->end(), m) - u->members->begin());
  u->rows[i].resize(u->b->n);
  return upsert_rows(m, u->b, u->rows[i].data(), u->transient);
}

static int group_upsert(dk_ctx* g, const dk_batch* b, uint32_t* rows_out, bool transient) {
  GroupUpsert u{b, transient, &g->members, std::vector<std::vector<uint32_t>>(g->members.size())};
  const int rc = group_each(g, upsert_member, &u);
  if (rc) return rc;
  for (size_t i = 1; i < u.rows.size(); ++i)
    if (u.rows[i] != u.rows[0]) {
      g->broken = true;
      return fail(DK_E_STATE, "device %zu assigned other rows", i);
    }
  if (rows_out && b->n) memcpy(rows_out, u.rows[0].data(), b->n * 4);
  return DK_OK;
}

static int group_match(dk_ctx* g, const uint32_t* q, uint64_t nq, int flags, dk_result** out) {
  const auto t0 = std::chrono::steady_clock::now();
  if (g->broken) return fail(DK_E_STATE, "a replicated update failed on some devices only");
  if (nq && !q) return fail(DK_E_INVALID, "query_rows is NULL");
  if (flags & DK_MATCH_DEVICE)
    return fail(DK_E_UNSUPPORTED, "a multi-device ctx hands its list over in host memory");
  if (flags) return fail(DK_E_INVALID, "unknown flags 0x%x", flags);
  const int nd = (int)g->members.size();
  // contiguous tiles of equal estimated cost: the query's candidates + one padded wave
  // (dukehip.dist.cost_bounds); every member holds the same index, so member 0 counts
  std::vector<uint64_t> bound(nd + 1, nq);
  bound[0] = 0;
  if (nq) {
    std::vector<uint64_t> cnt(nq);
    const int rc = candidate_counts_impl(g->members[0], q, nq, cnt.data());
    if (rc) return rc;
    double total = 0.0;
    for (uint64_t i = 0; i < nq; ++i) total += (double)cnt[i] + 32.0;
    double acc = 0.0;
    int t = 1;
    for (uint64_t i = 0; i < nq && t < nd; ++i) {
      while (t < nd && acc >= total * t / nd) bound[t++] = i;
      acc += (double)cnt[i] + 32.0;
    }
  }
  std::vector<dk_result*> part(nd, nullptr);
  std::vector<int> rc(nd, DK_OK);
  std::vector<std::string> msg(nd);
  dk_run_parts(nd, [&](int i) {
    rc[i] = guarded([&] {
      return match_impl(g->members[i], q + bound[i], bound[i + 1] - bound[i], DK_MATCH_DEVICE, &part[i]);
    });
    if (rc[i]) msg[i] = g_err;
  });
  auto release = [&] {
    for (dk_result*& r : part) {
      dk_free_result(r);
      r = nullptr;
    }
  };
  for (int i = 0; i < nd; ++i)
    if (rc[i]) {
      release();
      g_err = msg[i];
      return rc[i];
    }
  std::vector<uint64_t> base(nd + 1, 0);
  uint64_t scored = 0, generated = 0;
  for (int i = 0; i < nd; ++i) {
    base[i + 1] = base[i] + part[i]->n;
    scored += part[i]->pairs_scored;
    generated += part[i]->pairs_generated;
  }
  const uint64_t n = base[nd];
  std::unique_ptr<ResultHolder> R(new ResultHolder());
  R->pool = g->pool;
  R->bufs = g->pool->take();
  R->device = g->device;
  R->host_only = true;
  ResultBufs& B = *R->bufs;
  hipError_t e = B.h_first.reserve((nq + 1) * 8);
  if (e == hipSuccess) e = B.h_cand.reserve(n * 4 + 4);
  if (e == hipSuccess) e = B.h_prob.reserve(n * 8 + 8);
  if (e == hipSuccess) e = B.h_kind.reserve(n + 1);
  if (e != hipSuccess) {
    release();
    R->pool->give(std::move(R->bufs));
    return fail(DK_E_NOMEM, "pinned host memory for the list: %s", hipGetErrorString(e));
  }
  // every member copies its tile's list into its slice, on its own stream and host link
  dk_run_parts(nd, [&](int i) {
    rc[i] = guarded([&] {
      const ResultHolder* P = reinterpret_cast<const ResultHolder*>(part[i]);
      const ResultBufs& D = *P->bufs;
      const uint64_t nqi = bound[i + 1] - bound[i], ni = part[i]->n;
      HIPCHK(hipSetDevice(P->device));
      hipStream_t s = P->stream;
      if (nqi)
        HIPCHK(hipMemcpyAsync(B.h_first.as<uint64_t>() + bound[i], D.d_first.p, nqi * 8, hipMemcpyDeviceToHost, s));
      if (ni) {
        HIPCHK(hipMemcpyAsync(B.h_cand.as<uint32_t>() + base[i], D.d_cand.p, ni * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(B.h_prob.as<double>() + base[i], D.d_prob.p, ni * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(B.h_kind.as<uint8_t>() + base[i], D.d_kind.p, ni, hipMemcpyDeviceToHost, s));
      }
      HIPCHK(hipStreamSynchronize(s));
      uint64_t* f = B.h_first.as<uint64_t>() + bound[i];
      for (uint64_t k = 0; k < nqi; ++k) f[k] += base[i];  // tile-local -> list offsets
      return DK_OK;
    });
    if (rc[i]) msg[i] = g_err;
  });
  release();
  for (int i = 0; i < nd; ++i)
    if (rc[i]) {
      R->pool->give(std::move(R->bufs));
      g_err = msg[i];
      return rc[i];
    }
  B.h_first.as<uint64_t>()[nq] = n;
  dk_result& r = R->r;
  r.nqueries = nq;
  r.n = n;
  r.first = B.h_first.as<uint64_t>();
  r.candidate = B.h_cand.as<uint32_t>();
  r.prob = B.h_prob.as<double>();
  r.kind = B.h_kind.as<uint8_t>();
  r.pairs_scored = scored;
  r.pairs_generated = generated;
  if (g->profiling)
    g->prof.ms_total += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out = &R.release()->r;
  return DK_OK;
}
