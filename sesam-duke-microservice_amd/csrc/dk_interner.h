// dk_interner.h — exact UTF-16 string interning for the host-side units: record IDs (native
// ingestion, the link database) and blocking-key strings (dk_upsert).  Not part of the ABI.
//
// An open-addressing table over a string arena: ids are dense in first-insertion order.
// The slot array is split into kShards shards by the hash's top bits, so a batch is
// interned shard-parallel (intern_batch): each worker probes / inserts the batch's strings
// of its shards in batch order under provisional ids, one sequential pass over the batch
// then numbers the new strings in first-appearance order, and the workers patch their
// slots and copy the new strings into the arena.  A slot holds the hash's high half as a
// tag plus id + 1, so a probe compares units only on a tag hit.
#pragma once

#include <sys/mman.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <new>
#include <thread>
#include <vector>

// f(i) for i < n, parts 1.. on their own threads and part 0 on the caller's.  Exception-safe:
// a thread that cannot be started runs its part on the caller instead, every started thread
// is joined, and the first exception any part threw is rethrown on the caller afterwards (an
// exception escaping a std::thread would std::terminate the host process -- the JVM).
template <typename F>
inline void dk_run_parts(int n, F&& f) {
  if (n <= 1) {
    if (n == 1) f(0);
    return;
  }
  std::vector<std::exception_ptr> err((size_t)n);
  auto part = [&](int i) {
    try {
      f(i);
    } catch (...) {
      err[(size_t)i] = std::current_exception();
    }
  };
  std::vector<std::thread> th;
  int started = 1;
  try {
    th.reserve((size_t)n - 1);
    for (; started < n; ++started) th.emplace_back(part, started);
  } catch (...) {
    // no more threads: the remaining parts run here
  }
  part(0);
  for (int i = started; i < n; ++i) part(i);
  for (auto& t : th) t.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}

// A growable array of trivially copyable T whose growth leaves the new tail unwritten, so
// the workers that fill it also take its first-touch page faults, in parallel.
template <typename T>
struct PodVec {
  T* p = nullptr;
  uint64_t n = 0, cap = 0;
  PodVec() = default;
  PodVec(const PodVec&) = delete;
  PodVec& operator=(const PodVec&) = delete;
  PodVec(PodVec&& o) noexcept : p(o.p), n(o.n), cap(o.cap) { o.p = nullptr; o.n = o.cap = 0; }
  PodVec& operator=(PodVec&& o) noexcept {
    std::swap(p, o.p);
    std::swap(n, o.n);
    std::swap(cap, o.cap);
    return *this;
  }
  ~PodVec() { free(p); }
  // large arrays on 2 MB-aligned transparent huge pages: a 1M-record batch first-touches a
  // few dozen pages instead of ~10^4 (page faults dominate a cold batch otherwise)
  static T* alloc(uint64_t c) {
    const size_t bytes = (size_t)c * sizeof(T);
    void* q = nullptr;
    if (bytes >= (4u << 20)) {
      if (posix_memalign(&q, 2u << 20, bytes)) throw std::bad_alloc();
      (void)madvise(q, bytes, MADV_HUGEPAGE);
    } else {
      q = malloc(bytes ? bytes : 1);
      if (!q) throw std::bad_alloc();
    }
    return static_cast<T*>(q);
  }
  uint64_t size() const { return n; }
  T* data() { return p; }
  const T* data() const { return p; }
  T& operator[](uint64_t i) { return p[i]; }
  const T& operator[](uint64_t i) const { return p[i]; }
  void clear() { n = 0; }
  void reserve(uint64_t c) {  // geometric: streams of small batches stay linear
    if (c <= cap) return;
    c = std::max<uint64_t>(c, 2 * cap);
    T* q = alloc(c);  // uninitialised: no writes
    if (n) memcpy(q, p, n * sizeof(T));
    free(p);
    p = q;
    cap = c;
  }
  // reserve, the old contents copied by T threads (a 10M-ID arena is hundreds of MB)
  void reserve_par(uint64_t c, int threads) {
    if (c <= cap) return;
    c = std::max<uint64_t>(c, 2 * cap);
    T* q = alloc(c);
    const uint64_t bytes = n * sizeof(T), parts = bytes >= (64u << 20) ? (uint64_t)std::max(1, threads) : 1;
    dk_run_parts((int)parts, [&](int t) {
      const uint64_t a = bytes * t / parts, b = bytes * (t + 1) / parts;
      if (b > a) memcpy(reinterpret_cast<char*>(q) + a, reinterpret_cast<const char*>(p) + a, b - a);
    });
    free(p);
    p = q;
    cap = c;
  }
  void resize_uninit(uint64_t m) {
    reserve(m);
    n = m;
  }
  void reset_uninit(uint64_t m) {  // m elements, old contents dropped, nothing written
    if (m > cap) {
      T* q = alloc(m);  // first: a failed allocation leaves the vector as it was
      free(p);
      p = q;
      cap = m;
    }
    n = m;
  }
  void push_back(const T& v) {
    reserve(n + 1);
    p[n++] = v;
  }
  void append(const T* v, uint64_t m) {
    reserve(n + m);
    if (m) memcpy(p + n, v, m * sizeof(T));
    n += m;
  }
};

struct U16Table {
  static constexpr int kShardBits = 4, kShards = 1 << kShardBits;
  static constexpr uint32_t kProv = 0x80000000u;  // slot id field: batch index of a new string
  static constexpr uint64_t kAhead = 8;            // slot prefetch distance of the batch probes

  PodVec<char16_t> arena;
  PodVec<uint64_t> start;          // id -> [start[id], start[id + 1]) in the arena
  PodVec<uint64_t> hashes;         // id -> its hash (rehash without re-reading strings)
  PodVec<uint64_t> slots;          // kShards x shard_cap: (tag << 32) | (id + 1); 0 = empty
  uint64_t shard_cap = 0;          // power of two
  uint64_t fill[kShards] = {};

  U16Table() { start.push_back(0); }

  static uint64_t hash(const char16_t* s, uint64_t n) {
    // 8-byte words, multiply-xorshift mixing; the length seeds it ("" != "\0")
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xC2B2AE3D27D4EB4Full);
    const uint8_t* p = reinterpret_cast<const uint8_t*>(s);
    uint64_t nb = n * 2, w;
    for (; nb >= 8; nb -= 8, p += 8) {
      memcpy(&w, p, 8);
      h = (h ^ w) * 0xFF51AFD7ED558CCDull;
      h ^= h >> 29;
    }
    w = 0;
    memcpy(&w, p, nb);
    h = (h ^ w) * 0xC4CEB9FE1A85EC53ull;
    h ^= h >> 32;
    h *= 0x9E3779B97F4A7C15ull;
    return h ^ (h >> 29);
  }
  static int shard_of(uint64_t h) { return (int)(h >> (64 - kShardBits)); }

  uint64_t size() const { return hashes.size(); }
  const char16_t* str(uint64_t id) const { return arena.data() + start[id]; }
  uint64_t len(uint64_t id) const { return start[id + 1] - start[id]; }
  void clear() {
    arena.clear();
    start.clear();
    start.push_back(0);
    hashes.clear();
    slots.clear();
    shard_cap = 0;
    std::fill(fill, fill + kShards, 0);
  }

  bool find(const char16_t* s, uint64_t n, uint64_t h, uint64_t* id) const {
    if (!shard_cap) return false;
    const uint64_t* sh = slots.data() + (uint64_t)shard_of(h) * shard_cap;
    const uint64_t m = shard_cap - 1, tag = h >> 32;
    for (uint64_t i = h & m;; i = (i + 1) & m) {
      const uint64_t e = sh[i];
      if (!e) return false;
      if ((e >> 32) == tag) {
        const uint64_t x = (uint32_t)e - 1;
        if (len(x) == n && (n == 0 || memcmp(str(x), s, n * 2) == 0)) {
          *id = x;
          return true;
        }
      }
    }
  }
  bool find(const char16_t* s, uint64_t n, uint64_t* id) const { return find(s, n, hash(s, n), id); }

  // the id of s, interned if new
  uint64_t find_or_add(const char16_t* s, uint64_t n, uint64_t h) {
    uint64_t id;
    if (find(s, n, h, &id)) return id;
    id = size();
    const int sh = shard_of(h);
    ensure_shard(sh, fill[sh] + 1);
    arena.append(s, n);
    start.push_back(arena.size());
    hashes.push_back(h);
    place(h, id);
    return id;
  }
  uint64_t find_or_add(const char16_t* s, uint64_t n) { return find_or_add(s, n, hash(s, n)); }

  // out[i] = id of string i (ptr[i], n[i], hash h[i]); new strings get ids in the order of
  // their first appearance in the batch, exactly as n sequential find_or_add calls would
  void intern_batch(uint64_t cnt, const char16_t* const* ptr, const uint32_t* n, const uint64_t* h,
                    uint64_t* out, int threads) {
    if (cnt < 4096 || threads <= 1) {
      for (uint64_t i = 0; i < cnt; ++i) out[i] = find_or_add(ptr[i], n[i], h[i]);
      return;
    }
    const int T = std::min(threads, kShards);
    // the batch's indices per shard, in batch order (parallel counting sort)
    std::vector<uint64_t> cnts((size_t)T * kShards, 0);
    run(T, [&](int t) {
      uint64_t* c = cnts.data() + (size_t)t * kShards;
      for (uint64_t i = cnt * t / T; i < cnt * (t + 1) / T; ++i) ++c[shard_of(h[i])];
    });
    std::vector<uint64_t> base((size_t)T * kShards), shard_lo(kShards + 1, 0);
    uint64_t acc = 0;
    for (int s = 0; s < kShards; ++s) {
      shard_lo[s] = acc;
      for (int t = 0; t < T; ++t) {
        base[(size_t)t * kShards + s] = acc;
        acc += cnts[(size_t)t * kShards + s];
      }
    }
    shard_lo[kShards] = acc;
    // order[k]: the batch index at shard-order position k; oh[k] its hash, so the probe
    // passes read the hashes in sequence (prefetching the slots ahead) instead of gathering
    PodVec<uint32_t> order;
    PodVec<uint64_t> oh;
    PodVec<const char16_t*> op;  // and its string (prefetched ahead: a hit compares it)
    order.reset_uninit(cnt);
    oh.reset_uninit(cnt);
    op.reset_uninit(cnt);
    run(T, [&](int t) {
      uint64_t* b = base.data() + (size_t)t * kShards;
      for (uint64_t i = cnt * t / T; i < cnt * (t + 1) / T; ++i) {
        const uint64_t k = b[shard_of(h[i])]++;
        order[k] = (uint32_t)i;
        oh[k] = h[i];
        op[k] = ptr[i];
      }
    });
    // room for the batch's new strings (load <= 1/2 per shard): bounded by the batch's count
    // per shard, or -- when that bound would grow the table -- by a read-only lookup pass
    // first (a re-posted batch then never grows it)
    uint64_t need = 0;
    for (int s = 0; s < kShards; ++s) need = std::max(need, fill[s] + (shard_lo[s + 1] - shard_lo[s]));
    std::vector<char> known;  // per order position: found by the lookup pass (out[] set)
    if (shard_cap && 2 * need > shard_cap) {
      known.assign(cnt, 0);
      std::vector<uint64_t> miss(kShards, 0);
      run(T, [&](int t) {
        for (int s = t; s < kShards; s += T) {
          const uint64_t* sh = slots.data() + (uint64_t)s * shard_cap;
          uint64_t ms = 0;  // a local count: the shared array would bounce between workers
          for (uint64_t k = shard_lo[s]; k < shard_lo[s + 1]; ++k) {
            if (k + kAhead < shard_lo[s + 1]) {
              __builtin_prefetch(sh + (oh[k + kAhead] & (shard_cap - 1)));
              __builtin_prefetch(op[k + kAhead]);
            }
            const uint32_t i = order[k];
            uint64_t id;
            if (find(op[k], n[i], oh[k], &id)) {
              out[i] = id;
              known[k] = 1;
            } else {
              ++ms;
            }
          }
          miss[s] = ms;
        }
      });
      need = 0;
      for (int s = 0; s < kShards; ++s) need = std::max(need, fill[s] + miss[s]);
    }
    ensure_all(need, T);
    // Every allocation happens before the first provisional slot is written (the workers
    // and the numbering pass below allocate nothing): a std::bad_alloc leaves the table as
    // it was.  Worst case: every string of the batch is new.
    // slot positions of new strings: shard s's at placed[shard_lo[s] ..], placed_n[s] of them
    // (the workers keep their counts local: adjacent shared counters would bounce)
    PodVec<uint64_t> placed;
    placed.reset_uninit(cnt);
    std::vector<uint64_t> placed_n(kShards, 0);
    uint64_t units_max = 0;
    for (uint64_t i = 0; i < cnt; ++i) units_max += n[i];
    arena.reserve_par(arena.size() + units_max, T);
    start.reserve_par(start.size() + cnt, T);
    hashes.reserve_par(hashes.size() + cnt, T);
    std::vector<uint32_t> fresh;
    fresh.reserve(cnt);
    std::vector<uint64_t> rfresh(T + 1, 0), runits(T + 1, 0);  // the numbering's range prefixes
    // per shard, in batch order: existing id, or provisional (kProv | first index)
    run(T, [&](int t) {
      for (int s = t; s < kShards; s += T) {
        uint64_t* sh = slots.data() + (uint64_t)s * shard_cap;
        const uint64_t m = shard_cap - 1, k1 = shard_lo[s + 1];
        uint64_t* pl = placed.data() + shard_lo[s];
        uint64_t npl = 0;
        for (uint64_t k = shard_lo[s]; k < k1; ++k) {
          if (k + kAhead < k1) {
            __builtin_prefetch(sh + (oh[k + kAhead] & m), 1);
            __builtin_prefetch(op[k + kAhead]);
          }
          if (!known.empty() && known[k]) continue;
          const uint32_t i = order[k];
          const uint64_t hh = oh[k], tag = hh >> 32;
          uint64_t pos = hh & m;
          for (;; pos = (pos + 1) & m) {
            const uint64_t e = sh[pos];
            if (!e) {
              sh[pos] = (tag << 32) | (kProv | i);
              pl[npl++] = pos;
              out[i] = kProv | (uint64_t)i;
              break;
            }
            if ((e >> 32) != tag) continue;
            const uint32_t v = (uint32_t)e;
            if (v & kProv) {
              const uint32_t j = v & ~kProv;
              if (n[j] == n[i] && (n[i] == 0 || memcmp(ptr[j], ptr[i], (size_t)n[i] * 2) == 0)) {
                out[i] = kProv | (uint64_t)j;
                break;
              }
            } else {
              const uint64_t x = v - 1;
              if (len(x) == n[i] && (n[i] == 0 || memcmp(str(x), ptr[i], (size_t)n[i] * 2) == 0)) {
                out[i] = x;
                break;
              }
            }
          }
        }
        placed_n[s] = npl;
        fill[s] += npl;
      }
    });
    uint64_t nplaced = 0;
    for (int s = 0; s < kShards; ++s) nplaced += placed_n[s];
    if (nplaced == 0) return;  // every string was known (a re-posted batch): out[] is final
    // number the new strings in first-appearance order: per batch range, its first
    // appearances counted, then numbered from the range's prefix, then the repeats copy
    // their first appearance's id (final by then)
    const uint64_t id0 = size();
    run(T, [&](int t) {
      uint64_t f = 0, u = 0;
      for (uint64_t i = cnt * t / T; i < cnt * (t + 1) / T; ++i)
        if (out[i] == (kProv | i)) {
          ++f;
          u += n[i];
        }
      rfresh[t + 1] = f;
      runits[t + 1] = u;
    });
    for (int t = 0; t < T; ++t) {
      rfresh[t + 1] += rfresh[t];
      runits[t + 1] += runits[t];
    }
    const uint64_t units = runits[T];
    fresh.resize(rfresh[T]);
    run(T, [&](int t) {
      uint64_t f = rfresh[t];
      for (uint64_t i = cnt * t / T; i < cnt * (t + 1) / T; ++i)
        if (out[i] == (kProv | i)) {
          out[i] = id0 + f;
          fresh[f++] = (uint32_t)i;
        }
    });
    run(T, [&](int t) {
      for (uint64_t i = cnt * t / T; i < cnt * (t + 1) / T; ++i)
        if (out[i] & kProv) out[i] = out[out[i] & ~(uint64_t)kProv];
    });
    // slots, ids -> strings, arena
    const uint64_t a0 = arena.size();
    arena.resize_uninit(a0 + units);
    start.resize_uninit(start.size() + fresh.size());
    hashes.resize_uninit(id0 + fresh.size());
    uint64_t at = a0;
    for (size_t f = 0; f < fresh.size(); ++f) {
      at += n[fresh[f]];
      start[id0 + 1 + f] = at;
    }
    run(T, [&](int t) {
      for (int s = t; s < kShards; s += T) {
        uint64_t* sh = slots.data() + (uint64_t)s * shard_cap;
        const uint64_t* pl = placed.data() + shard_lo[s];
        for (uint64_t q = 0; q < placed_n[s]; ++q) {
          if (q + kAhead < placed_n[s]) __builtin_prefetch(sh + pl[q + kAhead], 1);
          const uint64_t pos = pl[q];
          const uint32_t i = (uint32_t)sh[pos] & ~kProv;
          sh[pos] = (sh[pos] & ~0xFFFFFFFFull) | (out[i] + 1);
        }
      }
      for (size_t f = fresh.size() * t / T; f < fresh.size() * (t + 1) / T; ++f) {
        const uint32_t i = fresh[f];
        hashes[id0 + f] = h[i];
        if (n[i]) memcpy(arena.data() + start[id0 + f], ptr[i], (size_t)n[i] * 2);
      }
    });
  }

  // String.compareTo order of two ids (UTF-16 units, unsigned)
  int compare(uint64_t a, uint64_t b) const {
    const uint64_t la = len(a), lb = len(b), m = la < lb ? la : lb;
    const char16_t *x = str(a), *y = str(b);
    for (uint64_t i = 0; i < m; ++i)
      if (x[i] != y[i]) return x[i] < y[i] ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
  }

 private:
  template <typename F>
  static void run(int T, F&& f) {
    dk_run_parts(T, f);
  }
  void place(uint64_t h, uint64_t id) {
    const int s = shard_of(h);
    uint64_t* sh = slots.data() + (uint64_t)s * shard_cap;
    const uint64_t m = shard_cap - 1;
    uint64_t i = h & m;
    while (sh[i]) i = (i + 1) & m;
    sh[i] = ((h >> 32) << 32) | (id + 1);
    ++fill[s];
  }
  void ensure_shard(int, uint64_t n) { ensure_all(n, 1); }
  // every shard holds n entries at load <= 1/2 (all shards share one capacity); a growth
  // leaves load <= 1/4, so a next batch as large as this one neither rehashes nor needs the
  // lookup pass (a cold database taking two 10M-record bodies rehashed 10M IDs otherwise)
  void ensure_all(uint64_t n, int T) {
    if (shard_cap && 2 * n <= shard_cap) return;
    uint64_t cap = shard_cap ? shard_cap : 64;
    while (cap < 4 * n) cap *= 2;
    slots.reset_uninit((uint64_t)kShards * cap);
    shard_cap = cap;
    std::fill(fill, fill + kShards, 0);
    // zero and refill the shards in parallel (each worker owns whole shards)
    const uint64_t nid = size();
    const int TT = std::max(1, std::min(T, kShards));
    run(TT, [&](int t) {
      for (int s = t; s < kShards; s += TT) memset(slots.data() + (uint64_t)s * cap, 0, cap * 8);
      for (uint64_t id = 0; id < nid; ++id) {
        const int s = shard_of(hashes[id]);
        if (s % TT != t) continue;
        uint64_t* sh = slots.data() + (uint64_t)s * cap;
        uint64_t i = hashes[id] & (cap - 1);
        while (sh[i]) i = (i + 1) & (cap - 1);
        sh[i] = ((hashes[id] >> 32) << 32) | (id + 1);
        ++fill[s];
      }
    });
  }
};

// the record-ID interner handle of the C-ABI (dk_interner_*)
struct dk_interner : U16Table {};
