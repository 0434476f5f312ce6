// dk_interner.h — exact UTF-16 string interning for the host-side units: record IDs (native
// ingestion, the link database) and blocking-key strings (dk_upsert).  Not part of the ABI.
//
// One open-addressing table over a string arena: ids are dense in first-insertion order, a
// slot holds the hash's high half as a tag plus id + 1, so a probe touches one cache line of
// slots and compares units only on a tag hit.  Hashes are computed by the caller (ingestion
// workers hash their records in parallel; the ordered insert is then one sequential pass).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

struct U16Table {
  std::vector<char16_t> arena;
  std::vector<uint64_t> start{0};  // id -> [start[id], start[id + 1]) in the arena
  std::vector<uint64_t> hashes;    // id -> its hash (rehash without re-reading strings)
  std::vector<uint64_t> slots;     // (tag << 32) | (id + 1); 0 = empty
  uint64_t mask = 0;

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

  uint64_t size() const { return hashes.size(); }
  const char16_t* str(uint64_t id) const { return arena.data() + start[id]; }
  uint64_t len(uint64_t id) const { return start[id + 1] - start[id]; }
  void clear() {
    arena.clear();
    start.assign(1, 0);
    hashes.clear();
    slots.clear();
    mask = 0;
  }
  // room for nstrings more strings of nunits units in total (geometric, so a stream of small
  // batches into a large table does not copy the arena each time)
  void reserve(uint64_t nstrings, uint64_t nunits) {
    auto room = [](auto& v, uint64_t add) {
      if (v.capacity() < v.size() + add) v.reserve(std::max<uint64_t>(v.size() + add, 2 * v.capacity()));
    };
    room(arena, nunits);
    room(start, nstrings);
    room(hashes, nstrings);
    grow_to(size() + nstrings);
  }

  bool find(const char16_t* s, uint64_t n, uint64_t h, uint64_t* id) const {
    if (slots.empty()) return false;
    const uint64_t tag = h >> 32;
    for (uint64_t i = h & mask;; i = (i + 1) & mask) {
      const uint64_t e = slots[i];
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

  // the id of s, interned if new (ids < 2^32 - 1; the callers bound their tables far below)
  uint64_t find_or_add(const char16_t* s, uint64_t n, uint64_t h) {
    uint64_t id;
    if (find(s, n, h, &id)) return id;
    id = size();
    grow_to(id + 1);
    arena.insert(arena.end(), s, s + n);
    start.push_back(arena.size());
    hashes.push_back(h);
    place(h, id);
    return id;
  }
  uint64_t find_or_add(const char16_t* s, uint64_t n) { return find_or_add(s, n, hash(s, n)); }

  // String.compareTo order of two ids (UTF-16 units, unsigned)
  int compare(uint64_t a, uint64_t b) const {
    const uint64_t la = len(a), lb = len(b), m = la < lb ? la : lb;
    const char16_t *x = str(a), *y = str(b);
    for (uint64_t i = 0; i < m; ++i)
      if (x[i] != y[i]) return x[i] < y[i] ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
  }

 private:
  void place(uint64_t h, uint64_t id) {
    uint64_t i = h & mask;
    while (slots[i]) i = (i + 1) & mask;
    slots[i] = ((h >> 32) << 32) | (id + 1);
  }
  void grow_to(uint64_t n) {  // load factor <= 1/2
    if (!slots.empty() && 2 * n <= slots.size()) return;
    uint64_t cap = slots.empty() ? 64 : slots.size();
    while (cap < 2 * n) cap *= 2;
    slots.assign(cap, 0);
    mask = cap - 1;
    for (uint64_t id = 0; id < size(); ++id) place(hashes[id], id);
  }
};

// the record-ID interner handle of the C-ABI (dk_interner_*)
struct dk_interner : U16Table {};
