// dk_device.h — device helpers shared by the scoring kernels (dk_kernels.hip,
// dk_score_grouped.hip): wave reductions, Java arithmetic, the string view over the
// arenas, and the comparator pieces both kernel families use.  Compiled with
// -ffp-contract=off (Makefile): every double operation rounds once, as in the JVM.
#pragma once

#include <hip/hip_runtime.h>

#include "dk_internal.h"

namespace dk {

// ------------------------------------------------------------------------------------
// small helpers
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

__device__ __forceinline__ uint32_t mask_rank(uint64_t m) {  // set bits below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ int imin3(int a, int b, int c) { return min(min(a, b), c); }

// Whole-wave max / sum, wave-uniform result (every lane active).  DPP steps instead of
// __shfl_xor's LDS crossbar (ds_bpermute + lgkm waits per step, and loop-invariant lane
// addresses that the fused kernels spilled): quad permutes, row half-mirror and mirror
// (16-lane rows), then row_bcast:15 / row_bcast:31 carry rows into lane 63.
template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_max_step(int v) {
  return max(v, __builtin_amdgcn_update_dpp(v, v, CTRL, ROWS, 0xF, false));
}
__device__ __forceinline__ int wave_max_i32(int v) {
  v = dpp_max_step<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
  v = dpp_max_step<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
  v = dpp_max_step<0x141, 0xF>(v);  // row_half_mirror
  v = dpp_max_step<0x140, 0xF>(v);  // row_mirror
  v = dpp_max_step<0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
  v = dpp_max_step<0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3
  return __builtin_amdgcn_readlane(v, 63);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_add_step(uint32_t v) {
  // lanes outside ROWS add 0 (old = 0)
  return v + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v = dpp_add_step<0xB1, 0xF>(v);
  v = dpp_add_step<0x4E, 0xF>(v);
  v = dpp_add_step<0x141, 0xF>(v);
  v = dpp_add_step<0x140, 0xF>(v);
  v = dpp_add_step<0x142, 0xA>(v);
  v = dpp_add_step<0x143, 0xC>(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// java.lang.Math.max(double, double)
__device__ __forceinline__ double java_max(double a, double b) {
  if (a != a) return a;
  if (b != b) return b;
  if (a == 0.0 && b == 0.0) return __signbit(a) ? b : a;
  return a >= b ? a : b;
}

// [Duke 1.2] utils.Utils.computeBayes
__device__ __forceinline__ double compute_bayes(double p1, double p2) {
  return (p1 * p2) / ((p1 * p2) + ((1.0 - p1) * (1.0 - p2)));
}

// A Java String's code units, read a 32-bit word (4 Latin-1 or 2 UTF-16 units) at a time.
// Words of one value are `wstride` words apart: 1 in the canonical arena (strings start
// 4-byte aligned, zero padded), the replica's position count in the candidate replica
// ([word k][position g]: the 64 lanes of a wave read 64 consecutive words).  Units past
// a value's length read as 0 in both layouts.
template <typename CT>
struct Str {
  static constexpr int UPW = 4 / (int)sizeof(CT);  // units per word
  const uint32_t* w;
  uint64_t wstride;
  int kmax;  // last word that may be read speculatively (replica: its row count - 1)
  __device__ __forceinline__ uint32_t word(int k) const { return w[(uint64_t)k * wstride]; }
  // a word read without a per-lane branch (the caller masks words past the value): the
  // canonical arena keeps >= 512 zero bytes after the last value, the replica is clamped
  __device__ __forceinline__ uint32_t word_any(int k) const { return w[(uint64_t)min(k, kmax) * wstride]; }
  // the same read issued where it stands: an invariant load may be sunk to its use by the
  // compiler (undoing a software prefetch); a relaxed atomic load is a plain global_load
  // that stays put
  __device__ __forceinline__ uint32_t word_pf(int k) const {
    return __hip_atomic_load(w + (uint64_t)min(k, kmax) * wstride, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
  static __device__ __forceinline__ uint32_t unit(uint32_t x, int u) {
    return sizeof(CT) == 1 ? (x >> (8 * u)) & 0xFFu : (x >> (16 * u)) & 0xFFFFu;
  }
  __device__ __forceinline__ uint32_t operator[](int j) const { return unit(word(j / UPW), j % UPW); }
};

// Length of the common prefix of a and b, at most `last` (<= 4 and <= both lengths), from
// their first words by XOR and trailing-zero count (units past a value read as 0 in both
// layouts, and `last` cuts at the shorter value) — no per-unit loop of dependent loads.
template <typename CT>
__device__ __forceinline__ int common_prefix4(const Str<CT>& a, const Str<CT>& b, int last) {
  constexpr int UB = 8 * (int)sizeof(CT);
  int p;
  const uint32_t x0 = a.word(0) ^ b.word(0);
  if (sizeof(CT) == 1) {
    p = x0 ? (int)(__builtin_ctz(x0) / UB) : 4;
  } else {
    const uint32_t x1 = a.word_any(1) ^ b.word_any(1);
    p = x0 ? (int)(__builtin_ctz(x0) / UB) : (x1 ? 2 + (int)(__builtin_ctz(x1) / UB) : 4);
  }
  return min(p, last);
}

template <typename CT>
__device__ __forceinline__ bool str_equal(const Str<CT>& a, int na, const Str<CT>& b, int nb) {
  if (na != nb) return false;
  const int nw = (na + Str<CT>::UPW - 1) / Str<CT>::UPW;
  // the first word alone (most unequal values differ in it: all-pairs Levenshtein pays
  // for extra loads there), then four words per round with their loads issued together: a
  // 10-unit date is two round trips instead of three dependent ones (word_any stays inside
  // both layouts' padding; words past the value are masked)
  if (nw == 0) return true;
  if (a.word(0) != b.word(0)) return false;
  for (int k = 1; k < nw; k += 4) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t x = a.word_any(k + i) ^ b.word_any(k + i);
      d |= k + i < nw ? x : 0u;
    }
    if (d) return false;
  }
  return true;
}

// ------------------------------------------------------------------------------------
// Per-wave query tables.  Every wave of k_score holds ONE query record (the candidate
// slots of a query are padded to a multiple of 64), so the query's value of a property
// is wave-uniform.  For it the wave builds, in its LDS slice, the position-mask table
// Peq[c] = {i : q[i] == c} (Myers' "Peq"): 256 entries for Latin-1 units; UTF-16 units
// use a low-byte and a high-byte table whose AND is exact.  A candidate code unit x then
// yields all query positions holding x with one or two LDS reads.
// ------------------------------------------------------------------------------------
constexpr int kPeqEntries = 512;  // per wave: [0,256) low byte, [256,512) high byte

__device__ __forceinline__ void wave_lds_sync() {
  // orders this wave's LDS accesses (no other wave touches its slice)
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
}

// [Duke 1.2] comparators.QGramComparator.compare over precomputed sorted unique gram sets
__device__ __forceinline__ double qgram_formula(int common, int m1, int m2, int formula) {
  if (formula == DK_QGRAM_JACCARD) return (double)common / (double)(m1 + m2 - common);
  if (formula == DK_QGRAM_DICE) return (2.0 * (double)common) / (double)(m1 + m2);
  return (double)common / fmin((double)m1, (double)m2);
}

// |Q ∩ C| with the query's gram set Q in a per-wave LDS hash table (open addressing,
// load <= 1/2, key + 1 stored so 0 marks an empty slot; the caller excludes a set holding
// the all-ones code) and each lane probing its candidate's grams in order — the loads of a
// lane's own list are independent of the probes, so they are issued one gram ahead instead
// of the data-dependent two-list merge.  Wave-uniform call; the table is cleared on exit
// (the LDS slice is the query's Peq table between properties, all zero).
constexpr int kQgramHashMax = 128;  // grams of a query held in the table (<= 256 slots)

__device__ __forceinline__ uint32_t gram_hash(uint64_t code, int lt) {
  return (((uint32_t)code ^ (uint32_t)(code >> 32)) * 0x9E3779B1u) >> (32 - lt);
}

template <typename GT>
__device__ __forceinline__ int qgram_common_hashed(uint64_t* tab, const uint64_t* __restrict__ g1, int m1,
                                                   const GT* __restrict__ g2, uint64_t gstride,
                                                   int gmax, int m2) {
  const int lt = m1 <= 32 ? 6 : (m1 <= 64 ? 7 : 8);
  const uint32_t tmask = (1u << lt) - 1u;
  for (int i = (int)lane_id(); i < m1; i += 64) {
    const uint64_t key = g1[i] + 1ull;
    uint32_t h = gram_hash(g1[i], lt);
    while (atomicCAS((unsigned long long*)&tab[h], 0ull, (unsigned long long)key) != 0ull)
      h = (h + 1u) & tmask;  // the set is unique: a taken slot holds another gram
  }
  wave_lds_sync();
  // the lane's grams in chunks of 8 independent loads (clamped indices: no branch around a
  // load), the next chunk in flight while the current one probes
  int common = 0;
  constexpr int CH = 8;
  uint64_t cur[CH], nxt[CH];
#pragma unroll
  for (int u = 0; u < CH; ++u) cur[u] = (uint64_t)g2[(uint64_t)min(u, gmax) * gstride];
  for (int k0 = 0; k0 < m2; k0 += CH) {
#pragma unroll
    for (int u = 0; u < CH; ++u) nxt[u] = (uint64_t)g2[(uint64_t)min(k0 + CH + u, gmax) * gstride];
    // first probes of the chunk issued together (one LDS latency for 8 grams); a slot
    // holding another gram sends that gram down its probe sequence
    uint32_t h[CH];
    uint64_t v[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      h[u] = gram_hash(cur[u], lt);
      v[u] = tab[h[u]];
    }
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      if (k0 + u < m2) {
        const uint64_t key = cur[u] + 1ull;
        uint64_t x = v[u];
        uint32_t hh = h[u];
        while (x != key && x != 0ull) {
          hh = (hh + 1u) & tmask;
          x = tab[hh];
        }
        common += x == key ? 1 : 0;
      }
    }
#pragma unroll
    for (int u = 0; u < CH; ++u) cur[u] = nxt[u];
  }
  wave_lds_sync();
  for (int e = (int)lane_id(); e <= (int)tmask; e += 64) tab[e] = 0ull;
  wave_lds_sync();
  return common;
}

// |Q ∩ C| of two sorted unique code lists (a merge)
__device__ __forceinline__ int intersect_sorted(const uint64_t* __restrict__ g1, int m1,
                                                const uint64_t* __restrict__ g2, int m2) {
  int i = 0, j = 0, common = 0;
  while (i < m1 && j < m2) {
    const uint64_t x = g1[i], y = g2[j];
    common += (x == y);
    i += (x <= y);
    j += (y <= x);
  }
  return common;
}

// [Duke 1.2] comparators.NumericComparator.compare on host-parsed values
__device__ __forceinline__ double numeric(double d1, bool ok1, double d2, bool ok2, double minratio) {
  if (!ok1 || !ok2) return 0.5;
  if (d1 == 0.0 && d2 == 0.0) return 1.0;
  if (d2 < d1) { const double t = d2; d2 = d1; d1 = t; }
  const double ratio = d1 / d2;
  if (ratio < minratio) return 0.0;
  return ratio;
}

// [Duke 1.2, recalled; parity unpinned] comparators.GeopositionComparator.compare with
// utils.Geoposition.distance: haversine on a sphere of radius 6371000 m, Java 8's
// Math.toRadians (angdeg / 180.0 * PI); an unparsable position -> 0.5; beyond max-distance
// -> 0.0; else ((1 - dist / maxdist) * 0.5) + 0.5.  The same operation order as
// oracle/duke_oracle.c dko_geoposition (no FMA contraction); sin / cos / atan2 may differ
// from libm / Java by an ulp, hence the 1e-12 relative bar of the north star.
__device__ __forceinline__ double geoposition(double lat1d, double lng1d, bool ok1, double lat2d, double lng2d,
                                              bool ok2, double maxdist) {
  if (!ok1 || !ok2) return 0.5;
  const double pi = 3.141592653589793;
  const double lat1 = lat1d / 180.0 * pi, lat2 = lat2d / 180.0 * pi;
  const double dlat = (lat2d - lat1d) / 180.0 * pi, dlng = (lng2d - lng1d) / 180.0 * pi;
  const double sl = sin(dlat / 2), sg = sin(dlng / 2);
  const double a = sl * sl + sg * sg * cos(lat1) * cos(lat2);
  const double dist = 6371000.0 * (2 * atan2(sqrt(a), sqrt(1 - a)));
  if (dist > maxdist) return 0.0;
  return ((1.0 - (dist / maxdist)) * 0.5) + 0.5;
}

// the visiting order of order class oc (wave-uniform): ScoreParams::order[oc] by a select,
// and its k-th property
__device__ __forceinline__ uint64_t order_word(const ScoreParams& P, int oc) {
  return oc == 0 ? P.order[0] : oc == 1 ? P.order[1] : oc == 2 ? P.order[2] : P.order[3];
}
__device__ __forceinline__ int order_at(uint64_t ow, int k) { return (int)((ow >> (4 * k)) & 15u); }

// [Duke 1.2] Processor.compareCandidatesSimple: strict thresholds
__device__ __forceinline__ uint32_t decide(double prob, double threshold, double maybe) {
  if (prob > threshold) return DK_KIND_MATCH;
  if (maybe != 0.0 && prob > maybe) return DK_KIND_MAYBE;
  return 0;
}

// [Duke 1.2] PropertyImpl.compare then the start of Processor.compare's java_max
__device__ __forceinline__ double property_prob(const DevProp& D, double sim) {
  const double v = D.op == DK_CMP_NONE ? 0.5
                   : (sim < 0.5 ? D.low : ((D.high - 0.5) * (sim * sim)) + 0.5);
  return java_max(0.0, v);
}

// [Duke 1.2] PropertyImpl.compare for a property with a comparator (QGram / Numeric roles
// of k_score_gq / k_tile) + the start of Processor.compare's Math.max(0.0, .)
__device__ __forceinline__ double gq_prob(double low, double high, double sim) {
  return java_max(0.0, sim < 0.5 ? low : ((high - 0.5) * (sim * sim)) + 0.5);
}

}  // namespace dk
