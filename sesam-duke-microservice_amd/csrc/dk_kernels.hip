// dk_kernels.hip — gfx950 kernels of the Duke candidate-pair scoring path.
//
// Compiled with -ffp-contract=off and without fast-math: every double operation is a
// single IEEE round-to-nearest operation, as in the JVM, so probabilities reproduce
// Duke's bit for bit when evaluated in the same order.
//
// Hot path (SURVEY §3.1 loops 2-4): k_score — one lane per (query, candidate) slot and
// one query per wave, all properties fused: comparator -> PropertyImpl low/high mapping
// -> computeBayes -> strict threshold -> block-ordered compaction of match / maybe
// entries.  Candidate values are read from the per-match replica (dk_internal.h), where
// the 64 lanes of a wave read 64 consecutive elements.
#include <cstring>

#include <algorithm>
#include <type_traits>
#include <utility>
#include <rocprim/rocprim.hpp>

#include "dk_internal.h"
#include "dk_device.h"

#ifndef DK_WAVES_COUNT
#define DK_WAVES_COUNT 1  // k_sym_count occupancy floor (A/B)
#endif
#define DK_JW_NARROW 32  // JaroWinkler on 32-bit position masks up to this query length (kPeqNarrow)
#ifndef DK_WAVES_SYM2
#define DK_WAVES_SYM2 7  // k_score_sym2 up to 40 rows (5 / 6 / 7 waves: configs[1] ms_score 23.9 / 23.2 / 22.3)
#endif
#ifndef DK_WAVES_SHORT
#define DK_WAVES_SHORT 7  // k_score waves per SIMD up to 40 Levenshtein rows (5 / 6 / 7: all-pairs Levenshtein 821 / 825 / 772 ms, UTF-16 dedup 30.4 / 28.7 / 28.3 ms)
#endif
#ifndef DK_WAVES_NODP
#define DK_WAVES_NODP 8   // k_score_nodp waves per SIMD (no DP comparator: latency bound)
#endif
#ifndef DK_WAVES_LONG8
#define DK_WAVES_LONG8 5  // k_score_long waves per SIMD (the DP an out-of-line call)
#endif
#ifndef DK_WAVES_LONG16
#define DK_WAVES_LONG16 5  // k_score_long_geo waves per SIMD (the DP in the fused kernel)
#endif

namespace dk {

struct RowKeys {
  uint64_t* p[kMaxKeys];
};

// Peq tables of a query value (bit i of entry c: unit i is c; UTF-16 units split into a low-
// and a high-byte table whose entries are ANDed).  A query of up to kPeqNarrow units gets
// NARROW tables of 32-bit entries (entry c at dword c): its readers take 32-bit masks
// (JaroWinkler's, and Levenshtein's row buckets up to 32), and consecutive characters then
// fall in distinct LDS banks -- entry c of a 64-bit table read as its low dword sits at
// dword 2c, so characters 16 apart ('a' / 'q') share a bank (scripts/micro/lds_probe.hip).
// Longer queries: 64-bit entries.
constexpr int kPeqNarrow = 32;
__device__ __forceinline__ bool peq_narrow(int n) { return n <= kPeqNarrow; }

// this lane's query unit (prefetched by the caller) set into / cleared from the tables
template <typename CT>
__device__ __forceinline__ void peq_set_unit(uint64_t* peq, uint32_t ch, int n, bool on) {
  const int lane = (int)lane_id();
  if (lane < n && peq_narrow(n)) {
    uint32_t* p32 = reinterpret_cast<uint32_t*>(peq);
    const uint32_t bit = 1u << lane;
    if (sizeof(CT) == 1) {
      if (on) atomicOr(&p32[ch], bit);
      else p32[ch] = 0;
    } else {
      if (on) {
        atomicOr(&p32[ch & 0xFF], bit);
        atomicOr(&p32[256 + (ch >> 8)], bit);
      } else {
        p32[ch & 0xFF] = 0;
        p32[256 + (ch >> 8)] = 0;
      }
    }
  } else if (lane < n) {
    const uint64_t bit = 1ull << lane;
    if (sizeof(CT) == 1) {
      if (on) atomicOr((unsigned long long*)&peq[ch], (unsigned long long)bit);
      else peq[ch] = 0;
    } else {
      if (on) {
        atomicOr((unsigned long long*)&peq[ch & 0xFF], (unsigned long long)bit);
        atomicOr((unsigned long long*)&peq[256 + (ch >> 8)], (unsigned long long)bit);
      } else {
        peq[ch & 0xFF] = 0;
        peq[256 + (ch >> 8)] = 0;
      }
    }
  }
  wave_lds_sync();
}

template <typename CT>
__device__ __forceinline__ uint64_t peq_eq(const uint64_t* peq, uint32_t x) {
  if (sizeof(CT) == 1) return peq[x];
  return peq[x & 0xFF] & peq[256 + (x >> 8)];
}

// Peq lookups and window masks at the width of the query's position masks: 32 bits when
// the query value has <= kPeqNarrow units (wave-uniform), which halves the mask arithmetic;
// the tables are then narrow (peq_set_unit).
template <typename MT, typename CT>
__device__ __forceinline__ MT peq_eq_t(const uint64_t* peq, uint32_t x) {
  if (sizeof(MT) == 8) return (MT)peq_eq<CT>(peq, x);
  const uint32_t* p32 = reinterpret_cast<const uint32_t*>(peq);
  if (sizeof(CT) == 1) return (MT)p32[x];
  return (MT)(p32[x & 0xFF] & p32[256 + (x >> 8)]);
}

__device__ __forceinline__ uint64_t range_mask(int lo, int hi) {  // bits [lo, hi), 0<=lo<=hi<=64
  const uint64_t up = hi >= 64 ? ~0ull : ((1ull << hi) - 1ull);
  const uint64_t dn = lo >= 64 ? ~0ull : ((1ull << lo) - 1ull);
  return up & ~dn;
}

__device__ __forceinline__ int ffs64(uint64_t m) { return (int)__builtin_ctzll(m); }

// ------------------------------------------------------------------------------------
// [Duke 1.2] comparators.Levenshtein.compactDistance with a wave-uniform s1 (the query
// value, Processor.compare's r1).  One lane per candidate s2; the DP column over s1's
// rows lives in VGPRs, unrolled to the row bucket R and cut at the uniform n1 by scalar
// branches.  The cell is Duke's min(above, aboveleft, left) + cost; the cost bit of row i
// in column j is bit i of ~Peq[s2[j]].
//
// Two rows per VGPR: the column is split into a top half (rows 1..H)
// and a bottom half (rows H+1..2H), the bottom half running one column behind: at step t
// the register of pair i holds (lo) top row i of column t and (hi) bottom row H+i of
// column t-1.  The two halves of a register are then independent, so one packed 3-way
// min + one 32-bit add (values < 2^15, no carry crosses the halves) computes two cells.
// Bottom row H+1 reads top row H of columns t-1 / t-2 (kept from earlier steps).
//
// Values are biased by B = 0x4000 - (maxdist + 1): a cell exceeds Duke's maxdist exactly
// when its bit 14 is set (values stay below 0x7000), so the cutoff test "column minimum > maxdist" is an AND of the
// column's cells (v_bitop3), not a min chain.  The test of column t-1 reads the top half's
// AND from step t-1 and the bottom half's from step t.
//
// Outcome contract: when the cutoff fires this returns maxdist + 1 rather than Duke's
// column minimum.  Both exceed min(n1, n2) / 2, so Levenshtein.compare's similarity is
// < 0.5 either way and PropertyImpl maps the pair to `low` (the distance itself is never
// reported).  Likewise the last column's cutoff is not tested: a cut-off value and
// D(n1, n2-1) are then both > maxdist.
//
// Boundaries (Duke's virtual first row / first column, re-indexed): D(0, t) = t + 1,
// D(i, -1) = i.  Before step 0 the registers hold top column -1 (D(i,-1) = i) and an
// all-BIG bottom "column -2"; bottom's step-0 costs are all 1, which turns that into
// D(H+i, -1) = H + i.
// ------------------------------------------------------------------------------------
// min of three packed pairs: one v_pk_minimum3_f16 — every DP value is kept in
// [0x3F00, 0x7000], positive normal half floats, whose order is their bit patterns' order
// (no NaN, infinity, denormal or sign bit can occur), so the f16 minimum is the u16 minimum.
__device__ __forceinline__ uint32_t pk_min3_u16(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// ------------------------------------------------------------------------------------
// The column loop is unrolled over one candidate word (UPW columns) with two register
// sets used in turn (ping-pong): column t reads set A and writes set B,
// column t+1 reads B and writes A.  In the rolled loop a cell's `diag` is the previous
// column's value of the row above, which the row above has already overwritten, so the
// compiler kept two sets anyway and copied the new one back at every back-edge (one
// v_mov per packed pair per column, and the copy of the prefetched word forced a vmcnt(0)
// wait in the same column).  Unrolled, every value has a fixed register, the unit offset
// inside the word is a constant, and the next word is issued a whole word (UPW columns)
// ahead.  Lanes whose DP ended keep stepping (their result is latched; a masked lane
// costs the SIMD nothing) until no lane of the wave is live, checked after every column.
// Outcome: Duke's distance when it is <= maxdist, else some value > maxdist (maxdist + 1 at
// a cutoff, D(n1, n2) when the lane reaches its last column), as stated above; the raw
// similarity of a cut-off pair comes from k_lev_exact.
// ------------------------------------------------------------------------------------
// PERLANE (k_score_sym2: two queries per wave): n1 differs between the wave's halves and
// may lie anywhere in (0, R]; the result row is then looked up among all R rows.
template <int R, typename CT, bool PERLANE = false>
__device__ __forceinline__ int compact_distance_pp(const uint64_t* peq, int n1, const Str<CT>& s2,
                                                   int n2, bool act) {
  constexpr int UPW = Str<CT>::UPW;
  static_assert(UPW % 2 == 0, "the register sets alternate within one word");
  constexpr int H = R / 2;
  constexpr int TAIL = R <= 32 ? 4 : 8;  // rows past n1 lie in (R - TAIL, R]
  constexpr int NC = (H + 15) / 16;      // cost words
  constexpr uint32_t BIG = 0x7000u;
  const int maxdist = min(n1, n2) >> 1;
  const uint32_t B = 0x4000u - (uint32_t)(maxdist + 1);
  uint32_t PA[H + 1], PB[H + 1];
#pragma unroll
  for (int i = 1; i <= H; ++i) PA[i] = ((uint32_t)i + B) | (BIG << 16);
  // The cutoff AND covers the rows past n1 too (at most TAIL - 1 of them): they can only
  // keep the AND false longer, i.e. delay a lane's exit to a later cutoff or to its last
  // column, whose D(n1, n2) then exceeds maxdist as well (a column minimum above maxdist
  // stays above it in every later column), so the probability (low) is the same; masking
  // them cost one v_or per tail pair per column (-1.6 % dedup step without it).
  const bool bottom_result = n1 > H;
  int result = 0;  // |s2| == 1: Duke returns its initial `above` (0)
  bool live = act && n2 > 1;
  const int fin = n2 - 1 + (bottom_result ? 1 : 0);

  uint32_t w = act ? s2.word(0) : 0u;  // units of columns [t0, t0 + UPW)
  uint32_t wn = s2.word_pf(1);         // the next word
  // cost masks at the width the column needs: rows [0, H + 16) of a Peq entry, so 32 bits
  // up to 32 rows (a 32-bit LDS read leaves no dead half whose register reuse would force
  // the read's wait in the column that issues it)
  constexpr bool kNarrow = H <= 16;
  using NT = typename std::conditional<kNarrow, uint32_t, uint64_t>::type;
  auto ne_of = [&](uint32_t x) -> NT {
    if constexpr (sizeof(NT) == 4) return (NT)~peq_eq_t<uint32_t, CT>(peq, x);
    else return (NT)~peq_eq<CT>(peq, x);
  };
  NT ne_cur = ne_of(Str<CT>::unit(w, 0));
  NT ne_prev = (NT)~(NT)0;
  uint32_t h2 = BIG;  // top row H of column t-2
  uint32_t acc_prev = 0;
  // column t = t0 + U from Pin into Pout; false once no lane of the wave is live
  auto step = [&](auto U_, uint32_t(&Pin)[H + 1], uint32_t(&Pout)[H + 1], int t0) -> bool {
    constexpr int U = decltype(U_)::value;
    const int t = t0 + U;
    const uint32_t xn = U + 1 < UPW ? Str<CT>::unit(w, U + 1) : Str<CT>::unit(wn, 0);
    const NT ne_nx = ne_of(xn);
    uint32_t C[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c)
      C[c] = ((uint32_t)(ne_cur >> (16 * c)) & 0xFFFFu) | ((uint32_t)(ne_prev >> (H + 16 * c)) << 16);
    const uint32_t h1 = Pin[H] & 0xFFFFu;  // top row H of column t-1
    uint32_t above = ((uint32_t)t + 1u + B) | (h1 << 16);
    uint32_t diag = ((uint32_t)t + B) | (h2 << 16);
    uint32_t acc = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 1; i <= H; ++i) {
      const uint32_t cost = (C[(i - 1) >> 4] >> ((i - 1) & 15)) & 0x10001u;
      const uint32_t v = pk_min3_u16(above, diag, Pin[i]) + cost;
      diag = Pin[i];
      Pout[i] = v;
      above = v;
      acc &= v;  // rows past n1 in the cutoff AND: see above
    }
    h2 = h1;
    if (live) {
      if (t >= 2 && (acc_prev & acc & 0x40004000u) == 0x40004000u) {  // column t-1 cut off
        result = maxdist + 1;
        live = false;
      } else if (t == fin) {
        uint32_t r = 0;
        // PERLANE: n1 through an opaque copy, so the R row compares are made here (once per
        // lane) rather than hoisted out of the column loop as R live lane masks
        int nr = n1;
        if (PERLANE) asm volatile("" : "+v"(nr));
#pragma unroll
        for (int row = PERLANE ? 1 : R - TAIL + 1; row <= R; ++row)
          if (row == nr) r = row <= H ? (Pout[row] & 0xFFFFu) : (Pout[row - H] >> 16);
        result = (int)(r - B);
        live = false;
      }
    }
    acc_prev = acc;
    ne_prev = ne_cur;
    ne_cur = ne_nx;
    return __ballot(live) != 0ull;
  };
  if (__ballot(live) != 0ull) {
    for (int t0 = 0;; t0 += UPW) {
      const uint32_t wn2 = s2.word_pf(t0 / UPW + 2);  // a whole word of columns ahead
      if (!step(std::integral_constant<int, 0>{}, PA, PB, t0)) break;
      if (!step(std::integral_constant<int, 1>{}, PB, PA, t0)) break;
      if constexpr (UPW == 4) {
        if (!step(std::integral_constant<int, 2>{}, PA, PB, t0)) break;
        if (!step(std::integral_constant<int, 3>{}, PB, PA, t0)) break;
      }
      w = wn;
      wn = wn2;
    }
  }
  return result;
}

// [Duke 1.2] comparators.Levenshtein.compare.  RMAX: the largest row bucket this kernel
// variant instantiates (the host picks the variant from the longest Levenshtein value),
// which bounds the VGPRs of the whole fused kernel and so its occupancy.
// PERLANE: n1 per lane (k_score_sym2), `nsel` (wave-uniform, >= every lane's n1) picks the
// row bucket
template <int RMAX, typename CT, bool PERLANE = false>
__device__ __forceinline__ double levenshtein_peq(const uint64_t* peq, const Str<CT>& s1, int n1,
                                                  const Str<CT>& s2, int n2, bool act, int nsel = 0) {
  const int len = min(n1, n2);
  const int maxlen = max(n1, n2);
  double r = 0.0;
  bool run = act;
  if (act) {
    // (double)len / maxlen <= 0.5  <=>  2 * len <= maxlen: for ints below 2^52 the
    // quotient is either exactly 0.5 or 1/(2*maxlen) away from it, far beyond rounding
    if (2 * len <= maxlen) run = false;
    else if (len == maxlen && str_equal(s1, n1, s2, n2)) { r = 1.0; run = false; }
  }
  // row buckets of 2 up to 16 rows (a date "YYYY-MM-DD" takes 10 rows, not 12), of 4 up to
  // 32, of 8 above (n1 is wave-uniform: a scalar switch)
  int d;
  const int ns = PERLANE ? nsel : n1;
#define DK_CD(R_) compact_distance_pp<R_, CT, PERLANE>(peq, n1, s2, n2, run)
  if (ns <= 16) {
    switch ((ns + 1) >> 1) {
      case 1: case 2: d = DK_CD(4); break;
      case 3: d = DK_CD(6); break;
      case 4: d = DK_CD(8); break;
      case 5: d = DK_CD(10); break;
      case 6: d = DK_CD(12); break;
      case 7: d = DK_CD(14); break;
      default: d = DK_CD(16); break;
    }
  } else
  switch ((ns + 3) >> 2) {
    case 1: d = DK_CD(4); break;
    case 2: d = DK_CD(8); break;
    case 3: d = DK_CD(12); break;
    case 4: d = DK_CD(16); break;
    case 5: d = DK_CD(20); break;
    case 6: d = DK_CD(24); break;
    case 7: d = DK_CD(28); break;
    case 8: d = DK_CD(32); break;
    case 9: case 10: d = DK_CD((RMAX < 40 ? 4 : 40)); break;
    case 11: case 12: d = DK_CD((RMAX < 48 ? 4 : 48)); break;
    case 13: case 14: d = DK_CD((RMAX < 56 ? 4 : 56)); break;
    default: d = DK_CD((RMAX < 64 ? 4 : 64)); break;
  }
#undef DK_CD
  if (run) {
    const int dist = min(d, len);
    r = 1.0 - ((double)dist / (double)len);
  }
  return r;
}

// ------------------------------------------------------------------------------------
// Long-value DP: WeightedLevenshtein (any length) and Levenshtein with a query value over
// 64 units, both up to kMaxLongUnits.  One candidate per 16-lane DPP row (4 pairs per
// wave, all against the wave's query); lane k of a row owns query rows
// i in (k*R, k*R + R] and, at step t, computes DP column j = t - k + 1 of them
// (anti-diagonal / systolic schedule).  Row k*R of column j arrives from lane k-1 by DPP
// row_shr:1; lane 0 takes the matrix's top boundary instead.  Every cell is a pure
// function of its three neighbours, so this order yields the cells of the Java loop nest
// bit for bit.
//
// Both comparators reduce to a full (n1+1) x (n2+1) matrix D with D(i,0) = i:
//  * Levenshtein.compactDistance: D(0,j) = j, D(i,j) = min(D(i-1,j), D(i-1,j-1),
//    D(i,j-1)) + cost — Duke's column loop with its virtual first row (ix2+1) and first
//    column min(column[ix1-1], ix1-1) + cost, re-indexed by one column.  The early-exit
//    cutoff is not replayed: when it fires (column minimum m > min(n1,n2)/2) the full
//    matrix's D(n1,n2) >= min(m, j) > maxdist as well, so the similarity is < 0.5 either
//    way and PropertyImpl maps both to `low`.
//  * WeightedLevenshtein.distance over the flat array of stride s1len: cell (s1len, c)
//    aliases (0, c+1), which leaves D(0,1) = n1 (the row init overwrites it) and, for
//    n1 == 1, makes row 0 of column j read the row-1 value of column j-1.  Cell:
//    min(D(i-1,j) + w(s1[i-1]), D(i,j-1) + w(s2[j-1]), D(i-1,j-1) + cost).
// ------------------------------------------------------------------------------------

// [Duke 1.2] comparators.WeightedLevenshtein.DefaultWeightEstimator: letters 1.0,
// digits 2.0, punctuation 0.1, anything else 1.0
__device__ __forceinline__ double wl_weight(uint32_t ch) {
  if ((ch | 0x20u) - 'a' < 26u) return 1.0;
  if (ch - '0' < 10u) return 2.0;
  // ' ' '"' '\'' ',' '-' '.' '/' below 64, and '\\'
  constexpr uint64_t kPunct = (1ull << ' ') | (1ull << '"') | (1ull << '\'') | (1ull << ',') |
                              (1ull << '-') | (1ull << '.') | (1ull << '/');
  if ((ch < 64u && ((kPunct >> ch) & 1ull)) || ch == '\\') return 0.1;
  return 1.0;
}

__device__ __forceinline__ int dpp_row_shr1(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, 0x111, 0xF, 0xF, false);
}

__device__ __forceinline__ double dpp_row_shr1(double old, double v) {
  const uint64_t o = (uint64_t)__double_as_longlong(old), x = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)o, (int)(uint32_t)x, 0x111, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(o >> 32), (int)(uint32_t)(x >> 32),
                                                            0x111, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// DPP wave_shr:1 (a gfx9-family control): lane l receives lane l-1's value across the
// whole wave; lane 0 keeps `old`
__device__ __forceinline__ int dpp_wave_shr1(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, 0x138, 0xF, 0xF, false);
}

__device__ __forceinline__ double dpp_wave_shr1(double old, double v) {
  const uint64_t o = (uint64_t)__double_as_longlong(old), x = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)o, (int)(uint32_t)x, 0x138, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(o >> 32), (int)(uint32_t)(x >> 32),
                                                            0x138, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// the value of lane k-1 of this lane's G-lane group (k = 0 takes `top`)
template <int G, typename T>
__device__ __forceinline__ T from_left(T top, T v, int k) {
  if (G == 16) return dpp_row_shr1(top, v);  // DPP rows are 16 lanes: lane 0 of a row keeps top
  const T x = dpp_wave_shr1(top, v);
  return k == 0 ? top : x;
}

// Per-wave LDS of the long-value section, inside the wave's table slice (zeroed on exit so
// the Peq tables stay clear), in u64 words:
//   [kLongPtr, +64)   candidate unit pointers by sorted position
//   [kLongMeta, +32)  u32 by sorted position: n2 | src lane << 16 (first the sort keys)
//   [kLongRes, +64)   D(n1, n2) by lane (f64 or int bits)
//   [kLongRing, +256) u32 unit rings [4 groups][128]: unit | weight class << 16
constexpr int kLongPtr = 0, kLongMeta = 64, kLongRes = 96, kLongRing = 160;
// the scoring kernels' per-wave table slices (namespace scope, so the out-of-line long DP
// addresses them as LDS)
__shared__ uint64_t g_wave_tables[kScoreBlock / 64][kPeqEntries];
constexpr int kLongLdsWords = kLongRing + 256;
static_assert(kLongLdsWords <= kPeqEntries, "the long section lives in the wave's Peq slice");

// [Duke 1.2] WeightedLevenshtein.DefaultWeightEstimator weight class of a unit: 0 = 1.0
// (letters, anything else), 1 = 2.0 (digits), 2 = 0.1 (punctuation and space)
__device__ __forceinline__ uint32_t wl_class(uint32_t ch) {
  if ((ch | 0x20u) - 'a' < 26u) return 0u;
  if (ch - '0' < 10u) return 1u;
  constexpr uint64_t kPunct = (1ull << ' ') | (1ull << '"') | (1ull << '\'') | (1ull << ',') |
                              (1ull << '-') | (1ull << '.') | (1ull << '/');
  if ((ch < 64u && ((kPunct >> ch) & 1ull)) || ch == '\\') return 2u;
  return 0u;
}

__device__ __forceinline__ double wl_class_weight(uint32_t cls) {
  return cls == 1u ? 2.0 : (cls == 2u ? 0.1 : 1.0);
}

// The wave's candidates stream through NG = 64/G lane groups.  long_sims sorts them
// longest first; group grp takes sorted positions grp, 2NG-1-grp, 2NG+grp, ... (dealt
// snake-wise, so the groups' column totals come out nearly equal) and runs their DP
// matrices back to back as ONE systolic stream of columns: lane k works on stream column
// t - k at step t, so a lane moves on to its next candidate one step after its left
// neighbour and the pipeline never drains between candidates.  Stream units come from a
// 128-unit LDS ring per group (two 64-unit blocks): block b+1 is written at step 64b + 32,
// from registers loaded 64 steps earlier, into the half the group's last lane left 32+
// steps before; every lane reads its unit one step ahead.  D(n1, n2) leaves as raw bits
// (long_sims turns it into the similarity), so the candidate switch stays small.
//
// Out of line: the stream's registers (column, weights, units, ring cursor) get an
// allocation of their own instead of competing with the fused kernel's live state, which
// spilled the weights and units inside the cell loop.
// f(integral_constant<int, i>) for i = 0 .. N-1, unrolled at compile time
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// long_dp_body runs as long_dp, an out-of-line call: the call saves the fused kernel's live
// state to its scratch frame, so the DP's column, weights and units get the registers, at 5
// waves per SIMD.  Inlined (one variant per kernel, zero scratch at 3-4 waves, or 4-5 waves
// with spills inside the DP) it ran 1.5-1.6x slower.
template <int G, int R, bool WL, typename CT>
__device__ __forceinline__ void long_dp_body(uint64_t wstride, const CT* s1p, int n1, int nneed) {
  uint64_t* lds = g_wave_tables[threadIdx.x >> 6];
  using T = typename std::conditional<WL, double, int>::type;
  constexpr int UPW = 4 / (int)sizeof(CT);
  constexpr int NG = 64 / G;  // candidate streams
  constexpr int UL = 64 / G;  // ring units a lane stages per block
  static_assert(G <= 32, "the ring half is rewritten 32 steps into the block");
  const uint64_t* cptr = lds + kLongPtr;
  const uint32_t* meta = reinterpret_cast<const uint32_t*>(lds + kLongMeta);
  uint64_t* rbits = lds + kLongRes;
  const int lane = (int)lane_id();
  const int grp = lane / G, k = lane % G;
  uint32_t* ring = reinterpret_cast<uint32_t*>(lds + kLongRing) + grp * 128;
  const int kstar = (n1 - 1) / R, rstar = n1 - kstar * R;
  auto spos = [&](int m) { return m * NG + ((m & 1) ? NG - 1 - grp : grp); };
  const int cnt = nneed / NG + (spos(nneed / NG) < nneed ? 1 : 0);
  int tlen = 0;
  for (int m = 0; m < cnt; ++m) tlen += (int)(meta[spos(m)] & 0xFFFFu);
  tlen = wave_max_i32(tlen);
  const int tend = tlen + kstar + 1;  // lane kstar closes its last matrix at step tlen + kstar

  // this lane's query rows, packed like the ring units (equal packed values <=> equal
  // units: the class is a function of the unit)
  uint32_t c1[R];
  double w1[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = k * R + r;
    const uint32_t ch = i < n1 ? (uint32_t)s1p[i] : 0u;
    c1[r] = i < n1 ? (ch | (wl_class(ch) << 16)) : 0xFFFFFFFFu;  // rows past n1 never match
    w1[r] = WL ? wl_weight(ch) : 0.0;
  }

  // staging cursor: this lane loads stream units k + G*i of each 64-unit block
  int lm = 0, loff = 0, ln2 = 0;
  const uint32_t* lptr = nullptr;
  if (cnt > 0) {
    ln2 = (int)(meta[spos(0)] & 0xFFFFu);
    lptr = reinterpret_cast<const uint32_t*>(cptr[spos(0)]);
  }
  auto advance = [&](int step) {
    loff += step;
    while (lm < cnt && loff >= ln2) {
      loff -= ln2;
      if (++lm < cnt) {
        ln2 = (int)(meta[spos(lm)] & 0xFFFFu);
        lptr = reinterpret_cast<const uint32_t*>(cptr[spos(lm)]);
      }
    }
  };
  uint32_t stg[UL];
  uint32_t subs = 0;
  auto load_block = [&]() {
    subs = 0;
#pragma unroll
    for (int i = 0; i < UL; ++i) {
      stg[i] = lm < cnt ? lptr[(uint64_t)(loff / UPW) * wstride] : 0u;
      subs |= (uint32_t)(loff % UPW) << (2 * i);
      advance(G);
    }
  };
  auto write_block = [&](int half) {
#pragma unroll
    for (int i = 0; i < UL; ++i) {
      const uint32_t ch = Str<CT>::unit(stg[i], (int)((subs >> (2 * i)) & 3u));
      ring[half * 64 + k + G * i] = ch | (wl_class(ch) << 16);
    }
  };
  advance(k);
  load_block();
  write_block(0);
  load_block();
  wave_lds_sync();

  // The lane's DP column.  In the steady state logical row r lives in col[(r + rho) %
  // (R + 1)], rho = -t mod (R + 1): a step writes row r's new value into the slot row r-1
  // vacated (row r-1's old value was row r's diagonal), so the column rotates one slot per
  // step instead of being moved back (a register move per cell), and the steady-state loop
  // is unrolled R + 1 steps, which makes every slot index a constant.  The pipeline fill
  // (t < G: lane k starts its first column at step k) runs in place, rho = 0.
  T col[R + 1];
#pragma unroll
  for (int r = 0; r < R; ++r) col[r] = (T)(k * R + r + 1);  // D(i, 0) = i
  col[R] = (T)0;
  T prev = (T)(k * R);                                      // D(k*R, j-1)
  T bot = col[R - 1];
  int m = 0, j = 1 - k;  // this lane's candidate and its column at this step
  int n2c = 0, srcc = 0;
  if (cnt > 0) {
    const uint32_t x = meta[spos(0)];
    n2c = (int)(x & 0xFFFFu);
    srcc = (int)(x >> 16);
  }
  uint32_t lu = ring[(0 - k) & 127];  // the unit of stream column t - k, read a step ahead
  auto step = [&](auto rho_c, int t, auto fill_c) {
    constexpr int rho = decltype(rho_c)::value;
    constexpr bool FILL = decltype(fill_c)::value;
    if ((t & 63) == 32) {  // block b+1 into the half block b-1 held, then load block b+2
      write_block(((t >> 6) + 1) & 1);
      load_block();
    }
    const uint32_t u = lu;
    lu = ring[(t + 1 - k) & 127];
    while (m < cnt && j > n2c) {
      // column n2c done: D(n1, n2) sits in lane kstar's row rstar
      if (k == kstar) {
        // col[rstar - 1] as a mask-or (a select chain becomes a dynamically indexed load)
        uint64_t bits = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const T x = col[(r + rho) % (R + 1)];
          const uint64_t b = WL ? (uint64_t)__double_as_longlong((double)x) : (uint64_t)(uint32_t)(int)x;
          bits |= b & (0ull - (uint64_t)(r + 1 == rstar));
        }
        rbits[srcc] = bits;
      }
      j -= n2c;
      if (++m < cnt) {
        const uint32_t x = meta[spos(m)];
        n2c = (int)(x & 0xFFFFu);
        srcc = (int)(x >> 16);
      }
      // D(i, 0) = i again, computed here (an opaque base: hoisted constants get spilled)
      int kb = k * R;
      asm volatile("" : "+v"(kb));
#pragma unroll
      for (int r = 0; r < R; ++r) col[(r + rho) % (R + 1)] = (T)(kb + r + 1);
      prev = (T)kb;
    }
    // lane 0's row above: the matrix's top boundary D(0, j)
    T top;
    if (WL) top = n1 == 1 ? col[rho % (R + 1)] : (T)(j == 1 ? n1 : j);
    else top = (T)j;
    const T recv = from_left<G>(top, bot, k);  // D(k*R, j)
    // the fill computes only lanes that have started (in place); the steady state computes
    // every lane (finished lanes produce values no running lane reads: a lane only takes
    // its left neighbour's column while that neighbour was still running)
    if (FILL ? (j >= 1 && m < cnt) : true) {
      T up = recv, dg = prev;
      const double w2 = WL ? wl_class_weight(u >> 16) : 0.0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const T old = col[(r + rho) % (R + 1)];
        T v;
        if (WL) {
          const double cost = c1[r] == u ? 0.0 : fmax(w1[r], w2);
          // Math.min(left, Math.min(above, aboveleft)) on non-negative values
          v = (T)fmin((double)up + w1[r], fmin((double)old + w2, (double)dg + cost));
        } else {
          v = (T)(imin3((int)up, (int)dg, (int)old) + (c1[r] == u ? 0 : 1));
        }
        col[FILL ? (r + rho) % (R + 1) : (r + rho + R) % (R + 1)] = v;
        dg = old;
        up = v;
      }
      prev = recv;
      bot = up;
    }
    ++j;
  };
  const int tfill = min(tend, G);
  for (int t = 0; t < tfill; ++t) step(std::integral_constant<int, 0>{}, t, std::true_type{});
  for (int t = tfill; t < tend; t += R + 1)
    static_for<R + 1>([&](auto q) {
      constexpr int qq = decltype(q)::value;
      if (t + qq < tend) step(std::integral_constant<int, (R + 1 - qq) % (R + 1)>{}, t + qq, std::false_type{});
    });
}

template <int G, int R, bool WL, typename CT>
__device__ __attribute__((noinline)) void long_dp(uint64_t wstride, const CT* s1p, int n1, int nneed) {
  long_dp_body<G, R, WL, CT>(wstride, s1p, n1, nneed);
}

// The DP variant of a query of n1 units in a kernel of up to LR rows per lane (0..11):
// 16-lane groups (4 streams, DPP row_shr) up to 128 rows, 32-lane groups (2 streams,
// wave_shr) beyond; LR caps the variants a kernel carries.
template <int LR>
__host__ __device__ constexpr int long_variant(int n1) {
  return n1 <= 16 ? 0 : n1 <= 32 ? 1 : n1 <= 48 ? 2 : (n1 <= 64 || LR <= 4) ? 3 : n1 <= 80 ? 4
       : n1 <= 96 ? 5 : n1 <= 112 ? 6 : (n1 <= 128 || LR <= 8) ? 7 : n1 <= 160 ? 8 : n1 <= 192 ? 9
       : n1 <= 224 ? 10 : 11;
}

// Similarity of every lane with `need` set (the others keep `sim`) through long_dp.
// Wave-uniform call: all 64 lanes enter.
template <int LR, bool WL, typename CT>
__device__ __forceinline__ double long_sims(const DevProp& D, uint64_t rstride, uint64_t* lds, uint32_t q,
                                            int n1, uint32_t g, uint32_t crow, int lc, bool need,
                                            double sim) {
  const uint64_t nm = __ballot(need);
  if (nm == 0) return sim;
  const int nneed = __popcll(nm);
  const uint32_t lane = lane_id();
  uint32_t* meta = reinterpret_cast<uint32_t*>(lds + kLongMeta);
  // sorted position: longest candidate first, ties in lane order (keys are distinct)
  const uint32_t key = need ? (((uint32_t)lc << 6) | (63u - lane)) + 1u : 0u;
  meta[lane] = key;
  wave_lds_sync();
  int rank = 0;
  if (need) {
    for (int i = 0; i < 64; i += 4) {
      const uint4 v = *reinterpret_cast<const uint4*>(meta + i);
      rank += (int)(v.x > key) + (int)(v.y > key) + (int)(v.z > key) + (int)(v.w > key);
    }
  }
  wave_lds_sync();
  const CT* base = reinterpret_cast<const CT*>(D.units);
  if (need) {
    meta[rank] = (uint32_t)lc | (lane << 16);
    const uint32_t* p = D.rlmax ? reinterpret_cast<const uint32_t*>(D.runits) + g
                                : reinterpret_cast<const uint32_t*>(base + D.off[crow]);
    lds[kLongPtr + rank] = (uint64_t)p;
  }
  wave_lds_sync();
  const uint64_t wstride = D.rlmax ? rstride : 1u;
  const CT* s1p = base + D.off[q];
  // query rows per lane (n1 is wave-uniform: a scalar switch): 16-lane groups (4 streams,
  // DPP row_shr) up to 128 rows, 32-lane groups (2 streams, wave_shr) beyond; R = rows /
  // lanes rounded up, so most of a group's lanes hold rows, and R <= 8 keeps the column,
  // weights and units in VGPRs.  LR caps the variants a kernel carries.
  const int vi = long_variant<LR>(n1);
#define DK_LDP(V_, G_, R_) \
  if (vi == (V_)) long_dp<G_, R_, WL, CT>(wstride, s1p, n1, nneed);
  DK_LDP(0, 16, 1)
  DK_LDP(1, 16, 2)
  DK_LDP(2, 16, 3)
  DK_LDP(3, 16, 4)
  DK_LDP(4, 16, 5)
  DK_LDP(5, 16, 6)
  DK_LDP(6, 16, 7)
  DK_LDP(7, 16, 8)
  DK_LDP(8, 32, (LR < 16 ? 4 : 5))
  DK_LDP(9, 32, (LR < 16 ? 4 : 6))
  DK_LDP(10, 32, (LR < 16 ? 4 : 7))
  DK_LDP(11, 32, (LR < 16 ? 4 : 8))
#undef DK_LDP
  wave_lds_sync();
  if (need) {
    const uint64_t bits = lds[kLongRes + lane];
    if (WL) {
      // [Duke 1.2] WeightedLevenshtein.compare
      const double maxlen = (double)max(n1, lc);
      const double dist = __longlong_as_double((long long)bits);
      sim = dist > maxlen ? 0.0 : 1.0 - (dist / maxlen);
    } else {
      // [Duke 1.2] Levenshtein.compare: 1 - min(dist, len) / len
      const int len = min(n1, lc);
      sim = 1.0 - ((double)min((int)(uint32_t)bits, len) / (double)len);
    }
  }
  wave_lds_sync();
  for (int e = (int)lane; e < kLongLdsWords; e += 64) lds[e] = 0;  // Peq slice stays zero
  wave_lds_sync();
  return sim;
}

// [Duke 1.2] comparators.JaroWinkler.similarity — per-lane form for values over 64 units
template <typename CT>
__device__ __forceinline__ double jarowinkler(Str<CT> s1, int n1, Str<CT> s2, int n2) {
  if (str_equal(s1, n1, s2, n2)) return 1.0;
  if (n1 > n2) {
    const Str<CT> ts = s2; s2 = s1; s1 = ts;
    int tn = n2; n2 = n1; n1 = tn;
  }
  const int maxdist = n2 >> 1;
  int c = 0, t = 0, prevpos = -1;
  for (int ix = 0; ix < n1; ++ix) {
    const uint32_t ch = s1[ix];
    const int hi = min(n2, ix + maxdist);
    for (int ix2 = max(0, ix - maxdist); ix2 < hi; ++ix2) {
      if (ch == s2[ix2]) {
        ++c;
        if (prevpos != -1 && ix2 < prevpos) ++t;
        prevpos = ix2;
        break;
      }
    }
  }
  if (c == 0) return 0.0;
  double score = ((c / (double)n1) + (c / (double)n2) + ((c - t) / (double)c)) / 3.0;
  const int p = common_prefix4(s1, s2, min(4, n1));
  score += ((p * (1 - score)) / 10);
  return score;
}

// [Duke 1.2] comparators.JaroWinkler.similarity with the query's Peq table (both values
// <= 64 units).  s1 is the shorter value (the query on a tie).  One sweep over the
// candidate's units j serves both cases, so lanes of either kind share it:
//  * candidate shorter (s1 = candidate, rows = its units): row j's first match is the
//    lowest set bit of Peq[cand[j]] inside the window over the query;
//  * query shorter or equal (rows = query units): Peq[cand[j]] gives every query row
//    holding that unit, masked to the rows whose window contains j and not yet matched
//    (Duke takes the FIRST match in the window); the step j that matched each row is kept
//    in six bit-planes.  The transposition count (a row matching before the previous
//    matched row did) then comes bit-parallel: each plane's bit is carried from one
//    matched row to the next by an add through the unmatched rows between them, and a
//    bit-sliced compare of the two 6-bit steps counts the descents.
template <typename MT>
__device__ __forceinline__ MT carry_to_next(MT plane, MT found) {
  // bit i of the result = bit of `plane` at the matched row before matched row i
  return (((plane & found) << 1) + ~found) & found;
}

template <typename MT>
__device__ __forceinline__ MT range_mask_t(int lo, int hi) {  // bits [lo, hi), 0<=lo<=hi<=width
  if (sizeof(MT) == 8) return (MT)range_mask(lo, hi);
  const uint32_t up = hi >= 32 ? ~0u : ((1u << hi) - 1u);
  const uint32_t dn = lo >= 32 ? ~0u : ((1u << lo) - 1u);
  return (MT)(up & ~dn);
}

template <typename MT>
__device__ __forceinline__ int popc_t(MT m) {
  return sizeof(MT) == 8 ? __popcll((uint64_t)m) : __popc((uint32_t)m);
}

// DUAL (symmetric dedup schedule): also the similarity with the roles swapped, *rev =
// JaroWinkler(r1 = candidate, r2 = query).  Only equal-length pairs differ (Duke keeps r1
// as s1 on a tie); for them the same sweep runs the candidate-rows form over the query
// window [j - md, j + md) beside the query-rows form.
template <typename MT, typename CT, bool DUAL>
__device__ __forceinline__ double jarowinkler_peq(const uint64_t* peq, const Str<CT>& qs, int nq,
                                                  const Str<CT>& cs, int nc, bool act, double* rev) {
  if (act && str_equal(qs, nq, cs, nc)) act = false;  // 1.0 below
  const bool rows_cand = act && nc < nq;
  const bool rows_query = act && !rows_cand;
  const bool eqlen = DUAL && act && nc == nq;  // the reversed orientation, candidate rows
  // window over the query: [j - md, j + md) for candidate row j (md = |query| / 2), or the
  // rows i with j in [i - md, i + md) (md = |candidate| / 2) — both as [lo_off + j, hi_off + j)
  const int md = rows_cand ? (nq >> 1) : (nc >> 1);
  const int lo_off = rows_cand ? -md : 1 - md, hi_off = rows_cand ? md : md + 1;
  const int md2 = nq >> 1;
  int c = 0, t = 0, prev = -1;  // prev = -1: the first match never counts (jj >= 0)
  MT found = 0, p0 = 0, p1 = 0, p2 = 0, p3 = 0, p4 = 0, p5 = 0;
  const int maxn = act ? nc : 0;
  int wmax = maxn;
  wmax = wave_max_i32(wmax);
  constexpr int UPW = Str<CT>::UPW;
  // Units past a candidate's end read as 0 (zero padded): Peq[0] is empty unless the
  // query itself holds U+0000 (wave-uniform), and only then do lanes mask past-end units.
  const bool nul = peq_eq_t<MT, CT>(peq, 0u) != (MT)0;
  if (sizeof(MT) == 4) {
    // 32-bit masks (query <= 32 units): the window [j + lo_off, j + hi_off) slides one
    // position per unit, so it is a 64-bit register shifted left once per step whose high
    // word holds query positions [0, 32) (positions below 0 live in the low word; Peq has
    // no bits at or past nq, so no upper clip is needed)
    const int width = hi_off - lo_off;  // 2 md <= 64
    uint64_t W = (width >= 64 ? ~0ull : ((1ull << width) - 1ull)) << (32 + lo_off);
    uint64_t W2 = ((1ull << (2 * md2)) - 1ull) << (32 - md2);  // DUAL: [j - md2, j + md2)
    auto sweep_word = [&](uint32_t w, int k) {
#pragma unroll
      for (int u = 0; u < UPW; ++u) {
        const int j = k * UPW + u;  // wave-uniform: the plane updates are scalar branches
        uint32_t pv = (uint32_t)peq_eq_t<MT, CT>(peq, Str<CT>::unit(w, u));
        if (nul) pv = j < maxn ? pv : 0u;
        const uint32_t e = pv & (uint32_t)(W >> 32);
        W <<= 1;
        // candidate rows: first match of row j
        uint32_t ec = rows_cand ? e : 0u;
        if (DUAL) {
          if (eqlen) ec = pv & (uint32_t)(W2 >> 32);
          W2 <<= 1;
        }
        const int jj = __ffs(ec) - 1;
        const bool has = ec != 0u;
        c += has ? 1 : 0;
        t += (has && jj < prev) ? 1 : 0;
        prev = has ? jj : prev;
        // query rows: rows first matched at step j
        const MT m = rows_query ? (MT)(e & ~(uint32_t)found) : (MT)0;
        found |= m;
        if (j & 1) p0 |= m;
        if (j & 2) p1 |= m;
        if (j & 4) p2 |= m;
        if (j & 8) p3 |= m;
        if (j & 16) p4 |= m;
        if (j & 32) p5 |= m;
      }
    };
    // candidate words two ahead in two fixed registers (the loop is unrolled by two words,
    // so a word is consumed two words after its load was issued); word_pf: loads the
    // compiler keeps where they are issued
    uint32_t wa = cs.word_pf(0), wb = cs.word_pf(1);
    for (int k = 0; k * UPW < wmax; k += 2) {
      sweep_word(wa, k);
      wa = cs.word_pf(k + 2);
      if ((k + 1) * UPW < wmax) {
        sweep_word(wb, k + 1);
        wb = cs.word_pf(k + 3);
      }
    }
  } else {
    for (int k = 0; k * UPW < wmax; ++k) {
      const uint32_t w = cs.word_any(k);  // units past maxn are never used (j < maxn)
#pragma unroll
      for (int u = 0; u < UPW; ++u) {
        const int j = k * UPW + u;  // wave-uniform: the plane updates are scalar branches
        MT pv = peq_eq_t<MT, CT>(peq, Str<CT>::unit(w, u));
        if (nul) pv = j < maxn ? pv : (MT)0;
        const MT e = pv & range_mask_t<MT>(max(0, j + lo_off), min(nq, j + hi_off));
        // candidate rows: first match of row j
        MT ec = rows_cand ? e : (MT)0;
        if (DUAL && eqlen) ec = pv & range_mask_t<MT>(max(0, j - md2), min(nq, j + md2));
        const int jj = ffs64((uint64_t)ec | (1ull << 63));
        const bool has = ec != 0;
        c += has ? 1 : 0;
        t += (has && jj < prev) ? 1 : 0;
        prev = has ? jj : prev;
        // query rows: rows first matched at step j
        const MT m = rows_query ? (MT)(e & ~found) : (MT)0;
        found |= m;
        if (j & 1) p0 |= m;
        if (j & 2) p1 |= m;
        if (j & 4) p2 |= m;
        if (j & 8) p3 |= m;
        if (j & 16) p4 |= m;
        if (j & 32) p5 |= m;
      }
    }
  }
  const int cc = c, tc = t;  // candidate-rows counts (rows_cand lanes, or the reversed pair)
  if (rows_query) {
    c = popc_t(found);
    // descents p(i) < p(previous matched row), MSB-first bit-sliced compare
    const MT P[6] = {p0, p1, p2, p3, p4, p5};
    MT lt = 0, eq = (MT)~(MT)0;
#pragma unroll
    for (int b = 5; b >= 0; --b) {
      const MT a = P[b], q = carry_to_next<MT>(P[b], found);
      lt |= eq & ~a & q;
      eq &= ~(a ^ q);
    }
    t = popc_t<MT>(lt & found);
  }
  if (!act) {  // equal values (inactive lanes discard the result)
    if (DUAL) *rev = 1.0;
    return 1.0;
  }
  double score = 0.0;
  const Str<CT>& s1 = rows_cand ? cs : qs;
  const Str<CT>& s2 = rows_cand ? qs : cs;
  const int n1 = rows_cand ? nc : nq, n2 = rows_cand ? nq : nc;
  const int p = common_prefix4(s1, s2, min(4, n1));  // symmetric in s1 / s2
  if (c != 0) {
    score = ((c / (double)n1) + (c / (double)n2) + ((c - t) / (double)c)) / 3.0;
    score += ((p * (1 - score)) / 10);
  }
  if (DUAL) {
    double r = score;
    if (eqlen) {  // r1 = candidate = s1 (n1 == n2)
      r = 0.0;
      if (cc != 0) {
        r = ((cc / (double)nc) + (cc / (double)nq) + ((cc - tc) / (double)cc)) / 3.0;
        r += ((p * (1 - r)) / 10);
      }
    }
    *rev = r;
  }
  return score;
}

// [Duke 1.2, recalled] DiceCoefficientComparator / JaccardIndexComparator with the
// ExactComparator sub-comparator: the tokens of the shorter list (s1 on a tie) that occur
// in the other, counted with multiplicity (sorted token ids, duplicates kept)
__device__ __forceinline__ int count_members(const uint64_t* __restrict__ g1, int m1,
                                             const uint64_t* __restrict__ g2, int m2) {
  int i = 0, j = 0, hit = 0;
  while (i < m1 && j < m2) {
    const uint64_t x = g1[i], y = g2[j];
    hit += (x == y);
    i += (x <= y);
    j += (y < x);
  }
  return hit;
}

// |Q ∩ C| for Latin-1 bigram sets (DevProp::g16).  The query's keys go to their slots of a
// per-wave LDS table under the query row's perfect-hash seed, so each candidate key is ONE
// table read and compare -- no probe chain, no divergence.  Each lane streams its
// candidate's key words (four keys per u64: the wave's 64 lanes read one 512-B row per word)
// two words at a time, the next two in flight.  Lanes past their own set read padding keys
// (0); slot 0 -- where key 0 hashes -- is never left 0, so padding never counts, and empty
// slots hold 0, which no real key equals.  Wave-uniform call; the table is left zero.
__device__ __forceinline__ int qgram_common_perfect(uint32_t* tab, const uint64_t* __restrict__ g1, int m1,
                                                    uint32_t seed, const uint64_t* __restrict__ rg,
                                                    uint64_t rstride, uint32_t g, int m2) {
  const int lt = kGramLtMin + (int)(seed >> 8);
  const uint32_t mult = gram_mult(seed & 0xFFu);
  const int sh = 32 - lt;
  const int lane = (int)lane_id();
  if (lane == 0) tab[0] = ~0u;  // a real key landing in slot 0 overwrites the sentinel below
  uint32_t s0 = 0u;             // this lane's query slot (m1 <= kGramPerfectMax = 64)
  if (lane < m1) {
    const uint32_t key = gram_key(g1[lane]);
    s0 = (uint32_t)__umul24(key, mult) >> sh;
    tab[s0] = key;
  }
  wave_lds_sync();
  int njw = (m2 + 3) >> 2;  // word rows: this lane's, then the wave's most (the trip count)
  njw = wave_max_i32(njw);
  // the word row's base is wave-uniform, the lane adds a 32-bit byte offset
  const char* base = reinterpret_cast<const char*>(rg);
  const uint32_t boff = g * 8u;
  const uint64_t rowb = rstride * 8u;
  auto ld = [&](int j) -> uint64_t {
    return __hip_atomic_load(reinterpret_cast<const uint64_t*>(base + (uint64_t)j * rowb + boff),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  int common = 0;
  auto probe = [&](uint64_t w) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t key = (uint32_t)(w >> (16 * e)) & 0xFFFFu;
      common += tab[(uint32_t)__umul24(key, mult) >> sh] == key ? 1 : 0;
    }
  };
  if (njw > 0) {
    uint64_t c0 = ld(0), c1 = ld(1);  // rgrows is even and >= 2
    for (int j = 0; j < njw; j += 2) {
      uint64_t n0 = 0, n1 = 0;
      if (j + 2 < njw) {  // wave-uniform; j + 3 < rgrows
        n0 = ld(j + 2);
        n1 = ld(j + 3);
      }
      probe(c0);
      probe(c1);
      c0 = n0;
      c1 = n1;
    }
  }
  wave_lds_sync();
  if (lane < m1) tab[s0] = 0u;
  if (lane == 0) tab[0] = 0u;
  wave_lds_sync();
  return common;
}

// ------------------------------------------------------------------------------------
// The fused scoring kernel.  One lane per slot, one query per wave.
// ------------------------------------------------------------------------------------
// SYM: `rev` receives Comparator.compare(candidate, query) where it can differ from
// compare(query, candidate) (JaroWinkler on equal lengths); it is left alone otherwise.
template <int RMAX, int LR, typename CT, bool SYM, bool DP, bool GR>
__device__ __forceinline__ double string_sim(const DevProp& D, uint64_t rstride, uint64_t* peq,
                                             uint32_t q, uint32_t g, uint32_t crow, int lq,
                                             int lc, bool cmp, double& rev, uint32_t qch) {
  const CT* base = reinterpret_cast<const CT*>(D.units);
  const Str<CT> s1{reinterpret_cast<const uint32_t*>(base + D.off[q]), 1, 1 << 30};
  const Str<CT> s2 = D.rlmax ? Str<CT>{reinterpret_cast<const uint32_t*>(D.runits) + g, rstride,
                                       D.rlmax / Str<CT>::UPW - 1}
                             : Str<CT>{reinterpret_cast<const uint32_t*>(base + D.off[crow]), 1, 1 << 30};
  double sim = 0.0;
  switch (D.op) {
    case DK_CMP_WEIGHTED_LEVENSHTEIN:
      if (DP && LR > 0) {  // the host only schedules WeightedLevenshtein on LR > 0 variants
        const bool same = cmp && str_equal(s1, lq, s2, lc);
        sim = same ? 1.0 : 0.0;
        sim = long_sims<LR, true, CT>(D, rstride, peq, q, lq, g, crow, lc, cmp && !same, sim);
      }
      break;
    case DK_CMP_LEVENSHTEIN:
      if (!DP) break;  // the DP-free variant is only launched without DP comparators
      if (LR > 0 && lq > kMaxUnits) {  // query over 64 units: long-value DP
        bool need = false;
        if (cmp) {
          const int len = min(lq, lc), maxlen = max(lq, lc);
          if (2 * len <= maxlen) sim = 0.0;
          else if (len == maxlen && str_equal(s1, lq, s2, lc)) sim = 1.0;
          else need = true;
        }
        sim = long_sims<LR, false, CT>(D, rstride, peq, q, lq, g, crow, lc, need, sim);
        break;
      }
      [[fallthrough]];
    case DK_CMP_JAROWINKLER: {
      if (!DP) break;
      const bool table = lq <= 64 && (D.op == DK_CMP_LEVENSHTEIN || __ballot(cmp && lc > 64) == 0);
      if (table) {
        peq_set_unit<CT>(peq, qch, lq, true);
        if (D.op == DK_CMP_LEVENSHTEIN) {
          sim = levenshtein_peq<RMAX>(peq, s1, lq, s2, lc, cmp);
        } else {
          double r = 0.0;
          sim = lq <= DK_JW_NARROW ? jarowinkler_peq<uint32_t, CT, SYM>(peq, s1, lq, s2, lc, cmp, &r)
                                   : jarowinkler_peq<uint64_t, CT, SYM>(peq, s1, lq, s2, lc, cmp, &r);
          if (SYM) rev = r;
        }
        peq_set_unit<CT>(peq, qch, lq, false);
      } else if (cmp) {
        sim = jarowinkler(s1, lq, s2, lc);
        if (SYM) rev = lq == lc ? jarowinkler(s2, lc, s1, lq) : sim;
      }
      break;
    }
    case DK_CMP_EXACT:
      if (cmp) sim = str_equal(s1, lq, s2, lc) ? 1.0 : 0.0;
      break;
    case DK_CMP_QGRAM: {
      if (!GR) break;  // the host launches GR = false only for schemas without gram sets
      const int m1 = (int)__builtin_amdgcn_readfirstlane((uint32_t)D.gcnt[q]);
      const uint64_t* g1 = D.grams + D.goff[q];
      if (D.g16) {
        const uint32_t sd = __builtin_amdgcn_readfirstlane((uint32_t)D.gseed[q]);
        if (m1 > 0 && sd != kGramSeedNone) {  // wave-uniform
          // no string compare: equal values have equal non-empty gram sets, for which every
          // formula is exactly 1.0
          const int m2 = cmp ? (int)D.rgcnt[g] : 0;
          const int common = qgram_common_perfect(reinterpret_cast<uint32_t*>(peq), g1, m1, sd,
                                                  reinterpret_cast<const uint64_t*>(D.rgrams),
                                                  rstride, g, m2);
          if (m2 > 0) sim = qgram_formula(common, m1, m2, D.formula);
          break;
        }
      }
      const bool same = cmp && str_equal(s1, lq, s2, lc);
      if (m1 > 0 && m1 <= kQgramHashMax && g1[m1 - 1] != ~0ull) {  // wave-uniform
        sim = same ? 1.0 : 0.0;
        const int m2 = cmp && !same ? (int)D.rgcnt[g] : 0;
        // candidate codes: the transposed replica (coalesced), or in place (no replica, or
        // a bigram-key replica and a query without a perfect hash)
        const int common =
            !D.rgmax || D.g16 ? qgram_common_hashed(peq, g1, m1, D.grams + D.rgoff[g], 1, max(m2 - 1, 0), m2)
            : D.rg32 ? qgram_common_hashed(peq, g1, m1, reinterpret_cast<const uint32_t*>(D.rgrams) + g,
                                           rstride, D.rgmax - 1, m2)
                     : qgram_common_hashed(peq, g1, m1, reinterpret_cast<const uint64_t*>(D.rgrams) + g,
                                           rstride, D.rgmax - 1, m2);
        if (m2 > 0) sim = qgram_formula(common, m1, m2, D.formula);
      } else if (cmp) {
        if (same) {
          sim = 1.0;
        } else {
          const int m2 = D.rgcnt[g];
          if (m1 == 0 || m2 == 0) sim = 0.0;
          else sim = qgram_formula(intersect_sorted(g1, m1, D.grams + D.rgoff[g], m2), m1, m2, D.formula);
        }
      }
      break;
    }
    case DK_CMP_DICE_TOKENS:
    case DK_CMP_JACCARD_TOKENS:
      if (GR && cmp) {
        if (str_equal(s1, lq, s2, lc)) {
          sim = 1.0;
        } else {
          int m1 = D.gcnt[q], m2 = D.rgcnt[g];
          const uint64_t* t1 = D.grams + D.goff[q];
          const uint64_t* t2 = D.grams + D.rgoff[g];
          if (m1 > m2) {
            const uint64_t* tt = t1; t1 = t2; t2 = tt;
            const int tm = m1; m1 = m2; m2 = tm;
          }
          const int hit = count_members(t1, m1, t2, m2);
          // exact small integers in doubles: sum = hit, union = m1 + m2 - hit
          sim = D.op == DK_CMP_JACCARD_TOKENS ? (double)hit / (double)(m1 + m2 - hit)
                                              : ((double)hit * 2) / (double)(m1 + m2);
        }
      }
      break;
    default:
      break;
  }
  return sim;
}

// Block-ordered compaction of a 256-slot block's decisions: wave ballots -> per-wave
// counts in LDS -> slot-ordered entries at the block's staging region (no atomics on
// entries), plus the block's scored-pair and operand-byte sums.
__device__ __forceinline__ void block_emit_at(const StageOut& out, uint64_t blk, uint32_t kind,
                                              double prob, uint32_t crow, uint32_t qi,
                                              uint32_t scored, uint32_t bytes) {
  __shared__ uint32_t wcount[kScoreBlock / 64], wscored[kScoreBlock / 64], wbytes[kScoreBlock / 64];
  const uint32_t wave = threadIdx.x >> 6;
  const uint64_t em = __ballot(kind != 0);
  const uint32_t sb = wave_sum_u32(bytes), ss = wave_sum_u32(scored);
  if (lane_id() == 0) {
    wcount[wave] = (uint32_t)__popcll(em);
    wscored[wave] = ss;
    wbytes[wave] = sb;
  }
  __syncthreads();
  uint32_t before = 0, total = 0;
#pragma unroll
  for (int w = 0; w < kScoreBlock / 64; ++w) {
    const uint32_t cw = wcount[w];
    before += (uint32_t)w < wave ? cw : 0u;
    total += cw;
  }
  if (kind != 0) {
    const uint64_t e = blk * kScoreBlock + before + mask_rank(em);
    out.prob[e] = prob;
    out.cand[e] = crow | (kind << kKindShift);
    out.qidx[e] = qi;
  }
  if (threadIdx.x == 0) {
    uint32_t ns = 0, nb = 0;
#pragma unroll
    for (int w = 0; w < kScoreBlock / 64; ++w) {
      ns += wscored[w];
      nb += wbytes[w];
    }
    out.bcnt[blk] = total;
    out.bscored[blk] = ns;
    out.bbytes[blk] = nb;
  }
  __syncthreads();  // the counts in LDS are reused by the block's next call
}

__device__ __forceinline__ void block_emit(const StageOut& out, uint32_t kind, double prob,
                                           uint32_t crow, uint32_t qi, uint32_t scored,
                                           uint32_t bytes) {
  block_emit_at(out, blockIdx.x, kind, prob, crow, qi, scored, bytes);
}

// SYM: the owner slots of the symmetric dedup schedule (PairSource::sym): every owned pair
// is scored in both directions in one pass and the two probabilities go to S.ores; the
// emission pass (k_sym_emit) turns them into the match list.
template <int RMAX, int LR, bool SYM, bool DP, bool GR = true, bool GEO = false>
__device__ __forceinline__ void score_body(const ScoreParams& P, const PairSource& S, uint64_t slot0,
                                           uint64_t nslots, const StageOut& out) {
  uint64_t* peq = g_wave_tables[threadIdx.x >> 6];
  for (int e = (int)lane_id(); e < kPeqEntries; e += 64) peq[e] = 0;

  const uint64_t bid = blockIdx.x;
  const uint64_t idx = bid * blockDim.x + threadIdx.x;
  const bool in_launch = idx < nslots;
  bool valid = in_launch;
  const uint64_t s = slot0 + min(idx, nslots - 1);
  uint32_t qi = 0, g = 0;
  bool mirror = false;  // SYM: the candidate is a query too (the reverse pair is owned here)
  int ksel = 0;         // SYM: key function of the slot, and the query's offset in the
  uint32_t moff = 0;    // candidate's mirror run (its own bucket position - the run's start)
  if (S.allpairs) {
    // slots of a query: [qi * mpad, qi * mpad + m), mpad = m rounded up to 64
    qi = (uint32_t)(s / S.mpad);
    const uint64_t t = s - (uint64_t)qi * S.mpad;
    valid = valid && t < S.m;
    g = valid ? (uint32_t)t : 0u;
  } else {
    // one query per wave by construction (padded slot layout): the wave's first slot,
    // computed wave-uniformly, so the map read is a scalar load at the head of the chain
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t sw = slot0 + min(bid * blockDim.x + (uint64_t)wave * 64u, nslots - 1);
    qi = S.wq[sw >> 6];
  }
  qi = __builtin_amdgcn_readfirstlane(qi);
  const uint32_t q = __builtin_amdgcn_readfirstlane(S.queries[qi]);
  if (!S.allpairs) {
    // Candidate t of the query: key function k's range first, then (group, row) order
    // inside it.  Filters: isSameAs (identity), and "already a candidate under an
    // earlier key function" (Duke returns candidates as a set).  The ranges and the
    // query's keys are wave-uniform.
    uint64_t t = s - S.qoff[qi];
    int k = -1;
    // the first kPre segments' ranges issued together (clamped: no branch around the loads);
    // the loop is unrolled, so each segment's range is a register, not a serial load + wait
    constexpr int kPre = 4;
    uint4 pre4[kPre];
    uint2 pre2[kPre];
#pragma unroll
    for (int kk = 0; kk < kPre; ++kk) {
      const uint64_t at = (uint64_t)min(kk, S.nseg - 1) * S.nq + qi;
      if (SYM) pre4[kk] = S.sranges[at];
      else pre2[kk] = S.ranges[at];
    }
#pragma unroll
    for (int kk = 0; kk < kMaxSegs; ++kk) {
      if (kk >= S.nseg) break;  // wave-uniform
      if (SYM) {  // owned candidates: [lo, qa) then (pq, hi)
        const uint4 r = kk < kPre ? pre4[kk < kPre ? kk : 0] : S.sranges[(uint64_t)kk * S.nq + qi];
        const bool in_t = r.w != kNoPos;
        const uint64_t nlow = r.z - r.x;
        const uint64_t len = nlow + (in_t ? (uint64_t)(r.y - r.w - 1) : 0);
        if (k < 0) {
          if (t < len) {
            k = kk;
            const uint64_t x = t < nlow ? r.x + t : r.w + 1 + (t - nlow);
            g = (uint32_t)(S.segoff[kk] + x);
            mirror = in_t;
            ksel = kk;
            moff = r.w - r.z;
          } else {
            t -= len;
          }
        }
      } else {
        const uint2 r = kk < kPre ? pre2[kk < kPre ? kk : 0] : S.ranges[(uint64_t)kk * S.nq + qi];
        const uint64_t len = (uint64_t)(r.y - r.x);
        if (k < 0) {
          if (t < len) {
            k = kk;
            g = (uint32_t)(S.segoff[kk] + r.x + t);
          } else {
            t -= len;
          }
        }
      }
    }
    valid = valid && k >= 0;
    if (!valid) g = 0u;  // lanes without a pair read replica position 0 (always in range)
    // isSameAs, and a base position superseded since the base was sorted (kDeadIdent)
    const uint64_t rid = S.rident[g];
    bool ok = rid != P.ident[q] && rid != kDeadIdent;
    const int kf = k >> S.seg_shift;  // the segment's key function
    for (int j = 0; j < S.nkeys - 1; ++j)
      if (j < kf) ok = ok && S.rkeys[j][g] != S.qkeys[j][q];
    valid = valid && ok;
  }
  const uint32_t crow = P.rowof[g];
  if (S.allpairs && !S.same_ok) valid = valid && P.ident[crow] != P.ident[q];  // Processor.isSameAs
  // the high segment (pq, hi) holds rows above the query's own; those below r1 are queries
  if (SYM) mirror = mirror && valid && crow >= S.r0 && crow < S.r1;
  wave_lds_sync();

  double prob = P.raw_prop < 0 ? 0.5 : __builtin_nan("");
  double prob2 = 0.5;  // SYM: Processor.compare(candidate, query)
  bool asym = false;   // SYM: a JaroWinkler property came before (prob2 may differ from prob)
  uint32_t bytes = valid ? 9u : 0u;  // two row ids + decision (SURVEY §8d B_pair)
  // property p+1's query length, this lane's query unit (its Peq bit) and the candidate's
  // length are loaded while property p computes: a property then starts without the
  // length -> offset -> unit chain of dependent loads
  auto prefetch = [&](int pp, int& lq_, uint32_t& ch_, int& lc_) {
    const DevProp& E = P.props[pp];
    lq_ = (int)__builtin_amdgcn_readfirstlane((uint32_t)E.len[q]);
    const int lane = (int)lane_id();
    ch_ = 0u;
    const bool table = DP && (E.op == DK_CMP_LEVENSHTEIN || E.op == DK_CMP_JAROWINKLER);  // Peq users
    if (table && lq_ != (int)kMissing && lane < lq_ && lane < 64) {
      const uint32_t o = __builtin_amdgcn_readfirstlane(E.off[q]);
      ch_ = E.width == 1 ? (uint32_t)reinterpret_cast<const uint8_t*>(E.units)[o + lane]
                         : (uint32_t)reinterpret_cast<const uint16_t*>(E.units)[o + lane];
    }
    lc_ = valid ? (int)__hip_atomic_load(E.rlen + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (int)kMissing;
  };
  int lq_n = 0, lc_n = (int)kMissing;
  uint32_t qch_n = 0u;
  // Processor.compare visits r1's (the query's) properties in its RecordImpl HashMap order,
  // which depends on the map's capacity: the query row's order class (dk_schema.orders)
  const uint64_t ow =
      order_word(P, P.norders > 1 ? (int)__builtin_amdgcn_readfirstlane((uint32_t)P.oclass[q]) : 0);
  if (P.nprops > 0) prefetch(order_at(ow, 0), lq_n, qch_n, lc_n);
  for (int p = 0; p < P.nprops; ++p) {
    const int pp = order_at(ow, p);
    const DevProp& D = P.props[pp];
    const int lq = lq_n;
    const int lc = lc_n;
    const uint32_t qch = qch_n;
    if (p + 1 < P.nprops) prefetch(order_at(ow, p + 1), lq_n, qch_n, lc_n);
    if (lq == (int)kMissing) continue;  // r1 has no value: property skipped for the wave
    const bool present = lc != (int)kMissing;
    const bool cmp = present && lq > 0 && lc > 0;
    double sim = 0.0, rev = 0.0;
    // algorithmic bytes: the CANDIDATE's operands at their stored
    // width -- the query's value is read once per wave (LDS tables), not per pair
    if (present) bytes += 2u;  // rlen
    if (D.op == DK_CMP_NUMERIC) {
      if (cmp) sim = numeric(D.num[q], D.numok[q] != 0, D.rnum[g], D.rnumok[g] != 0, D.min_ratio);
      if (cmp) bytes += 9u;   // rnum + rnumok
      rev = sim;
    } else if (GEO && D.op == DK_CMP_GEOPOSITION) {
      if (cmp) {
        const uint32_t ok1 = D.numok[q], ok2 = D.rnumok[g];
        if (ok1 == 2u || ok2 == 2u)  // a value without ',': Duke raises on this comparison
          __hip_atomic_fetch_or(P.raised, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sim = geoposition(D.num[2 * q], D.num[2 * q + 1], ok1 == 1u, D.rnum[2 * g], D.rnum[2 * g + 1],
                          ok2 == 1u, D.min_ratio);
      }
      if (cmp) bytes += 17u;  // rnum pair + rnumok
      rev = sim;
    } else if (D.op != DK_CMP_NONE) {
      rev = __builtin_nan("");  // marks "same as sim" unless the comparator sets it
      // a property on the long-value DP for this wave (wave-uniform): the pre-pass's slot
      sim = D.width == 1 ? string_sim<RMAX, LR, uint8_t, SYM, DP, GR>(D, P.rstride, peq, q, g, crow, lq, lc, cmp, rev, qch)
                         : string_sim<RMAX, LR, uint16_t, SYM, DP, GR>(D, P.rstride, peq, q, g, crow, lq, lc, cmp, rev, qch);
      if (!SYM || rev != rev) rev = sim;
      if (cmp) {
        if (D.op == DK_CMP_QGRAM)  // the candidate's gram codes (u32 replica codes for q <= 2,
                                   // 16-bit keys for Latin-1 bigrams)
          bytes += 6u + (D.g16 ? 2u : D.rg32 && D.rgmax ? 4u : 8u) * (uint32_t)D.rgcnt[g];
        else if (uses_codes(D.op))  // token ids
          bytes += 6u + 8u * (uint32_t)D.rgcnt[g];
        else
          bytes += (uint32_t)lc * (uint32_t)D.width;
      }
    }
    if (SYM && D.op == DK_CMP_JAROWINKLER) asym = true;  // wave-uniform
    if (pp == P.raw_prop) {  // Comparator.compare(v1, v2) itself (wave-uniform branch)
      if (cmp) prob = sim;
      break;
    }
    if (present) {
      // [Duke 1.2] Processor.compare: high = max(0.0, PropertyImpl.compare) over the value
      // pairs (one each here), then computeBayes
      prob = compute_bayes(prob, cmp ? property_prob(D, sim) : 0.0);
      // the reverse direction differs only from the first JaroWinkler property on (every
      // other comparator of the symmetric schedule has rev == sim): until then prob2 == prob
      // bit for bit, and its computeBayes would repeat prob's
      if (SYM) prob2 = asym ? compute_bayes(prob2, cmp ? property_prob(D, rev) : 0.0) : prob;
    }
  }

  if (SYM) {
    // the owner decision byte for this query's list (its probability only for an entry); the
    // reverse direction into the candidate's mirror segment (scattered stores while the
    // VALU-bound wave keeps computing) when it is an entry -- the rest of that segment keeps
    // its cleared decision bytes
    const uint32_t kind = valid ? decide(prob, P.threshold, P.maybe) : 0u;
    if (in_launch) {
      S.okind[s] = (uint8_t)kind;
      if (kind != 0u) S.ores[s] = prob;
    }
    const uint32_t kind2 = mirror ? decide(prob2, P.threshold, P.maybe) : 0u;
    if (kind2 != 0u) {
      const uint64_t m = S.mbase[(uint64_t)ksel * S.nq + (crow - S.r0)] + moff;
      S.mkind[m] = (uint8_t)kind2;
      S.mres[m] = prob2;
    }
    block_emit_at(out, bid, 0u, 0.0, 0u, qi, valid ? (mirror ? 2u : 1u) : 0u, bytes);  // operands read once
  } else {
    const uint32_t kind = valid ? decide(prob, P.threshold, P.maybe) : 0u;
    block_emit_at(out, bid, kind, prob, crow, qi, valid ? 1u : 0u, bytes);
  }
}

// The fused scoring kernel.  Short-value variants pin the occupancy (the DP is
// latency-bound: 7 waves/SIMD up to 40 rows -- spills and all, measured faster than 5 or 6 -- 4 above); the long-value variants (LR > 0)
// carry the systolic DP's f64 rows and take what the register allocator needs.
// GR = false: no QGram / token property (the dedup headline's Levenshtein + JaroWinkler):
// the gram-set code and its registers are compiled out.
template <int RMAX, bool SYM, bool GR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RMAX <= 40 ? DK_WAVES_SHORT : 4, 8)))
void k_score(const ScoreParams P, const PairSource S, uint64_t slot0, uint64_t nslots, StageOut out) {
  score_body<RMAX, 0, SYM, true, GR>(P, S, slot0, nslots, out);
}

// The symmetric owner schedule with TWO queries per wave (PairSource::two): the owner slots
// are packed so that a wave holds at most two queries, the second from any lane on (k_opack)
// -- configs[1]'s owned lists waste ~2 % of their slots on padding, against 13.3 % with every
// query padded to a wave (6.7 % to a half-wave).
// Schemas of Latin-1 Levenshtein / JaroWinkler, Exact and Numeric properties in one HashMap
// order class (the host checks: dk_api.cpp sym2_ok): the wave's two Peq tables fit its LDS
// slice (256 entries each), the row bucket covers the longer query value, and the query side
// of every comparator is per lane (its query); the rest is score_body's SYM path.
template <int RMAX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RMAX <= 40 ? DK_WAVES_SYM2 : 4, 8)))
void k_score_sym2(const ScoreParams P, const PairSource S, uint64_t slot0, uint64_t nslots, StageOut out) {
  uint64_t* tab = g_wave_tables[threadIdx.x >> 6];
  for (int e = (int)lane_id(); e < kPeqEntries; e += 64) tab[e] = 0;
  const int lane = (int)lane_id();
  const uint64_t bid = blockIdx.x;
  const uint64_t idx = bid * blockDim.x + threadIdx.x;
  const uint64_t s = slot0 + min(idx, nslots - 1);
  // slot0 is wave-aligned: the launch's first wave may start with the previous launch's
  // query (slots below olo: neither scored nor written)
  const bool in_launch = idx < nslots && s >= S.olo;
  bool valid = in_launch;
  // the wave's two queries (scalar loads; equal when one query fills the wave): A from lane
  // 0, B from its first slot qoff[B] on
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t w0 = bid * blockDim.x + (uint64_t)wave * 64u;
  const uint2 wqp = S.wq2[(slot0 + min(w0, nslots - 1)) >> 6];
  const uint32_t qiA = __builtin_amdgcn_readfirstlane(wqp.x);
  const uint32_t qiB = __builtin_amdgcn_readfirstlane(wqp.y);
  const bool two = qiA != qiB;  // wave-uniform
  const uint64_t offA = S.qoff[qiA], offB = S.qoff[qiB];
  const bool hi = two && s >= offB;
  const uint32_t qA = __builtin_amdgcn_readfirstlane(S.queries[qiA]);
  const uint32_t qB = __builtin_amdgcn_readfirstlane(S.queries[qiB]);
  const uint32_t q = hi ? qB : qA;
  uint64_t* peq = tab + (hi ? 256 : 0);  // this lane's query's Peq table
  uint32_t g = 0;
  bool mirror = false;
  int ksel = 0;
  uint32_t moff = 0;
  {
    // owner slot t of the lane's query: key function k's owned range [lo, qa) then (pq, hi)
    uint64_t t = s - (hi ? offB : offA);
    int k = -1;
    constexpr int kPre = 2;  // the two queries' first ranges as scalars (SGPR budget)
    uint4 pa[kPre], pb[kPre];
#pragma unroll
    for (int kk = 0; kk < kPre; ++kk) {
      const uint64_t at = (uint64_t)min(kk, S.nseg - 1) * S.nq;
      pa[kk] = S.sranges[at + qiA];
      pb[kk] = S.sranges[at + qiB];
    }
#pragma unroll
    for (int kk = 0; kk < kMaxSegs; ++kk) {
      if (kk >= S.nseg) break;  // wave-uniform
      const uint4 ra = kk < kPre ? pa[kk < kPre ? kk : 0] : S.sranges[(uint64_t)kk * S.nq + qiA];
      const uint4 rb = kk < kPre ? pb[kk < kPre ? kk : 0] : S.sranges[(uint64_t)kk * S.nq + qiB];
      const uint4 r = hi ? rb : ra;
      const bool in_t = r.w != kNoPos;
      const uint64_t nlow = r.z - r.x;
      const uint64_t len = nlow + (in_t ? (uint64_t)(r.y - r.w - 1) : 0);
      if (k < 0) {
        if (t < len) {
          k = kk;
          const uint64_t x = t < nlow ? r.x + t : r.w + 1 + (t - nlow);
          g = (uint32_t)(S.segoff[kk] + x);
          mirror = in_t;
          ksel = kk;
          moff = r.w - r.z;
        } else {
          t -= len;
        }
      }
    }
    valid = valid && k >= 0;
    if (!valid) g = 0u;
    const uint64_t rid = S.rident[g];
    const uint64_t ida = P.ident[qA], idb = P.ident[qB];
    bool ok = rid != (hi ? idb : ida) && rid != kDeadIdent;
    const int kf = k >> S.seg_shift;
    for (int j = 0; j < S.nkeys - 1; ++j) {
      const uint64_t ka = S.qkeys[j][qA], kb = S.qkeys[j][qB];
      if (j < kf) ok = ok && S.rkeys[j][g] != (hi ? kb : ka);
    }
    valid = valid && ok;
  }
  const uint32_t crow = P.rowof[g];
  mirror = mirror && valid && crow >= S.r0 && crow < S.r1;
  wave_lds_sync();

  double prob = 0.5, prob2 = 0.5;
  bool asym = false;
  uint32_t bytes = valid ? 9u : 0u;
  // the next property's query lengths, this lane's unit of each query (Peq bits) and the
  // candidate's length, loaded while the current property computes
  auto prefetch = [&](int pp, int& la, int& lb, uint32_t& ca, uint32_t& cb, int& lc_) {
    const DevProp& E = P.props[pp];
    la = (int)__builtin_amdgcn_readfirstlane((uint32_t)E.len[qA]);
    lb = (int)__builtin_amdgcn_readfirstlane((uint32_t)E.len[qB]);
    ca = cb = 0u;
    if (E.op == DK_CMP_LEVENSHTEIN || E.op == DK_CMP_JAROWINKLER) {
      const uint8_t* u = reinterpret_cast<const uint8_t*>(E.units);
      if (la != (int)kMissing && lane < la && lane < 64)
        ca = u[__builtin_amdgcn_readfirstlane(E.off[qA]) + lane];
      if (two && lb != (int)kMissing && lane < lb && lane < 64)
        cb = u[__builtin_amdgcn_readfirstlane(E.off[qB]) + lane];
    }
    lc_ = valid ? (int)__hip_atomic_load(E.rlen + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (int)kMissing;
  };
  // the wave's Peq tables: query A's in [0, 256), query B's in [256, 512) (two queries) --
  // set (on) or cleared
  // (narrow: 32-bit entries, peq_set_unit, when both queries have <= kPeqNarrow units)
  auto tables = [&](int la, int lb, uint32_t ca, uint32_t cb, bool on) {
    if (peq_narrow(max(la, lb))) {
      uint32_t* t32 = reinterpret_cast<uint32_t*>(tab);
      const uint32_t bit = 1u << (lane & 31);
      if (lane < la) {
        if (on) atomicOr(&t32[ca], bit);
        else t32[ca] = 0;
      }
      if (two && lane < lb) {
        if (on) atomicOr(&t32[512 + cb], bit);
        else t32[512 + cb] = 0;
      }
    } else {
      const uint64_t bit = 1ull << lane;
      if (lane < la) {
        if (on) atomicOr((unsigned long long*)&tab[ca], (unsigned long long)bit);
        else tab[ca] = 0;
      }
      if (two && lane < lb) {
        if (on) atomicOr((unsigned long long*)&tab[256 + cb], (unsigned long long)bit);
        else tab[256 + cb] = 0;
      }
    }
    wave_lds_sync();
  };
  const uint64_t ow = P.order[0];
  int la_n = 0, lb_n = 0, lc_n = (int)kMissing;
  uint32_t ca_n = 0u, cb_n = 0u;
  if (P.nprops > 0) prefetch(order_at(ow, 0), la_n, lb_n, ca_n, cb_n, lc_n);
  for (int p = 0; p < P.nprops; ++p) {
    const int pp = order_at(ow, p);
    const DevProp& D = P.props[pp];
    const int la = la_n, lb = lb_n, lc = lc_n;
    const uint32_t ca = ca_n, cb = cb_n;
    if (p + 1 < P.nprops) prefetch(order_at(ow, p + 1), la_n, lb_n, ca_n, cb_n, lc_n);
    const bool ma = la == (int)kMissing, mb = !two || lb == (int)kMissing;
    if (ma && (mb || !two)) continue;  // no query of the wave has a value: skipped
    const int lq = hi ? lb : la;
    const bool qmiss = lq == (int)kMissing;  // r1 has no value: the property is skipped
    const bool present = !qmiss && lc != (int)kMissing;
    const bool cmp = present && lq > 0 && lc > 0;
    double sim = 0.0, rev = __builtin_nan("");
    if (present) bytes += 2u;
    const Str<uint8_t> s1{reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(D.units) + D.off[q]),
                          1, 1 << 30};
    const Str<uint8_t> s2 = D.rlmax ? Str<uint8_t>{reinterpret_cast<const uint32_t*>(D.runits) + g, P.rstride,
                                                   D.rlmax / 4 - 1}
                                    : Str<uint8_t>{reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(D.units) + D.off[crow]),
                                                   1, 1 << 30};
    if (D.op == DK_CMP_NUMERIC) {
      if (cmp) sim = numeric(D.num[q], D.numok[q] != 0, D.rnum[g], D.rnumok[g] != 0, D.min_ratio);
      if (cmp) bytes += 9u;
    } else if (D.op == DK_CMP_EXACT) {
      if (cmp) sim = str_equal(s1, lq, s2, lc) ? 1.0 : 0.0;
      if (cmp) bytes += (uint32_t)lc;
    } else if (D.op == DK_CMP_LEVENSHTEIN || D.op == DK_CMP_JAROWINKLER) {
      const int nmax = max(ma ? 0 : la, mb ? 0 : lb);  // wave-uniform: the row bucket / mask width
      const int n1 = qmiss ? 0 : lq;
      const bool table = nmax <= 64 && (D.op == DK_CMP_LEVENSHTEIN || __ballot(cmp && lc > 64) == 0);
      if (table) {
        tables(ma ? 0 : la, mb ? 0 : lb, ca, cb, true);
        if (D.op == DK_CMP_LEVENSHTEIN) {
          sim = levenshtein_peq<RMAX, uint8_t, true>(peq, s1, n1, s2, lc, cmp, nmax);
        } else {
          double r = 0.0;
          sim = nmax <= DK_JW_NARROW ? jarowinkler_peq<uint32_t, uint8_t, true>(peq, s1, n1, s2, lc, cmp, &r)
                                     : jarowinkler_peq<uint64_t, uint8_t, true>(peq, s1, n1, s2, lc, cmp, &r);
          rev = r;
        }
        tables(ma ? 0 : la, mb ? 0 : lb, ca, cb, false);
      } else if (cmp) {
        sim = jarowinkler(s1, lq, s2, lc);
        rev = lq == lc ? jarowinkler(s2, lc, s1, lq) : sim;
      }
      if (cmp) bytes += (uint32_t)lc;
    }
    if (rev != rev) rev = sim;
    if (D.op == DK_CMP_JAROWINKLER) asym = true;  // wave-uniform
    if (present) {
      prob = compute_bayes(prob, cmp ? property_prob(D, sim) : 0.0);
      prob2 = asym ? compute_bayes(prob2, cmp ? property_prob(D, rev) : 0.0) : prob;
    }
  }
  const uint32_t kind = valid ? decide(prob, P.threshold, P.maybe) : 0u;
  if (in_launch) {  // padding slots too (the count pass reads them as 0)
    S.okind[s] = (uint8_t)kind;
    if (kind != 0u) S.ores[s] = prob;
  }
  const uint32_t kind2 = mirror ? decide(prob2, P.threshold, P.maybe) : 0u;
  if (kind2 != 0u) {
    const uint64_t m = S.mbase[(uint64_t)ksel * S.nq + (crow - S.r0)] + moff;
    S.mkind[m] = (uint8_t)kind2;
    S.mres[m] = prob2;
  }
  block_emit_at(out, bid, 0u, 0.0, 0u, 0u, valid ? (mirror ? 2u : 1u) : 0u, bytes);
}

// Schemas without a DP comparator (QGram / Numeric / Exact / token comparators: configs[2]'s
// linkage): none of the DP code, its registers or its spills; the kernel is memory-latency
// bound, so it takes the occupancy instead.
template <bool SYM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DK_WAVES_NODP, 8)))
void k_score_nodp(const ScoreParams P, const PairSource S, uint64_t slot0, uint64_t nslots, StageOut out) {
  score_body<16, 0, SYM, false>(P, S, slot0, nslots, out);
}

// Long values (WeightedLevenshtein, Levenshtein over 64 units): the fused kernel with the DP
// as an out-of-line call (long_dp).
template <int RMAX, int LR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DK_WAVES_LONG8, 8)))
void k_score_long(const ScoreParams P, const PairSource S, uint64_t slot0, uint64_t nslots, StageOut out) {
  score_body<RMAX, LR, false, true, true, false>(P, S, slot0, nslots, out);
}

// Schemas with a GeopositionComparator (P.has_geo; never the symmetric schedule): the direct
// schedule's widest variants with the haversine compiled in -- the f64 sin / cos keep a
// scratch frame for large-argument reduction, which only these variants carry.  Their
// occupancy targets are the widest plain variants': long_dp is a called function, whose
// register budget follows the most permissive of its callers.
template <bool DP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_score_geo(const ScoreParams P, const PairSource S, uint64_t slot0,
                                                   uint64_t nslots, StageOut out) {
  score_body<64, 0, false, DP, true, true>(P, S, slot0, nslots, out);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DK_WAVES_LONG16, 8))) void k_score_long_geo(const ScoreParams P, const PairSource S, uint64_t slot0,
                                                        uint64_t nslots, StageOut out) {
  score_body<64, 16, false, true, true, true>(P, S, slot0, nslots, out);
}

// Emission pass of the symmetric dedup schedule: one wave per query walks
// its candidates in Duke's order -- per segment k the bucket positions [lo, hi) without
// its own position pq: [lo, qa) and (pq, hi) it owns (okind / ores at its owner slots),
// [qa, pq) are owned by the earlier queries there, which pushed their reverse decision to
// its mirror run (mkind / mres) -- reading one decision byte per candidate, kEmitBatch
// steps of 64 candidates with their loads issued together (the pass is latency bound).
// WRITE = false: the query's entries -> ecount[qi].  WRITE = true (after the inclusive scan
// of the chunk's counts): its entries in order at list position base + eincl[qi] -
// ecount[qi] on, with their candidate rows and probabilities, and first[qi] (the chunk's
// last query first[qi + 1] too).  No staging, no compaction and no per-entry query index:
// the list is written where it ends up.
#ifndef DK_EMIT_BATCH
#define DK_EMIT_BATCH 8
#endif
constexpr int kEmitBatch = DK_EMIT_BATCH;

struct EmitSeg {
  uint64_t start;       // first index of the segment in the query's candidate order
  uint64_t ob, mb, so;  // owner slot / mirror slot of position qa, first replica position
  uint32_t lo, qa, pq, pad;
};

// The count pass: kCountLanes threads per query count the non-zero decision bytes of its
// owner slots [oqoff[qi], + ocnt[qi]) (padding slots hold 0) and of its mirror slots
// [mqoff[qi], mqoff[qi + 1]) -- both contiguous runs, read 16 bytes per thread and step --
// instead of walking the candidate order (a wave per query was latency bound; a thread per
// query left a chunk's launch a few waves per CU).
constexpr int kCountLanes = 8;

__device__ __forceinline__ uint32_t nz_bytes(uint32_t x) {  // decision bytes are 0, 1 or 2
  return (uint32_t)__popc((x | (x >> 1)) & 0x01010101u);
}

// this thread's share (16-B blocks k, k + kCountLanes, ...) of the run [a, e) of base
__device__ __forceinline__ uint32_t nz_run(const uint8_t* base, uint64_t a, uint64_t e, uint32_t k) {
  uint32_t n = 0;
  for (uint64_t p = (a & ~(uint64_t)15) + 16u * k; p < e; p += 16u * kCountLanes) {
    const uint4 v = *reinterpret_cast<const uint4*>(base + p);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t b0 = p + 4 * j;  // bytes [b0, b0 + 4) of the run's buffer
      uint32_t x = w[j];
      if (b0 < a) x = a - b0 >= 4 ? 0u : x & (~0u << (8 * (a - b0)));
      if (b0 + 4 > e) x = b0 >= e ? 0u : x & (~0u >> (8 * (b0 + 4 - e)));
      n += nz_bytes(x);
    }
  }
  return n;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DK_WAVES_COUNT, 8))) void k_sym_count(const EmitSource S, uint64_t q0, uint64_t nqc) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t i = t / kCountLanes;
  const uint32_t k = (uint32_t)(t % kCountLanes);
  uint32_t n = 0;
  const uint64_t qi = q0 + min(i, nqc - 1);
  if (i < nqc) {
    const uint64_t oa = S.oqoff[qi], oe = S.ocnt ? oa + S.ocnt[qi] : S.oqoff[qi + 1];
    n = nz_run(S.okind, oa, oe, k) + nz_run(S.mkind, S.mqoff[qi], S.mqoff[qi + 1], k);
  }
#pragma unroll
  for (int o = kCountLanes / 2; o > 0; o >>= 1) n += __shfl_xor(n, o, kCountLanes);
  if (i < nqc && k == 0) S.ecount[qi] = n;
}

// the write pass is latency bound: 8 waves per SIMD (<= 64 VGPRs) rather than the 6 its
// registers would give (configs[1] write pass 2.19 -> 1.68 ms per step)
#ifndef DK_WAVES_EMIT
#define DK_WAVES_EMIT 8
#endif
template <bool WRITE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DK_WAVES_EMIT, 8))) void k_sym_emit(const EmitSource S, uint64_t q0, uint64_t nqc,
                                                  uint64_t base, MatchList out,
                                                  uint64_t* __restrict__ first) {
  __shared__ EmitSeg seg[kScoreBlock / 64][kMaxSegs];
  const uint32_t wave = threadIdx.x >> 6, lane = lane_id();
  const uint64_t wi = (uint64_t)blockIdx.x * (kScoreBlock / 64) + wave;
  if (wi >= nqc) return;  // wave-uniform; no block barrier follows
  const uint64_t qi = q0 + wi;
  const int nseg = S.nseg;
  EmitSeg* sg = seg[wave];
  uint64_t len = 0;
  if ((int)lane < nseg) {  // lane k: segment k's record
    const uint64_t at = (uint64_t)lane * S.nq + qi;
    const uint4 r = S.sranges[at];
    len = (uint64_t)(r.y - r.x) - (r.w != kNoPos ? 1u : 0u);
    uint64_t so = 0;
#pragma unroll
    for (int j = 0; j < kMaxSegs; ++j) so = (int)lane == j ? S.segoff[j] : so;
    sg[lane].ob = S.obase[at];
    sg[lane].mb = S.mbase[at];
    sg[lane].so = so;
    sg[lane].lo = r.x;
    sg[lane].qa = r.z;
    sg[lane].pq = r.w;
  }
  uint64_t incl = len;  // inclusive prefix over the segments (lanes past nseg add 0)
#pragma unroll
  for (int o = 1; o < kMaxSegs; o <<= 1) {
    const uint64_t y = __shfl_up(incl, (unsigned)o);
    if ((int)lane >= o) incl += y;
  }
  if ((int)lane < nseg) sg[lane].start = incl - len;
  const uint64_t tot = __shfl(incl, nseg - 1);
  const uint64_t L = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(tot >> 32)) << 32) |
                     __builtin_amdgcn_readfirstlane((uint32_t)tot);
  wave_lds_sync();
  uint64_t at0 = 0;
  if (WRITE) at0 = base + S.eincl[qi] - S.ecount[qi];
  uint64_t n = 0;  // entries so far (wave-uniform)
  for (uint64_t t0 = 0; t0 < L; t0 += 64 * kEmitBatch) {
    uint32_t kind[kEmitBatch], pos[kEmitBatch];
    uint64_t idx[kEmitBatch];
    bool mir[kEmitBatch];
#pragma unroll
    for (int u = 0; u < kEmitBatch; ++u) {
      const uint64_t t = t0 + (uint64_t)u * 64 + lane;
      int k = 0;
      for (int j = 1; j < nseg; ++j) k = t >= sg[j].start ? j : k;
      const EmitSeg& e = sg[k];
      uint32_t x = e.lo + (uint32_t)(t - e.start);
      if (x >= e.pq) ++x;  // past the query's own position (kNoPos: not in the table)
      const bool m = x >= e.qa && x < e.pq;
      idx[u] = m ? e.mb + (x - e.qa) : (x < e.qa ? e.ob - (uint64_t)(e.qa - x) : e.ob + (x - e.pq - 1u));
      mir[u] = m;
      pos[u] = (uint32_t)(e.so + x);
      kind[u] = t < L ? (uint32_t)(m ? S.mkind[idx[u]] : S.okind[idx[u]]) : 0u;
    }
    if (WRITE) {
      // every in-range candidate's probability and row loaded with its decision byte (one
      // memory round trip, not two: at ~1 entry in 4 candidates an entry-only load touches
      // the same cache lines)
      double pr[kEmitBatch];
      uint32_t crow[kEmitBatch];
#pragma unroll
      for (int u = 0; u < kEmitBatch; ++u) {
        const bool in = t0 + (uint64_t)u * 64 + lane < L;
        pr[u] = in ? (mir[u] ? S.mres[idx[u]] : S.ores[idx[u]]) : 0.0;
        crow[u] = in ? S.rowof[pos[u]] : 0u;
      }
#pragma unroll
      for (int u = 0; u < kEmitBatch; ++u) {
        const uint64_t em = __ballot(kind[u] != 0u);
        if (kind[u] != 0u) {
          const uint64_t o = at0 + n + mask_rank(em);
          out.cand[o] = crow[u];
          out.kind[o] = (uint8_t)kind[u];
          out.prob[o] = pr[u];
        }
        n += (uint64_t)__popcll(em);
      }
    } else {
#pragma unroll
      for (int u = 0; u < kEmitBatch; ++u) n += (uint64_t)__popcll(__ballot(kind[u] != 0u));
    }
  }
  if (lane == 0) {
    if (!WRITE) {
      S.ecount[qi] = (uint32_t)n;
    } else {
      first[qi] = at0;
      if (wi + 1 == nqc) first[qi + 1] = at0 + n;
    }
  }
}

// Sum the per-block counters of a chunk into counters[0..1]: one atomic pair per block
// of this kernel (a same-address atomic per score wave serialises at the memory side).
__global__ __launch_bounds__(256) void k_reduce_blocks(const StageOut st, uint64_t nblocks) {
  uint64_t a = 0, b = 0, x = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nblocks;
       i += (uint64_t)gridDim.x * blockDim.x) {
    a += st.bscored[i];
    b += st.bbytes[i];
    if (st.bexact) x += st.bexact[i];
  }
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    b += __shfl_xor(b, o);
    x += __shfl_xor(x, o);
  }
  __shared__ uint64_t sa[4], sbb[4], sx[4];
  if (lane_id() == 0) {
    sa[threadIdx.x >> 6] = a;
    sbb[threadIdx.x >> 6] = b;
    sx[threadIdx.x >> 6] = x;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    a = sa[0] + sa[1] + sa[2] + sa[3];
    b = sbb[0] + sbb[1] + sbb[2] + sbb[3];
    x = sx[0] + sx[1] + sx[2] + sx[3];
    if (a) atomicAdd((unsigned long long*)&st.counters[0], (unsigned long long)a);
    if (b) atomicAdd((unsigned long long*)&st.counters[1], (unsigned long long)b);
    if (x) atomicAdd((unsigned long long*)&st.counters[3], (unsigned long long)x);
  }
}

// Concatenate the per-block staged entries in block order.  A wave takes kCompactRun
// consecutive staging blocks at a time: their counts in one read, then the run's entries as
// ONE sequence, 64 per step (entry i of the run: the block whose inclusive count prefix first
// exceeds i), so a step's lanes are full across block boundaries -- configs[1] stages ~70
// entries per block, which a step per block left half idle -- and the run's destination is
// contiguous.  (One workgroup per staging block spent most of its time dispatching
// workgroups with nothing to copy: sparse match lists, configs[2].)
constexpr int kCompactRun = 16;

__global__ __launch_bounds__(256) void k_compact(const StageOut st, const uint64_t* __restrict__ boff,
                                                 uint64_t nblocks, uint64_t base, MatchList out) {
  const uint32_t lane = lane_id();
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t b0 = wave * kCompactRun; b0 < nblocks; b0 += nwaves * kCompactRun) {
    const uint64_t b = b0 + lane;
    const uint32_t n = lane < (uint32_t)kCompactRun && b < nblocks ? st.bcnt[b] : 0u;
    uint32_t incl = n;  // inclusive prefix over the run's blocks (lanes past them add 0)
#pragma unroll
    for (int o = 1; o < kCompactRun; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)incl, (unsigned)o);
      if (lane >= (uint32_t)o) incl += y;
    }
    uint32_t pre[kCompactRun];  // wave-uniform
#pragma unroll
    for (int k = 0; k < kCompactRun; ++k) pre[k] = (uint32_t)__builtin_amdgcn_readlane((int)incl, k);
    const uint32_t total = pre[kCompactRun - 1];
    if (total == 0u) continue;  // wave-uniform
    const uint64_t dst0 = base + boff[b0];  // the run's first entry (boff: exclusive prefix)
    for (uint32_t i = lane; i < total; i += 64) {
      uint32_t j = 0, start = 0;  // block of entry i within the run, its first entry
#pragma unroll
      for (int k = 0; k < kCompactRun - 1; ++k)
        if (pre[k] <= i) {
          j = (uint32_t)k + 1u;
          start = pre[k];
        }
      const uint64_t src = (b0 + j) * kScoreBlock + (i - start);
      const uint32_t w = st.cand[src];
      out.cand[dst0 + i] = w & ((1u << kKindShift) - 1u);
      out.kind[dst0 + i] = (uint8_t)(w >> kKindShift);
      out.prob[dst0 + i] = st.prob[src];
      out.qidx[dst0 + i] = st.qidx[src];
    }
  }
}

// first[i] = first entry of query i (entries are grouped by query index, ascending)
__global__ void k_first(const uint32_t* __restrict__ qidx, uint64_t n, uint64_t nq,
                        uint64_t* __restrict__ first) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nq) return;
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if ((uint64_t)qidx[mid] < i) lo = mid + 1; else hi = mid;
  }
  first[i] = lo;
}

// ------------------------------------------------------------------------------------
// candidate replica: position g <- row rowof[g], units transposed
// ------------------------------------------------------------------------------------
template <typename CT>
__device__ __forceinline__ void replicate_units(const ReplicaJob& J, uint64_t g, uint32_t row, int l) {
  // canonical words are zero padded past the value; words past it are written as 0
  const uint32_t* src = reinterpret_cast<const uint32_t*>(reinterpret_cast<const CT*>(J.units) + J.off[row]);
  uint32_t* dst = reinterpret_cast<uint32_t*>(J.runits) + g;
  const int n = l == (int)kMissing ? 0 : l;
  const int upw = 4 / (int)sizeof(CT);
  const int nw = (n + upw - 1) / upw, rw = J.rlmax / upw;
  for (int k = 0; k < rw; ++k) dst[(uint64_t)k * J.stride] = k < nw ? src[k] : 0u;
}

// [Duke 1.2] comparators.Levenshtein.compare for ONE pair, serially, with compactDistance's
// early exit returning the column minimum exactly as Duke does.  Comparator.compare's raw
// similarity (dk_property_similarity): the fused kernels return maxdist + 1 (short values) or
// the full-matrix distance (long values) when the cutoff fires -- the same `low` probability,
// a different raw similarity.  One thread; rows r1 (s1, the column) and r2 (s2).
__global__ void k_lev_exact(const uint32_t* __restrict__ off, const uint16_t* __restrict__ len,
                            const void* __restrict__ units, int width, uint32_t r1, uint32_t r2,
                            double* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int n1 = len[r1], n2 = len[r2];
  if (n1 == (int)kMissing || n2 == (int)kMissing || n1 == 0 || n2 == 0) {
    *out = __builtin_nan("");  // Processor.compare skips the property
    return;
  }
  auto u = [&](uint32_t row, int i) -> uint32_t {
    return width == 1 ? (uint32_t)reinterpret_cast<const uint8_t*>(units)[off[row] + i]
                      : (uint32_t)reinterpret_cast<const uint16_t*>(units)[off[row] + i];
  };
  const int ln = min(n1, n2), maxlen = max(n1, n2);
  if (2 * ln <= maxlen) {  // (double)len / maxlen <= 0.5
    *out = 0.0;
    return;
  }
  bool same = n1 == n2;
  for (int i = 0; i < n1 && same; ++i) same = u(r1, i) == u(r2, i);
  if (same) {
    *out = 1.0;
    return;
  }
  // compactDistance: one column over s1's rows, virtual first row ix2 + 1
  int column[kMaxLongUnits + 1];
  const int maxdist = ln / 2;
  uint32_t ch2 = u(r2, 0);
  column[0] = 1;
  for (int i = 1; i <= n1; ++i) column[i] = min(column[i - 1], i - 1) + (u(r1, i - 1) == ch2 ? 0 : 1);
  int above = 0, result = -1;
  for (int j = 1; j < n2; ++j) {
    ch2 = u(r2, j);
    above = j + 1;
    int smallest = 2 * n1;
    for (int i = 1; i <= n1; ++i) {
      const int v = min(min(above, column[i - 1]), column[i]) + (u(r1, i - 1) == ch2 ? 0 : 1);
      column[i - 1] = above;
      above = v;
      smallest = min(smallest, v);
    }
    column[n1] = above;
    if (smallest > maxdist) {
      result = smallest;
      break;
    }
  }
  if (result < 0) result = above;
  const int dist = min(result, ln);
  *out = 1.0 - ((double)dist / (double)ln);
}

// Per-row perfect hash of a Latin-1 bigram set (DevProp::g16): the first multiplier of
// gram_mult's sequence under which the set's keys land in distinct slots of a 2^lt table
// (one thread per row, its occupancy bitmap in its own LDS words).  Rows of more than
// kGramPerfectMax grams, with the key-0 bigram, or without a seed in kGramSeedTries tries
// get kGramSeedNone (k_score then reads the candidate sets in place).
__global__ __launch_bounds__(256) void k_gram_seed(const uint64_t* __restrict__ grams,
                                                   const uint32_t* __restrict__ goff,
                                                   const uint16_t* __restrict__ gcnt,
                                                   const uint16_t* __restrict__ len, uint64_t row0,
                                                   uint64_t n, uint16_t* __restrict__ seed) {
  __shared__ uint32_t occ[256][17];  // 512 bits per thread (+1 word: rows spread over banks)
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t row = row0 + i;
  const int m = len[row] == kMissing ? 0 : (int)gcnt[row];
  uint16_t out = kGramSeedNone;
  if (m > 0 && m <= kGramPerfectMax) {
    const uint64_t* g = grams + goff[row];
    uint32_t* bits = occ[threadIdx.x];
    bool zero = false;
    for (int k = 0; k < m; ++k) zero = zero || gram_key(g[k]) == 0u;
    // the smallest table first: a probe's LDS bank conflicts grow with the table's words per
    // bank (none at 64 16-bit slots, scripts/micro/lds_probe.hip); m <= kGramPerfectMax = 64
    // (the smaller sizes get a few tries each: a failed try stops at its first collision, but
    // an upsert seeds every row)
    const int lt_hi = m <= 32 ? 8 : 9;
    for (int lt = lt_hi - 2; lt <= lt_hi && out == kGramSeedNone && !zero; ++lt) {
      const int words = 1 << (lt - 5);
      const int tries = lt == lt_hi ? kGramSeedTries : (lt == lt_hi - 1 ? 32 : 16);
      for (int t = 0; t < tries; ++t) {
        const uint32_t mult = gram_mult((uint32_t)t);
        // k_score_gq's slot-0 sentinel is a key in 1..64 whose slot is not 0
        if (((64u * mult) >> (32 - lt)) == 0u) continue;
        for (int w = 0; w < words; ++w) bits[w] = 0u;
        bool ok = true;
        for (int k = 0; k < m && ok; ++k) {
          const uint32_t h = (gram_key(g[k]) * mult) >> (32 - lt);
          const uint32_t b = 1u << (h & 31u);
          ok = (bits[h >> 5] & b) == 0u;
          bits[h >> 5] |= b;
        }
        if (ok) {
          out = (uint16_t)(((lt - kGramLtMin) << 8) | t);
          break;
        }
      }
    }
  }
  seed[row] = out;
}

__global__ __launch_bounds__(256) void k_replicate(const ReplicaJob J, const uint32_t* __restrict__ rowof,
                                                   uint64_t pos0, uint64_t npos) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npos) return;
  const uint64_t g = pos0 + i;
  const uint32_t row = rowof[g];
  const int l = J.len[row];
  J.rlen[g] = (uint16_t)l;
  if (J.rlmax) {
    if (J.width == 1) replicate_units<uint8_t>(J, g, row, l);
    else replicate_units<uint16_t>(J, g, row, l);
  }
  if (J.has_num == 2) {  // (latitude, longitude): the 64 lanes of a score wave read 1 KiB
    J.rnum[2 * g] = J.num[2 * (uint64_t)row];
    J.rnum[2 * g + 1] = J.num[2 * (uint64_t)row + 1];
    J.rnumok[g] = J.numok[row];
  } else if (J.has_num) {
    J.rnum[g] = J.num[row];
    J.rnumok[g] = J.numok[row];
  }
  if (J.has_qgram) {
    J.rgoff[g] = J.goff[row];
    J.rgcnt[g] = J.gcnt[row];
    if (J.rgmax) {  // codes transposed: the 64 lanes of a score wave read row k as 512 B
      const uint64_t* src = J.grams + J.goff[row];
      const int m = l == (int)kMissing ? 0 : (int)J.gcnt[row];
      if (J.g16) {  // four bigram keys per word, the wave's 64 lanes read a word row as 512 B
        uint64_t* dst = reinterpret_cast<uint64_t*>(J.rgrams);
        for (int j = 0; j < J.rgrows; ++j) {
          uint64_t w = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (4 * j + e < m) w |= (uint64_t)gram_key(src[4 * j + e]) << (16 * e);
          dst[(uint64_t)j * J.stride + g] = w;
        }
      } else if (J.rg32) {
        uint32_t* dst = reinterpret_cast<uint32_t*>(J.rgrams);
        for (int k = 0; k < J.rgmax; ++k) dst[(uint64_t)k * J.stride + g] = k < m ? (uint32_t)src[k] : 0u;
      } else {
        uint64_t* dst = reinterpret_cast<uint64_t*>(J.rgrams);
        for (int k = 0; k < J.rgmax; ++k) dst[(uint64_t)k * J.stride + g] = k < m ? src[k] : 0ull;
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// blocking: candidate counting and pair emission
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t lower_bound_u64(const uint64_t* a, uint64_t n, uint64_t v) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ uint64_t upper_bound_u64(const uint64_t* a, uint64_t lo, uint64_t hi,
                                                    uint64_t v) {
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Per query and key function: the candidate range [lo, hi) in sorted table k.  The
// query's own key is looked up by value, so a superseded or deleted query still finds
// its block.  LINKAGE keeps only the other group's sub-range (rows are sorted by
// (key, group, row) and groups are 1 and 2; IncrementalDataSource.java:80-84).
template <int PAD>  // 0: exact counts; else rounded up to PAD slots
__global__ void k_count(const uint32_t* __restrict__ queries, uint64_t nq, const BlockTables T,
                        uint2* __restrict__ ranges, uint64_t* __restrict__ counts,
                        uint64_t* __restrict__ real) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t total = 0;
  if (i < nq) {
    const uint32_t q = queries[i];
    for (int k = 0; k < T.nseg; ++k) {
      const uint64_t key = T.keys[k >> T.seg_shift][q];
      const uint64_t lo = lower_bound_u64(T.skeys[k], T.seg_len[k], key);
      const uint64_t hi = upper_bound_u64(T.skeys[k], lo, T.seg_len[k], key);
      uint64_t a = lo, b = hi;
      if (T.linkage) {
        uint64_t s = lo, e = hi;  // first position with group >= 2
        while (s < e) {
          const uint64_t mid = (s + e) >> 1;
          if (T.sgroup[k][mid] < 2) s = mid + 1; else e = mid;
        }
        if (T.group[q] < 2) a = s; else b = s;
      }
      ranges[(uint64_t)k * nq + i] = make_uint2((uint32_t)a, (uint32_t)b);
      total += b - a;
    }
    counts[i] = PAD ? (total + PAD - 1) / PAD * PAD : total;
  }
  if (!PAD) return;
  uint64_t w = total;
  for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o);
  if (lane_id() == 0 && w) atomicAdd((unsigned long long*)real, (unsigned long long)w);
}

// Symmetric dedup schedule (PairSource::sym): per query and key function its bucket
// [lo, hi), the first position qa of a query row (rows >= r0; the bucket is sorted by row)
// and its own position pq, by binary search; full slot counts padded to 64, owner slot
// counts to opad (64, or 32 for k_score_sym2's half-wave queries).
__device__ __forceinline__ uint64_t lower_bound_u32(const uint32_t* a, uint64_t lo, uint64_t hi,
                                                    uint32_t v) {
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// The symmetric schedule's bucket lookup of large batches (SymIndex, built once per table
// build): per segment k and row, the row's position in the segment (kNoPos: not in it), and per
// replica position its bucket's first position and, at that first position, the bucket's end
// (segment-relative) -- three dependent loads per (query, segment) instead of four binary
// searches (~50 dependent loads, 0.59 ms of a configs[1] step).
__global__ void k_symidx_pos(const BlockTables T, int k, uint64_t nrows, uint32_t* __restrict__ posof,
                             uint32_t* __restrict__ hflag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T.seg_len[k]) return;
  const uint64_t off = T.seg_off[k];
  posof[(uint64_t)k * nrows + T.rowof[off + i]] = (uint32_t)i;
  hflag[off + i] = i == 0 || T.skeys[k][i] != T.skeys[k][i - 1] ? (uint32_t)i : 0u;
}

__global__ void k_symidx_end(const BlockTables T, int k, const uint32_t* __restrict__ bstart,
                             uint32_t* __restrict__ bend) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t n = T.seg_len[k];
  if (i >= n) return;
  const uint64_t off = T.seg_off[k];
  if (i + 1 == n || T.skeys[k][i + 1] != T.skeys[k][i]) bend[off + bstart[off + i]] = (uint32_t)(i + 1);
}

// per position {bucket start, bucket end}: k_count_sym's bucket in one load
__global__ void k_symidx_pair(const BlockTables T, int k, const uint32_t* __restrict__ bstart,
                              const uint32_t* __restrict__ bend, uint2* __restrict__ bse) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T.seg_len[k]) return;
  const uint64_t off = T.seg_off[k];
  const uint32_t b = bstart[off + i];
  bse[off + i] = make_uint2(b, bend[off + b]);
}

__global__ void k_count_sym(const uint32_t* __restrict__ queries, uint64_t nq, const BlockTables T,
                            uint32_t r0, uint4* __restrict__ sranges, uint64_t* __restrict__ counts,
                            uint64_t* __restrict__ ocounts, uint64_t* __restrict__ mcounts,
                            uint64_t* __restrict__ real, uint32_t opad, const SymIndex X) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t total = 0, own = 0, mir = 0;
  if (i < nq) {
    const uint32_t q = queries[i];
    for (int k = 0; k < T.nseg; ++k) {
      const uint32_t* rows = T.rowof + T.seg_off[k];
      const uint32_t px = X.posof ? X.posof[(uint64_t)k * X.nrows + q] : kNoPos;
      uint64_t lo, hi, qa, p;
      bool self = false;  // rows[p] == q is known (posof)
      if (px != kNoPos) {  // the query's own entry: its bucket from the index
        const uint2 be = X.bse[T.seg_off[k] + px];
        lo = be.x;
        hi = be.y;
        // (r0 == 0: every row of the bucket is a batch row -- no load)
        qa = r0 == 0 || rows[lo] >= r0 ? lo : lower_bound_u32(rows, lo, hi, r0);
        p = px;
        self = true;
      } else {
        const uint64_t key = T.keys[k >> T.seg_shift][q];
        lo = lower_bound_u64(T.skeys[k], T.seg_len[k], key);
        hi = upper_bound_u64(T.skeys[k], lo, T.seg_len[k], key);
        qa = lower_bound_u32(rows, lo, hi, r0);
        p = lower_bound_u32(rows, qa, hi, q);
      }
      // a superseded base entry is no candidate, so its query is not "in" the segment
      // either: it owns its whole bucket and expects no mirrored results
      const bool in_t = p < hi && (self || rows[p] == q) && T.rident[T.seg_off[k] + p] != kDeadIdent;
      const uint32_t qa_eff = in_t ? (uint32_t)qa : (uint32_t)hi;
      sranges[(uint64_t)k * nq + i] =
          make_uint4((uint32_t)lo, (uint32_t)hi, qa_eff, in_t ? (uint32_t)p : kNoPos);
      total += hi - lo;
      own += (qa_eff - lo) + (in_t ? hi - p - 1 : 0);
      mir += in_t ? p - qa : 0;
    }
    counts[i] = (total + 63) & ~(uint64_t)63;
    ocounts[i] = (own + opad - 1) / opad * opad;
    mcounts[i] = mir;
  }
  uint64_t w = total;
  for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o);
  if (lane_id() == 0 && w) atomicAdd((unsigned long long*)real, (unsigned long long)w);
}

// obase[k][qi] = owner slot of bucket position qa for (k, qi): the query's owner slots
// start at oqoff[qi] and hold its owned candidates key function by key function
// and mbase[k][qi] = mirror slot of bucket position qa (the query's mirror runs [qa, pq)
// start at mqoff[qi], key function by key function)
__global__ void k_obase(const uint4* __restrict__ sranges, const uint64_t* __restrict__ oqoff,
                        const uint64_t* __restrict__ mqoff, uint64_t nq, int nseg,
                        uint64_t* __restrict__ obase, uint64_t* __restrict__ mbase) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  uint64_t cum = oqoff[i], mcum = mqoff[i];
  for (int k = 0; k < nseg; ++k) {
    const uint4 r = sranges[(uint64_t)k * nq + i];
    const uint64_t nlow = r.z - r.x;
    const bool in_t = r.w != kNoPos;
    obase[(uint64_t)k * nq + i] = cum + nlow;
    mbase[(uint64_t)k * nq + i] = mcum;
    cum += nlow + (in_t ? (uint64_t)(r.y - r.w - 1) : 0);
    mcum += in_t ? (uint64_t)(r.w - r.z) : 0;
  }
}

__global__ void k_gather_u64(const uint64_t* __restrict__ src, const uint64_t* __restrict__ idx,
                             uint64_t n, uint64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = src[idx[i]];
}

__global__ void k_iota_u32(uint32_t* __restrict__ out, uint64_t n, uint32_t start) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = start + (uint32_t)i;
}

// wq[w] = qi for every wave w of query qi's slots (one thread per query, its waves in a
// short loop: a query spans a few waves on average)
__global__ void k_wavemap(const uint64_t* __restrict__ qoff, uint64_t nq, uint32_t* __restrict__ wq, int shift) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  for (uint64_t w = qoff[i] >> shift, e = qoff[i + 1] >> shift; w < e; ++w) wq[w] = (uint32_t)i;
}

// k_score_sym2's owner slot layout: waves hold at most two queries, each from any lane on.
// One workgroup per tile of kPackTile queries (tiles start at a wave and end at one): the
// tile's queries ordered by `klen` (the query's length on the schema's longest Levenshtein
// property, when given: a wave's DP row bucket follows its longer query, so neighbours of
// similar length waste fewer rows), then placed greedily by one thread -- a query starts on
// the next free lane unless a query already started inside that wave (the wave's rest is
// then padding, at the end of the previous query's slots).  own[i] (the query's owned slots)
// becomes its slots with trailing padding, loc[i] its first slot within the tile, ttot[t]
// the tile's slots.  Padding is ~2 % of the slots, against ~7 % with every query padded to
// a half-wave.

__global__ __launch_bounds__(kPackTile) void k_opack(uint64_t* __restrict__ own, uint64_t nq,
                                                     const uint32_t* __restrict__ queries,
                                                     const uint16_t* __restrict__ klen,
                                                     uint32_t* __restrict__ loc, uint64_t* __restrict__ ttot) {
  __shared__ uint32_t sk[kPackTile];  // key << 8 | local index, sorted
  __shared__ uint64_t so[kPackTile];  // owned slots -> slots with padding
  __shared__ uint32_t sl[kPackTile];  // first slot within the tile
  const uint32_t j = threadIdx.x;
  const uint64_t q0 = (uint64_t)blockIdx.x * kPackTile;
  const uint32_t n = (uint32_t)min<uint64_t>(kPackTile, nq - q0);
  uint32_t key = 0xFFFFu;  // past the tile's queries: last
  if (j < n) {
    key = 0u;
    if (klen) {
      const uint32_t l = klen[queries[q0 + j]];
      key = l == kMissing ? 0u : min(l, 0xFFFEu);
    }
    so[j] = own[q0 + j];
  }
  sk[j] = (key << 8) | j;
  __syncthreads();
  for (uint32_t k = 2; k <= kPackTile; k <<= 1) {  // bitonic sort, ascending
    for (uint32_t h = k >> 1; h > 0; h >>= 1) {
      const uint32_t x = j ^ h;
      if (x > j) {
        const uint32_t a = sk[j], b = sk[x];
        if (((j & k) == 0) == (a > b)) {
          sk[j] = b;
          sk[x] = a;
        }
      }
      __syncthreads();
    }
  }
  if (j == 0) {
    uint64_t cur = 0;       // next free slot of the tile
    bool started = false;   // a query started inside the current wave (not at lane 0)
    uint32_t last = kPackTile;
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t jj = sk[i] & 0xFFu;
      const uint64_t L = so[jj];
      uint32_t p = (uint32_t)(cur & 63u);
      if (L > 0 && p > 0 && started) {  // a third query would share the wave: pad it
        so[last] += 64u - p;
        cur += 64u - p;
        p = 0;
        started = false;
      }
      sl[jj] = (uint32_t)cur;
      if (L == 0) continue;
      started = p > 0;
      if (p + L >= 64) started = false;  // the query reaches the next wave: it is that wave's first
      cur += L;
      last = jj;
    }
    const uint32_t p = (uint32_t)(cur & 63u);
    if (p && last < kPackTile) {
      so[last] += 64u - p;
      cur += 64u - p;
    }
    ttot[blockIdx.x] = cur;
  }
  __syncthreads();
  if (j < n) {
    own[q0 + j] = so[j];
    loc[q0 + j] = sl[j];
  }
}

// oqoff[i] = the tile's first slot + the query's first slot within it; oqoff[nq] = the total
__global__ void k_opack_fin(const uint32_t* __restrict__ loc, const uint64_t* __restrict__ tbase,
                            uint64_t nq, uint64_t* __restrict__ oqoff) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nq) oqoff[i] = tbase[i / kPackTile] + loc[i];
  if (i == 0) oqoff[nq] = tbase[(nq + kPackTile - 1) / kPackTile];
}

// wave w of k_score_sym2's owner slots -> {query of its first slot, query of its last slot}
// (one thread per query over the waves whose first / last slot lies in its range
// [qoff[i], qoff[i] + occ[i]))
__global__ void k_wavemap2(const uint64_t* __restrict__ qoff, const uint64_t* __restrict__ occ, uint64_t nq,
                           uint2* __restrict__ wq2) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  const uint64_t a = qoff[i], e = a + occ[i];
  for (uint64_t w = (a + 63) >> 6, we = (e + 63) >> 6; w < we; ++w) wq2[w].x = (uint32_t)i;
  for (uint64_t w = a >> 6, we = e >> 6; w < we; ++w) wq2[w].y = (uint32_t)i;
}

// replica-ordered identity and keys (the score kernel's candidate filters read them
// coalesced, 64 consecutive positions per wave)
__global__ __launch_bounds__(256) void k_replicate_rows(const uint32_t* __restrict__ rowof, uint64_t pos0,
                                                        uint64_t npos, const uint64_t* __restrict__ ident,
                                                        uint64_t* __restrict__ rident, const BlockTables T,
                                                        RowKeys rk) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npos) return;
  const uint64_t g = pos0 + i;
  const uint32_t row = rowof[g];
  rident[g] = ident[row];
  for (int j = 0; j < T.nkeys - 1; ++j) rk.p[j][g] = T.keys[j][row];
}

// A row superseded after the base was sorted (delete-by-ID of a re-posted ID): find its
// entry in key function k's base segment -- its key's bucket, its group's sub-range
// (LINKAGE), then the row, the bucket being sorted by row within a group -- and retire it.
// One thread per (row, key function).
__global__ void k_mark_dead(const BlockTables T, const uint32_t* __restrict__ rows, uint64_t n,
                            uint64_t* __restrict__ rident) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * (uint64_t)T.nkeys) return;
  const uint32_t row = rows[i / T.nkeys];
  const int k = (int)(i % T.nkeys);
  const int sg = k << T.seg_shift;  // the key function's base segment
  const uint64_t key = T.keys[k][row];
  uint64_t lo = lower_bound_u64(T.skeys[sg], T.seg_len[sg], key);
  uint64_t hi = upper_bound_u64(T.skeys[sg], lo, T.seg_len[sg], key);
  if (T.linkage) {
    const uint8_t g = T.group[row];
    uint64_t s = lo, e = hi;  // first position with group >= 2
    while (s < e) {
      const uint64_t mid = (s + e) >> 1;
      if (T.sgroup[sg][mid] < 2) s = mid + 1; else e = mid;
    }
    if (g < 2) hi = s; else lo = s;
  }
  const uint32_t* rs = T.rowof + T.seg_off[sg];
  const uint64_t p = lower_bound_u32(rs, lo, hi, row);
  if (p < hi && rs[p] == row) rident[T.seg_off[sg] + p] = kDeadIdent;
}

// ------------------------------------------------------------------------------------
// Lucene-compatible candidate source (DK_CAND_LUCENE): IncrementalLuceneDatabase.
// findCandidateMatches + EstimateResultTracker.doQuery over a postings table
// ------------------------------------------------------------------------------------
// The postings and maxDoc of the collection statistics: rows with a bit of `mask` set --
// kAlive (merged: superseded versions gone) or kIndexed (unmerged: superseded versions still
// counted, as Lucene counts deleted documents until their segment is merged).
__global__ void k_lucene_prep(const uint64_t* __restrict__ key, uint64_t npost,
                              const uint8_t* __restrict__ flags, uint64_t nrows, uint8_t mask,
                              uint64_t* __restrict__ out_key, uint64_t* __restrict__ counts) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t kept = 0, docs = 0;
  if (i < npost) {
    const uint64_t k = key[i];
    const bool in = (flags[(uint32_t)k] & mask) != 0;
    out_key[i] = in ? k : ~0ull;
    kept = in;
  }
  if (i < nrows) docs = (flags[i] & mask) != 0;
  for (int o = 32; o > 0; o >>= 1) {
    kept += __shfl_xor(kept, o);
    docs += __shfl_xor(docs, o);
  }
  if (lane_id() == 0) {
    if (kept) atomicAdd((unsigned long long*)&counts[0], (unsigned long long)kept);
    if (docs) atomicAdd((unsigned long long*)&counts[1], (unsigned long long)docs);
  }
}

__device__ __forceinline__ uint64_t lower_bound_key(const uint64_t* a, uint64_t lo, uint64_t hi,
                                                    uint64_t v) {
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// SmallFloat.byte315ToFloat: the decoded length norm
__device__ __forceinline__ float decode_norm(uint32_t b) {
  return b == 0 ? 0.0f : __uint_as_float((b << 21) + ((63u - 15u) << 24));
}

// One workgroup per query.  The query's clauses (its lookup values' tokens, escaped) are
// TermQuerys on the postings; DefaultSimilarity [Lucene 4.x, recalled]:
//   idf = (float)(ln(maxDoc / (double)(df + 1)) + 1), queryNorm = (float)(1 / sqrt(sum idf^2)),
//   clause weight = (idf * queryNorm) * idf, term score = ((float)sqrt(tf) * weight) * norm,
//   document score = (float)(sum over matching clauses in clause order, in double) * coord,
//   coord = overlap / (float)clauses.
// Rows are visited in tiles of kLuceneTile (only tiles holding a posting): the clauses add
// into a per-tile LDS accumulator one after another (a barrier between clauses keeps the sum
// order), then rows that reach min_relevance and beat the current max_hits-th hit are merged
// into the hit list (score descending, row ascending: Lucene's doc-id tie break).
__global__ __launch_bounds__(256) void k_lucene_topk(const LuceneParams L) {
  __shared__ double acc[kLuceneTile];
  __shared__ uint16_t cnt[kLuceneTile];
  __shared__ uint64_t cur[kLuceneMaxClauses], endp[kLuceneMaxClauses], hip_[kLuceneMaxClauses];
  __shared__ uint32_t cft[kLuceneMaxClauses];
  __shared__ float w[kLuceneMaxClauses];
  __shared__ float coordf[kLuceneMaxClauses + 1];
  __shared__ float topS[kLuceneMaxHits];
  __shared__ uint32_t topR[kLuceneMaxHits];
  __shared__ float cbS[kLuceneTile];
  __shared__ uint32_t cbR[kLuceneTile];
  __shared__ int ntop, ncb;
  __shared__ uint32_t tile0;
  __shared__ float qnorm;
  const uint64_t qi = blockIdx.x;
  const int tid = threadIdx.x;
  const uint32_t q = L.queries[qi];
  const uint64_t c0 = L.qoff[q];
  const int nc = (int)(L.qoff[q + 1] - c0);  // <= kLuceneMaxClauses (checked by dk_upsert)
  const int K = L.max_hits;
  const uint8_t qgroup = L.group[q];
  if (tid < nc) {
    const uint32_t ft = L.qterm[c0 + tid];
    const uint64_t lo = lower_bound_key(L.skey, 0, L.npost, (uint64_t)ft << 32);
    const uint64_t hi = lower_bound_key(L.skey, lo, L.npost, (uint64_t)(ft + 1) << 32);
    cft[tid] = ft;
    cur[tid] = lo;
    hip_[tid] = hi;
    w[tid] = (float)(log((double)L.max_doc / (double)(hi - lo + 1)) + 1.0);  // idf
  }
  for (int k = tid; k <= nc; k += 256) coordf[k] = nc ? (float)k / (float)nc : 0.0f;
  if (tid == 0) {
    ntop = 0;
    float ssw = 0.0f;  // BooleanWeight.getValueForNormalization: float, clause order
    for (int c = 0; c < nc; ++c) ssw += w[c] * w[c];
    float qn = (float)(1.0 / sqrt((double)ssw));
    if (!(qn == qn) || qn == __builtin_inff()) qn = 1.0f;
    qnorm = qn;
  }
  __syncthreads();
  if (tid < nc) w[tid] = (w[tid] * qnorm) * w[tid];
  __syncthreads();
  for (;;) {
    if (tid == 0) {
      uint32_t m = 0xFFFFFFFFu;
      for (int c = 0; c < nc; ++c)
        if (cur[c] < hip_[c]) m = min(m, (uint32_t)L.skey[cur[c]]);
      tile0 = m == 0xFFFFFFFFu ? m : m / kLuceneTile * kLuceneTile;
      ncb = 0;
    }
    __syncthreads();
    const uint32_t t0 = tile0;
    if (t0 == 0xFFFFFFFFu) break;
    for (int j = tid; j < kLuceneTile; j += 256) {
      acc[j] = 0.0;
      cnt[j] = 0;
    }
    if (tid < nc) {  // the clause's postings inside this tile
      const uint64_t end = ((uint64_t)cft[tid] << 32) | ((uint64_t)t0 + kLuceneTile);
      endp[tid] = lower_bound_key(L.skey, cur[tid], hip_[tid], end);
    }
    __syncthreads();
    for (int c = 0; c < nc; ++c) {
      const int f = (int)(cft[c] >> 24);
      const float wc = w[c];
      for (uint64_t e = cur[c] + tid; e < endp[c]; e += 256) {
        const uint32_t row = (uint32_t)L.skey[e];
        const float tf = (float)sqrt((double)L.stf[e]);
        const float sc = (tf * wc) * decode_norm(L.norm[(uint64_t)row * L.nfields + f]);
        acc[row - t0] += (double)sc;
        cnt[row - t0] += 1;
      }
      __syncthreads();
    }
    if (tid < nc) cur[tid] = endp[tid];
    // candidates of the tile: eligible rows that reach min_relevance and the hit list
    const int full = ntop == K;
    const float worst = full ? topS[K - 1] : 0.0f;
    for (int j = tid; j < kLuceneTile; j += 256) {
      const int k = cnt[j];
      if (!k) continue;
      const uint32_t row = t0 + (uint32_t)j;
      if ((L.flags[row] & (kAlive | kDeleted)) != kAlive) continue;  // liveDocs; dukeDeleted
      if (L.linkage && L.group[row] == qgroup) continue;
      const float score = (float)(acc[j] * (double)coordf[k]);
      if (!(score >= L.min_relevance)) continue;
      if (full && !(score > worst)) continue;  // later rows lose ties (doc-id order)
      const int at = atomicAdd(&ncb, 1);
      cbS[at] = score;
      cbR[at] = row;
    }
    __syncthreads();
    if (tid == 0) {  // insertion into the sorted hit list
      int n = ntop;
      for (int i = 0; i < ncb; ++i) {
        const float sc = cbS[i];
        const uint32_t r = cbR[i];
        int pos = n;
        while (pos > 0 && (topS[pos - 1] < sc || (topS[pos - 1] == sc && topR[pos - 1] > r))) --pos;
        if (pos >= K) continue;
        for (int m = min(n, K - 1); m > pos; --m) {
          topS[m] = topS[m - 1];
          topR[m] = topR[m - 1];
        }
        topS[pos] = sc;
        topR[pos] = r;
        if (n < K) ++n;
      }
      ntop = n;
    }
    __syncthreads();
  }
  const int n = ntop;
  if (tid < n) L.hits[qi * (uint64_t)K + tid] = topR[tid];
  if (tid == 0) {
    L.ranges[qi] = make_uint2((uint32_t)(qi * (uint64_t)K), (uint32_t)(qi * (uint64_t)K + n));
    L.counts[qi] = ((uint64_t)n + 63) & ~(uint64_t)63;
    if (L.exact) L.exact[qi] = (uint64_t)n;
    if (L.real && n) atomicAdd((unsigned long long*)L.real, (unsigned long long)n);
  }
}

// ------------------------------------------------------------------------------------
// small utility kernels
// ------------------------------------------------------------------------------------
__global__ void k_widen_u8(const uint8_t* __restrict__ src, uint16_t* __restrict__ dst, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

__global__ void k_clear_flag(uint8_t* flags, const uint32_t* rows, uint64_t n, uint8_t bit) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flags[rows[i]] &= (uint8_t)~bit;
}

__global__ void k_gather_keys(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ rows,
                              uint64_t* __restrict__ out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = keys[rows[i]];
}

__global__ void k_gather_u8(const uint8_t* __restrict__ src, const uint32_t* __restrict__ rows,
                            uint8_t* __restrict__ out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = src[rows[i]];
}

// usable = alive and not deleted; LINKAGE selects one group per pass (want_group > 0)
__global__ void k_select_rows(const uint8_t* __restrict__ flags, const uint8_t* __restrict__ group,
                              uint64_t row0, uint64_t n, int want_group, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t r = row0 + i;
  bool ok = (flags[r] & (kAlive | kDeleted)) == kAlive;
  if (want_group > 0) ok = ok && ((int)group[r] == want_group || (want_group == 2 && group[r] > 2));
  out[i] = ok ? 1u : 0u;
}

__global__ void k_scatter_rows(const uint32_t* __restrict__ flag, const uint32_t* __restrict__ pos,
                               uint64_t row0, uint64_t n, uint32_t base, uint32_t* __restrict__ rows) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && flag[i]) rows[base + pos[i]] = (uint32_t)(row0 + i);
}

__global__ void k_fill_u32(uint32_t* p, uint32_t v, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void k_iota_u32(uint32_t* p, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (uint32_t)i;
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
static inline unsigned grid1d(uint64_t n, unsigned b = 256) {
  return (unsigned)((n + b - 1) / b);
}

#define DK_LAUNCH_GUARD(n) \
  if ((n) == 0) return hipSuccess;

hipError_t launch_widen_u8(const uint8_t* src, uint16_t* dst, uint64_t n, hipStream_t s) {
  DK_LAUNCH_GUARD(n);
  k_widen_u8<<<grid1d(n), 256, 0, s>>>(src, dst, n);
  return hipGetLastError();
}

hipError_t launch_clear_flag(uint8_t* flags, const uint32_t* rows, uint64_t n, uint8_t bit,
                             hipStream_t s) {
  DK_LAUNCH_GUARD(n);
  k_clear_flag<<<grid1d(n), 256, 0, s>>>(flags, rows, n, bit);
  return hipGetLastError();
}

hipError_t launch_gather_keys(const uint64_t* keys, const uint32_t* rows, uint64_t* out,
                              uint64_t n, hipStream_t s) {
  DK_LAUNCH_GUARD(n);
  k_gather_keys<<<grid1d(n), 256, 0, s>>>(keys, rows, out, n);
  return hipGetLastError();
}

hipError_t launch_gather_u8(const uint8_t* src, const uint32_t* rows, uint8_t* out, uint64_t n,
                            hipStream_t s) {
  DK_LAUNCH_GUARD(n);
  k_gather_u8<<<grid1d(n), 256, 0, s>>>(src, rows, out, n);
  return hipGetLastError();
}

hipError_t launch_select_rows(const uint8_t* flags, const uint8_t* group, uint64_t row0,
                              uint64_t nrows, int want_group, uint32_t* flag_out, hipStream_t s) {
  DK_LAUNCH_GUARD(nrows);
  k_select_rows<<<grid1d(nrows), 256, 0, s>>>(flags, group, row0, nrows, want_group, flag_out);
  return hipGetLastError();
}

hipError_t launch_scatter_rows(const uint32_t* flag, const uint32_t* pos, uint64_t row0,
                               uint64_t nrows, uint32_t base, uint32_t* rows_out, hipStream_t s) {
  DK_LAUNCH_GUARD(nrows);
  k_scatter_rows<<<grid1d(nrows), 256, 0, s>>>(flag, pos, row0, nrows, base, rows_out);
  return hipGetLastError();
}

hipError_t launch_lev_exact(const uint32_t* off, const uint16_t* len, const void* units, int width,
                            uint32_t r1, uint32_t r2, double* out, hipStream_t s) {
  k_lev_exact<<<1, 64, 0, s>>>(off, len, units, width, r1, r2, out);
  return hipGetLastError();
}

hipError_t launch_gram_seed(const uint64_t* grams, const uint32_t* goff, const uint16_t* gcnt,
                            const uint16_t* len, uint64_t row0, uint64_t n, uint16_t* seed,
                            hipStream_t s) {
  DK_LAUNCH_GUARD(n);
  k_gram_seed<<<grid1d(n), 256, 0, s>>>(grams, goff, gcnt, len, row0, n, seed);
  return hipGetLastError();
}

hipError_t launch_replicate(const ReplicaJob& J, const uint32_t* rowof, uint64_t pos0, uint64_t npos,
                            hipStream_t s) {
  DK_LAUNCH_GUARD(npos);
  k_replicate<<<grid1d(npos), 256, 0, s>>>(J, rowof, pos0, npos);
  return hipGetLastError();
}

hipError_t launch_mark_dead(const BlockTables& T, const uint32_t* rows, uint64_t n, uint64_t* rident,
                            hipStream_t s) {
  DK_LAUNCH_GUARD(n);
  k_mark_dead<<<grid1d(n * (uint64_t)T.nkeys), 256, 0, s>>>(T, rows, n, rident);
  return hipGetLastError();
}

hipError_t launch_count(const uint32_t* queries, uint64_t nq, const BlockTables& T, uint2* ranges,
                        uint64_t* counts, uint64_t* real, int pad, hipStream_t s) {
  DK_LAUNCH_GUARD(nq);
  if (pad == kScoreBlock) k_count<kScoreBlock><<<grid1d(nq), 256, 0, s>>>(queries, nq, T, ranges, counts, real);
  else if (pad == 64) k_count<64><<<grid1d(nq), 256, 0, s>>>(queries, nq, T, ranges, counts, real);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_count_exact(const uint32_t* queries, uint64_t nq, const BlockTables& T,
                              uint2* ranges, uint64_t* counts, hipStream_t s) {
  DK_LAUNCH_GUARD(nq);
  k_count<0><<<grid1d(nq), 256, 0, s>>>(queries, nq, T, ranges, counts, nullptr);
  return hipGetLastError();
}

hipError_t launch_wavemap(const uint64_t* qoff, uint64_t nq, uint32_t* wq, hipStream_t s, int shift) {
  DK_LAUNCH_GUARD(nq);
  k_wavemap<<<grid1d(nq), 256, 0, s>>>(qoff, nq, wq, shift);
  return hipGetLastError();
}

uint64_t opack_tiles(uint64_t nq) { return (nq + kPackTile - 1) / kPackTile; }

hipError_t launch_opack(uint64_t* own, uint64_t nq, const uint32_t* queries, const uint16_t* klen,
                        uint32_t* loc, uint64_t* ttot, hipStream_t s) {
  DK_LAUNCH_GUARD(nq);
  k_opack<<<(unsigned)opack_tiles(nq), kPackTile, 0, s>>>(own, nq, queries, klen, loc, ttot);
  return hipGetLastError();
}

hipError_t launch_opack_fin(const uint32_t* loc, const uint64_t* tbase, uint64_t nq, uint64_t* oqoff,
                            hipStream_t s) {
  DK_LAUNCH_GUARD(nq);
  k_opack_fin<<<grid1d(nq), 256, 0, s>>>(loc, tbase, nq, oqoff);
  return hipGetLastError();
}

hipError_t launch_wavemap2(const uint64_t* qoff, const uint64_t* occ, uint64_t nq, uint2* wq2, hipStream_t s) {
  DK_LAUNCH_GUARD(nq);
  k_wavemap2<<<grid1d(nq), 256, 0, s>>>(qoff, occ, nq, wq2);
  return hipGetLastError();
}

hipError_t launch_replicate_rows(const uint32_t* rowof, uint64_t pos0, uint64_t npos,
                                 const uint64_t* ident, uint64_t* rident, const BlockTables& T,
                                 uint64_t* const* rkeys, hipStream_t s) {
  DK_LAUNCH_GUARD(npos);
  RowKeys rk{};
  for (int j = 0; j < T.nkeys - 1; ++j) rk.p[j] = rkeys[j];
  k_replicate_rows<<<grid1d(npos), 256, 0, s>>>(rowof, pos0, npos, ident, rident, T, rk);
  return hipGetLastError();
}

hipError_t launch_count_sym(const uint32_t* queries, uint64_t nq, const BlockTables& T, uint32_t r0,
                            uint4* sranges, uint64_t* counts, uint64_t* ocounts, uint64_t* mcounts,
                            uint64_t* real, uint32_t opad, const SymIndex& X, hipStream_t s) {
  DK_LAUNCH_GUARD(nq);
  k_count_sym<<<grid1d(nq), 256, 0, s>>>(queries, nq, T, r0, sranges, counts, ocounts, mcounts, real, opad, X);
  return hipGetLastError();
}

hipError_t launch_symidx(const BlockTables& T, uint64_t nrows, uint32_t* posof, uint32_t* hflag,
                         uint32_t* bstart, uint32_t* bend, uint2* bse, void* tmp, size_t tmp_bytes, hipStream_t s) {
  for (int k = 0; k < T.nseg; ++k) {
    const uint64_t n = T.seg_len[k];
    if (!n) continue;
    k_symidx_pos<<<grid1d(n), 256, 0, s>>>(T, k, nrows, posof, hflag);
    size_t b = tmp_bytes;
    hipError_t e = rocprim::inclusive_scan(tmp, b, hflag + T.seg_off[k], bstart + T.seg_off[k], (size_t)n,
                                           rocprim::maximum<uint32_t>(), s);
    if (e != hipSuccess) return e;
    k_symidx_end<<<grid1d(n), 256, 0, s>>>(T, k, bstart, bend);
    k_symidx_pair<<<grid1d(n), 256, 0, s>>>(T, k, bstart, bend, bse);
  }
  return hipGetLastError();
}

hipError_t symidx_scan_bytes(uint64_t n, size_t* bytes) {
  return rocprim::inclusive_scan(nullptr, *bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n,
                                 rocprim::maximum<uint32_t>(), (hipStream_t)0);
}

hipError_t launch_obase(const uint4* sranges, const uint64_t* oqoff, const uint64_t* mqoff,
                        uint64_t nq, int nseg, uint64_t* obase, uint64_t* mbase, hipStream_t s) {
  DK_LAUNCH_GUARD(nq);
  k_obase<<<grid1d(nq), 256, 0, s>>>(sranges, oqoff, mqoff, nq, nseg, obase, mbase);
  return hipGetLastError();
}

hipError_t launch_sym_emit(const EmitSource& src, uint64_t q0, uint64_t nqc, bool write, uint64_t base,
                           const MatchList& out, uint64_t* first, hipStream_t s) {
  DK_LAUNCH_GUARD(nqc);
  const unsigned grid = grid1d(nqc, kScoreBlock / 64);
  if (write) k_sym_emit<true><<<grid, kScoreBlock, 0, s>>>(src, q0, nqc, base, out, first);
  else k_sym_count<<<grid1d(nqc * kCountLanes), 256, 0, s>>>(src, q0, nqc);
  return hipGetLastError();
}

hipError_t launch_gather_u64(const uint64_t* src, const uint64_t* idx, uint64_t n, uint64_t* out,
                             hipStream_t s) {
  DK_LAUNCH_GUARD(n);
  k_gather_u64<<<grid1d(n), 256, 0, s>>>(src, idx, n, out);
  return hipGetLastError();
}

hipError_t launch_iota_u32(uint32_t* out, uint64_t n, uint32_t start, hipStream_t s) {
  DK_LAUNCH_GUARD(n);
  k_iota_u32<<<grid1d(n), 256, 0, s>>>(out, n, start);
  return hipGetLastError();
}

// DK_GRAM_VARIANT=0: always the kernels with the gram-set code (A/B)
static bool gram_variant_off() {
  static const bool off = [] {
    const char* e = getenv("DK_GRAM_VARIANT");
    return e && e[0] == '0';
  }();
  return off;
}

hipError_t launch_score(const ScoreParams& P, const PairSource& src, uint64_t slot0,
                        uint64_t nslots, const StageOut& out, hipStream_t s) {
  DK_LAUNCH_GUARD(nslots);
  const unsigned grid = grid1d(nslots, kScoreBlock);
  // kernel variant by the longest Levenshtein query value (rows of the lane-per-pair DP
  // column) and the longest value of the long-value DP (WeightedLevenshtein, or a
  // Levenshtein value over 64 units): both bound the VGPRs of the fused kernel
#define DK_SHORT(RM)                                                               \
  do {                                                                             \
    if (P.has_grams || gram_variant_off()) {                                                \
      if (src.sym) k_score<RM, true, true><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out); \
      else k_score<RM, false, true><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out);        \
    } else {                                                                                  \
      if (src.sym) k_score<RM, true, false><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out); \
      else k_score<RM, false, false><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out);        \
    }                                                                                         \
  } while (0)
#define DK_LONG(RM, L) k_score_long<RM, L><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out)
  if (src.sym && P.long_rows > 0) return hipErrorInvalidValue;  // the host never schedules it
  if (P.has_geo) {
    if (src.sym) return hipErrorInvalidValue;  // the host never schedules it (sym_schema_ok)
    if (!P.has_dp) k_score_geo<false><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out);
    else if (P.long_rows > 0) k_score_long_geo<<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out);
    else k_score_geo<true><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out);
  } else if (!P.has_dp) {
    if (src.sym) k_score_nodp<true><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out);
    else k_score_nodp<false><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out);
  } else if (P.long_rows > 0) {
    const bool lev64 = P.lev_rows > 16;
    if (P.long_rows <= 64) { if (lev64) DK_LONG(64, 4); else DK_LONG(16, 4); }
    else if (P.long_rows <= 128) { if (lev64) DK_LONG(64, 8); else DK_LONG(16, 8); }
    else { if (lev64) DK_LONG(64, 16); else DK_LONG(16, 16); }
  } else if (src.sym && src.two) {
    if (P.lev_rows <= 16) k_score_sym2<16><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out);
    else if (P.lev_rows <= 32) k_score_sym2<32><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out);
    else if (P.lev_rows <= 40) k_score_sym2<40><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out);
    else if (P.lev_rows <= 48) k_score_sym2<48><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out);
    else k_score_sym2<64><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, out);
  } else if (P.lev_rows <= 16) DK_SHORT(16);
  else if (P.lev_rows <= 32) DK_SHORT(32);
  else if (P.lev_rows <= 40) DK_SHORT(40);
  else if (P.lev_rows <= 48) DK_SHORT(48);
  else DK_SHORT(64);
#undef DK_SHORT
#undef DK_LONG
  return hipGetLastError();
}


hipError_t launch_reduce_blocks(const StageOut& st, uint64_t nblocks, hipStream_t s) {
  DK_LAUNCH_GUARD(nblocks);
  const unsigned g = (unsigned)std::min<uint64_t>((nblocks + 1023) / 1024, 512);
  k_reduce_blocks<<<g, 256, 0, s>>>(st, nblocks);
  return hipGetLastError();
}

hipError_t launch_compact(const StageOut& st, const uint64_t* boff, uint64_t nblocks,
                          uint64_t base, const MatchList& out, hipStream_t s) {
  DK_LAUNCH_GUARD(nblocks);
  const uint64_t runs = (nblocks + kCompactRun - 1) / kCompactRun;   // one per wave
  const unsigned grid = (unsigned)std::min<uint64_t>((runs + 3) / 4, 8192);
  k_compact<<<grid, 256, 0, s>>>(st, boff, nblocks, base, out);
  return hipGetLastError();
}

hipError_t launch_first(const uint32_t* qidx, uint64_t n, uint64_t nq, uint64_t* first,
                        hipStream_t s) {
  k_first<<<grid1d(nq + 1), 256, 0, s>>>(qidx, n, nq, first);
  return hipGetLastError();
}

hipError_t launch_lucene_prep(const uint64_t* key, uint64_t npost, const uint8_t* flags, uint64_t nrows,
                              uint8_t mask, uint64_t* out_key, uint64_t* counts, hipStream_t s) {
  const uint64_t n = std::max(npost, nrows);
  DK_LAUNCH_GUARD(n);
  k_lucene_prep<<<grid1d(n), 256, 0, s>>>(key, npost, flags, nrows, mask, out_key, counts);
  return hipGetLastError();
}

// IndexWriter.forceMerge: superseded versions leave the statistics
__global__ void k_lucene_merge(uint8_t* flags, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && !(flags[i] & kAlive)) flags[i] &= (uint8_t)~kIndexed;
}

hipError_t launch_lucene_merge(uint8_t* flags, uint64_t nrows, hipStream_t s) {
  if (!nrows) return hipSuccess;
  DK_LAUNCH_GUARD(nrows);
  k_lucene_merge<<<grid1d(nrows), 256, 0, s>>>(flags, nrows);
  return hipGetLastError();
}

hipError_t launch_lucene_topk(const LuceneParams& L, hipStream_t s) {
  DK_LAUNCH_GUARD(L.nq);
  if (L.max_hits < 1 || L.max_hits > kLuceneMaxHits || L.nq > 0x7FFFFFFFull) return hipErrorInvalidValue;
  k_lucene_topk<<<(unsigned)L.nq, 256, 0, s>>>(L);
  return hipGetLastError();
}

hipError_t launch_fill_u32(uint32_t* p, uint32_t v, uint64_t n, hipStream_t s) {
  DK_LAUNCH_GUARD(n);
  k_fill_u32<<<grid1d(n), 256, 0, s>>>(p, v, n);
  return hipGetLastError();
}

hipError_t launch_iota_u32(uint32_t* p, uint64_t n, hipStream_t s) {
  DK_LAUNCH_GUARD(n);
  k_iota_u32<<<grid1d(n), 256, 0, s>>>(p, n);
  return hipGetLastError();
}

hipError_t sort_pairs_u64_u32(void* tmp, size_t& tmp_bytes, const uint64_t* kin, uint64_t* kout,
                              const uint32_t* vin, uint32_t* vout, uint64_t n, hipStream_t s) {
  return rocprim::radix_sort_pairs(tmp, tmp_bytes, kin, kout, vin, vout, (size_t)n, 0, 64, s);
}

hipError_t sort_pairs_u64_u32_bits(void* tmp, size_t& tmp_bytes, const uint64_t* kin, uint64_t* kout,
                                   const uint32_t* vin, uint32_t* vout, uint64_t n, int end_bit,
                                   hipStream_t s) {
  return rocprim::radix_sort_pairs(tmp, tmp_bytes, kin, kout, vin, vout, (size_t)n, 0, end_bit, s);
}

hipError_t exclusive_scan_u64(void* tmp, size_t& tmp_bytes, const uint64_t* in, uint64_t* out,
                              uint64_t n, hipStream_t s) {
  return rocprim::exclusive_scan(tmp, tmp_bytes, in, out, (uint64_t)0, (size_t)n,
                                 rocprim::plus<uint64_t>(), s);
}

hipError_t exclusive_scan_u32_u64(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint64_t* out,
                                  uint64_t n, hipStream_t s) {
  return rocprim::exclusive_scan(tmp, tmp_bytes, in, out, (uint64_t)0, (size_t)n,
                                 rocprim::plus<uint64_t>(), s);
}

hipError_t inclusive_scan_u32_u64(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint64_t* out,
                                  uint64_t n, hipStream_t s) {
  return rocprim::inclusive_scan(tmp, tmp_bytes, in, out, (size_t)n, rocprim::plus<uint64_t>(), s);
}

hipError_t exclusive_scan_u32(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint32_t* out,
                              uint64_t n, hipStream_t s) {
  return rocprim::exclusive_scan(tmp, tmp_bytes, in, out, (uint32_t)0, (size_t)n,
                                 rocprim::plus<uint32_t>(), s);
}

}  // namespace dk
