// dk_kernels.hip — gfx950 kernels of the Duke candidate-pair scoring path.
//
// Compiled with -ffp-contract=off and without fast-math: every double operation is a
// single IEEE round-to-nearest operation, as in the JVM, so probabilities reproduce
// Duke's bit for bit when evaluated in the same order.
//
// Hot path (SURVEY §3.1 loops 2-4): k_score — one lane per (query, candidate) slot,
// all properties fused: comparator -> PropertyImpl low/high mapping -> computeBayes ->
// strict threshold -> wave-ballot compaction of match / maybe entries.
#include <cstring>

#include <algorithm>
#include <rocprim/rocprim.hpp>

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

template <typename CT>
__device__ __forceinline__ bool units_equal(const CT* a, int na, const CT* b, int nb) {
  if (na != nb) return false;
  // strings start 4-byte aligned and are zero padded to a 4-byte multiple
  const uint32_t* wa = reinterpret_cast<const uint32_t*>(a);
  const uint32_t* wb = reinterpret_cast<const uint32_t*>(b);
  const int nw = (na * (int)sizeof(CT) + 3) >> 2;
  for (int i = 0; i < nw; ++i)
    if (wa[i] != wb[i]) return false;
  return true;
}

// ------------------------------------------------------------------------------------
// [Duke 1.2] comparators.Levenshtein.compactDistance, lane per pair.
// s1 (the query value, Processor.compare's r1) indexes the DP column, kept in VGPRs and
// unrolled to MAXM rows; s2 (candidate) streams one code unit per column.  Rows past
// n1 compute garbage that never feeds rows <= n1 (the recurrence only looks up and
// left); they are excluded from the cutoff minimum.  Preconditions: 1 <= n1 <= MAXM,
// n2 >= 1, arena over-read of MAXM units past s1 is in bounds (tail padding).
// ------------------------------------------------------------------------------------
template <int MAXM, typename CT>
__device__ __forceinline__ int compact_distance(const CT* __restrict__ s1, int n1,
                                                const CT* __restrict__ s2, int n2) {
  uint32_t a[MAXM];
#pragma unroll
  for (int i = 0; i < MAXM; ++i) a[i] = s1[i];
  int col[MAXM + 1];
  const int maxdist = min(n1, n2) >> 1;
  uint32_t ch = s2[0];
  col[0] = 1;  // virtual first row
#pragma unroll
  for (int i = 1; i <= MAXM; ++i) col[i] = min(col[i - 1], i - 1) + (a[i - 1] != ch ? 1 : 0);
  int above = 0;
  int result = -1;
  for (int j = 1; j < n2; ++j) {
    ch = s2[j];
    above = j + 1;  // virtual first row
    int smallest = 2 * n1;
#pragma unroll
    for (int i = 1; i <= MAXM; ++i) {
      const int v = imin3(above, col[i - 1], col[i]) + (a[i - 1] != ch ? 1 : 0);
      col[i - 1] = above;
      above = v;
      smallest = (i <= n1) ? min(smallest, v) : smallest;
    }
    col[MAXM] = above;
    if (smallest > maxdist) {
      result = smallest;
      break;
    }
  }
  if (result < 0) {
    if (n2 == 1) return 0;  // Duke returns its initial `above` when |s2| == 1
    // D[n1][n2-1] was parked in col[n1] (written at unrolled row n1+1, or row MAXM above)
    int r = col[0];
#pragma unroll
    for (int i = 1; i <= MAXM; ++i) r = (i == n1) ? col[i] : r;
    result = r;
  }
  return result;
}

// [Duke 1.2] comparators.Levenshtein.compare
template <typename CT>
__device__ __forceinline__ double levenshtein(const CT* s1, int n1, const CT* s2, int n2,
                                              int bucket) {
  const int len = min(n1, n2);
  const int maxlen = max(n1, n2);
  if ((double)len / (double)maxlen <= 0.5) return 0.0;
  if (len == maxlen && units_equal(s1, n1, s2, n2)) return 1.0;
  int d;
  if (bucket <= 16) d = compact_distance<16>(s1, n1, s2, n2);
  else if (bucket <= 32) d = compact_distance<32>(s1, n1, s2, n2);
  else d = compact_distance<64>(s1, n1, s2, n2);
  const int dist = min(d, len);
  return 1.0 - ((double)dist / (double)len);
}

// [Duke 1.2] comparators.JaroWinkler.similarity
template <typename CT>
__device__ __forceinline__ double jarowinkler(const CT* s1, int n1, const CT* s2, int n2) {
  if (units_equal(s1, n1, s2, n2)) return 1.0;
  if (n1 > n2) {
    const CT* ts = s2; s2 = s1; s1 = ts;
    int tn = n2; n2 = n1; n1 = tn;
  }
  const int maxdist = n2 >> 1;
  int c = 0, t = 0, prevpos = -1;
  for (int ix = 0; ix < n1; ++ix) {
    const uint32_t ch = s1[ix];
    const int hi = min(n2, ix + maxdist);
    for (int ix2 = max(0, ix - maxdist); ix2 < hi; ++ix2) {
      if (ch == (uint32_t)s2[ix2]) {
        ++c;
        if (prevpos != -1 && ix2 < prevpos) ++t;
        prevpos = ix2;
        break;
      }
    }
  }
  if (c == 0) return 0.0;
  double score = ((c / (double)n1) + (c / (double)n2) + ((c - t) / (double)c)) / 3.0;
  int p = 0;
  const int last = min(4, n1);
  while (p < last && s1[p] == s2[p]) ++p;
  score += ((p * (1 - score)) / 10);
  return score;
}

// [Duke 1.2] comparators.QGramComparator.compare over precomputed sorted unique gram sets
__device__ __forceinline__ double qgram_formula(int common, int m1, int m2, int formula) {
  if (formula == DK_QGRAM_JACCARD) return (double)common / (double)(m1 + m2 - common);
  if (formula == DK_QGRAM_DICE) return (2.0 * (double)common) / (double)(m1 + m2);
  return (double)common / fmin((double)m1, (double)m2);
}

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

// ------------------------------------------------------------------------------------
// The fused scoring kernel.
// ------------------------------------------------------------------------------------
template <typename CT>
__device__ __forceinline__ double string_sim(const DevProp& D, uint32_t q, uint32_t c, int lq,
                                             int lc, int bucket) {
  const CT* base = reinterpret_cast<const CT*>(D.units);
  const CT* s1 = base + D.off[q];
  const CT* s2 = base + D.off[c];
  switch (D.op) {
    case DK_CMP_LEVENSHTEIN: return levenshtein(s1, lq, s2, lc, bucket);
    case DK_CMP_JAROWINKLER: return jarowinkler(s1, lq, s2, lc);
    case DK_CMP_EXACT: return units_equal(s1, lq, s2, lc) ? 1.0 : 0.0;
    case DK_CMP_QGRAM: {
      if (units_equal(s1, lq, s2, lc)) return 1.0;
      const int m1 = D.gcnt[q], m2 = D.gcnt[c];
      if (m1 == 0 || m2 == 0) return 0.0;
      const int common = intersect_sorted(D.grams + D.goff[q], m1, D.grams + D.goff[c], m2);
      return qgram_formula(common, m1, m2, D.formula);
    }
    default: return 0.5;
  }
}

__global__ __launch_bounds__(256) void k_score(const ScoreParams P, const PairSource S,
                                               uint64_t slot0, uint64_t nslots, StageOut out) {
  const uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool valid = idx < nslots;
  uint32_t qi = 0, q = 0, c = 0;
  if (valid) {
    if (S.allpairs) {
      const uint64_t g = slot0 + idx;
      qi = (uint32_t)(g / S.m);
      c = S.usable[g - (uint64_t)qi * S.m];
      q = S.queries[qi];
      valid = P.ident[c] != P.ident[q];  // Processor.isSameAs
    } else {
      qi = S.pq[idx];
      const uint32_t w = S.pc[idx];
      valid = w != kSentinel;
      c = w & kRowMask;
      q = S.queries[qi];
    }
  }

  double prob = 0.5;
  uint32_t bytes = valid ? 9u : 0u;  // two row ids + decision (SURVEY §8d B_pair)
  for (int p = 0; p < P.nprops; ++p) {
    const DevProp& D = P.props[p];
    const int lq = valid ? (int)D.len[q] : (int)kMissing;
    const int lc = valid ? (int)D.len[c] : (int)kMissing;
    const bool present = lq != (int)kMissing && lc != (int)kMissing;
    const bool cmp = present && lq > 0 && lc > 0;
    int bucket = 64;
    if (D.op == DK_CMP_LEVENSHTEIN) {
      // wave-uniform row bucket for the DP column: the longest query value in the wave
      bucket = __ballot(cmp && lq > 32) ? 64 : (__ballot(cmp && lq > 16) ? 32 : 16);
    }
    if (present) {
      double high = 0.0;
      if (cmp) {
        double sim;
        if (D.op == DK_CMP_NUMERIC) {
          sim = numeric(D.num[q], D.numok[q] != 0, D.num[c], D.numok[c] != 0, D.min_ratio);
          bytes += 16;
        } else if (D.op == DK_CMP_NONE) {
          sim = -1.0;
        } else {
          sim = D.width == 1 ? string_sim<uint8_t>(D, q, c, lq, lc, bucket)
                             : string_sim<uint16_t>(D, q, c, lq, lc, bucket);
          bytes += 8u + (uint32_t)(lq + lc) * (uint32_t)D.width;
          if (D.op == DK_CMP_QGRAM) bytes += 8u + 8u * (uint32_t)(D.gcnt[q] + D.gcnt[c]);
        }
        // [Duke 1.2] PropertyImpl.compare
        const double v = D.op == DK_CMP_NONE ? 0.5
                         : (sim < 0.5 ? D.low : ((D.high - 0.5) * (sim * sim)) + 0.5);
        high = java_max(high, v);
      }
      prob = compute_bayes(prob, high);
    }
  }

  // [Duke 1.2] Processor.compareCandidatesSimple: strict thresholds
  uint32_t kind = 0;
  if (valid) {
    if (prob > P.threshold) kind = DK_KIND_MATCH;
    else if (P.maybe != 0.0 && prob > P.maybe) kind = DK_KIND_MAYBE;
  }

  // block-ordered compaction: wave ballots -> per-wave counts in LDS -> slot-ordered
  // entries at the block's staging region; no atomics on entries
  __shared__ uint32_t wcount[kScoreBlock / 64];
  const uint64_t em = __ballot(kind != 0);
  const uint64_t vm = __ballot(valid);
  const uint32_t wave = threadIdx.x >> 6;
  uint32_t wbytes = bytes;
  for (int o = 32; o > 0; o >>= 1) wbytes += __shfl_xor(wbytes, o);
  if (lane_id() == 0) {
    wcount[wave] = (uint32_t)__popcll(em);
    if (vm) {
      atomicAdd((unsigned long long*)&out.counters[0], (unsigned long long)__popcll(vm));
      atomicAdd((unsigned long long*)&out.counters[1], (unsigned long long)wbytes);
    }
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
    const uint64_t e = (uint64_t)blockIdx.x * kScoreBlock + before + mask_rank(em);
    out.prob[e] = prob;
    out.cand[e] = c | (kind << kKindShift);
    out.qidx[e] = qi;
  }
  if (threadIdx.x == 0) out.bcnt[blockIdx.x] = total;
}

// Concatenate the per-block staged entries in block order (one block per score block).
__global__ __launch_bounds__(256) void k_compact(const StageOut st, const uint64_t* __restrict__ boff,
                                                 uint64_t base, MatchList out) {
  const uint32_t b = blockIdx.x;
  const uint32_t n = st.bcnt[b];
  const uint32_t i = threadIdx.x;
  if (i >= n) return;
  const uint64_t src = (uint64_t)b * kScoreBlock + i;
  const uint64_t dst = base + boff[b] + i;
  const uint32_t w = st.cand[src];
  out.cand[dst] = w & ((1u << kKindShift) - 1u);
  out.kind[dst] = (uint8_t)(w >> kKindShift);
  out.prob[dst] = st.prob[src];
  out.qidx[dst] = st.qidx[src];
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

// Per query and key function: the candidate range [lo, hi) in the sorted table.  The
// query's own key is looked up by value, so a superseded or deleted query still finds
// its block.  LINKAGE keeps only the other group's sub-range (rows are sorted by
// (key, group, row) and groups are 1 and 2; IncrementalDataSource.java:80-84).
__global__ void k_count(const uint32_t* __restrict__ queries, uint64_t nq, const BlockTables T,
                        uint2* __restrict__ ranges, uint64_t* __restrict__ counts) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  const uint32_t q = queries[i];
  uint64_t total = 0;
  for (int k = 0; k < T.nkeys; ++k) {
    const uint64_t key = T.keys[k][q];
    const uint64_t lo = lower_bound_u64(T.skeys[k], T.n[k], key);
    const uint64_t hi = upper_bound_u64(T.skeys[k], lo, T.n[k], key);
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
  counts[i] = total;
}

// One wave per query (grid-stride): writes the query's candidate slots that fall in
// [s0, s1).  Slot order inside a query = key function, then (group, row) order of the
// sorted table.  Filters: isSameAs (identity) and "already a candidate under an
// earlier key function" (Duke returns candidates as a set).
__global__ __launch_bounds__(256) void k_emit(const uint32_t* __restrict__ queries, uint64_t q0,
                                              uint64_t q1, const uint64_t* __restrict__ qoff,
                                              const uint2* __restrict__ ranges, uint64_t nq,
                                              const BlockTables T, const uint64_t* __restrict__ ident,
                                              uint64_t s0, uint64_t s1, uint32_t* __restrict__ pq,
                                              uint32_t* __restrict__ pc) {
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t qi = q0 + wave; qi < q1; qi += nwaves) {
    const uint64_t qa = qoff[qi], qb = qoff[qi + 1];
    const uint64_t a = max(qa, s0), b = min(qb, s1);
    if (a >= b) continue;
    const uint32_t q = queries[qi];
    const uint64_t idq = ident[q];
    for (uint64_t s = a + lane; s < b; s += 64) {
      uint64_t t = s - qa;
      int k = 0;
      uint2 r = ranges[qi];
      for (; k < T.nkeys - 1; ++k) {
        r = ranges[(uint64_t)k * nq + qi];
        const uint64_t len = (uint64_t)(r.y - r.x);
        if (t < len) break;
        t -= len;
      }
      if (k == T.nkeys - 1) r = ranges[(uint64_t)k * nq + qi];
      const uint32_t c = T.srows[k][r.x + t];
      bool ok = ident[c] != idq;
      for (int j = 0; j < k && ok; ++j)
        ok = T.keys[j][c] != T.keys[j][q];
      pq[s - s0] = (uint32_t)qi;
      pc[s - s0] = ok ? (c | ((uint32_t)k << kKeyShift)) : kSentinel;
    }
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
                              uint64_t n, int want_group, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool ok = (flags[i] & (kAlive | kDeleted)) == kAlive;
  if (want_group > 0) ok = ok && ((int)group[i] == want_group || (want_group == 2 && group[i] > 2));
  out[i] = ok ? 1u : 0u;
}

__global__ void k_scatter_rows(const uint32_t* __restrict__ flag, const uint32_t* __restrict__ pos,
                               uint64_t n, uint32_t base, uint32_t* __restrict__ rows) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && flag[i]) rows[base + pos[i]] = (uint32_t)i;
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

hipError_t launch_select_rows(const uint8_t* flags, const uint8_t* group, uint64_t nrows,
                              int want_group, uint32_t* flag_out, hipStream_t s) {
  DK_LAUNCH_GUARD(nrows);
  k_select_rows<<<grid1d(nrows), 256, 0, s>>>(flags, group, nrows, want_group, flag_out);
  return hipGetLastError();
}

hipError_t launch_scatter_rows(const uint32_t* flag, const uint32_t* pos, uint64_t nrows,
                               uint32_t base, uint32_t* rows_out, hipStream_t s) {
  DK_LAUNCH_GUARD(nrows);
  k_scatter_rows<<<grid1d(nrows), 256, 0, s>>>(flag, pos, nrows, base, rows_out);
  return hipGetLastError();
}

hipError_t launch_count(const uint32_t* queries, uint64_t nq, const BlockTables& T, uint2* ranges,
                        uint64_t* counts, hipStream_t s) {
  DK_LAUNCH_GUARD(nq);
  k_count<<<grid1d(nq), 256, 0, s>>>(queries, nq, T, ranges, counts);
  return hipGetLastError();
}

hipError_t launch_emit(const uint32_t* queries, uint64_t q0, uint64_t q1, const uint64_t* qoff,
                       const uint2* ranges, uint64_t nq, const BlockTables& T,
                       const uint64_t* ident, uint64_t s0, uint64_t s1, uint32_t* pq,
                       uint32_t* pc, hipStream_t s) {
  if (q1 <= q0 || s1 <= s0) return hipSuccess;
  const uint64_t waves = q1 - q0;
  const unsigned blocks = (unsigned)std::min<uint64_t>((waves + 3) / 4, 256u * 32u);
  k_emit<<<blocks, 256, 0, s>>>(queries, q0, q1, qoff, ranges, nq, T, ident, s0, s1, pq, pc);
  return hipGetLastError();
}

hipError_t launch_score(const ScoreParams& P, const PairSource& src, uint64_t slot0,
                        uint64_t nslots, const StageOut& out, hipStream_t s) {
  DK_LAUNCH_GUARD(nslots);
  k_score<<<grid1d(nslots, kScoreBlock), kScoreBlock, 0, s>>>(P, src, slot0, nslots, out);
  return hipGetLastError();
}

hipError_t launch_compact(const StageOut& st, const uint64_t* boff, uint64_t nblocks,
                          uint64_t base, const MatchList& out, hipStream_t s) {
  DK_LAUNCH_GUARD(nblocks);
  k_compact<<<(unsigned)nblocks, kScoreBlock, 0, s>>>(st, boff, base, out);
  return hipGetLastError();
}

hipError_t launch_first(const uint32_t* qidx, uint64_t n, uint64_t nq, uint64_t* first,
                        hipStream_t s) {
  k_first<<<grid1d(nq + 1), 256, 0, s>>>(qidx, n, nq, first);
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

hipError_t exclusive_scan_u32(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint32_t* out,
                              uint64_t n, hipStream_t s) {
  return rocprim::exclusive_scan(tmp, tmp_bytes, in, out, (uint32_t)0, (size_t)n,
                                 rocprim::plus<uint32_t>(), s);
}

}  // namespace dk
