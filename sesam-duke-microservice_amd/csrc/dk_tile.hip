// dk_tile.hip — configs[2]'s schemas (bigram QGram + Numeric roles, GQArgs) on a
// BUCKET-TILED schedule (round 5).
//
// Every query record of one blocking bucket (a key function's sorted-table range: in linkage
// the other group's part of the key's bucket) has the SAME candidate range.  k_score_gq walks
// each query's range on its own: per pair every candidate bigram key is hashed and probed in
// the query's LDS table (~50 probes of ~5 VALU instructions per pair on configs[2]).  Here a
// workgroup takes one CHUNK of 64 candidates of a bucket and up to 256 of the bucket's
// queries (one wave per 64):
//  * wave 0 stages the chunk's candidate operands in LDS and builds, per QGram role, the
//    chunk's bigram -> candidate-mask table: key k's dictionary id (a dense renumbering of
//    the keys the index holds, TileArgs::lut) indexes a u64 whose bit c says candidate c of
//    the chunk has k (one LDS atomic OR per candidate key, once per chunk);
//  * each lane of a wave holds ONE query: per query key it reads its row of the mask table
//    (one LDS read for 64 candidates) and adds it into 7 bit-planes -- after its m1 keys,
//    bit c of plane p is bit p of |Q ∩ C_c| for all 64 candidates at once;
//  * then the wave walks the chunk's candidates c = 0..63 (wave-uniform operands from LDS):
//    every lane extracts its count for c from the planes and finishes the pair exactly as
//    k_score_gq (PropertyImpl.compare, computeBayes in the query's HashMap order,
//    compareCandidatesSimple's strict thresholds).
// The intersection costs ~30 bit operations per query key for 64 pairs instead of ~5
// VALU instructions per candidate key per pair.  Entries leave unordered, keyed by (query
// index, slot t of the query's concatenated candidate ranges); the host sorts them into
// Duke's order (k_score_gq's block order) -- the list is identical.
#include "dk_internal.h"
#include "dk_device.h"

#include <type_traits>

#ifndef DK_WAVES_TILE
#define DK_WAVES_TILE 4  // k_tile waves per SIMD
#endif

namespace dk {

// bit planes of the per-(query, candidate) common-gram counts: PL = 6 for sets of at most 63
// grams, 7 for 64 (k_tile<NQ, NN, PL>)

// one candidate of the chunk, staged in LDS by wave 0 (wave-uniform reads afterwards)
struct TileCand {
  uint64_t rid;       // rident (kDeadIdent: superseded, or past the bucket)
  uint64_t rk0;       // rkeys[0]: the candidate under key function 0 already (Duke's set)
  uint32_t crow;      // row
  uint16_t lq[2];     // QGram roles: rlen
  uint8_t cq[2];      // gram counts
  uint8_t c0[2];      // first unit (a one-unit value against a query without grams)
  uint16_t ln[3];     // Numeric roles: rlen
  uint8_t cok[3];
  uint8_t pad[3];
  double cn[3];
};
static_assert(sizeof(TileCand) == 64, "four ds_read_b128");

// the launch's per-role constants and outputs, in LDS: the candidate loop re-reads them per
// candidate through an address the compiler cannot hoist (kernel-argument values hoisted out
// of the loop would be held -- and spilled -- in scalar registers)
struct TileHdr {
  double low[kGroupedTabs + kGQMaxNum], high[kGroupedTabs + kGQMaxNum];
  double min_ratio[kGQMaxNum];
  double threshold, maybe;
  int32_t formula[kGroupedTabs];
  uint64_t* ecount;
  uint64_t ecap;
  uint64_t* ekey;
  uint32_t* eval;
  double* eprob;
  uint32_t* ecand;
};
using TileHdrL = const __attribute__((address_space(3))) TileHdr;
__device__ __forceinline__ TileHdrL* tl_hdr(TileHdrL* h) {
  uint32_t v = (uint32_t)(uintptr_t)h;
  asm volatile("" : "+v"(v));
  return (TileHdrL*)(uintptr_t)v;
}
template <typename T>
__device__ __forceinline__ T* tl_uptr(T* p) {  // a uniform pointer held in a VGPR -> scalar
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<T*>(((uint64_t)hi << 32) | lo);
}

template <typename T>
__device__ __forceinline__ T tl_ld(const T* p, uint64_t i) {
  return ((const __attribute__((address_space(1))) T*)(p))[i];
}
typedef unsigned int tl_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 tl_ld4(const void* p, uint64_t i) {  // 16 B at p + 16 i
  const tl_v4u v = ((const __attribute__((address_space(1))) tl_v4u*)(p))[i];
  return make_uint4(v.x, v.y, v.z, v.w);
}

// DK_TILE_CHECK: every indexed access of k_tile checked; a violation sets its bit in T.dbg and
// reads index 0 instead (fault hunting without faulting the GPU)
#ifdef DK_TILE_CHECK
#define TL_CHK(cond, bit, idx) ((cond) ? (idx) : (atomicOr(T.dbg, 1u << (bit)), (std::decay_t<decltype(idx)>)0))
#else
#define TL_CHK(cond, bit, idx) (idx)
#endif

// one work-group = two waves (the launch and __launch_bounds__ share this)
constexpr int kTileThreads = 128;

template <int NQ, int NN, int PL>
__global__ __launch_bounds__(kTileThreads) __attribute__((amdgpu_waves_per_eu(DK_WAVES_TILE, 8)))
void k_tile(const ScoreParams P, const PairSource S, const GQArgs* __restrict__ A, const TileArgs T) {
  constexpr int NR = NQ + NN;
  constexpr int NQ1 = NQ > 0 ? NQ : 1;
  extern __shared__ uint64_t masks[];  // role a: rows [T.toff[a], T.toff[a] + T.dict[a]] (the last one zero)
  __shared__ TileCand cand[64];
  __shared__ TileHdr hdr;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = lane_id();

  // ---- the item: bucket, chunk, query group ----
  const uint64_t item = blockIdx.x;
  const uint64_t b = TL_CHK(T.ibucket[item] < T.nbuckets, 0, (uint64_t)T.ibucket[item]);
  const uint32_t blen = T.blen[b], bnq = T.bnq[b], bpos = T.bpos[b], bfirst = T.bfirst[b];
  const int seg = (int)T.bseg[b];
  const uint32_t nch = (blen + 63) >> 6;
  const uint32_t local = (uint32_t)(item - T.bitem[b]);
  const uint32_t chunk = local % nch, qgroup = local / nch;
  const uint32_t clen = min(64u, blen - chunk * 64u);
  const int kf = seg >> S.seg_shift;

  for (uint32_t e = threadIdx.x; e < T.tsize; e += 128) masks[e] = 0ull;
  if (threadIdx.x == 0) {
    TileHdr h{};
    for (int a = 0; a < NQ; ++a) {
      h.low[a] = A->q[a].low;
      h.high[a] = A->q[a].high;
      h.formula[a] = A->q[a].formula;
    }
    for (int bb = 0; bb < NN; ++bb) {
      h.low[NQ + bb] = A->n[bb].low;
      h.high[NQ + bb] = A->n[bb].high;
      h.min_ratio[bb] = A->n[bb].min_ratio;
    }
    h.threshold = P.threshold;
    h.maybe = P.maybe;
    h.ecount = T.ecount;
    h.ecap = T.ecap;
    h.ekey = T.ekey;
    h.eval = T.eval;
    h.eprob = T.eprob;
    h.ecand = T.ecand;
    hdr = h;
  }
  __syncthreads();

  // ---- wave 0: the chunk's candidates -> LDS operands and the key -> candidate-mask tables ----
  if (wave == 0) {
    const bool v = lane < clen;
    const uint32_t g = TL_CHK(bpos + chunk * 64u + (v ? lane : 0u) < T.npos, 1, bpos + chunk * 64u + (v ? lane : 0u));
    TileCand tc{};
    tc.rid = v ? tl_ld(S.rident, g) : kDeadIdent;
    tc.rk0 = S.nkeys > 1 ? tl_ld(S.rkeys[0], g) : 0ull;
    tc.crow = tl_ld(P.rowof, g);
    uint32_t nwq[NQ1];
#pragma unroll
    for (int a = 0; a < NQ; ++a) {
      tc.lq[a] = tl_ld(A->q[a].rlen, g);
      const uint32_t cnt = v ? (tl_ld(A->q[a].rgcnt, g) & 0xFFu) : 0u;
      tc.cq[a] = (uint8_t)cnt;
      nwq[a] = (cnt + 3u) >> 2;
      const DevProp& D = P.props[A->q[a].prop];
      tc.c0[a] = tc.lq[a] != kMissing && tc.lq[a] > 0
                     ? static_cast<const uint8_t*>(D.units)[D.off[tc.crow]] : (uint8_t)0;
    }
#pragma unroll
    for (int bb = 0; bb < NN; ++bb) {
      tc.ln[bb] = tl_ld(A->n[bb].rlen, g);
      tc.cok[bb] = tl_ld(A->n[bb].rnumok, g);
      tc.cn[bb] = tl_ld(A->n[bb].rnum, g);
    }
    cand[lane] = tc;
    // key -> bit `lane` of the key's mask row: the rows a lane has, four keys each
#pragma unroll
    for (int a = 0; a < NQ; ++a) {
      uint64_t* tab = masks + T.toff[a];
      const uint64_t* rows = A->q[a].rows;
      const uint64_t rstride = P.rstride;
      const int nj = wave_max_i32((int)nwq[a]);
      for (int j0 = 0; j0 < nj; j0 += 4) {
        uint64_t w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t j = (uint32_t)(j0 + i);
          w[i] = j < nwq[a] ? tl_ld(rows, TL_CHK(j < A->q[a].nrows, 2, (uint64_t)j * rstride + g)) : 0ull;
        }
        uint32_t id[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t key = (uint32_t)(w[i >> 2] >> (16 * (i & 3))) & 0xFFFFu;
          id[i] = key ? (uint32_t)tl_ld(T.lut[a], key) : ~0u;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (id[i] != ~0u)
            __hip_atomic_fetch_or(tab + TL_CHK(id[i] <= T.dict[a], 3, id[i]), 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
  __syncthreads();

  // ---- the wave's blocks of 64 of the group's queries, one query per lane ----
  uint32_t scored = 0, bytes = 0;
  const uint32_t gend = min(bnq, (qgroup + 1) * kTileQueryGroup);
  for (uint32_t blk = qgroup * kTileQueryGroup + wave * 64u; blk < gend; blk += 128u) {
    const uint32_t qb = blk + lane;
    const bool qv = qb < gend;
    const uint32_t qi = TL_CHK(!qv || (uint64_t)bfirst + qb < T.nvalid, 4, qv ? (uint32_t)tl_ld(T.bkey, (uint64_t)bfirst + qb) : 0u);
#ifdef DK_TILE_CHECK
    if (qi >= T.nq) atomicOr(T.dbg, 1u << 5);
#endif
    // the query's precomputed record, its slot offset, its first key ids (one batch of loads)
    const void* rp = T.qrec + qi;
    const uint4 r0 = tl_ld4(rp, 0), r1 = tl_ld4(rp, 1), r2 = tl_ld4(rp, 2), r3 = tl_ld4(rp, 3);
    uint4 idw[NQ1];
#pragma unroll
    for (int a = 0; a < NQ; ++a)
      idw[a] = tl_ld4(T.qids + ((uint64_t)qi * NQ + a) * kTileIdsPerRole, 0);
    // slot t of candidate c = the query's candidates under earlier segments + chunk * 64 + c
    uint32_t toff = chunk * 64u;
    for (int k = 0; k < seg; ++k) {
      const uint64_t r = tl_ld(reinterpret_cast<const uint64_t*>(S.ranges), (uint64_t)k * S.nq + qi);
      toff += (uint32_t)(r >> 32) - (uint32_t)r;
    }
    TileQRec R;
    __builtin_memcpy(reinterpret_cast<uint4*>(&R) + 0, &r0, 16);
    __builtin_memcpy(reinterpret_cast<uint4*>(&R) + 1, &r1, 16);
    __builtin_memcpy(reinterpret_cast<uint4*>(&R) + 2, &r2, 16);
    __builtin_memcpy(reinterpret_cast<uint4*>(&R) + 3, &r3, 16);
    const uint64_t qident = R.ident, qk0 = R.key0;
    const uint64_t ro = A->rorder[R.oc & 3u];
    uint32_t qlen[NR > 0 ? NR : 1];
#pragma unroll
    for (int r = 0; r < NR; ++r) qlen[r] = qv ? (uint32_t)R.len[r] : (uint32_t)kMissing;
    uint32_t m1[NQ1];
#pragma unroll
    for (int a = 0; a < NQ; ++a) m1[a] = qlen[a] != kMissing ? (uint32_t)R.m1[a] : 0u;

    // ---- |Q ∩ C_c| for the 64 candidates: bit planes of the counts ----
    uint64_t pl[NQ1][PL];
#pragma unroll
    for (int a = 0; a < NQ; ++a) {
#pragma unroll
      for (int p = 0; p < PL; ++p) pl[a][p] = 0ull;
      const int mmax = wave_max_i32((int)m1[a]);
      const uint64_t* tab = masks + T.toff[a];
      const uint32_t zrow = T.dict[a];  // the zero row
      const uint16_t* ids = T.qids + ((uint64_t)qi * NQ + a) * kTileIdsPerRole;
      uint4 w = idw[a];
      for (int i0 = 0; i0 < mmax; i0 += 8) {
        const uint4 wn = tl_ld4(ids, (uint64_t)min(i0 / 8 + 1, kTileIdsPerRole / 8 - 1));  // the next 8, early
        uint64_t m[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t word = e < 2 ? w.x : e < 4 ? w.y : e < 6 ? w.z : w.w;
          const uint32_t id = (word >> (16 * (e & 1))) & 0xFFFFu;
          m[e] = tab[TL_CHK(((uint32_t)(i0 + e) < m1[a] ? id : zrow) <= T.dict[a], 6, (uint32_t)(i0 + e) < m1[a] ? id : zrow)];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          uint64_t carry = m[e];
#pragma unroll
          for (int p = 0; p < PL; ++p) {
            const uint64_t t = pl[a][p] & carry;
            pl[a][p] ^= carry;
            carry = t;
          }
        }
        w = wn;
      }
    }
    // ---- the chunk's candidates, one at a time (wave-uniform operands); candidates 0..31
    //      read the planes' low words, 32..63 the high ones ----
    auto pass = [&](auto hi_c, uint32_t c0, uint32_t c1) {
      constexpr bool HI = decltype(hi_c)::value;
      uint32_t plw[NQ1][PL];
  #pragma unroll
      for (int a = 0; a < NQ; ++a)
  #pragma unroll
        for (int p = 0; p < PL; ++p) plw[a][p] = HI ? (uint32_t)(pl[a][p] >> 32) : (uint32_t)pl[a][p];
      for (uint32_t c = c0; c < c1; ++c) {
        TileHdrL* const H = tl_hdr((TileHdrL*)&hdr);
        const TileCand tc = cand[c];
        const uint32_t cb = c & 31u;
        bool valid = qv && tc.rid != qident && tc.rid != kDeadIdent;
        if (kf > 0) valid = valid && tc.rk0 != qk0;
        uint32_t by = valid ? 9u : 0u;  // two row ids + decision (SURVEY §8d B_pair)
        double pp[NR > 0 ? NR : 1];
        bool ap[NR > 0 ? NR : 1];
  #pragma unroll
        for (int a = 0; a < NQ; ++a) {
          // the count of candidate c: bit c of each plane
          uint32_t common = 0;
  #pragma unroll
          for (int p = PL - 1; p >= 0; --p) common = (common << 1) | __builtin_amdgcn_ubfe(plw[a][p], cb, 1u);
          const uint32_t lc = tc.lq[a];
          const bool present = valid && lc != kMissing && qlen[a] != kMissing;
          const bool cmp = present && lc > 0 && qlen[a] > 0;
          const uint32_t m2 = tc.cq[a];
          double sim = 0.0;
          if (m1[a] > 0) {
            if (cmp && m2 > 0)
              sim = qgram_formula((int)common, (int)m1[a], (int)m2, (int)__builtin_amdgcn_readfirstlane(H->formula[a]));
          } else if (cmp) {  // a one-unit query value (no grams): String.equals
            sim = lc == qlen[a] && tc.c0[a] == (uint32_t)R.c0[a] ? 1.0 : 0.0;
          }
          if (present) by += 2u;
          if (cmp) by += 6u + 2u * m2;
          pp[a] = cmp ? gq_prob(H->low[a], H->high[a], sim) : 0.0;
          ap[a] = present;
        }
  #pragma unroll
        for (int bb = 0; bb < NN; ++bb) {
          const uint32_t lc = tc.ln[bb];
          const bool present = valid && lc != kMissing && qlen[NQ + bb] != kMissing;
          const bool cmp = present && lc > 0 && qlen[NQ + bb] > 0;
          double sim = 0.0;
          if (cmp) sim = numeric(R.num[bb], R.ok[bb] != 0u, tc.cn[bb], tc.cok[bb] != 0u, H->min_ratio[bb]);
          if (present) by += 2u;
          if (cmp) by += 9u;
          pp[NQ + bb] = cmp ? gq_prob(H->low[NQ + bb], H->high[NQ + bb], sim) : 0.0;
          ap[NQ + bb] = present;
        }
        // [Duke 1.2] Processor.compare: computeBayes over r1's properties in its HashMap order
        double prob = 0.5;
  #pragma unroll
        for (int k = 0; k < NR; ++k) {
          const uint32_t r = (uint32_t)(ro >> (4 * k)) & 15u;
          const int ri = r >= 8u ? NQ + (int)(r - 8u) : (int)r;
          double x = 0.5;
          bool use = false;
  #pragma unroll
          for (int i = 0; i < NR; ++i)
            if (ri == i) {
              x = pp[i];
              use = ap[i];
            }
          const double nb = compute_bayes(prob, x);
          prob = use ? nb : prob;
        }
        // [Duke 1.2] Processor.compareCandidatesSimple: strict thresholds; entries leave keyed
        // by (query index, slot) for the host's ordering sort
        const uint32_t kind = valid ? decide(prob, H->threshold, H->maybe) : 0u;
        const uint64_t em = __ballot(kind != 0u);
        if (em) {
          const int first = __builtin_ffsll((long long)em) - 1;
          uint64_t base = 0;
          if ((int)lane == first)
            base = atomicAdd((unsigned long long*)tl_uptr(H->ecount), (unsigned long long)__popcll(em));
          const uint32_t blo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)base, first);
          const uint32_t bhi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(base >> 32), first);
          base = ((uint64_t)bhi << 32) | blo;
          if (kind != 0u) {
            const uint64_t e = base + mask_rank(em);
            if (e < H->ecap) {
              tl_uptr(H->ekey)[e] = ((uint64_t)qi << 32) | (toff + c);
              tl_uptr(H->eval)[e] = (uint32_t)e;
              tl_uptr(H->eprob)[e] = prob;
              tl_uptr(H->ecand)[e] = tc.crow | (kind << kKindShift);
            }
          }
        }
        scored += valid ? 1u : 0u;
        bytes += by;
      }
    };
    pass(std::integral_constant<bool, false>{}, 0u, min(clen, 32u));
    if (clen > 32u) pass(std::integral_constant<bool, true>{}, 32u, clen);
  }
  const uint32_t ss = wave_sum_u32(scored), sb = wave_sum_u32(bytes);
  if (lane == 0) {
    if (ss) atomicAdd((unsigned long long*)&T.counters[0], (unsigned long long)ss);
    if (sb) atomicAdd((unsigned long long*)&T.counters[1], (unsigned long long)sb);
  }
}

hipError_t launch_tile(const ScoreParams& P, const PairSource& src, const GQArgs* A, int nq, int nn,
                       int planes, const TileArgs& T, hipStream_t s) {
  if (T.nitems == 0) return hipSuccess;
  if (T.nitems >= (1ull << 31)) return hipErrorInvalidValue;
  const size_t lds = (size_t)T.tsize * 8;
#define DK_TILE_CASE(NQ_, NN_)                                                                  \
  if (nq == NQ_ && nn == NN_) {                                                                 \
    if (planes == 6) k_tile<NQ_, NN_, 6><<<(unsigned)T.nitems, kTileThreads, lds, s>>>(P, src, A, T);    \
    else k_tile<NQ_, NN_, 7><<<(unsigned)T.nitems, kTileThreads, lds, s>>>(P, src, A, T);                \
    return hipGetLastError();                                                                   \
  }
  DK_TILE_CASE(1, 0) DK_TILE_CASE(1, 1) DK_TILE_CASE(1, 2) DK_TILE_CASE(1, 3)
  DK_TILE_CASE(2, 0) DK_TILE_CASE(2, 1) DK_TILE_CASE(2, 2) DK_TILE_CASE(2, 3)
#undef DK_TILE_CASE
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------
// the dictionary: every bigram key the property's gram arena holds -> a dense id
// ---------------------------------------------------------------------------------------
__global__ void k_tile_mark(const uint64_t* __restrict__ grams, uint64_t g0, uint64_t n,
                            uint32_t* __restrict__ present) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t key = gram_key(grams[g0 + i]);
  if (!present[key]) present[key] = 1u;  // racing writers all store 1
}

hipError_t launch_tile_mark(const uint64_t* grams, uint64_t g0, uint64_t n, uint32_t* present, hipStream_t s) {
  if (n == 0) return hipSuccess;
  k_tile_mark<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(grams, g0, n, present);
  return hipGetLastError();
}

// lut[key] = exclusive prefix of present (the id), as u16
__global__ void k_tile_lut(const uint32_t* __restrict__ scan, uint16_t* __restrict__ lut) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < 65536u) lut[k] = (uint16_t)scan[k];
}

hipError_t launch_tile_lut(const uint32_t* scan, uint16_t* lut, hipStream_t s) {
  k_tile_lut<<<256, 256, 0, s>>>(scan, lut);
  return hipGetLastError();
}

// per query: the values k_tile reads of it (TileQRec)
__global__ void k_tile_qrec(const ScoreParams P, const PairSource S, const GQArgs* __restrict__ A,
                            TileQRec* __restrict__ out) {
  const uint64_t qi = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (qi >= S.nq) return;
  const uint32_t q = S.queries[qi];
  TileQRec R{};
  R.ident = P.ident[q];
  R.key0 = S.nkeys > 1 ? S.qkeys[0][q] : 0ull;
  R.oc = P.norders > 1 ? P.oclass[q] : 0;
  for (int a = 0; a < A->nq; ++a) {
    const DevProp& D = P.props[A->q[a].prop];
    const uint16_t l = D.len[q];
    R.len[a] = l;
    R.m1[a] = l != kMissing ? (uint8_t)D.gcnt[q] : 0;
    R.c0[a] = l != kMissing && l > 0 ? static_cast<const uint8_t*>(D.units)[D.off[q]] : 0;
  }
  for (int b = 0; b < A->nn; ++b) {
    const DevProp& D = P.props[A->n[b].prop];
    R.len[A->nq + b] = D.len[q];
    R.ok[b] = D.numok[q];
    R.num[b] = D.num[q];
  }
  out[qi] = R;
}

hipError_t launch_tile_qrec(const ScoreParams& P, const PairSource& src, const GQArgs* A, TileQRec* qrec,
                            hipStream_t s) {
  if (src.nq == 0) return hipSuccess;
  k_tile_qrec<<<(unsigned)((src.nq + 255) / 256), 256, 0, s>>>(P, src, A, qrec);
  return hipGetLastError();
}

// per query and QGram role: its keys' ids (kTileIdsPerRole slots, ids past its grams 0)
__global__ void k_tile_qids(const ScoreParams P, const uint32_t* __restrict__ queries, uint64_t nq,
                            const GQArgs* __restrict__ A, int nqr, const uint16_t* lut0, const uint16_t* lut1,
                            uint16_t* __restrict__ qids) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq * (uint64_t)nqr) return;
  const uint64_t qi = i / (uint64_t)nqr;
  const int a = (int)(i % (uint64_t)nqr);
  const uint32_t q = queries[qi];
  const DevProp& D = P.props[A->q[a].prop];
  const uint16_t* lut = a == 0 ? lut0 : lut1;
  const int m = D.len[q] == kMissing ? 0 : (int)D.gcnt[q];
  const uint64_t* g = D.grams + D.goff[q];
  uint16_t* out = qids + i * kTileIdsPerRole;
  for (int k = 0; k < kTileIdsPerRole; ++k) out[k] = k < m ? lut[gram_key(g[k])] : (uint16_t)0;
}

hipError_t launch_tile_qids(const ScoreParams& P, const uint32_t* queries, uint64_t nq, const GQArgs* A,
                            int nqr, const uint16_t* lut0, const uint16_t* lut1, uint16_t* qids,
                            hipStream_t s) {
  const uint64_t n = nq * (uint64_t)nqr;
  if (n == 0) return hipSuccess;
  k_tile_qids<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(P, queries, nq, A, nqr, lut0, lut1, qids);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// buckets: every (segment, query) with candidates, keyed by its range's first replica
// position (a range is a bucket, or in linkage the other group's part of one: equal
// starts = equal ranges), sorted; runs of equal starts are the buckets
// ---------------------------------------------------------------------------------------
__global__ void k_tile_bkeys(const PairSource S, uint64_t* __restrict__ key, uint64_t* __restrict__ nvalid) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool v = false;
  if (i < (uint64_t)S.nseg * S.nq) {
    const uint64_t k = i / S.nq, qi = i % S.nq;
    const uint2 r = S.ranges[i];
    v = r.y > r.x;
    key[i] = v ? ((S.segoff[k] + r.x) << 32) | qi : ~0ull;
  }
  const uint64_t m = __ballot(v);
  if (lane_id() == 0 && m) atomicAdd((unsigned long long*)nvalid, (unsigned long long)__popcll(m));
}

hipError_t launch_tile_bkeys(const PairSource& S, uint64_t* key, uint64_t* nvalid, hipStream_t s) {
  const uint64_t n = (uint64_t)S.nseg * S.nq;
  if (n == 0) return hipSuccess;
  k_tile_bkeys<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(S, key, nvalid);
  return hipGetLastError();
}

// head[i] = 1 where sorted key i starts a bucket (i < nvalid)
__global__ void k_tile_heads(const uint64_t* __restrict__ key, uint64_t n, uint32_t* __restrict__ head) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = key[i];
  head[i] = k != ~0ull && (i == 0 || (key[i - 1] >> 32) != (k >> 32)) ? 1u : 0u;
}

hipError_t launch_tile_heads(const uint64_t* key, uint64_t n, uint32_t* head, hipStream_t s) {
  if (n == 0) return hipSuccess;
  k_tile_heads<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(key, n, head);
  return hipGetLastError();
}

// per bucket (bid[i] = exclusive prefix of head): first key, position, segment, length and
// its items (chunks of 64 candidates x groups of kTileQueryGroup queries; the query count is filled by
// the next bucket's head, or n)
__global__ void k_tile_buckets(const PairSource S, const uint64_t* __restrict__ key, uint64_t n,
                               const uint32_t* __restrict__ head, const uint32_t* __restrict__ bid,
                               uint32_t* __restrict__ bfirst, uint32_t* __restrict__ bpos,
                               uint32_t* __restrict__ bseg, uint32_t* __restrict__ blen) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !head[i]) return;
  const uint64_t k = key[i];
  const uint32_t pos = (uint32_t)(k >> 32), qi = (uint32_t)k;
  int seg = 0;
  for (int s2 = 1; s2 < S.nseg; ++s2)
    if (S.segoff[s2] <= pos) seg = s2;
  const uint2 r = S.ranges[(uint64_t)seg * S.nq + qi];
  const uint32_t b = bid[i];
  bfirst[b] = (uint32_t)i;
  bpos[b] = pos;
  bseg[b] = (uint32_t)seg;
  blen[b] = r.y - r.x;
}

__global__ void k_tile_items(const uint32_t* __restrict__ bfirst, const uint32_t* __restrict__ blen,
                             uint64_t nb, uint64_t nvalid, uint32_t* __restrict__ bnq,
                             uint64_t* __restrict__ nitems) {
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  const uint32_t nq = (uint32_t)((b + 1 < nb ? bfirst[b + 1] : nvalid) - bfirst[b]);
  bnq[b] = nq;
  nitems[b] = (uint64_t)((blen[b] + 63) / 64) * ((nq + kTileQueryGroup - 1) / kTileQueryGroup);
}

hipError_t launch_tile_buckets(const PairSource& S, const uint64_t* key, uint64_t n, uint64_t nvalid,
                               const uint32_t* head, const uint32_t* bid, uint64_t nb, uint32_t* bfirst,
                               uint32_t* bpos, uint32_t* bseg, uint32_t* blen, uint32_t* bnq,
                               uint64_t* nitems, hipStream_t s) {
  if (n == 0 || nb == 0) return hipSuccess;
  k_tile_buckets<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(S, key, n, head, bid, bfirst, bpos, bseg, blen);
  k_tile_items<<<(unsigned)((nb + 255) / 256), 256, 0, s>>>(bfirst, blen, nb, nvalid, bnq, nitems);
  return hipGetLastError();
}

// item -> its bucket (binary search over the buckets' first items; off the scoring kernel's
// critical path)
__global__ void k_tile_itemmap(const uint64_t* __restrict__ bitem, uint64_t nb, uint64_t nitems,
                               uint32_t* __restrict__ ibucket) {
  const uint64_t item = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= nitems) return;
  uint64_t lo = 0, hi = nb;
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (bitem[mid] <= item) lo = mid; else hi = mid;
  }
  ibucket[item] = (uint32_t)lo;
}

hipError_t launch_tile_itemmap(const uint64_t* bitem, uint64_t nb, uint64_t nitems, uint32_t* ibucket,
                               hipStream_t s) {
  if (nitems == 0) return hipSuccess;
  k_tile_itemmap<<<(unsigned)((nitems + 255) / 256), 256, 0, s>>>(bitem, nb, nitems, ibucket);
  return hipGetLastError();
}

// the sorted entries -> the match list (candidate row, kind, probability, query index)
__global__ void k_tile_emit(const uint64_t* __restrict__ skey, const uint32_t* __restrict__ sval, uint64_t n,
                            const double* __restrict__ eprob, const uint32_t* __restrict__ ecand,
                            MatchList out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t e = sval[i];
  const uint32_t cw = ecand[e];
  out.cand[i] = cw & ((1u << kKindShift) - 1u);
  out.kind[i] = (uint8_t)(cw >> kKindShift);
  out.prob[i] = eprob[e];
  out.qidx[i] = (uint32_t)(skey[i] >> 32);
}

hipError_t launch_tile_emit(const uint64_t* skey, const uint32_t* sval, uint64_t n, const double* eprob,
                            const uint32_t* ecand, const MatchList& out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  k_tile_emit<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(skey, sval, n, eprob, ecand, out);
  return hipGetLastError();
}

}  // namespace dk
