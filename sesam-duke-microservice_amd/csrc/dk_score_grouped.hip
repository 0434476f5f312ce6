// dk_score_grouped.hip — the scoring kernel of schemas made of Latin-1 bigram QGram and
// Numeric properties (BASELINE configs[2]: NAME / ADDRESS QGram q=2, BIRTHYEAR / ZIP
// Numeric), the north-star linkage.
//
// Same semantics as k_score (dk_kernels.hip: Processor.compareCandidatesSimple ->
// Processor.compare -> PropertyImpl.compare -> computeBayes, strict thresholds), on a
// schedule built for latency instead of arithmetic: these comparators do a few dozen
// operations per pair, so k_score_nodp's waves spent 0.75 of their cycles parked on a
// chain of ~10 dependent memory round trips (wave map, ranges, candidate position,
// lengths, code counts, key words, per property in turn) and rebuilt the query's
// perfect-hash tables for every 64 candidates.
//
//  * One wave owns a TASK: 256 consecutive slots (four groups of 64 candidates) of ONE
//    query -- the host pads every query's slots to 256 (launch_count pad 256).  The
//    query's bigram tables are built once per task, and the task's slots are the staging
//    block of the block-ordered compaction (k_compact), so the list order is unchanged.
//  * Waves are independent: four tasks per 256-thread workgroup, no workgroup barrier;
//    each wave's LDS slice holds its query's tables.
//  * Candidate operands are loaded one PROPERTY ahead: while property p of a group is
//    probed, property p+1's lengths, code counts, first key-word rows (or numeric value)
//    are in flight; after a group's last property the next group's candidate positions,
//    filters and first property follow.  One round trip per property, overlapped.
#include "dk_internal.h"
#include "dk_device.h"

#include <type_traits>

#ifndef DK_WAVES_GROUPED
#define DK_WAVES_GROUPED 8  // k_score_grouped waves per SIMD
#endif
#ifndef DK_GROUPED_KEYS
#define DK_GROUPED_KEYS 1   // key functions whose filter operand is prefetched (+1: the first)
#endif
#ifndef DK_GROUPED_TAIL
#define DK_GROUPED_TAIL 4   // rows per load batch past 2 * DK_GROUPED_ROWS
#endif
#ifndef DK_GROUPED_ROWS
#define DK_GROUPED_ROWS 2   // key-word rows (4 bigram keys each) loaded one property ahead
#endif

namespace dk {

constexpr int kTaskGroups = kScoreBlock / 64;  // groups of 64 slots per task
constexpr int kPreRows = DK_GROUPED_ROWS;
static_assert(2 * kPreRows <= kGroupedHeadRows, "the head rows' resource covers rows < kGroupedHeadRows");
constexpr int kTabWords = 512;  // u32 per bigram table (lt <= 9)
constexpr int kPreKeys = DK_GROUPED_KEYS;  // key-function filters loaded one step ahead
constexpr int kTailRows = DK_GROUPED_TAIL;
constexpr uint32_t kRsrcWord3 = 0x00020000u;  // gfx9 raw buffer: 32-bit data format

// Candidate operands are read with raw buffer loads: every load of the prefetch is issued
// unconditionally -- no branch, hence no wait at a join that would drain the loads in
// flight -- and a load past a resource's size (a row the property does not have) returns 0
// without a memory access.
using rsrc_t = __amdgpu_buffer_rsrc_t;

// The query's per-property values, staged in LDS once per task (LDS reads wait on lgkmcnt
// only; a vector load of a uniform u16 would wait on vmcnt, draining the prefetch).
struct QueryVals {
  uint16_t len, gcnt, seed;
  uint8_t numok, pad;
  double num;
};
static_assert(sizeof(QueryVals) == 16, "one ds_read_b128");

// One property's candidate operands of one group, loaded one step ahead.
struct PreOps {
  uint32_t lc;            // rlen (kMissing: no value)
  uint32_t x;             // bigram QGram: rgcnt (its low byte: sets <= 64 grams); Numeric: rnumok
  uint64_t w[kPreRows];   // bigram QGram: key-word rows 0..kPreRows-1; Numeric: w[0] = rnum's bits
};

// Per-property buffer resources of the candidate operands (wave-uniform), from the host's
// GroupedProp record.  Key-word row j of a bigram property (a Numeric property's value is
// its row 0) sits at byte g * 8 + j * rowb of w.  MODE 0: one resource over the property's
// rows, offsets below 2^32 (the host checks, tail rows included), so a row past the
// property's rows is out of range (0, no data moved).  Replicas past that (configs[2] at
// 10M x 10M: 40M positions x 8 B per row): the head rows (the first 2 kPreRows, read for
// every pair) through one resource over the rows that fit under 4 GiB, and the tail rows
// MODE 1: through one resource over the rows past the head (under 4 GiB; a tail row index
// is clamped to the property's last row and its word masked, so no offset passes the
// resource), or MODE 2: a resource per tail row, based at w + j * rowb, one row long or
// empty past the rows (any size; more scalar work per load: 3 % at 1M x 1M).
struct OpRes {
  rsrc_t len, x, w, t;
  const char* wb;
  uint32_t rowb, rows, xsh;
};

template <int MODE>
__device__ __forceinline__ OpRes op_res(const GroupedProp* gp, int p) {
  const GroupedProp G = gp[p];
  OpRes r;
  r.len = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(G.len), (short)0, (int)G.len_n, kRsrcWord3);
  r.x = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(G.x), (short)0, (int)G.x_n, kRsrcWord3);
  r.wb = static_cast<const char*>(G.w);
  r.rowb = G.rowb;
  r.rows = G.w_rows;
  r.w = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(G.w), (short)0, (int)(G.w_head * G.rowb), kRsrcWord3);
  if (MODE == 1)
    r.t = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(static_cast<const char*>(G.w) + (uint64_t)kGroupedHeadRows * G.rowb), (short)0,
        (int)G.w_tailb, kRsrcWord3);
  r.xsh = G.xsh;
  return r;
}

// head rows j < 2 kPreRows: the first resource, in either form
__device__ __forceinline__ uint64_t ld_row_head(const OpRes& R, int j, uint32_t g) {
  return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(R.w, g * 8u + (uint32_t)j * R.rowb, 0, 0));
}

// tail rows j >= kGroupedHeadRows
template <int MODE>
__device__ __forceinline__ uint64_t ld_row(const OpRes& R, int j, uint32_t g) {
  if (MODE == 0)
    return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(R.w, g * 8u + (uint32_t)j * R.rowb, 0, 0));
  if (MODE == 1) {
    const int jj = min(j, (int)R.rows - 1);
    const uint64_t v = __builtin_bit_cast(
        uint64_t, __builtin_amdgcn_raw_buffer_load_b64(R.t, g * 8u + (uint32_t)(jj - kGroupedHeadRows) * R.rowb, 0, 0));
    return j < (int)R.rows ? v : 0ull;
  }
  // the row's base and size are wave-uniform (readfirstlane keeps the resource in SGPRs: a
  // resource in VGPRs would make the load a waterfall loop)
  const uint64_t at = (uint64_t)(uintptr_t)R.wb + (uint64_t)(uint32_t)j * R.rowb;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)at);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(at >> 32));
  const uint32_t nb = __builtin_amdgcn_readfirstlane((uint32_t)j < R.rows ? R.rowb : 0u);
  const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>((uintptr_t)(((uint64_t)hi << 32) | lo)), (short)0, (int)nb, kRsrcWord3);
  return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(rs, g * 8u, 0, 0));
}

// property p's candidate operands at replica position g (lanes without a pair read
// position 0), all loads unconditional
__device__ __forceinline__ void load_ops(const OpRes& R, uint32_t g, bool valid, PreOps& o) {
  const uint32_t lc = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(R.len, g * 2u, 0, 0);
  o.lc = valid ? lc : (uint32_t)kMissing;
  o.x = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(R.x, g << R.xsh, 0, 0);
#pragma unroll
  for (int j = 0; j < kPreRows; ++j) o.w[j] = ld_row_head(R, j, g);
}

// |Q ∩ C| of one bigram key word (four 16-bit keys) against the query's perfect-hash table
__device__ __forceinline__ int probe_word(const uint32_t* tab, uint64_t w, uint32_t mult, int sh) {
  int c = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t key = (uint32_t)(w >> (16 * e)) & 0xFFFFu;
    c += tab[(uint32_t)__umul24(key, mult) >> sh] == key ? 1 : 0;
  }
  return c;
}

// A query without a perfect hash for this property (a set with the key-0 bigram, or none
// found in kGramSeedTries tries), or without grams.  Every set of the property has at most
// kMaxReplicaGrams grams (it has a key replica), so a merge of the two sorted code lists
// (the candidate's read in place) is short and needs no table.  Same result as k_score's
// generic QGram path: for m1 > 0, equal values have equal non-empty sets, whose formula
// is exactly 1.0, so only a query without grams (a value shorter than q) compares strings.
template <typename CT>
__device__ __forceinline__ double qgram_generic(const DevProp& D, uint64_t rstride, uint32_t q,
                                                uint32_t g, uint32_t crow, int m1, int lq, int lc,
                                                bool cmp) {
  if (!cmp) return 0.0;
  if (m1 == 0) {
    const CT* base = reinterpret_cast<const CT*>(D.units);
    const Str<CT> s1{reinterpret_cast<const uint32_t*>(base + D.off[q]), 1, 1 << 30};
    const Str<CT> s2 = D.rlmax ? Str<CT>{reinterpret_cast<const uint32_t*>(D.runits) + g, rstride,
                                         D.rlmax / Str<CT>::UPW - 1}
                               : Str<CT>{reinterpret_cast<const uint32_t*>(base + D.off[crow]), 1, 1 << 30};
    return str_equal(s1, lq, s2, lc) ? 1.0 : 0.0;
  }
  const int m2 = D.rgcnt[g];
  if (m2 == 0) return 0.0;
  const int common = intersect_sorted(D.grams + D.goff[q], m1, D.grams + D.rgoff[g], m2);
  return qgram_formula(common, m1, m2, D.formula);
}

// Candidate t of the query (its concatenated segment ranges) -> replica position.
struct Cand {
  uint32_t g;    // replica position (0 for a slot without a pair)
  int kf;        // key function of its segment
  bool valid;
};

// Execution order -> task.  The launch's tasks run in the order of their first candidate's
// replica position (perm, sorted per chunk by k_task_keys + a radix sort), so consecutive
// tasks read the same blocking bucket's replica rows; and blocks b, b+8, b+16, ... (one XCD
// under the round-robin dispatch, observed, not guaranteed: speed only) take consecutive
// stretches of that order, so a bucket's rows are re-read from one XCD's L2 instead of HBM.
__device__ __forceinline__ uint64_t grouped_task(const uint32_t* perm, uint64_t task0, uint64_t ntask,
                                                 uint32_t wave) {
  const uint64_t nb = gridDim.x, b = blockIdx.x;
  const uint64_t m = nb / 8;
  const uint64_t sb = b < 8 * m ? (b % 8) * m + b / 8 : b;
  const uint64_t e = sb * (kScoreBlock / 64) + wave;
  if (e >= ntask) return ~0ull;
  return perm ? (uint64_t)perm[task0 + e] - task0 : e;
}

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DK_WAVES_GROUPED, 8)))
void k_score_grouped(const ScoreParams P, const PairSource S, uint64_t slot0, uint64_t nslots,
                     const uint32_t* __restrict__ perm, const GroupedProp* __restrict__ gp,
                     StageOut out) {
  __shared__ uint32_t lds[kScoreBlock / 64][kGroupedTabs * kTabWords];
  __shared__ QueryVals qlds[kScoreBlock / 64][kMaxProps];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = lane_id();
  const uint64_t task = grouped_task(perm, slot0 / kScoreBlock, nslots / kScoreBlock, wave);
  if (task == ~0ull) return;  // the whole wave: no workgroup barrier follows
  uint32_t* tabs = lds[wave];
  QueryVals* qv = qlds[wave];

  // ---- the task's query (wave-uniform, scalar loads) ----
  const uint64_t sb = slot0 + task * kScoreBlock;
  const uint32_t qi = __builtin_amdgcn_readfirstlane(S.wq[sb >> 6]);
  const uint32_t q = __builtin_amdgcn_readfirstlane(S.queries[qi]);
  const uint64_t tbase = sb - S.qoff[qi];
  uint64_t total = 0;
  for (int k = 0; k < S.nseg; ++k) {
    const uint2 r = S.ranges[(uint64_t)k * S.nq + qi];
    total += r.y - r.x;
  }
  const uint64_t rest = (total - tbase + 63) >> 6;
  const int ngroups = rest < (uint64_t)kTaskGroups ? (int)rest : kTaskGroups;
  const uint64_t qident = P.ident[q];

  // candidate t -> (segment, position): key function k's range first, then (group, row)
  // order inside it (Duke's candidate order); filters: isSameAs (identity), a base
  // position superseded since the sort (kDeadIdent), and "already a candidate under an
  // earlier key function" (Duke returns a set).  The ranges are re-read per group from
  // the scalar cache rather than held in SGPRs.
  auto resolve = [&](int grp) -> Cand {
    uint64_t t = tbase + (uint64_t)grp * 64 + lane;
    Cand c{0u, 0, false};
    for (int k = 0; k < S.nseg; ++k) {
      const uint2 r = S.ranges[(uint64_t)k * S.nq + qi];
      const uint64_t len = r.y - r.x;
      if (!c.valid && t < len) {
        c.g = (uint32_t)(S.segoff[k] + r.x + t);
        c.kf = k >> S.seg_shift;
        c.valid = true;
      }
      t -= c.valid ? 0 : len;
    }
    return c;
  };
  // the filters' operands and the output row of a group's candidates (unconditional loads:
  // a key function past nkeys - 1 reads rident)
  auto load_filters = [&](const Cand& c, uint64_t& rid, uint64_t (&rk)[kPreKeys], uint32_t& crow) {
    rid = S.rident[c.g];
#pragma unroll
    for (int j = 0; j < kPreKeys; ++j) rk[j] = (j < S.nkeys - 1 ? S.rkeys[j] : S.rident)[c.g];
    crow = P.rowof[c.g];
  };

  // ---- the query's values in LDS, group 0 in flight, then the query's tables ----
  {
    // lane p < nprops reads property p's query values (pointers selected per lane: one
    // batch of loads, one wait)
    const uint16_t* plen = nullptr;
    const uint16_t* pgc = nullptr;
    const uint16_t* psd = nullptr;
    const uint8_t* pok = nullptr;
    const double* pnum = nullptr;
    for (int p = 0; p < P.nprops; ++p) {
      const DevProp& D = P.props[p];
      if ((int)lane == p) {
        plen = D.len;
        if (D.op == DK_CMP_QGRAM) { pgc = D.gcnt; psd = D.gseed; }
        if (D.op == DK_CMP_NUMERIC) { pok = D.numok; pnum = D.num; }
      }
    }
    if ((int)lane < P.nprops) {
      QueryVals v{};
      v.len = plen[q];
      v.gcnt = pgc ? pgc[q] : 0;
      v.seed = psd ? psd[q] : kGramSeedNone;
      v.numok = pok ? pok[q] : 0;
      v.num = pnum ? pnum[q] : 0.0;
      qv[lane] = v;
    }
  }
  // Processor.compare's visiting order for this query (its RecordImpl HashMap's order class)
  const uint64_t ow =
      order_word(P, P.norders > 1 ? (int)__builtin_amdgcn_readfirstlane((uint32_t)P.oclass[q]) : 0);
  Cand cn = resolve(0);
  uint64_t rid_n;
  uint64_t rk_n[kPreKeys];
  uint32_t crow_n;
  load_filters(cn, rid_n, rk_n, crow_n);
  PreOps nx;
  load_ops(op_res<MODE>(gp, order_at(ow, 0)), cn.g, cn.valid, nx);

  // the query's bigram sets in its perfect-hash tables (one per bigram property)
  for (int e = (int)lane * 4; e < kGroupedTabs * kTabWords; e += 256)
    *reinterpret_cast<uint4*>(tabs + e) = make_uint4(0u, 0u, 0u, 0u);
  wave_lds_sync();
  {
    int ts = 0;
    for (int p = 0; p < P.nprops; ++p) {
      const DevProp& D = P.props[p];
      if (D.op != DK_CMP_QGRAM) continue;
      const QueryVals v = qv[p];
      const uint32_t lq = __builtin_amdgcn_readfirstlane((uint32_t)v.len);
      const int m1 = (int)__builtin_amdgcn_readfirstlane((uint32_t)v.gcnt);
      const uint32_t sd = __builtin_amdgcn_readfirstlane((uint32_t)v.seed);
      if (lq != kMissing && m1 > 0 && sd != kGramSeedNone) {
        uint32_t* tab = tabs + ts * kTabWords;
        const uint32_t mult = gram_mult(sd & 0xFFu);
        const int sh = 32 - kGramLtMin - (int)(sd >> 8);  // 32 - lt
        if (lane == 0) tab[0] = ~0u;  // a real key landing in slot 0 overwrites the sentinel
        if ((int)lane < m1) {
          const uint32_t key = gram_key(D.grams[D.goff[q] + lane]);
          tab[(uint32_t)__umul24(key, mult) >> sh] = key;
        }
      }
      ++ts;
    }
  }
  wave_lds_sync();

  uint32_t cnt = 0, scored = 0, bytes = 0;
  const uint64_t blk = task;  // staging block of the task (k_compact: block order = slot order)
  for (int grp = 0; grp < ngroups; ++grp) {
    const Cand c = cn;
    const uint64_t rid = rid_n;
    uint64_t rk[kPreKeys];
#pragma unroll
    for (int j = 0; j < kPreKeys; ++j) rk[j] = rk_n[j];
    const uint32_t crow = crow_n;
    bool valid = c.valid && rid != qident && rid != kDeadIdent;
#pragma unroll
    for (int j = 0; j < kPreKeys; ++j)
      if (j < S.nkeys - 1 && j < c.kf) valid = valid && rk[j] != S.qkeys[j][q];
    for (int j = kPreKeys; j < S.nkeys - 1; ++j)  // more than kPreKeys + 1 key functions
      if (j < c.kf) valid = valid && S.rkeys[j][c.g] != S.qkeys[j][q];

    double prob = 0.5;
    uint32_t by = valid ? 9u : 0u;  // two row ids + decision (SURVEY §8d B_pair)
    for (int k = 0; k < P.nprops; ++k) {
      const int p = order_at(ow, k);
      const DevProp& D = P.props[p];
      const PreOps o = nx;
      const bool isq = D.op == DK_CMP_QGRAM;
      const QueryVals v = qv[p];
      const uint32_t lq = __builtin_amdgcn_readfirstlane((uint32_t)v.len);
      const int m1 = (int)__builtin_amdgcn_readfirstlane((uint32_t)v.gcnt);
      const uint32_t sd = __builtin_amdgcn_readfirstlane((uint32_t)v.seed);
      const int lc = (int)o.lc;
      const bool present = valid && lc != (int)kMissing;
      const bool cmp = present && lq != kMissing && lq > 0 && lc > 0;
      const bool perfect = isq && lq != kMissing && m1 > 0 && sd != kGramSeedNone;  // wave-uniform
      // rows kPreRows .. 2 kPreRows - 1 of this property, issued before the next step's
      // prefetch (loads complete in order: waiting for these then never waits for that)
      const int m2 = cmp ? (int)(o.x & 0xFFu) : 0;
      const int njw = perfect ? wave_max_i32((m2 + 3) >> 2) : 0;  // key-word rows the wave needs
      const OpRes R = op_res<MODE>(gp, p);
      uint64_t ex[kPreRows];
      if (njw > kPreRows) {
#pragma unroll
        for (int j = 0; j < kPreRows; ++j) ex[j] = ld_row_head(R, kPreRows + j, c.g);
      }
      // the next step's operands: property p+1 of this group, or the next group's
      // positions, filters and property 0
      if (k + 1 < P.nprops) {
        load_ops(op_res<MODE>(gp, order_at(ow, k + 1)), c.g, c.valid, nx);
      } else if (grp + 1 < ngroups) {
        cn = resolve(grp + 1);
        load_filters(cn, rid_n, rk_n, crow_n);
        load_ops(op_res<MODE>(gp, order_at(ow, 0)), cn.g, cn.valid, nx);
      }
      const int tslot = (int)gp[p].tslot;
      if (lq == kMissing) continue;  // r1 has no value: property skipped for the wave
      double sim = 0.0;
      if (present) by += 2u;  // rlen
      if (D.op == DK_CMP_NUMERIC) {
        if (cmp) {
          sim = numeric(v.num, v.numok != 0, __builtin_bit_cast(double, o.w[0]), o.x != 0u, D.min_ratio);
          by += 9u;  // rnum + rnumok
        }
      } else if (isq) {
        if (perfect) {
          // no string compare: equal values have equal non-empty gram sets, for which every
          // formula is exactly 1.0
          const uint32_t* tab = tabs + tslot * kTabWords;
          const uint32_t mult = gram_mult(sd & 0xFFu);
          const int sh = 32 - kGramLtMin - (int)(sd >> 8);
          int common = 0;
#pragma unroll
          for (int j = 0; j < kPreRows; ++j)
            if (j < njw) common += probe_word(tab, o.w[j], mult, sh);
          if (njw > kPreRows) {
#pragma unroll
            for (int j = 0; j < kPreRows; ++j)
              if (kPreRows + j < njw) common += probe_word(tab, ex[j], mult, sh);
            // longer sets: the rest DK_GROUPED_TAIL rows at a time (loads issued together;
            // rows past the property's rows are out of range, free)
            for (int j = 2 * kPreRows; j < njw; j += kTailRows) {
              uint64_t w[kTailRows];
#pragma unroll
              for (int i = 0; i < kTailRows; ++i) w[i] = ld_row<MODE>(R, j + i, c.g);
#pragma unroll
              for (int i = 0; i < kTailRows; ++i)
                if (j + i < njw) common += probe_word(tab, w[i], mult, sh);
            }
          }
          if (m2 > 0) sim = qgram_formula(common, m1, m2, D.formula);
        } else {  // g16 properties have a width-1 arena
          sim = qgram_generic<uint8_t>(D, P.rstride, q, c.g, crow, m1, (int)lq, lc, cmp);
        }
        if (cmp) by += 6u + 2u * (o.x & 0xFFu);  // rgoff + rgcnt + the candidate's 16-bit keys
      }
      if (present) {
        // [Duke 1.2] Processor.compare: high = max(0.0, PropertyImpl.compare), then
        // computeBayes
        prob = compute_bayes(prob, cmp ? property_prob(D, sim) : 0.0);
      }
    }

    // [Duke 1.2] Processor.compareCandidatesSimple; block-ordered compaction within the task
    const uint32_t kind = valid ? decide(prob, P.threshold, P.maybe) : 0u;
    const uint64_t em = __ballot(kind != 0u);
    if (kind != 0u) {
      const uint64_t e = blk * kScoreBlock + cnt + mask_rank(em);
      out.prob[e] = prob;
      out.cand[e] = crow | (kind << kKindShift);
      out.qidx[e] = qi;
    }
    cnt += (uint32_t)__popcll(em);
    scored += valid ? 1u : 0u;
    bytes += by;
  }
  const uint32_t ss = wave_sum_u32(scored), sbytes = wave_sum_u32(bytes);
  if (lane == 0) {
    out.bcnt[blk] = cnt;
    out.bscored[blk] = ss;
    out.bbytes[blk] = sbytes;
  }
}

hipError_t launch_score_grouped(const ScoreParams& P, const PairSource& src, uint64_t slot0,
                                uint64_t nslots, const uint32_t* perm, const GroupedProp* gp,
                                int mode, const StageOut& out, hipStream_t s) {
  if (nslots == 0) return hipSuccess;
  if (nslots % kScoreBlock || slot0 % kScoreBlock) return hipErrorInvalidValue;
  const uint64_t ntask = nslots / kScoreBlock;
  const uint64_t grid = (ntask + kScoreBlock / 64 - 1) / (kScoreBlock / 64);
  if (mode == 2) k_score_grouped<2><<<(unsigned)grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, perm, gp, out);
  else if (mode == 1) k_score_grouped<1><<<(unsigned)grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, perm, gp, out);
  else k_score_grouped<0><<<(unsigned)grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, perm, gp, out);
  return hipGetLastError();
}

// =======================================================================================
// k_score_gq<NQ, NN> (round 5): k_score_grouped's schemas on a schedule with ONE memory
// round trip per group of 64 candidates instead of one per property plus one or two for the
// key-word rows past the first two.  k_score_grouped<1> at configs[2] 10M x 10M spent 0.53
// of its wave cycles waiting (rows 2-3 of each QGram property were loaded when the
// property began, rows 4+ one batch later behind the next property's prefetch, and a
// Numeric property's compute was too short to cover the next one's loads), and issued
// nearly as many scalar instructions as vector ones (the per-property operand sources
// rebuilt per group from a runtime property index).  Here:
//  * Properties are ROLES of a fixed kind (NQ bigram QGram, NN Numeric; GQArgs), unrolled
//    at compile time: every per-role constant sits at a fixed offset, and the HashMap
//    visiting order only selects which role's probability enters computeBayes next (a
//    uniform branch), after all roles are computed.
//  * The FRONT of group g+1 (candidate positions and gram counts: what the row loads need)
//    is loaded while group g computes; at group g's start its BACK operands -- every
//    key-word row each lane needs (per-lane offsets past the lane's own rows are out of
//    range: no data moved), lengths, filters, Numeric values -- are issued in one batch.
//  * The waves of a SIMD (DK_WAVES_GQ) cover that one round trip.
// =======================================================================================
#ifndef DK_WAVES_GQ
#define DK_WAVES_GQ 8  // k_score_gq waves per SIMD (<= 64 VGPRs; 15 KB LDS per 4 waves; 7 -> 8: configs[2] 1M ms_score 8.50 -> 8.20)
#endif
#ifndef DK_GQ_ABL
#define DK_GQ_ABL 0  // timing ablations only (wrong results): 1 probes, 2 f64 math, 4 row traffic
#endif
#ifndef DK_GQ_GUARD
#define DK_GQ_GUARD 0  // 1: probe a register row only when some lane has it (uniform branches: the
                       // ballot masks then cost SGPRs and every probe its own LDS wait)
#endif
#ifndef DK_GQ_ROWS0
#define DK_GQ_ROWS0 5  // key-word rows held in registers: QGram role 0 (24 grams)
#endif
#ifndef DK_GQ_ROWS1
#define DK_GQ_ROWS1 8  // role 1 (36 grams); longer sets read the rest in batches of 4
#endif

template <int A>
struct GQRows {
  static constexpr int v = A == 0 ? DK_GQ_ROWS0 : DK_GQ_ROWS1;
};

// element i of a global array whose pointer was read from memory (GQArgs): a generic
// pointer would make it a FLAT load, which the wait-count pass cannot order against the
// buffer loads in flight (every later wait becomes vmcnt(0))
template <typename T>
__device__ __forceinline__ T gq_ld(const T* p, uint32_t i) {
  return ((const __attribute__((address_space(1))) T*)(p))[i];
}
template <typename T>
__device__ __forceinline__ void gq_st(T* p, uint64_t i, T v) {
  ((__attribute__((address_space(1))) T*)(p))[i] = v;
}

using GQLds = const __attribute__((address_space(3))) GQArgs;

// The launch's GQArgs as this wave's LDS copy, through an address the compiler cannot prove
// loop-invariant: per-group reads are LDS reads (no vector-memory wait, no scalar registers
// held -- and spilled -- across the group loop); uniform values are made scalar at their use
__device__ __forceinline__ GQLds* gq_hdr(GQLds* h) {
  uint32_t v = (uint32_t)(uintptr_t)h;
  asm volatile("" : "+v"(v));
  return (GQLds*)(uintptr_t)v;
}
template <typename T>
__device__ __forceinline__ T* gq_uptr(T* p) {  // a uniform pointer (VGPR copy) -> scalar
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<T*>(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t gq_u(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ rsrc_t gq_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, kRsrcWord3);
}


// |Q ∩ C| of one key word against a table of 16-bit entries (k_score_gq): the same slots
// as probe_word, half the LDS
__device__ __forceinline__ int probe_word16(const uint16_t* tab, uint64_t w, uint32_t mult, int sh) {
  int c = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t key = (uint32_t)(w >> (16 * e)) & 0xFFFFu;
    c += (uint32_t)tab[(uint32_t)__umul24(key, mult) >> sh] == key ? 1 : 0;
  }
  return c;
}

// the query's values of one role (wave-uniform), staged in LDS once per task
struct GQQuery {
  uint16_t len, m1, seed;  // QGram: grams, perfect-hash seed
  uint8_t ok, pad;         // Numeric: parsed
  double num;              // Numeric: value
};
static_assert(sizeof(GQQuery) == 16, "one ds_read_b128");
static_assert(sizeof(GQArgs) % 16 == 0, "GQArgs copied to LDS in 16-B pieces");

template <int NQ, int NN, int DEF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DEF < 0 && NQ == 2 ? DK_WAVES_GQ - 2 : DK_WAVES_GQ, 8)))
void k_score_gq(const ScoreParams P, const PairSource S, uint64_t slot0, uint64_t nslots,
                const uint32_t* __restrict__ perm, const GQArgs* __restrict__ A, StageOut out) {
  constexpr int NR = NQ + NN;
  constexpr int NQ1 = NQ > 0 ? NQ : 1, NN1 = NN > 0 ? NN : 1, NR1 = NR > 0 ? NR : 1;
  static_assert(DEF < NQ, "the deferred role is a QGram role");
  // per QGram role a table of 512 16-bit slots (a key, 0 = empty; slot 0 starts with a
  // sentinel key that hashes elsewhere, so neither a padding key 0 nor any other key that
  // lands on slot 0 finds it)
  __shared__ uint16_t lds[kScoreBlock / 64][kGroupedTabs * kTabWords];
  __shared__ uint64_t queue_lds[kScoreBlock / 64][kGQQueue];
  __shared__ GQQuery qlds[kScoreBlock / 64][kGroupedTabs + kGQMaxNum];
  __shared__ uint2 slds[kScoreBlock / 64][kMaxSegs];  // per segment: {first position, length}
  __shared__ GQArgs hlds[kScoreBlock / 64];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = lane_id();
  const uint64_t task = grouped_task(perm, slot0 / kScoreBlock, nslots / kScoreBlock, wave);
  if (task == ~0ull) return;  // the whole wave: no workgroup barrier follows
  uint16_t* tabs = lds[wave];
  GQQuery* qv = qlds[wave];
  uint2* seg = slds[wave];
  uint64_t* queue = queue_lds[wave];
  for (int e = (int)lane; e < (int)(sizeof(GQArgs) / 16); e += 64)
    reinterpret_cast<uint4*>(&hlds[wave])[e] = reinterpret_cast<const uint4*>(A)[e];
  GQLds* const hdr0 = (GQLds*)&hlds[wave];

  // ---- the task's query: its segment ranges in LDS (the group loop then reads no uniform
  //      value from global memory: a vector load there would wait for every row in flight) ----
  const uint64_t sb = slot0 + task * kScoreBlock;
  const uint32_t qi = __builtin_amdgcn_readfirstlane(S.wq[sb >> 6]);
  const uint32_t q = __builtin_amdgcn_readfirstlane(S.queries[qi]);
  const uint64_t tbase = sb - S.qoff[qi];
  const int nseg = S.nseg;
  uint32_t slen = 0;
  if ((int)lane < nseg) {
    const uint2 r = S.ranges[(uint64_t)lane * S.nq + qi];
    slen = r.y - r.x;
    uint64_t so = 0;
    for (int k = 0; k < nseg; ++k)
      if (k == (int)lane) so = S.segoff[k];
    seg[lane] = make_uint2((uint32_t)(so + r.x), slen);
  }
  const uint64_t total = wave_sum_u32(slen);
  const uint64_t rest = (total - tbase + 63) >> 6;
  const int ngroups = rest < (uint64_t)kTaskGroups ? (int)rest : kTaskGroups;
  const uint64_t qident = P.ident[q];
  const uint64_t qk0 = S.nkeys > 1 ? S.qkeys[0][q] : 0ull;
  const int seg_shift = S.seg_shift;
  const int nkeys = S.nkeys;

  // candidate t of the query -> (segment, position), as k_score_grouped; the FRONT of a
  // group: its positions (kf << 1 | pair in fk) and the QGram roles' gram counts
  auto load_front = [&](GQLds* H, int grp, uint32_t& g, uint32_t& fk, uint32_t (&cq)[NQ1]) {
    uint32_t t = (uint32_t)(tbase + (uint64_t)grp * 64) + lane;  // a task's t < 2^32
    bool v = false;
    g = 0u;
    fk = 0u;
    for (int k = 0; k < nseg; ++k) {
      const uint2 r = seg[k];
      if (!v && t < r.y) {
        g = r.x + t;
        fk = (uint32_t)(k >> seg_shift) << 1 | 1u;
        v = true;
      }
      t -= v ? 0u : r.y;
    }
#pragma unroll
    for (int a = 0; a < NQ; ++a) cq[a] = gq_ld(gq_uptr(H->q[a].rgcnt), g) & 0xFFu;
  };

  // lane r < NR stages role r's query values in LDS (one batch of loads, one wait)
  if ((int)lane < NR) {
    const int r = (int)lane;
    const DevProp& D = P.props[r < NQ ? A->q[r].prop : A->n[r - NQ].prop];
    GQQuery v{};
    v.len = D.len[q];
    if (r < NQ) {
      v.m1 = D.gcnt[q];
      v.seed = D.gseed[q];
      v.pad = (uint8_t)D.formula;
    } else {
      v.ok = D.numok[q];
      v.num = D.num[q];
    }
    qv[r] = v;
  }
  // Processor.compare's visiting order for this query, as roles (this wave's header copy:
  // re-read per group, like the rest of it)
  {
    const uint64_t ro = A->rorder[P.norders > 1 ? (int)__builtin_amdgcn_readfirstlane((uint32_t)P.oclass[q]) : 0];
    if (lane == 0) hlds[wave].rorder[0] = ro;
  }
  for (int e = (int)lane * 8; e < NQ * kTabWords; e += 512)
    *reinterpret_cast<uint4*>(tabs + e) = make_uint4(0u, 0u, 0u, 0u);
  wave_lds_sync();
  uint32_t gn, fkn, cqn[NQ1];
  load_front(hdr0, 0, gn, fkn, cqn);
  // the query's bigram sets in its perfect-hash tables (table a = QGram role a)
#pragma unroll
  for (int a = 0; a < NQ; ++a) {
    const GQQuery v = qv[a];
    const uint32_t sd = __builtin_amdgcn_readfirstlane((uint32_t)v.seed);
    const uint32_t m1 = __builtin_amdgcn_readfirstlane((uint32_t)v.m1);
    if (__builtin_amdgcn_readfirstlane((uint32_t)v.len) != kMissing && m1 > 0 && sd != kGramSeedNone) {
      uint16_t* tab = tabs + a * kTabWords;
      const DevProp& D = P.props[A->q[a].prop];
      const uint32_t mult = gram_mult(sd & 0xFFu);
      const int sh = 32 - kGramLtMin - (int)(sd >> 8);
      // the sentinel: the smallest key in 1..64 whose slot is not 0
      const uint64_t off0 = __ballot(((uint32_t)__umul24(lane + 1u, mult) >> sh) != 0u);
      if (off0 == 0ull) {
        if (lane == 0) qv[a].seed = kGramSeedNone;  // (no such key: the sorted-list path)
      } else {
        if (lane == 0) tab[0] = (uint16_t)(__builtin_ctzll(off0) + 1);  // a real key in slot 0 overwrites it
        if (lane < m1) {
          const uint32_t key = gram_key(D.grams[D.goff[q] + lane]);
          tab[(uint32_t)__umul24(key, mult) >> sh] = (uint16_t)key;
        }
      }
    }
  }
  wave_lds_sync();

  uint32_t cnt = 0, scored = 0, bytes = 0, nexact = 0;
  const uint64_t blk = task;  // staging block of the task (k_compact: block order = slot order)

  // the query's role constants (LDS, uniform)
  auto query_roles = [&](uint32_t (&qlen)[NR1], bool (&perfect)[NQ1], uint32_t (&m1)[NQ1], uint32_t (&sd)[NQ1]) {
#pragma unroll
    for (int r = 0; r < NR; ++r) qlen[r] = gq_u((uint32_t)qv[r].len);
#pragma unroll
    for (int a = 0; a < NQ; ++a) {
      m1[a] = gq_u((uint32_t)qv[a].m1);
      sd[a] = gq_u((uint32_t)qv[a].seed);
      perfect[a] = qlen[a] != kMissing && m1[a] > 0 && sd[a] != kGramSeedNone;
    }
  };
  // key-word rows [0, GQRows<a>) of role a at position g, nw of them in range (one batch)
  auto issue_rows = [&](GQLds* H, auto ic, uint32_t g, uint32_t nw, uint64_t* w) {
    constexpr int a = decltype(ic)::value;
    const rsrc_t rh = gq_rsrc(gq_uptr(H->q[a].rows), gq_u(H->q[a].head_bytes));
    const rsrc_t rt = gq_rsrc(gq_uptr(H->q[a].tail), gq_u(H->q[a].tail_bytes));
    const uint32_t rowb = gq_u(H->q[a].rowb);
    const uint32_t g8 = g * 8u;
#pragma unroll
    for (int j = 0; j < GQRows<a>::v; ++j) {
      const uint32_t off = g8 + (uint32_t)(j < kGroupedHeadRows ? j : j - kGroupedHeadRows) * rowb;
      const uint32_t o = (DK_GQ_ABL & 4) ? 0xFFFFFFFFu : (uint32_t)j < nw ? off : 0xFFFFFFFFu;
      w[j] = __builtin_bit_cast(uint64_t,
                                __builtin_amdgcn_raw_buffer_load_b64(j < kGroupedHeadRows ? rh : rt, o, 0, 0));
    }
  };
  // |Q ∩ C| of role a: the rows held in registers, then the rest kTailRows at a time
  auto role_common = [&](GQLds* H, auto ic, uint32_t g, uint32_t nw, uint32_t sdv, const uint64_t* w) -> int {
    constexpr int a = decltype(ic)::value;
    const uint16_t* tab = tabs + a * kTabWords;
    const uint32_t mult = gram_mult(sdv & 0xFFu);
    const int sh = 32 - kGramLtMin - (int)(sdv >> 8);  // 32 - lt
    int common = 0;
#pragma unroll
    for (int j = 0; j < GQRows<a>::v; ++j)
      if (!DK_GQ_GUARD || __builtin_amdgcn_ballot_w64((uint32_t)j < nw))  // uniform: a lane has row j
        if (!(DK_GQ_ABL & 1)) common += probe_word16(tab, w[j], mult, sh);
    if (__builtin_amdgcn_ballot_w64(nw > (uint32_t)GQRows<a>::v)) {
      const rsrc_t rt = gq_rsrc(gq_uptr(H->q[a].tail), gq_u(H->q[a].tail_bytes));
      const uint32_t rowb = gq_u(H->q[a].rowb);
      const int nrows = (int)gq_u(H->q[a].nrows);
      const uint32_t g8 = g * 8u;
      for (int j = GQRows<a>::v; j < nrows; j += kTailRows) {
        uint64_t wt[kTailRows];
#pragma unroll
        for (int i = 0; i < kTailRows; ++i) {
          const uint32_t off = g8 + (uint32_t)(j + i - kGroupedHeadRows) * rowb;
          wt[i] = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(
                                                   rt, (uint32_t)(j + i) < nw ? off : 0xFFFFFFFFu, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < kTailRows; ++i) common += probe_word16(tab, wt[i], mult, sh);
        if (!__builtin_amdgcn_ballot_w64(nw > (uint32_t)(j + kTailRows))) break;
      }
    }
    return common;
  };

  // ---- EXACT pass over queued pairs (lanes < n hold queue entries head..head+n-1, in
  //      candidate order): the deferred role's rows and probes, every role's probability
  //      in double precision, computeBayes in the visiting order, the decision, emission ----
  auto exact = [&](uint32_t head, uint32_t n) {
    GQLds* const H = gq_hdr(hdr0);
    const bool act = lane < n;
    nexact += n;
    const uint64_t ent = act ? queue[(head + lane) & (kGQQueue - 1)] : 0ull;
    const uint32_t g = (uint32_t)ent;
    uint32_t qlen[NR1], m1[NQ1], sd[NQ1];
    bool perfect[NQ1];
    query_roles(qlen, perfect, m1, sd);
    int common[NQ1];
    uint32_t cq[NQ1];
#pragma unroll
    for (int a = 0; a < NQ; ++a) {
      common[a] = (int)((ent >> (32 + 8 * a)) & 0xFFu);
      cq[a] = (uint32_t)((ent >> (48 + 8 * a)) & 0xFFu);
    }
    uint64_t wd[DEF >= 0 ? GQRows<DEF < 0 ? 0 : DEF>::v : 1];
    const uint32_t nwd = DEF >= 0 && act && perfect[DEF < 0 ? 0 : DEF] ? (cq[DEF < 0 ? 0 : DEF] + 3u) >> 2 : 0u;
    if constexpr (DEF >= 0) issue_rows(H, std::integral_constant<int, DEF < 0 ? 0 : DEF>{}, g, nwd, wd);
    const uint32_t crow = gq_ld(gq_uptr(H->rowof), g);
    uint32_t lq[NQ1], ln[NN1], cok[NN1];
    double cn[NN1];
#pragma unroll
    for (int a = 0; a < NQ; ++a) lq[a] = gq_ld(gq_uptr(H->q[a].rlen), g);
#pragma unroll
    for (int b = 0; b < NN; ++b) {
      ln[b] = gq_ld(gq_uptr(H->n[b].rlen), g);
      cn[b] = gq_ld(gq_uptr(H->n[b].rnum), g);
      cok[b] = gq_ld(gq_uptr(H->n[b].rnumok), g);
    }
    if constexpr (DEF >= 0)
      if (perfect[DEF < 0 ? 0 : DEF]) common[DEF < 0 ? 0 : DEF] = role_common(H, std::integral_constant<int, DEF < 0 ? 0 : DEF>{}, g, nwd, sd[DEF < 0 ? 0 : DEF], wd);
    // algorithmic bytes: the deferred role's candidate keys, read by this pass only
    if constexpr (DEF >= 0)
      if (act && lq[DEF < 0 ? 0 : DEF] != kMissing && lq[DEF < 0 ? 0 : DEF] > 0 && qlen[DEF < 0 ? 0 : DEF] > 0 &&
          qlen[DEF < 0 ? 0 : DEF] != kMissing)
        bytes += 2u * cq[DEF < 0 ? 0 : DEF];
    double pp[NR1];
    bool ap[NR1];
#pragma unroll
    for (int a = 0; a < NQ; ++a) {
      const bool present = act && lq[a] != kMissing;
      const bool cmp = present && lq[a] > 0 && qlen[a] > 0;
      double sim = 0.0;
      if (qlen[a] != kMissing) {
        if (perfect[a]) {
          const int m2 = cmp ? (int)cq[a] : 0;
          if (m2 > 0) sim = (DK_GQ_ABL & 2) ? (double)common[a] * 0.015625 : qgram_formula(common[a], (int)m1[a], m2, (int)gq_u(qv[a].pad));
        } else {  // no perfect hash for the query: the sorted lists (rare), as k_score_grouped
          const DevProp& D = P.props[gq_u((uint32_t)H->q[a].prop)];
          sim = qgram_generic<uint8_t>(D, P.rstride, q, g, crow, (int)m1[a], (int)qlen[a], (int)lq[a], cmp);
        }
      }
      pp[a] = cmp ? gq_prob(H->q[a].low, H->q[a].high, sim) : 0.0;
      ap[a] = present;
    }
#pragma unroll
    for (int b = 0; b < NN; ++b) {
      const bool present = act && ln[b] != kMissing;
      const bool cmp = present && ln[b] > 0 && qlen[NQ + b] > 0;
      double sim = 0.0;
      if (qlen[NQ + b] != kMissing && cmp) {
        const GQQuery v = qv[NQ + b];
        sim = (DK_GQ_ABL & 2) ? cn[b] * v.num : numeric(v.num, v.ok != 0, cn[b], cok[b] != 0u, H->n[b].min_ratio);
      }
      pp[NQ + b] = cmp ? gq_prob(H->n[b].low, H->n[b].high, sim) : 0.0;
      ap[NQ + b] = present;
    }
    // [Duke 1.2] Processor.compare: per property of r1 in its HashMap order, skipping those
    // r1 or r2 has no value of, prob = computeBayes(prob, max(0.0, PropertyImpl.compare))
    double prob = 0.5;
    const uint64_t ro = ((uint64_t)gq_u((uint32_t)(H->rorder[0] >> 32)) << 32) | gq_u((uint32_t)H->rorder[0]);
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const uint32_t r = (uint32_t)(ro >> (4 * k)) & 15u;
      const int ri = r >= 8u ? NQ + (int)(r - 8u) : (int)r;  // wave-uniform
      double x = 0.5;
      bool use = false;
#pragma unroll
      for (int i = 0; i < NR; ++i)
        if (ri == i) {
          x = pp[i];
          use = qlen[i] != kMissing && ap[i];
        }
      const double nb = (DK_GQ_ABL & 2) ? prob * x : compute_bayes(prob, x);
      prob = use ? nb : prob;
    }
    // [Duke 1.2] Processor.compareCandidatesSimple; block-ordered compaction within the task
    const uint32_t kind = act ? decide(prob, H->threshold, H->maybe) : 0u;
    const uint64_t em = __ballot(kind != 0u);
    if (kind != 0u) {
      const uint64_t e = blk * kScoreBlock + cnt + mask_rank(em);
      gq_st(gq_uptr(H->oprob), e, prob);
      gq_st(gq_uptr(H->ocand), e, crow | (kind << kKindShift));
      gq_st(gq_uptr(H->oqidx), e, qi);
    }
    cnt += (uint32_t)__popcll(em);
  };

  // ---- SCREEN pass, per group of 64 candidates: the non-deferred QGram roles' counts and
  //      the Numeric roles, then a single-precision upper bound of the pair's probability
  //      (the deferred role at its maximum); the pairs whose bound can reach the list go to
  //      the queue, the exact pass takes 64 of them at a time ----
  uint32_t qn = 0, qh = 0;  // queue: pushed, taken
  for (int grp = 0; grp < ngroups; ++grp) {
    GQLds* const H = gq_hdr(hdr0);
    const uint32_t g = gn, fk = fkn;
    uint32_t cq[NQ1];
#pragma unroll
    for (int a = 0; a < NQ; ++a) cq[a] = cqn[a];
    const bool pair = (fk & 1u) != 0u;
    uint32_t qlen[NR1], m1[NQ1], sd[NQ1];
    bool perfect[NQ1];
    query_roles(qlen, perfect, m1, sd);

    // ---- back operands, one batch: key-word rows of the screened roles, lengths, filters,
    //      Numeric values ----
    uint32_t nw[NQ1];
#pragma unroll
    for (int a = 0; a < NQ; ++a) nw[a] = a != DEF && pair && perfect[a] ? (cq[a] + 3u) >> 2 : 0u;
    uint64_t w0[DEF == 0 ? 1 : GQRows<0>::v];
    uint64_t w1[DEF == 1 ? 1 : GQRows<1>::v];
    if constexpr (NQ > 0 && DEF != 0) issue_rows(H, std::integral_constant<int, 0>{}, g, nw[0], w0);
    if constexpr (NQ > 1 && DEF != 1) issue_rows(H, std::integral_constant<int, 1>{}, g, nw[1], w1);
    const uint64_t rid = gq_ld(gq_uptr(H->rident), g);
    const uint64_t rk = nkeys > 1 && fk > 1u ? gq_ld(gq_uptr(H->rkey0), g) : 0ull;
    uint32_t lq[NQ1], ln[NN1], cok[NN1];
    double cn[NN1];
#pragma unroll
    for (int a = 0; a < NQ; ++a) lq[a] = gq_ld(gq_uptr(H->q[a].rlen), g);
#pragma unroll
    for (int b = 0; b < NN; ++b) {
      ln[b] = gq_ld(gq_uptr(H->n[b].rlen), g);
      cn[b] = gq_ld(gq_uptr(H->n[b].rnum), g);
      cok[b] = gq_ld(gq_uptr(H->n[b].rnumok), g);
    }
    // the next group's front (past the last group: position 0, no pair)
    load_front(H, grp + 1, gn, fkn, cqn);

    // ---- filters: Processor.isSameAs, a superseded base position, a candidate already
    //      returned under an earlier key function (Duke's candidate set) ----
    const int kf = (int)(fk >> 1);
    bool valid = pair && rid != qident && rid != kDeadIdent;
    if (kf > 0) valid = valid && rk != qk0;
    for (int j = 1; j < nkeys - 1; ++j)  // more than two key functions
      if (j < kf) valid = valid && S.rkeys[j][g] != S.qkeys[j][q];

    // ---- the bound: odds = prod x / (1 - x) over the roles applied (the HashMap order does
    //      not change the product); a role whose bound is outside [kScreenLo, kScreenHi]
    //      (where single precision is not enough, or Bayes is not monotone) sends the pair on ----
    uint32_t by = valid ? 9u : 0u;  // two row ids + decision (SURVEY §8d B_pair)
    float odds = 1.0f;
    bool wide = false;
    int common[NQ1];
#pragma unroll
    for (int a = 0; a < NQ; ++a) common[a] = 0;
    auto screen_x = [&](float x) {
      if (!(x >= kScreenLo && x <= kScreenHi)) wide = true;
      else odds *= x * __builtin_amdgcn_rcpf(1.0f - x);
    };
    auto screen_role = [&](auto ic, const uint64_t* w) {
      constexpr int a = decltype(ic)::value;
      if (qlen[a] == kMissing) return;
      const bool present = valid && lq[a] != kMissing;
      const bool cmp = present && lq[a] > 0 && qlen[a] > 0;
      if (present) by += 2u;
      if (cmp) by += 6u + (a == DEF ? 0u : 2u * cq[a]);  // the deferred role's keys: the exact pass
      if constexpr (a != DEF)
        if (perfect[a]) common[a] = role_common(H, ic, g, nw[a], sd[a], w);
      if (!present) return;
      float x;
      if (!cmp) {
        x = 0.0f;
      } else if (a == DEF || !perfect[a] || cq[a] == 0u) {
        x = cq[a] == 0u && perfect[a] ? H->q[a].flow0 : H->q[a].fub;
      } else {  // sim in [s (1 - 1e-5), s (1 + 1e-5)]: the f32 quotient is within 2 ulp
        const int f = (int)gq_u(qv[a].pad);
        const float c = (float)common[a], fm1 = (float)m1[a], fm2 = (float)cq[a];
        const float num = f == DK_QGRAM_DICE ? 2.0f * c : c;
        const float den = f == DK_QGRAM_JACCARD ? fm1 + fm2 - c : f == DK_QGRAM_DICE ? fm1 + fm2 : fminf(fm1, fm2);
        const float sm = num * __builtin_amdgcn_rcpf(den);
        const float slo = sm * (1.0f - 1e-5f), shi = sm * (1.0f + 1e-5f);
        const float hi5 = H->q[a].fhigh - 0.5f;
        float xb = slo < 0.5f ? H->q[a].flow : -1.0f;
        if (shi >= 0.5f) {
          const float s0 = fmaxf(slo, 0.5f);
          xb = fmaxf(xb, fmaxf(hi5 * (s0 * s0) + 0.5f, hi5 * (shi * shi) + 0.5f));
        }
        x = fmaxf(xb, 0.0f);
      }
      screen_x(x);
    };
    if constexpr (NQ > 0) screen_role(std::integral_constant<int, 0>{}, w0);
    if constexpr (NQ > 1) screen_role(std::integral_constant<int, 1>{}, w1);
#pragma unroll
    for (int b = 0; b < NN; ++b) {
      if (qlen[NQ + b] == kMissing) continue;
      const bool present = valid && ln[b] != kMissing;
      const bool cmp = present && ln[b] > 0 && qlen[NQ + b] > 0;
      if (present) by += 2u;
      if (!present) continue;
      float x = 0.0f;
      if (cmp) {
        by += 9u;  // rnum + rnumok
        const GQQuery v = qv[NQ + b];
        x = (float)gq_prob(H->n[b].low, H->n[b].high,
                           numeric(v.num, v.ok != 0, cn[b], cok[b] != 0u, H->n[b].min_ratio));
      }
      screen_x(x);
    }
    const bool pass = valid && (wide || odds >= H->screen);
    const uint64_t pm = __ballot(pass);
    if (pass) {
      uint64_t ent = (uint64_t)g;
#pragma unroll
      for (int a = 0; a < NQ; ++a) ent |= (uint64_t)((uint32_t)common[a] & 0xFFu) << (32 + 8 * a) | (uint64_t)cq[a] << (48 + 8 * a);
      queue[(qn + mask_rank(pm)) & (kGQQueue - 1)] = ent;
    }
    qn += (uint32_t)__popcll(pm);
    scored += valid ? 1u : 0u;
    bytes += by;
    if (qn - qh >= 64u) {
      wave_lds_sync();
      exact(qh, 64u);
      qh += 64u;
    }
  }
  if (qn > qh) {
    wave_lds_sync();
    exact(qh, qn - qh);
  }
  const uint32_t ss = wave_sum_u32(scored), sbytes = wave_sum_u32(bytes);
  if (lane == 0) {
    out.bcnt[blk] = cnt;
    out.bscored[blk] = ss;
    out.bbytes[blk] = sbytes;
    if (out.bexact) out.bexact[blk] = nexact;
  }
}

hipError_t launch_score_gq(const ScoreParams& P, const PairSource& src, uint64_t slot0, uint64_t nslots,
                           const uint32_t* perm, const GQArgs* A, int nq, int nn, int defer,
                           const StageOut& out, hipStream_t s) {
  if (nslots == 0) return hipSuccess;
  if (nslots % kScoreBlock || slot0 % kScoreBlock) return hipErrorInvalidValue;
  const uint64_t ntask = nslots / kScoreBlock;
  const unsigned grid = (unsigned)((ntask + kScoreBlock / 64 - 1) / (kScoreBlock / 64));
#define DK_GQ_CASE(NQ_, NN_, DEF_)                                                                 \
  if (nq == NQ_ && nn == NN_ && defer == DEF_) {                                                   \
    k_score_gq<NQ_, NN_, DEF_><<<grid, kScoreBlock, 0, s>>>(P, src, slot0, nslots, perm, A, out);  \
    return hipGetLastError();                                                                      \
  }
#ifdef DK_GQ_MIN  // timing variants (csrc/Makefile gvariant): configs[2]'s case only
  DK_GQ_CASE(2, 2, 0)
#else
  DK_GQ_CASE(1, 0, -1) DK_GQ_CASE(1, 1, -1) DK_GQ_CASE(1, 2, -1) DK_GQ_CASE(1, 3, -1)
  DK_GQ_CASE(2, 0, -1) DK_GQ_CASE(2, 1, -1) DK_GQ_CASE(2, 2, -1) DK_GQ_CASE(2, 3, -1)
  DK_GQ_CASE(2, 0, 0) DK_GQ_CASE(2, 1, 0) DK_GQ_CASE(2, 2, 0) DK_GQ_CASE(2, 3, 0)
  DK_GQ_CASE(2, 0, 1) DK_GQ_CASE(2, 1, 1) DK_GQ_CASE(2, 2, 1) DK_GQ_CASE(2, 3, 1)
#endif
#undef DK_GQ_CASE
  return hipErrorInvalidValue;
}

// Sort keys of the tasks (kScoreBlock slots of one query each): chunk << 32 | the replica
// position of the task's first candidate; cb[0..nchunks] = the chunks' first tasks.
__global__ void k_task_keys(const PairSource S, uint64_t ntask, const uint64_t* __restrict__ cb,
                            int nchunks, uint64_t* __restrict__ key, uint32_t* __restrict__ val) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntask) return;
  const uint32_t qi = S.wq[t * (kScoreBlock / 64)];
  uint64_t x = t * kScoreBlock - S.qoff[qi];
  uint64_t g = 0;
  for (int k = 0; k < S.nseg; ++k) {
    const uint2 r = S.ranges[(uint64_t)k * S.nq + qi];
    const uint64_t len = r.y - r.x;
    if (x < len) {
      g = S.segoff[k] + r.x + x;
      break;
    }
    x -= len;
  }
  int lo = 0, hi = nchunks;  // the chunk c with cb[c] <= t < cb[c + 1]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (cb[mid] <= t) lo = mid; else hi = mid;
  }
  key[t] = ((uint64_t)lo << 32) | (g & 0xFFFFFFFFull);
  val[t] = (uint32_t)t;
}

hipError_t launch_task_keys(const PairSource& src, uint64_t ntask, const uint64_t* cb, int nchunks,
                            uint64_t* key, uint32_t* val, hipStream_t s) {
  if (ntask == 0) return hipSuccess;
  k_task_keys<<<(unsigned)((ntask + 255) / 256), 256, 0, s>>>(src, ntask, cb, nchunks, key, val);
  return hipGetLastError();
}

}  // namespace dk
