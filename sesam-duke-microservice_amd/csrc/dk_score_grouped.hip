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
        const int sh = 24 - (int)(sd >> 8);  // 32 - lt
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
          const int sh = 24 - (int)(sd >> 8);
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
