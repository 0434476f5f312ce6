// dk_internal.h — shared definitions between the C-ABI host layer (dk_api.cpp) and the
// gfx950 kernels (dk_kernels.hip).  Not part of the public ABI (include/dukehip.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dukehip.h"

namespace dk {

constexpr int kMaxProps = 16;
constexpr int kMaxOrders = DK_MAX_ORDER_CLASSES;  // Processor.compare visiting orders (dk_schema)
static_assert(kMaxProps <= 16 && kMaxOrders == 4, "ScoreParams::order packs 4-bit positions");
constexpr int kMaxKeys = 8;
constexpr int kMaxSegs = 2 * kMaxKeys;  // per key function: sorted base + sorted delta
constexpr uint16_t kMissing = 0xFFFF;  // length sentinel: record has no value
constexpr int kMaxUnits = 64;          // Levenshtein query limit of the lane-per-pair DP
constexpr int kMaxLongUnits = 256;     // WeightedLevenshtein / long Levenshtein value limit
constexpr int kMaxReplicaUnits = 64;   // longer columns are read in place (canonical arena)
constexpr int kMaxReplicaGrams = 64;   // QGram sets with more grams are read in place
constexpr uint32_t kSentinel = 0xFFFFFFFFu;  // filtered candidate slot

// Latin-1 bigram keys and their per-row perfect hash (DevProp::g16).  A QGram q = 2 code is
// (u0 << 16) | u1 (16 bits per UTF-16 unit); with both units < 256 the 16-bit bigram
// (u0 << 8) | u1 is injective, and key = bigram + 1 (mod 2^16) is never 0 except for the
// bigram U+00FF U+00FF, whose rows get no seed -- so a zero key is padding.  A row's seed
// s = (lt - kGramLtMin) << 8 | i names the table size 2^lt (lt 6..9: the smallest that has a
// seed, k_gram_seed) and multiplier gram_mult(i) under which slot(key) = low32(key * mult)
// >> (32 - lt) is injective on the row's keys.
constexpr int kGramLtMin = 6;
constexpr uint16_t kGramSeedNone = 0xFFFF;
constexpr int kGramSeedTries = 256;
// grams of a set that get a seed (table <= 512 u32): a property whose longest set has more
// grams has no candidate replica (kMaxReplicaGrams), so no seed of it would ever be read
constexpr int kGramPerfectMax = kMaxReplicaGrams;
__host__ __device__ inline uint32_t gram_key(uint64_t code) {
  return ((((uint32_t)(code >> 8) & 0xFF00u) | ((uint32_t)code & 0xFFu)) + 1u) & 0xFFFFu;
}
__host__ __device__ inline uint32_t gram_mult(uint32_t i) {  // odd, < 2^24 (v_mul_u32_u24)
  return ((0x9E3779u ^ (i * 0x5851F5u)) & 0xFFFFFFu) | 1u;
}

// comparators whose values carry a precomputed sorted code list (goff/gcnt/grams):
// QGram sets (sorted unique packed grams) and the token comparators (sorted token ids,
// duplicates kept)
__host__ __device__ constexpr bool uses_codes(int op) {
  return op == DK_CMP_QGRAM || op == DK_CMP_DICE_TOKENS || op == DK_CMP_JACCARD_TOKENS;
}

constexpr uint8_t kAlive = 1;    // not superseded by a later upsert of the same ID
constexpr uint8_t kDeleted = 2;  // dukeDeleted == "true" (IncrementalLuceneDatabase.java:478)
// entered the index (not transient); kept when the row is superseded, so a superseded version
// still counts in the Lucene source's unmerged statistics until dk_lucene_merge
constexpr uint8_t kIndexed = 4;
// replica identity of a base-table position whose row was superseded after the base was
// sorted (delete-by-ID, IncrementalLuceneDatabase.java:516-517): never a candidate.  dk_upsert
// rejects this identity value.
constexpr uint64_t kDeadIdent = ~0ull;

// ---------------------------------------------------------------------------------------
// HBM layout
//  canonical index (row-indexed, grows with dk_upsert):
//    per property: off[row] (first code unit, 4-byte aligned), len[row] (kMissing = no
//    value), units arena (u8 or u16, zero padded), num/numok (NUMERIC), goff/gcnt/grams
//    (QGRAM: sorted unique packed grams; DICE/JACCARD_TOKENS: sorted token ids with
//    duplicates); per row: ident, flags, group; per key function
//    keys[k][row].
//  candidate replica (rebuilt by every dk_match after the blocking sort): the K key
//    functions' sorted candidate lists concatenated — position g = k * M + i holds row
//    rowof[g] = k-th table's i-th row — and per property its values in that order:
//    rlen[g], runits transposed [unit j][g] (so the 64 lanes of a wave, which hold 64
//    consecutive candidates, read unit j of their values as 64 consecutive elements),
//    rnum/rnumok, rgoff/rgcnt, and for QGram sets of <= kMaxReplicaGrams grams the codes
//    transposed rgrams[k][g] (zero past a set's count).
// ---------------------------------------------------------------------------------------

struct DevProp {
  int32_t op;         // DK_CMP_*
  int32_t width;      // 1 or 2 bytes per code unit in `units`
  int32_t q, formula, tokenizer;
  int32_t rlmax;      // replica units per value (0 = read candidates in place)
  double low, high, min_ratio;
  // canonical (query side; candidate side when rlmax == 0)
  const uint32_t* off;
  const uint16_t* len;
  const void* units;
  const double* num;
  const uint8_t* numok;
  const uint32_t* goff;
  const uint16_t* gcnt;
  const uint64_t* grams;
  // replica (candidate side), indexed by replica position
  const uint16_t* rlen;
  const void* runits;     // [j * rstride + g]
  const double* rnum;
  const uint8_t* rnumok;
  const uint32_t* rgoff;
  const uint16_t* rgcnt;
  const void* rgrams;      // QGram: [k * rstride + g], k < rgmax (0 = read grams in place)
  int32_t rgmax;
  int32_t rg32;            // replica codes are u32 (every code of the property < 2^32)
  // Latin-1 bigrams (QGram q = 2, BASIC / ENDS, a width-1 arena): rgrams holds per position
  // rgrows u64 words [j * rstride + g], word j = the gram keys 4j .. 4j+3 (16 bits each,
  // gram_key(), 0 past the set), and gseed[row] is the row's perfect-hash seed of its own
  // gram set (kGramSeedNone: none) -- the query side's LDS table is then collision-free.
  int32_t g16;
  int32_t rgrows;
  const uint16_t* gseed;
};

struct ScoreParams {
  int32_t nprops;
  int32_t mode;
  int32_t lev_rows;       // longest Levenshtein value in the index (selects the variant)
  int32_t long_rows;      // longest value on the long-value DP (0 = none; selects the variant)
  int32_t raw_prop;       // >= 0: emit property raw_prop's comparator similarity instead of
                          // the probability (dk_property_similarity); -1 = normal scoring
  int32_t has_dp;         // some property is Levenshtein / JaroWinkler / WeightedLevenshtein
                          // (0: the DP-free kernel variant, no DP code or registers)
  int32_t has_grams;      // some property is QGram / Dice / Jaccard tokens (0: the short
                          // kernels' variant without the gram-set code or its registers)
  int32_t has_geo;        // some property is GeopositionComparator: the GEO kernel variants
                          // (libm's f64 sin / cos reduce large arguments in scratch memory,
                          // which the other variants must not carry)
  double threshold;
  double maybe;
  const uint64_t* ident;
  const uint32_t* rowof;  // replica position -> row
  uint64_t rstride;       // replica positions (K * M)
  // Processor.compare's visiting order of a query row: the k-th property of order class c
  // is bits [4k, 4k + 4) of order[c] (dk_schema.orders); norders 1: order[0] is the
  // identity.  Packed words, read by a uniform select (order_word): a dynamically indexed
  // byte array in the kernel argument sends the whole ScoreParams to scratch.
  int32_t norders;
  uint64_t order[kMaxOrders];
  const uint8_t* oclass;  // per row: its order class (norders > 1)
  // GeopositionComparator: set (non-zero) by a kernel that compared a value without ','
  // (numok 2) -- stock Duke raises there; the host then fails the call
  uint32_t* raised;
  DevProp props[kMaxProps];
};

// Where the (query, candidate) of a slot comes from.  Every query's slots are padded to
// a multiple of 64, so each wave of k_score holds exactly one query.
struct PairSource {
  const uint32_t* queries;  // query rows
  // blocked modes: slot s of query qi (qoff[qi] <= s < qoff[qi+1]) is candidate t = s -
  // qoff[qi] of its concatenated key-function ranges; t past their total is padding
  const uint32_t* wq;       // global wave (slot / 64) -> query index
  const uint64_t* qoff;     // query index -> first slot
  const uint2* ranges;      // [k * nq + qi]: candidate range of query qi in sorted table k
  uint64_t nq;
  int32_t nkeys;            // key functions
  int32_t allpairs;
  // candidate segments (BlockTables): segment k of nseg belongs to key function
  // k >> seg_shift; its replica positions start at segoff[k]; ranges / sranges / mbase /
  // obase are indexed [segment * nq + qi]
  int32_t nseg, seg_shift;
  uint64_t segoff[kMaxSegs];
  const uint64_t* qkeys[kMaxKeys];  // key of every row (the query side's keys)
  const uint64_t* rident;   // per replica position: ident of its row (Processor.isSameAs)
  const uint64_t* rkeys[kMaxKeys];  // per replica position: key j of its row, j < nkeys - 1
  // ALLPAIRS: slot s -> (s / mpad, replica position s % mpad if < m)
  uint64_t m;               // usable rows (= replica positions per key function)
  uint64_t mpad;            // m rounded up to a wave (64)
  int32_t same_ok;          // score pairs of one identity too (dk_compare_rows)
  int32_t sym;              // 1: owner slots of the symmetric dedup schedule (below)
  int32_t two;              // SYM: k_score_sym2's packed owner slots (k_opack): wq2 per wave
  const uint2* wq2;         // {query of the wave's first slot, query of its last slot}
  uint64_t olo;             // first owner slot of the launch's queries (slot0 is wave-aligned)
  // Symmetric dedup schedule: queries are the contiguous rows [r0, r1);
  // per (key function k, query qi) sranges[k * nq + qi] = {lo, hi, qa, pq}: the bucket
  // [lo, hi) of the query's key in sorted table k, qa = first position with row >= r0,
  // pq = the query's own position (kNoPos when it is not in the table: then qa = hi).
  // The query OWNS candidates [lo, qa) and (pq, hi): it scores them and, for those that
  // are queries themselves, also the reverse direction; candidates in [qa, pq) are owned
  // by those (earlier) queries.  Owner slot t of a query is its t-th owned candidate over
  // k; qoff / wq then describe owner slots.  Results: okind[s] = the decision (0 none,
  // DK_KIND_*) of compare(query, cand) at owner slot s and, for an entry, ores[s] = its
  // probability; compare(cand, query) goes to the candidate's MIRROR segment for key k,
  // position m = mbase[k * nq + cand] + (pq - qa) -- the candidate's mirror candidates are
  // the bucket positions [qa, pq_cand) in order -- as mkind[m] / mres[m], written only for
  // an entry (mkind is cleared per call), so the emission pass (k_sym_emit) reads one
  // decision byte per candidate from contiguous runs.
  const uint4* sranges;
  uint8_t* okind;
  double* ores;
  uint8_t* mkind;
  double* mres;
  const uint64_t* mbase;
  uint32_t r0, r1;
};

constexpr uint32_t kNoPos = 0xFFFFFFFFu;

// k_score_grouped (dk_score_grouped.hip): schemas of Numeric properties and at most
// kGroupedTabs Latin-1 bigram QGram properties (DevProp::g16), direct schedule; each
// query's slots are padded to kScoreBlock (one task = one wave = one staging block)
constexpr int kGroupedTabs = 2;

// k_score_grouped's per-property operand sources, built by the host for each match (raw
// buffer resources: base + size in bytes; size 0 = nothing to read) and read by the kernel
// with scalar loads -- the resources then cost no per-group arithmetic or SGPRs to keep.
struct GroupedProp {
  const void* len;    // rlen (u16 per position)
  const void* x;      // QGram: rgcnt (u16; its low byte); Numeric: rnumok (u8)
  const void* w;      // QGram: rgrams rows (u64 key words); Numeric: rnum
  uint32_t len_n, x_n;
  uint32_t w_rows;    // rows of w: QGram rgrows, Numeric 1 (rnum), none 0
  uint32_t rowb;      // bytes per row of w (replica positions x 8)
  uint32_t xsh;       // x element = 1 << xsh bytes
  uint32_t tslot;     // QGram: the query table of this property (rank among the QGram ones)
  uint32_t w_head;    // rows of w under the first resource (all of them unless they pass 4 GiB)
  uint32_t w_tailb;   // k_score_grouped<1>: bytes of the tail rows' resource (rows past the
                      // first kGroupedHeadRows)
  uint32_t pad[2];
};
static_assert(sizeof(GroupedProp) == 64, "two s_load_dwordx8");
constexpr int kGroupedHeadRows = 4;  // k_score_grouped reads rows [0, 2 DK_GROUPED_ROWS) per pair

// k_score_gq<NQ, NN> (dk_score_grouped.hip, round 5): the same schemas as k_score_grouped
// without DK_CMP_NONE properties, NQ <= kGroupedTabs bigram QGram properties and NN <=
// kGQMaxNum Numeric ones, each in a ROLE of its kind (QGram roles ordered by key-word rows,
// fewest first).  Per role the host gives the candidate operands' bases and sizes and the
// comparator constants, so every per-role value the kernel reads sits at a fixed offset
// (scalar loads, no per-group property indexing).  Key-word row j of a QGram role is read
// through the head buffer resource (rows < kGroupedHeadRows, based at row 0) or the tail
// one (based at row kGroupedHeadRows); both must stay below 2^32 bytes (the host checks).
constexpr int kGQMaxNum = 3;
struct GQRoleQ {
  const uint16_t* rlen;
  const uint16_t* rgcnt;
  const uint64_t* rows;   // key-word rows [j * rstride + g]
  const uint64_t* tail;   // rows + kGroupedHeadRows * rstride
  uint32_t nrows;         // rgrows
  uint32_t head_bytes;    // min(nrows, kGroupedHeadRows) rows
  uint32_t tail_bytes;    // the rows past kGroupedHeadRows
  uint32_t rowb;          // bytes per row (replica positions x 8)
  int32_t prop, formula;
  double low, high;
  // the screen's single-precision constants: low, high, max(0, low) (a candidate without
  // grams), and the most PropertyImpl.compare can give over sim in [0, 1] (a deferred role)
  float flow, fhigh, flow0, fub;
};
struct GQRoleN {
  const uint16_t* rlen;
  const uint8_t* rnumok;
  const double* rnum;
  int32_t prop;
  uint32_t pad;
  double low, high, min_ratio;
};
struct alignas(16) GQArgs {
  int32_t nq, nn;
  uint32_t len_bytes;     // replica positions x 2 (rlen / rgcnt resources)
  uint32_t pos_n;         // replica positions
  // the group loop's other operands (the kernel copies GQArgs to LDS and re-reads it per
  // group, so none of this is held in scalar registers across the loop)
  const uint64_t* rident;
  const uint64_t* rkey0;  // rkeys[0] (nkeys > 1)
  const uint32_t* rowof;
  double* oprob;          // the launch's staging set (StageOut)
  uint32_t* ocand;
  uint32_t* oqidx;
  double threshold, maybe;
  // Processor.compare's visiting order per order class as ROLES, 4 bits per position: a
  // QGram role a is a, a Numeric role b is 8 + b
  uint64_t rorder[kMaxOrders];
  GQRoleQ q[kGroupedTabs];
  GQRoleN n[kGQMaxNum];
  // k_score_gq's screen: a pair goes to the exact pass when its probability bound's odds
  // reach `screen` (0: every valid pair); `defer`: the QGram role left to the exact pass
  // (-1: none)
  float screen;
  int32_t defer;
  uint32_t pad_[2];
};
// queue of screened pairs per wave (k_score_gq), and the bounds inside which a role's
// single-precision probability keeps Bayes monotone and the odds accurate
constexpr int kGQQueue = 128;
constexpr float kScreenLo = 0.011f, kScreenHi = 0.989f;

// The emission pass of the symmetric schedule (k_sym_emit): per query of a chunk its
// candidates in Duke's order, each read as a decision byte from the owner results (okind,
// ores: the chunk's half, indexed by absolute owner slot) or the mirror results (mkind, mres).
struct EmitSource {
  const uint4* sranges;
  const uint64_t* obase;    // [k * nq + qi]: owner slot of candidate position qa of (k, qi)
  const uint64_t* mbase;    // [k * nq + qi]: mirror slot of candidate position qa of (k, qi)
  const uint8_t* okind;
  const double* ores;
  const uint8_t* mkind;
  const double* mres;
  const uint32_t* rowof;
  uint64_t nq;
  int32_t nseg;
  uint32_t pad;
  uint64_t segoff[kMaxSegs];
  uint32_t* ecount;         // per query: its entries (the count pass)
  const uint64_t* eincl;    // per query: inclusive prefix of ecount over its chunk's queries
  const uint64_t* oqoff;    // per query: first owner slot (its owned run: up to oqoff[qi + 1])
  const uint64_t* mqoff;    // per query: first mirror slot (its mirror runs: up to mqoff[qi + 1])
  const uint64_t* ocnt;     // non-null (k_opack's tile order): the owned run is [oqoff, + ocnt)
};

// Per-chunk staging of the score kernel.  Block b (256 slots) writes its emitted entries,
// in slot order, to [b*256, b*256 + bcnt[b]); k_compact then concatenates the blocks in
// block order, so the final list is in slot order (query, key function, candidate)
// without a sort or any atomic on the entries.
constexpr int kScoreBlock = 256;
constexpr int kKindShift = 30;  // staged candidate word = row | kind << 30
struct StageOut {
  uint64_t* counters;  // [0] pairs scored, [1] operand bytes, [3] pairs that took k_score_gq's
                       // exact pass (summed by k_reduce_blocks)
  uint32_t* bcnt;      // per block: emitted entries
  uint32_t* bscored;   // per block: pairs scored
  uint32_t* bbytes;    // per block: algorithmic operand bytes
  double* prob;
  uint32_t* cand;
  uint32_t* qidx;
  uint32_t* bexact;    // per block: pairs through the exact pass (k_score_gq; null: none)
};

// Device-resident match list of one dk_match call.
struct MatchList {
  uint32_t* cand;
  uint8_t* kind;
  double* prob;
  uint32_t* qidx;
};

// Blocking tables (index state): per key function the usable rows (alive, not deleted)
// sorted by (key, group, row).  Each key function has a BASE segment (the rows below
// base_rows when the tables were last fully sorted) and, once rows were added after that,
// a DELTA segment (the usable rows from base_rows on, re-sorted per index change; SURVEY
// §8f-1).  Segment s belongs to key function s >> seg_shift (seg_shift 0: no delta, one
// segment per key function); its entries are replica positions [seg_off[s], seg_off[s] +
// seg_len[s]) with rows rowof[...].  All delta rows are above all base rows, so a bucket's
// base entries followed by its delta entries are in (group, row) order -- the full sort's.
struct BlockTables {
  int32_t nkeys;
  int32_t linkage;
  int32_t nseg, seg_shift;
  const uint64_t* keys[kMaxKeys];   // per key function, per row
  const uint8_t* group;             // per row (LINKAGE)
  const uint64_t* skeys[kMaxSegs];  // sorted keys of segment s
  const uint8_t* sgroup[kMaxSegs];  // group of segment s's entries (LINKAGE)
  uint64_t seg_len[kMaxSegs];
  uint64_t seg_off[kMaxSegs];
  const uint32_t* rowof;            // replica position -> row
  const uint64_t* rident;           // replica position -> identity (kDeadIdent: superseded)
};

// One property's replica build.
struct ReplicaJob {
  int32_t width;
  int32_t rlmax;      // 0: no unit replica (long values, or non-string comparator)
  int32_t has_num;        // doubles per row in num / rnum (1 Numeric, 2 Geoposition; 0 none)
  int32_t has_qgram;
  int32_t rgmax;      // QGram replica rows (0: none)
  int32_t rg32;       // u32 replica codes
  int32_t g16;        // Latin-1 bigram keys, 4 per u64 word, rgrows words (DevProp::g16)
  int32_t rgrows;
  uint64_t stride;    // replica positions
  const uint32_t* off;
  const uint16_t* len;
  const void* units;
  const double* num;
  const uint8_t* numok;
  const uint32_t* goff;
  const uint16_t* gcnt;
  uint16_t* rlen;
  void* runits;
  double* rnum;
  uint8_t* rnumok;
  uint32_t* rgoff;
  uint16_t* rgcnt;
  const uint64_t* grams;
  void* rgrams;
};

// Lucene-compatible candidate source (DK_CAND_LUCENE, include/dukehip.h dk_lucene).
// Postings: one entry per (lookup field, term, row) of the rows in the index, key =
// (field << 24 | term) << 32 | row, value = the term's frequency in the row's value; sorted by
// key they give every term's documents in row order (= Lucene doc id order).
constexpr int kLuceneMaxClauses = 256;
constexpr int kLuceneMaxHits = 100;
constexpr int kLuceneTile = 2048;      // rows per accumulation tile (LDS)

struct LuceneParams {
  const uint32_t* queries;
  uint64_t nq;
  const uint64_t* qoff;     // per row: its query clauses [qoff[row], qoff[row+1]) in qterm
  const uint32_t* qterm;    // field << 24 | term of each clause, in clause order
  const uint64_t* skey;     // sorted postings keys
  const uint32_t* stf;      // their term frequencies
  uint64_t npost;
  const uint8_t* norm;      // [row * nfields + field]: SmallFloat-encoded length norm
  int32_t nfields;
  int32_t linkage;
  const uint8_t* flags;     // kDeleted rows are never hits (MUST_NOT dukeDeleted:true)
  const uint8_t* group;     // LINKAGE: MUST_NOT dukeGroupNo == the query's group
  uint64_t max_doc;         // documents in the index (IndexReader.maxDoc of a merged index)
  int32_t max_hits;
  float min_relevance;
  uint32_t* hits;           // [qi * max_hits + j]: row of hit j of query qi (score order)
  uint2* ranges;            // [qi]: its hit positions {qi * max_hits, + nhits}
  uint64_t* counts;         // [qi]: nhits rounded up to 64 (score slots)
  uint64_t* exact;          // [qi]: nhits (NULL: not written)
  uint64_t* real;           // += nhits
};

// The q-gram sets of a batch built on the device (dk_grams.hip): rows [row0, row0 + n) of a
// QGram property whose units, off and len are in place.
struct GramJob {
  const void* units;
  int32_t width, q, tokenizer;
  const uint32_t* off;
  const uint16_t* len;
  uint64_t row0, n;
  const uint64_t* soff;  // per batch row: its scratch run (values of more than 64 raw grams)
  uint64_t* scratch;
  uint16_t* gcnt;        // count pass: [row0 + i] = the set's size
  uint32_t* gcnt32;      // count pass: [i] = the same (scanned into gpos)
  uint32_t* maxg;        // count pass: atomicMax of the sizes
  const uint32_t* gpos;  // write pass: [i] = exclusive prefix of the sizes
  uint32_t gbase;        // write pass: the arena's fill before the batch
  uint32_t* goff;        // write pass: [row0 + i] = gbase + gpos[i]
  uint64_t* grams;       // write pass: the arena
};
hipError_t launch_qgram_sets(const GramJob& J, bool write, hipStream_t s);
hipError_t exclusive_scan_u32_dev(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint32_t* out,
                                  uint64_t n, hipStream_t s);

// ---- launchers (dk_kernels.hip) ----
// postings of rows that are in the index (kAlive): key kept, others set to ~0 (sorted last);
// counts[0] += entries kept, counts[1] += rows in the index among [0, nrows)
hipError_t launch_lucene_prep(const uint64_t* key, uint64_t npost, const uint8_t* flags, uint64_t nrows,
                              uint8_t mask, uint64_t* out_key, uint64_t* counts, hipStream_t s);
hipError_t launch_lucene_merge(uint8_t* flags, uint64_t nrows, hipStream_t s);
hipError_t launch_lucene_topk(const LuceneParams& L, hipStream_t s);
hipError_t launch_widen_u8(const uint8_t* src, uint16_t* dst, uint64_t n, hipStream_t s);
hipError_t launch_clear_flag(uint8_t* flags, const uint32_t* rows, uint64_t n, uint8_t bit,
                             hipStream_t s);
hipError_t launch_gather_keys(const uint64_t* keys, const uint32_t* rows, uint64_t* out,
                              uint64_t n, hipStream_t s);
hipError_t launch_gather_u8(const uint8_t* src, const uint32_t* rows, uint8_t* out, uint64_t n,
                            hipStream_t s);
// rows [row0, row0 + nrows): flag_out[i] = row row0 + i is usable (of want_group)
hipError_t launch_select_rows(const uint8_t* flags, const uint8_t* group, uint64_t row0,
                              uint64_t nrows, int want_group, uint32_t* flag_out, hipStream_t s);
hipError_t launch_scatter_rows(const uint32_t* flag, const uint32_t* pos, uint64_t row0,
                               uint64_t nrows, uint32_t base, uint32_t* rows_out, hipStream_t s);
// *out = Levenshtein.compare(row r1's value, row r2's value) with Duke's exact early exit
// (NaN when either value is missing or empty)
hipError_t launch_lev_exact(const uint32_t* off, const uint16_t* len, const void* units, int width,
                            uint32_t r1, uint32_t r2, double* out, hipStream_t s);
// rows [row0, row0 + n): seed[row] = the perfect-hash seed of the row's bigram keys
hipError_t launch_gram_seed(const uint64_t* grams, const uint32_t* goff, const uint16_t* gcnt,
                            const uint16_t* len, uint64_t row0, uint64_t n, uint16_t* seed,
                            hipStream_t s);
// replica positions [pos0, pos0 + npos)
hipError_t launch_replicate(const ReplicaJob& J, const uint32_t* rowof, uint64_t pos0, uint64_t npos,
                            hipStream_t s);
// superseded base rows: their positions in every base segment get rident = kDeadIdent
hipError_t launch_mark_dead(const BlockTables& T, const uint32_t* rows, uint64_t n, uint64_t* rident,
                            hipStream_t s);
// counts[i] = candidate slots of query i rounded up to `pad` (64: one query per score wave;
// kScoreBlock: one query per k_score_grouped task); real[0] += the unpadded total
hipError_t launch_count(const uint32_t* queries, uint64_t nq, const BlockTables& T, uint2* ranges,
                        uint64_t* counts, uint64_t* real, int pad, hipStream_t s);
// counts[i] = candidate slots of query i, unpadded (dk_candidate_counts)
hipError_t launch_count_exact(const uint32_t* queries, uint64_t nq, const BlockTables& T,
                              uint2* ranges, uint64_t* counts, hipStream_t s);
// wq[w] = qi for every group w of 2^shift slots of query qi (qoff in multiples of 2^shift)
hipError_t launch_wavemap(const uint64_t* qoff, uint64_t nq, uint32_t* wq, hipStream_t s, int shift = 6);
// k_score_sym2's owner slots, per tile of kPackTile queries (k_opack): own[i] (owned candidates)
// -> the query's slots with the padding that keeps every wave to two queries, loc[i] its
// first slot within the tile (queries ordered by klen[queries[i]] when klen is given),
// ttot[t] the tile's slots; oqoff[i] = tbase[tile] + loc[i] with tbase the exclusive scan
// of ttot (k_opack_fin); wq2[w] = {query of wave w's first slot, query of its last slot}
constexpr int kPackTile = 64;  // queries per k_opack tile (one wave walks it)
uint64_t opack_tiles(uint64_t nq);
hipError_t launch_opack(uint64_t* own, uint64_t nq, const uint32_t* queries, const uint16_t* klen,
                        uint32_t* loc, uint64_t* ttot, hipStream_t s);
hipError_t launch_opack_fin(const uint32_t* loc, const uint64_t* tbase, uint64_t nq, uint64_t* oqoff,
                            hipStream_t s);
hipError_t launch_wavemap2(const uint64_t* qoff, const uint64_t* occ, uint64_t nq, uint2* wq2, hipStream_t s);
// replica-ordered identity and keys 0..nkeys-2 of the rows at replica positions
hipError_t launch_replicate_rows(const uint32_t* rowof, uint64_t pos0, uint64_t npos,
                                 const uint64_t* ident, uint64_t* rident, const BlockTables& T,
                                 uint64_t* const* rkeys, hipStream_t s);
hipError_t launch_score(const ScoreParams& P, const PairSource& src, uint64_t slot0,
                        uint64_t nslots, const StageOut& out, hipStream_t s);
// k_score_grouped: slot0 and nslots multiples of kScoreBlock, slots padded per query to it;
// perm (or NULL: task order) = the tasks in execution order (k_task_keys, sorted)
// mode (replicas whose key-word rows pass 2^32 bytes): 0 one buffer resource per property;
// 1 a head and a tail resource; 2 a resource per tail row (k_score_grouped<MODE>)
hipError_t launch_score_grouped(const ScoreParams& P, const PairSource& src, uint64_t slot0,
                                uint64_t nslots, const uint32_t* perm, const GroupedProp* gp,
                                int mode, const StageOut& out, hipStream_t s);
// k_score_gq<nq, nn> (A: device copy of the host's GQArgs, whose nq / nn are passed too)
hipError_t launch_score_gq(const ScoreParams& P, const PairSource& src, uint64_t slot0, uint64_t nslots,
                           const uint32_t* perm, const GQArgs* A, int nq, int nn, int defer, const StageOut& out,
                           hipStream_t s);
// key[t] = chunk << 32 | first candidate's replica position of task t, val[t] = t;
// cb[0..nchunks] = first task of each chunk
hipError_t launch_task_keys(const PairSource& src, uint64_t ntask, const uint64_t* cb, int nchunks,
                            uint64_t* key, uint32_t* val, hipStream_t s);
// symmetric dedup schedule: per query its bucket positions (sranges), full and owner slot
// counts (each padded to 64), real[0] += the unpadded full total
// the symmetric schedule's bucket lookup (k_count_sym's fast path; posof null: binary searches)
struct SymIndex {
  const uint32_t* posof;   // [segment * nrows + row]: position in the segment, kNoPos: none
  const uint32_t* bstart;  // [replica position]: its bucket's first position (segment-relative)
  const uint32_t* bend;    // [replica position of a bucket's first entry]: the bucket's end
  uint64_t nrows;
  const uint2* bse;        // [replica position]: {its bucket's first position, end} in one load
};
hipError_t launch_count_sym(const uint32_t* queries, uint64_t nq, const BlockTables& T, uint32_t r0,
                            uint4* sranges, uint64_t* counts, uint64_t* ocounts, uint64_t* mcounts,
                            uint64_t* real, uint32_t opad, const SymIndex& X, hipStream_t s);
// builds SymIndex over every segment of T (hflag: scratch of one u32 per replica position;
// tmp: symidx_scan_bytes of the longest segment)
hipError_t launch_symidx(const BlockTables& T, uint64_t nrows, uint32_t* posof, uint32_t* hflag,
                         uint32_t* bstart, uint32_t* bend, uint2* bse, void* tmp, size_t tmp_bytes, hipStream_t s);
hipError_t symidx_scan_bytes(uint64_t n, size_t* bytes);
hipError_t launch_obase(const uint4* sranges, const uint64_t* oqoff, const uint64_t* mqoff,
                        uint64_t nq, int nseg, uint64_t* obase, uint64_t* mbase, hipStream_t s);
// k_sym_emit over the chunk's queries [q0, q0 + nqc): write = false counts each query's
// entries into src.ecount; write = true writes them to `out` from list position base +
// src.eincl[qi] - src.ecount[qi] on, and first[qi] (the chunk's last query: first[qi + 1] too)
hipError_t launch_sym_emit(const EmitSource& src, uint64_t q0, uint64_t nqc, bool write, uint64_t base,
                           const MatchList& out, uint64_t* first, hipStream_t s);
hipError_t launch_gather_u64(const uint64_t* src, const uint64_t* idx, uint64_t n, uint64_t* out,
                             hipStream_t s);
// out[i] = start + i (a contiguous batch's query rows, written on the device)
hipError_t launch_iota_u32(uint32_t* out, uint64_t n, uint32_t start, hipStream_t s);
hipError_t launch_reduce_blocks(const StageOut& st, uint64_t nblocks, hipStream_t s);
hipError_t launch_compact(const StageOut& st, const uint64_t* boff, uint64_t nblocks,
                          uint64_t base, const MatchList& out, hipStream_t s);
hipError_t launch_first(const uint32_t* qidx, uint64_t n, uint64_t nq, uint64_t* first,
                        hipStream_t s);
hipError_t launch_fill_u32(uint32_t* p, uint32_t v, uint64_t n, hipStream_t s);
hipError_t launch_iota_u32(uint32_t* p, uint64_t n, hipStream_t s);

// rocPRIM wrappers (dk_kernels.hip)
hipError_t sort_pairs_u64_u32(void* tmp, size_t& tmp_bytes, const uint64_t* kin, uint64_t* kout,
                              const uint32_t* vin, uint32_t* vout, uint64_t n, hipStream_t s);
// the same over key bits [0, end_bit)
hipError_t sort_pairs_u64_u32_bits(void* tmp, size_t& tmp_bytes, const uint64_t* kin, uint64_t* kout,
                                   const uint32_t* vin, uint32_t* vout, uint64_t n, int end_bit,
                                   hipStream_t s);
hipError_t exclusive_scan_u64(void* tmp, size_t& tmp_bytes, const uint64_t* in, uint64_t* out,
                              uint64_t n, hipStream_t s);
hipError_t exclusive_scan_u32(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint32_t* out,
                              uint64_t n, hipStream_t s);
hipError_t exclusive_scan_u32_u64(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint64_t* out,
                                  uint64_t n, hipStream_t s);
hipError_t inclusive_scan_u32_u64(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint64_t* out,
                                  uint64_t n, hipStream_t s);

}  // namespace dk
