// dk_internal.h — shared definitions between the C-ABI host layer (dk_api.cpp) and the
// gfx950 kernels (dk_kernels.hip).  Not part of the public ABI (include/dukehip.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dukehip.h"

namespace dk {

constexpr int kMaxProps = 16;
constexpr int kMaxKeys = 8;
constexpr uint16_t kMissing = 0xFFFF;  // length sentinel: record has no value
constexpr int kMaxUnits = 64;          // per-value limit of the lane-per-pair kernels
constexpr uint32_t kSentinel = 0xFFFFFFFFu;  // filtered candidate slot
constexpr int kKeyShift = 29;          // candidate word = row | (key function << 29)
constexpr uint32_t kRowMask = (1u << kKeyShift) - 1u;

constexpr uint8_t kAlive = 1;    // not superseded by a later upsert of the same ID
constexpr uint8_t kDeleted = 2;  // dukeDeleted == "true" (IncrementalLuceneDatabase.java:478)

// One scored property as the fused kernel sees it (HBM SoA, row-indexed).
struct DevProp {
  int32_t op;         // DK_CMP_*
  int32_t width;      // 1 or 2 bytes per code unit in `units`
  int32_t q, formula, tokenizer, pad;
  double low, high, min_ratio;
  const uint32_t* off;   // row -> first code unit (4-byte aligned string starts)
  const uint16_t* len;   // row -> code units, kMissing = no value
  const void* units;     // arena, zero-padded, tail-padded for over-reads
  const double* num;     // NUMERIC: parsed Double.parseDouble value
  const uint8_t* numok;  // NUMERIC: 1 = parsed, 0 = NumberFormatException
  const uint32_t* goff;  // QGRAM: row -> first gram
  const uint16_t* gcnt;  // QGRAM: row -> unique grams
  const uint64_t* grams; // QGRAM: sorted unique packed grams
};

struct ScoreParams {
  int32_t nprops;
  int32_t mode;
  double threshold;
  double maybe;
  const uint64_t* ident;
  DevProp props[kMaxProps];
};

// Where the (query, candidate) of a slot comes from.
struct PairSource {
  // blocked modes: materialised chunk of slots
  const uint32_t* pq;  // query index (into the query list)
  const uint32_t* pc;  // candidate word (row | k << 29) or kSentinel
  // ALLPAIRS: implicit slots s -> (s / m, usable[s % m])
  const uint32_t* queries;  // query rows
  const uint32_t* usable;   // candidate rows
  uint64_t m;
  int32_t allpairs;
};

// Per-chunk staging of the score kernel.  Block b (256 slots) writes its emitted entries,
// in slot order, to [b*256, b*256 + bcnt[b]); k_compact then concatenates the blocks in
// block order, so the final list is in slot order (query, key function, candidate)
// without a sort or any atomic on the entries.
constexpr int kScoreBlock = 256;
constexpr int kKindShift = 30;  // staged candidate word = row | kind << 30
struct StageOut {
  uint64_t* counters;  // [0] pairs scored, [1] operand bytes
  uint32_t* bcnt;      // per block: emitted entries
  double* prob;
  uint32_t* cand;
  uint32_t* qidx;
};

// Device-resident match list of one dk_match call.
struct MatchList {
  uint32_t* cand;
  uint8_t* kind;
  double* prob;
  uint32_t* qidx;
};

// ---- launchers (dk_kernels.hip) ----
hipError_t launch_widen_u8(const uint8_t* src, uint16_t* dst, uint64_t n, hipStream_t s);
hipError_t launch_clear_flag(uint8_t* flags, const uint32_t* rows, uint64_t n, uint8_t bit,
                             hipStream_t s);
hipError_t launch_gather_keys(const uint64_t* keys, const uint32_t* rows, uint64_t* out,
                              uint64_t n, hipStream_t s);
hipError_t launch_gather_u8(const uint8_t* src, const uint32_t* rows, uint8_t* out, uint64_t n,
                            hipStream_t s);
hipError_t launch_select_rows(const uint8_t* flags, const uint8_t* group, uint64_t nrows,
                              int want_group, uint32_t* flag_out, hipStream_t s);
hipError_t launch_scatter_rows(const uint32_t* flag, const uint32_t* pos, uint64_t nrows,
                               uint32_t base, uint32_t* rows_out, hipStream_t s);
// Blocking tables of one dk_match call: per key function, the usable rows (alive, not
// deleted) sorted by (key, group, row).
struct BlockTables {
  int32_t nkeys;
  int32_t linkage;
  const uint64_t* keys[kMaxKeys];  // per key function, per row
  const uint8_t* group;  // per row (LINKAGE)
  const uint64_t* skeys[kMaxKeys];
  const uint32_t* srows[kMaxKeys];
  const uint8_t* sgroup[kMaxKeys];
  uint64_t n[kMaxKeys];
};

hipError_t launch_count(const uint32_t* queries, uint64_t nq, const BlockTables& T, uint2* ranges,
                        uint64_t* counts, hipStream_t s);
hipError_t launch_emit(const uint32_t* queries, uint64_t q0, uint64_t q1, const uint64_t* qoff,
                       const uint2* ranges, uint64_t nq, const BlockTables& T,
                       const uint64_t* ident, uint64_t s0, uint64_t s1, uint32_t* pq,
                       uint32_t* pc, hipStream_t s);
hipError_t launch_score(const ScoreParams& P, const PairSource& src, uint64_t slot0,
                        uint64_t nslots, const StageOut& out, hipStream_t s);
hipError_t launch_compact(const StageOut& st, const uint64_t* boff, uint64_t nblocks,
                          uint64_t base, const MatchList& out, hipStream_t s);
hipError_t launch_first(const uint32_t* qidx, uint64_t n, uint64_t nq, uint64_t* first,
                        hipStream_t s);
hipError_t launch_fill_u32(uint32_t* p, uint32_t v, uint64_t n, hipStream_t s);
hipError_t launch_iota_u32(uint32_t* p, uint64_t n, hipStream_t s);

// rocPRIM wrappers (dk_kernels.hip)
hipError_t sort_pairs_u64_u32(void* tmp, size_t& tmp_bytes, const uint64_t* kin, uint64_t* kout,
                              const uint32_t* vin, uint32_t* vout, uint64_t n, hipStream_t s);
hipError_t exclusive_scan_u64(void* tmp, size_t& tmp_bytes, const uint64_t* in, uint64_t* out,
                              uint64_t n, hipStream_t s);
hipError_t exclusive_scan_u32(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint32_t* out,
                              uint64_t n, hipStream_t s);
hipError_t exclusive_scan_u32_u64(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint64_t* out,
                                  uint64_t n, hipStream_t s);

}  // namespace dk
