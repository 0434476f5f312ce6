// dk_grams.hip — the q-gram sets of an upserted batch, built on the device from the units
// arena (QGramComparator's HashSet<String> of q-grams as sorted unique packed codes, SURVEY
// §8a-12; the same codes as the host restatement qgram_codes in dk_api.cpp, which the token
// comparators still use).  dk_upsert copies the batch's units, then:
//
//   k_qgram_sets<false>: per row (one thread), the value's raw codes -> sorted in registers
//     by a Batcher network (<= kNetMax codes; longer values sort in their own scratch run)
//     -> its unique count gcnt[row], the batch's longest set by atomicMax;
//   an exclusive scan of the counts (rocPRIM);
//   k_qgram_sets<true>: the same codes again, the unique ones written to the grams arena at
//     goff[row] = grams_used + the scan.
//
// Replaces the host's per-value sort, which was most of a 2M-row linkage upsert.
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "dk_internal.h"
#include "dk_sortnet.h"

namespace dk {

constexpr int kNetMax = 64;  // codes of a value sorted in registers

// unit j of the gram source: s, or "^" + s + "$" for ENDS [recalled] (qgram_codes)
template <typename CT>
__device__ __forceinline__ uint32_t gram_unit(const CT* s, int L, int j, int tok) {
  if (tok == DK_QGRAM_ENDS) return j == 0 ? (uint32_t)'^' : (j == L + 1 ? (uint32_t)'$' : (uint32_t)s[j - 1]);
  return (uint32_t)s[j];
}

// code of the gram at ix: 16 bits per unit, POSITIONAL adds ix << 48
template <typename CT>
__device__ __forceinline__ uint64_t gram_code(const CT* s, int L, int ix, int q, int tok) {
  uint64_t c = 0;
  for (int k = 0; k < q; ++k) c = (c << 16) | gram_unit(s, L, ix + k, tok);
  if (tok == DK_QGRAM_POSITIONAL) c |= (uint64_t)ix << 48;
  return c;
}

template <bool WRITE, typename CT>
__device__ __forceinline__ void qgram_row(const GramJob& J, uint64_t i) {
  const uint64_t row = J.row0 + i;
  const int L = J.len[row] == kMissing ? -1 : (int)J.len[row];
  const int m = L < 0 ? 0 : max(0, L + (J.tokenizer == DK_QGRAM_ENDS ? 2 : 0) - J.q + 1);
  const CT* s = reinterpret_cast<const CT*>(J.units) + J.off[row];
  uint64_t* dst = WRITE ? J.grams + J.gbase + J.gpos[i] : nullptr;
  int u = 0;
  if (m <= kNetMax) {
    // the codes in registers, padded with the largest code (the first m after sorting are
    // the value's own); reads past the value stay inside the arena's zero tail
    uint64_t c[kNetMax];
#pragma unroll
    for (int ix = 0; ix < kNetMax; ++ix) c[ix] = ix < m ? gram_code(s, L, ix, J.q, J.tokenizer) : ~0ull;
#define DK_CS(a, b)                                   \
    {                                                 \
      const uint64_t x_ = c[a], y_ = c[b];            \
      c[a] = x_ < y_ ? x_ : y_;                       \
      c[b] = x_ < y_ ? y_ : x_;                       \
    }
    if (__ballot(m > 32) == 0ull) {  // wave-uniform: no lane of the wave has more than 32
      DK_SORTNET32(DK_CS);
    } else {
      DK_SORTNET64(DK_CS);
    }
#undef DK_CS
#pragma unroll
    for (int ix = 0; ix < kNetMax; ++ix) {
      const bool first = ix < m && (ix == 0 || c[ix] != c[ix - 1]);
      if (WRITE && first) dst[u] = c[ix];
      u += first ? 1 : 0;
    }
  } else {
    // a long value: its raw codes in its scratch run, Shell-sorted there (Ciura's gaps:
    // a 254-gram text value takes ~2k compares instead of insertion sort's ~16k)
    uint64_t* r = J.scratch + J.soff[i];
    if (!WRITE) {
      for (int ix = 0; ix < m; ++ix) r[ix] = gram_code(s, L, ix, J.q, J.tokenizer);
      constexpr int kGaps[8] = {701, 301, 132, 57, 23, 10, 4, 1};
      for (int gi = 0; gi < 8; ++gi) {
        const int gap = kGaps[gi];
        for (int ix = gap; ix < m; ++ix) {
          const uint64_t x = r[ix];
          int k = ix;
          while (k >= gap && r[k - gap] > x) {
            r[k] = r[k - gap];
            k -= gap;
          }
          r[k] = x;
        }
      }
    }
    for (int ix = 0; ix < m; ++ix) {
      const bool first = ix == 0 || r[ix] != r[ix - 1];
      if (WRITE && first) dst[u] = r[ix];
      u += first ? 1 : 0;
    }
  }
  if (WRITE) {
    J.goff[row] = J.gbase + J.gpos[i];
  } else {
    J.gcnt[row] = (uint16_t)u;
    J.gcnt32[i] = (uint32_t)u;
    atomicMax(J.maxg, (uint32_t)u);
  }
}

template <bool WRITE>
__global__ __launch_bounds__(256) void k_qgram_sets(const GramJob J) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= J.n) return;
  if (J.width == 1) qgram_row<WRITE, uint8_t>(J, i);
  else qgram_row<WRITE, uint16_t>(J, i);
}

hipError_t launch_qgram_sets(const GramJob& J, bool write, hipStream_t s) {
  if (J.n == 0) return hipSuccess;
  const unsigned grid = (unsigned)((J.n + 255) / 256);
  if (write) k_qgram_sets<true><<<grid, 256, 0, s>>>(J);
  else k_qgram_sets<false><<<grid, 256, 0, s>>>(J);
  return hipGetLastError();
}

hipError_t exclusive_scan_u32_dev(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint32_t* out,
                                  uint64_t n, hipStream_t s) {
  return rocprim::exclusive_scan(tmp, tmp_bytes, in, out, 0u, (size_t)n, rocprim::plus<uint32_t>(), s);
}

}  // namespace dk
