// LDS bank conflicts of random hash-table probes on gfx950: the probe
// k_score_gq issues (probe_word16: a 16-bit entry at a perfect-hash slot of the query's
// 512-entry table, one table per wave) against the layouts proposed to cut its conflicts.
// Every lane probes pseudo-random slots (an LCG per lane); each kernel runs the same probe
// count, 4 waves per block, 8 blocks per CU.  Prints ns per probe instruction per CU; the
// conflict cycles per LDS instruction come from a rocprofv3 --pmc pass over the same binary
// (SQ_INSTS_LDS, SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE), and --mc prints the Monte-Carlo
// expectation of the extra cycles for uniform random slots under the microarch guide's
// banking rule (ds_read_b32 / u16: two 32-lane groups, bank = dword mod 32, one extra cycle
// per extra distinct dword on a bank).
//
//   V0 u16 table, 512 entries (1 KB per wave)          -- k_score_gq's probe
//   V1 two half-wave copies of V0 (lanes 32..63 read the second 1 KB)
//   V2 4-way interleaved copies: entry e of copy (lane & 3) at dword 4e + (lane & 3) (8 KB)
//   V3 u32 table, 512 entries (2 KB)                   -- k_score_grouped's probe_word
//   V4 V0 with the slot's dword rotated by the lane's half (bank + 16 for lanes 32..63)
//   V5 u16 table, 256 entries (lt 8: 4 dwords per bank)
//   V6 u16 table, 128 entries (lt 7: 2 dwords per bank)
//   V7 u16 table,  64 entries (lt 6: one dword per bank -- no conflict can occur)
//
// hipcc --offload-arch=gfx950 -O3 -o lds_probe lds_probe.hip && ./lds_probe [--mc]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>

constexpr int kIters = 4096;
constexpr int kUnroll = 16;

template <int V>
__global__ __launch_bounds__(256) void k_probe(unsigned* out, unsigned seed) {
  __shared__ unsigned lds[4][2048];  // 8 KB per wave: the largest layout (V2)
  const unsigned wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  unsigned* t32 = lds[wave];
  for (unsigned i = lane; i < 2048; i += 64) t32[i] = i * 2654435761u;
  __syncthreads();
  unsigned x = seed ^ (blockIdx.x * 256u + threadIdx.x) * 747796405u;
  unsigned acc = 0;
  const unsigned short* t16 = reinterpret_cast<const unsigned short*>(t32);
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      x = x * 1664525u + 1013904223u;
      const unsigned slot = x >> 23;  // 0..511
      if constexpr (V == 0) acc += t16[slot];
      if constexpr (V == 1) acc += t16[(lane >= 32 ? 512u : 0u) + slot];
      if constexpr (V == 2) acc += t32[4u * slot + (lane & 3u)] & 0xFFFFu;
      if constexpr (V == 3) acc += t32[slot];
      if constexpr (V == 4) acc += t16[((((slot >> 1) + (lane >= 32 ? 16u : 0u)) & 255u) << 1) | (slot & 1u)];
      if constexpr (V == 5) acc += t16[slot >> 1];
      if constexpr (V == 6) acc += t16[slot >> 2];
      if constexpr (V == 7) acc += t16[slot >> 3];
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// Monte Carlo: extra LDS cycles per wave instruction for uniform random slots
static double mc(int V, int trials) {
  std::mt19937 rng(1234);
  double extra = 0;
  for (int t = 0; t < trials; ++t) {
    for (int g = 0; g < 2; ++g) {
      std::set<unsigned> dw[32];
      for (int l = 0; l < 32; ++l) {
        const unsigned lane = 32u * g + l, slot = rng() & 511u;
        unsigned dword = 0;
        if (V == 0) dword = slot >> 1;
        if (V == 1) dword = (lane >= 32 ? 256u : 0u) + (slot >> 1);
        if (V == 2) dword = 4u * slot + (lane & 3u);
        if (V == 3) dword = slot;
        if (V == 4) dword = ((slot >> 1) + (lane >= 32 ? 16u : 0u)) & 255u;
        if (V >= 5) dword = (slot >> (V - 4)) >> 1;
        dw[dword % 32].insert(dword);
      }
      size_t mx = 0;
      for (auto& b : dw) mx = b.size() > mx ? b.size() : mx;
      extra += (double)mx - 1.0;
    }
  }
  return extra / trials;
}

#define CHK(x)                                                             \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

template <int V>
static int run(unsigned* d, int blocks, const char* name) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  k_probe<V><<<blocks, 256>>>(d, 1u);  // warm-up
  CHK(hipEventRecord(a));
  k_probe<V><<<blocks, 256>>>(d, 2u);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const double insts = (double)blocks * 4 * kIters * kUnroll;  // wave-level probe instructions
  printf("{\"variant\": \"%s\", \"ms\": %.4f, \"ns_per_probe_inst_per_cu\": %.4f, \"mc_extra_cycles\": %.3f}\n",
         name, ms, ms * 1e6 / (insts / cus), mc(V, 20000));
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "--mc")) {
    for (int v = 0; v < 8; ++v) printf("V%d extra cycles per instruction %.3f\n", v, mc(v, 200000));
    return 0;
  }
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus * 8;
  unsigned* d = nullptr;
  CHK(hipMalloc(&d, (size_t)blocks * 256 * 4));
  if (run<0>(d, blocks, "V0_u16_512") || run<1>(d, blocks, "V1_two_half_wave_tables") ||
      run<2>(d, blocks, "V2_4way_interleaved") || run<3>(d, blocks, "V3_u32_512") ||
      run<4>(d, blocks, "V4_half_rotated") || run<5>(d, blocks, "V5_u16_256") ||
      run<6>(d, blocks, "V6_u16_128") || run<7>(d, blocks, "V7_u16_64"))
    return 1;
  CHK(hipFree(d));
  return 0;
}
