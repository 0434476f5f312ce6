// Issue rate of the integer VALU ops the Levenshtein DP uses, on gfx950: 8 independent
// chains per lane, 8 waves per SIMD; prints cycles per wave64 instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define OP_MIN3 "v_min3_u32 %0, %0, %1, %2"
#define OP_ADD "v_add_u32 %0, %0, %1"
#define OP_BFE "v_bfe_u32 %0, %1, 5, 1"
#define OP_BITOP3 "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96"
#define OP_PKMIN "v_pk_min_u16 %0, %0, %1"

template <int K>
__global__ __launch_bounds__(256) void k(unsigned* out, int iters, unsigned a, unsigned b) {
  unsigned x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  unsigned y = a + threadIdx.x, z = b ^ threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (K == 0) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 2) asm volatile("v_bfe_u32 %0, %0, 5, 1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 4) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 5) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 6) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 7) asm volatile("v_min_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 8) asm volatile("v_min_i32 %0, %0, %1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 9) asm volatile("v_min_u16 %0, %0, %1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 10) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 11) asm volatile("v_lshrrev_b32 %0, 1, %0" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 12) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 13) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 14) asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 15) asm volatile("v_alignbit_b32 %0, %0, %1, 3" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 16) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 17) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 18) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 19) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 20) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 21) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 22) asm volatile("v_max_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 23) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 24) asm volatile("v_min3_u16 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 25) asm volatile("v_sad_u8 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 26) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 27) asm volatile("v_add_u16 %0, %0, %1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 28) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 29) asm volatile("v_cmp_lt_u32 vcc, %0, %1" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
        if constexpr (K == 30) asm volatile("v_pk_minimum3_f16 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z) : "vcc");
      }
    }
  }
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// dependent chain: one accumulator, measures latency-bound rate with W waves per SIMD
template <int K>
__global__ __launch_bounds__(256) void kdep(unsigned* out, int iters, unsigned a, unsigned b) {
  unsigned x = threadIdx.x, y = a + threadIdx.x, z = b ^ threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 128; ++r) {
      if constexpr (K == 0) asm volatile(OP_MIN3 : "+v"(x) : "v"(y), "v"(z));
      if constexpr (K == 1) asm volatile(OP_ADD : "+v"(x) : "v"(y));
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = x;
}

template <typename F>
static void run(const char* name, F kern, int blocks, int iters, int per_iter, unsigned* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 2, 1u, 2u);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, iters, 1u, 2u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  int dev;
  hipGetDevice(&dev);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, dev);
  const double waves = blocks * 4.0, instr = waves * iters * per_iter;
  const double simds = p.multiProcessorCount * 4.0, clk = p.clockRate * 1e3;
  printf("%-12s blocks %5d  %.3f ms  %.2f cycles per wave-instr per SIMD (clk %.0f MHz, %d CUs)\n",
         name, blocks, ms, simds * clk * ms * 1e-3 / instr, clk / 1e6, p.multiProcessorCount);
}

int main() {
  unsigned* d;
  hipMalloc(&d, 1 << 26);
  int cus;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int b8 = cus * 8;  // 8 waves per SIMD (blocks of 4 waves, 8 blocks per CU)
  run("min3", k<0>, b8, 1000, 128, d);
  run("add", k<1>, b8, 1000, 128, d);
  run("bfe", k<2>, b8, 1000, 128, d);
  run("bitop3", k<3>, b8, 1000, 128, d);
  run("pk_min_u16", k<4>, b8, 1000, 128, d);
  run("pk_add_u16", k<5>, b8, 1000, 128, d);
  run("add_f32", k<6>, b8, 1000, 128, d);
  run("min_u32", k<7>, b8, 1000, 128, d);
  run("min_i32", k<8>, b8, 1000, 128, d);
  run("min_u16", k<9>, b8, 1000, 128, d);
  run("and", k<10>, b8, 1000, 128, d);
  run("lshr", k<11>, b8, 1000, 128, d);
  run("sub", k<12>, b8, 1000, 128, d);
  run("add3", k<13>, b8, 1000, 128, d);
  run("lshl_add", k<14>, b8, 1000, 128, d);
  run("alignbit", k<15>, b8, 1000, 128, d);
  run("perm", k<16>, b8, 1000, 128, d);
  run("mul_u24", k<17>, b8, 1000, 128, d);
  run("med3", k<18>, b8, 1000, 128, d);
  run("cndmask", k<19>, b8, 1000, 128, d);
  run("add_sdwa", k<20>, b8, 1000, 128, d);
  run("addc", k<21>, b8, 1000, 128, d);
  run("max_u32", k<22>, b8, 1000, 128, d);
  run("max3", k<23>, b8, 1000, 128, d);
  run("min3_u16", k<24>, b8, 1000, 128, d);
  run("sad_u8", k<25>, b8, 1000, 128, d);
  run("xad", k<26>, b8, 1000, 128, d);
  run("add_i16", k<27>, b8, 1000, 128, d);
  run("or3", k<28>, b8, 1000, 128, d);
  run("cmp_lt", k<29>, b8, 1000, 128, d);
  run("pk_minimum3_f16", k<30>, b8, 1000, 128, d);
  for (int w : {1, 2, 4, 8}) {
    char nm[32];
    snprintf(nm, sizeof nm, "dep min3 w%d", w);
    run(nm, kdep<0>, cus * w, 2000, 128, d);
    snprintf(nm, sizeof nm, "dep add w%d", w);
    run(nm, kdep<1>, cus * w, 2000, 128, d);
  }
  hipFree(d);
  return 0;
}
