// FETCH_SIZE calibration for the scoring kernels' access widths ("calibrate
// FETCH_SIZE for 4-B-per-lane word reads with a known-byte microkernel of this access
// pattern", MI355X_MICROARCH.md §HBM: FETCH_SIZE is calibrated only for 16 B per lane).
//
// Each kernel reads a 1 GiB buffer exactly once, in the scoring kernels' pattern: the 64
// lanes of a wave read 64 consecutive elements of one row (the candidate replica's
// [row][position] layout), one global load per lane per row, W bytes per lane
// (W = 2: rlen, 4: unit words / u32 codes, 8: bigram key words / rnum, 16: the guide's
// calibrated case).  Far larger than the 256 MiB Infinity Cache and read once, so every
// byte comes from HBM.  Every thread XORs its data into one word (nothing is dead code).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/micro/fetch_calib scripts/micro/fetch_calib.hip
// Run each width under its own PMC pass:
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE -d OUT -o pmc -- scripts/micro/fetch_calib
// factor(W) = 2^30 B / (FETCH_SIZE(kernel W) * 1024).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

template <typename T>
__global__ __launch_bounds__(256) void k_read(const T* __restrict__ p, uint64_t n, uint32_t* out) {
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = i0; i < n; i += stride) {
    const T v = p[i];
    if constexpr (sizeof(T) == 16) {
      const uint4 u = *reinterpret_cast<const uint4*>(&v);
      acc ^= u.x ^ u.y ^ u.z ^ u.w;
    } else if constexpr (sizeof(T) == 8) {
      acc ^= (uint32_t)v ^ (uint32_t)(v >> 32);
    } else {
      acc ^= (uint32_t)v;
    }
  }
  atomicXor(out, acc);  // keeps every lane's loads live (one atomic per thread: noise)
}

int main() {
  const size_t bytes = 1ull << 30;
  void* buf = nullptr;
  uint32_t* out = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  (void)hipMemset(buf, 0x5A, bytes);
  (void)hipDeviceSynchronize();
  const unsigned grid = 256 * 8;  // 8 workgroups per CU
  k_read<uint16_t><<<grid, 256>>>((const uint16_t*)buf, bytes / 2, out);
  k_read<uint32_t><<<grid, 256>>>((const uint32_t*)buf, bytes / 4, out);
  k_read<uint64_t><<<grid, 256>>>((const uint64_t*)buf, bytes / 8, out);
  k_read<uint4><<<grid, 256>>>((const uint4*)buf, bytes / 16, out);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("read %zu bytes per kernel: widths 2, 4, 8, 16 B per lane\n", bytes);
  (void)hipFree(buf);
  (void)hipFree(out);
  return 0;
}
