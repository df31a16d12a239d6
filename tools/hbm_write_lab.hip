// Lab (GPU, round 5): the HBM write ceiling the 4-bit dequantise works against (k_dequantize_4bit_stream moves
// 1 byte read : 4 bytes written, 22.5 MB -> 90 MB at the metric shape, measured 4.4-5 TB/s in the step).
// Streams over a 2 GiB buffer (beyond the 256 MB MALL), 16-B stores per lane, 8 per lane per pass:
//   write-only with plain / write-through (sc1) / non-temporal (nt) stores, and the dequantise's mix (one 16-B load of a
//   separate 512 MiB source per 4 16-B stores), each as GB/s over the bytes moved.  Also a 90 MB write (the dequantise's
//   size) repeated back to back, MALL-resident after the first pass.
// Build: hipcc -O3 --offload-arch=gfx950 tools/hbm_write_lab.hip -o tools/_bin/hbm_write_lab
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int POL>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
  if constexpr (POL == 0) *p = v;
  else if constexpr (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(v) : "memory");
  else __builtin_nontemporal_store(v, p);
}

// write-only: every lane stores 16 B at i, i + stride, ... (grid-stride, 8 per pass)
template <int POL>
__global__ void __launch_bounds__(256) k_write(u32x4* __restrict__ dst, long long n16, unsigned seed) {
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const u32x4 v = {seed ^ (unsigned)i, seed, ~seed, (unsigned)threadIdx.x};
  for (; i + 7 * stride < n16; i += 8 * stride) {
#pragma unroll
    for (int u = 0; u < 8; ++u) st16<POL>(dst + i + u * stride, v);
  }
  for (; i < n16; i += stride) st16<POL>(dst + i, v);
}

// the dequantise's mix: per 16-B load of the source, four 16-B stores; like the dequantise, every store instruction
// writes 1 KiB contiguous (a wave's 64 loads at source index i0 + lane go to destination 4 i0 + 64 u + lane)
template <int POL>
__global__ void __launch_bounds__(256) k_mix(const u32x4* __restrict__ src, u32x4* __restrict__ dst, long long nsrc16) {
  const long long stride = (long long)gridDim.x * 256;
  const int lane = threadIdx.x & 63;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nsrc16; i += stride) {
    const u32x4 a = __builtin_nontemporal_load(src + i);
    const long long i0 = i - lane;
#pragma unroll
    for (int u = 0; u < 4; ++u) st16<POL>(dst + 4 * i0 + 64 * u + lane, a + (unsigned)u);
  }
}

static float time_ms(void (*fn)(void*), void* arg, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  fn(arg);
  (void)hipEventRecord(a);
  for (int r = 0; r < reps; ++r) fn(arg);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms / reps;
}

struct Args {
  u32x4* dst;
  const u32x4* src;
  long long n16;
  int blocks;
};

template <int POL> static void run_write(void* p) {
  Args* a = (Args*)p;
  hipLaunchKernelGGL(k_write<POL>, dim3(a->blocks), dim3(256), 0, 0, a->dst, a->n16, 7u);
}
template <int POL> static void run_mix(void* p) {
  Args* a = (Args*)p;
  hipLaunchKernelGGL(k_mix<POL>, dim3(a->blocks), dim3(256), 0, 0, a->src, a->dst, a->n16 / 4);
}

int main() {
  const long long big = 2LL << 30, src_bytes = 512LL << 20, small = 90LL << 20;
  u32x4 *dst = nullptr, *src = nullptr;
  if (hipMalloc(&dst, big) != hipSuccess || hipMalloc(&src, src_bytes) != hipSuccess) return 1;
  (void)hipMemset(src, 1, src_bytes);
  const char* pol[3] = {"plain", "sc1 (write-through)", "nt"};
  for (int blocks : {1024, 2048, 4096}) {
    Args w{dst, src, big / 16, blocks};
    float t[3] = {time_ms(run_write<0>, &w, 5), time_ms(run_write<1>, &w, 5), time_ms(run_write<2>, &w, 5)};
    for (int p = 0; p < 3; ++p)
      std::printf("write-only 2 GiB, %4d blocks, %-20s: %8.1f GB/s\n", blocks, pol[p], big / (t[p] * 1e6));
    Args m{dst, src, (src_bytes * 4) / 16, blocks};
    float tm[3] = {time_ms(run_mix<0>, &m, 5), time_ms(run_mix<1>, &m, 5), time_ms(run_mix<2>, &m, 5)};
    for (int p = 0; p < 3; ++p)
      std::printf("1:4 read:write (512 MiB -> 2 GiB), %4d blocks, %-20s: %8.1f GB/s moved\n", blocks, pol[p],
                  (src_bytes * 5) / (tm[p] * 1e6));
    Args s{dst, src, small / 16, blocks};
    float ts[3] = {time_ms(run_write<0>, &s, 20), time_ms(run_write<1>, &s, 20), time_ms(run_write<2>, &s, 20)};
    for (int p = 0; p < 3; ++p)
      std::printf("write-only 90 MiB back to back, %4d blocks, %-20s: %8.1f GB/s (%.1f us)\n", blocks, pol[p],
                  small / (ts[p] * 1e6), ts[p] * 1e3);
  }
  (void)hipFree(dst);
  (void)hipFree(src);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
