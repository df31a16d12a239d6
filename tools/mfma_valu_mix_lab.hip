// Lab (GPU, round 5): how much VALU / LDS-read issue one wave per SIMD can put beside v_mfma_f32_16x16x32_bf16 before
// the matrix pipe slows -- the question DESIGN §7b answers for an in-register NF4 decode inside k_hgemm (2 VALU +
// 0.5 ds_read_b64 per MFMA: per 2 weights one v_perm_b32, two v_mul_f32, one v_cvt_pk_bf16_f32, one table read).
// Each wave issues groups of 8 independent AGPR-accumulated MFMAs; between consecutive MFMAs it issues V2/2 VALU ops of
// the decode mix (independent of the MFMAs, rotating temporaries) and, every 2 MFMAs, L ds_read_b64 of a bank-clean
// LDS address; one lgkmcnt wait per group.  One workgroup of 4 waves per CU (the LDS claim keeps it to one).
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_valu_mix_lab.hip -o tools/_bin/mfma_valu_mix_lab
// Usage: tools/_bin/mfma_valu_mix_lab   (prints one line per configuration)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

template <int V2, int L>
__global__ void __launch_bounds__(256, 1) k_mix(int iters, float* __restrict__ sink) {
  extern __shared__ uint8_t lds[];
  const unsigned t = threadIdx.x;
  for (int i = t; i < 96 * 1024 / 4; i += 256) reinterpret_cast<unsigned*>(lds)[i] = i * 0x9E3779B9u;
  __syncthreads();
  const u32x4 av = {0x3F003F01u ^ t, 0x3F103F11u, 0x3F203F21u, 0x3F303F31u};
  const u32x4 bv = {0x3E803E81u, 0x3E903E91u ^ t, 0x3EA03EA1u, 0x3EB03EB1u};
  f32x4 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc[j]) : "v"(av), "v"(bv));
  unsigned p0 = t, p1 = t * 3u, tb = 0;
  float f0 = 1.0f + t, f1 = 2.0f, s0 = 0.5f, s1 = 0.25f, m0 = 0.f, m1 = 0.f;
  unsigned cv = 0;
  uint2 rd = {0u, 0u};
  const unsigned laddr = (unsigned)(uintptr_t)lds + ((t & 63) * 8) + ((t >> 6) * 4096);
  // one op of the decode mix, by index (perm, mul, mul, cvt)
  auto valu = [&](int k) {
    switch (k & 3) {
      case 0: asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(tb) : "v"(p0), "v"(p1), "v"(0x05010400u)); break;
      case 1: asm volatile("v_mul_f32 %0, %1, %2" : "=v"(m0) : "v"(f0), "v"(s0)); break;
      case 2: asm volatile("v_mul_f32 %0, %1, %2" : "=v"(m1) : "v"(f1), "v"(s1)); break;
      default: asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(cv) : "v"(f0), "v"(f1)); break;
    }
  };
  for (int it = 0; it < iters; ++it) {
    int k = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(av), "v"(bv));
      // V2 ops per 2 MFMAs: the first MFMA of the pair gets the odd one
      const int nv = (j & 1) ? V2 / 2 : V2 - V2 / 2;
#pragma unroll
      for (int v = 0; v < nv; ++v) valu(k++);
      if ((j & 1) && L > 0) {
#pragma unroll
        for (int l = 0; l < L; ++l) asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(rd) : "v"(laddr), "i"(512 * l));
      }
    }
    if (L > 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    p0 += tb; f0 += m0 + m1; p1 ^= cv + rd.x;
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  float s = f0 + (float)p1 + (float)p0;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    for (int r = 0; r < 4; ++r) s += acc[j][r];
  sink[blockIdx.x * 256 + t] = s;
}

template <int V2, int L>
static void run(float* sink, int blocks, int iters, double pure_ns) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto launch = [&] { hipLaunchKernelGGL((k_mix<V2, L>), dim3(blocks), dim3(256), 96 * 1024, 0, iters, sink); };
  for (int w = 0; w < 3; ++w) launch();
  hipEventRecord(a);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double per = ms * 1e6 / reps;
  const double flop = (double)blocks * 4 * 8 * iters * 16 * 16 * 32 * 2;
  std::printf("VALU per MFMA %.1f  ds_read_b64 per MFMA %.1f:  %8.1f us  %7.1f TFLOP/s  MFMA rate vs pure %.3f\n",
              V2 / 2.0, L / 2.0, per / 1e3, flop / per / 1e3, pure_ns > 0 ? pure_ns / per : 1.0);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

template <int V2, int L>
static double time_only(float* sink, int blocks, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_mix<V2, L>), dim3(blocks), dim3(256), 96 * 1024, 0, iters, sink);
  hipEventRecord(a);
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL((k_mix<V2, L>), dim3(blocks), dim3(256), 96 * 1024, 0, iters, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms * 1e6 / 10;
}

int main() {
  const int blocks = 256 * 4, iters = 4000;
  float* sink = nullptr;
  if (hipMalloc(&sink, (size_t)blocks * 256 * sizeof(float)) != hipSuccess) return 1;
  const double pure = time_only<0, 0>(sink, blocks, iters);
  run<0, 0>(sink, blocks, iters, pure);
  run<1, 0>(sink, blocks, iters, pure);
  run<2, 0>(sink, blocks, iters, pure);
  run<3, 0>(sink, blocks, iters, pure);
  run<4, 0>(sink, blocks, iters, pure);
  run<6, 0>(sink, blocks, iters, pure);
  run<8, 0>(sink, blocks, iters, pure);
  run<0, 1>(sink, blocks, iters, pure);
  run<2, 1>(sink, blocks, iters, pure);
  run<4, 1>(sink, blocks, iters, pure);
  run<4, 2>(sink, blocks, iters, pure);
  run<6, 1>(sink, blocks, iters, pure);
  hipFree(sink);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
