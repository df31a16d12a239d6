// Measured ceilings for the bench's roofline ("report both the spec and the measured peak").
//   k_probe_mfma<bf16 | i8>: the dense MFMA issue rate the chip holds on random operands -- one wave per SIMD
//     (256 threads per CU), operands in registers, 8 independent accumulators per wave, the 16x16 shapes the GEMMs use
//     (v_mfma_f32_16x16x32_bf16, v_mfma_i32_16x16x64_i8).  No memory traffic in the loop; the accumulators are
//     written once at the end so nothing is dead code.
//   k_probe_hbm_read: the HBM streaming read ceiling -- every lane keeps 8 x 16-B non-temporal loads in flight over
//     a buffer larger than the 256 MB Infinity Cache, xor-folded, one dword per workgroup written.
// Not on the product path: bench.py calls them once to put measured peaks beside the spec peaks.
#include "common.hpp"

namespace bnb {

typedef __attribute__((ext_vector_type(8))) __bf16 pb_bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float pb_f32x4_t;
typedef __attribute__((ext_vector_type(4))) int pb_i32x4_t;

template <int KIND>
__global__ void __launch_bounds__(512, 1) k_probe_mfma(int iters, uint32_t seed, float* __restrict__ sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  // random operand bits per lane (bf16: exponent kept in range, so the products are ordinary values)
  auto rnd = [&](uint32_t i) {
    uint32_t x = (t * 0x9E3779B9u) ^ (seed + i * 0x85EBCA6Bu);
    x ^= x >> 15; x *= 0x2C1B3C6Du; x ^= x >> 12; x *= 0x297A2D39u; x ^= x >> 15;
    return x;
  };
  uint4 a, b;
  if constexpr (KIND == 0) {
    auto bf = [&](uint32_t i) { return (rnd(i) & 0x807F807Fu) | 0x3F003F00u; };   // |v| in [0.5, 1)
    a = make_uint4(bf(0), bf(1), bf(2), bf(3));
    b = make_uint4(bf(4), bf(5), bf(6), bf(7));
  } else {
    a = make_uint4(rnd(0), rnd(1), rnd(2), rnd(3));
    b = make_uint4(rnd(4), rnd(5), rnd(6), rnd(7));
  }
  // accumulators pinned to AGPRs by inline asm (with the builtin, hipcc shuffles them through VGPRs every iteration
  // -- the pathology hgemm.hip documents -- and the loop measures the shuffles, not the matrix pipe)
  pb_f32x4_t accf[8];
  pb_i32x4_t acci[8];
  typedef __attribute__((ext_vector_type(4))) unsigned u4;
  const u4 av = __builtin_bit_cast(u4, a), bv = __builtin_bit_cast(u4, b);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if constexpr (KIND == 0) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(accf[j]) : "v"(av), "v"(bv));
    else asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, 0" : "=a"(acci[j]) : "v"(av), "v"(bv));
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (KIND == 0) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(accf[j]) : "v"(av), "v"(bv));
      else asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+a"(acci[j]) : "v"(av), "v"(bv));
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");   // MFMA -> accvgpr_read wait states (asm MFMAs)
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    for (int r = 0; r < 4; ++r) s += (KIND == 0) ? accf[j][r] : (float)acci[j][r];
  sink[t] = s;
}

typedef __attribute__((ext_vector_type(4))) unsigned pb_u32x4_t;

__global__ void __launch_bounds__(256) k_probe_hbm_read(const pb_u32x4_t* __restrict__ p, long long n16,
                                                        uint32_t* __restrict__ sink) {
  const long long stride = (long long)gridDim.x * 256;
  uint32_t x = 0;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 7 * stride < n16; i += 8 * stride) {
    pb_u32x4_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(p + i + u * stride);
#pragma unroll
    for (int u = 0; u < 8; ++u) x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n16; i += stride) {
    const pb_u32x4_t v = __builtin_nontemporal_load(p + i);
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x12345678u) sink[blockIdx.x] = x;   // practically never taken: keeps the loads live without traffic
}

}  // namespace bnb

// LDS poisoning (test support): every workgroup takes the whole 160 KiB LDS of its CU and fills it with `pattern`, so
// the next kernel's workgroups find that pattern in any LDS byte they read before writing it (LDS is not cleared
// between kernels).  With 0xFFFFFFFF (a NaN in fp32, bf16 and fp16) a kernel that reads a staged LDS slot before its
// DMA landed, or a slot its loads never write, returns NaN or different bits than an unpoisoned run
// (tests/test_lds_poison_gpu.py).  k_probe_lds_peek is the positive control: it reads LDS it never wrote.
constexpr int PB_LDS_WORDS = 160 * 1024 / 4;
__global__ void __launch_bounds__(256) k_probe_lds_poison(unsigned pattern) {
  __shared__ unsigned lds[PB_LDS_WORDS];
  for (int i = threadIdx.x; i < PB_LDS_WORDS; i += blockDim.x) lds[i] = pattern;
  __syncthreads();
  asm volatile("" ::"v"(lds[(threadIdx.x * 613) % PB_LDS_WORDS]));
}
__global__ void __launch_bounds__(256) k_probe_lds_peek(unsigned* __restrict__ out) {
  __shared__ unsigned lds[PB_LDS_WORDS];
  unsigned v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((unsigned)(uintptr_t)&lds[threadIdx.x * 157]));
  out[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

extern "C" {

// [additive, measurement] kind 0 = bf16 (v_mfma_f32_16x16x32_bf16), 1 = int8 (v_mfma_i32_16x16x64_i8), + 2 for
// 8-wave workgroups (two waves per SIMD) instead of 4: `blocks` workgroups, every wave issues 8 x iters MFMAs;
// sink >= blocks * 512 floats.  Returns 0 / 1 (bad kind) / 2 (launch).
int cprobe_mfma(int kind, int blocks, int iters, unsigned seed, float* sink) {
  BNB_RANGE("cprobe_mfma");
  const int threads = (kind & 2) ? 512 : 256;
  if ((kind & 1) == 0)
    hipLaunchKernelGGL((bnb::k_probe_mfma<0>), dim3(blocks), dim3(threads), 0, bnb::current_stream(), iters, seed, sink);
  else if (kind < 4)
    hipLaunchKernelGGL((bnb::k_probe_mfma<1>), dim3(blocks), dim3(threads), 0, bnb::current_stream(), iters, seed, sink);
  else
    return 1;
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
// [additive, measurement] streaming read of `bytes` (multiple of 16) at p by `blocks` workgroups of 256 threads;
// sink >= blocks dwords.
int cprobe_hbm_read(const void* p, long long bytes, int blocks, unsigned* sink) {
  BNB_RANGE("cprobe_hbm_read");
  hipLaunchKernelGGL(bnb::k_probe_hbm_read, dim3(blocks), dim3(256), 0, bnb::current_stream(),
                     reinterpret_cast<const bnb::pb_u32x4_t*>(p), bytes / 16, sink);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// [additive, testing] fill the LDS of every CU with `pattern` (blocks: >= the CU count; one launch on the current stream)
int cprobe_lds_poison(unsigned pattern, int blocks) {
  BNB_RANGE("cprobe_lds_poison");
  hipLaunchKernelGGL(k_probe_lds_poison, dim3(blocks), dim3(256), 0, bnb::current_stream(), pattern);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
// [additive, testing] positive control of the poisoning: out[b * 256 + t] = an LDS word the kernel never wrote
int cprobe_lds_peek(unsigned* out, int blocks) {
  BNB_RANGE("cprobe_lds_peek");
  hipLaunchKernelGGL(k_probe_lds_peek, dim3(blocks), dim3(256), 0, bnb::current_stream(), out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
}  // extern "C"
