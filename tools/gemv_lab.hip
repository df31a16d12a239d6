// Decode GEMV design lab: times kernel variants of the 4-bit M=1 product on synthetic data
// (11008 x 4096 NF4 weight, bs 64, 14 rotating copies > MALL).  Not part of the library.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I../bitsandbytes-sycl_amd/csrc gemv_lab.hip -o gemv_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "common.hpp"
#include "gemm_common.hpp"

using namespace bnb;
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float dot2(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), c, false);
}

// MODE 0: shared 256-entry pair LUT; MODE 1: no LUT (memory floor); MODE 2: 32 bank-private LUT copies
// addressed by v_perm (byte*256 + lane4)
template <int MODE, int R, int U, int NT, int THREADS>
__global__ void __launch_bounds__(THREADS)
k_lab(int M, int K, const uint16_t* __restrict__ A, const uint8_t* __restrict__ B, const float* __restrict__ absmax,
      const float* __restrict__ datatype, uint16_t* __restrict__ out, int ldb, int bs_shift) {
  extern __shared__ __attribute__((aligned(16))) uint32_t gsm[];
  constexpr int LUT_DW = (MODE == 2 || MODE == 5) ? 16384 : MODE == 6 ? 8192 : 256;
  uint32_t* lut = gsm;
  uint32_t* xs = gsm + LUT_DW;
  constexpr int WPB = THREADS / 64;
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * WPB + (threadIdx.x >> 6)) * R;
  const int nch = K >> 5;
  const long long two_ldb = 2LL * ldb;
  uint4 b[U][R];
  float am[U][R];
  typedef const __attribute__((address_space(1))) uint8_t* gbyte_p;
  typedef const __attribute__((address_space(1))) float* gfloat_p;
  typedef const __attribute__((address_space(1))) u32x4_t* gvec_p;
  const uint8_t* Bq = B;
  const float* Aq = absmax;
  constexpr int NB = 2048 / THREADS;
  uint32_t tv[NB];
  if constexpr (MODE >= 3) {
    // table first, then x by LDS-DMA (older than every weight load), then the weights
    if constexpr (MODE == 3 || MODE == 4)
      for (int i = threadIdx.x; i < 256; i += THREADS) lut[i] = pack_bf16x2(datatype[i >> 4], datatype[i & 15]);
    if constexpr (MODE == 5 || MODE == 6)
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        const int e = (threadIdx.x + k * THREADS) >> 3;
        tv[k] = pack_bf16x2(datatype[e >> 4], datatype[e & 15]);
      }
    const int nx = K >> 3, wave = threadIdx.x >> 6;
    for (int j = 0; j * THREADS < nx; ++j) {
      const int idx = (j * WPB + wave) * 64 + lane;
      if (idx < nx) glds16(A + 8 * idx, reinterpret_cast<uint8_t*>(xs) + (j * WPB + wave) * 1024);
    }
    // launder the weight pointers so their loads stay between the DMA and the vmcnt wait below
    uintptr_t bp = (uintptr_t)B, ap = (uintptr_t)absmax;
    asm volatile("" : "+s"(bp), "+s"(ap)::"memory");
    Bq = (const uint8_t*)bp;
    Aq = (const float*)ap;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = min(lane + 64 * u, nch - 1);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = min(row0 + r, M - 1);
      if (NT) {
        const u32x4_t v = __builtin_nontemporal_load((gvec_p)((gbyte_p)Bq + (long long)row * ldb + 16LL * c));
        b[u][r] = make_uint4(v.x, v.y, v.z, v.w);
      }
      else b[u][r] = *reinterpret_cast<const uint4*>(Bq + (long long)row * ldb + 16LL * c);
      am[u][r] = ((gfloat_p)Aq)[(two_ldb * row + 32LL * c) >> bs_shift];
    }
  }
  if (MODE == 0) {
    for (int i = threadIdx.x; i < 256; i += THREADS) lut[i] = pack_bf16x2(datatype[i >> 4], datatype[i & 15]);
  } else if (MODE == 2) {
    // entry e at dwords [64e, 64e+32): copy j in bank j
    for (int i = threadIdx.x; i < 256 * 8; i += THREADS) {
      const int e = i >> 3, q = i & 7;
      const uint32_t v = pack_bf16x2(datatype[e >> 4], datatype[e & 15]);
      reinterpret_cast<uint4*>(lut)[e * 16 + q] = make_uint4(v, v, v, v);
    }
  }
  if constexpr (MODE == 5 || MODE == 6) {
    // bank-private copies: entry e for lane-bank j at byte e*STRIDE + 4j (STRIDE 256 for v_perm addressing)
    constexpr int STRIDE = MODE == 5 ? 256 : 128;
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int i = threadIdx.x + k * THREADS, e = i >> 3, q = i & 7;
      *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(lut) + e * STRIDE + 16 * q) = make_uint4(tv[k], tv[k], tv[k], tv[k]);
    }
  }
  if constexpr (MODE >= 3) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * R * U) : "memory");   // x landed; weights still in flight
    __builtin_amdgcn_s_waitcnt(0xC07F);                                   // lgkmcnt(0): table writes
    __builtin_amdgcn_s_barrier();
  } else {
    for (int i = threadIdx.x; i < (K >> 3); i += THREADS) reinterpret_cast<uint4*>(xs)[i] = reinterpret_cast<const uint4*>(A)[i];
    __syncthreads();
  }
  if (row0 >= M) return;
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0f;
  const uint32_t lane4 = (lane & 31) * 4;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool valid = lane + 64 * u < nch;
    const int c = min(lane + 64 * u, nch - 1);
    uint32_t x[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(xs + 16 * c)[q];
      x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t w[4] = {b[u][r].x, b[u][r].y, b[u][r].z, b[u][r].w};
      uint32_t l[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (MODE == 5) {
          const uint32_t sel = 0x0C0C0000u | ((4u + (uint32_t)(i & 3)) << 8);
          const uint32_t addr = __builtin_amdgcn_perm(w[i >> 2], lane4, sel);
          l[i] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(lut) + addr);
        } else if (MODE == 6) {
          const uint32_t addr = (((w[i >> 2] >> (8 * (i & 3))) & 0xFF) << 7) | lane4;
          l[i] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(lut) + addr);
        } else if (MODE == 0 || MODE == 3) l[i] = lut[(w[i >> 2] >> (8 * (i & 3))) & 0xFF];
        else if (MODE == 1 || MODE == 4) l[i] = w[i >> 2];
        else {
          // byte i&3 of w -> bits 8..15, lane4 -> bits 0..7
          const uint32_t sel = 0x0C0C0000u | ((4u + (uint32_t)(i & 3)) << 8);   // src0 bytes are 4..7
          const uint32_t addr = __builtin_amdgcn_perm(w[i >> 2], lane4, sel);
          l[i] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(lut) + addr);
        }
      }
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        s0 = dot2(x[i], l[i], s0);
        s1 = dot2(x[i + 1], l[i + 1], s1);
      }
      const float part = (s0 + s1) * am[u][r];
      acc[r] += valid ? part : 0.0f;
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (row0 + r < M) out[row0 + r] = (uint16_t)(__float_as_uint(acc[r]) >> 16);
  }
}

template <int MODE> constexpr int LUTB() { return ((MODE == 2 || MODE == 5) ? 16384 : MODE == 6 ? 8192 : 256) * 4; }
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
  const int N = 11008, K = 4096, BS = 64, COPIES = 14, REPS = 20;
  const size_t wbytes = (size_t)N * K / 2, nabs = (size_t)N * K / BS;
  std::vector<uint8_t*> Bs(COPIES);
  std::vector<float*> As(COPIES);
  std::vector<uint8_t> hb(wbytes);
  std::vector<float> ha(nabs);
  srand(1);
  for (auto& v : hb) v = rand() & 0xFF;
  for (auto& v : ha) v = 0.01f + (rand() & 1023) / 1024.0f;
  for (int i = 0; i < COPIES; ++i) {
    CK(hipMalloc(&Bs[i], wbytes));
    CK(hipMalloc(&As[i], nabs * 4));
    CK(hipMemcpy(Bs[i], hb.data(), wbytes, hipMemcpyHostToDevice));
    CK(hipMemcpy(As[i], ha.data(), nabs * 4, hipMemcpyHostToDevice));
  }
  uint16_t *x, *out;
  float* code;
  CK(hipMalloc(&x, K * 2));
  CK(hipMalloc(&out, N * 2));
  CK(hipMalloc(&code, 64));
  std::vector<uint16_t> hx(K);
  for (auto& v : hx) v = 0x3F80 ^ (rand() & 0x807F);
  CK(hipMemcpy(x, hx.data(), K * 2, hipMemcpyHostToDevice));
  float hc[16];
  for (int i = 0; i < 16; ++i) hc[i] = (i - 7.5f) / 8.0f;
  CK(hipMemcpy(code, hc, 64, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = wbytes + nabs * 4.0 + K * 2 + N * 2;
  auto run = [&](const char* name, auto kern, int R, int threads, size_t lds) {
    const int waves = (N + R - 1) / R, wpb = threads / 64;
    const int grid = (waves + wpb - 1) / wpb;
    if (lds > 65536) CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    for (int i = 0; i < COPIES; ++i)
      hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), lds, 0, N, K, x, Bs[i], As[i], code, out, K / 2, 6);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < REPS; ++r)
      for (int i = 0; i < COPIES; ++i)
        hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), lds, 0, N, K, x, Bs[i], As[i], code, out, K / 2, 6);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / (REPS * COPIES);
    printf("%-34s %8.2f us  %7.0f GB/s\n", name, us, bytes / us / 1e3);
  };
  const size_t xl = K * 2;
#define RUN(MODE, R, U, NT, T) \
  run("mode" #MODE " R" #R " U" #U " nt" #NT " T" #T, k_lab<MODE, R, U, NT, T>, R, T, (size_t)LUTB<MODE>() + xl)
  RUN(3, 4, 2, 1, 256);
  RUN(4, 4, 2, 1, 256);
  RUN(5, 4, 2, 1, 512);
  RUN(5, 8, 2, 1, 256);
  RUN(5, 4, 2, 1, 256);
  RUN(6, 4, 2, 1, 512);
  RUN(6, 4, 2, 1, 256);
  RUN(6, 2, 2, 1, 256);
  return 0;
}
