// DESIGN LAB (not built into the library): 256 x 256-tile fused 4-bit weight GEMM with ONE wave per
// SIMD (4 waves x 512 VGPRs).  Round-1 result at 4096x4096x11008: 355-358 us vs 345-347 us for
// csrc/gemm4bit_256.hip (profiles/lab/r01_nf4_gemm_designs_*.txt): 19 % more wave-cycles at a 16 %
// higher clock.  Across the three designs MFMA-busy x clock stays ~1.0e9 MFMA-cycles/s per SIMD.
// Wave w owns output columns n0 + 64w .. +63 for all 256 token rows:
// 8 x 2 accumulators of v_mfma_f32_32x32x16 (256 VGPRs), so each A fragment read from LDS feeds two
// MFMAs (half the LDS reads per MFMA of an 8-wave 256x256 tile) and the weights are dequantised in
// the lane that feeds them to the MFMA (no LDS round trip of the dequantised tile).
//   lane (c, h) = (lane & 31, lane >> 5), column fragment j: weight row n0 + 64w + 32j + c,
//   bytes 16h .. 16h+15 of the row's 32-byte k-step chunk -> dword ks = elements 32h + 8ks .. +7,
//   which the A operand of the same lane reads from 16-B slot 4h + ks of the activation row.
// Pair table (byte -> {code[hi], code[lo]}) in 32 bank-private copies addressed by one v_perm;
// two fp32 multiplies by absmax and one RNE cast per byte (kernel_quant.cpp:1428-1453 values).
// LDS: [0,64K) table, [64K,128K) 2 activation stages (LDS-DMA, XOR swizzle on the source),
//      [128K,152K) 3 packed-weight stages, [152K,155K) 3 absmax stages (all LDS-DMA).
#include "gemm_common.hpp"

namespace bnb {

constexpr int W4_BM = 256, W4_BN = 256, W4_BK = 64, W4_THREADS = 256;
constexpr int W4_LUT = 256 * 32 * 8;
constexpr int W4_XT = W4_BM * W4_BK * 2;        // 32 KiB
constexpr int W4_WT = W4_BN * W4_BK / 2;        // 8 KiB
constexpr int W4_AT = W4_BN * 4;                // 1 KiB
constexpr int W4_OFF_X = W4_LUT;
constexpr int W4_OFF_W = W4_OFF_X + 2 * W4_XT;
constexpr int W4_OFF_AM = W4_OFF_W + 3 * W4_WT;
constexpr int W4_LDS = W4_OFF_AM + 3 * W4_AT;   // 158,720 B

typedef float f32x2w_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2w_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int w4_swz(int r, int s) { return r * 128 + ((s ^ ((r >> 1) & 7)) << 4); }
__device__ __forceinline__ float w4_mul(float a, float b) {
  float r;
  asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <typename T> __device__ __forceinline__ uint32_t w4_cvt2(float lo, float hi);
template <> __device__ __forceinline__ uint32_t w4_cvt2<bf16_t>(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2w_t){lo, hi}, bf16x2w_t));
}
template <> __device__ __forceinline__ uint32_t w4_cvt2<fp16_t>(float lo, float hi) { return Mfma<fp16_t>::pack2(lo, hi); }

// FL: 1 = no activation DMA in the loop, 2 = no dequant (raw bytes as B), 4 = s_setprio around MFMAs
template <typename T, int FL = 0>
__global__ void __launch_bounds__(W4_THREADS, 1)
k_gemm_4bit_w4(int N, int M, int K, const T* __restrict__ A, const uint8_t* __restrict__ B,
               const float* __restrict__ absmax, const float* __restrict__ datatype, T* __restrict__ out,
               int lda, int ldb, int ldc, int blocksize) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[W4_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 31, h = lane >> 5;

  // ---- pair table: thread (j = tid & 31, g = tid >> 5 in 0..7) writes entries 32g .. 32g+31 of copy j
  {
    const int j = tid & 31, g = tid >> 5;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const float vhi = datatype[2 * g + s];
      float2* dst = reinterpret_cast<float2*>(smem + 256 * 16 * (2 * g + s) + 8 * j);
#pragma unroll
      for (int lo = 0; lo < 16; ++lo) dst[32 * lo] = make_float2(vhi, datatype[lo]);
    }
  }

  const int tilesN = (N + W4_BN - 1) / W4_BN, tilesM = (M + W4_BM - 1) / W4_BM;
  const int wg = xcd_remap(blockIdx.x, tilesN * tilesM);
  constexpr int GROUP = 4;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * W4_BM, n0 = tn * W4_BN;

  // ---- DMA roles.  X: piece i of wave w fills rows 8(8w+i) .. +7.  W: piece p of wave w fills rows
  // 64w + 32p .. +31 (lane l -> row l >> 1, half l & 1).  absmax: lane l -> row 64w + l.
  const T* xsrc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = 8 * (8 * wave + i) + (lane >> 3);
    xsrc[i] = A + (long long)min(m0 + row, M - 1) * lda + 8 * ((lane & 7) ^ ((row >> 1) & 7));
  }
  const uint8_t* wsrc[2];
#pragma unroll
  for (int p = 0; p < 2; ++p)
    wsrc[p] = B + (long long)min(n0 + 64 * wave + 32 * p + (lane >> 1), N - 1) * ldb + 16 * (lane & 1);
  const long long abase = 2LL * ldb * min(n0 + 64 * wave + lane, N - 1);
  const int bs_shift = __builtin_ctz(blocksize);
  const uint32_t lanebase = 8u * c;
  const int nk = K / W4_BK;

  auto dma_x = [&](int kt, int buf, int i) {
    glds16(xsrc[i] + (long long)kt * W4_BK, smem + W4_OFF_X + buf * W4_XT + (8 * wave + i) * 1024);
  };
  auto dma_w = [&](int kt) {
    const int st = kt % 3;
#pragma unroll
    for (int p = 0; p < 2; ++p)
      glds16(wsrc[p] + (long long)kt * (W4_BK / 2), smem + W4_OFF_W + st * W4_WT + (2 * wave + p) * 1024);
    glds4(absmax + ((abase + (long long)kt * W4_BK) >> bs_shift), smem + W4_OFF_AM + st * W4_AT + wave * 256);
  };
  auto read_w = [&](int kt, uint32_t (&wd)[2][4], float (&am)[2]) {
    const int st = kt % 3;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int rl = 64 * wave + 32 * j + c;
      const uint4 v = *reinterpret_cast<const uint4*>(smem + W4_OFF_W + st * W4_WT + 32 * rl + 16 * h);
      wd[j][0] = v.x; wd[j][1] = v.y; wd[j][2] = v.z; wd[j][3] = v.w;
      am[j] = *reinterpret_cast<const float*>(smem + W4_OFF_AM + st * W4_AT + 4 * rl);
    }
  };
  auto lut_read = [&](uint32_t wd, float2 (&cv)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t addr = __builtin_amdgcn_perm(wd, lanebase, 0x0C0C0000u | ((4u + q) << 8));
      cv[q] = *reinterpret_cast<const float2*>(smem + addr);
    }
  };
  auto finish = [&](const float2 (&cv)[4], float am) -> uint4 {
    uint32_t p[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) p[q] = w4_cvt2<T>(w4_mul(cv[q].x, am), w4_mul(cv[q].y, am));
    return make_uint4(p[0], p[1], p[2], p[3]);
  };
  auto fake_b = [&](uint32_t wd) { return make_uint4(wd, wd ^ 0x11111111u, wd >> 1, wd + 7u); };
  auto read_a = [&](const uint8_t* xs, int ks, uint4 (&a)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const uint4*>(xs + w4_swz(32 * i + c, 4 * h + ks));
  };

  f32x16_t acc[8][2];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // ---- prologue
#pragma unroll
  for (int i = 0; i < 8; ++i) dma_x(0, 0, i);
  dma_w(0);
  dma_w(min(1, nk - 1));
  wait_vmcnt0();
  __syncthreads();

  uint32_t wd[2][4];
  float am[2];
  uint4 b[2][2];          // [ks parity][j]
  float2 cv[2][4];
  read_w(0, wd, am);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (FL & 2) b[0][j] = fake_b(wd[j][0]);
    else { lut_read(wd[j][0], cv[j]); b[0][j] = finish(cv[j], am[j]); }
  }

  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    const uint8_t* xs = smem + W4_OFF_X + s * W4_XT;
    uint4 a[2][8];
    read_a(xs, 0, a[0]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int cur = ks & 1, nxt = cur ^ 1;
      uint32_t wn[2][4];
      float amn[2] = {am[0], am[1]};
      // operands of the next sub-step in flight
      if (ks < 3) {
        if (!(FL & 2)) { lut_read(wd[0][ks + 1], cv[0]); lut_read(wd[1][ks + 1], cv[1]); }
        read_a(xs, ks + 1, a[nxt]);
      } else if (t + 1 < nk) {
        read_w(t + 1, wn, amn);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (FL & 4) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = Mfma32<T>::mma(a[cur][i], b[cur][j], acc[i][j]);
      if (FL & 4) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if (ks == 0) {
        if (!(FL & 1)) {
#pragma unroll
          for (int i = 0; i < 8; ++i) dma_x(min(t + 1, nk - 1), s ^ 1, i);
        }
        dma_w(min(t + 2, nk - 1));
      }
      if (ks < 3) {
#pragma unroll
        for (int j = 0; j < 2; ++j) b[nxt][j] = (FL & 2) ? fake_b(wd[j][ks + 1]) : finish(cv[j], am[j]);
      } else if (t + 1 < nk) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
#pragma unroll
          for (int q = 0; q < 4; ++q) wd[j][q] = wn[j][q];
          am[j] = amn[j];
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (FL & 2) b[nxt][j] = fake_b(wd[j][0]);
          else { lut_read(wd[j][0], cv[j]); b[nxt][j] = finish(cv[j], am[j]); }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (FL & 4) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 4; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = Mfma32<T>::mma(a[cur][i], b[cur][j], acc[i][j]);
      if (FL & 4) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // b[0] now holds B(ks = 0) of step t+1 (ks = 3 wrote b[nxt = 0])
    wait_vmcnt0();
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- epilogue: per-wave [256][64] T staged in LDS (128-B rows), 16-B stores of 128 B per row
  uint8_t* ep = smem + wave * (256 * 128);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 32 * i + 8 * (r >> 2) + 4 * h + (r & 3);
        *reinterpret_cast<T*>(ep + row * 128 + 2 * (32 * j + c)) = Io<T>::from_f32(acc[i][j][r]);
      }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  const int gcol0 = n0 + 64 * wave;
  const bool vec_ok = ((ldc & 7) == 0) && (((uintptr_t)out & 15) == 0);
#pragma unroll
  for (int it = 0; it < 32; ++it) {
    const int id = lane + 64 * it;
    const int row = id >> 3, part = id & 7;
    const int grow = m0 + row, gcol = gcol0 + 8 * part;
    if (grow >= M) continue;
    const uint4 v = *reinterpret_cast<const uint4*>(ep + row * 128 + 16 * part);
    T* dst = out + (long long)grow * ldc + gcol;
    if (vec_ok && gcol + 8 <= N) {
      *reinterpret_cast<uint4*>(dst) = v;
    } else {
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      for (int e = 0; e < 8 && gcol + e < N; ++e) dst[e] = __builtin_bit_cast(T, (uint16_t)(w4[e >> 1] >> (16 * (e & 1))));
    }
  }
}

}  // namespace bnb
