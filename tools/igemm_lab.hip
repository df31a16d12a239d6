// int8 GEMM design lab: the library's 256x256 kernel (csrc/igemm_256.hip: BK = 128, 2 LDS stages, one
// barrier per k-step, fragments pipelined across it -- the 'cross-barrier' variant below, adopted) against
// a 3-stage variant (BK = 64 bytes, DMA two tiles ahead,
// counted vmcnt, raw s_barrier) on the fused igemmlt + mm_dequant path, row-major A [M,K], B [N,K].
// Outputs must be bit-identical (exact int32 + the same epilogue).  Usage: igemm_lab [M N K]
#include "igemm_256.hip"
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#include <functional>

namespace bnb {
hipStream_t current_stream() { return nullptr; }
void set_error(int, const char* what) { printf("error: %s\n", what); }

constexpr int K3_BK = 64, K3_TILE = 256 * K3_BK, K3_STAGE = 2 * K3_TILE;   // 16 KiB per operand, 32 KiB per stage
constexpr int K3_LDS = J_LDS_EPI > 3 * K3_STAGE ? J_LDS_EPI : 3 * K3_STAGE;

// [rows][64 B] tile, 16-B slot s of row r at slot s ^ (((r >> 3) & 1) << 1): the ds_read_b128 lane
// groups of a 16-row fragment read (rows l & 15, slot l >> 4) hit 16 distinct bank quads
__device__ __forceinline__ int swz64(int r, int s) { return r * 64 + ((s ^ (((r >> 3) & 1) << 1)) << 4); }

template <int FL>
__global__ void __launch_bounds__(J_THREADS, 1)
k_igemm_3s(int M, int N, int K, const int8_t* __restrict__ A, const int8_t* __restrict__ B, fp16_t* __restrict__ out,
           long long lda, long long ldb, long long ldc, const float* __restrict__ rowStats,
           const float* __restrict__ colStats, const fp16_t* __restrict__ bias) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[K3_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tilesN = (N + 255) / 256, tilesM = (M + 255) / 256;
  const int wg = xcd_remap(blockIdx.x, tilesN * tilesM);
  constexpr int GROUP = 4;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * 256, n0 = tn * 256;

  // DMA: piece p = 2*wave + i covers rows 16p .. 16p+15 (lane -> row 16p + (lane >> 2), LDS slot lane & 3)
  const int8_t* asrc[2];
  const int8_t* bsrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * (2 * wave + i) + (lane >> 2);
    const int gslot = (lane & 3) ^ (((row >> 3) & 1) << 1);
    asrc[i] = A + (long long)min(m0 + row, M - 1) * lda + 16 * gslot;
    bsrc[i] = B + (long long)min(n0 + row, N - 1) * ldb + 16 * gslot;
  }
  const int nk = K / K3_BK;
  auto dma = [&](int kt, int st) {
    const long long k0 = (long long)min(kt, nk - 1) * K3_BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      glds16(asrc[i] + k0, smem + st * K3_STAGE + (2 * wave + i) * 1024);
      glds16(bsrc[i] + k0, smem + st * K3_STAGE + K3_TILE + (2 * wave + i) * 1024);
    }
  };
  const int wm = wave >> 2, wn = wave & 3;
  i32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = i32x4_t{0, 0, 0, 0};

  dma(0, 0);
  dma(1, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");     // tile 0 landed (tile 1 may be in flight)
  __builtin_amdgcn_s_barrier();
  int st = 0;
  for (int t = 0; t < nk; ++t) {
    int st2 = st + 2;
    if (st2 >= 3) st2 -= 3;
    dma(t + 2, st2);                                    // stage of tile t-1: every wave passed its reads
    const uint8_t* as = smem + st * K3_STAGE;
    const uint8_t* bs = as + K3_TILE;
    const int slot = lane >> 4;
    uint4 b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const uint4*>(bs + swz64(64 * wn + 16 * j + (lane & 15), slot));
    if (FL & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint4 a = *reinterpret_cast<const uint4*>(as + swz64(128 * wm + 16 * i + (lane & 15), slot));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4_t, a), __builtin_bit_cast(i32x4_t, b[j]),
                                                          acc[i][j], 0, 0, 0);
    }
    if (FL & 1) __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // tile t+1 landed; tile t+2 stays in flight
    __builtin_amdgcn_s_waitcnt(0xC07F);                // this wave's LDS reads of tile t are done
    __builtin_amdgcn_s_barrier();
    st = st == 2 ? 0 : st + 1;
  }
  wait_vmcnt0();
  __syncthreads();

  // epilogue: fused mm_dequant (kernel_quant.cpp:3969 order), staged for 16-B stores
  const int grow0 = m0 + 128 * wm, gcol0 = n0 + 64 * wn;
  uint8_t* ep = smem + wave * (128 * J_EPI_STRIDE);
  float cs[4], bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = min(gcol0 + 16 * j + (lane & 15), N - 1);
    cs[j] = colStats[col];
    bv[j] = bias ? (float)bias[col] : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * i + 4 * (lane >> 4) + r;
      const float rs = rowStats[min(grow0 + row, M - 1)];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<fp16_t*>(ep + row * J_EPI_STRIDE + 2 * (16 * j + (lane & 15))) =
            mm_dequant_value(acc[i][j][r], rs, cs[j], bv[j]);
    }
  __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = lane + 64 * it;
    const int row = id >> 3, c8 = id & 7;
    const int grow = grow0 + row, gcol = gcol0 + 8 * c8;
    if (grow >= M || gcol + 8 > N) continue;
    const uint2 lo = *reinterpret_cast<const uint2*>(ep + row * J_EPI_STRIDE + 16 * c8);
    const uint2 hi = *reinterpret_cast<const uint2*>(ep + row * J_EPI_STRIDE + 16 * c8 + 8);
    *reinterpret_cast<uint4*>(out + (long long)grow * ldc + gcol) = make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
}

// Cross-barrier pipeline on the library geometry (BK = 128, 2 stages): the ks = 1 fragments are read
// into registers before the ks = 0 MFMAs, so after the barrier the wave reads tile t+1's ks = 0
// fragments while it runs tile t's ks = 1 MFMAs -- the barrier and the first LDS latency of a tile
// are covered by 32 MFMAs instead of exposed.
template <int FL>
__global__ void __launch_bounds__(J_THREADS, 1)
k_igemm_xb(int M, int N, int K, const int8_t* __restrict__ A, const int8_t* __restrict__ B, fp16_t* __restrict__ out,
           long long lda, long long ldb, long long ldc, const float* __restrict__ rowStats,
           const float* __restrict__ colStats, const fp16_t* __restrict__ bias) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[J_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tilesN = (N + 255) / 256, tilesM = (M + 255) / 256;
  const int wg = xcd_remap(blockIdx.x, tilesN * tilesM);
  constexpr int GROUP = 4;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * 256, n0 = tn * 256;
  const int8_t* asrc[4];
  const int8_t* bsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wave + i) + (lane >> 3);
    const int ks = 16 * ((lane & 7) ^ (row & 7));
    asrc[i] = A + (long long)min(m0 + row, M - 1) * lda + ks;
    bsrc[i] = B + (long long)min(n0 + row, N - 1) * ldb + ks;
  }
  auto dma = [&](int kt, int buf) {
    const long long k0 = (long long)kt * J_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      glds16(asrc[i] + k0, smem + buf * J_TILE + (4 * wave + i) * 1024);
      glds16(bsrc[i] + k0, smem + 2 * J_TILE + buf * J_TILE + (4 * wave + i) * 1024);
    }
  };
  const int wm = wave >> 2, wn = wave & 3;
  i32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = i32x4_t{0, 0, 0, 0};
  uint4 fa[2][8], fb[2][4];
  auto frag = [&](int buf, int ks, uint4 (&a)[8], uint4 (&b)[4]) {
    const uint8_t* as = smem + buf * J_TILE;
    const uint8_t* bs = smem + 2 * J_TILE + buf * J_TILE;
    const int slot = 4 * ks + (lane >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const uint4*>(bs + swz(64 * wn + 16 * j + (lane & 15), slot));
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const uint4*>(as + swz(128 * wm + 16 * i + (lane & 15), slot));
  };
  auto mma = [&](const uint4 (&a)[8], const uint4 (&b)[4]) {
    if (FL & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4_t, a[i]), __builtin_bit_cast(i32x4_t, b[j]),
                                                          acc[i][j], 0, 0, 0);
    if (FL & 1) __builtin_amdgcn_s_setprio(0);
  };
  const int nk = K / J_BK;
  dma(0, 0);
  if (nk > 1) dma(1, 1);
  if (nk > 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else wait_vmcnt0();
  __syncthreads();
  frag(0, 0, fa[0], fb[0]);
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    frag(s, 1, fa[1], fb[1]);
    mma(fa[0], fb[0]);
    if (FL & 2) __builtin_amdgcn_sched_barrier(0);      // keep the ks = 0 MFMAs ahead of the barrier
    wait_vmcnt0();                                     // tile t+1 landed (this wave's part)
    __builtin_amdgcn_s_waitcnt(0xC07F);                // this wave's reads of tile t are done
    __builtin_amdgcn_s_barrier();
    if (t + 2 < nk) dma(t + 2, s);
    if (t + 1 < nk) frag(s ^ 1, 0, fa[0], fb[0]);
    if (FL & 4) __builtin_amdgcn_sched_barrier(0);      // reads issued before the ks = 1 MFMAs
    mma(fa[1], fb[1]);
    if (FL & 2) __builtin_amdgcn_sched_barrier(0);
  }
  wait_vmcnt0();
  __syncthreads();

  const int grow0 = m0 + 128 * wm, gcol0 = n0 + 64 * wn;
  uint8_t* ep = smem + wave * (128 * J_EPI_STRIDE);
  float cs[4], bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = min(gcol0 + 16 * j + (lane & 15), N - 1);
    cs[j] = colStats[col];
    bv[j] = bias ? (float)bias[col] : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * i + 4 * (lane >> 4) + r;
      const float rs = rowStats[min(grow0 + row, M - 1)];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<fp16_t*>(ep + row * J_EPI_STRIDE + 2 * (16 * j + (lane & 15))) =
            mm_dequant_value(acc[i][j][r], rs, cs[j], bv[j]);
    }
  __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = lane + 64 * it;
    const int row = id >> 3, c8 = id & 7;
    const int grow = grow0 + row, gcol = gcol0 + 8 * c8;
    if (grow >= M || gcol + 8 > N) continue;
    const uint2 lo = *reinterpret_cast<const uint2*>(ep + row * J_EPI_STRIDE + 16 * c8);
    const uint2 hi = *reinterpret_cast<const uint2*>(ep + row * J_EPI_STRIDE + 16 * c8 + 8);
    *reinterpret_cast<uint4*>(out + (long long)grow * ldc + gcol) = make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
}

// One wave per SIMD: 256 threads = 4 waves (2 x 2), 128 x 128 outputs per wave (8 x 8 tiles, 256
// accumulator registers), so each fragment read from LDS feeds 8 MFMAs (4 in the 8-wave kernel).
// Same stages, swizzle and cross-barrier fragment pipeline as the library kernel.
__global__ void __launch_bounds__(256, 1)
k_igemm_w4(int M, int N, int K, const int8_t* __restrict__ A, const int8_t* __restrict__ B, fp16_t* __restrict__ out,
           long long lda, long long ldb, long long ldc, const float* __restrict__ rowStats,
           const float* __restrict__ colStats, const fp16_t* __restrict__ bias) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[J_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tilesN = (N + 255) / 256, tilesM = (M + 255) / 256;
  const int wg = xcd_remap(blockIdx.x, tilesN * tilesM);
  constexpr int GROUP = 4;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * 256, n0 = tn * 256;
  const int8_t* asrc[8];
  const int8_t* bsrc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = 8 * (8 * wave + i) + (lane >> 3);
    const int ks = 16 * ((lane & 7) ^ (row & 7));
    asrc[i] = A + (long long)min(m0 + row, M - 1) * lda + ks;
    bsrc[i] = B + (long long)min(n0 + row, N - 1) * ldb + ks;
  }
  auto dma = [&](int kt, int buf) {
    const long long k0 = (long long)kt * J_BK;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      glds16(asrc[i] + k0, smem + buf * J_TILE + (8 * wave + i) * 1024);
      glds16(bsrc[i] + k0, smem + 2 * J_TILE + buf * J_TILE + (8 * wave + i) * 1024);
    }
  };
  const int wm = wave >> 1, wn = wave & 1;
  i32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = i32x4_t{0, 0, 0, 0};
  uint4 fa[2][8], fb[2][8];
  auto frag = [&](int buf, int ks, uint4 (&a)[8], uint4 (&b)[8]) {
    const uint8_t* as = smem + buf * J_TILE;
    const uint8_t* bs = smem + 2 * J_TILE + buf * J_TILE;
    const int slot = 4 * ks + (lane >> 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = *reinterpret_cast<const uint4*>(bs + swz(128 * wn + 16 * j + (lane & 15), slot));
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const uint4*>(as + swz(128 * wm + 16 * i + (lane & 15), slot));
  };
  auto mma = [&](const uint4 (&a)[8], const uint4 (&b)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4_t, a[i]), __builtin_bit_cast(i32x4_t, b[j]),
                                                          acc[i][j], 0, 0, 0);
  };
  const int nk = K / J_BK;
  dma(0, 0);
  if (nk > 1) {
    dma(1, 1);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    wait_vmcnt0();
  }
  __syncthreads();
  frag(0, 0, fa[0], fb[0]);
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    frag(s, 1, fa[1], fb[1]);
    mma(fa[0], fb[0]);
    wait_vmcnt0();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    if (t + 2 < nk) dma(t + 2, s);
    if (t + 1 < nk) frag(s ^ 1, 0, fa[0], fb[0]);
    mma(fa[1], fb[1]);
  }
  __syncthreads();

  // epilogue: fused mm_dequant, two 64-column halves through the per-wave [128][64] staging
  const int grow0 = m0 + 128 * wm;
  uint8_t* ep = smem + wave * (128 * J_EPI_STRIDE);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int gcol0 = n0 + 128 * wn + 64 * h;
    float cs[4], bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = min(gcol0 + 16 * j + (lane & 15), N - 1);
      cs[j] = colStats[col];
      bv[j] = bias ? (float)bias[col] : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * i + 4 * (lane >> 4) + r;
        const float rs = rowStats[min(grow0 + row, M - 1)];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<fp16_t*>(ep + row * J_EPI_STRIDE + 2 * (16 * j + (lane & 15))) =
              mm_dequant_value(acc[i][4 * h + j][r], rs, cs[j], bv[j]);
      }
    __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int id = lane + 64 * it;
      const int row = id >> 3, c8 = id & 7;
      const int grow = grow0 + row, gcol = gcol0 + 8 * c8;
      if (grow >= M || gcol + 8 > N) continue;
      const uint2 lo = *reinterpret_cast<const uint2*>(ep + row * J_EPI_STRIDE + 16 * c8);
      const uint2 hi = *reinterpret_cast<const uint2*>(ep + row * J_EPI_STRIDE + 16 * c8 + 8);
      *reinterpret_cast<uint4*>(out + (long long)grow * ldc + gcol) = make_uint4(lo.x, lo.y, hi.x, hi.y);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
}

// v_mfma_i32_32x32x32_i8 variant of the library kernel (ROW A, ROW B, fused fp16 dequant): per wave 128 x 64 as
// 4 x 2 tiles of 32x32, k32 per MFMA (4 sub-steps per 128-B k-tile) -> 6 fragment reads per 8 MFMAs (the 16x16x64
// form reads 12 per 32).  Lane l holds 16 k of row l & 31, k-chunk l >> 5 (A and B alike); the (row >> 1) & 7 swizzle
// makes the 32-row fragment reads conflict-free.  D[r]: row 8 (r >> 2) + 4 (l >> 5) + (r & 3), col l & 31.
typedef __attribute__((ext_vector_type(16))) int i32x16_t;
__device__ __forceinline__ int swzh(int r, int s) { return r * 128 + ((s ^ ((r >> 1) & 7)) << 4); }

template <int FL>
__global__ void __launch_bounds__(J_THREADS, 1)
k_igemm_32(int M, int N, int K, const int8_t* __restrict__ A, const int8_t* __restrict__ B, fp16_t* __restrict__ out,
           long long lda, long long ldb, long long ldc, const float* __restrict__ rowStats,
           const float* __restrict__ colStats, const fp16_t* __restrict__ bias) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[J_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tilesN = (N + J_BN - 1) / J_BN, tilesM = (M + J_BM - 1) / J_BM;
  const int wg = xcd_remap(blockIdx.x, tilesN * tilesM);
  constexpr int GROUP = 4;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * J_BM, n0 = tn * J_BN;
  long long arow[4], brow[4];
  int kslot[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wave + i) + (lane >> 3);
    arow[i] = min(m0 + row, M - 1);
    brow[i] = min(n0 + row, N - 1);
    kslot[i] = 16 * ((lane & 7) ^ ((row >> 1) & 7));
  }
  auto dma = [&](int kt, int buf) {
    const long long k0 = (long long)kt * J_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      glds16(A + arow[i] * lda + k0 + kslot[i], smem + buf * J_TILE + (4 * wave + i) * 1024);
      glds16(B + brow[i] * ldb + k0 + kslot[i], smem + 2 * J_TILE + buf * J_TILE + (4 * wave + i) * 1024);
    }
  };
  const int wm = wave >> 2, wn = wave & 3;
  i32x16_t acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;
  // fragments of sub-steps (ks, ks + 1) in one set: a[2][4], b[2][2]
  auto frag = [&](int buf, int kp, uint4 (&a)[2][4], uint4 (&b)[2][2]) {
    const uint8_t* as = smem + buf * J_TILE;
    const uint8_t* bs = smem + 2 * J_TILE + buf * J_TILE;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int slot = 2 * (2 * kp + h) + (lane >> 5);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[h][j] = *reinterpret_cast<const uint4*>(bs + swzh(64 * wn + 32 * j + (lane & 31), slot));
#pragma unroll
      for (int i = 0; i < 4; ++i) a[h][i] = *reinterpret_cast<const uint4*>(as + swzh(128 * wm + 32 * i + (lane & 31), slot));
    }
  };
  auto mma = [&](const uint4 (&a)[2][4], const uint4 (&b)[2][2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i32x4_t, a[h][i]), __builtin_bit_cast(i32x4_t, b[h][j]),
                                                            acc[i][j], 0, 0, 0);
  };
  const int nk = K / J_BK;
  dma(0, 0);
  if (nk > 1) {
    dma(1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    wait_vmcnt0();
  }
  __syncthreads();
  uint4 fa[2][2][4], fb[2][2][2];
  frag(0, 0, fa[0], fb[0]);
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    frag(s, 1, fa[1], fb[1]);
    mma(fa[0], fb[0]);
    wait_vmcnt0();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    if (t + 2 < nk) dma(t + 2, s);
    if (t + 1 < nk) frag(s ^ 1, 0, fa[0], fb[0]);
    mma(fa[1], fb[1]);
  }
  __syncthreads();
  const int grow0 = m0 + 128 * wm, gcol0 = n0 + 64 * wn;
  uint8_t* ep = smem + wave * (128 * J_EPI_STRIDE);
  float cs[2], bv[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = min(gcol0 + 32 * j + (lane & 31), N - 1);
    cs[j] = colStats[col];
    bv[j] = bias ? (float)bias[col] : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * i + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
      const float rs = rowStats[min(grow0 + row, M - 1)];
#pragma unroll
      for (int j = 0; j < 2; ++j)
        *reinterpret_cast<fp16_t*>(ep + row * J_EPI_STRIDE + 2 * (32 * j + (lane & 31))) = mm_dequant_value(acc[i][j][r], rs, cs[j], bv[j]);
    }
  __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = lane + 64 * it;
    const int row = id >> 3, c8 = id & 7;
    const int grow = grow0 + row, gcol = gcol0 + 8 * c8;
    if (grow >= M) continue;
    const uint2 lo = *reinterpret_cast<const uint2*>(ep + row * J_EPI_STRIDE + 16 * c8);
    const uint2 hi = *reinterpret_cast<const uint2*>(ep + row * J_EPI_STRIDE + 16 * c8 + 8);
    fp16_t* dst = out + (long long)grow * ldc + gcol;
    if (gcol + 8 <= N) *reinterpret_cast<uint4*>(dst) = make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
}
}  // namespace bnb
using namespace bnb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 4096, K = argc > 3 ? atoi(argv[3]) : 11008;
  int8_t *A, *B;
  fp16_t *C0, *C1;
  float *rs, *cs;
  CK(hipMalloc(&A, (size_t)M * K)); CK(hipMalloc(&B, (size_t)N * K));
  CK(hipMalloc(&C0, (size_t)M * N * 2)); CK(hipMalloc(&C1, (size_t)M * N * 2));
  CK(hipMalloc(&rs, M * 4)); CK(hipMalloc(&cs, N * 4));
  {
    std::vector<int8_t> h((size_t)std::max(M, N) * K);
    srand(5);
    for (auto& v : h) v = (int8_t)((rand() % 255) - 127);
    CK(hipMemcpy(A, h.data(), (size_t)M * K, hipMemcpyHostToDevice));
    for (auto& v : h) v = (int8_t)((rand() % 255) - 127);
    CK(hipMemcpy(B, h.data(), (size_t)N * K, hipMemcpyHostToDevice));
    std::vector<float> f(std::max(M, N));
    for (auto& v : f) v = 0.5f + (rand() & 0xFFFF) / 65536.0f;
    CK(hipMemcpy(rs, f.data(), M * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(cs, f.data(), N * 4, hipMemcpyHostToDevice));
  }
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto lib = [&]() { launch_igemm_256<ROW, ROW, EPI_F16_ROW_DEQUANT>(M, N, K, A, B, C0, nullptr, K, K, N, rs, cs, nullptr); };
  auto v3 = [&](auto kern) {
    return [=]() { hipLaunchKernelGGL(kern, dim3(tiles), dim3(512), 0, 0, M, N, K, A, B, C1, (long long)K, (long long)K, (long long)N, rs, cs, (const fp16_t*)nullptr); };
  };
  auto time = [&](const char* name, auto fn) {
    for (int i = 0; i < 3; ++i) fn();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 30; ++i) fn();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / 30;
    printf("%-22s %8.1f us  %7.1f TOPS\n", name, us, 2.0 * M * N * K / us / 1e6);
    fflush(stdout);
  };
  for (int i = 0; i < 100; ++i) lib();
  CK(hipDeviceSynchronize());
  auto check = [&]() {
    std::vector<uint16_t> a((size_t)M * N), b((size_t)M * N);
    CK(hipMemcpy(a.data(), C0, a.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), C1, b.size() * 2, hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (size_t i = 0; i < a.size(); ++i) diff += a[i] != b[i];
    printf("  bit-identical: %s (%zu differ)\n", diff ? "NO" : "yes", diff);
  };
  // correctness once, then interleaved timing (clock under load drifts; alternate the variants)
  struct V { const char* name; std::function<void()> fn; std::vector<double> us; };
  std::vector<V> vs;
  vs.push_back({"lib 256 BK128 2-stage", lib, {}});
  vs.push_back({"3-stage BK64", v3(k_igemm_3s<0>), {}});
  vs.push_back({"cross-barrier", v3(k_igemm_xb<0>), {}});
  auto w4 = [=]() { hipLaunchKernelGGL(k_igemm_w4, dim3(tiles), dim3(256), 0, 0, M, N, K, (const int8_t*)A, (const int8_t*)B, C1, (long long)K, (long long)K, (long long)N, (const float*)rs, (const float*)cs, (const fp16_t*)nullptr); };
  vs.push_back({"one wave per SIMD", w4, {}});
  vs.push_back({"32x32x32 MFMA", v3(k_igemm_32<0>), {}});
  for (size_t v = 1; v < vs.size(); ++v) { vs[v].fn(); CK(hipDeviceSynchronize()); printf("%s", vs[v].name); check(); }
  for (int rep = 0; rep < 12; ++rep)
    for (auto& v : vs) {
      for (int i = 0; i < 2; ++i) v.fn();
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) v.fn();
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1e3 / 10);
    }
  for (auto& v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double med = v.us[v.us.size() / 2];
    printf("%-24s median %7.1f us  min %7.1f  max %7.1f  %7.1f TOPS\n", v.name, med, v.us.front(), v.us.back(), 2.0 * M * N * K / med / 1e6);
  }
  return 0;
}
