// NF4 GEMM design lab: the 256x256 kernel with parts switched off (FL bit 1: no in-loop DMA,
// 2: no dequant, 4: no per-step barrier) to find what bounds it.  Results are garbage for FL != 0.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstring>
#include "gemm_common.hpp"
namespace bnb {
constexpr int Q_BM = 256, Q_BN = 256, Q_BK = 64, Q_THREADS = 512;
constexpr int Q_XT = Q_BM * Q_BK * 2;          // 32 KiB
constexpr int Q_WT = Q_BN * Q_BK * 2;          // 32 KiB
constexpr int Q_PT = Q_BN * Q_BK / 2;          // 8 KiB
constexpr int Q_AT = 2 * Q_BN * 4;             // 2 KiB (absmax + spare copy)
constexpr int Q_OFF_X = 0;
constexpr int Q_OFF_W = 2 * Q_XT;
constexpr int Q_OFF_P = Q_OFF_W + 2 * Q_WT;
constexpr int Q_OFF_A = Q_OFF_P + 2 * Q_PT;
constexpr int Q_OFF_L = Q_OFF_A + 2 * Q_AT;
constexpr int Q_LDS = Q_OFF_L + 256 * 8;       // 151,552 B
constexpr int Q_EPI_STRIDE = 136;              // staged output row: 128 B + 8 B pad
static_assert(8 * 128 * Q_EPI_STRIDE <= Q_OFF_L, "epilogue staging must not overlap the LUT");

typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// one packed byte -> {T(code[hi]*am), T(code[lo]*am)} as a dword: ds_read_b64 of the pair table,
// v_pk_mul_f32 by the broadcast absmax, one v_cvt_pk (RNE) -- the reference's dequantised values.
template <typename T> __device__ __forceinline__ uint32_t deq_byte(const f32x2_t* lut, uint32_t byte, f32x2_t am2);
template <> __device__ __forceinline__ uint32_t deq_byte<bf16_t>(const f32x2_t* lut, uint32_t byte, f32x2_t am2) {
  const f32x2_t p = lut[byte] * am2;
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(p, bf16x2_t));
}
template <> __device__ __forceinline__ uint32_t deq_byte<fp16_t>(const f32x2_t* lut, uint32_t byte, f32x2_t am2) {
  const f32x2_t p = lut[byte] * am2;
  return Mfma<fp16_t>::pack2(p.x, p.y);
}

template <typename T>
__device__ __forceinline__ void dequant_slot_pair(uint8_t* ws, const float2* lut, uint32_t w0, uint32_t w1, float am,
                                                  int row, int slot0) {
  const uint32_t w[2] = {w0, w1};
  const f32x2_t am2 = {am, am};
  const f32x2_t* lut2 = reinterpret_cast<const f32x2_t*>(lut);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    uint32_t pk[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) pk[j] = deq_byte<T>(lut2, (w[s] >> (8 * j)) & 0xFF, am2);
    *reinterpret_cast<uint4*>(ws + swz(row, slot0 + s)) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  }
}

template <typename T, int FL>
__global__ void __launch_bounds__(Q_THREADS, 1)
k_lab(int N, int M, int K, const T* __restrict__ A, const uint8_t* __restrict__ B,
                const float* __restrict__ absmax, const float* __restrict__ datatype, T* __restrict__ out,
                int lda, int ldb, int ldc, int blocksize) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[Q_LDS];
  float2* lut = reinterpret_cast<float2*>(smem + Q_OFF_L);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);        // provably wave-uniform (SGPR math)
  if (tid < 256) lut[tid] = make_float2(datatype[tid >> 4], datatype[tid & 15]);

  // ---- tile order: XCD-contiguous ids, grouped 4 token-tiles x all feature-tiles
  const int tilesN = (N + Q_BN - 1) / Q_BN, tilesM = (M + Q_BM - 1) / Q_BM;
  const int wg = xcd_remap(blockIdx.x, tilesN * tilesM);
  constexpr int GROUP = 4;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * Q_BM, n0 = tn * Q_BN;

  // ---- DMA source addresses (k = 0); per k-step they advance by 64 elements / 32 bytes
  const T* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wave + i) + (lane >> 3);
    xsrc[i] = A + (long long)min(m0 + row, M - 1) * lda + 8 * ((lane & 7) ^ (row & 7));
  }
  const int prow = tid >> 1, phalf = tid & 1;                       // this lane's packed 16 B
  const uint8_t* psrc = B + (long long)min(n0 + prow, N - 1) * ldb + 16 * phalf;
  // absmax DMA: one row per lane; waves 4-7 repeat waves 0-3 into the stage's spare copy (branch-free)
  const int arow = 64 * (wave & 3) + lane;
  const int bs_shift = __builtin_ctz(blocksize);                    // blocksize: power of two >= 64
  const long long abase = 2LL * ldb * min(n0 + arow, N - 1);        // element index of (row, k = 0)

  const int nk = K / Q_BK;
  auto dma_w = [&](int kt, int buf) {                               // packed weights + absmax of k-tile kt
    glds16(psrc + (long long)kt * (Q_BK / 2), smem + Q_OFF_P + buf * Q_PT + wave * 1024);
    glds4(absmax + ((abase + (long long)kt * Q_BK) >> bs_shift), smem + Q_OFF_A + buf * Q_AT + wave * 256);
  };
  auto dma_x = [&](int kt, int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds16(xsrc[i] + (long long)kt * Q_BK, smem + Q_OFF_X + buf * Q_XT + (4 * wave + i) * 1024);
  };
  auto dequant_half = [&](int buf_src, int buf_dst, int h) {       // h = 0/1: first/second 8 packed bytes
    const uint8_t* p = smem + Q_OFF_P + buf_src * Q_PT + 16 * tid;
    const uint2 w = *reinterpret_cast<const uint2*>(p + 8 * h);
    const float am = *reinterpret_cast<const float*>(smem + Q_OFF_A + buf_src * Q_AT + 4 * prow);
    dequant_slot_pair<T>(smem + Q_OFF_W + buf_dst * Q_WT, lut, w.x, w.y, am, prow, 4 * phalf + 2 * h);
  };

  const int wm = wave >> 2, wn = wave & 3;
  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: X(0), W(0), W(1) in flight; dequantise W(0) into Ws[0]
  dma_x(0, 0);
  dma_w(0, 0);
  dma_w(min(1, nk - 1), 1);
  wait_vmcnt0();
  __syncthreads();
  dequant_half(0, 0, 0);
  dequant_half(0, 0, 1);
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    if (!(FL & 1)) {
      dma_x(min(t + 1, nk - 1), s ^ 1);
      dma_w(min(t + 2, nk - 1), s);
    }
    const uint8_t* xs = smem + Q_OFF_X + s * Q_XT;
    const uint8_t* ws = smem + Q_OFF_W + s * Q_WT;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int slot = 4 * ks + (lane >> 4);
      uint4 b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const uint4*>(ws + swz(64 * wn + 16 * j + (lane & 15), slot));
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint4 a = *reinterpret_cast<const uint4*>(xs + swz(128 * wm + 16 * i + (lane & 15), slot));
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = Mfma<T>::mma(a, b[j], acc[i][j]);
      }
      if (!(FL & 2)) dequant_half(s ^ 1, s ^ 1, ks);   // W(t+1): Wp[(t+1)&1] -> Ws[(t+1)&1]
    }
    wait_vmcnt0();
    if (!(FL & 4)) __syncthreads();
  }

  // ---- epilogue: acc -> LDS (per-wave [128][64] T, 136-B rows) -> 16-B coalesced stores
  uint8_t* ep = smem + wave * (128 * Q_EPI_STRIDE);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * i + 4 * (lane >> 4) + r, col = 16 * j + (lane & 15);
        *reinterpret_cast<T*>(ep + row * Q_EPI_STRIDE + 2 * col) = Io<T>::from_f32(acc[i][j][r]);
      }
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the wave reads back only its own region
  const int grow0 = m0 + 128 * wm, gcol0 = n0 + 64 * wn;
  const bool vec_ok = ((ldc & 7) == 0) && (((uintptr_t)out & 15) == 0);
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = lane + 64 * it;
    const int row = id >> 3, c8 = id & 7;
    const int grow = grow0 + row, gcol = gcol0 + 8 * c8;
    if (grow >= M) continue;
    const uint2 lo = *reinterpret_cast<const uint2*>(ep + row * Q_EPI_STRIDE + 16 * c8);
    const uint2 hi = *reinterpret_cast<const uint2*>(ep + row * Q_EPI_STRIDE + 16 * c8 + 8);
    T* dst = out + (long long)grow * ldc + gcol;
    if (vec_ok && gcol + 8 <= N) {
      *reinterpret_cast<uint4*>(dst) = make_uint4(lo.x, lo.y, hi.x, hi.y);
    } else {
      const uint32_t w4[4] = {lo.x, lo.y, hi.x, hi.y};
      for (int e = 0; e < 8 && gcol + e < N; ++e) dst[e] = __builtin_bit_cast(T, (uint16_t)(w4[e >> 1] >> (16 * (e & 1))));
    }
  }
}


// ---- variant: 32x32x16 MFMA, (r>>1)-XOR swizzle, scalar muls, conflict-free dequant writes
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
__device__ __forceinline__ int swz2(int r, int s) { return r * 128 + ((s ^ ((r >> 1) & 7)) << 4); }
__device__ __forceinline__ float mul_nopk(float a, float b) {
  float r;
  asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <int FL>
__global__ void __launch_bounds__(Q_THREADS, 1)
k_lab32(int N, int M, int K, const bf16_t* __restrict__ A, const uint8_t* __restrict__ B,
        const float* __restrict__ absmax, const float* __restrict__ datatype, bf16_t* __restrict__ out,
        int lda, int ldb, int ldc, int blocksize) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[Q_LDS];
  float2* lut = reinterpret_cast<float2*>(smem + Q_OFF_L);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid < 256) lut[tid] = make_float2(datatype[tid >> 4], datatype[tid & 15]);
  const int tilesN = (N + Q_BN - 1) / Q_BN, tilesM = (M + Q_BM - 1) / Q_BM;
  const int wg = xcd_remap(blockIdx.x, tilesN * tilesM);
  constexpr int GROUP = 4;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * Q_BM, n0 = tn * Q_BN;
  const bf16_t* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wave + i) + (lane >> 3);
    xsrc[i] = A + (long long)min(m0 + row, M - 1) * lda + 8 * ((lane & 7) ^ ((row >> 1) & 7));
  }
  // packed-weight DMA stays lane-linear: [256 rows][2 halves][16 B]
  const uint8_t* psrc = B + (long long)min(n0 + (tid >> 1), N - 1) * ldb + 16 * (tid & 1);
  const int arow = 64 * (wave & 3) + lane;
  const int bs_shift = __builtin_ctz(blocksize);
  const long long abase = 2LL * ldb * min(n0 + arow, N - 1);
  const int nk = K / Q_BK;
  auto dma_w = [&](int kt, int buf) {
    glds16(psrc + (long long)kt * (Q_BK / 2), smem + Q_OFF_P + buf * Q_PT + wave * 1024);
    glds4(absmax + ((abase + (long long)kt * Q_BK) >> bs_shift), smem + Q_OFF_A + buf * Q_AT + wave * 256);
  };
  auto dma_x = [&](int kt, int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds16(xsrc[i] + (long long)kt * Q_BK, smem + Q_OFF_X + buf * Q_XT + (4 * wave + i) * 1024);
  };
  // dequant role: 8 consecutive lanes take rows 2i+p (distinct XOR keys) -> conflict-free ds_write_b128
  const int g = lane & 31;
  const int drow = 16 * (tid >> 5) + 2 * (g & 7) + ((g >> 3) & 1);
  const int dhalf = (g >> 4) & 1;
  auto dequant_half = [&](int buf_src, int buf_dst, int h) {
    const uint8_t* p = smem + Q_OFF_P + buf_src * Q_PT + drow * 32 + 16 * dhalf;
    const uint2 w = *reinterpret_cast<const uint2*>(p + 8 * h);
    const float am = *reinterpret_cast<const float*>(smem + Q_OFF_A + buf_src * Q_AT + 4 * drow);
    const uint32_t ww[2] = {w.x, w.y};
    uint8_t* ws = smem + Q_OFF_W + buf_dst * Q_WT;
#pragma unroll
    for (int sidx = 0; sidx < 2; ++sidx) {
      uint32_t pk[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float2 c = lut[(ww[sidx] >> (8 * j)) & 0xFF];
        const float lo = mul_nopk(c.x, am), hi = mul_nopk(c.y, am);
        pk[j] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
      }
      *reinterpret_cast<uint4*>(ws + swz2(drow, 4 * dhalf + 2 * h + sidx)) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    }
  };
  const int wm = wave >> 2, wn = wave & 3;
  f32x16_t acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  dma_x(0, 0);
  dma_w(0, 0);
  dma_w(min(1, nk - 1), 1);
  wait_vmcnt0();
  __syncthreads();
  dequant_half(0, 0, 0);
  dequant_half(0, 0, 1);
  __syncthreads();
  if ((FL & 8) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    if (!(FL & 1) && !(FL & 16)) {
      dma_x(min(t + 1, nk - 1), s ^ 1);
      dma_w(min(t + 2, nk - 1), s);
    }
    const uint8_t* xs = smem + Q_OFF_X + s * Q_XT;
    const uint8_t* ws = smem + Q_OFF_W + s * Q_WT;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (FL & 16) {   // one X piece per ks, the weight pieces with the first
        glds16(xsrc[ks] + (long long)min(t + 1, nk - 1) * Q_BK, smem + Q_OFF_X + (s ^ 1) * Q_XT + (4 * wave + ks) * 1024);
        if (ks == 0) dma_w(min(t + 2, nk - 1), s);
      }
      const int slot = 2 * ks + (lane >> 5);
      uint4 b[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = *reinterpret_cast<const uint4*>(ws + swz2(64 * wn + 32 * j + (lane & 31), slot));
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint4 a = *reinterpret_cast<const uint4*>(xs + swz2(128 * wm + 32 * i + (lane & 31), slot));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b[j]),
                                                              acc[i][j], 0, 0, 0);
      }
      if (!(FL & 2) && (ks & 1)) dequant_half(s ^ 1, s ^ 1, ks >> 1);
    }
    wait_vmcnt0();
    if (!(FL & 4)) __syncthreads();
  }
  // epilogue: C/D 32x32: col = lane&31, row = 8*(r>>2) + 4*(lane>>5) + (r&3)
  uint8_t* ep = smem + wave * (128 * Q_EPI_STRIDE);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 32 * i + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3), col = 32 * j + (lane & 31);
        *reinterpret_cast<bf16_t*>(ep + row * Q_EPI_STRIDE + 2 * col) = Io<bf16_t>::from_f32(acc[i][j][r]);
      }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  const int grow0 = m0 + 128 * wm, gcol0 = n0 + 64 * wn;
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = lane + 64 * it;
    const int row = id >> 3, c8 = id & 7;
    const int grow = grow0 + row, gcol = gcol0 + 8 * c8;
    if (grow >= M) continue;
    const uint2 lo = *reinterpret_cast<const uint2*>(ep + row * Q_EPI_STRIDE + 16 * c8);
    const uint2 hi = *reinterpret_cast<const uint2*>(ep + row * Q_EPI_STRIDE + 16 * c8 + 8);
    *reinterpret_cast<uint4*>(out + (long long)grow * ldc + gcol) = make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
}
template <int FL>
__global__ void __launch_bounds__(Q_THREADS, 1)
k_lab32b(int N, int M, int K, const bf16_t* __restrict__ A, const uint8_t* __restrict__ B,
        const float* __restrict__ absmax, const float* __restrict__ datatype, bf16_t* __restrict__ out,
        int lda, int ldb, int ldc, int blocksize) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[Q_LDS];
  float2* lut = reinterpret_cast<float2*>(smem + Q_OFF_L);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid < 256) lut[tid] = make_float2(datatype[tid >> 4], datatype[tid & 15]);
  const int tilesN = (N + Q_BN - 1) / Q_BN, tilesM = (M + Q_BM - 1) / Q_BM;
  const int wg = xcd_remap(blockIdx.x, tilesN * tilesM);
  constexpr int GROUP = 4;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * Q_BM, n0 = tn * Q_BN;
  const bf16_t* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wave + i) + (lane >> 3);
    xsrc[i] = A + (long long)min(m0 + row, M - 1) * lda + 8 * ((lane & 7) ^ ((row >> 1) & 7));
  }
  // packed-weight DMA stays lane-linear: [256 rows][2 halves][16 B]
  const uint8_t* psrc = B + (long long)min(n0 + (tid >> 1), N - 1) * ldb + 16 * (tid & 1);
  const int arow = 64 * (wave & 3) + lane;
  const int bs_shift = __builtin_ctz(blocksize);
  const long long abase = 2LL * ldb * min(n0 + arow, N - 1);
  const int nk = K / Q_BK;
  auto dma_w = [&](int kt, int buf) {
    glds16(psrc + (long long)kt * (Q_BK / 2), smem + Q_OFF_P + buf * Q_PT + wave * 1024);
    glds4(absmax + ((abase + (long long)kt * Q_BK) >> bs_shift), smem + Q_OFF_A + buf * Q_AT + wave * 256);
  };
  auto dma_x = [&](int kt, int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds16(xsrc[i] + (long long)kt * Q_BK, smem + Q_OFF_X + buf * Q_XT + (4 * wave + i) * 1024);
  };
  // dequant role: 8 consecutive lanes take rows 2i+p (distinct XOR keys) -> conflict-free ds_write_b128
  const int g = lane & 31;
  const int drow = 16 * (tid >> 5) + 2 * (g & 7) + ((g >> 3) & 1);
  const int dhalf = (g >> 4) & 1;
  const int wm = wave >> 2, wn = wave & 3;
  f32x16_t acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // quarter q of this thread's 16 packed bytes -> one 16-B slot (8 bf16) of its W row
  auto lut_reads = [&](uint32_t word, float2 (&c)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = lut[(word >> (8 * j)) & 0xFF];
  };
  auto finish = [&](const float2 (&c)[4], float am, uint8_t* ws, int q) {
    uint32_t pk[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float lo = mul_nopk(c[j].x, am), hi = mul_nopk(c[j].y, am);
      pk[j] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
    }
    *reinterpret_cast<uint4*>(ws + swz2(drow, 4 * dhalf + q)) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  };
  auto dequant_all = [&](int buf) {   // prologue only
    const uint4 pw = *reinterpret_cast<const uint4*>(smem + Q_OFF_P + buf * Q_PT + drow * 32 + 16 * dhalf);
    const float am = *reinterpret_cast<const float*>(smem + Q_OFF_A + buf * Q_AT + 4 * drow);
    const uint32_t w4[4] = {pw.x, pw.y, pw.z, pw.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float2 c[4];
      lut_reads(w4[q], c);
      finish(c, am, smem + Q_OFF_W + buf * Q_WT, q);
    }
  };
  dma_x(0, 0);
  dma_w(0, 0);
  dma_w(min(1, nk - 1), 1);
  wait_vmcnt0();
  __syncthreads();
  dequant_all(0);
  __syncthreads();
  if ((FL & 8) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    const uint8_t* xs = smem + Q_OFF_X + s * Q_XT;
    const uint8_t* ws = smem + Q_OFF_W + s * Q_WT;
    uint8_t* wsn = smem + Q_OFF_W + (s ^ 1) * Q_WT;
    const uint4 pw = *reinterpret_cast<const uint4*>(smem + Q_OFF_P + (s ^ 1) * Q_PT + drow * 32 + 16 * dhalf);
    const float am = *reinterpret_cast<const float*>(smem + Q_OFF_A + (s ^ 1) * Q_AT + 4 * drow);
    const uint32_t w4[4] = {pw.x, pw.y, pw.z, pw.w};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (!(FL & 1)) {   // one X piece per ks, the weight pieces with the first
        glds16(xsrc[ks] + (long long)min(t + 1, nk - 1) * Q_BK, smem + Q_OFF_X + (s ^ 1) * Q_XT + (4 * wave + ks) * 1024);
        if (ks == 0) dma_w(min(t + 2, nk - 1), s);
      }
      const int slot = 2 * ks + (lane >> 5);
      uint4 b[2], a[4];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = *reinterpret_cast<const uint4*>(ws + swz2(64 * wn + 32 * j + (lane & 31), slot));
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const uint4*>(xs + swz2(128 * wm + 32 * i + (lane & 31), slot));
      float2 c[4];
      if (!(FL & 2)) lut_reads(w4[ks], c);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a[i]), __builtin_bit_cast(bf16x8_t, b[j]),
                                                              acc[i][j], 0, 0, 0);
      if (!(FL & 2)) finish(c, am, wsn, ks);
    }
    wait_vmcnt0();
    __syncthreads();
  }
  // epilogue: C/D 32x32: col = lane&31, row = 8*(r>>2) + 4*(lane>>5) + (r&3)
  uint8_t* ep = smem + wave * (128 * Q_EPI_STRIDE);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 32 * i + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3), col = 32 * j + (lane & 31);
        *reinterpret_cast<bf16_t*>(ep + row * Q_EPI_STRIDE + 2 * col) = Io<bf16_t>::from_f32(acc[i][j][r]);
      }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  const int grow0 = m0 + 128 * wm, gcol0 = n0 + 64 * wn;
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = lane + 64 * it;
    const int row = id >> 3, c8 = id & 7;
    const int grow = grow0 + row, gcol = gcol0 + 8 * c8;
    if (grow >= M) continue;
    const uint2 lo = *reinterpret_cast<const uint2*>(ep + row * Q_EPI_STRIDE + 16 * c8);
    const uint2 hi = *reinterpret_cast<const uint2*>(ep + row * Q_EPI_STRIDE + 16 * c8 + 8);
    *reinterpret_cast<uint4*>(out + (long long)grow * ldc + gcol) = make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
}
template <int FL>
__global__ void __launch_bounds__(Q_THREADS, 1)
k_lab32c(int N, int M, int K, const bf16_t* __restrict__ A, const uint8_t* __restrict__ B,
        const float* __restrict__ absmax, const float* __restrict__ datatype, bf16_t* __restrict__ out,
        int lda, int ldb, int ldc, int blocksize) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[Q_LDS];
  float2* lut = reinterpret_cast<float2*>(smem + Q_OFF_L);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid < 256) lut[tid] = make_float2(datatype[tid >> 4], datatype[tid & 15]);
  const int tilesN = (N + Q_BN - 1) / Q_BN, tilesM = (M + Q_BM - 1) / Q_BM;
  const int wg = xcd_remap(blockIdx.x, tilesN * tilesM);
  constexpr int GROUP = 4;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * Q_BM, n0 = tn * Q_BN;
  const bf16_t* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wave + i) + (lane >> 3);
    xsrc[i] = A + (long long)min(m0 + row, M - 1) * lda + 8 * ((lane & 7) ^ ((row >> 1) & 7));
  }
  // packed-weight DMA stays lane-linear: [256 rows][2 halves][16 B]
  const uint8_t* psrc = B + (long long)min(n0 + (tid >> 1), N - 1) * ldb + 16 * (tid & 1);
  const int arow = 64 * (wave & 3) + lane;
  const int bs_shift = __builtin_ctz(blocksize);
  const long long abase = 2LL * ldb * min(n0 + arow, N - 1);
  const int nk = K / Q_BK;
  auto dma_w = [&](int kt, int buf) {
    glds16(psrc + (long long)kt * (Q_BK / 2), smem + Q_OFF_P + buf * Q_PT + wave * 1024);
    glds4(absmax + ((abase + (long long)kt * Q_BK) >> bs_shift), smem + Q_OFF_A + buf * Q_AT + wave * 256);
  };
  auto dma_x = [&](int kt, int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds16(xsrc[i] + (long long)kt * Q_BK, smem + Q_OFF_X + buf * Q_XT + (4 * wave + i) * 1024);
  };
  // dequant role: 8 consecutive lanes take rows 2i+p (distinct XOR keys) -> conflict-free ds_write_b128
  const int g = lane & 31;
  const int drow = 16 * (tid >> 5) + 2 * (g & 7) + ((g >> 3) & 1);
  const int dhalf = (g >> 4) & 1;
  const int wm = wave >> 2, wn = wave & 3;
  f32x16_t acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // quarter q of this thread's 16 packed bytes -> one 16-B slot (8 bf16) of its W row
  auto lut_reads = [&](uint32_t word, float2 (&c)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = lut[(word >> (8 * j)) & 0xFF];
  };
  auto finish = [&](const float2 (&c)[4], float am, uint8_t* ws, int q) {
    uint32_t pk[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float lo = mul_nopk(c[j].x, am), hi = mul_nopk(c[j].y, am);
      pk[j] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
    }
    *reinterpret_cast<uint4*>(ws + swz2(drow, 4 * dhalf + q)) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  };
  auto dequant_all = [&](int buf) {   // prologue only
    const uint4 pw = *reinterpret_cast<const uint4*>(smem + Q_OFF_P + buf * Q_PT + drow * 32 + 16 * dhalf);
    const float am = *reinterpret_cast<const float*>(smem + Q_OFF_A + buf * Q_AT + 4 * drow);
    const uint32_t w4[4] = {pw.x, pw.y, pw.z, pw.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float2 c[4];
      lut_reads(w4[q], c);
      finish(c, am, smem + Q_OFF_W + buf * Q_WT, q);
    }
  };
  dma_x(0, 0);
  dma_w(0, 0);
  dma_w(min(1, nk - 1), 1);
  wait_vmcnt0();
  __syncthreads();
  dequant_all(0);
  __syncthreads();
  if ((FL & 8) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    const uint8_t* xs = smem + Q_OFF_X + s * Q_XT;
    const uint8_t* ws = smem + Q_OFF_W + s * Q_WT;
    uint8_t* wsn = smem + Q_OFF_W + (s ^ 1) * Q_WT;
    const uint4 pw = *reinterpret_cast<const uint4*>(smem + Q_OFF_P + (s ^ 1) * Q_PT + drow * 32 + 16 * dhalf);
    const float am = *reinterpret_cast<const float*>(smem + Q_OFF_A + (s ^ 1) * Q_AT + 4 * drow);
    const uint32_t w4[4] = {pw.x, pw.y, pw.z, pw.w};
    uint4 a[2][4], b[2][2];
    float2 c[2][4];
    auto rd = [&](int ks, int buf) {
      const int slot = 2 * ks + (lane >> 5);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[buf][j] = *reinterpret_cast<const uint4*>(ws + swz2(64 * wn + 32 * j + (lane & 31), slot));
#pragma unroll
      for (int i = 0; i < 4; ++i) a[buf][i] = *reinterpret_cast<const uint4*>(xs + swz2(128 * wm + 32 * i + (lane & 31), slot));
    };
    rd(0, 0);
    if (!(FL & 2)) lut_reads(w4[0], c[0]);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int cb = ks & 1;
      if (!(FL & 1)) {   // one X piece per ks (a scheduling-region boundary), the weight pieces with the first
        glds16(xsrc[ks] + (long long)min(t + 1, nk - 1) * Q_BK, smem + Q_OFF_X + (s ^ 1) * Q_XT + (4 * wave + ks) * 1024);
        if (ks == 0) dma_w(min(t + 2, nk - 1), s);
      }
      if (ks < 3) {
        rd(ks + 1, cb ^ 1);
        if (!(FL & 2)) lut_reads(w4[ks + 1], c[cb ^ 1]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a[cb][i]),
                                                              __builtin_bit_cast(bf16x8_t, b[cb][j]), acc[i][j], 0, 0, 0);
      if (!(FL & 2)) finish(c[cb], am, wsn, ks);
      // order: all DS reads first, then MFMA / VALU alternating, the W store last
      __builtin_amdgcn_sched_group_barrier(0x100, 10, 0);
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
    }
    wait_vmcnt0();
    __syncthreads();
  }
  // epilogue: C/D 32x32: col = lane&31, row = 8*(r>>2) + 4*(lane>>5) + (r&3)
  uint8_t* ep = smem + wave * (128 * Q_EPI_STRIDE);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 32 * i + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3), col = 32 * j + (lane & 31);
        *reinterpret_cast<bf16_t*>(ep + row * Q_EPI_STRIDE + 2 * col) = Io<bf16_t>::from_f32(acc[i][j][r]);
      }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  const int grow0 = m0 + 128 * wm, gcol0 = n0 + 64 * wn;
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = lane + 64 * it;
    const int row = id >> 3, c8 = id & 7;
    const int grow = grow0 + row, gcol = gcol0 + 8 * c8;
    if (grow >= M) continue;
    const uint2 lo = *reinterpret_cast<const uint2*>(ep + row * Q_EPI_STRIDE + 16 * c8);
    const uint2 hi = *reinterpret_cast<const uint2*>(ep + row * Q_EPI_STRIDE + 16 * c8 + 8);
    *reinterpret_cast<uint4*>(out + (long long)grow * ldc + gcol) = make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
}

// ---- v3: X ring of 3 stages (DMA two steps ahead), single W buffer with a mid-step barrier,
// B fragments of the whole step read up front
constexpr int V3_OFF_X = 0;                         // 3 x 32 KiB
constexpr int V3_OFF_W = 3 * Q_XT;                  // 32 KiB
constexpr int V3_OFF_P = V3_OFF_W + Q_WT;           // 2 x 8 KiB
constexpr int V3_OFF_A = V3_OFF_P + 2 * Q_PT;       // 2 x 1 KiB
constexpr int V3_OFF_L = V3_OFF_A + 2 * 1024;       // 2 KiB
constexpr int V3_LDS = V3_OFF_L + 2048;
template <int FL>
__global__ void __launch_bounds__(Q_THREADS, 1)
k_lab3(int N, int M, int K, const bf16_t* __restrict__ A, const uint8_t* __restrict__ B,
       const float* __restrict__ absmax, const float* __restrict__ datatype, bf16_t* __restrict__ out,
       int lda, int ldb, int ldc, int blocksize) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  float2* lut = reinterpret_cast<float2*>(smem + V3_OFF_L);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid < 256) lut[tid] = make_float2(datatype[tid >> 4], datatype[tid & 15]);
  const int tilesN = (N + Q_BN - 1) / Q_BN, tilesM = (M + Q_BM - 1) / Q_BM;
  const int wg = xcd_remap(blockIdx.x, tilesN * tilesM);
  constexpr int GROUP = 4;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * Q_BM, n0 = tn * Q_BN;
  const bf16_t* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wave + i) + (lane >> 3);
    xsrc[i] = A + (long long)min(m0 + row, M - 1) * lda + 8 * ((lane & 7) ^ ((row >> 1) & 7));
  }
  const uint8_t* psrc = B + (long long)min(n0 + (tid >> 1), N - 1) * ldb + 16 * (tid & 1);
  const int arow = 64 * (wave & 3) + lane;
  const int bs_shift = __builtin_ctz(blocksize);
  const long long abase = 2LL * ldb * min(n0 + arow, N - 1);
  const int nk = K / Q_BK;
  auto dma_w = [&](int kt, int buf) {
    glds16(psrc + (long long)kt * (Q_BK / 2), smem + V3_OFF_P + buf * Q_PT + wave * 1024);
    if (wave < 4) glds4(absmax + ((abase + (long long)kt * Q_BK) >> bs_shift), smem + V3_OFF_A + buf * 1024 + wave * 256);
  };
  auto dma_x_piece = [&](int kt, int buf, int i) {
    glds16(xsrc[i] + (long long)kt * Q_BK, smem + V3_OFF_X + buf * Q_XT + (4 * wave + i) * 1024);
  };
  const int g = lane & 31;
  const int drow = 16 * (tid >> 5) + 2 * (g & 7) + ((g >> 3) & 1);
  const int dhalf = (g >> 4) & 1;
  auto lut_reads = [&](uint32_t word, float2 (&c)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = lut[(word >> (8 * j)) & 0xFF];
  };
  uint8_t* wbuf = smem + V3_OFF_W;
  auto finish = [&](const float2 (&c)[4], float am, int q) {
    uint32_t pk[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float lo = mul_nopk(c[j].x, am), hi = mul_nopk(c[j].y, am);
      pk[j] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
    }
    *reinterpret_cast<uint4*>(wbuf + swz2(drow, 4 * dhalf + q)) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  };
  auto packed_of = [&](int buf, uint32_t (&w4)[4], float& am) {
    const uint4 pw = *reinterpret_cast<const uint4*>(smem + V3_OFF_P + buf * Q_PT + drow * 32 + 16 * dhalf);
    w4[0] = pw.x; w4[1] = pw.y; w4[2] = pw.z; w4[3] = pw.w;
    am = *reinterpret_cast<const float*>(smem + V3_OFF_A + buf * 1024 + 4 * drow);
  };
  const int wm = wave >> 2, wn = wave & 3;
  f32x16_t acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // prologue: X(0), X(1), W(0), W(1); W(0) dequantised
#pragma unroll
  for (int i = 0; i < 4; ++i) dma_x_piece(0, 0, i);
#pragma unroll
  for (int i = 0; i < 4; ++i) dma_x_piece(min(1, nk - 1), 1, i);
  dma_w(0, 0);
  dma_w(min(1, nk - 1), 1);
  wait_vmcnt0();
  __syncthreads();
  {
    uint32_t w4[4];
    float am;
    packed_of(0, w4, am);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float2 c[4];
      lut_reads(w4[q], c);
      finish(c, am, q);
    }
  }
  __syncthreads();
  int sx = 0;                                   // X stage of step t (t % 3)
  for (int t = 0; t < nk; ++t) {
    const uint8_t* xs = smem + V3_OFF_X + sx * Q_XT;
    const int sx2 = sx == 0 ? 2 : sx - 1;       // (t + 2) % 3
    uint4 b[4][2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        b[ks][j] = *reinterpret_cast<const uint4*>(wbuf + swz2(64 * wn + 32 * j + (lane & 31), 2 * ks + (lane >> 5)));
    uint32_t w4[4];
    float am;
    packed_of((t + 1) & 1, w4, am);
    __builtin_amdgcn_s_waitcnt(0xC07F);         // lgkmcnt(0): every B fragment of W(t) is in registers
    __builtin_amdgcn_s_barrier();               // ... in every wave, so W(t+1) may overwrite the buffer
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (ks == 0) dma_w(min(t + 2, nk - 1), t & 1);
      dma_x_piece(min(t + 2, nk - 1), sx2, ks);
      const int slot = 2 * ks + (lane >> 5);
      uint4 a[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const uint4*>(xs + swz2(128 * wm + 32 * i + (lane & 31), slot));
      float2 c[4];
      if (!(FL & 2)) lut_reads(w4[ks], c);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a[i]),
                                                              __builtin_bit_cast(bf16x8_t, b[ks][j]), acc[i][j], 0, 0, 0);
      if (!(FL & 2)) finish(c, am, ks);
    }
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // X(t+2) may stay in flight; W(t+2), X(t+1) landed
    __syncthreads();
    sx = sx == 2 ? 0 : sx + 1;
  }
  uint8_t* ep = smem + wave * (128 * Q_EPI_STRIDE);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 32 * i + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3), col = 32 * j + (lane & 31);
        *reinterpret_cast<bf16_t*>(ep + row * Q_EPI_STRIDE + 2 * col) = Io<bf16_t>::from_f32(acc[i][j][r]);
      }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  const int grow0 = m0 + 128 * wm, gcol0 = n0 + 64 * wn;
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = lane + 64 * it;
    const int row = id >> 3, c8 = id & 7;
    const int grow = grow0 + row, gcol = gcol0 + 8 * c8;
    if (grow >= M) continue;
    const uint2 lo = *reinterpret_cast<const uint2*>(ep + row * Q_EPI_STRIDE + 16 * c8);
    const uint2 hi = *reinterpret_cast<const uint2*>(ep + row * Q_EPI_STRIDE + 16 * c8 + 8);
    *reinterpret_cast<uint4*>(out + (long long)grow * ldc + gcol) = make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
}
}
using namespace bnb;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
int main() {
  const int M = 4096, N = 4096, K = 11008, BS = 64;
  uint16_t *X, *Y; uint8_t* W; float *am, *code;
  CK(hipMalloc(&X, (size_t)M * K * 2)); CK(hipMalloc(&Y, (size_t)M * N * 2));
  CK(hipMalloc(&W, (size_t)N * K / 2)); CK(hipMalloc(&am, (size_t)N * K / BS * 4)); CK(hipMalloc(&code, 64));
  {
    std::vector<uint16_t> hx((size_t)M * K);
    srand(3);
    for (auto& v : hx) { float f = ((rand() & 0xFFFF) - 32768) / 16384.0f; uint32_t u; memcpy(&u, &f, 4); v = (uint16_t)(u >> 16); }
    CK(hipMemcpy(X, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
    std::vector<uint8_t> hw((size_t)N * K / 2);
    for (auto& v : hw) v = rand() & 0xFF;
    CK(hipMemcpy(W, hw.data(), hw.size(), hipMemcpyHostToDevice));
  }
  std::vector<float> h(N * (K / BS), 0.01f); CK(hipMemcpy(am, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  float hc[16]; for (int i = 0; i < 16; ++i) hc[i] = (i - 7.5f) / 8; CK(hipMemcpy(code, hc, 64, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int tiles = (M / 256) * (N / 256);
  auto run = [&](const char* name, auto kern, size_t dyn = 0) {
    if (dyn) CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(tiles), dim3(512), dyn, 0, N, M, K, (const bf16_t*)X, W, am, code, (bf16_t*)Y, K, K / 2, N, BS);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int R = 20;
    for (int i = 0; i < R; ++i) hipLaunchKernelGGL(kern, dim3(tiles), dim3(512), dyn, 0, N, M, K, (const bf16_t*)X, W, am, code, (bf16_t*)Y, K, K / 2, N, BS);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / R;
    printf("%-28s %8.1f us  %7.1f TFLOP/s\n", name, us, 2.0 * M * N * K / us / 1e6);
  };
  for (int rep = 0; rep < 2; ++rep) {
  run("32b full", k_lab32b<0>);
  run("32b no-dma", k_lab32b<1>);
  run("v3 full", k_lab3<0>, V3_LDS);
  run("v3 no-dequant", k_lab3<2>, V3_LDS);
  }
  return 0;
}
