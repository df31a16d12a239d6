// 256 x 256-tile fused 4-bit weight GEMM (the large-problem kernel behind cgemm_4bit_inference*,
// see gemm4bit.hip for the ABI / semantics; ref:sycl/pythonInterface.cpp:377-378, kernel_gemm.cpp:1015).
//
// Geometry: 512 threads = 8 waves (2 along tokens x 4 along out-features), 128 x 64 outputs per wave
// (8 x 4 tiles of v_mfma_f32_16x16x32, or 4 x 2 of 32x32x16 with M16 = false), BK = 64, one workgroup
// per CU (148 KiB LDS).
//
// Every operand arrives by LDS-DMA (global_load_lds), so no VGPR-destination load is ever in flight
// in the k-loop (hipcc otherwise drains the prefetch early, cdna_hip_programming.md §5):
//   Xs[2]  activations   2 x 32 KiB  [256][64] T, 16-B slots XOR-swizzled by (row >> 1) & 7
//   Ws[2]  weights (T)   2 x 32 KiB  same layout, written by the in-kernel dequantisation
//   Wp[2]  packed 4-bit  2 x  8 KiB  [256 rows][2 halves][16 B], lane-linear
//   Am[2]  absmax        2 x  1 KiB  one fp32 per weight row and k-step (bs >= 64)
//   LUT                      2 KiB   byte -> {code[hi], code[lo]}
// The swizzle makes the 32-row fragment reads (ds_read_b128 lane groups) and the dequant stores
// (8 consecutive lanes -> rows 2i+p, distinct XOR keys) conflict-free.
// k-step t (one barrier): the four k16 sub-steps each issue one X(t+1) DMA piece (W(t+2) and its
// absmax ride with the first), run 8 MFMAs on stage t, and dequantise one quarter of this thread's
// 16 packed bytes of W(t+1) (LUT -> *absmax -> one RNE cast -> Ws) -- the reference's dequantised
// values; vmcnt(0) + barrier.
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
// the byte -> {code[hi], code[lo]} LUT as Q_LUTC interleaved copies (entry b of copy j at b * Q_LUTC + j,
// lane l reads copy l % Q_LUTC): random-byte ds_read_b64 lookups of one copy serialise on bank conflicts
constexpr int Q_LUTC = 4;
constexpr int Q_LDS = Q_OFF_L + 256 * 8 * Q_LUTC;   // 157,696 B
constexpr int Q_EPI_STRIDE = 136;              // staged output row: 128 B + 8 B pad
static_assert(8 * 128 * Q_EPI_STRIDE <= Q_OFF_L, "epilogue staging must not overlap the LUT");

typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int swz2(int r, int s) { return r * 128 + ((s ^ ((r >> 1) & 7)) << 4); }

// scalar v_mul_f32 (hipcc would SLP-pack the pair into v_pk_mul_f32, which costs ~4x the issue
// slots beside MFMAs on gfx950)
__device__ __forceinline__ float mul_f32(float a, float b) {
  float r;
  asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// {T(lo), T(hi)} with one RNE cast each (v_cvt_pk_bf16_f32 for bf16)
template <typename T> __device__ __forceinline__ uint32_t cvt2(float lo, float hi);
template <> __device__ __forceinline__ uint32_t cvt2<bf16_t>(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
}
template <> __device__ __forceinline__ uint32_t cvt2<fp16_t>(float lo, float hi) { return Mfma<fp16_t>::pack2(lo, hi); }

// M16 (the launched form): v_mfma_f32_16x16x32 (8 x 4 tiles of 16x16 per wave, k32 per sub-step)
// instead of 32x32x16.  Same cycles per FLOP, but the chip holds a higher clock on the 16x16 shape under
// load (MI355X_MICROARCH.md 'DVFS give-back' item 7): 326 vs 346 us at 4096 x 4096 x 11008, bit-identical
// outputs (tools/gemm_m16_lab.hip).  The fragment reads (rows l & 15, slot 4 s + (l >> 4)) stay
// conflict-free under the (row >> 1) & 7 swizzle.
template <typename T, bool SPLIT, bool M16 = false, int LUTC = Q_LUTC, bool XB = false>
__global__ void __launch_bounds__(Q_THREADS, 1)
k_gemm_4bit_256(int N, int M, int K, const T* __restrict__ A, const uint8_t* __restrict__ B,
                const float* __restrict__ absmax, const float* __restrict__ datatype, T* __restrict__ out,
                int lda, int ldb, int ldc, int blocksize, float* __restrict__ ws, int ksplit_arg) {
  const int ksplit = SPLIT ? ksplit_arg : 1;    // the unsplit instance keeps the k-loop free of split terms
  __shared__ __attribute__((aligned(16))) uint8_t smem[Q_LDS];
  float2* lut = reinterpret_cast<float2*>(smem + Q_OFF_L);
  const float2* lutc = lut + (threadIdx.x & (LUTC - 1));
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);        // provably wave-uniform (SGPR math)
  for (int e = tid; e < 256 * LUTC; e += Q_THREADS) lut[e] = make_float2(datatype[(e / LUTC) >> 4], datatype[(e / LUTC) & 15]);

  // ---- tile order: XCD-contiguous ids, grouped 4 token-tiles x all feature-tiles; with split-K
  // (ksplit > 1) the split is the outer index, so an XCD's workgroups share one K range
  const int tilesN = (N + Q_BN - 1) / Q_BN, tilesM = (M + Q_BM - 1) / Q_BM;
  const int ntiles = tilesN * tilesM;
  const int wg_all = xcd_remap(blockIdx.x, ntiles * ksplit);
  const int split = wg_all / ntiles, wg = wg_all - split * ntiles;
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
    xsrc[i] = A + (long long)min(m0 + row, M - 1) * lda + 8 * ((lane & 7) ^ ((row >> 1) & 7));
  }
  const uint8_t* psrc = B + (long long)min(n0 + (tid >> 1), N - 1) * ldb + 16 * (tid & 1);   // lane-linear
  // absmax DMA: one row per lane; waves 4-7 repeat waves 0-3 into the stage's spare copy (branch-free)
  const int arow = 64 * (wave & 3) + lane;
  const int bs_shift = __builtin_ctz(blocksize);                    // blocksize: power of two >= 64
  const long long abase = 2LL * ldb * min(n0 + arow, N - 1);        // element index of (row, k = 0)

  // this workgroup's k-tiles: [kb, kb + nk) of the K / 64 (the host keeps ksplit <= K / 64)
  const int nk_all = K / Q_BK;
  const int kb = SPLIT ? (int)((long long)split * nk_all / ksplit) : 0;
  const int nk = SPLIT ? (int)((long long)(split + 1) * nk_all / ksplit) - kb : nk_all;
  auto dma_w = [&](int kt, int buf) {                               // packed weights + absmax of k-tile kt
    kt += kb;
    glds16(psrc + (long long)kt * (Q_BK / 2), smem + Q_OFF_P + buf * Q_PT + wave * 1024);
    glds4(absmax + ((abase + (long long)kt * Q_BK) >> bs_shift), smem + Q_OFF_A + buf * Q_AT + wave * 256);
  };
  auto dma_x_piece = [&](int kt, int buf, int i) {
    glds16(xsrc[i] + (long long)(kb + kt) * Q_BK, smem + Q_OFF_X + buf * Q_XT + (4 * wave + i) * 1024);
  };

  // ---- dequant role: this thread owns 16 packed bytes (32 k) of one W row; 8 consecutive lanes take
  // rows 2i+p so their 16-B stores land on distinct swizzle keys
  const int g = lane & 31;
  const int drow = 16 * (tid >> 5) + 2 * (g & 7) + ((g >> 3) & 1);
  const int dhalf = (g >> 4) & 1;
  auto lut_reads = [&](uint32_t word, float2 (&c)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = lutc[((word >> (8 * j)) & 0xFF) * LUTC];
  };
  auto finish = [&](const float2 (&c)[4], float am, uint8_t* ws, int q) {   // 4 bytes -> one 16-B slot
    uint32_t pk[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) pk[j] = cvt2<T>(mul_f32(c[j].x, am), mul_f32(c[j].y, am));
    *reinterpret_cast<uint4*>(ws + swz2(drow, 4 * dhalf + q)) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  };
  auto packed_of = [&](int buf, uint32_t (&w4)[4], float& am) {
    const uint4 pw = *reinterpret_cast<const uint4*>(smem + Q_OFF_P + buf * Q_PT + drow * 32 + 16 * dhalf);
    w4[0] = pw.x; w4[1] = pw.y; w4[2] = pw.z; w4[3] = pw.w;
    am = *reinterpret_cast<const float*>(smem + Q_OFF_A + buf * Q_AT + 4 * drow);
  };

  const int wm = wave >> 2, wn = wave & 3;
  f32x16_t acc[4][2];
  f32x4_t acc16[M16 ? 8 : 1][M16 ? 4 : 1];
  if constexpr (M16) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc16[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  }

  // ---- prologue: X(0), W(0), W(1) in flight; dequantise W(0) into Ws[0]
#pragma unroll
  for (int i = 0; i < 4; ++i) dma_x_piece(0, 0, i);
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
      finish(c, am, smem + Q_OFF_W, q);
    }
  }
  __syncthreads();

  if constexpr (M16 && XB) {
    // Cross-barrier pipeline (as igemm_256.hip): tile t's k2 = 1 fragments are read into registers
    // under its k2 = 0 MFMAs; after the barrier the wave reads tile t+1's k2 = 0 fragments under tile
    // t's k2 = 1 MFMAs.  W(t+1) is dequantised into Ws[t+1] before the barrier as before.
    // One set of A fragments is recycled row by row (a[i] is re-read right after its last MFMA), so
    // only B is double-buffered: acc + 8 A + 2 x 4 B fragments fit the 256-VGPR budget.
    uint4 a[8], b0[4], b1[4];
    auto rd_a = [&](int buf, int k2, int i) {
      return *reinterpret_cast<const uint4*>(smem + Q_OFF_X + buf * Q_XT + swz2(128 * wm + 16 * i + (lane & 15), 4 * k2 + (lane >> 4)));
    };
    auto rd_b = [&](int buf, int k2, uint4 (&b)[4]) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = *reinterpret_cast<const uint4*>(smem + Q_OFF_W + buf * Q_WT + swz2(64 * wn + 16 * j + (lane & 15), 4 * k2 + (lane >> 4)));
    };
    rd_b(0, 0, b0);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = rd_a(0, 0, i);
    for (int t = 0; t < nk; ++t) {
      const int s = t & 1;
      uint8_t* wsn = smem + Q_OFF_W + (s ^ 1) * Q_WT;
      uint32_t w4[4];
      float am;
      packed_of(s ^ 1, w4, am);                                    // W(t+1), landed during step t-1
      rd_b(s, 1, b1);
      if (t + 1 < nk) {
#pragma unroll
        for (int i = 0; i < 4; ++i) dma_x_piece(t + 1, s ^ 1, i);  // every wave is past tile t-1's reads
      }
      if (t + 2 < nk) dma_w(t + 2, s);
      float2 c0[4], c1[4];
      lut_reads(w4[0], c0);
      lut_reads(w4[1], c1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc16[i][j] = Mfma<T>::mma(a[i], b0[j], acc16[i][j]);
        a[i] = rd_a(s, 1, i);
      }
      finish(c0, am, wsn, 0);
      finish(c1, am, wsn, 1);
      lut_reads(w4[2], c0);
      lut_reads(w4[3], c1);
      finish(c0, am, wsn, 2);
      finish(c1, am, wsn, 3);
      wait_vmcnt0();                                               // X(t+1), W(t+2) of this wave landed
      __builtin_amdgcn_s_waitcnt(0xC07F);                          // its Ws[t+1] stores and tile-t reads done
      __builtin_amdgcn_s_barrier();
      const int sn = t + 1 < nk ? s ^ 1 : s;                       // (last step: harmless re-reads)
      rd_b(sn, 0, b0);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc16[i][j] = Mfma<T>::mma(a[i], b1[j], acc16[i][j]);
        a[i] = rd_a(sn, 0, i);
      }
    }
    __syncthreads();                                               // the epilogue reuses the stages
  } else
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    const uint8_t* xs = smem + Q_OFF_X + s * Q_XT;
    const uint8_t* ws = smem + Q_OFF_W + s * Q_WT;
    uint8_t* wsn = smem + Q_OFF_W + (s ^ 1) * Q_WT;
    uint32_t w4[4];
    float am;
    packed_of(s ^ 1, w4, am);                                      // W(t+1), landed during step t-1
    if constexpr (M16) {
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        dma_x_piece(min(t + 1, nk - 1), s ^ 1, 2 * k2);   // spread over the sub-steps (all at the top of
        dma_x_piece(min(t + 1, nk - 1), s ^ 1, 2 * k2 + 1);   // the step measured 3 % slower)
        if (k2 == 0) dma_w(min(t + 2, nk - 1), s);
        const int slot = 4 * k2 + (lane >> 4);
        uint4 a[8], b[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const uint4*>(ws + swz2(64 * wn + 16 * j + (lane & 15), slot));
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const uint4*>(xs + swz2(128 * wm + 16 * i + (lane & 15), slot));
        float2 c0[4], c1[4];
        lut_reads(w4[2 * k2], c0);
        lut_reads(w4[2 * k2 + 1], c1);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc16[i][j] = Mfma<T>::mma(a[i], b[j], acc16[i][j]);
        finish(c0, am, wsn, 2 * k2);
        finish(c1, am, wsn, 2 * k2 + 1);
      }
      wait_vmcnt0();
      __syncthreads();
      continue;
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      dma_x_piece(min(t + 1, nk - 1), s ^ 1, ks);
      if (ks == 0) dma_w(min(t + 2, nk - 1), s);
      const int slot = 2 * ks + (lane >> 5);
      uint4 a[4], b[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = *reinterpret_cast<const uint4*>(ws + swz2(64 * wn + 32 * j + (lane & 31), slot));
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const uint4*>(xs + swz2(128 * wm + 32 * i + (lane & 31), slot));
      float2 c[4];
      lut_reads(w4[ks], c);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = Mfma32<T>::mma(a[i], b[j], acc[i][j]);
      finish(c, am, wsn, ks);
    }
    wait_vmcnt0();
    __syncthreads();
  }

  if (SPLIT) {
    // split-K: fp32 partial tile -> ws[split][M][N]; k_splitk_reduce sums the splits in order
    float* wsp = ws + (long long)split * M * N;
    if constexpr (M16) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = m0 + 128 * wm + 16 * i + 4 * (lane >> 4) + r;
            const int col = n0 + 64 * wn + 16 * j + (lane & 15);
            if (row < M && col < N) wsp[(long long)row * N + col] = acc16[i][j][r];
          }
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + 128 * wm + 32 * i + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
          const int col = n0 + 64 * wn + 32 * j + (lane & 31);
          if (row < M && col < N) wsp[(long long)row * N + col] = acc[i][j][r];
        }
    return;
  }

  // ---- epilogue: acc -> LDS (per-wave [128][64] T, 136-B rows) -> 16-B coalesced stores
  uint8_t* ep = smem + wave * (128 * Q_EPI_STRIDE);
  if constexpr (M16) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * i + 4 * (lane >> 4) + r, col = 16 * j + (lane & 15);
          *reinterpret_cast<T*>(ep + row * Q_EPI_STRIDE + 2 * col) = Io<T>::from_f32(acc16[i][j][r]);
        }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = 32 * i + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3), col = 32 * j + (lane & 31);
          *reinterpret_cast<T*>(ep + row * Q_EPI_STRIDE + 2 * col) = Io<T>::from_f32(acc[i][j][r]);
        }
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

// out[r, c] = T(sum_s ws[s][r][c]) in split order (fp32), one RNE cast
template <typename T>
__global__ void __launch_bounds__(256)
k_splitk_reduce(const float* __restrict__ ws, int ksplit, int rows, int cols, T* __restrict__ out, int ldc) {
  const long long mn = (long long)rows * cols;
  const long long i4 = 4LL * (blockIdx.x * 256LL + threadIdx.x);
  if (i4 >= mn) return;
  if ((cols & 3) == 0) {
    float4 s = *reinterpret_cast<const float4*>(ws + i4);
    for (int k = 1; k < ksplit; ++k) {
      const float4 v = *reinterpret_cast<const float4*>(ws + k * mn + i4);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    const long long r = i4 / cols, c = i4 - r * cols;
    T* dst = out + r * ldc + c;
    dst[0] = Io<T>::from_f32(s.x); dst[1] = Io<T>::from_f32(s.y);
    dst[2] = Io<T>::from_f32(s.z); dst[3] = Io<T>::from_f32(s.w);
  } else {
    for (long long i = i4; i < i4 + 4 && i < mn; ++i) {
      float s = ws[i];
      for (int k = 1; k < ksplit; ++k) s += ws[k * mn + i];
      const long long r = i / cols, c = i - r * cols;
      out[r * ldc + c] = Io<T>::from_f32(s);
    }
  }
}

template <typename T>
void launch_gemm_4bit_256(int m, int n, int k, const T* A, const uint8_t* B, const float* absmax, const float* datatype,
                          T* out, int lda, int ldb, int ldc, int blocksize, float* ws, int ksplit) {
  const long long tiles = (long long)((m + Q_BN - 1) / Q_BN) * ((n + Q_BM - 1) / Q_BM);
  if (ksplit <= 1) {
    hipLaunchKernelGGL((k_gemm_4bit_256<T, false, true>), dim3((unsigned)tiles), dim3(Q_THREADS), 0, current_stream(), m, n,
                       k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize, ws, 1);
  } else {
    hipLaunchKernelGGL((k_gemm_4bit_256<T, true, true>), dim3((unsigned)(tiles * ksplit)), dim3(Q_THREADS), 0,
                       current_stream(), m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize, ws, ksplit);
    const long long mn = (long long)m * n;
    hipLaunchKernelGGL((k_splitk_reduce<T>), dim3((unsigned)((mn / 4 + 255) / 256 + 1)), dim3(256), 0,
                       current_stream(), ws, ksplit, n, m, out, ldc);
  }
}

template void launch_gemm_4bit_256<bf16_t>(int, int, int, const bf16_t*, const uint8_t*, const float*, const float*,
                                           bf16_t*, int, int, int, int, float*, int);
template void launch_gemm_4bit_256<fp16_t>(int, int, int, const fp16_t*, const uint8_t*, const float*, const float*,
                                           fp16_t*, int, int, int, int, float*, int);

}  // namespace bnb
