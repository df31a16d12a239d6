// Hand-written bf16 / fp16 GEMM for gfx950, C[m][n] = sum_k A[m][k] * B[n][k] (both operands k-contiguous,
// the F.linear shape).  It is the GEMM half of the large-prefill NF4 path: the reference dequantises the
// 4-bit weight and calls F.linear (ref:python_src_quants/autograd/_functions.py:507, MatMul4Bit.forward);
// here k_dequantize_4bit_stream writes the weight once and this kernel multiplies it (no vendor GEMM).
//
// Geometry (the shape a tuned library GEMM uses on this chip): 256 x 256 output tile, BK = 64, FOUR waves
// (256 threads, one wave per SIMD, one workgroup per CU), each wave 128 x 128 outputs = 8 x 8 accumulators of
// v_mfma_f32_16x16x32 (256 accumulator registers).  Every fragment read from LDS feeds 8 MFMAs, so a k32 step
// is 16 ds_read_b128 per 64 MFMAs -- a third fewer LDS bytes per MFMA than the 8-wave 128 x 64 split
// (MI355X_MICROARCH.md 'DVFS give-back': LDS read bytes cost clock).
//
// Pipeline: two LDS stages of 64 KiB (A and B tiles [256][64], 16-B slots XOR-swizzled by (row >> 1) & 7 through
// the DMA source address, conflict-free for the fragment reads).  Both operands move by LDS-DMA
// (global_load_lds_dwordx4, scalar base + one 32-bit lane offset per piece, so ragged edges are clamped once in
// the offsets and a k-step advances only the scalar base).  Per k-tile t, two halves:
//   half 1: the 64 MFMAs of k32 step 0 (fragments already in registers) while this wave reads step 1's fragments;
//           lgkmcnt(0) + barrier: every wave is done with stage t & 1;
//   half 2: DMA of tile t+2 into that stage, interleaved with step 1's MFMAs; vmcnt(16) (tile t+1 landed) +
//           barrier; tile t+1's step-0 fragments read under the remaining MFMAs.
// The DMA of a tile is therefore in flight for a whole k-tile (~2k MFMA cycles), and no vmcnt(0) drain sits in
// the loop (cdna_hip_programming.md §5 'Pipelining across barriers').
#include "gemm_common.hpp"

#include <type_traits>

namespace bnb {

constexpr int HG_BM = 256, HG_BN = 256, HG_BK = 64, HG_THREADS = 256;
constexpr int HG_TILE = HG_BM * HG_BK * 2;        // 32 KiB per operand per stage
constexpr int HG_STAGE = 2 * HG_TILE;             // A + B
constexpr int HG_LDS = 2 * HG_STAGE;              // 128 KiB

// LDS-DMA with a scalar base: lane address = sbase + voff (unsigned 32-bit), 16 B per lane to lds + 16 * lane.
// M0 (the LDS destination) is written and restored inside the statement (it is compiler-reserved).
__device__ __forceinline__ void glds16_sv(const void* sbase, uint32_t voff, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds)
               : "memory");
}

typedef float hg_f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 hg_bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 hg_f16x2_t __attribute__((ext_vector_type(2)));
// {T(lo), T(hi)}: one RNE conversion each (v_cvt_pk_bf16_f32 / v_cvt_pkrtz is NOT used for fp16: RNE per element)
template <typename T> __device__ __forceinline__ uint32_t cvt_pk(float lo, float hi);
template <> __device__ __forceinline__ uint32_t cvt_pk<bf16_t>(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((hg_f32x2_t){lo, hi}, hg_bf16x2_t));
}
template <> __device__ __forceinline__ uint32_t cvt_pk<fp16_t>(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((hg_f32x2_t){lo, hi}, hg_f16x2_t));
}

// MFMA operand type kept native end to end (no uint4 <-> bf16x8 bit casts in the k-loop)
// The MFMA is issued from inline asm with the accumulator pinned to AGPRs ("+a") and the fragments to VGPRs ("v"):
// with the builtin, hipcc's allocator treats both as either-file operands and, at 256 accumulator registers, shuffles
// them between the files every iteration (v_accvgpr_read/write/mov).  What the asm hides from hipcc is handled here:
// the fragment reads are ordinary LDS loads (hipcc waits on lgkmcnt before the statement that reads them), each
// accumulator is re-read 63 MFMAs after it was written, and the epilogue pads the MFMA -> accvgpr_read hazard itself.
typedef unsigned hg_u32x4_t __attribute__((ext_vector_type(4)));
template <typename T> struct HgFrag;
template <> struct HgFrag<bf16_t> {
  typedef hg_u32x4_t type;
  __device__ static __forceinline__ f32x4_t mma(const type& a, const type& b, f32x4_t c) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
    return c;
  }
  __device__ static __forceinline__ f32x4_t mma0(const type& a, const type& b) {
    f32x4_t c;
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
    return c;
  }
};
template <> struct HgFrag<fp16_t> {
  typedef hg_u32x4_t type;
  __device__ static __forceinline__ f32x4_t mma(const type& a, const type& b, f32x4_t c) {
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
    return c;
  }
  __device__ static __forceinline__ f32x4_t mma0(const type& a, const type& b) {
    f32x4_t c;
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
    return c;
  }
};

__device__ __forceinline__ int hg_swz(int r, int s) { return r * 128 + ((s ^ ((r >> 1) & 7)) << 4); }

// V: schedule variant bits (A/B arms of tools/hgemm_lab.hip; HG_V is the launched one):
//   1 = step-1 fragment reads all after half 1's MFMAs, 2 = no sched_barrier fences in half 2,
//   4 = next-step fragments read in MFMA-need order, 8 = DMA spread (8 pieces before the wait, 8 after, one per
//   4 MFMAs) -- 1.6 PFLOP/s vs 1.44 for 0 at 4096 x 4096 x 11008 (profiles/lab/r03_hgemm_variants.txt)
constexpr int HG_V = 8;
template <typename T, int V = 0>
__global__ void __launch_bounds__(HG_THREADS, 1)
k_hgemm(int M, int N, int K, const T* __restrict__ A, long long lda, const T* __restrict__ B, long long ldb,
        T* __restrict__ C, long long ldc) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[HG_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // ---- tile order: XCD-contiguous ids; groups of 4 M-tiles x all N-tiles (an XCD's 32 tiles share A / B rows)
  const int tilesN = (N + HG_BN - 1) / HG_BN, tilesM = (M + HG_BM - 1) / HG_BM;
  const int wg = xcd_remap(blockIdx.x, tilesN * tilesM);
  constexpr int GROUP = 4;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * HG_BM, n0 = tn * HG_BN;

  // ---- DMA: wave w fills pieces p = 8w + i (tile rows 8p .. 8p+7) of both operands; lane -> (row, slot)
  // (32-bit arithmetic: the host keeps every offset below 4 GiB; 64-bit products made hipcc park each offset in a
  // 4-register tuple)
  uint32_t aoff[8], boff[8];
  const uint32_t lda2 = (uint32_t)lda * 2u, ldb2 = (uint32_t)ldb * 2u;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = 8 * (8 * wave + i) + (lane >> 3);
    const uint32_t slot = (uint32_t)((lane & 7) ^ ((row >> 1) & 7));
    aoff[i] = (uint32_t)min(m0 + row, M - 1) * lda2 + 16u * slot;
    boff[i] = (uint32_t)min(n0 + row, N - 1) * ldb2 + 16u * slot;
  }
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem) + wave * 8192;
  auto dma_a = [&](int kt, int st, int i) {
    glds16_sv(A + (long long)kt * HG_BK, aoff[i], lds0 + st * HG_STAGE + i * 1024);
  };
  auto dma_b = [&](int kt, int st, int i) {
    glds16_sv(B + (long long)kt * HG_BK, boff[i], lds0 + st * HG_STAGE + HG_TILE + i * 1024);
  };

  // ---- fragments: MFMA A operand = B rows (n), MFMA B operand = A rows (m), so D[n][m] and a lane's 4 results
  // are 4 consecutive n of one m: one 8-B store per accumulator.  Row keys ((row >> 1) & 7) do not depend on the
  // fragment index, so each operand needs one lane offset per k32 step.
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fg = lane >> 4, key = (fr >> 1) & 7;
  const int xo0 = (128 * wm + fr) * 128 + ((fg ^ key) << 4), xo1 = (128 * wm + fr) * 128 + (((4 + fg) ^ key) << 4);
  const int wo0 = HG_TILE + (128 * wn + fr) * 128 + ((fg ^ key) << 4);
  const int wo1 = HG_TILE + (128 * wn + fr) * 128 + (((4 + fg) ^ key) << 4);
  using frag_t = typename HgFrag<T>::type;
  auto rd = [&](int st, int off, int f) -> frag_t {
    return *reinterpret_cast<const frag_t*>(smem + st * HG_STAGE + off + f * 2048);
  };

  f32x4_t acc[8][8];
  frag_t w0[8], x0[8], w1[8], x1[8];
  const int nk = K / HG_BK;

  // half 1 of k-tile t (stage st): the 64 MFMAs of k32 step 0, step 1's fragments of the stage read underneath (one
  // read per 4 MFMAs); then this wave's reads are retired and the barrier says every wave is done with the stage.
  // FIRST: tile 0 starts the accumulators (SrcC = 0, so no zero-fill of the AGPRs is needed).
  auto half1 = [&](auto first, int st) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (decltype(first)::value) acc[j][i] = HgFrag<T>::mma0(w0[j], x0[i]);
        else acc[j][i] = HgFrag<T>::mma(w0[j], x0[i], acc[j][i]);
        if (!(V & 1) && (i & 3) == 3) {
          const int q = 2 * j + (i >> 2);               // 0..15
          if (q < 8) w1[q] = rd(st, wo1, q);
          else x1[q - 8] = rd(st, xo1, q - 8);
        }
      }
      if (!(V & 1)) __builtin_amdgcn_sched_barrier(0);
    }
    if (V & 1) {
#pragma unroll
      for (int f = 0; f < 8; ++f) { w1[f] = rd(st, wo1, f); x1[f] = rd(st, xo1, f); }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);                   // lgkmcnt(0): this wave's reads of stage st are done
    __builtin_amdgcn_s_barrier();                         // ... and every other wave's
    __builtin_amdgcn_sched_barrier(0);
  };
  // half 2 of k-tile t: the 64 MFMAs of step 1.  Unless LAST: tile t+2's DMA into stage st under the first 32 (one
  // piece per 2 MFMAs; past the end the last tile is re-loaded into a stage nobody reads again, so the body stays
  // branch-free), vmcnt(16) = tile t+1 landed for this wave + barrier = for every wave, and tile t+1's step-0
  // fragments read under the last 32.
  auto half2 = [&](auto last, int t, int st) {
    constexpr bool L = decltype(last)::value;
    constexpr bool SPREAD = (V & 8) != 0;    // 8 DMA pieces before the wait, 8 after (one per 4 MFMAs throughout)
    const int kn = min(t + 2, nk - 1);
    auto dma = [&](int q) {
      if (q < 8) dma_a(kn, st, q);
      else dma_b(kn, st, q - 8);
    };
    // fragment q of the next step 0, in the order its MFMAs need them (w0[0], x0[0..7], w0[1..7]) unless V & 4 == 0
    auto rdn = [&](int q) {
      if constexpr ((V & 4) != 0) {
        if (q == 0) w0[0] = rd(st ^ 1, wo0, 0);
        else if (q <= 8) x0[q - 1] = rd(st ^ 1, xo0, q - 1);
        else w0[q - 8] = rd(st ^ 1, wo0, q - 8);
      } else {
        if (q < 8) w0[q] = rd(st ^ 1, wo0, q);
        else x0[q - 8] = rd(st ^ 1, xo0, q - 8);
      }
    };
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[j][i] = HgFrag<T>::mma(w1[j], x1[i], acc[j][i]);
        if constexpr (!L) {
          if (SPREAD) {
            if ((i & 3) == 3) dma(2 * j + (i >> 2));            // pieces 0..7
          } else if ((i & 1) == 1) {
            dma(4 * j + (i >> 1));                              // pieces 0..15
          }
        }
      }
      if (!(V & 2)) __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (!L) {
      if (SPREAD) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");    // tile t+1 landed (this wave's pieces)
      else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      __builtin_amdgcn_s_barrier();                                    // ... every wave's pieces
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = 4; j < 8; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[j][i] = HgFrag<T>::mma(w1[j], x1[i], acc[j][i]);
        if constexpr (!L) {
          if ((i & 1) == 1) rdn(4 * (j - 4) + (i >> 1));       // fragments 0..15
          if (SPREAD && (i & 3) == 0) dma(8 + 2 * (j - 4) + (i >> 2));   // pieces 8..15
        }
      }
      if (!(V & 2)) __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- prologue: tiles 0 and 1 in flight, tile 0 landed, its step-0 fragments in registers
#pragma unroll
  for (int i = 0; i < 8; ++i) { dma_a(0, 0, i); dma_b(0, 0, i); }
  {
    const int k1 = min(1, nk - 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) { dma_a(k1, 1, i); dma_b(k1, 1, i); }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int f = 0; f < 8; ++f) { w0[f] = rd(0, wo0, f); x0[f] = rd(0, xo0, f); }

  half1(std::true_type{}, 0);
  for (int t = 0; t + 1 < nk; ++t) {
    half2(std::false_type{}, t, t & 1);
    half1(std::false_type{}, (t + 1) & 1);
  }
  half2(std::true_type{}, nk - 1, (nk - 1) & 1);
  wait_vmcnt0();                                          // no LDS-DMA may outlive the workgroup
  // MFMA (asm, invisible to hipcc's hazard recognizer) -> v_accvgpr_read: pad the wait states by hand
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  // ---- epilogue: acc[j][i][r] = C[m0 + 128 wm + 16 i + fr][n0 + 128 wn + 16 j + 4 fg + r]; 8-B stores.
  // Full tiles (the common case) store unconditionally; edge tiles check every row / column.
  const int mb = m0 + 128 * wm + fr, nb = n0 + 128 * wn + 4 * fg;
  const bool full = (m0 + HG_BM <= M) && (n0 + HG_BN <= N) && ((ldc & 3) == 0) && (((uintptr_t)C & 7) == 0);
  if (full) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      T* crow = C + (long long)(mb + 16 * i) * ldc + nb;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        uint2 v;
        v.x = cvt_pk<T>(acc[j][i][0], acc[j][i][1]);
        v.y = cvt_pk<T>(acc[j][i][2], acc[j][i][3]);
        *reinterpret_cast<uint2*>(crow + 16 * j) = v;
        __builtin_amdgcn_sched_barrier(0);   // one accumulator at a time: no VGPR burst that displaces AGPRs
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mb + 16 * i;
      T* crow = C + (long long)min(m, M - 1) * ldc;
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = nb + 16 * j + r;
          if (m < M && n < N) crow[n] = Io<T>::from_f32(acc[j][i][r]);
          __builtin_amdgcn_sched_barrier(0);
        }
    }
  }
}

// Host rule: K % 64 == 0, 16-B aligned rows (lda, ldb % 8 == 0, 16-B aligned bases), and every lane offset
// (row * ld * 2 bytes) below 4 GiB.
bool hgemm_fits(int m, int n, int k, long long lda, long long ldb, const void* A, const void* B) {
  if (m <= 0 || n <= 0 || k <= 0 || (k % HG_BK) != 0) return false;
  if ((lda & 7) || (ldb & 7) || lda < k || ldb < k) return false;
  if (((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return false;
  if ((long long)(m - 1) * lda * 2 + 2LL * k > 0xFFFFFFFFLL) return false;
  if ((long long)(n - 1) * ldb * 2 + 2LL * k > 0xFFFFFFFFLL) return false;
  return true;
}

template <typename T>
int hgemm_tn(int m, int n, int k, const T* A, long long lda, const T* B, long long ldb, T* C, long long ldc) {
  if (!hgemm_fits(m, n, k, lda, ldb, A, B) || ldc < n) return 1;
  const long long tiles = (long long)((m + HG_BM - 1) / HG_BM) * ((n + HG_BN - 1) / HG_BN);
  hipLaunchKernelGGL((k_hgemm<T, HG_V>), dim3((unsigned)tiles), dim3(HG_THREADS), 0, current_stream(), m, n, k, A, lda, B,
                     ldb, C, ldc);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error((int)e, "k_hgemm launch");
    return 2;
  }
  return 0;
}

}  // namespace bnb

extern "C" {

// [additive] C[m, n] = A[m, k] . W[n, k]^T, row-major, bf16 / fp16 in and out, fp32 accumulation, on the hand-written
// k_hgemm (the GEMM of the large-prefill 4-bit path after cdequantize_blockwise_* into W; replaces the F.linear of
// ref:python_src_quants/autograd/_functions.py:507).  Returns 0 = launched, 1 = shape / alignment not supported
// (k % 64, 16-B aligned rows; nothing launched), 2 = launch error (cget_last_error*).
int chgemm_tn_bf16(int m, int n, int k, const bf16_t* A, int lda, const bf16_t* W, int ldw, bf16_t* C, int ldc) {
  return bnb::hgemm_tn<bf16_t>(m, n, k, A, lda, W, ldw, C, ldc);
}
int chgemm_tn_fp16(int m, int n, int k, const fp16_t* A, int lda, const fp16_t* W, int ldw, fp16_t* C, int ldc) {
  return bnb::hgemm_tn<fp16_t>(m, n, k, A, lda, W, ldw, C, ldc);
}

}  // extern "C"
