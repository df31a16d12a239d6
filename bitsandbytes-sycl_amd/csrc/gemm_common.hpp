// Shared MFMA / LDS helpers for the 4-bit GEMM kernels (gfx950).
#pragma once

#include "common.hpp"

namespace bnb {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

// v_mfma_f32_16x16x32_{bf16,f16}: lane l holds A[row l&15][k 8(l>>4)..+7], B[k ..][col l&15];
// C/D: col = l&15, row = 4(l>>4) + reg.
template <typename T> struct Mfma;
template <> struct Mfma<bf16_t> {
  __device__ static __forceinline__ f32x4_t mma(const uint4& a, const uint4& b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
  }
  __device__ static __forceinline__ uint32_t pack2(float lo, float hi) { return pack_bf16x2(lo, hi); }
};
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
// 32x32x16 (gfx950): lane l holds A[row l&31][k 8(l>>5)..+8] and B[k 8(l>>5)..+8][col l&31];
// D[r]: row 8(r>>2) + 4(l>>5) + (r&3), col l&31.  An MFMA holds the SIMD's vector issue for 8 of
// its 32 cycles (vs 8 of 16 for 16x16x32), leaving 3x the issue slots for the in-loop dequant.
template <typename T> struct Mfma32;
template <> struct Mfma32<bf16_t> {
  __device__ static __forceinline__ f32x16_t mma(const uint4& a, const uint4& b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
  }
};
template <> struct Mfma32<fp16_t> {
  __device__ static __forceinline__ f32x16_t mma(const uint4& a, const uint4& b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
  }
};

template <> struct Mfma<fp16_t> {
  __device__ static __forceinline__ f32x4_t mma(const uint4& a, const uint4& b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
  }
  __device__ static __forceinline__ uint32_t pack2(float lo, float hi) {
    return (uint32_t)__builtin_bit_cast(uint16_t, Io<fp16_t>::from_f32(lo)) |
           ((uint32_t)__builtin_bit_cast(uint16_t, Io<fp16_t>::from_f32(hi)) << 16);
  }
};

// LDS-DMA: 16 B (or 4 B) per lane from a per-lane global address to lds_base + lane*size.
// Issued from inline asm on purpose: with __builtin_amdgcn_global_load_lds, hipcc (ROCm 7.2) treats
// every later ds_read of the same __shared__ array as aliasing the in-flight DMA and drains it with
// s_waitcnt vmcnt(0) right there, serialising the prefetch.  The asm form is invisible to that
// bookkeeping, so the caller owns the wait: `s_waitcnt vmcnt(0)` before the barrier that publishes
// the stage.  lds_base must be wave-uniform (it goes to M0; M0 is saved/restored in the statement).
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_base) {
  unsigned keep;
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_base);
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
}
__device__ __forceinline__ void glds4(const void* gsrc, void* lds_base) {
  unsigned keep;
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_base);
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
}
__device__ __forceinline__ void wait_vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// byte offset of 16-B slot s (0..7) of row r in a [rows][64] 16-bit tile, XOR swizzled so that
// 16 lanes reading one slot of 16 consecutive rows (MFMA fragment) hit distinct banks
__device__ __forceinline__ int swz(int r, int s) { return r * 128 + ((s ^ (r & 7)) << 4); }

// bijective XCD-aware remap of the workgroup id (consecutive ids land on one XCD's L2)
__device__ __forceinline__ int xcd_remap(int wg, int nwg) {
  const int xcd = wg & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (wg >> 3);
}

extern Knob<int> g_tile_override;   // 0 = auto, 128 / 256 = force that tile kernel (tests / A-B benchmarks)

// ws/ksplit: split-K over ksplit workgroups per tile with fp32 partials in ws[ksplit][n][m]
// (ksplit == 1: ws unused, direct T output)
template <typename T>
void launch_gemm_4bit_256(int m, int n, int k, const T* A, const uint8_t* B, const float* absmax, const float* datatype,
                          T* out, int lda, int ldb, int ldc, int blocksize, float* ws, int ksplit);

// Few-token kernel (gemm4bit_skinny.hip): 1..64 activation rows (SK_MAX_TOKENS), K % 128 == 0.  Statistics either plain
// fp32 absmax or nested (q8 + code2 + absmax2 + offset, decoded in-kernel).
struct SkStats {
  const float* absmax;
  const uint8_t* q8;
  const float* code2;
  const float* absmax2;
  const float* offset;
  int bs_shift, bs2_shift;
};
long long skinny_workspace_bytes(int m, int n, int k);
// the 33..64-token kernel (gemm4bit_t64.hip): fp32 split partials it needs (0: unsplit), and its launch (false: not
// applicable, nothing launched)
long long t64_workspace_bytes(int m, int n, int k);
template <typename T>
bool launch_gemm_4bit_t64(int m, int n, int k, const T* A, int lda, const uint8_t* B, int ldb, SkStats st,
                          int blocksize, int blocksize2, const float* code, T* out, int ldc, float* ws,
                          long long ws_bytes);
int device_cu_count();
// out[t, n] = T(sum_s ws[s][t][n]) (fp32 split partials, row-major [rows][cols] per split), splits summed in order
template <typename T>
void launch_splitk_rows_reduce(const float* ws, int nsplit, int rows, int cols, T* out, int ldc);
template <typename T>
bool launch_gemm_4bit_skinny(int m, int n, int k, const T* A, int lda, const uint8_t* B, int ldb, SkStats st,
                             int blocksize, int blocksize2, const float* code, T* out, int ldc, float* ws,
                             long long ws_bytes);

// Few-token kernel on the 32x32x16 MFMA, whole K per workgroup, no workspace (gemm4bit_fewtok.hip): 1..32 activation
// rows, K % 64 == 0, K >= 256.  False when the shape / alignment does not fit (nothing launched).
template <typename T>
bool launch_gemm_4bit_fewtok(int m, int n, int k, const T* A, int lda, const uint8_t* B, int ldb, SkStats st,
                             int blocksize, int blocksize2, const float* code, T* out, int ldc);

// Few-token kernel with whole K per workgroup (gemm4bit_wk.hip): 1..32 activation rows, K % 128 == 0, no workspace.
// False when the shape / alignment does not fit or the A/B knob selects the skinny kernel.
template <typename T>
bool launch_gemm_4bit_wk(int m, int n, int k, const T* A, int lda, const uint8_t* B, int ldb, SkStats st,
                         int blocksize, int blocksize2, const float* code, T* out, int ldc);

}  // namespace bnb
