// Shared LLM.int8 device helpers: tile layouts, int8 rounding, the mm_dequant formula, epilogue kinds.
#pragma once

#include "common.hpp"

namespace bnb {

enum Fmt { ROW = 0, COL32 = 2, TURING = 3, AMPERE = 4 };

__host__ __device__ __forceinline__ long long pad_to(long long v, long long m) { return (v + m - 1) / m * m; }

__device__ __forceinline__ int ampere_row(int x) { return 8 * ((x & 7) >> 1) + 2 * (x >> 3) + (x & 1); }

// offset of element (r, c) in format F, `ld` = the format's leading dimension:
//   ROW r*ld + c; COL32 ld = 32*rows; TURING ld = 32*pad8(rows); AMPERE ld = 32*pad32(rows)
// (ref:sycl/sycl_code/blas_utils.h:244-346; kernel_quant.cpp:3640-3835)
template <int F>
__device__ __forceinline__ long long fmt_offset(long long r, long long c, long long ld) {
  if constexpr (F == ROW) return r * ld + c;
  else if constexpr (F == COL32) return (c >> 5) * ld + 32 * r + (c & 31);
  else if constexpr (F == TURING)
    return (c >> 5) * ld + (r >> 3) * 256 + 128 * (r & 1) + 16 * ((c & 31) >> 2) + 4 * ((r & 7) >> 1) + (c & 3);
  else return (c >> 5) * ld + (r >> 5) * 1024 + 32 * ampere_row((int)(r & 31)) + (c & 31);
}

__device__ __forceinline__ int8_t rint_i8(float v) {
  // (char)rint(v): half-to-even; NaN -> 0; saturating (|v| <= 127 for in-range data)
  float r = rintf(v);
  if (r != r) r = 0.0f;
  r = fminf(fmaxf(r, -128.0f), 127.0f);
  return (int8_t)(int)r;
}

// out = half( ((float(C) * 6.200012e-05f) * rowStat) * colStat + bias )  (kernel_quant.cpp:3969 order;
// explicit _rn ops + an opaque barrier forbid contraction and the f16 fma_mix fold)
__device__ __forceinline__ fp16_t mm_dequant_value(int32_t acc, float rs, float cs, float bias) {
  float v = __fmul_rn((float)acc, 6.200012e-05f);
  v = __fmul_rn(v, rs);
  v = opaque(__fmul_rn(v, cs));
  v = __fadd_rn(v, bias);
  return Io<fp16_t>::from_f32(v);
}

enum Epi { EPI_I32_COL32 = 0, EPI_I8_COL32 = 1, EPI_I8_COL32_ROWSCALE = 2, EPI_F16_ROW_DEQUANT = 3, EPI_I32_ROW = 4 };

// 256x256-tile int8 GEMM (igemm_256.hip); returns false when the shape/layout is not covered
// ws / ws_bytes: a caller workspace that lets small tile grids of row-major operands run split-K (int32 partials,
// summed exactly by a reduce launch that also applies the epilogue); NULL or too small: no split
template <int AF, int BF, int EPI>
bool launch_igemm_256(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, const float* row_scale,
                      long long lda, long long ldb, long long ldc, const float* rowStats, const float* colStats,
                      const fp16_t* bias, int32_t* ws = nullptr, long long ws_bytes = 0);
int igemm_splitk_factor(int m, int n, int k);
// row-major int8 product on the 4-wave 256 x 256 kernel (hgemm.hip): 0 = launched, 1 = not covered, 2 = launch error
int igemm_4wave(int m, int n, int k, const int8_t* A, long long lda, const int8_t* B, long long ldb, void* C,
                long long ldc, bool dequant, const float* rowStats, const float* colStats, const fp16_t* bias);
long long hgemm_tiles(int m, int n);
long long igemm_workspace_bytes(int m, int n, int k);

}  // namespace bnb
