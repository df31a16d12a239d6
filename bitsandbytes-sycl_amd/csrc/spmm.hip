// Sparse (COO) x dense products of the LLM.int8 outlier decomposition, gfx950.
//
//   cspmm_coo_very_sparse_naive_{fp16,int8}  ref:sycl/pythonInterface.cpp:362-366
//                                            -> kspmm_coo_very_sparse_naive  ref:sycl/sycl_code/kernel_gemm.cpp:1398-1545
//                                               launcher spmm_coo_very_sparse_naive op_gemm.cpp:933-979
//   cspmm_coo                                ref:sycl/pythonInterface.cpp:358-361 (commented out there, Q18;
//                                            the Python wrapper functional.py:2656 still calls it -> upstream
//                                            cuSPARSE SpMM: C = A_coo @ B, fp32 compute, beta = 0)
//
// very_sparse semantics (kernel_gemm.cpp:1431-1540): workgroup b takes the row group max_idx[b] (rows
// sorted by nonzero count, descending), its `count = max_count[b]` nonzeros start at offset_rowidx[max_idx
// - 1] (0 for the first group) and belong to row rowidx[offset].  Per output column c the products are
// accumulated in an fp16 register in nonzero order -- every `acc = (float)acc + (float)b * (float)a`
// rounds to fp16 -- and the row of `out` is updated in place, out = (float)out + (float)acc (fp16).  With
// int8 B and dequant_stats: acc = (float)acc + (((float)half(stats[c]) * (1/127)) * b) * a, skipped when
// a or b is 0 (the stats pass through the kernel's fp16 shared memory).
//
// MI355X design: one 256-thread workgroup per nonzero row, 8 consecutive columns per thread (16-B fp16
// or 8-B int8 loads of B rows, 16-B read-modify-write of out), the <= 32 nonzeros of the row in SGPR-
// uniform registers.  The products are HBM-bound on B rows: count * colsB * sizeof(T) bytes per row.
#include "common.hpp"

namespace bnb {

constexpr int SPMM_THREADS = 256, SPMM_COLS = 8, SPMM_MAX_COUNT = 32;

template <typename T>
__global__ void __launch_bounds__(SPMM_THREADS)
k_spmm_coo_very_sparse(const int* __restrict__ max_count, const int* __restrict__ max_idx,
                       const int* __restrict__ offset_rowidx, const int* __restrict__ rowidx,
                       const int* __restrict__ colidx, const fp16_t* __restrict__ values, const T* __restrict__ B,
                       fp16_t* __restrict__ out, const float* __restrict__ dequant_stats, int colsB) {
  const int count = min(max_count[blockIdx.x], SPMM_MAX_COUNT);
  const int group = max_idx[blockIdx.x];
  const int offset = group == 0 ? 0 : offset_rowidx[group - 1];
  const int row = rowidx[offset];
  float a[SPMM_MAX_COUNT];
  int kcol[SPMM_MAX_COUNT];
#pragma unroll
  for (int i = 0; i < SPMM_MAX_COUNT; ++i) {
    a[i] = i < count ? (float)values[offset + i] : 0.0f;
    kcol[i] = i < count ? colidx[offset + i] : 0;
  }
  constexpr float DENORM = 1.0f / 127.0f;
  for (int c0 = SPMM_COLS * threadIdx.x; c0 < colsB; c0 += SPMM_COLS * SPMM_THREADS) {
    fp16_t acc[SPMM_COLS];
    float st[SPMM_COLS];
#pragma unroll
    for (int k = 0; k < SPMM_COLS; ++k) {
      acc[k] = (fp16_t)0.0f;
      st[k] = 0.0f;
      if (sizeof(T) == 1 && dequant_stats != nullptr && c0 + k < colsB)
        st[k] = __fmul_rn((float)(fp16_t)dequant_stats[c0 + k], DENORM);
    }
    for (int i = 0; i < count; ++i) {
      const T* brow = B + (long long)kcol[i] * colsB + c0;
      float b[SPMM_COLS];
#pragma unroll
      for (int k = 0; k < SPMM_COLS; ++k) b[k] = (c0 + k < colsB) ? (float)brow[k] : 0.0f;
#pragma unroll
      for (int k = 0; k < SPMM_COLS; ++k) {
        if (sizeof(T) == 1 && dequant_stats != nullptr) {
          if (b[k] != 0.0f && a[i] != 0.0f)
            acc[k] = Io<fp16_t>::from_f32(__fadd_rn((float)acc[k], __fmul_rn(__fmul_rn(st[k], b[k]), a[i])));
        } else {
          acc[k] = Io<fp16_t>::from_f32(__fadd_rn((float)acc[k], __fmul_rn(b[k], a[i])));
        }
      }
    }
    fp16_t* orow = out + (long long)row * colsB + c0;
#pragma unroll
    for (int k = 0; k < SPMM_COLS; ++k)
      if (c0 + k < colsB) orow[k] = Io<fp16_t>::from_f32(__fadd_rn((float)orow[k], (float)acc[k]));
  }
}

// C[r, :] = sum over the nonzeros of row r (in index order) of value * B[col, :], fp32 accumulation, one
// fp16 rounding; row_ptr[r] .. row_ptr[r+1] index the row-sorted COO (built by the Python wrapper).
// B element (k, j) at B[k * ldb + j] (row-major) or B[j * ldb + k] (transposed_B).
__global__ void __launch_bounds__(SPMM_THREADS)
k_spmm_coo_rows(const int* __restrict__ row_ptr, const int* __restrict__ colidx, const fp16_t* __restrict__ values,
                const fp16_t* __restrict__ B, fp16_t* __restrict__ C, int B_cols, int ldb, int ldc, bool transposed_B) {
  const int r = blockIdx.x;
  const int e0 = row_ptr[r], e1 = row_ptr[r + 1];
  for (int j = threadIdx.x; j < B_cols; j += SPMM_THREADS) {
    float acc = 0.0f;
    for (int e = e0; e < e1; ++e) {
      const long long k = colidx[e];
      const float b = (float)(transposed_B ? B[(long long)j * ldb + k] : B[k * ldb + j]);
      acc = __fadd_rn(acc, __fmul_rn((float)values[e], b));
    }
    C[(long long)r * ldc + j] = Io<fp16_t>::from_f32(acc);
  }
}

template <typename T>
void spmm_coo_very_sparse(int* max_count, int* max_idx, int* offset_rowidx, int* rowidx, int* colidx, fp16_t* values,
                          T* B, fp16_t* out, float* dequant_stats, int nnz_rows, int colsB) {
  if (nnz_rows <= 0 || colsB <= 0) return;
  hipLaunchKernelGGL((k_spmm_coo_very_sparse<T>), dim3(nnz_rows), dim3(SPMM_THREADS), 0, current_stream(), max_count,
                     max_idx, offset_rowidx, rowidx, colidx, values, B, out, dequant_stats, colsB);
  BNB_LAUNCH_CHECK("spmm_coo_very_sparse_naive");
}

}  // namespace bnb

using namespace bnb;

extern "C" {

// ref:sycl/pythonInterface.cpp:362-366 (argument list kept; nnz, rowsA, rowsB are not needed here)
void cspmm_coo_very_sparse_naive_fp16(int* max_count, int* max_idx, int* offset_rowidx, int* rowidx, int* colidx,
                                      fp16_t* values, fp16_t* B, fp16_t* out, float* dequant_stats, int nnz_rows,
                                      int nnz, int rowsA, int rowsB, int colsB) {
  BNB_RANGE("cspmm_coo_very_sparse_naive_fp16");
  (void)nnz; (void)rowsA; (void)rowsB;
  spmm_coo_very_sparse<fp16_t>(max_count, max_idx, offset_rowidx, rowidx, colidx, values, B, out, dequant_stats,
                               nnz_rows, colsB);
}
void cspmm_coo_very_sparse_naive_int8(int* max_count, int* max_idx, int* offset_rowidx, int* rowidx, int* colidx,
                                      fp16_t* values, signed char* B, fp16_t* out, float* dequant_stats, int nnz_rows,
                                      int nnz, int rowsA, int rowsB, int colsB) {
  BNB_RANGE("cspmm_coo_very_sparse_naive_int8");
  (void)nnz; (void)rowsA; (void)rowsB;
  spmm_coo_very_sparse<int8_t>(max_count, max_idx, offset_rowidx, rowidx, colidx, values, (int8_t*)B, out,
                               dequant_stats, nnz_rows, colsB);
}

// [additive] C = A_coo @ B over a row-sorted COO with row pointers (the Python wrapper sorts and builds
// row_ptr[A_rows + 1]); replaces the cuSPARSE-backed cspmm_coo of the reference's Python wrapper
// (functional.py:2656-2701).  Every row of C is written (0 for empty rows).
void cspmm_coo_rows(int* row_ptr, int* A_colidx, fp16_t* A_vals, int A_rows, int B_cols, int ldb, fp16_t* B, int ldc,
                    fp16_t* C, bool transposed_B) {
  BNB_RANGE("cspmm_coo_rows");
  if (A_rows <= 0 || B_cols <= 0) return;
  hipLaunchKernelGGL(k_spmm_coo_rows, dim3(A_rows), dim3(SPMM_THREADS), 0, current_stream(), row_ptr, A_colidx, A_vals,
                     B, C, B_cols, ldb, ldc, transposed_B);
  BNB_LAUNCH_CHECK("spmm_coo");
}

}  // extern "C"
