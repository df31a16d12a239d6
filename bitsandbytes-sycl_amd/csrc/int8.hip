// LLM.int8 hot path on gfx950: row/col statistics, double_quant, tile layouts,
// igemmlt on the int8 MFMA and the int32 -> fp16 dequant (standalone and fused).
//
// Replaces (same C-ABI names, argument order and meaning):
//   cget_col_row_stats            ref:sycl/pythonInterface.cpp:335  -> kgetColRowStats    kernel_quant.cpp:3214-3379
//   cdouble_rowcol_quant          ref:sycl/pythonInterface.cpp:338  -> kDoubleRowColQuant kernel_quant.cpp:3384-3512
//   ctransform_row2{col32,turing,ampere}{,T}  ref:sycl/pythonInterface.cpp:341-357 -> kTransformRowToFormat 3516-3840
//   cigemmlt_{turing,ampere}_{32,8,8_rowscale} ref:sycl/pythonInterface.cpp:298-316 -> igemmlt op_gemm.cpp:541-655
//   cdequant_mm_int32_fp16        ref:sycl/pythonInterface.cpp:333  -> kdequant_mm_int32_fp16 kernel_quant.cpp:3846-3987
//   cextractOutliers_{turing,ampere} ref:sycl/pythonInterface.cpp:368-369 -> kExtractOutliers 3992-
// Additive: ctransform_{turing,ampere,col32}2row (called by functional.py:2645-2647, never exported by the
// reference, Q18) and cigemmlt_row_dequant_fp16 (row-major int8 A and B, int32 accumulators dequantised
// to fp16 in the epilogue = igemmlt + mm_dequant in one launch).
//
// Layout maps (offset of element (r, c) of a [rows, cols] matrix), blas_utils.h:244-346:
//   col32      (c/32)*ld + 32 r + c%32                                  ld = 32*rows
//   col_turing (c/32)*ld + (r/8)*256 + 128(r%2) + 16((c%32)/4) + 4((r%8)/2) + c%4     ld = 32*pad8(rows)
//   col_ampere (c/32)*ld + (r/32)*1024 + 32*arow(r%32) + c%32, arow(x) = 8((x%8)/2) + 2(x/8) + x%2   ld = 32*pad32(rows)
#include "int8_common.hpp"

namespace bnb {

// ============================================================================ row/col statistics
// Tile: 16 rows x 256 cols per 256-thread workgroup (the reference's TILE_ROWS/TILE_COLS, which also
// fix the layout of nnz_count_row: entry (tile*16 + r + 1), tile = row_tile*col_tiles + col_tile).
// Thread t: 8 consecutive columns (t%32) of rows (t/32) and (t/32)+8.

__device__ __forceinline__ void load8_half(const fp16_t* A, long long row, int c0, int cols, bool vec, float (&v)[8]) {
  const fp16_t* p = A + row * (long long)cols + c0;
  if (vec && c0 + 8 <= cols) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = (float)__builtin_bit_cast(fp16_t, (uint16_t)(w[i] & 0xFFFF));
      v[2 * i + 1] = (float)__builtin_bit_cast(fp16_t, (uint16_t)(w[i] >> 16));
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (c0 + i < cols) ? (float)p[i] : 0.0f;
  }
}

__device__ __forceinline__ void atomic_max_nonneg(float* addr, float v) {
  // valid for v >= 0 against any existing value (negative init or non-negative maxima)
  atomicMax(reinterpret_cast<int*>(addr), __float_as_int(v));
}

template <bool SPARSE>
__global__ void __launch_bounds__(256)
k_colrow_stats(const fp16_t* __restrict__ A, float* __restrict__ rowStats, float* __restrict__ colStats,
               int* __restrict__ nnz_count_row, float threshold, int rows, int cols, int col_tiles, bool vec) {
  __shared__ float s_col[8][256];
  __shared__ int s_nnz[16];
  const int tid = threadIdx.x;
  const int row_tile = blockIdx.x / col_tiles, col_tile = blockIdx.x % col_tiles;
  const int base_row = row_tile * 16, base_col = col_tile * 256;
  const int cg = tid & 31, rs = tid >> 5;
  const int c0 = base_col + 8 * cg;
  if (tid < 16) s_nnz[tid] = 0;
  float cmax[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) cmax[i] = -3.402823466e+38f;
  float rmax[2];
  int rnnz[2] = {0, 0};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = base_row + rs + 8 * h;
    rmax[h] = -3.402823466e+38f;
    if (row < rows && c0 < cols) {
      float v[8];
      load8_half(A, row, c0, cols, vec, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float a = fabsf(v[i]);
        if (c0 + i >= cols) a = -3.402823466e+38f;
        if (SPARSE && c0 + i < cols && a >= threshold) { rnnz[h] += 1; a = 0.0f; }
        cmax[i] = fmaxf(cmax[i], a);
        rmax[h] = fmaxf(rmax[h], a);
      }
    }
    // row reduce over the 32 lanes that share this row (lanes 0-31 / 32-63 of the wave)
    rmax[h] = wave_max_xor(rmax[h], 32);
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = base_row + rs + 8 * h;
    if ((tid & 31) == 0 && row < rows && rmax[h] >= 0.0f) atomic_max_nonneg(&rowStats[row], rmax[h]);
    if (SPARSE) {
      int c = rnnz[h];
      for (int o = 1; o < 32; o <<= 1) c += __shfl_xor(c, o, 64);
      if ((tid & 31) == 0) s_nnz[rs + 8 * h] = c;
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) s_col[rs][8 * cg + i] = cmax[i];
  __syncthreads();
  {
    float m = s_col[0][tid];
#pragma unroll
    for (int r = 1; r < 8; ++r) m = fmaxf(m, s_col[r][tid]);
    const int col = base_col + tid;
    if (col < cols && m >= 0.0f) atomic_max_nonneg(&colStats[col], m);
  }
  if (SPARSE && tid < 16) nnz_count_row[blockIdx.x * 16 + tid + 1] = s_nnz[tid];
}

// ============================================================================ double row/col quant

template <bool SPARSE>
__global__ void __launch_bounds__(256)
k_double_rowcol_quant(const fp16_t* __restrict__ A, const float* __restrict__ rowStats,
                      const float* __restrict__ colStats, int8_t* __restrict__ out_col, int8_t* __restrict__ out_row,
                      int* __restrict__ rowidx, int* __restrict__ colidx, fp16_t* __restrict__ val,
                      const int* __restrict__ nnz_block_ptr, float threshold, int rows, int cols, int col_tiles,
                      bool vec) {
  __shared__ unsigned s_next[16];
  const int tid = threadIdx.x;
  const int row_tile = blockIdx.x / col_tiles, col_tile = blockIdx.x % col_tiles;
  const int base_row = row_tile * 16, base_col = col_tile * 256;
  const int cg = tid & 31, rs = tid >> 5;
  const int c0 = base_col + 8 * cg;
  if (SPARSE) {
    if (tid < 16) s_next[tid] = (unsigned)nnz_block_ptr[blockIdx.x * 16 + tid];
    __syncthreads();
  }
  if (c0 >= cols) return;
  float cs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) cs[i] = (c0 + i < cols) ? __fdiv_rn(127.0f, colStats[c0 + i]) : 0.0f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = base_row + rs + 8 * h;
    if (row >= rows) continue;
    float v[8];
    load8_half(A, row, c0, cols, vec, v);
    const float rsc = __fdiv_rn(127.0f, rowStats[row]);
    uint32_t qr[2] = {0, 0}, qc[2] = {0, 0};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int8_t r8 = rint_i8(__fmul_rn(v[i], rsc));
      if (SPARSE && c0 + i < cols && fabsf(v[i]) >= threshold) {
        r8 = 0;
        const unsigned slot = atomicAdd(&s_next[rs + 8 * h], 1u);
        rowidx[slot] = row;
        colidx[slot] = c0 + i;
        val[slot] = (fp16_t)v[i];
      }
      const int8_t c8 = rint_i8(__fmul_rn(v[i], cs[i]));
      qr[i >> 2] |= (uint32_t)(uint8_t)r8 << (8 * (i & 3));
      qc[i >> 2] |= (uint32_t)(uint8_t)c8 << (8 * (i & 3));
    }
    const long long off = (long long)row * cols + c0;
    if (vec && c0 + 8 <= cols) {
      *reinterpret_cast<uint2*>(out_row + off) = make_uint2(qr[0], qr[1]);
      *reinterpret_cast<uint2*>(out_col + off) = make_uint2(qc[0], qc[1]);
    } else {
      for (int i = 0; i < 8 && c0 + i < cols; ++i) {
        out_row[off + i] = (int8_t)(qr[i >> 2] >> (8 * (i & 3)));
        out_col[off + i] = (int8_t)(qc[i >> 2] >> (8 * (i & 3)));
      }
    }
  }
}

// ============================================================================ wide-tile stats + double quant
// The threshold == 0 path (no outliers, no COO) on 16-B aligned rows with cols % 8 == 0: 32 x 512 tiles,
// thread t owns 8 columns (t % 64) of the 8 rows (t / 64) + 4 i, so each thread keeps 8 x 16-B loads in
// flight and each wave covers a whole 512-column row segment (row max by one wave reduction).  Column
// atomics drop 2x (one per column per 32-row tile instead of per 16-row tile), row atomics 2x, and
// workgroups carry 32 KiB instead of 8.  Same maxima / roundings as the 16 x 256 kernels above (the
// max is order-free; the quantisation is the same expression per element).
constexpr int W_ROWS = 32, W_COLS = 512;

__global__ void __launch_bounds__(256)
k_colrow_stats_wide(const fp16_t* __restrict__ A, float* __restrict__ rowStats, float* __restrict__ colStats,
                    int rows, int cols, int col_tiles) {
  __shared__ float s_col[4][W_COLS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row_tile = blockIdx.x / col_tiles, col_tile = blockIdx.x % col_tiles;
  const int base_row = row_tile * W_ROWS, c0 = col_tile * W_COLS + 8 * lane;
  const bool has_cols = c0 < cols;
  uint4 raw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = base_row + wave + 4 * i;
    raw[i] = (has_cols && row < rows) ? *reinterpret_cast<const uint4*>(A + (long long)row * cols + c0)
                                      : make_uint4(0, 0, 0, 0);
  }
  float cmax[8], rmax[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cmax[j] = -3.402823466e+38f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t w[4] = {raw[i].x, raw[i].y, raw[i].z, raw[i].w};
    const int row = base_row + wave + 4 * i;
    const bool ok = has_cols && row < rows;
    rmax[i] = -3.402823466e+38f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = (float)__builtin_bit_cast(fp16_t, (uint16_t)(w[j >> 1] >> (16 * (j & 1))));
      const float a = ok ? fabsf(v) : -3.402823466e+38f;
      cmax[j] = fmaxf(cmax[j], a);
      rmax[i] = fmaxf(rmax[i], a);
    }
  }
  // the 8 row maxima over the wave's 64 lanes by a halving butterfly: across lane bits 5, 4, 3 each lane
  // keeps half of its rows (4 + 2 + 1 shuffles), then bits 0-2 reduce the one left (3) -- 10 shuffles
  // instead of 8 full reductions (48); lane 8r' + 0 ends with row i = 4 b5 + 2 b4 + b3 of its lane id
  {
    const int h5 = (lane >> 5) & 1, h4 = (lane >> 4) & 1, h3 = (lane >> 3) & 1;
    float r4[4], r2[2], r1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float send = h5 ? rmax[k] : rmax[k + 4];
      const float mine = h5 ? rmax[k + 4] : rmax[k];
      r4[k] = fmaxf(mine, __shfl_xor(send, 32, 64));
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const float send = h4 ? r4[k] : r4[k + 2];
      const float mine = h4 ? r4[k + 2] : r4[k];
      r2[k] = fmaxf(mine, __shfl_xor(send, 16, 64));
    }
    {
      const float send = h3 ? r2[0] : r2[1];
      const float mine = h3 ? r2[1] : r2[0];
      r1 = fmaxf(mine, __shfl_xor(send, 8, 64));
    }
    r1 = fmaxf(r1, __shfl_xor(r1, 1, 64));
    r1 = fmaxf(r1, __shfl_xor(r1, 2, 64));
    r1 = fmaxf(r1, __shfl_xor(r1, 4, 64));
    const int i = 4 * h5 + 2 * h4 + h3;
    const int row = base_row + wave + 4 * i;
    if ((lane & 7) == 0 && row < rows && r1 >= 0.0f) atomic_max_nonneg(&rowStats[row], r1);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) s_col[wave][8 * lane + j] = cmax[j];
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int cl = tid + 256 * h;
    const float m = fmaxf(fmaxf(s_col[0][cl], s_col[1][cl]), fmaxf(s_col[2][cl], s_col[3][cl]));
    const int col = col_tile * W_COLS + cl;
    if (col < cols && m >= 0.0f) atomic_max_nonneg(&colStats[col], m);
  }
}

__global__ void __launch_bounds__(256)
k_double_rowcol_quant_wide(const fp16_t* __restrict__ A, const float* __restrict__ rowStats,
                           const float* __restrict__ colStats, int8_t* __restrict__ out_col,
                           int8_t* __restrict__ out_row, int rows, int cols, int col_tiles) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row_tile = blockIdx.x / col_tiles, col_tile = blockIdx.x % col_tiles;
  const int base_row = row_tile * W_ROWS, c0 = col_tile * W_COLS + 8 * lane;
  if (c0 >= cols) return;
  uint4 raw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = base_row + wave + 4 * i;
    if (row < rows) raw[i] = *reinterpret_cast<const uint4*>(A + (long long)row * cols + c0);
  }
  float cs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cs[j] = __fdiv_rn(127.0f, colStats[c0 + j]);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = base_row + wave + 4 * i;
    if (row >= rows) break;
    const float rsc = __fdiv_rn(127.0f, rowStats[row]);
    const uint32_t w[4] = {raw[i].x, raw[i].y, raw[i].z, raw[i].w};
    uint32_t qr[2] = {0, 0}, qc[2] = {0, 0};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = (float)__builtin_bit_cast(fp16_t, (uint16_t)(w[j >> 1] >> (16 * (j & 1))));
      qr[j >> 2] |= (uint32_t)(uint8_t)rint_i8(__fmul_rn(v, rsc)) << (8 * (j & 3));
      qc[j >> 2] |= (uint32_t)(uint8_t)rint_i8(__fmul_rn(v, cs[j])) << (8 * (j & 3));
    }
    const long long off = (long long)row * cols + c0;
    *reinterpret_cast<uint2*>(out_row + off) = make_uint2(qr[0], qr[1]);
    *reinterpret_cast<uint2*>(out_col + off) = make_uint2(qc[0], qc[1]);
  }
}

// ============================================================================ one-pass row quantisation
// The forward of LLM.int8 without outliers and without a backward needs only the row-normalised CA and
// its row statistics (CAt / column stats serve the backward, autograd/_functions.py:436-483).  One wave
// per row keeps the whole row in registers (cols <= 64 * 8 * RQ_MAX_VEC), so A is read once: the row
// max (the row half of kgetColRowStats, kernel_quant.cpp:3214-3379) and the row quantisation (the row
// half of kDoubleRowColQuant, 3384-3512) with the same expressions -- rowStats = max |a| (or the
// -50000 the callers pre-fill when a row has no finite |a|), CA = rint(a * (127 / rowStats)).
constexpr int RQ_MAX_VEC = 32;   // 16-B vectors per lane: K <= 16384
typedef uint32_t rq_u32x2_t __attribute__((ext_vector_type(2)));
// cint8_set_row_quant_store; off: measured neutral (row quantise 30.5 vs 30.7 us, + igemmlt 156.7 vs 156.8 us at
// 4096 x 11008; the 90 MB fp16 read, not the 45 MB int8 write, sets its time; profiles/lab/r04_store_policy.txt)
static Knob<int> g_rq_wt{0};

// NV = 16-B vectors per lane (the smallest instance that holds the row: registers decide how many rows a CU keeps in
// flight -- 32 vectors cost 171 VGPRs, two waves per SIMD)
// WT: the int8 row stores write-through (device scope), so the GEMM launch that reads CA next inherits no dirty L2
// lines to write back at its boundary (cint8_set_row_quant_store)
template <int NV, bool WT = false>
__global__ void __launch_bounds__(256)
k_row_quant(const fp16_t* __restrict__ A, float* __restrict__ rowStats, int8_t* __restrict__ out, int rows, int cols) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nvec = cols >> 3;
  const uint4* src = reinterpret_cast<const uint4*>(A + (long long)row * cols);
  uint4 v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < nvec) v[i] = src[c];
  }
  float m = -3.402823466e+38f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (lane + 64 * i < nvec) {
      const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf((float)__builtin_bit_cast(fp16_t, (uint16_t)(w[j >> 1] >> (16 * (j & 1))))));
    }
  }
  m = wave_max_xor(m, 64);
  if (!(m >= 0.0f)) m = -50000.0f;               // the callers' pre-fill, untouched by atomicMax
  if (lane == 0) rowStats[row] = m;
  const float rsc = __fdiv_rn(127.0f, m);
  uint2* dst = reinterpret_cast<uint2*>(out + (long long)row * cols);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < nvec) {
      const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
      uint32_t q[2] = {0, 0};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = (float)__builtin_bit_cast(fp16_t, (uint16_t)(w[j >> 1] >> (16 * (j & 1))));
        q[j >> 2] |= (uint32_t)(uint8_t)rint_i8(__fmul_rn(a, rsc)) << (8 * (j & 3));
      }
      if constexpr (WT)
        asm volatile("global_store_dwordx2 %0, %1, off sc1" : : "v"(dst + c), "v"((rq_u32x2_t){q[0], q[1]}) : "memory");
      else
        dst[c] = make_uint2(q[0], q[1]);
    }
  }
}

// ============================================================================ layout transforms
// One thread per element (row-major source index i).  These are load-time / small-tensor ops.

template <int F, bool TRANSPOSE, bool INVERSE>
__global__ void k_transform(const int8_t* __restrict__ src, int8_t* __restrict__ dst, int rows, int cols) {
  const long long n = (long long)rows * cols;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / cols, c = i % cols;
    // logical matrix in the target format: A (rows x cols) or A^T (cols x rows)
    const long long lr = TRANSPOSE ? c : r, lc = TRANSPOSE ? r : c;
    const long long lrows = TRANSPOSE ? cols : rows;
    long long ld;
    if constexpr (F == COL32) ld = 32 * lrows;
    else if constexpr (F == TURING) ld = 32 * pad_to(lrows, 8);
    else ld = 32 * pad_to(lrows, 32);
    const long long o = fmt_offset<F>(lr, lc, ld);
    if (INVERSE) dst[i] = src[o];
    else dst[o] = src[i];
  }
}

// Row-major -> col32 / col_ampere, 16 B per lane: a 16-column run of one row stays contiguous in both formats
// (c % 32 is the fastest index), so each lane moves one 16-B chunk with one load and one store.  Needs
// cols % 16 == 0 and 16-B aligned pointers; the padding of the output is not written (the reference's buffers
// come zero-filled, functional.py:482-518).
// Lanes walk the OUTPUT in order (consecutive lanes store consecutive 16 B): chunk i = (column block cb, row r,
// half h) for col32 -- output byte 16 i; for col_ampere the row order inside a 32-row block is the format's
// interleave, so the lane's source row is found through the inverse map.
template <int F>
__global__ void __launch_bounds__(256)
k_transform16(const int8_t* __restrict__ src, int8_t* __restrict__ dst, int rows, int cols) {
  const long long rp = (F == COL32) ? rows : pad_to(rows, 32);   // rows held per column block
  const long long nq = (long long)((cols + 31) >> 5) * rp * 2;   // a half-filled last block skips its h = 1 lanes
  const long long ld = 32 * rp;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += (long long)gridDim.x * blockDim.x) {
    const long long cb = i / (2 * rp), rem = i - cb * 2 * rp;
    const int h = (int)(rem & 1);
    long long r = rem >> 1;                                   // row slot inside the column block
    if constexpr (F == AMPERE) {
      // slot s = 32 (r / 32) + x holds source row 32 (r / 32) + a^-1(x), a(y) = 8 ((y % 8) / 2) + 2 (y / 8) + y % 2
      const int x = (int)(r & 31);
      const int y = 8 * ((x >> 1) & 3) + 2 * (x >> 3) + (x & 1);   // the inverse interleave
      r = (r & ~31LL) + y;
    }
    const int c = (int)(32 * cb + 16 * h);
    if (r >= rows || c >= cols) continue;
    const uint4 v = *reinterpret_cast<const uint4*>(src + r * cols + c);
    *reinterpret_cast<uint4*>(dst + fmt_offset<F>(r, c, ld)) = v;
  }
}

template <int F, bool TRANSPOSE, bool INVERSE>
static void launch_transform(const int8_t* A, int8_t* out, int rows, int cols) {
  const long long n = (long long)rows * cols;
  if (n <= 0) return;
  if constexpr ((F == COL32 || F == AMPERE) && !TRANSPOSE && !INVERSE) {
    if (cols % 16 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)out & 15) == 0) {
      long long g = (n / 16 + 255) / 256;
      if (g > 16384) g = 16384;
      hipLaunchKernelGGL((k_transform16<F>), dim3((unsigned)g), dim3(256), 0, current_stream(), A, out, rows, cols);
      BNB_LAUNCH_CHECK("transform");
      return;
    }
  }
  long long g = (n + 255) / 256;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL((k_transform<F, TRANSPOSE, INVERSE>), dim3((unsigned)g), dim3(256), 0, current_stream(), A, out, rows, cols);
  BNB_LAUNCH_CHECK("transform");
}

// ============================================================================ dequant_mm_int32_fp16

// C in col32 layout (the reference's igemmlt output, ldc = 32*numRows); 4 consecutive columns per thread
__global__ void __launch_bounds__(256)
k_dequant_mm_col32(const int32_t* __restrict__ C, const float* __restrict__ rowStats, const float* __restrict__ colStats,
                   fp16_t* __restrict__ out, const fp16_t* __restrict__ bias, int numRows, int numCols) {
  const long long groups = (long long)numRows * ((numCols + 3) / 4);
  const int cgroups = (numCols + 3) / 4;
  for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(g / cgroups), c0 = 4 * (int)(g % cgroups);
    const float rs = rowStats[r];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + j;
      if (c >= numCols) break;
      const int32_t acc = C[(long long)(c >> 5) * 32 * numRows + 32LL * r + (c & 31)];
      out[(long long)r * numCols + c] = mm_dequant_value(acc, rs, colStats[c], bias ? (float)bias[c] : 0.0f);
    }
  }
}

// 8 consecutive columns per lane (numCols % 8 == 0, 16-B aligned): two 16-B int32 loads (one col32 run), the
// column statistics and bias as 16-B loads, one 16-B fp16 store; same per-element arithmetic (mm_dequant_value)
__global__ void __launch_bounds__(256)
k_dequant_mm_col32_v8(const int32_t* __restrict__ C, const float* __restrict__ rowStats,
                      const float* __restrict__ colStats, fp16_t* __restrict__ out, const fp16_t* __restrict__ bias,
                      int numRows, int numCols) {
  const int cg = numCols >> 3;
  const long long groups = (long long)numRows * cg;
  for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(g / cg), c0 = 8 * (int)(g - (long long)r * cg);
    const int32_t* src = C + (long long)(c0 >> 5) * 32 * numRows + 32LL * r + (c0 & 31);
    const int4 a0 = reinterpret_cast<const int4*>(src)[0], a1 = reinterpret_cast<const int4*>(src)[1];
    const float4 s0 = reinterpret_cast<const float4*>(colStats + c0)[0];
    const float4 s1 = reinterpret_cast<const float4*>(colStats + c0)[1];
    float bv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (bias) {
      const uint4 bw = *reinterpret_cast<const uint4*>(bias + c0);
      const uint32_t w[4] = {bw.x, bw.y, bw.z, bw.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bv[2 * j] = (float)__builtin_bit_cast(fp16_t, (uint16_t)(w[j] & 0xFFFF));
        bv[2 * j + 1] = (float)__builtin_bit_cast(fp16_t, (uint16_t)(w[j] >> 16));
      }
    }
    const float rs = rowStats[r];
    const int32_t acc[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const float cs[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      o[j] = (uint32_t)__builtin_bit_cast(uint16_t, mm_dequant_value(acc[2 * j], rs, cs[2 * j], bv[2 * j])) |
             ((uint32_t)__builtin_bit_cast(uint16_t, mm_dequant_value(acc[2 * j + 1], rs, cs[2 * j + 1], bv[2 * j + 1]))
              << 16);
    *reinterpret_cast<uint4*>(out + (long long)r * numCols + c0) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// ============================================================================ igemmlt (int8 MFMA)
// C[i, j] = sum_k A[i, k] * B[j, k]   (A m x k, B n x k, both K-contiguous per row)
// 128 x 128 output tile per 256-thread workgroup (2x2 waves, 64x64 per wave, v_mfma_i32_16x16x64_i8),
// BK = 128 bytes, two LDS stages with register staging (issue loads before the MFMA phase, write to
// LDS after the next barrier).  Operand fragments: lane l holds 16 consecutive k of row (l&15),
// k-chunk (l>>4) — the same k assignment for A and B, so the dot product is exact for any internal
// k order of the instruction.

typedef __attribute__((ext_vector_type(4))) int i32x4_t;


constexpr int Q_BM = 128, Q_BN = 128, Q_BK = 128, Q_THREADS = 256;
constexpr int Q_TILE = Q_BM * Q_BK;   // 16 KiB

__device__ __forceinline__ int qswz(int r, int s) { return r * 128 + ((s ^ (r & 7)) << 4); }

// Stage one 128 x 128 operand tile into registers: thread t -> row t>>1, k-half (t&1)*64, 4 x 16 B.
template <int F>
__device__ __forceinline__ void load_tile(const int8_t* __restrict__ P, long long ld, int row0, int nrows, int k0,
                                          int K, uint4 (&v)[4]) {
  const int tr = threadIdx.x >> 1, th = threadIdx.x & 1;
  const long long r = min(row0 + tr, nrows - 1);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = k0 + 64 * th + 16 * s;
    if (k + 16 <= K) {
      if constexpr (F == TURING) {
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) w[q] = *reinterpret_cast<const uint32_t*>(P + fmt_offset<F>(r, k + 4 * q, ld));
        v[s] = make_uint4(w[0], w[1], w[2], w[3]);
      } else {
        v[s] = *reinterpret_cast<const uint4*>(P + fmt_offset<F>(r, k, ld));
      }
    } else {
      uint32_t w[4] = {0, 0, 0, 0};
      for (int b = 0; b < 16; ++b)
        if (k + b < K) w[b >> 2] |= (uint32_t)(uint8_t)P[fmt_offset<F>(r, k + b, ld)] << (8 * (b & 3));
      v[s] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

__device__ __forceinline__ void store_tile(uint8_t* lds, const uint4 (&v)[4]) {
  const int tr = threadIdx.x >> 1, th = threadIdx.x & 1;
#pragma unroll
  for (int s = 0; s < 4; ++s) *reinterpret_cast<uint4*>(lds + qswz(tr, 4 * th + s)) = v[s];
}

template <int AF, int BF, int EPI>
__global__ void __launch_bounds__(Q_THREADS, 2)
k_igemm(int M, int N, int K, const int8_t* __restrict__ A, const int8_t* __restrict__ B, void* __restrict__ Cout,
        const float* __restrict__ row_scale, long long lda, long long ldb, long long ldc,
        const float* __restrict__ rowStats, const float* __restrict__ colStats, const fp16_t* __restrict__ bias) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[4 * Q_TILE];
  uint8_t* As = smem;
  uint8_t* Bs = smem + 2 * Q_TILE;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  const int tilesN = (N + Q_BN - 1) / Q_BN, tilesM = (M + Q_BM - 1) / Q_BM;
  const int nwg = tilesN * tilesM;
  int wg = blockIdx.x;
  {
    const int xcd = wg & 7, q = nwg >> 3, r = nwg & 7;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (wg >> 3);
  }
  constexpr int GROUP = 8;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * Q_BM, n0 = tn * Q_BN;

  const int wm = wave >> 1, wn = wave & 1;
  i32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = i32x4_t{0, 0, 0, 0};

  const int nk = (K + Q_BK - 1) / Q_BK;
  uint4 ra[4], rb[4];
  load_tile<AF>(A, lda, m0, M, 0, K, ra);
  load_tile<BF>(B, ldb, n0, N, 0, K, rb);
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    uint8_t* as = As + cur * Q_TILE;
    uint8_t* bs = Bs + cur * Q_TILE;
    store_tile(as, ra);
    store_tile(bs, rb);
    __syncthreads();
    if (t + 1 < nk) {
      load_tile<AF>(A, lda, m0, M, (t + 1) * Q_BK, K, ra);
      load_tile<BF>(B, ldb, n0, N, (t + 1) * Q_BK, K, rb);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 a[4], b[4];
      const int slot = 4 * ks + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const uint4*>(as + qswz(64 * wm + 16 * i + (lane & 15), slot));
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const uint4*>(bs + qswz(64 * wn + 16 * j + (lane & 15), slot));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4_t, a[i]),
                                                            __builtin_bit_cast(i32x4_t, b[j]), acc[i][j], 0, 0, 0);
    }
  }

#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + 64 * wm + 16 * i + 4 * (lane >> 4) + r;
      if (row >= M) continue;
      float rs = 0.0f;
      if constexpr (EPI == EPI_F16_ROW_DEQUANT) rs = rowStats[row];
      if constexpr (EPI == EPI_I8_COL32_ROWSCALE) rs = row_scale[row];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + 64 * wn + 16 * j + (lane & 15);
        if (col >= N) continue;
        const int32_t v = acc[i][j][r];
        if constexpr (EPI == EPI_I32_COL32) {
          reinterpret_cast<int32_t*>(Cout)[fmt_offset<COL32>(row, col, ldc)] = v;
        } else if constexpr (EPI == EPI_I32_ROW) {
          reinterpret_cast<int32_t*>(Cout)[(long long)row * ldc + col] = v;
        } else if constexpr (EPI == EPI_I8_COL32) {
          reinterpret_cast<int8_t*>(Cout)[fmt_offset<COL32>(row, col, ldc)] = rint_i8((float)v);
        } else if constexpr (EPI == EPI_I8_COL32_ROWSCALE) {
          reinterpret_cast<int8_t*>(Cout)[fmt_offset<COL32>(row, col, ldc)] = rint_i8(__fmul_rn((float)v, rs));
        } else {
          reinterpret_cast<fp16_t*>(Cout)[(long long)row * ldc + col] =
              mm_dequant_value(v, rs, colStats[col], bias ? (float)bias[col] : 0.0f);
        }
      }
    }
  }
}

static Knob<int> g_igemm_tile{0};   // 0 = auto, 128 = force the 128x128 register-staged kernel, 4 = force the 4-wave
                               // hgemm.hip kernel for row-major operands, 8 = force the 8-wave igemm_256 (tests / A-B)

template <int AF, int BF, int EPI>
static int launch_igemm(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, const float* row_scale, long long lda,
                        long long ldb, long long ldc, const float* rowStats = nullptr, const float* colStats = nullptr,
                        const fp16_t* bias = nullptr, int32_t* ws = nullptr, long long ws_bytes = 0) {
  if (m <= 0 || n <= 0 || k <= 0) return 0;
  // Row-major operands with the fused dequant on the 4-wave kernel (hgemm.hip HG_I8_DEQ, one wave per SIMD, 128 x 128
  // per wave, the three-barrier schedule) wherever its grid is one mostly full round (>= 192 tiles of 256 x 256):
  // bit-identical to igemm_256's 8 waves and faster since round 4 -- 127.3-129.3 vs 138.4-141.3 us at
  // 4096 x 4096 x 11008, 54.4-55.2 vs 58.8-59.6 us at 4096^3 (tools/hgemm_variant_ab.py,
  // profiles/lab/r04_hgemm_variants.txt).  Round 3 measured it slower (163 vs 142 us): its epilogue loaded the column
  // statistics and bias once per accumulator (256 dependent loads per lane, ~34 us of fixed cost per launch); they
  // are loaded once per lane now.  Smaller grids keep igemm_256's exact split-K; the int32 form stays there too.
  if constexpr (AF == ROW && BF == ROW && (EPI == EPI_F16_ROW_DEQUANT || EPI == EPI_I32_ROW)) {
    if (g_igemm_tile == 4 || (g_igemm_tile == 0 && EPI == EPI_F16_ROW_DEQUANT && hgemm_tiles(m, n) >= 192)) {
      const int rc = igemm_4wave(m, n, k, A, lda, B, ldb, C, ldc, EPI == EPI_F16_ROW_DEQUANT, rowStats, colStats, bias);
      if (rc != 1) return rc == 0 ? 0 : 1;
    }
  }
  // large problems: 256x256 LDS-DMA kernel (igemm_256.hip; split-K over ws for small tile grids); small /
  // col_turing / ragged-k: 128x128 here
  if (g_igemm_tile != 128 &&
      launch_igemm_256<AF, BF, EPI>(m, n, k, A, B, C, row_scale, lda, ldb, ldc, rowStats, colStats, bias, ws,
                                    ws_bytes)) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) { set_error((int)e, "igemmlt launch"); return 1; }
    return 0;
  }
  const int tiles = ((m + Q_BM - 1) / Q_BM) * ((n + Q_BN - 1) / Q_BN);
  hipLaunchKernelGGL((k_igemm<AF, BF, EPI>), dim3(tiles), dim3(Q_THREADS), 0, current_stream(), m, n, k, A, B, C,
                     row_scale, lda, ldb, ldc, rowStats, colStats, bias);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_error((int)e, "igemmlt launch"); return 1; }
  return 0;
}

// ============================================================================ extract outliers
// out is row-major [rows, idx_size]: out[r * idx_size + j] = B_fmt[r, idx[j]]  (kernel_quant.cpp:3992-4052)
template <int F>
__global__ void k_extract_outliers(const int8_t* __restrict__ A, const int* __restrict__ idx, int8_t* __restrict__ out,
                                   int idx_size, int rows, int cols) {
  const int c_out = blockIdx.x;
  if (c_out >= idx_size) return;
  const long long ld = (F == TURING) ? 32 * pad_to(rows, 8) : 32 * pad_to(rows, 32);
  const int col = idx[c_out];
  for (int r = threadIdx.x; r < rows; r += blockDim.x) out[(long long)r * idx_size + c_out] = A[fmt_offset<F>(r, col, ld)];
}

}  // namespace bnb

using namespace bnb;

extern "C" {

void cget_col_row_stats(fp16_t* A, float* rowStats, float* colStats, int* nnz_count_row, float nnz_threshold, int rows,
                        int cols) {
  if (rows <= 0 || cols <= 0) return;
  const int col_tiles = (cols + 255) / 256, row_tiles = (rows + 15) / 16;
  const bool vec = (((uintptr_t)A & 15) == 0) && (cols % 8 == 0);
  if (vec && !(nnz_threshold > 0.0f && nnz_count_row != nullptr)) {
    const int wct = (cols + W_COLS - 1) / W_COLS, wrt = (rows + W_ROWS - 1) / W_ROWS;
    hipLaunchKernelGGL(k_colrow_stats_wide, dim3(wrt * wct), dim3(256), 0, current_stream(), A, rowStats, colStats,
                       rows, cols, wct);
  } else if (nnz_threshold > 0.0f && nnz_count_row != nullptr)
    hipLaunchKernelGGL(k_colrow_stats<true>, dim3(row_tiles * col_tiles), dim3(256), 0, current_stream(), A, rowStats,
                       colStats, nnz_count_row, nnz_threshold, rows, cols, col_tiles, vec);
  else
    hipLaunchKernelGGL(k_colrow_stats<false>, dim3(row_tiles * col_tiles), dim3(256), 0, current_stream(), A, rowStats,
                       colStats, nnz_count_row, nnz_threshold, rows, cols, col_tiles, vec);
  BNB_LAUNCH_CHECK("get_col_row_stats");
}

// [additive] CA and row statistics in one pass (the row halves of cget_col_row_stats + cdouble_rowcol_quant,
// threshold 0).  Returns 0 when launched, 1 when the shape needs the two-kernel path.
int cint8_row_quant_fp16(fp16_t* A, float* rowStats, char* out_row, int rows, int cols) {
  BNB_RANGE("cint8_row_quant_fp16");
  if (rows <= 0 || cols <= 0) return 0;
  if (cols % 8 || cols > 64 * 8 * RQ_MAX_VEC || ((uintptr_t)A & 15) || ((uintptr_t)out_row & 7)) return 1;
  const int per_lane = (cols / 8 + 63) / 64;
  auto go = [&](auto kern, auto kern_wt) {
    hipLaunchKernelGGL(g_rq_wt ? kern_wt : kern, dim3((rows + 3) / 4), dim3(256), 0, current_stream(), A, rowStats,
                       (int8_t*)out_row, rows, cols);
  };
  if (per_lane <= 4) go(k_row_quant<4>, k_row_quant<4, true>);
  else if (per_lane <= 8) go(k_row_quant<8>, k_row_quant<8, true>);
  else if (per_lane <= 12) go(k_row_quant<12>, k_row_quant<12, true>);
  else if (per_lane <= 16) go(k_row_quant<16>, k_row_quant<16, true>);
  else if (per_lane <= 22) go(k_row_quant<22>, k_row_quant<22, true>);   // K = 11008: 22 vectors, 4 waves per SIMD
  else if (per_lane <= 24) go(k_row_quant<24>, k_row_quant<24, true>);
  else go(k_row_quant<RQ_MAX_VEC>, k_row_quant<RQ_MAX_VEC, true>);
  BNB_LAUNCH_CHECK("int8_row_quant");
  return 0;
}

// [additive, testing] 1: cint8_row_quant_fp16 stores CA write-through (device scope), 0: write-back; returns the previous
int cint8_set_row_quant_store(int wt) {
  const int prev = bnb::g_rq_wt;
  bnb::g_rq_wt = wt ? 1 : 0;
  return prev;
}

void cdouble_rowcol_quant(fp16_t* A, float* rowStats, float* colStats, char* out_col_normed, char* out_row_normed,
                          int* rowidx, int* colidx, fp16_t* val, int* nnz_row_ptr, float threshold, int rows, int cols) {
  BNB_RANGE("cdouble_rowcol_quant");
  if (rows <= 0 || cols <= 0) return;
  const int col_tiles = (cols + 255) / 256, row_tiles = (rows + 15) / 16;
  const bool vec = (((uintptr_t)A & 15) == 0) && (cols % 8 == 0) && (((uintptr_t)out_col_normed & 7) == 0) &&
                   (((uintptr_t)out_row_normed & 7) == 0);
  if (vec && !(threshold > 0.0f && rowidx && colidx && val && nnz_row_ptr)) {
    const int wct = (cols + W_COLS - 1) / W_COLS, wrt = (rows + W_ROWS - 1) / W_ROWS;
    hipLaunchKernelGGL(k_double_rowcol_quant_wide, dim3(wrt * wct), dim3(256), 0, current_stream(), A, rowStats,
                       colStats, (int8_t*)out_col_normed, (int8_t*)out_row_normed, rows, cols, wct);
  } else if (threshold > 0.0f && rowidx && colidx && val && nnz_row_ptr)
    hipLaunchKernelGGL(k_double_rowcol_quant<true>, dim3(row_tiles * col_tiles), dim3(256), 0, current_stream(), A,
                       rowStats, colStats, (int8_t*)out_col_normed, (int8_t*)out_row_normed, rowidx, colidx, val,
                       nnz_row_ptr, threshold, rows, cols, col_tiles, vec);
  else
    hipLaunchKernelGGL(k_double_rowcol_quant<false>, dim3(row_tiles * col_tiles), dim3(256), 0, current_stream(), A,
                       rowStats, colStats, (int8_t*)out_col_normed, (int8_t*)out_row_normed, rowidx, colidx, val,
                       nnz_row_ptr, threshold, rows, cols, col_tiles, vec);
  BNB_LAUNCH_CHECK("double_rowcol_quant");
}

void ctransform_row2col32(char* A, char* out, int rows, int cols) { launch_transform<COL32, false, false>((int8_t*)A, (int8_t*)out, rows, cols); }
void ctransform_row2col32T(char* A, char* out, int rows, int cols) { launch_transform<COL32, true, false>((int8_t*)A, (int8_t*)out, rows, cols); }
void ctransform_row2turing(char* A, char* out, int rows, int cols) { launch_transform<TURING, false, false>((int8_t*)A, (int8_t*)out, rows, cols); }
void ctransform_row2turingT(char* A, char* out, int rows, int cols) { launch_transform<TURING, true, false>((int8_t*)A, (int8_t*)out, rows, cols); }
void ctransform_row2ampere(char* A, char* out, int rows, int cols) { launch_transform<AMPERE, false, false>((int8_t*)A, (int8_t*)out, rows, cols); }
void ctransform_row2ampereT(char* A, char* out, int rows, int cols) { launch_transform<AMPERE, true, false>((int8_t*)A, (int8_t*)out, rows, cols); }
// inverse transforms (out is the row-major rows x cols matrix)
void ctransform_col322row(char* A, char* out, int rows, int cols) { launch_transform<COL32, false, true>((int8_t*)A, (int8_t*)out, rows, cols); }
void ctransform_turing2row(char* A, char* out, int rows, int cols) { launch_transform<TURING, false, true>((int8_t*)A, (int8_t*)out, rows, cols); }
void ctransform_ampere2row(char* A, char* out, int rows, int cols) { launch_transform<AMPERE, false, true>((int8_t*)A, (int8_t*)out, rows, cols); }

int cigemmlt_turing_32(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, float* row_scale, int lda, int ldb, int ldc) {
  BNB_RANGE("cigemmlt_turing_32");
  return launch_igemm<COL32, TURING, EPI_I32_COL32>(m, n, k, A, B, C, row_scale, lda, ldb, ldc);
}
int cigemmlt_turing_8(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, float* row_scale, int lda, int ldb, int ldc) {
  BNB_RANGE("cigemmlt_turing_8");
  return launch_igemm<COL32, TURING, EPI_I8_COL32>(m, n, k, A, B, C, row_scale, lda, ldb, ldc);
}
int cigemmlt_turing_8_rowscale(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, float* row_scale, int lda, int ldb, int ldc) {
  BNB_RANGE("cigemmlt_turing_8_rowscale");
  return launch_igemm<COL32, TURING, EPI_I8_COL32_ROWSCALE>(m, n, k, A, B, C, row_scale, lda, ldb, ldc);
}
int cigemmlt_ampere_32(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, float* row_scale, int lda, int ldb, int ldc) {
  BNB_RANGE("cigemmlt_ampere_32");
  return launch_igemm<COL32, AMPERE, EPI_I32_COL32>(m, n, k, A, B, C, row_scale, lda, ldb, ldc);
}
int cigemmlt_ampere_8(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, float* row_scale, int lda, int ldb, int ldc) {
  BNB_RANGE("cigemmlt_ampere_8");
  return launch_igemm<COL32, AMPERE, EPI_I8_COL32>(m, n, k, A, B, C, row_scale, lda, ldb, ldc);
}
int cigemmlt_ampere_8_rowscale(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, float* row_scale, int lda, int ldb, int ldc) {
  BNB_RANGE("cigemmlt_ampere_8_rowscale");
  return launch_igemm<COL32, AMPERE, EPI_I8_COL32_ROWSCALE>(m, n, k, A, B, C, row_scale, lda, ldb, ldc);
}

// Additive fast path: row-major int8 A [m, k] (lda) and B [n, k] (ldb); epilogue = mm_dequant to fp16
// row-major out [m, n] (ldc), i.e. igemmlt + cdequant_mm_int32_fp16 fused into one launch.
int cigemmlt_row_dequant_fp16(int m, int n, int k, const int8_t* A, const int8_t* B, fp16_t* out, const float* rowStats,
                              const float* colStats, const fp16_t* bias, int lda, int ldb, int ldc) {
  BNB_RANGE("cigemmlt_row_dequant_fp16");
  return launch_igemm<ROW, ROW, EPI_F16_ROW_DEQUANT>(m, n, k, A, B, out, nullptr, lda, ldb, ldc, rowStats, colStats, bias);
}
// Additive: row-major int8 GEMM with int32 row-major output (exact igemm, test_matmulqlt.py:194-204).
int cigemm_row_i32(int m, int n, int k, const int8_t* A, const int8_t* B, int32_t* out, int lda, int ldb, int ldc) {
  BNB_RANGE("cigemm_row_i32");
  return launch_igemm<ROW, ROW, EPI_I32_ROW>(m, n, k, A, B, out, nullptr, lda, ldb, ldc);
}
// Additive: the two row-major entry points with a caller workspace (size: cigemmlt_workspace_bytes) that lets
// small tile grids -- the column shards of the multi-GPU step -- run split-K; the result is the same bits.
int cigemmlt_row_dequant_ws_fp16(int m, int n, int k, const int8_t* A, const int8_t* B, fp16_t* out,
                                 const float* rowStats, const float* colStats, const fp16_t* bias, int lda, int ldb,
                                 int ldc, int32_t* workspace, long long workspace_bytes) {
  BNB_RANGE("cigemmlt_row_dequant_ws_fp16");
  return launch_igemm<ROW, ROW, EPI_F16_ROW_DEQUANT>(m, n, k, A, B, out, nullptr, lda, ldb, ldc, rowStats, colStats,
                                                     bias, workspace, workspace_bytes);
}
int cigemm_row_i32_ws(int m, int n, int k, const int8_t* A, const int8_t* B, int32_t* out, int lda, int ldb, int ldc,
                      int32_t* workspace, long long workspace_bytes) {
  BNB_RANGE("cigemm_row_i32_ws");
  return launch_igemm<ROW, ROW, EPI_I32_ROW>(m, n, k, A, B, out, nullptr, lda, ldb, ldc, nullptr, nullptr, nullptr,
                                             workspace, workspace_bytes);
}
long long cigemmlt_workspace_bytes(int m, int n, int k) { return igemm_workspace_bytes(m, n, k); }

void cdequant_mm_int32_fp16(int* A, float* rowStats, float* colStats, fp16_t* out, float* newRowStats,
                            float* newcolStats, fp16_t* bias, int numRows, int numCols) {
  BNB_RANGE("cdequant_mm_int32_fp16");
  (void)newRowStats; (void)newcolStats;   // unused by the reference kernel as well
  if (numRows <= 0 || numCols <= 0) return;
  if (numCols % 8 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)out & 15) == 0 && ((uintptr_t)colStats & 15) == 0 &&
      ((uintptr_t)bias & 15) == 0) {
    long long g = ((long long)numRows * (numCols / 8) + 255) / 256;
    if (g > 16384) g = 16384;
    hipLaunchKernelGGL(k_dequant_mm_col32_v8, dim3((unsigned)g), dim3(256), 0, current_stream(), (const int32_t*)A,
                       rowStats, colStats, out, bias, numRows, numCols);
    BNB_LAUNCH_CHECK("dequant_mm_int32_fp16");
    return;
  }
  const long long groups = (long long)numRows * ((numCols + 3) / 4);
  long long g = (groups + 255) / 256;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(k_dequant_mm_col32, dim3((unsigned)g), dim3(256), 0, current_stream(), A, rowStats, colStats, out, bias,
                     numRows, numCols);
  BNB_LAUNCH_CHECK("dequant_mm_int32_fp16");
}

void cextractOutliers_turing(char* A, int* idx, char* out, int idx_size, int rows, int cols) {
  if (idx_size <= 0) return;
  hipLaunchKernelGGL(k_extract_outliers<TURING>, dim3(idx_size), dim3(256), 0, current_stream(), (int8_t*)A, idx,
                     (int8_t*)out, idx_size, rows, cols);
  BNB_LAUNCH_CHECK("extract_outliers");
}
void cextractOutliers_ampere(char* A, int* idx, char* out, int idx_size, int rows, int cols) {
  if (idx_size <= 0) return;
  hipLaunchKernelGGL(k_extract_outliers<AMPERE>, dim3(idx_size), dim3(256), 0, current_stream(), (int8_t*)A, idx,
                     (int8_t*)out, idx_size, rows, cols);
  BNB_LAUNCH_CHECK("extract_outliers");
}

// [additive, testing] 0 = auto, 128 = force the 128x128 int8 GEMM kernel, 4 = the 4-wave kernel (row-major operands),
// 8 = the 8-wave igemm_256
void cigemm_set_tile(int tile) { g_igemm_tile = tile; }

}  // extern "C"
