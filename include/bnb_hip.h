/* C-ABI of libbitsandbytes_hip.so — the drop-in boundary for the quantized-matmul hot path.
 *
 * Every entry point below keeps the name, argument order, types and meaning of the reference's
 * exported symbol (abhilash1910/bitsandbytes-SYCL, ref:sycl/pythonInterface.cpp, cited per line),
 * so the reference's ctypes layer (ref:python_src_quants/functional.py) can bind it unchanged.
 * Device pointers are HIP device pointers on the current device; launches go to the stream set
 * by cset_stream (default: the null stream).  Launches are asynchronous.
 *
 * Types: fp16 = IEEE binary16 (passed as `unsigned short` bit patterns here, `sycl::half` in the
 * reference); bf16 = bfloat16 (`unsigned short` bits, `sycl::ext::oneapi::bfloat16` in the reference).
 * Symbols marked [additive] are not in the reference ABI and never change the meaning of one that is.
 */
#ifndef BNB_HIP_H
#define BNB_HIP_H

#include <stddef.h>
#include <stdint.h>
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef unsigned short bnb_fp16;
typedef unsigned short bnb_bf16;

/* ---- context / loader probes: ref:sycl/pythonInterface.cpp:295-296, 380-398 ---- */
void* get_context(void);                                   /* pythonInterface.cpp:295 */
void* get_cusparse(void);                                  /* pythonInterface.cpp:296 */
void* cget_managed_ptr(size_t bytes);                      /* pythonInterface.cpp:380 */
void cprefetch(void* ptr, size_t bytes, int device);       /* pythonInterface.cpp:389 */

/* ---- blockwise quantize: ref:sycl/pythonInterface.cpp:203-217 ----
 * absmax[b] = max|A| over block b (fp32); code = NULL for fp4/nf4, the 256-entry map for 8-bit.
 * out: ceil(n/2) bytes for fp4/nf4 (high nibble = even element), n bytes for 8-bit. */
void cquantize_blockwise_fp16(float* code, bnb_fp16* A, float* absmax, unsigned char* out, int blocksize, const int n);     /* :203 */
void cquantize_blockwise_fp16_fp4(float* code, bnb_fp16* A, float* absmax, unsigned char* out, int blocksize, const int n); /* :204 */
void cquantize_blockwise_fp16_nf4(float* code, bnb_fp16* A, float* absmax, unsigned char* out, int blocksize, const int n); /* :205 */
void cquantize_blockwise_fp32(float* code, float* A, float* absmax, unsigned char* out, int blocksize, const int n);        /* :207 */
void cquantize_blockwise_fp32_fp4(float* code, float* A, float* absmax, unsigned char* out, int blocksize, const int n);    /* :208 */
void cquantize_blockwise_fp32_nf4(float* code, float* A, float* absmax, unsigned char* out, int blocksize, const int n);    /* :209 */
void cquantize_blockwise_bf16(float* code, bnb_bf16* A, float* absmax, unsigned char* out, int blocksize, const int n);     /* :215 */
void cquantize_blockwise_bf16_fp4(float* code, bnb_bf16* A, float* absmax, unsigned char* out, int blocksize, const int n); /* :216 */
void cquantize_blockwise_bf16_nf4(float* code, bnb_bf16* A, float* absmax, unsigned char* out, int blocksize, const int n); /* :217 */

/* ---- blockwise dequantize: ref:sycl/pythonInterface.cpp:199-221 ---- out[i] = T(code[q_i] * absmax[i/bs]) */
void cdequantize_blockwise_fp16_fp4(float* code, unsigned char* A, float* absmax, bnb_fp16* out, int blocksize, const int n); /* :199 */
void cdequantize_blockwise_fp16(float* code, unsigned char* A, float* absmax, bnb_fp16* out, int blocksize, const int n);     /* :200 */
void cdequantize_blockwise_fp16_nf4(float* code, unsigned char* A, float* absmax, bnb_fp16* out, int blocksize, const int n); /* :201 */
void cdequantize_blockwise_fp32(float* code, unsigned char* A, float* absmax, float* out, int blocksize, const int n);        /* :211 */
void cdequantize_blockwise_fp32_fp4(float* code, unsigned char* A, float* absmax, float* out, int blocksize, const int n);    /* :212 */
void cdequantize_blockwise_fp32_nf4(float* code, unsigned char* A, float* absmax, float* out, int blocksize, const int n);    /* :213 */
void cdequantize_blockwise_bf16(float* code, unsigned char* A, float* absmax, bnb_bf16* out, int blocksize, const int n);     /* :219 */
void cdequantize_blockwise_bf16_fp4(float* code, unsigned char* A, float* absmax, bnb_bf16* out, int blocksize, const int n); /* :220 */
void cdequantize_blockwise_bf16_nf4(float* code, unsigned char* A, float* absmax, bnb_bf16* out, int blocksize, const int n); /* :221 */

/* ---- host-pointer CPU-path entry points: ref:sycl/pythonInterface.cpp:419-420 (cpu_ops.cpp semantics:
 * division A/absmax, nearest code with ties to the left, code[0] := -1 in place).  Run on the host cores
 * (csrc/cpu_ops.cpp; no HIP call, so they work without a GPU), synchronous on return. */
void cquantize_blockwise_cpu_fp32(float* code, float* A, float* absmax, unsigned char* out, long long blocksize, long long n);   /* :419 */
void cdequantize_blockwise_cpu_fp32(float* code, unsigned char* A, float* absmax, float* out, long long blocksize, long long n); /* :420 */
/* [additive] worker threads of the two host entry points (0 = default: BNB_CPU_THREADS, else OMP_NUM_THREADS,
 * else the hardware threads, at most 64); returns the count in effect */
int cset_cpu_threads(int threads);
/* [additive] device-pointer forms of the CPU-path quantize / dequantize, executed on the GPU (one byte per
 * element, any blocksize; the quantize does not rewrite the caller's code table) */
void cquantize_blockwise_bytes_fp32(float* code, float* A, float* absmax, unsigned char* out, long long blocksize, long long n);
void cdequantize_blockwise_bytes_fp32(float* code, unsigned char* A, float* absmax, float* out, long long blocksize, long long n);

/* ---- 4-bit GEMV (M == 1): ref:sycl/pythonInterface.cpp:408-415 ----
 * out[r] = sum_k A[k] * datatype[q(r,k)] * absmax[(2*ldb*r + k)/blocksize]; m = out_features, k = in_features */
void cgemm_4bit_inference_naive_fp16(int m, int n, int k, bnb_fp16* A, unsigned char* B, float* absmax, float* datatype,
                                     bnb_fp16* out, int lda, int ldb, int ldc, int blocksize);   /* :408 */
void cgemm_4bit_inference_naive_bf16(int m, int n, int k, bnb_bf16* A, unsigned char* B, float* absmax, float* datatype,
                                     bnb_bf16* out, int lda, int ldb, int ldc, int blocksize);   /* :411 */
void cgemm_4bit_inference_naive_fp32(int m, int n, int k, float* A, unsigned char* B, float* absmax, float* datatype,
                                     float* out, int lda, int ldb, int ldc, int blocksize);      /* :414 */
/* Additive: the same GEMV with compressed statistics (compress_statistics=True) decoded in-kernel,
 * absmax[j] = code2[absmax_q[j]] * absmax2[j / blocksize2] + *offset (fp32), replacing the
 * dequantize_blockwise launch of ref:python_src_quants/functional.py:1982-1984.  `offset` is a device
 * pointer to one float.  Returns 0 when launched, 1 when the shape needs the two-step path, 2 when the
 * launch failed (the error is also recorded for cget_last_error). */
int cgemm_4bit_inference_naive_nested_fp16(int m, int n, int k, bnb_fp16* A, unsigned char* B, unsigned char* absmax_q,
                                           float* code2, float* absmax2, float* offset, float* datatype, bnb_fp16* out,
                                           int lda, int ldb, int ldc, int blocksize, int blocksize2);
int cgemm_4bit_inference_naive_nested_bf16(int m, int n, int k, bnb_bf16* A, unsigned char* B, unsigned char* absmax_q,
                                           float* code2, float* absmax2, float* offset, float* datatype, bnb_bf16* out,
                                           int lda, int ldb, int ldc, int blocksize, int blocksize2);

/* [additive, testing] few-token (1..64 activation rows; the whole-K kernel 1..32) GEMM kernel choice: 0 = auto (the whole-K kernel,
 * gemm4bit_wk.hip, no workspace, at <= 6 rows on weights of < 2 row tiles per CU; else the split-K kernel),
 * 1 = the split-K kernel (gemm4bit_skinny.hip + its ordered reduce) only, 2 = the whole-K kernel wherever it fits */
void cgemm_4bit_set_fewtoken_kernel(int which);

/* [additive, testing] the whole-K few-token kernel (gemm4bit_fewtok.hip; 1..32 activation rows, LDS-DMA weight ring,
 * 16x16x32 MFMA, tried before the kernels above): 0 = auto (where its shape rule takes it), 1 = off, 2 = wherever it fits */
void cgemm_4bit_set_fewtok_mode(int mode);
/* [additive] 1 when the 4-bit GEMM entry points (cgemm_4bit_inference*, the few-token ws / nested entries) run that
 * kernel for m out features, n activation rows, k in features and this blocksize, else 0 */
int cgemm_4bit_fewtok_takes(int m, int n, int k, int blocksize);

/* [additive, testing] GEMV kernel choice: 0 = auto (the balanced-range kernel where the shape fits, else the
 * 4-waves-x-R-rows kernel), 1 = the 4-waves-x-R-rows kernel only; both give identical bits */
void cgemv_4bit_set_kernel(int which);
/* [additive, testing] the balanced GEMV's nested statistics decoded per chunk where it is consumed (1; round 5, measured
 * 0.2-1.9 % slower) or all before the first dot (0, default); bit-identical; returns the previous setting */
int cgemv_4bit_set_lazy_nested(int on);
/* [additive, testing] 1 = the wide GEMV (narrow / long-K weights) one row per workgroup; 0 = rows per workgroup
   by the launch rule (up to 4, sharing one activation load and table fill) */
void cgemv_4bit_set_wide_rows(int mode);

/* ---- 4-bit GEMM (any number of activation rows): ref:sycl/pythonInterface.cpp:377-378 (slot of the
 * broken kgemm_4bit_inference, re-implemented as a fused NF4 GEMM) ----
 * m = out_features, n = activation rows, k = in_features (k % 64 == 0):
 * out[t*ldc + r] = sum_k A[t*lda + k] * W[r, k],  W[r, k] = T(code[q(r,k)] * absmax[(2*ldb*r + k)/blocksize]) */
void cgemm_4bit_inference(int m, int n, int k, bnb_fp16* A, unsigned char* B, float* absmax, bnb_fp16* out, int lda,
                          int ldb, int ldc, int blocksize);                                      /* :377, NF4 table */
/* [additive] bf16 sibling (NF4) and table-driven variants (any 16-entry code, e.g. FP4) */
void cgemm_4bit_inference_bf16(int m, int n, int k, bnb_bf16* A, unsigned char* B, float* absmax, bnb_bf16* out, int lda,
                               int ldb, int ldc, int blocksize);
void cgemm_4bit_inference_code_fp16(int m, int n, int k, bnb_fp16* A, unsigned char* B, float* absmax, float* datatype,
                                    bnb_fp16* out, int lda, int ldb, int ldc, int blocksize);
void cgemm_4bit_inference_code_bf16(int m, int n, int k, bnb_bf16* A, unsigned char* B, float* absmax, float* datatype,
                                    bnb_bf16* out, int lda, int ldb, int ldc, int blocksize);
/* [additive] the same with a caller-owned fp32 workspace that lets small tile grids (narrow column
 * shards, few tokens) run split-K; size it with cgemm_4bit_workspace_bytes (0 = split-K not used for this
 * shape).  A NULL or smaller workspace falls back to the unsplit kernels. */
void cgemm_4bit_inference_code_ws_fp16(int m, int n, int k, bnb_fp16* A, unsigned char* B, float* absmax,
                                       float* datatype, bnb_fp16* out, int lda, int ldb, int ldc, int blocksize,
                                       float* workspace, long long workspace_bytes);
void cgemm_4bit_inference_code_ws_bf16(int m, int n, int k, bnb_bf16* A, unsigned char* B, float* absmax,
                                       float* datatype, bnb_bf16* out, int lda, int ldb, int ldc, int blocksize,
                                       float* workspace, long long workspace_bytes);
long long cgemm_4bit_workspace_bytes(int m, int n, int k);
/* [additive] few tokens (n <= 64, k % 128 == 0): the weight-streaming kernel with compressed statistics
 * (absmax_q uint8 codes, code2 256-entry map, absmax2 per blocksize2 codes, offset: one fp32 on the
 * device) decoded in-kernel -- replaces the absmax decode launch + GEMM of the M > 1 path
 * (ref:functional.py:1346-1350 + autograd/_functions.py:507).  The plain-absmax calls above use the
 * same kernel for n <= 64 when the workspace fits.  Returns 0 when launched, 1 when the shape,
 * alignment or workspace does not fit (the caller then decodes absmax and uses the _ws entry points). */
int cgemm_4bit_inference_nested_ws_fp16(int m, int n, int k, bnb_fp16* A, unsigned char* B, unsigned char* absmax_q,
                                        float* code2, float* absmax2, float* offset, float* datatype, bnb_fp16* out,
                                        int lda, int ldb, int ldc, int blocksize, int blocksize2, float* workspace,
                                        long long workspace_bytes);
/* [additive] 4-bit weight x 2..4 activation rows in one launch (gemv4bit_tok.hip; replaces the M > 1 pair
 * dequantize_4bit + F.linear, ref:autograd/_functions.py:491-507, for batched decode): out[t * ldc + r], t < ntok.
 * Statistics plain (absmax fp32, absmax_q = NULL) or compressed (absmax = NULL; absmax_q, code2, absmax2, offset,
 * blocksize2) decoded in the kernel.  Each row t is bit-identical to cgemm_4bit_inference_naive_* on row t.
 * Returns 0 when launched, 1 when the shape / alignment does not fit (nothing launched), 2 when the launch failed. */
int cgemm_4bit_inference_tokens_bf16(int m, int ntok, int k, bnb_bf16* A, int lda, unsigned char* B, int ldb,
                                     float* absmax, unsigned char* absmax_q, float* code2, float* absmax2,
                                     float* offset, float* datatype, bnb_bf16* out, int ldc, int blocksize,
                                     int blocksize2);
int cgemm_4bit_inference_tokens_fp16(int m, int ntok, int k, bnb_fp16* A, int lda, unsigned char* B, int ldb,
                                     float* absmax, unsigned char* absmax_q, float* code2, float* absmax2,
                                     float* offset, float* datatype, bnb_fp16* out, int ldc, int blocksize,
                                     int blocksize2);
int cgemm_4bit_inference_nested_ws_bf16(int m, int n, int k, bnb_bf16* A, unsigned char* B, unsigned char* absmax_q,
                                        float* code2, float* absmax2, float* offset, float* datatype, bnb_bf16* out,
                                        int lda, int ldb, int ldc, int blocksize, int blocksize2, float* workspace,
                                        long long workspace_bytes);
/* [additive, testing] force the GEMM tile kernel: 0 = auto, 128 = 128x128, 256 = 256x256 */
void cgemm_4bit_set_tile(int tile);

/* ---- LLM.int8 statistics and quantisation: ref:sycl/pythonInterface.cpp:333-339 ---- */
void cget_col_row_stats(bnb_fp16* A, float* rowStats, float* colStats, int* nnz_count_row, float nnz_threshold, int rows,
                        int cols);                                                               /* :335 */
/* [additive] CA and row statistics of cdouble_rowcol_quant (threshold 0) in one pass over A, for the
 * inference forward (no CAt needed).  Returns 0 when launched, 1 when the shape needs the two-kernel path
 * (cols % 8, cols > 16384, unaligned pointers). */
int cint8_row_quant_fp16(bnb_fp16* A, float* rowStats, char* out_row, int rows, int cols);
/* [additive, testing] 1: cint8_row_quant_fp16 stores CA write-through (device scope), 0: write-back; returns the
 * previous setting */
int cint8_set_row_quant_store(int wt);
void cdouble_rowcol_quant(bnb_fp16* A, float* rowStats, float* colStats, char* out_col_normed, char* out_row_normed,
                          int* rowidx, int* colidx, bnb_fp16* val, int* nnz_row_ptr, float threshold, int rows,
                          int cols);                                                             /* :338 */

/* ---- tile layouts: ref:sycl/pythonInterface.cpp:341-357 (row-major int8 -> format of A, or of A^T for *T) ---- */
void ctransform_row2col32(char* A, char* out, int rows, int cols);     /* :341 */
void ctransform_row2col32T(char* A, char* out, int rows, int cols);    /* :344 */
void ctransform_row2turing(char* A, char* out, int rows, int cols);    /* :347 */
void ctransform_row2turingT(char* A, char* out, int rows, int cols);   /* :350 */
void ctransform_row2ampere(char* A, char* out, int rows, int cols);    /* :353 */
void ctransform_row2ampereT(char* A, char* out, int rows, int cols);   /* :356 */
/* [additive] inverse transforms; functional.py:2645-2647 calls the first two (never exported by the reference, Q18) */
void ctransform_turing2row(char* A, char* out, int rows, int cols);
void ctransform_ampere2row(char* A, char* out, int rows, int cols);
void ctransform_col322row(char* A, char* out, int rows, int cols);

/* ---- int8 GEMM C = A @ B^T (A col32 m x k, B col_turing/col_ampere n x k, C col32): ref:sycl/pythonInterface.cpp:298-316.
 * Returns 0 on success, 1 on error (Python maps 1 -> NotImplementedError, functional.py:2341-2348). No context argument. */
int cigemmlt_turing_32(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, float* row_scale, int lda, int ldb, int ldc);          /* :298 */
int cigemmlt_turing_8(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, float* row_scale, int lda, int ldb, int ldc);           /* :303 */
int cigemmlt_turing_8_rowscale(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, float* row_scale, int lda, int ldb, int ldc);  /* :306 */
int cigemmlt_ampere_32(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, float* row_scale, int lda, int ldb, int ldc);          /* :309 */
int cigemmlt_ampere_8_rowscale(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, float* row_scale, int lda, int ldb, int ldc);  /* :312 */
int cigemmlt_ampere_8(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, float* row_scale, int lda, int ldb, int ldc);           /* :315 */
/* [additive] row-major operands: fused igemmlt + dequant_mm_int32_fp16 (fp16 [m, n] out), and exact int32 */
int cigemmlt_row_dequant_fp16(int m, int n, int k, const int8_t* A, const int8_t* B, bnb_fp16* out, const float* rowStats,
                              const float* colStats, const bnb_fp16* bias, int lda, int ldb, int ldc);
int cigemm_row_i32(int m, int n, int k, const int8_t* A, const int8_t* B, int32_t* out, int lda, int ldb, int ldc);
/* [additive] the two row-major int8 entry points with a caller-owned workspace (bytes: cigemmlt_workspace_bytes;
 * 0 = no split for this shape) that lets small tile grids (the column shards of the multi-GPU step) run split-K:
 * int32 partials summed exactly by a second launch that applies the epilogue -- the same bits as without it.  A NULL
 * or smaller workspace runs unsplit. */
int cigemmlt_row_dequant_ws_fp16(int m, int n, int k, const int8_t* A, const int8_t* B, bnb_fp16* out,
                                 const float* rowStats, const float* colStats, const bnb_fp16* bias, int lda, int ldb,
                                 int ldc, int32_t* workspace, long long workspace_bytes);
int cigemm_row_i32_ws(int m, int n, int k, const int8_t* A, const int8_t* B, int32_t* out, int lda, int ldb,
                      int ldc, int32_t* workspace, long long workspace_bytes);
long long cigemmlt_workspace_bytes(int m, int n, int k);
/* [additive] the library GEMM of the large-prefill 4-bit path (gemm_lib.hip): C[m, n] = A[m, k] . W[n, k]^T, row-major,
 * bf16 / fp16 in and out, fp32 accumulation, on rocBLAS with a per-shape solution search (first call of a shape, per
 * quarter-octave bucket of m; kept only when > 5 % faster than the standard algorithm; none during graph capture).
 * Replaces the F.linear of ref:autograd/_functions.py:507 after the dequantise.  Returns 0 / 1 (error recorded). */
int cgemm_tn_bf16(int m, int n, int k, const bnb_bf16* A, int lda, const bnb_bf16* W, int ldw, bnb_bf16* C, int ldc);
int cgemm_tn_fp16(int m, int n, int k, const bnb_fp16* A, int lda, const bnb_fp16* W, int ldw, bnb_fp16* C, int ldc);
/* [additive] search switch (0 = standard algorithm only), per-shape budget (ms, > 0 to set), clear != 0 forgets the
 * cached plans; returns the number of cached plans.  cgemm_tn_plan: the cached plan of a shape (dtype 0 = bf16,
 * 1 = fp16): 1 = a searched rocBLAS solution, 0 = the standard algorithm, -1 = not searched yet. */
int cgemm_tn_set_search(int on, double budget_ms, int clear);
int cgemm_tn_plan(int m, int n, int k, int dtype, int lda, int ldw, int ldc);
/* [additive] the same product on the hand-written gfx950 GEMM (hgemm.hip: 256 x 256 tile, 4 waves x 128 x 128 on
 * v_mfma_f32_16x16x32, both operands by LDS-DMA): the large-prefill route of the 4-bit path after the dequantise
 * (ref:autograd/_functions.py:507's F.linear).  Returns 0 = launched, 1 = shape not supported (k % 64 != 0, rows not
 * 16-B aligned; nothing launched), 2 = launch error (cget_last_error*). */
int chgemm_tn_bf16(int m, int n, int k, const bnb_bf16* A, int lda, const bnb_bf16* W, int ldw, bnb_bf16* C, int ldc);
int chgemm_tn_fp16(int m, int n, int k, const bnb_fp16* A, int lda, const bnb_fp16* W, int ldw, bnb_fp16* C, int ldc);
/* [additive] the same with a caller workspace: split-K (fp32 partials, summed in split order by one more launch) on
 * tile grids below 192 tiles of 256 x 256; chgemm_tn_workspace_bytes(m, n, k) gives the bytes the shape needs (0 = no
 * split); a smaller workspace runs the unsplit kernel.  Same return codes. */
int chgemm_tn_ws_bf16(int m, int n, int k, const bnb_bf16* A, int lda, const bnb_bf16* W, int ldw, bnb_bf16* C, int ldc,
                      float* ws, long long ws_bytes);
int chgemm_tn_ws_fp16(int m, int n, int k, const bnb_fp16* A, int lda, const bnb_fp16* W, int ldw, bnb_fp16* C, int ldc,
                      float* ws, long long ws_bytes);
long long chgemm_tn_workspace_bytes(int m, int n, int k);
/* [additive] chgemm_tn_ws_* that also dequantises the NEXT 4-bit weight inside the same launch, software-pipelined one
 * weight ahead (replaces the following call's cdequantize_blockwise_{bf16,fp16}_{nf4,fp4} / nested dequantise, i.e. the
 * dequantize_4bit of ref:python_src_quants/functional.py:1329 before that layer's F.linear, autograd/_functions.py:507):
 * next_n elements (% 32 == 0, < 2^31) of packed 4-bit next_packed (16-B aligned; fp4 = 1 FP4 code, 0 NF4) with fp32
 * statistics next_absmax (next_q8 == NULL) or nested ones (next_q8, next_code2[256], next_absmax2, next_offset[1],
 * blocksize2) into next_out (16-B aligned, the GEMM's element type); same bits as the dequantise kernel.  Returns 0 =
 * launched, 1 = not supported (nothing launched), 2 = launch error. */
int chgemm_tn_pf_bf16(int m, int n, int k, const bnb_bf16* A, int lda, const bnb_bf16* W, int ldw, bnb_bf16* C, int ldc,
                      float* ws, long long ws_bytes, const unsigned char* next_packed, const float* next_absmax,
                      const unsigned char* next_q8, const float* next_code2, const float* next_absmax2,
                      const float* next_offset, int fp4, int blocksize, int blocksize2, long long next_n,
                      bnb_bf16* next_out);
int chgemm_tn_pf_fp16(int m, int n, int k, const bnb_fp16* A, int lda, const bnb_fp16* W, int ldw, bnb_fp16* C, int ldc,
                      float* ws, long long ws_bytes, const unsigned char* next_packed, const float* next_absmax,
                      const unsigned char* next_q8, const float* next_code2, const float* next_absmax2,
                      const float* next_offset, int fp4, int blocksize, int blocksize2, long long next_n,
                      bnb_fp16* next_out);
/* [additive, testing] the 33..64-token 4-bit GEMM kernel (gemm4bit_t64.hip): 0 = auto (33..64 activation rows,
 * blocksize 64, K % 256 == 0), 1 = off, 2 = wherever it applies (1..64 rows); returns the previous setting */
int cgemm_4bit_set_t64_mode(int mode);
/* [additive, testing] that kernel's split-K count: ks > 0 forces it (within the GEMM tolerance of the rule's split;
 * the combine forms stay bit-identical to each other), 0 = the rule; returns the previous setting */
int cgemm_4bit_set_t64_splits(int ks);
/* [additive, testing] geometry of the split-K few-token kernel (gemm4bit_skinny.hip): -1 (default) = the rule, 0 = 4
 * waves, 1 = 8 waves with the same blocks per split, 2 = 8 waves with twice the blocks per split; results within the
 * GEMM tolerance */
void cgemm_4bit_set_skinny_config(int cfg);
/* [additive, testing] split-K combine of that kernel: 1 = by the last workgroup of each row tile to finish (device-scope
 * partials, vmcnt(0) + barrier, then a ticket; splits summed in order), 0 (default) = a separate reduce launch (faster:
 * DESIGN.md §4); returns the previous setting */
int cgemm_4bit_set_t64_combine(int on);
/* [additive, testing] that kernel's split-K partial stores: 0 = write-back, 1 = write-through dwords, 2 (default) =
 * write-through 16-B lines staged through LDS; returns the previous setting */
int cgemm_4bit_set_t64_pstore(int p);
/* [additive, testing] that kernel's waves per 48-row set: 1 = 4 waves (one per SIMD), 2 = 8 waves (two per SIMD, the
 * set's blocks alternated between them, partial sums added in LDS), 0 (default) = auto, 8 waves up to 48 activation
 * rows or where K is not split; returns the previous setting */
int cgemm_4bit_set_t64_waves(int kp);
/* [additive, testing] that kernel's register-fed form (48 weight rows x whole K per workgroup, the 4 waves splitting K,
 * operands straight into registers, K-parts summed in LDS: no reduce launch): 1 (default) = off (measured slower), 2 =
 * wherever the 33..64-token kernel applies, 0 = auto (where its row tiles alone fill >= 3/4 of the CUs); returns the
 * previous setting */
int cgemm_4bit_set_t64_regfed(int v);
/* [additive, testing] launch shape of the 4-bit streaming dequantise: p = packed dwords per lane per pass (4, 8, 16),
 * grid_cap = at most that many workgroups (0 = none); returns the previous p */
int cdequantize_set_stream_cfg(int p, int grid_cap);
/* [additive, testing] store policy of that kernel's bf16/fp16 outputs: 0 = write-back, 1 = non-temporal,
 * 2 (default) = device-scope write-through; returns the previous setting */
int cdequantize_set_store_policy(int policy);
/* [additive, testing] the nested-statistics dequantise reads each wave's 64 statistic codes and second-level scale by
 * scalar loads (1, where blocksize 64 / blocksize2 >= 64 / 64-B aligned codes allow) or per lane (0, default: measured
 * faster); bit-identical; returns the previous setting */
int cdequantize_set_nested_scalar(int on);
/* [additive, testing] k_hgemm side dequantise (chgemm_tn_pf_*): bit 1 (default) = non-temporal side loads / stores,
 * 0 = plain; other bits are ignored (the lab build's ablations); returns the previous value */
int chgemm_set_side_mode(int v);
/* [additive, testing] 1 (default): k_hgemm stores C and its split-K partials write-through (device scope), 0:
 * write-back, 2: write-through + non-temporal hint (256 x 256 tile, interleaved epilogue; others as 1); returns the
 * previous setting */
int chgemm_set_c_store(int wt);
/* [additive, testing] the 128 x 128 tile of the 16-bit k_hgemm (round 5): mode 0 = never, 1 = by the launch plan's cost
 * (default), 2 = forced wherever allowed (no side dequantise); kt_x1000 > 0 sets the tile's k-tile time for the cost
 * model (256 x 256 k-tile units x 1000); returns the previous mode */
int chgemm_set_quarter_tile(int mode, int kt_x1000);
/* [additive, testing] k_hgemm's 16-bit epilogue: 1 (default) = interleaved per 16-row group (conversion overlapped with
 * the previous group's stores), 0 = the round-4 form; bit-identical outputs; returns the previous setting */
int chgemm_set_epilogue(int v);
/* [additive, testing] the launch plan of chgemm_tn_ws_* for (m, n, k): out = {WI, WJ, splits, k-tiles per split};
 * the output tile is 32 WI x 32 WJ (256 x 256, 256 x 128 or 128 x 256) */
void chgemm_tn_plan(int m, int n, int k, int* out);
/* [additive, measurement] measured ceilings for the bench's roofline (probe.hip): the dense MFMA rate on random operands
 * in registers (kind 0 = bf16 v_mfma_f32_16x16x32_bf16, 1 = int8 v_mfma_i32_16x16x64_i8; one wave per SIMD, 8 x iters
 * MFMAs per wave; sink >= blocks * 256 floats) and the HBM streaming read rate (bytes % 16 == 0; sink >= blocks
 * dwords).  Return 0 = launched, 1 = bad kind, 2 = launch error. */
int cprobe_mfma(int kind, int blocks, int iters, unsigned seed, float* sink);
int cprobe_hbm_read(const void* p, long long bytes, int blocks, unsigned* sink);
/* [additive, testing] int8 split-K factor: -1 = auto, 1 = never, >= 2 = force where it applies */
void cigemm_set_splitk(int ks);
/* [additive, testing] force the int8 GEMM tile kernel: 0 = auto (256x256 when it applies), 128 = 128x128, 4 = the
 * 4-wave 256x256 kernel of hgemm.hip for row-major operands (A/B only: slower than the default for int8) */
void cigemm_set_tile(int tile);

/* ---- int32 -> fp16 dequant: ref:sycl/pythonInterface.cpp:333 ----
 * out[r, c] = half(((float(C[r,c]) * 6.200012e-05f) * rowStats[r]) * colStats[c] + bias[c]), C in col32 */
void cdequant_mm_int32_fp16(int* A, float* rowStats, float* colStats, bnb_fp16* out, float* newRowStats, float* newcolStats,
                            bnb_fp16* bias, int numRows, int numCols);                           /* :333 */

/* ---- outlier column gather: ref:sycl/pythonInterface.cpp:368-369 ---- */
void cextractOutliers_turing(char* A, int* idx, char* out, int idx_size, int rows, int cols);   /* :368 */
void cextractOutliers_ampere(char* A, int* idx, char* out, int idx_size, int rows, int cols);   /* :369 */
/* COO sparse x dense: ref:sycl/pythonInterface.cpp:362-366 -> kspmm_coo_very_sparse_naive
 * (kernel_gemm.cpp:1398-1545).  out (fp16 [rowsA, colsB]) += A_coo @ B, fp16 accumulation per nonzero;
 * int8 B scaled by dequant_stats[col] / 127.  nnz, rowsA, rowsB kept for the reference's argument list. */
void cspmm_coo_very_sparse_naive_fp16(int* max_count, int* max_idx, int* offset_rowidx, int* rowidx, int* colidx,
        bnb_fp16* values, bnb_fp16* B, bnb_fp16* out, float* dequant_stats, int nnz_rows, int nnz, int rowsA,
        int rowsB, int colsB);
void cspmm_coo_very_sparse_naive_int8(int* max_count, int* max_idx, int* offset_rowidx, int* rowidx, int* colidx,
        bnb_fp16* values, signed char* B, bnb_fp16* out, float* dequant_stats, int nnz_rows, int nnz, int rowsA,
        int rowsB, int colsB);
/* [additive] C = A_coo @ B over a row-sorted COO with row pointers (row_ptr[A_rows + 1]), fp32 accumulation;
 * replaces cspmm_coo (pythonInterface.cpp:358-361, commented out in the reference, Q18), whose Python
 * wrapper (functional.py:2656) targets a cuSPARSE SpMM. */
void cspmm_coo_rows(int* row_ptr, int* A_colidx, bnb_fp16* A_vals, int A_rows, int B_cols, int ldb, bnb_fp16* B,
        int ldc, bnb_fp16* C, bool transposed_B);

/* ---- optimizers, SURVEY §8(f) row 4 (bnb_opt_T = float / bnb_fp16 / bnb_bf16 storage) ----
 * 8-bit blockwise states, 2048-element blocks, dynamic maps: ref:sycl/pythonInterface.cpp:264-284
 *   (kernels kernel_quant.cpp:2715-3208).  Adam uses state1+state2, the others state1 only.  */
void cadam_8bit_blockwise_grad_fp32(float* p, float* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
void cadam_8bit_blockwise_grad_fp16(bnb_fp16* p, bnb_fp16* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
void cadam_8bit_blockwise_grad_bf16(bnb_bf16* p, bnb_bf16* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
void cmomentum_8bit_blockwise_grad_fp32(float* p, float* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
void cmomentum_8bit_blockwise_grad_fp16(bnb_fp16* p, bnb_fp16* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
void cmomentum_8bit_blockwise_grad_bf16(bnb_bf16* p, bnb_bf16* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
void crmsprop_8bit_blockwise_grad_fp32(float* p, float* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
void crmsprop_8bit_blockwise_grad_fp16(bnb_fp16* p, bnb_fp16* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
void crmsprop_8bit_blockwise_grad_bf16(bnb_bf16* p, bnb_bf16* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
void cadagrad_8bit_blockwise_grad_fp32(float* p, float* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
void cadagrad_8bit_blockwise_grad_fp16(bnb_fp16* p, bnb_fp16* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
void cadagrad_8bit_blockwise_grad_bf16(bnb_bf16* p, bnb_bf16* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
void clion_8bit_blockwise_grad_fp32(float* p, float* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
void clion_8bit_blockwise_grad_fp16(bnb_fp16* p, bnb_fp16* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
void clion_8bit_blockwise_grad_bf16(bnb_bf16* p, bnb_bf16* g, unsigned char* state1, unsigned char* state2, float beta1, float beta2,
        float eps, int step, float lr, float* quantiles1, float* quantiles2, float* absmax1, float* absmax2,
        float weight_decay, const float gnorm_scale, bool skip_zeros, int n);
/* [additive] 4-bit dequantise with compressed statistics decoded in the kernel, absmax = code2[absmax_q[b]] *
 * absmax2[b / blocksize2] + *offset (fp32): one launch instead of dequantize_blockwise(absmax) + the 4-bit
 * dequantise (functional.py:1342-1350).  Returns 0 when launched, 1 when the shape needs the two-step path. */
int cdequantize_blockwise_nested_fp16_fp4(unsigned char* A, unsigned char* absmax_q, float* code2, float* absmax2,
        float* offset, bnb_fp16* out, int blocksize, int blocksize2, long long n);
int cdequantize_blockwise_nested_fp16_nf4(unsigned char* A, unsigned char* absmax_q, float* code2, float* absmax2,
        float* offset, bnb_fp16* out, int blocksize, int blocksize2, long long n);
int cdequantize_blockwise_nested_bf16_fp4(unsigned char* A, unsigned char* absmax_q, float* code2, float* absmax2,
        float* offset, bnb_bf16* out, int blocksize, int blocksize2, long long n);
int cdequantize_blockwise_nested_bf16_nf4(unsigned char* A, unsigned char* absmax_q, float* code2, float* absmax2,
        float* offset, bnb_bf16* out, int blocksize, int blocksize2, long long n);
/* fp32 states: ref:sycl/pythonInterface.cpp:223-241 (reference suffixes; bf16 siblings additive).
 * max_unorm > 0 is not supported (reported through cget_last_error). */
void cadam32bit_grad_fp32(float* g, float* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);
void cadam32bit_grad_fp16(bnb_fp16* g, bnb_fp16* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);
void cadam32bit_grad_bf16(bnb_bf16* g, bnb_bf16* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);
void cmomentum32bit_grad_32(float* g, float* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);
void cmomentum32bit_grad_16(bnb_fp16* g, bnb_fp16* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);
void cmomentum32bit_grad_bf16(bnb_bf16* g, bnb_bf16* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);
void crmsprop32bit_grad_32(float* g, float* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);
void crmsprop32bit_grad_16(bnb_fp16* g, bnb_fp16* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);
void crmsprop32bit_grad_bf16(bnb_bf16* g, bnb_bf16* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);
void cadagrad32bit_grad_32(float* g, float* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);
void cadagrad32bit_grad_16(bnb_fp16* g, bnb_fp16* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);
void cadagrad32bit_grad_bf16(bnb_bf16* g, bnb_bf16* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);
void clion32bit_grad_fp32(float* g, float* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);
void clion32bit_grad_fp16(bnb_fp16* g, bnb_fp16* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);
void clion32bit_grad_bf16(bnb_bf16* g, bnb_bf16* p, float* state1, float* state2, float* unorm, float max_unorm,
        float param_norm, const float beta1, const float beta2, const float eps, const float weight_decay,
        const int step, const float lr, const float gnorm_scale, bool skip_zeros, const int n);

/* ---- [additive] nested statistics -> fp32 absmax in one launch:
 * out[i] = code2[q[i]] * absmax2[i / blocksize2] + *offset (fp32 product, then fp32 add), the result of
 * dequantize_blockwise + `absmax += offset` (ref:python_src_quants/functional.py:1346-1350) ---- */
void cdequantize_nested_absmax_fp32(float* code2, unsigned char* q, float* absmax2, float* offset, float* out,
                                    int blocksize2, long long n);

/* ---- [additive] one-shot decode all-gather over peer memory (csrc/ipc.hip; SURVEY §8(e): the M = 1 all-gather is
 * latency-bound, "prefer a custom hipIPC one-shot all-gather").  Not in the reference (no multi-GPU code there): the
 * RCCL all-gather stays the prefill path.  Each rank allocates one exchange buffer (cipc_alloc, bytes from
 * cipc_allgather_buffer_bytes), exports it (cipc_get_handle), opens every peer's (cipc_open_handle), and per decode
 * step launches callgather_ipc_16: its [n] shard is pushed into every rank's buffer with an epoch flag, the rank waits
 * (bounded) for all flags and copies the assembled [world * n] row out.  state: device u32[4] zeroed once (epoch,
 * timeout count, last timed-out rank + 1).  Fail-stop: a step whose wait timed out, and every step after it, writes a
 * NaN row (all 16-bit elements 0xFFFF) instead of stale slots; the host checks the sticky count. ---- */
long long cipc_allgather_buffer_bytes(int world, int n, int elem);
void* cipc_alloc(long long bytes, int* kind);   /* kind: 2 uncached, 1 fine-grained; NULL when neither (no
                                                   coarse-grained fallback: peers' stores could be served stale) */
void cipc_free(void* p);
int cipc_handle_size(void);
int cipc_get_handle(void* p, void* handle);
int cipc_open_handle(const void* handle, void** out);
int cipc_close_handle(void* p);
int callgather_ipc_16(const unsigned long long* bufs, int rank, int world, int n, const void* y, void* rows,
                      unsigned* state);

/* ---- [additive, testing] LDS poisoning: fill every CU's 160 KiB LDS with `pattern` (blocks >= CU count), and the
 * positive control that reads LDS it never wrote (csrc/probe.hip; tests/test_lds_poison_gpu.py) ---- */
int cprobe_lds_poison(unsigned pattern, int blocks);
int cprobe_lds_peek(unsigned* out, int blocks);

/* ---- [additive] runtime ---- */
void cset_stream(void* stream);            /* hipStream_t used by every launch (NULL = null stream) */
void* cget_stream(void);
int cget_last_error(void);                 /* returns and clears the last error code (0 = none) */
const char* cget_last_error_message(void);
int cget_abi_version(void);
int croctx_enabled(void);                  /* 1 when roctx ranges are on: BNB_ROCTX=1 at load and libroctx64 found */

#ifdef __cplusplus
}
#endif

#endif /* BNB_HIP_H */
