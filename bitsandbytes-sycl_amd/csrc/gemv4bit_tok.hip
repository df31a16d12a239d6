// 4-bit GEMV for a few activation rows (2..8 tokens: batched decode, speculative verification) for gfx950.
//
// Same slot as the few-token GEMM (cgemm_4bit_inference*, ref:sycl/pythonInterface.cpp:377-378; the M > 1 path it
// replaces is dequantize_4bit + F.linear, ref:autograd/_functions.py:491-507) and the arithmetic of the decode GEMV
// (gemv4bit.hip, ref:sycl/sycl_code/kernel_gemm.cpp:1271-1388) applied to every token: per packed byte one table
// lookup {T(code[hi]), T(code[lo])} and one v_dot2c_f32_{bf16,f16} per token against the matching activation pair;
// each 32-element chunk is scaled once by its fp32 absmax.  Every token's output row is bit-identical to the
// one-row GEMV on that row (same lane -> chunk map, same chains, same wave reduction).
//
// Structure (the balanced GEMV's, k_gemv_4bit_bal): G workgroups (two per CU where the LDS allows), workgroup g owns
// a balanced range of weight rows and the WHOLE K -- no split-K partials, no second launch; NW waves take rows
// r0 + w + NW*j.  The weight bytes are streamed once, non-temporal; the TOK activation rows sit in LDS (swizzled as
// in the balanced GEMV), the pair table is 32 bank-private copies at a 128-B stride (32 KiB, so two workgroups fit a
// CU with 2..4 rows of K = 4096 activations).  Per chunk: R x 16 lookups, then per token 4 ds_read_b128 of
// activations and R x 16 dot2 -- the lookups are shared by the tokens.
#include "common.hpp"
#include "gemm_common.hpp"
#include "gemv_common.hpp"

namespace bnb {

constexpr int GT_TABLE_BYTES = 256 * 128;
constexpr int GT_MAX_WAVES = 16;
constexpr size_t GT_TWO_PER_CU_LDS = 80 * 1024 - 1024;

template <typename T, int R, int U, bool NESTED, int TOK>
__global__ void __launch_bounds__(GT_MAX_WAVES * 64)
k_gemv_4bit_tok(int M, int K, int ntok, const T* __restrict__ A, int lda, const uint8_t* __restrict__ B, GemvStats st,
                const float* __restrict__ datatype, T* __restrict__ out, int ldb, int ldc, int G) {
  extern __shared__ __attribute__((aligned(16))) uint8_t gsm[];
  uint8_t* table = gsm;                               // GT_TABLE_BYTES
  uint8_t* xs = gsm + GT_TABLE_BYTES;                 // TOK rows of K * 2 bytes, each swizzled
  float* code2s = reinterpret_cast<float*>(xs + (size_t)TOK * 2 * K);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int NW = blockDim.x >> 6;
  const int r0 = (int)((long long)blockIdx.x * M / G), r1 = (int)((long long)(blockIdx.x + 1) * M / G);
  const int nch = K >> 5;
  const long long two_ldb = 2LL * ldb;
  auto row_of = [&](int j) { return min(r0 + wave + NW * j, r1 - 1); };
  auto chunk_of = [&](int u) { return min(lane + 64 * u, nch - 1); };

  // (1) code values (scalar), block statistics, activations by LDS-DMA (16-B piece q of chunk c of token row t
  //     at t * 2K + 64 c + 16 ((q + (c >> 2)) & 3); rows past ntok repeat the last row, never stored)
  float dt[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) dt[j] = datatype[j];
  float am[U][R];
  uint32_t q8[U][R];
  float a2[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const long long blk = (two_ldb * row_of(j) + 32LL * chunk_of(u)) >> st.bs_shift;
      if constexpr (NESTED) {
        q8[u][j] = st.q8[blk];
        a2[u][j] = st.absmax2[blk >> st.bs2_shift];
      } else {
        am[u][j] = st.absmax[blk];
      }
    }
  float offset = 0.0f, c2 = 0.0f;
  if constexpr (NESTED) {
    offset = *st.offset;
    c2 = st.code2[threadIdx.x & 255];                 // threads past 256 load a duplicate, stored by nobody
  }
  const int nx = K >> 3;                              // 16-B pieces per token row
  for (int p = wave; p * 64 < TOK * nx; p += NW) {
    const int i = p * 64 + lane;
    if (i < TOK * nx) {
      const int t = i / nx, ii = i - t * nx, c = ii >> 2;
      glds16(A + (long long)min(t, ntok - 1) * lda + 8 * (4 * c + (((ii & 3) - (c >> 2)) & 3)), xs + p * 1024);
    }
  }
  __builtin_amdgcn_s_barrier();                       // all statistics / activation requests are out
  // (2) this wave's weights, non-temporal, consumption order
  uintptr_t bp = (uintptr_t)B;
  asm volatile("" : "+s"(bp)::"memory");
  uint4 b[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const u32x4_t v =
          __builtin_nontemporal_load((gvec_p)((gbyte_p)bp + (long long)row_of(j) * ldb + 16LL * chunk_of(u)));
      b[u][j] = make_uint4(v.x, v.y, v.z, v.w);
    }
  // (3) table: thread t < 256 writes entry t, 32 copies at 128 e + 4 copy (16-B stores rotated by t)
  for (int t = threadIdx.x; t < 256; t += NW * 64) {
    float hi = dt[0], lo = dt[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) {
      hi = (t >> 4) == j ? dt[j] : hi;
      lo = (t & 15) == j ? dt[j] : lo;
    }
    const uint32_t v = Dot2<T>::pair(hi, lo);
#pragma unroll
    for (int k = 0; k < 8; ++k) *reinterpret_cast<uint4*>(table + 128 * t + 16 * ((k + t) & 7)) = make_uint4(v, v, v, v);
  }
  if constexpr (NESTED) {
    if (threadIdx.x < 256) code2s[threadIdx.x] = c2;
    for (int t = threadIdx.x + NW * 64; t < 256; t += NW * 64) code2s[t] = st.code2[t];   // < 4 waves
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R * U) : "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  if constexpr (NESTED) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < R; ++j) am[u][j] = __fadd_rn(__fmul_rn(code2s[q8[u][j]], a2[u][j]), offset);
  }
  float acc[TOK][R];
#pragma unroll
  for (int t = 0; t < TOK; ++t)
#pragma unroll
    for (int j = 0; j < R; ++j) acc[t][j] = 0.0f;
  const uint32_t lane4 = (lane & 31) * 4;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool valid = lane + 64 * u < nch;
    const int c = chunk_of(u);
    uint32_t l[R][16];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t w[4] = {b[u][j].x, b[u][j].y, b[u][j].z, b[u][j].w};
#pragma unroll
      for (int i = 0; i < 16; ++i)
        l[j][i] = *reinterpret_cast<const uint32_t*>(table + ((((w[i >> 2] >> (8 * (i & 3))) & 0xFF) << 7) | lane4));
    }
#pragma unroll
    for (int t = 0; t < TOK; ++t) {
      uint32_t x[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 v = reinterpret_cast<const uint4*>(xs + (size_t)t * 2 * K + 64 * c)[(q + (c >> 2)) & 3];
        x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          s0 = Dot2<T>::dot(x[i], l[j][i], s0);
          s1 = Dot2<T>::dot(x[i + 1], l[j][i + 1], s1);
        }
        const float part = (s0 + s1) * am[u][j];
        acc[t][j] += valid ? part : 0.0f;
      }
    }
  }
#pragma unroll
  for (int t = 0; t < TOK; ++t)
#pragma unroll
    for (int j = 0; j < R; ++j) acc[t][j] = wave_sum(acc[t][j]);
  if (lane == 0) {
#pragma unroll
    for (int t = 0; t < TOK; ++t) {
      if (t >= ntok) break;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int row = r0 + wave + NW * j;
        if (row < r1) out[(long long)t * ldc + row] = Io<T>::from_f32(acc[t][j]);
      }
    }
  }
}

constexpr int GT_MAX_TOKENS = 4;

// m = weight rows, ntok = activation rows (2..GT_MAX_TOKENS), k = in features.  False: shape, alignment or size
// does not fit (the caller then uses the few-token GEMM).
template <typename T, bool NESTED>
static bool launch_gemv_tok(int m, int ntok, int k, const T* A, int lda, const uint8_t* B, int ldb, GemvStats st,
                            const float* datatype, T* out, int ldc) {
  if (ntok < 2 || ntok > GT_MAX_TOKENS || k > GV_MAX_K) return false;
  // fewer weight rows than CUs leave most of the chip idle here (whole rows per workgroup): the split-K few-token
  // kernel is faster there (128 x 8192 at 4 rows 12.8 -> 9.0 us; profiles/lab/r02_gemv_wide.txt)
  if (m < device_cu_count()) return false;
  const int tok = ntok <= 2 ? 2 : 4;
  const size_t lds = GT_TABLE_BYTES + (size_t)tok * 2 * k + (NESTED ? 1024 : 0);
  if (lds > 160 * 1024) return false;
  const bool two = lds <= GT_TWO_PER_CU_LDS;
  int U = ((k >> 5) + 63) / 64;
  if (U > 4) U = U <= 6 ? 6 : 8;
  const int max_waves = two ? 8 : 16;
  const int r_max = min(4, (tok == 4 ? 6 : 8) / U);                 // R x U loads per lane (R 4 x U 2 at 4 tokens spills)
  if (r_max < 1) return false;
  // two (or one) balanced workgroups per CU; more when that many rows per wave would not fit the registers
  int G = (two ? 2 : 1) * device_cu_count();
  if ((long long)G * max_waves * r_max < m) G = (int)((m + (long long)max_waves * r_max - 1) / ((long long)max_waves * r_max));
  G = min(G, m);
  const int rows = (m + G - 1) / G;
  const int R = (rows + max_waves - 1) / max_waves;
  if (R > r_max) return false;
  const int nw = (rows + R - 1) / R;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(G), dim3(64 * nw), lds, current_stream(), m, k, ntok, A, lda, B, st, datatype, out,
                       ldb, ldc, G);
    return true;
  };
#define GT_CASES(TK)                                                                     \
  switch (R * 8 + U) {                                                                   \
    case 8 + 1: return go(k_gemv_4bit_tok<T, 1, 1, NESTED, TK>);                         \
    case 8 + 2: return go(k_gemv_4bit_tok<T, 1, 2, NESTED, TK>);                         \
    case 8 + 3: return go(k_gemv_4bit_tok<T, 1, 3, NESTED, TK>);                         \
    case 8 + 4: return go(k_gemv_4bit_tok<T, 1, 4, NESTED, TK>);                         \
    case 8 + 6: return go(k_gemv_4bit_tok<T, 1, 6, NESTED, TK>);                         \
    case 8 + 8: return go(k_gemv_4bit_tok<T, 1, 8, NESTED, TK>);                         \
    case 16 + 1: return go(k_gemv_4bit_tok<T, 2, 1, NESTED, TK>);                        \
    case 16 + 2: return go(k_gemv_4bit_tok<T, 2, 2, NESTED, TK>);                        \
    case 16 + 3: return go(k_gemv_4bit_tok<T, 2, 3, NESTED, TK>);                        \
    case 16 + 4: return go(k_gemv_4bit_tok<T, 2, 4, NESTED, TK>);                        \
    case 24 + 1: return go(k_gemv_4bit_tok<T, 3, 1, NESTED, TK>);                        \
    case 24 + 2: return go(k_gemv_4bit_tok<T, 3, 2, NESTED, TK>);                        \
    case 32 + 1: return go(k_gemv_4bit_tok<T, 4, 1, NESTED, TK>);                        \
    case 32 + 2: return go(k_gemv_4bit_tok<T, 4, 2, NESTED, TK>);                        \
    default: return false;                                                               \
  }
  if (tok == 2) { GT_CASES(2) }
  else { GT_CASES(4) }
#undef GT_CASES
}

template <typename T>
static int gemv_tokens(int m, int ntok, int k, const T* A, int lda, const uint8_t* B, int ldb, const float* absmax,
                       const uint8_t* absmax_q, const float* code2, const float* absmax2, const float* offset,
                       const float* datatype, T* out, int ldc, int blocksize, int blocksize2) {
  if (m <= 0) return 0;
  const bool nested = absmax_q != nullptr;
  if (k % 32 || ldb % 16 || lda % 8 || ((uintptr_t)A & 15) || ((uintptr_t)B & 15) || blocksize < 32 ||
      (blocksize & (blocksize - 1)) || (nested && (blocksize2 <= 0 || (blocksize2 & (blocksize2 - 1)))))
    return 1;
  GemvStats st{absmax, absmax_q, code2, absmax2, offset, __builtin_ctz(blocksize), nested ? __builtin_ctz(blocksize2) : 0};
  const bool ok = nested ? launch_gemv_tok<T, true>(m, ntok, k, A, lda, B, ldb, st, datatype, out, ldc)
                         : launch_gemv_tok<T, false>(m, ntok, k, A, lda, B, ldb, st, datatype, out, ldc);
  if (!ok) return 1;
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_error((int)e, "gemv_4bit_tokens"); return 2; }
  return 0;
}

}  // namespace bnb

using namespace bnb;

extern "C" {

// [additive] 4-bit weight x 2..4 activation rows in one launch (out[t, r] for t < ntok, row stride ldc): plain fp32
// statistics (absmax_q = NULL) or compressed ones decoded in-kernel (absmax = NULL).  Returns 0 when launched, 1 when
// the shape or alignment does not fit (nothing launched), 2 when the launch failed.
int cgemm_4bit_inference_tokens_bf16(int m, int ntok, int k, bf16_t* A, int lda, unsigned char* B, int ldb, float* absmax,
                                     unsigned char* absmax_q, float* code2, float* absmax2, float* offset,
                                     float* datatype, bf16_t* out, int ldc, int blocksize, int blocksize2) {
  BNB_RANGE("cgemm_4bit_inference_tokens_bf16");
  return gemv_tokens<bf16_t>(m, ntok, k, A, lda, B, ldb, absmax, absmax_q, code2, absmax2, offset, datatype, out, ldc,
                             blocksize, blocksize2);
}
int cgemm_4bit_inference_tokens_fp16(int m, int ntok, int k, fp16_t* A, int lda, unsigned char* B, int ldb, float* absmax,
                                     unsigned char* absmax_q, float* code2, float* absmax2, float* offset,
                                     float* datatype, fp16_t* out, int ldc, int blocksize, int blocksize2) {
  BNB_RANGE("cgemm_4bit_inference_tokens_fp16");
  return gemv_tokens<fp16_t>(m, ntok, k, A, lda, B, ldb, absmax, absmax_q, code2, absmax2, offset, datatype, out, ldc,
                             blocksize, blocksize2);
}

}  // extern "C"
