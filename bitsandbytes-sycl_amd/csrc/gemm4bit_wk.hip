// Few-token 4-bit weight GEMM, whole K per workgroup (1..32 activation rows) for gfx950.
//
// Same slot and semantics as gemm4bit_skinny.hip (cgemm_4bit_inference*, ref:sycl/pythonInterface.cpp:377-378;
// the M > 1 path it replaces is dequantize_4bit + F.linear, ref:autograd/_functions.py:491-507): every weight is
// dequantised in fp32 and rounded once to T (kernel_quant.cpp:1428-1453 values), products on the bf16/fp16 MFMA
// with fp32 sums.
//
// The skinny kernel splits K over workgroups (fp32 partials in a workspace, then an ordered reduce launch) and
// stages the activations of its K slice in LDS before any weight lands.  Here a workgroup owns 16 weight rows (one
// MFMA row tile) and ALL of K, so there is no workspace and no second launch:
//   * WAVES waves split K: wave w takes the 128-k blocks w, w + WAVES, ... (the workgroup's waves read 64-B pieces
//     of consecutive blocks of the same rows, so a row's bytes are fetched together);
//   * each wave streams its blocks through a register ring D blocks deep: the weights (16 B per lane: row
//     l & 15, elements 32c .. 32c + 31 with c = l >> 4), the block statistics and the token fragments (token
//     16g + (l & 15), elements 32c .. 32c + 31 of the block: four 16-B loads, read from L2 -- every workgroup
//     reads the same activations) of block i + D are issued before block i is consumed, so the weight stream and
//     the dequantise + MFMA work overlap from the first block on;
//   * sub-step s of a block feeds dword s of the lane's weights (elements 32c + 8s .. + 7, one 16-B A fragment)
//     and the matching 16-B token fragment to one MFMA per 16-token tile: the k order inside an MFMA is free as
//     long as both operands share it;
//   * at the end the waves' fp32 tiles are summed in LDS in wave order (deterministic) and wave 0 stores T.
// Dequantisation: 256-entry LDS pair table (byte -> {code[hi], code[lo]}), fp32 products by the block's absmax,
// one RNE cast per value; nested statistics decoded in-kernel (code2[q8] * absmax2 + offset, the
// dequantize_blockwise order).
#include "gemm_common.hpp"

namespace bnb {

typedef float wk_f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 wk_bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 wk_f16x2_t __attribute__((ext_vector_type(2)));
template <typename T> __device__ __forceinline__ uint32_t wk_cvt2(wk_f32x2_t v);
template <> __device__ __forceinline__ uint32_t wk_cvt2<bf16_t>(wk_f32x2_t v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, wk_bf16x2_t));
}
template <> __device__ __forceinline__ uint32_t wk_cvt2<fp16_t>(wk_f32x2_t v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, wk_f16x2_t));
}

template <typename T, int MT, int WAVES, int D, bool NESTED>
__global__ void __launch_bounds__(64 * WAVES)
k_gemm_4bit_wk(int N, int M, int K, const T* __restrict__ A, int lda, const uint8_t* __restrict__ B, int ldb,
               SkStats st, const float* __restrict__ code, T* __restrict__ out, int ldc) {
  __shared__ float2 lut[256];
  __shared__ float c2s[NESTED ? 256 : 1];
  __shared__ f32x4_t red[WAVES - 1][MT][64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, c = lane >> 4;
  const int row = min((int)blockIdx.x * 16 + r, N - 1);
  const int nblk = K >> 7;
  const int nb = (nblk - wave + WAVES - 1) / WAVES;          // this wave's blocks (wave-uniform, >= 0)

  // global address space: these loads count on vmcnt only (a flat load would also count on lgkmcnt)
  typedef const __attribute__((address_space(1))) u32x4_t* gvec_t;
  typedef const __attribute__((address_space(1))) uint8_t* gbyte_t;
  typedef const __attribute__((address_space(1))) float* gfloat_t;
  const gbyte_t wrow = (gbyte_t)B + (long long)row * ldb + 16 * c;
  const T* xrow[MT];
#pragma unroll
  for (int g = 0; g < MT; ++g) xrow[g] = A + (long long)min(16 * g + r, M - 1) * lda + 32 * c;
  const long long abase = 2LL * ldb * row + 32 * c;            // element index of (row, k = 32c)

  uint4 wv[D];
  uint4 xv[D][MT][4];
  float sa[D];
  uint32_t sq[D];
  // issue the loads of this wave's i-th block into ring slot j; past the last block the weight slot reads the
  // (L2-resident) activations instead and the other loads repeat the last block: no branch, no wasted HBM bytes
  auto issue = [&](int i, int j) {
    const bool live = i < nb;
    const int b = min(wave + WAVES * max(min(i, nb - 1), 0), nblk - 1);
    const gvec_t wsrc = live ? (gvec_t)(wrow + 64LL * b) : (gvec_t)(xrow[0]);
    const u32x4_t v = __builtin_nontemporal_load(wsrc);
    wv[j] = make_uint4(v.x, v.y, v.z, v.w);
    const long long sj = (abase + 128LL * b) >> st.bs_shift;
    if constexpr (NESTED) {
      sq[j] = ((gbyte_t)st.q8)[sj];
      sa[j] = ((gfloat_t)st.absmax2)[sj >> st.bs2_shift];
    } else {
      sa[j] = ((gfloat_t)st.absmax)[sj];
    }
#pragma unroll
    for (int g = 0; g < MT; ++g)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const u32x4_t x = *(gvec_t)(xrow[g] + 128LL * b + 8 * s);
        xv[j][g][s] = make_uint4(x.x, x.y, x.z, x.w);
      }
  };

  // the ring's first D blocks fly while the tables are staged
#pragma unroll
  for (int j = 0; j < D; ++j) issue(j, j);
  float off = 0.0f;
  for (int e = tid; e < 256; e += 64 * WAVES) {
    lut[e] = make_float2(code[e >> 4], code[e & 15]);
    if constexpr (NESTED) c2s[e] = st.code2[e];
  }
  if constexpr (NESTED) off = *st.offset;
  __syncthreads();

  f32x4_t acc[MT];
#pragma unroll
  for (int g = 0; g < MT; ++g) acc[g] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int i0 = 0; i0 < nb; i0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int i = i0 + j;
      if (i < nb) {                                            // wave-uniform
        const float a = NESTED ? __fadd_rn(__fmul_rn(c2s[sq[j]], sa[j]), off) : sa[j];
        const wk_f32x2_t aa = wk_f32x2_t{a, a};
        const uint32_t wd[4] = {wv[j].x, wv[j].y, wv[j].z, wv[j].w};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          uint32_t pk[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float2 p = lut[(wd[s] >> (8 * q)) & 0xFF];
            pk[q] = wk_cvt2<T>(wk_f32x2_t{p.x, p.y} * aa);     // fp32 products, one RNE cast each
          }
          const uint4 fa = make_uint4(pk[0], pk[1], pk[2], pk[3]);
#pragma unroll
          for (int g = 0; g < MT; ++g) acc[g] = Mfma<T>::mma(fa, xv[j][g][s], acc[g]);
        }
      }
      issue(i + D, j);
    }
  }

  // ordered cross-wave sum: wave 0 + wave 1 + ... (fp32), one RNE cast
  if (wave > 0) {
#pragma unroll
    for (int g = 0; g < MT; ++g) red[wave - 1][g][lane] = acc[g];
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int w = 1; w < WAVES; ++w)
#pragma unroll
    for (int g = 0; g < MT; ++g) acc[g] += red[w - 1][g][lane];
  // D[i]: weight row 4c + i of the tile, token 16g + r
  const int row0 = (int)blockIdx.x * 16 + 4 * c;
#pragma unroll
  for (int g = 0; g < MT; ++g) {
    const int t = 16 * g + r;
    if (t >= M) continue;
    T* dst = out + (long long)t * ldc + row0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (row0 + q < N) dst[q] = Io<T>::from_f32(acc[g][q]);
  }
}

int device_cu_count();      // CUs of the current device (cached; gemv4bit.hip)
// 0 = auto (this kernel at <= WK_MAX_TOKENS tokens on narrow weights, else the split-K kernel), 1 = the split-K
// skinny kernel only, 2 = this kernel for every shape it fits (A/B knob; tests)
Knob<int> g_fewtoken_kernel{0};
constexpr int WK_MAX_TOKENS = 6;

bool wk_applicable(int m, int n, int k, int lda, int ldb, int blocksize, const void* A, const void* B) {
  return g_fewtoken_kernel != 1 && n >= 1 && n <= 32 && m >= 1 && k >= 128 && k % 128 == 0 && blocksize >= 64 &&
         (blocksize & (blocksize - 1)) == 0 && lda % 8 == 0 && ldb % 16 == 0 && ((uintptr_t)A & 15) == 0 &&
         ((uintptr_t)B & 15) == 0;
}

// m = out features (weight rows), n = tokens, k = in features.  False: not applicable.
template <typename T>
bool launch_gemm_4bit_wk(int m, int n, int k, const T* A, int lda, const uint8_t* B, int ldb, SkStats st,
                         int blocksize, int blocksize2, const float* code, T* out, int ldc) {
  if (!wk_applicable(m, n, k, lda, ldb, blocksize, A, B)) return false;
  const bool nested = st.q8 != nullptr;
  if (nested && (blocksize2 <= 0 || (blocksize2 & (blocksize2 - 1)))) return false;
  st.bs_shift = __builtin_ctz(blocksize);
  st.bs2_shift = nested ? __builtin_ctz(blocksize2) : 0;
  const int tiles = (m + 15) / 16;
  // Where it is used (tools/fewtoken_ab.py, profiles/lab/r02_fewtoken_whole_k.txt): every workgroup reads the
  // token rows of all of K from L2, 16 weight rows per read, so the activation traffic grows with the tokens and
  // the split-K kernel (64 weight rows share one LDS copy) wins from ~8 tokens on, and on wide weights (>= 2 row
  // tiles per CU) at any count.  This kernel runs at <= WK_MAX_TOKENS tokens on narrower weights (8 waves per row
  // tile), e.g. 4096 x 11008 at 5 tokens 13.4 vs 16.0 us, 4096 x 4096 8.5 vs 9.3 us; g_fewtoken_kernel = 2 forces
  // it for every 1..32-token shape (tests, A/B).
  // Not on long K or on very narrow weights either (1024 x 28672 at 2..4 rows 26-29 vs 15.7 us split-K; 128 x 8192
  // 9.6 vs 8.8 us: profiles/lab/r02_gemv_wide.txt): every workgroup re-reads the token rows of all of K from L2.
  const bool forced = g_fewtoken_kernel == 2;
  if (!forced && (n > WK_MAX_TOKENS || tiles >= 2 * device_cu_count() || tiles < 64 || k > 16384)) return false;
  const bool wide = tiles >= 2 * device_cu_count();
  const dim3 grid((unsigned)tiles);
  auto go = [&](auto kern, int waves) {
    hipLaunchKernelGGL(kern, grid, dim3(64 * waves), 0, current_stream(), m, n, k, A, lda, B, ldb, st, code, out, ldc);
  };
  const bool mt1 = n <= 16;
  if (nested) {
    if (mt1) wide ? go(k_gemm_4bit_wk<T, 1, 4, 4, true>, 4) : go(k_gemm_4bit_wk<T, 1, 8, 4, true>, 8);
    else wide ? go(k_gemm_4bit_wk<T, 2, 4, 3, true>, 4) : go(k_gemm_4bit_wk<T, 2, 8, 3, true>, 8);
  } else {
    if (mt1) wide ? go(k_gemm_4bit_wk<T, 1, 4, 4, false>, 4) : go(k_gemm_4bit_wk<T, 1, 8, 4, false>, 8);
    else wide ? go(k_gemm_4bit_wk<T, 2, 4, 3, false>, 4) : go(k_gemm_4bit_wk<T, 2, 8, 3, false>, 8);
  }
  return true;
}

template bool launch_gemm_4bit_wk<bf16_t>(int, int, int, const bf16_t*, int, const uint8_t*, int, SkStats, int, int,
                                          const float*, bf16_t*, int);
template bool launch_gemm_4bit_wk<fp16_t>(int, int, int, const fp16_t*, int, const uint8_t*, int, SkStats, int, int,
                                          const float*, fp16_t*, int);

}  // namespace bnb

extern "C" {
// [additive, testing] few-token kernel choice: 0 = auto, 1 = the split-K skinny kernel (gemm4bit_skinny.hip) only,
// 2 = the whole-K kernel (gemm4bit_wk.hip) wherever it fits
void cgemm_4bit_set_fewtoken_kernel(int which) { bnb::g_fewtoken_kernel = which; }
}
