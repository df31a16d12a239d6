// Few-token 4-bit weight GEMM (batched decode / short prefill, 2..64 activation rows) for gfx950.
//
// Same slot and semantics as gemm4bit.hip (cgemm_4bit_inference*, ref:sycl/pythonInterface.cpp:377-378;
// the M > 1 path it replaces is dequantize_4bit + F.linear, ref:autograd/_functions.py:491-507): every
// weight is dequantised in fp32 and rounded once to T, products on the bf16/fp16 MFMA with fp32 sums.
//
// With few tokens the problem is a weight stream (0.5 B per weight, read once), so the design is the
// GEMV's, widened to MFMA: a workgroup of 4 waves owns 64 weight rows (16 per wave) and one K range.
//   * A operand = 16 weight rows: lane (r, c) = (l & 15, l >> 4) loads 16 packed bytes of row r per
//     128-k block (bytes 16c..16c+15, elements 32c..32c+31; one 64-element absmax block) and feeds the
//     MFMA of sub-step s with dword s dequantised (elements 32c + 8s .. +7).  The k order inside an MFMA
//     is a free choice as long as both operands use it: the B operand (16 tokens) lane (t, c) holds the
//     same elements 32c + 8s .. +7 of token t.
//   * All of a workgroup's loads are issued up front (GEMV schedule): statistics, then the K slice of
//     every token row by LDS-DMA (16-B slots XOR-swizzled by the token row through the source address,
//     shared by the 4 waves), then every weight chunk of the lane; each block is consumed as it lands.
//   * Dequantisation through a 256-entry LDS pair table (byte -> {code[hi], code[lo]}; one copy, so a
//     lookup address is one SDWA shift of the packed byte -- 1, 4, 8 and 16 interleaved copies measured
//     equal or slower, tools/skinny_lab.hip), a packed fp32 multiply by absmax and one packed RNE cast
//     per byte (kernel_quant.cpp:1428-1453 values).
//   * Nested statistics (NESTED) are decoded in-kernel: code2[q8[j]] * absmax2[j >> log2(bs2)] + offset
//     (the dequantize_blockwise order), removing the absmax decode launch.
//   * Split-K over workgroups when 64-row blocks alone would not fill the chip: fp32 partials
//     ws[split][token][row], summed in split order by k_skinny_reduce (deterministic).
#include "gemm_common.hpp"

#include <algorithm>
#include <type_traits>

namespace bnb {
#ifndef LUTC_DEF
#define LUTC_DEF 1
#endif

// timeline hooks for tools/fewtoken_lab.hip (no code in the library build)
#ifndef SK_STAMP
#define SK_STAMP(i)
#endif

[[maybe_unused]] constexpr int SK_THREADS = 256, SK_ROWS = 64;  // base form (labs)
constexpr int SK_LUTC = LUTC_DEF, SK_MAX_TOKENS = 64;


typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
// {T(v.x), T(v.y)}, one RNE cast each, as one packed convert
template <typename T> __device__ __forceinline__ uint32_t sk_cvt2v(f32x2_t v);
template <> __device__ __forceinline__ uint32_t sk_cvt2v<bf16_t>(f32x2_t v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}
template <> __device__ __forceinline__ uint32_t sk_cvt2v<fp16_t>(f32x2_t v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2_t));
}

// ABL (design lab only, tools/skinny_lab.hip): 1 = no weight loads, 2 = no activation DMA, 4 = no MFMA.
// W = waves per workgroup (16 W weight rows share one LDS copy of the token rows): 4, or 8 (half the activation
// DMA per weight row, one workgroup per CU).
template <typename T, int MT, int NB, bool NESTED, int ABL = 0, int W = 4>
__global__ void __launch_bounds__(64 * W, W == 4 ? 2 : 1)
k_gemm_4bit_skinny(int N, int M, int K, const T* __restrict__ A, int lda, const uint8_t* __restrict__ B, int ldb,
                   SkStats st, const float* __restrict__ code, float* __restrict__ ws, T* __restrict__ out, int ldc,
                   int nsplit) {
  constexpr int MP = 16 * MT;                    // token rows held (padded to the MFMA width)
  constexpr int XBLK = MP * 256;                 // LDS bytes of one 128-k block of all tokens
  constexpr int THREADS = 64 * W, ROWS = 16 * W;
  constexpr int XP = NB * MT * 4 / W;            // 1-KiB activation DMA pieces per wave
  static_assert((NB * MT * 4) % W == 0, "whole DMA pieces per wave");
  __shared__ __attribute__((aligned(16))) uint8_t xs[(NB + 1) * XBLK];   // + one zero block
  __shared__ float2 lut[256 * SK_LUTC];
  __shared__ float c2s[NESTED ? 256 : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rb = blockIdx.x / nsplit, split = blockIdx.x - rb * nsplit;
  const int r = lane & 15, c = lane >> 4;
  const int rowc = min(rb * ROWS + 16 * wave + r, N - 1);
  const int kb0 = split * NB;                                  // first 128-k block of this split
  const int nb = min(NB, (K >> 7) - kb0);                      // >= 1 by construction
  SK_STAMP(0);

  // (1a) table values and statistics first: their consumers must not wait on the weight loads below
  // (the VMEM counter retires in order)
  const int te = tid & 255;                                    // table entry of this thread (tid < 256 stores)
  const float code_hi = code[te >> 4], code_lo = code[te & 15];
  float off = 0.0f, c2v = 0.0f;
  if constexpr (NESTED) {
    c2v = st.code2[te];
    off = *st.offset;
  }
  const long long abase = 2LL * ldb * rowc + 32 * c + 128LL * kb0;   // element index of (row, k)
  float am[NB];
  uint32_t q8[NB];
  float a2[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const long long j = (abase + 128 * min(b, nb - 1)) >> st.bs_shift;
    if constexpr (NESTED) {
      q8[b] = st.q8[j];
      a2[b] = st.absmax2[j >> st.bs2_shift];
    } else {
      am[b] = st.absmax[j];
    }
  }
  // (1b) this split's activations for all tokens by LDS-DMA: piece p = (block, 4 token rows); lane ->
  // row 4 (p % 4MT) + (l >> 4), LDS slot l & 15 holding source slot (l & 15) ^ (row & 15)
#pragma unroll
  for (int i = 0; i < ((ABL & 2) ? 0 : XP); ++i) {
    const int p = wave + W * i;
    const int blk = p / (4 * MT), t = 4 * (p % (4 * MT)) + (lane >> 4);
    const int gslot = (lane & 15) ^ (t & 15);
    glds16(A + (long long)min(t, M - 1) * lda + 128LL * (kb0 + min(blk, nb - 1)) + 8 * gslot,
           xs + blk * XBLK + (p % (4 * MT)) * 1024);
  }
  // (1c) all of this lane's weight chunks (non-temporal: read once); the laundered pointer keeps them
  // behind the DMA, so vmcnt(NB) below means "activations landed"
  uintptr_t bp = (uintptr_t)B;
  asm volatile("" : "+s"(bp)::"memory");
  // (global address space: a flat load would also count on lgkmcnt and order against the LDS stores)
  typedef const __attribute__((address_space(1))) uint8_t* gbyte_t;
  typedef const __attribute__((address_space(1))) u32x4_t* gvec_t;
  const gbyte_t wp = (gbyte_t)bp + (long long)rowc * ldb + 16 * c + 64LL * kb0;
  uint4 w[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if constexpr ((ABL & 1) == 0) {
      const u32x4_t v = __builtin_nontemporal_load((gvec_t)(wp + 64 * min(b, nb - 1)));
      w[b] = make_uint4(v.x, v.y, v.z, v.w);
    } else {
      w[b] = make_uint4(b * 0x01010101u + rowc, 0x12345678u, 0x9abcdef0u, c);
    }
  }
  // (2) table (+ nested code map) while the loads fly: entry tid, copies 0..SK_LUTC-1
  if (tid < 256) {
#pragma unroll
    for (int j = 0; j < SK_LUTC; ++j) lut[tid * SK_LUTC + j] = make_float2(code_hi, code_lo);
    if constexpr (NESTED) c2s[tid] = c2v;
  }
  // a zero activation block: blocks past a short last split multiply it (exact zeros, no branch)
  for (int i = tid; i < XBLK / 16; i += THREADS) *reinterpret_cast<uint4*>(xs + NB * XBLK + 16 * i) = make_uint4(0, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NB) : "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  SK_STAMP(1);
  const float2* lutc = lut + (lane & (SK_LUTC - 1));

  // (3) per block, as its weights land: 16 table pairs (read one block ahead), one 16-row x 32-k A
  // fragment per sub-step, MT MFMAs against the token fragments.  One accumulator per sub-step keeps
  // the MFMAs independent; they are summed in a fixed order at the end.
  f32x4_t acc[4][MT];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int g = 0; g < MT; ++g) acc[s][g] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto pairs = [&](const uint4& wv, f32x2_t (&p)[16]) {
    const uint32_t wd[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float2 v = lutc[((wd[i >> 2] >> (8 * (i & 3))) & 0xFF) * SK_LUTC];
      p[i] = f32x2_t{v.x, v.y};
    }
  };
  f32x2_t pp[2][16];                                           // table pairs of blocks b (and b+1)
  pairs(w[0], pp[0]);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const uint8_t* xb = xs + (b < nb ? b : NB) * XBLK;         // (uniform) past a short split: zeros
    if (b + 1 < NB) pairs(w[b + 1], pp[(b + 1) & 1]);
    uint4 fx[4][MT];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int g = 0; g < MT; ++g) {
        const int t = 16 * g + r;
        fx[s][g] = *reinterpret_cast<const uint4*>(xb + t * 256 + 16 * ((4 * c + s) ^ (t & 15)));
      }
    float a;
    if constexpr (NESTED) a = __fadd_rn(__fmul_rn(c2s[q8[b]], a2[b]), off);
    else a = am[b];
    const f32x2_t aa = f32x2_t{a, a};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      uint32_t pk[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) pk[i] = sk_cvt2v<T>(pp[b & 1][4 * s + i] * aa);   // fp32 products (v_pk_mul_f32), one RNE cast
      const uint4 fa = make_uint4(pk[0], pk[1], pk[2], pk[3]);
      if constexpr ((ABL & 4) == 0) {
#pragma unroll
        for (int g = 0; g < MT; ++g) acc[s][g] = Mfma<T>::mma(fa, fx[s][g], acc[s][g]);
      }
    }
  }
#pragma unroll
  for (int g = 0; g < MT; ++g)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[0][g][i] = (acc[0][g][i] + acc[1][g][i]) + (acc[2][g][i] + acc[3][g][i]);

  SK_STAMP(2);
  // D[i]: weight row 4c + i of the wave's 16, token 16g + r -> 4 consecutive features per lane
  const int row0 = rb * ROWS + 16 * wave + 4 * c;
#pragma unroll
  for (int g = 0; g < MT; ++g) {
    const int t = 16 * g + r;
    if (t >= M) continue;
    if (nsplit > 1) {
      float* dst = ws + ((long long)split * M + t) * N + row0;
      if (row0 + 4 <= N && (N & 3) == 0) {
        *reinterpret_cast<float4*>(dst) = make_float4(acc[0][g][0], acc[0][g][1], acc[0][g][2], acc[0][g][3]);
      } else {
        for (int i = 0; i < 4; ++i)
          if (row0 + i < N) dst[i] = acc[0][g][i];
      }
    } else {
      T* dst = out + (long long)t * ldc + row0;
      for (int i = 0; i < 4; ++i)
        if (row0 + i < N) dst[i] = Io<T>::from_f32(acc[0][g][i]);
    }
  }
}

// out[t, n] = T(sum_s ws[s][t][n]), splits summed in order (fp32), one RNE cast; 4 outputs per thread.
// The partials were just written by other XCDs (read back through the MALL), so the loads of up to BATCH splits
// are issued together (indices clamped, unconditional) before any add: one round trip for the usual 2..8
// splits instead of one per split.  Same additions in the same order as a sequential loop.  BATCH (2, 4 or 8) is the
// smallest that covers the split count up to 8 (round 5: with BATCH 8 for 4 splits, half the loads re-read split 3).
template <typename T, int BATCH = 8>
__global__ void __launch_bounds__(256)
k_skinny_reduce(const float* __restrict__ ws, int nsplit, int M, int N, T* __restrict__ out, int ldc) {
  const long long mn = (long long)M * N;
  const long long i0 = 4 * ((long long)blockIdx.x * 256 + threadIdx.x);
  if (i0 >= mn) return;
  if ((N & 3) == 0) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k0 = 0; k0 < nsplit; k0 += BATCH) {
      float4 v[BATCH];
#pragma unroll
      for (int b = 0; b < BATCH; ++b)
        v[b] = *reinterpret_cast<const float4*>(ws + min(k0 + b, nsplit - 1) * mn + i0);
#pragma unroll
      for (int b = 0; b < BATCH; ++b) {
        const bool live = k0 + b < nsplit;
        if (k0 + b == 0) {
          s = v[0];
        } else {
          s.x = live ? s.x + v[b].x : s.x; s.y = live ? s.y + v[b].y : s.y;
          s.z = live ? s.z + v[b].z : s.z; s.w = live ? s.w + v[b].w : s.w;
        }
      }
    }
    const long long t = i0 / N, n = i0 - t * N;
    T* dst = out + t * ldc + n;
    if ((((uintptr_t)dst) & 7) == 0) {                 // one 8-B store of the four (one RNE cast each)
      *reinterpret_cast<uint2*>(dst) = make_uint2(sk_cvt2v<T>((f32x2_t){s.x, s.y}), sk_cvt2v<T>((f32x2_t){s.z, s.w}));
    } else {
      dst[0] = Io<T>::from_f32(s.x); dst[1] = Io<T>::from_f32(s.y);
      dst[2] = Io<T>::from_f32(s.z); dst[3] = Io<T>::from_f32(s.w);
    }
  } else {
    for (long long i = i0; i < i0 + 4 && i < mn; ++i) {
      float s = ws[i];
      for (int k = 1; k < nsplit; ++k) s += ws[k * mn + i];
      const long long t = i / N, n = i - t * N;
      out[t * ldc + n] = Io<T>::from_f32(s);
    }
  }
}

// Blocks of 128 k per workgroup: the activation slice ((NB + 1) x 16 MT rows x 256 B = 44 / 48 KiB at MT 1 / 2,
// plus the pair table and code2: 47 / 51 KiB in all) lets three workgroups fit a CU; at MT 4 (33..64 rows) three
// blocks, 64 KiB + 3 KiB, two per CU.  All of a workgroup's weights are in flight at once (NB x 16 B per lane).
template <int MT> constexpr int skinny_nb() { return MT == 1 ? 10 : (MT == 2 ? 5 : 3); }

// 16-token MFMA tiles held: 1, 2, or 4 (33..64 rows)
static int skinny_tiles(int n) { return n <= 16 ? 1 : (n <= 32 ? 2 : 4); }

bool skinny_applicable(int m, int n, int k, int lda, int ldb, int blocksize, const void* A, const void* B) {
  return n >= 1 && n <= SK_MAX_TOKENS && m >= 1 && k >= 128 && k % 128 == 0 && blocksize >= 64 &&
         (blocksize & (blocksize - 1)) == 0 && lda % 8 == 0 && ldb % 16 == 0 && ((uintptr_t)A & 15) == 0 &&
         ((uintptr_t)B & 15) == 0;
}

// Geometry (profiles/lab/r02_skinny_waves.txt).  The base form is 4 waves (64 weight rows) per workgroup with the NB
// above.  At 33..64 rows a second form, 8 waves (128 weight rows sharing one LDS copy of the token rows) with twice the
// blocks per split, halves the splits and so the fp32 partials the reduce re-reads: 4096 x 11008 at 64 rows 32.9 ->
// 28.0 us, 4096 x 4096 19.3 -> 17.4 us.  It has a quarter of the workgroups, so it loses when its last round of
// workgroups is mostly empty (11008 x 4096: 516 workgroups on 256 CUs, 30.2 -> 36.8 us at 48 rows); it is taken when
// that round is at least 70 % full.  At 1..32 rows the 8-wave forms lost everywhere (same NB: +1..3 us; 2 x NB: +5..14 us).
// g_skinny_cfg (cgemm_4bit_set_skinny_config, lab A/B): -1 = that rule, 0 = base, 1 = 8 waves same NB, 2 = 8 waves 2 x NB.
static Knob<int> g_skinny_cfg{-1};
extern Knob<int> g_fewtoken_kernel;   // gemm4bit_wk.hip
int skinny_cfg_knob() { return g_skinny_cfg; }

struct SkGeom {
  int cfg, waves, nb, splits;
};

int device_cu_count();   // CUs of the current device (cached; gemv4bit.hip)

static SkGeom skinny_geometry(int m, int n, int k) {
  const int mt = skinny_tiles(n), kb = k / 128;
  const int nb = mt == 1 ? skinny_nb<1>() : (mt == 2 ? skinny_nb<2>() : skinny_nb<4>());
  int cfg = g_skinny_cfg;
  if (cfg < 0) {
    cfg = 0;
    if (mt == 4) {
      const long long wg = (long long)((m + 127) / 128) * ((kb + 2 * nb - 1) / (2 * nb));
      const long long cus = device_cu_count(), rounds = (wg + cus - 1) / cus;
      if (10 * wg >= 7 * rounds * cus) cfg = 2;
    }
  }
  const int nbw = cfg == 2 ? 2 * nb : nb;
  return SkGeom{cfg, cfg == 0 ? 4 : 8, nbw, (kb + nbw - 1) / nbw};
}

// workspace for any geometry: the base form has the most splits
long long skinny_workspace_bytes(int m, int n, int k) {
  if (n < 1 || n > SK_MAX_TOKENS || k < 128 || k % 128) return 0;
  const int mt = skinny_tiles(n), nb = mt == 1 ? skinny_nb<1>() : (mt == 2 ? skinny_nb<2>() : skinny_nb<4>());
  const int s = (k / 128 + nb - 1) / nb;
  return std::max(s > 1 ? (long long)s * n * m * (long long)sizeof(float) : 0LL, t64_workspace_bytes(m, n, k));
}

// m = out features (weight rows), n = tokens, k = in features.  False: not applicable (shape, alignment
// or workspace); the caller then uses the tile kernels.
template <typename T>
bool launch_gemm_4bit_skinny(int m, int n, int k, const T* A, int lda, const uint8_t* B, int ldb, SkStats st,
                             int blocksize, int blocksize2, const float* code, T* out, int ldc, float* ws,
                             long long ws_bytes) {
  // 33..64 tokens: the split-K tile kernel that shares the token rows across 192 weight rows (gemm4bit_t64.hip); then
  // the whole-K MFMA kernel (gemm4bit_fewtok.hip), unless a lab / test knob selects one of the older kernels
  if (g_fewtoken_kernel == 0 && g_skinny_cfg < 0 &&
      launch_gemm_4bit_t64<T>(m, n, k, A, lda, B, ldb, st, blocksize, blocksize2, code, out, ldc, ws, ws_bytes))
    return true;
  if (g_fewtoken_kernel == 0 && g_skinny_cfg < 0 &&
      launch_gemm_4bit_fewtok<T>(m, n, k, A, lda, B, ldb, st, blocksize, blocksize2, code, out, ldc))
    return true;
  if (launch_gemm_4bit_wk<T>(m, n, k, A, lda, B, ldb, st, blocksize, blocksize2, code, out, ldc)) return true;
  if (!skinny_applicable(m, n, k, lda, ldb, blocksize, A, B)) return false;
  const bool nested = st.q8 != nullptr;
  if (nested && (blocksize2 <= 0 || (blocksize2 & (blocksize2 - 1)))) return false;
  const SkGeom geo = skinny_geometry(m, n, k);
  const int s = geo.splits;
  if (s > 1 && (ws == nullptr || ((uintptr_t)ws & 15) || (long long)s * n * m * (long long)sizeof(float) > ws_bytes))
    return false;
  st.bs_shift = __builtin_ctz(blocksize);
  st.bs2_shift = nested ? __builtin_ctz(blocksize2) : 0;
  const int waves = geo.waves;
  const dim3 grid((unsigned)(((m + 16 * waves - 1) / (16 * waves)) * s));
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(64 * waves), 0, current_stream(), m, n, k, A, lda, B, ldb, st, code, ws, out,
                       ldc, s);
  };
  const int mt = skinny_tiles(n);
  auto dispatch = [&](auto nested_tag) {
    constexpr bool NS = decltype(nested_tag)::value;
    if (geo.cfg == 0) {
      if (mt == 1) go(k_gemm_4bit_skinny<T, 1, skinny_nb<1>(), NS>);
      else if (mt == 2) go(k_gemm_4bit_skinny<T, 2, skinny_nb<2>(), NS>);
      else go(k_gemm_4bit_skinny<T, 4, skinny_nb<4>(), NS>);
    } else if (geo.cfg == 1) {
      if (mt == 1) go(k_gemm_4bit_skinny<T, 1, skinny_nb<1>(), NS, 0, 8>);
      else if (mt == 2) go(k_gemm_4bit_skinny<T, 2, skinny_nb<2>(), NS, 0, 8>);
      else go(k_gemm_4bit_skinny<T, 4, skinny_nb<4>(), NS, 0, 8>);
    } else {
      if (mt == 1) go(k_gemm_4bit_skinny<T, 1, 2 * skinny_nb<1>(), NS, 0, 8>);
      else if (mt == 2) go(k_gemm_4bit_skinny<T, 2, 2 * skinny_nb<2>(), NS, 0, 8>);
      else go(k_gemm_4bit_skinny<T, 4, 2 * skinny_nb<4>(), NS, 0, 8>);
    }
  };
  if (nested) dispatch(std::true_type{});
  else dispatch(std::false_type{});
  if (s > 1) launch_splitk_rows_reduce<T>(ws, s, n, m, out, ldc);
  return true;
}

// out[t, n] = T(sum_s ws[s][t][n]) for any producer of row-major fp32 split partials (the split-K of k_hgemm too)
template <typename T>
void launch_splitk_rows_reduce(const float* ws, int nsplit, int rows, int cols, T* out, int ldc) {
  const long long mn = (long long)rows * cols;
  const dim3 grid((unsigned)((mn / 4 + 255) / 256 + 1));
  if (nsplit <= 2)
    hipLaunchKernelGGL((k_skinny_reduce<T, 2>), grid, dim3(256), 0, current_stream(), ws, nsplit, rows, cols, out, ldc);
  else if (nsplit <= 4)
    hipLaunchKernelGGL((k_skinny_reduce<T, 4>), grid, dim3(256), 0, current_stream(), ws, nsplit, rows, cols, out, ldc);
  else
    hipLaunchKernelGGL((k_skinny_reduce<T, 8>), grid, dim3(256), 0, current_stream(), ws, nsplit, rows, cols, out, ldc);
}
template void launch_splitk_rows_reduce<bf16_t>(const float*, int, int, int, bf16_t*, int);
template void launch_splitk_rows_reduce<fp16_t>(const float*, int, int, int, fp16_t*, int);

template bool launch_gemm_4bit_skinny<bf16_t>(int, int, int, const bf16_t*, int, const uint8_t*, int, SkStats, int, int,
                                              const float*, bf16_t*, int, float*, long long);
template bool launch_gemm_4bit_skinny<fp16_t>(int, int, int, const fp16_t*, int, const uint8_t*, int, SkStats, int, int,
                                              const float*, fp16_t*, int, float*, long long);

}  // namespace bnb

using namespace bnb;

extern "C" {

// [lab, not in the header] A/B knob of the few-token split-K kernel's geometry: -1 = the measured rule (default),
// 0 / 1 / 2 = forced (see g_skinny_cfg)
void cgemm_4bit_set_skinny_config(int cfg) { bnb::g_skinny_cfg = cfg; }

// [additive] few-token 4-bit GEMM with compressed statistics decoded in-kernel (one launch instead of
// the absmax decode + GEMM; functional.py:1346-1350 order).  Returns 0 when launched, 1 when the shape,
// alignment or workspace (cgemm_4bit_workspace_bytes) does not fit this kernel.
int cgemm_4bit_inference_nested_ws_bf16(int m, int n, int k, bf16_t* A, unsigned char* B, unsigned char* absmax_q,
                                        float* code2, float* absmax2, float* offset, float* datatype, bf16_t* out,
                                        int lda, int ldb, int ldc, int blocksize, int blocksize2, float* workspace,
                                        long long workspace_bytes) {
  BNB_RANGE("cgemm_4bit_inference_nested_ws_bf16");
  SkStats st{nullptr, absmax_q, code2, absmax2, offset, 0, 0};
  if (m <= 0 || n <= 0) return 0;
  if (!launch_gemm_4bit_skinny<bf16_t>(m, n, k, A, lda, B, ldb, st, blocksize, blocksize2, datatype, out, ldc,
                                       workspace, workspace_bytes))
    return 1;
  BNB_LAUNCH_CHECK("gemm_4bit_nested");
  return 0;
}
int cgemm_4bit_inference_nested_ws_fp16(int m, int n, int k, fp16_t* A, unsigned char* B, unsigned char* absmax_q,
                                        float* code2, float* absmax2, float* offset, float* datatype, fp16_t* out,
                                        int lda, int ldb, int ldc, int blocksize, int blocksize2, float* workspace,
                                        long long workspace_bytes) {
  BNB_RANGE("cgemm_4bit_inference_nested_ws_fp16");
  SkStats st{nullptr, absmax_q, code2, absmax2, offset, 0, 0};
  if (m <= 0 || n <= 0) return 0;
  if (!launch_gemm_4bit_skinny<fp16_t>(m, n, k, A, lda, B, ldb, st, blocksize, blocksize2, datatype, out, ldc,
                                       workspace, workspace_bytes))
    return 1;
  BNB_LAUNCH_CHECK("gemm_4bit_nested");
  return 0;
}

}  // extern "C"
