// 33..64-token 4-bit weight GEMM (batched decode / short prefill) for gfx950: the M > 1 slot of cgemm_4bit_inference
// (ref:sycl/pythonInterface.cpp:377-378), i.e. dequantize_4bit + F.linear (ref:python_src_quants/autograd/
// _functions.py:491-507), in the arithmetic of the whole-K few-token kernel (gemm4bit_fewtok.hip; the reference GEMV's
// T-precision code values, ref:sycl/sycl_code/kernel_gemm.cpp:1291-1294): each weight enters the MFMA as T(code[q]),
// a 64-element block's two MFMAs sum T(code) x products in fp32, and the block sum is scaled by its fp32 absmax (one
// fma per output).  Tolerance class: the GEMV's.
//
// Why a separate kernel from 33 tokens on (round 4; the split-K weight stream k_gemm_4bit_skinny ran 11008 x 4096 at
// 64 tokens in 25.9 us + a 6.6 us reduce, 0.10 of HBM): per CU the traffic of a tile of R weight rows x Kc in-features
// x 64 tokens is 64 Kc x 2 B of tokens (from L2) + R Kc / 2 B of weights + R x 64 x 4 B of fp32 partials per split;
// for the whole product that is N K (128 / R + 512 / Kc) bytes beside the weights, least near R ~ 4 Kc / 16.  The
// skinny kernel runs 64 rows x 384 k (3.3 B of side traffic per weight), the whole-K kernel 48 rows x K (2.8 B, and
// its token fragments for 64 tokens do not fit the registers); here 192 rows x K / 4 at 11008 x 4096 (0.9 B).
//
// Geometry: 4 waves, each 48 weight rows (3 groups of 16) x all 64 tokens (4 MFMA tiles) x the workgroup's K range
// (whole 4-block groups of 256 k; split-K over workgroups, fp32 partials summed in split order by k_skinny_reduce).
// Every operand arrives by LDS-DMA, so the k-loop holds no VGPR-destination load and every wait is an explicit count:
//   tokens   shared by the 4 waves: 2 slots x 16 KiB ([64 tokens][128 k], 16-B slots XOR-swizzled by token row & 15:
//            the A-operand reads of 16 rows at one k are conflict-free), 16 pieces per 2-block half-group, 4 per wave;
//   weights  per wave: 2 slots x 6 KiB (48 rows x 128 B of one 4-block group, slots swizzled by (row >> 1) & 7 as in
//            the whole-K kernel), 6 pieces per group;
//   stats    per wave: 2 slots; plain: the row's 4 block absmax (16 B), nested: its 4 codes (dword) + absmax2;
//   table    {T(code[hi]), T(code[lo])} per packed byte, 32 bank-private copies (the whole-K kernel's layout, one
//            v_perm_b32 per lookup address), the nested code map in the rows' spare halves.
// Per 4-block group g (half-groups 2g, 2g + 1): wait for half-group h's tokens (vmcnt: the pieces issued since -- the
// next half-group's tokens and the next group's weights -- may fly) + barrier; consume its 2 blocks; barrier (every
// wave is done with that token slot); refill the slot with half-group h + 2.  After the second half the wave's
// weight slot is refilled with group g + 2.  Past the last group the refills re-load the last one into slots nobody
// reads (constant counts, no branches); vmcnt(0) before the end.
#include "gemm_common.hpp"
#include "gemv_common.hpp"

#include <algorithm>
#include <type_traits>

namespace bnb {

constexpr int T64_RG = 3, T64_WAVES = 4, T64_THREADS = 64 * T64_WAVES;
constexpr int T64_ROWS = 16 * T64_RG * T64_WAVES;            // 192 weight rows per workgroup
constexpr int T64_TABLE = 256 * 256;
constexpr int T64_TOK = 64 * 256;                            // one token slot: 64 tokens x 128 k
constexpr int T64_WGRP = 16 * T64_RG * 128;                  // one weight slot per wave: 48 rows x 128 B
constexpr int T64_STAT = 1024;                               // one statistics slot per wave
constexpr int T64_OFF_TOK = T64_TABLE;
constexpr int T64_OFF_W = T64_OFF_TOK + 2 * T64_TOK;
constexpr int T64_OFF_S = T64_OFF_W + T64_WAVES * 2 * T64_WGRP;
constexpr int T64_OFF_C2 = T64_OFF_S + T64_WAVES * 2 * T64_STAT;   // nested code map (256 floats)
constexpr int T64_OFF_OFS = T64_OFF_C2 + 1024;                   // the nested offset (64 copies)
constexpr int T64_LDS = T64_OFF_OFS + 256;                       // 153 KiB
constexpr int T64_WPIECES = 16 * T64_RG / 8;                 // 6 weight pieces per wave per group
constexpr int T64_TPIECES = 4;                               // token pieces per wave per half-group
constexpr int T64_STAGE_LD = T64_ROWS + 4;                  // staged partial tile row pitch (floats)
static_assert(64 * T64_STAGE_LD * 4 <= T64_TABLE, "staged tile fits the table");
typedef uint32_t hg_u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t t64_u32x2 __attribute__((ext_vector_type(2)));

template <typename T> struct T64Mfma;
template <> struct T64Mfma<bf16_t> {
  __device__ static __forceinline__ f32x4_t mma(const uint4& a, const uint4& b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                   0, 0, 0);
  }
};
template <> struct T64Mfma<fp16_t> {
  __device__ static __forceinline__ f32x4_t mma(const uint4& a, const uint4& b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0,
                                                  0, 0);
  }
};

// LDS-DMA, scalar base + 32-bit lane offset, M0 = the destination (written here; this kernel uses M0 for nothing else)
template <int BYTES>
__device__ __forceinline__ void t64_dma(const void* sbase, uint32_t voff, uint32_t lds) {
  if constexpr (BYTES == 16)
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" : : "v"(voff), "s"(sbase), "s"(lds) : "memory");
  else
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1" : : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}
template <int BYTES>
__device__ __forceinline__ void t64_dma_nt(const void* sbase, uint32_t voff, uint32_t lds) {
  static_assert(BYTES == 16, "16-B pieces");
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 nt" : : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}

typedef float t64_f32x2_t __attribute__((ext_vector_type(2)));
template <typename T> __device__ __forceinline__ uint32_t t64_cvt2(float a, float b) {   // one RNE cast each
  if constexpr (std::is_same<T, bf16_t>::value)
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((t64_f32x2_t){a, b}, bf16x2_t));
  else
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((t64_f32x2_t){a, b}, f16x2_t));
}

// device-scope (sc1) dword store / loads of the fp32 partials through a buffer resource (element offsets < 2^29)
__device__ __forceinline__ void t64_store_dev(__amdgpu_buffer_rsrc_t r, uint32_t e, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)(4u * e), 0, 16);
}
__device__ __forceinline__ float4 t64_load4_dev(__amdgpu_buffer_rsrc_t r, uint32_t e) {
  // (the whole vector cast: hipcc's bit_cast of one subscripted element of this builtin's result reads element 0)
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(4u * e), 0, 16));
}
__device__ __forceinline__ float t64_load_dev(__amdgpu_buffer_rsrc_t r, uint32_t e) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)(4u * e), 0, 16));
}

// The split-K combine of one row tile (rows row0 .. row0 + 191, every token), run by the row tile's last workgroup to
// finish: out[t][row] = T(ws[0][t][row] + ws[1][t][row] + ... ) -- k_skinny_reduce's additions in its order, so the
// outputs are bit-identical to the two-launch form.
template <typename T, int NT = T64_THREADS>
__device__ __forceinline__ void t64_combine(__amdgpu_buffer_rsrc_t wsr, int ks, int M, int N, int row0,
                                            T* __restrict__ out, int ldc, int tid) {
  const uint32_t mn = (uint32_t)M * (uint32_t)N;
  const int rows = min(T64_ROWS, N - row0);
  if ((N & 3) == 0) {                                        // row0 % 4 == 0 too: whole float4s
    // element e = tid + 256 j (j < 12 covers 64 tokens x 48 float4s): every load of KB splits x 12 elements in
    // flight before the adds -- one round trip per KB splits instead of one per element
    constexpr int EPT = (64 * T64_ROWS / 4) / NT, KB = 4;
    const int per_t = rows >> 2, total = M * per_t;
    const bool st8 = (((uintptr_t)out & 7) == 0) && (ldc & 3) == 0;
    uint32_t off[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int e = min(tid + NT * j, total - 1), t = e / per_t, c = e - t * per_t;
      off[j] = (uint32_t)t * (uint32_t)N + (uint32_t)(row0 + 4 * c);
    }
    float4 s[EPT];
    for (int k0 = 0; k0 < ks; k0 += KB) {
      float4 v[KB][EPT];
#pragma unroll
      for (int b = 0; b < KB; ++b)
#pragma unroll
        for (int j = 0; j < EPT; ++j)
          if (k0 + b < ks) v[b][j] = t64_load4_dev(wsr, (uint32_t)(k0 + b) * mn + off[j]);
#pragma unroll
      for (int b = 0; b < KB; ++b)
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
          if (k0 + b == 0) {
            s[j] = v[0][j];
          } else if (k0 + b < ks) {
            s[j].x += v[b][j].x; s[j].y += v[b][j].y; s[j].z += v[b][j].z; s[j].w += v[b][j].w;
          }
        }
    }
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int e = tid + NT * j;
      if (e >= total) break;
      const int t = e / per_t, c = e - t * per_t;
      T* dst = out + (long long)t * ldc + row0 + 4 * c;
      if (st8) {
        *reinterpret_cast<uint2*>(dst) = make_uint2(t64_cvt2<T>(s[j].x, s[j].y), t64_cvt2<T>(s[j].z, s[j].w));
      } else {
        dst[0] = Io<T>::from_f32(s[j].x); dst[1] = Io<T>::from_f32(s[j].y);
        dst[2] = Io<T>::from_f32(s[j].z); dst[3] = Io<T>::from_f32(s[j].w);
      }
    }
  } else {
    for (int e = tid; e < M * rows; e += NT) {
      const int t = e / rows, r = e - t * rows;
      const uint32_t off = (uint32_t)t * (uint32_t)N + (uint32_t)(row0 + r);
      float s = t64_load_dev(wsr, off);
      for (int k = 1; k < ks; ++k) s += t64_load_dev(wsr, (uint32_t)k * mn + off);
      out[(long long)t * ldc + row0 + r] = Io<T>::from_f32(s);
    }
  }
}

// lab timeline (ABL 512): per wave 8 s_memrealtime stamps (10 ns ticks) at g_t64_tl[(block * waves + wave) * 8 + i]:
// start, prologue issued, table built, first half-group landed, loop done, DMA drained, outputs issued, outputs landed
__device__ unsigned long long* g_t64_tl = nullptr;
__device__ __forceinline__ unsigned long long t64_now() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// N = out features (weight rows), M = tokens (1..64), K = in features (% 256 == 0), blocksize 64.  Workgroup
// (row tile rt, split sp): rows rt * 192 .., groups [sp * kc, min((sp + 1) * kc, K / 256)).  ksplit > 1: fp32
// partials ws[sp][token][row], combined by the row tile's last workgroup when `tickets` is given (one counter per row
// tile, zero between launches), else by k_skinny_reduce after the launch; ksplit == 1: the outputs.
// ABL (lab ablations, timing only): 1 = no vmcnt waits, 2 = no token DMA after the prologue, 4 = no weight DMA after
// the prologue, 8 = no MFMAs, 16 = no table lookups, 32 = no output / partial stores, 64 = no table build, 128 = no
// barriers in the loop, 256 = no token fragment reads
// KP (round 5): waves per 48-row set.  KP = 1: the round-4 kernel, 4 waves (one per SIMD), each wave both blocks of every
// 2-block half-group.  KP = 2: 8 waves (two per SIMD), the waves w and w + 4 of a row set take the half-group's first and
// second block -- the same LDS slots, DMA pieces split between them, half the registers each -- so one wave's VALU (the
// table lookups, the per-block absmax fmas) and LDS reads run beside the other's MFMAs; the two partial sums of a row
// set meet in LDS at the end (first + second, fixed order: deterministic).
template <typename T, bool NESTED, int ABL = 0, int KP = 1>
__global__ void __launch_bounds__(T64_THREADS * KP, KP)
k_gemm_4bit_t64(int N, int M, int K, const T* __restrict__ A, int lda, const uint8_t* __restrict__ B, int ldb,
                SkStats st, const float* __restrict__ code, T* __restrict__ out, int ldc, float* __restrict__ ws,
                int ksplit, int kc, uint32_t* __restrict__ tickets, int pstore) {
  static_assert(KP == 1 || KP == 2, "one or two waves per row set");
  constexpr int NT = T64_THREADS * KP;                       // threads of the workgroup
  constexpr int WPW = T64_WPIECES / KP;                      // weight pieces of a group issued by each wave of the set
  constexpr int WOPS = (NESTED ? 2 : 1) + WPW;               // VMEM instructions of one weight-group issue (per wave)
  constexpr int TOPS = T64_TPIECES / KP;                     // ... of one token half-group issue
  constexpr int NB2 = 2 / KP;                                // blocks of a half-group this wave consumes
  __shared__ __attribute__((aligned(16))) uint8_t sm[T64_LDS];
  uint8_t* table = sm;
  auto code2s_at = [&](uint32_t t) -> const float& { return *reinterpret_cast<const float*>(sm + T64_OFF_C2 + 4 * t); };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rs = wave & 3, kp = wave >> 2;                   // row set, k part (KP = 1: rs = wave, kp = 0)
  const int n = lane & 15, g = lane >> 4;
  const int bid = blockIdx.x, rt = bid / ksplit, sp = bid - rt * ksplit;
  const int r0 = rt * T64_ROWS + rs * 16 * T64_RG;           // this wave's first weight row
  const int ngr = K >> 8, gr0 = sp * kc, ng = min(kc, ngr - gr0);   // this workgroup's groups (>= 1, host rule)

  constexpr bool TL = (ABL & 512) != 0;
  unsigned long long tl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if constexpr (TL) tl[0] = t64_now();
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)sm);
  // token pieces: this wave's pieces q = 4 wave + i of a half-group slot; lane l -> token row t = 4 q + (l >> 4),
  // physical 16-B slot p = l & 15 holding logical slot p ^ (t & 15) (k = 8 x logical slot within the 128 k)
  uint32_t toff[TOPS];
#pragma unroll
  for (int i = 0; i < TOPS; ++i) {
    const int q = TOPS * wave + i, t = 4 * q + (lane >> 4), p = lane & 15;
    toff[i] = (uint32_t)min(t, M - 1) * (uint32_t)lda * 2u + 16u * (uint32_t)(p ^ (t & 15));
  }
  // weight pieces: piece j = rows 8 j .. 8 j + 7 of the wave's 48; lane l -> row 8 j + (l >> 3), LDS slot l & 7 holding
  // source slot (l & 7) ^ ((row >> 1) & 7)
  // (KP = 2: the pieces 3 kp .. 3 kp + 2 of the set's 6)
  uint32_t woff[WPW];
#pragma unroll
  for (int jj = 0; jj < WPW; ++jj) {
    const int j = WPW * kp + jj, rr = 8 * j + (lane >> 3);
    woff[jj] = (uint32_t)min(r0 + rr, N - 1) * (uint32_t)ldb + 16u * (uint32_t)((lane & 7) ^ ((rr >> 1) & 7));
  }
  // statistics: lane l -> the wave's row min(l, 47); its first block index (bs = 64: 2 ldb row / 64)
  const uint32_t sblk0 = (uint32_t)((2LL * ldb * min(r0 + min(lane, 16 * T64_RG - 1), N - 1)) >> 6);
  const uint32_t tok_lds = lds0 + T64_OFF_TOK;
  const uint32_t w_lds = lds0 + T64_OFF_W + rs * 2 * T64_WGRP;
  const uint32_t s_lds = lds0 + T64_OFF_S + rs * 2 * T64_STAT;

  auto issue_w = [&](int gi, int slot) {                     // weight group gi (clamped) -> this wave's slot
    if constexpr ((ABL & 4) != 0) if (gi >= 2) return;
    const int G = gr0 + min(gi, ng - 1);
    const uint32_t j0 = sblk0 + 4u * (uint32_t)G;
    if constexpr (NESTED) {
      t64_dma<4>(st.q8, j0, s_lds + slot * T64_STAT);
      t64_dma<4>(st.absmax2, 4u * (j0 >> st.bs2_shift), s_lds + slot * T64_STAT + 256);
    } else {
      t64_dma<16>(st.absmax, 4u * j0, s_lds + slot * T64_STAT);
    }
    // (both waves of a row set load its statistics: the same words into the same slot, so every wave's VMEM count per
    // group is the same constant)
    const uint8_t* src = B + 128LL * G;
#pragma unroll
    for (int jj = 0; jj < WPW; ++jj) t64_dma_nt<16>(src, woff[jj], w_lds + slot * T64_WGRP + 1024 * (WPW * kp + jj));
  };
  auto issue_t = [&](int hi, int slot) {                     // token half-group hi (clamped) -> token slot
    if constexpr ((ABL & 2) != 0) if (hi >= 2) return;
    const int h = min(hi, 2 * ng - 1);
    const T* src = A + 64LL * (4 * gr0 + 2 * h);             // k0 = 64 x (first block of the half-group)
#pragma unroll
    for (int i = 0; i < TOPS; ++i) t64_dma<16>(src, toff[i], tok_lds + slot * T64_TOK + 1024 * (TOPS * wave + i));
  };

  f32x4_t acc[T64_RG][4];
#pragma unroll
  for (int rg = 0; rg < T64_RG; ++rg)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[rg][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const uint32_t lane4 = (uint32_t)(lane & 31) * 4;

  // consume the 2 blocks of half-group `half` (0 / 1) of group gi: tokens from token slot `half`, weights and statistics
  // from slot gi & 1
  auto consume = [&](int gi, int half) {
    // One wave per SIMD: nothing else hides an LDS round trip, so every read of the half-group is issued before any
    // is used -- token fragments of both blocks, the weight words and statistics of all row groups, then all table
    // lookups -- and only then the 48 MFMAs (one basic block; hipcc waits on lgkmcnt just before each first use).
    // (KP = 2: only block kp of the half-group -- b2 below runs over this wave's NB2 blocks, bk = its block index)
    const int ws_slot = gi & 1;
    const uint8_t* tk = sm + T64_OFF_TOK + half * T64_TOK;
    const uint8_t* wr = sm + T64_OFF_W + (rs * 2 + ws_slot) * T64_WGRP;
    const uint8_t* sr = sm + T64_OFF_S + (rs * 2 + ws_slot) * T64_STAT;
    auto bk = [&](int b2) { return KP == 2 ? kp : b2; };
    uint2 wv[NB2][T64_RG];
    uint32_t q4[T64_RG];
    float a2[T64_RG], a[NB2][T64_RG];
#pragma unroll
    for (int rg = 0; rg < T64_RG; ++rg) {
      const int rr = 16 * rg + n;
#pragma unroll
      for (int b2 = 0; b2 < NB2; ++b2) {
        const int slot16 = (2 * (2 * half + bk(b2)) + (g >> 1)) ^ ((rr >> 1) & 7);
        wv[b2][rg] = *reinterpret_cast<const uint2*>(wr + rr * 128 + 16 * slot16 + 8 * (g & 1));
      }
      if constexpr (NESTED) {
        q4[rg] = *reinterpret_cast<const uint32_t*>(sr + 4 * rr);
        a2[rg] = *reinterpret_cast<const float*>(sr + 256 + 4 * rr);
      } else {
#pragma unroll
        for (int b2 = 0; b2 < NB2; ++b2) a[b2][rg] = *reinterpret_cast<const float*>(sr + 16 * rr + 4 * (2 * half + bk(b2)));
      }
    }
    uint4 xf[NB2][4][2];                                     // tokens: A tile mt, lane (t = n, g): row 16 mt + n
#pragma unroll
    for (int b2 = 0; b2 < NB2; ++b2)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int ls = 8 * bk(b2) + 2 * g + s;             // logical 16-B slot: k 64 b2 + 16 g + 8 s
          if constexpr ((ABL & 256) != 0) xf[b2][mt][s] = make_uint4(ls, mt, n, 0);
          else xf[b2][mt][s] = *reinterpret_cast<const uint4*>(tk + (16 * mt + n) * 256 + 16 * (ls ^ n));
        }
    if constexpr (NESTED) {
      const float offset = *reinterpret_cast<const float*>(sm + T64_OFF_OFS + 4 * (lane & 63));
#pragma unroll
      for (int rg = 0; rg < T64_RG; ++rg)
#pragma unroll
        for (int b2 = 0; b2 < NB2; ++b2)
          a[b2][rg] = __fadd_rn(__fmul_rn(code2s_at((q4[rg] >> (8 * (2 * half + bk(b2)))) & 0xFF), a2[rg]), offset);
    }
    uint4 bf[NB2][T64_RG][2];                                // weight operands: byte i of the word -> entry, lane copy
#pragma unroll
    for (int b2 = 0; b2 < NB2; ++b2)
#pragma unroll
      for (int rg = 0; rg < T64_RG; ++rg)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const uint32_t d = s ? wv[b2][rg].y : wv[b2][rg].x;
          uint32_t l[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if constexpr ((ABL & 16) != 0) l[i] = d + i;
            else l[i] = *reinterpret_cast<const uint32_t*>(table + __builtin_amdgcn_perm(d, lane4, 0x0C0C0000u | ((4u + i) << 8)));
          }
          bf[b2][rg][s] = make_uint4(l[0], l[1], l[2], l[3]);
        }
#pragma unroll
    for (int b2 = 0; b2 < NB2; ++b2)
#pragma unroll
      for (int rg = 0; rg < T64_RG; ++rg) {
        f32x4_t blk[4];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            if constexpr ((ABL & 8) != 0) {
              const f32x4_t z = s ? blk[mt] : f32x4_t{0.f, 0.f, 0.f, 0.f};
              blk[mt] = z + f32x4_t{__uint_as_float(xf[b2][mt][s].x ^ bf[b2][rg][s].x), 0.f, 0.f, 0.f};
            } else {
              blk[mt] = T64Mfma<T>::mma(xf[b2][mt][s], bf[b2][rg][s], s ? blk[mt] : f32x4_t{0.f, 0.f, 0.f, 0.f});
            }
          }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[rg][mt][i] = __builtin_fmaf(a[b2][rg], blk[mt][i], acc[rg][mt][i]);
      }
  };

  // ---- prologue: [code map], W(0), T(0), T(1), W(1) -- the steady state's order (at each wait the ops younger than
  // the awaited token half-group are exactly the next half-group's tokens and one weight group; the code map is older)
  if constexpr (NESTED) {
    // (the offset too: a plain load of it would be a VMEM load hipcc waits for with vmcnt(0) -- inside the loop, where
    // it drained every in-flight piece each group)
    if (wave < 4) t64_dma<4>(st.code2, 4u * (uint32_t)(64 * wave + lane), lds0 + T64_OFF_C2 + 256 * wave);
    if (wave == 0) t64_dma<4>(st.offset, 0u, lds0 + T64_OFF_OFS);
  }
  issue_w(0, 0);
  issue_t(0, 0);
  issue_t(1, 1);
  issue_w(1, 1);
  if constexpr (TL) tl[1] = t64_now();
  // ---- the pair table, built while the prologue's DMA is in flight (code values by scalar loads: lgkmcnt, not the
  // vmcnt the DMA counts; the nested code map travels by LDS-DMA with the first pieces)
  if constexpr ((ABL & 64) == 0) {
    float dt[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) dt[j] = code[j];
    float hi = dt[0], lo = dt[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) {
      hi = ((tid & 255) >> 4) == j ? dt[j] : hi;
      lo = (tid & 15) == j ? dt[j] : lo;
    }
    const uint32_t v = Dot2<T>::pair(hi, lo);
    // (KP = 2: threads 256.. write the same entries' other halves: entry tid & 255, copies 4 (tid >> 8) .. + 3)
#pragma unroll
    for (int k = 0; k < 8 / KP; ++k) {
      const int e = tid & 255, kk = k + (8 / KP) * (tid >> 8);
      *reinterpret_cast<uint4*>(table + 256 * e + 16 * ((kk + e) & 7)) = make_uint4(v, v, v, v);
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);                      // lgkmcnt(0): the table is written (barrier at the wait)
  if constexpr (TL) tl[2] = t64_now();

  for (int gi = 0; gi < ng; ++gi) {
    if constexpr ((ABL & 1) == 0)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(TOPS + WOPS) : "memory");   // T(2 gi) and W(gi) landed (this wave)
    if constexpr ((ABL & 128) == 0) __builtin_amdgcn_s_barrier();                                          // ... every wave's token pieces
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (TL) tl[3] = gi == 0 ? t64_now() : tl[3];
    consume(gi, 0);
    __builtin_amdgcn_s_waitcnt(0xC07F);                                    // lgkmcnt(0): this wave's reads are done
    if constexpr ((ABL & 128) == 0) __builtin_amdgcn_s_barrier();                                          // ... every wave's: token slot 0 is free
    __builtin_amdgcn_sched_barrier(0);
    issue_t(2 * gi + 2, 0);
    if constexpr ((ABL & 1) == 0)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(TOPS + WOPS) : "memory");   // T(2 gi + 1) landed
    if constexpr ((ABL & 128) == 0) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    consume(gi, 1);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if constexpr ((ABL & 128) == 0) __builtin_amdgcn_s_barrier();                                          // token slot 1 and this wave's weight slot
    __builtin_amdgcn_sched_barrier(0);                                     // are free
    issue_t(2 * gi + 3, 1);
    issue_w(gi + 2, gi & 1);
  }
  if constexpr (TL) tl[4] = t64_now();
  wait_vmcnt0();                                                           // no LDS-DMA may outlive the workgroup
  if constexpr (TL) tl[5] = t64_now();

  // ---- KP = 2: the second wave of each row set hands its partial sums to the first through LDS (the table region, free
  // once every wave is past its last lookup); the first adds them (first + second) and does the stores below
  if constexpr (KP == 2) {
    float* pb = reinterpret_cast<float*>(sm);                // 4 sets x 48 rows x 64 tokens x 4 B = 48 KiB
    __syncthreads();
    if (kp == 1) {
#pragma unroll
      for (int rg = 0; rg < T64_RG; ++rg)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int i = 0; i < 4; ++i) pb[(((rs * T64_RG + rg) * 4 + mt) * 4 + i) * 64 + lane] = acc[rg][mt][i];
    }
    __syncthreads();
    if (kp == 0) {
#pragma unroll
      for (int rg = 0; rg < T64_RG; ++rg)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[rg][mt][i] = acc[rg][mt][i] + pb[(((rs * T64_RG + rg) * 4 + mt) * 4 + i) * 64 + lane];
    }
  }
  const bool storer = KP == 1 || kp == 0;                   // (wave-uniform) the waves that hold the summed tile

  // ---- outputs: acc[rg][mt][i] = token 16 mt + 4 g + i, weight row r0 + 16 rg + n (ABL 32: stored only where the
  // value is an impossible one -- the computation stays live, the stores go).  A whole tile (64 tokens, 192 rows in
  // range) stores unpredicated from a wave-uniform base per (token tile, i) plus one 32-bit lane offset; edge tiles
  // check every element.
  const bool whole = M == 64 && rt * T64_ROWS + T64_ROWS <= N;
  const __amdgpu_buffer_rsrc_t wsr = __builtin_amdgcn_make_buffer_rsrc(ws, (short)0, 0x7FFFFFFF, 0x00020000);
  // partial stores: 0 plain, 1 device-scope (sc1) dwords, 2 device-scope 16-B lines staged through LDS (the combine
  // needs device scope; for the reduce launch it only saves the boundary's write-back of dirty lines)
  const int wt = tickets != nullptr ? 2 : pstore;
  if (whole && (ABL & 32) == 0) {
    const uint32_t loff = (uint32_t)(4 * g) * (uint32_t)N + (uint32_t)(r0 + n);
    if (ksplit > 1 && wt == 2 && (N & 3) == 0) {
      // device-scope stores (the combine reads them), whole lines: the tile through LDS ([token][row], rows padded to
      // 196 floats: the 4 token rows of one write are 2-way on the banks) then 16-B stores, each wave's 1 KiB contiguous
      float* stage = reinterpret_cast<float*>(sm);             // the table: every wave is past its last lookup
      __syncthreads();
      const int wr0 = rs * 16 * T64_RG;
      if (storer) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int rg = 0; rg < T64_RG; ++rg) stage[(16 * mt + 4 * g + i) * T64_STAGE_LD + wr0 + 16 * rg + n] = acc[rg][mt][i];
      }
      __syncthreads();
      const uint32_t b0 = (uint32_t)sp * 64u * (uint32_t)N + (uint32_t)(rt * T64_ROWS);
#pragma unroll
      for (int j = 0; j < (64 * T64_ROWS / 4) / NT; ++j) {
        const int e = tid + NT * j, t = e / (T64_ROWS / 4), c = e - t * (T64_ROWS / 4);
        const float4 v = *reinterpret_cast<const float4*>(stage + t * T64_STAGE_LD + 4 * c);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(hg_u32x4, v), wsr, (int)(4u * (b0 + (uint32_t)t * (uint32_t)N + 4u * c)), 0, 16);
      }
    } else if (!storer) {
    } else if (ksplit > 1 && wt != 0) {
      const uint32_t b0 = (uint32_t)sp * 64u * (uint32_t)N + loff;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int rg = 0; rg < T64_RG; ++rg)
            t64_store_dev(wsr, b0 + (uint32_t)(16 * mt + i) * (uint32_t)N + 16u * rg, acc[rg][mt][i]);
    } else if (ksplit > 1) {
      float* wsb = ws + (long long)sp * 64 * N;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float* p = wsb + (long long)(16 * mt + i) * N;
#pragma unroll
          for (int rg = 0; rg < T64_RG; ++rg) p[loff + 16 * rg] = acc[rg][mt][i];
        }
    } else {
      const uint32_t loo = (uint32_t)(4 * g) * (uint32_t)ldc + (uint32_t)(r0 + n);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          T* p = out + (long long)(16 * mt + i) * ldc;
#pragma unroll
          for (int rg = 0; rg < T64_RG; ++rg) p[loo + 16 * rg] = Io<T>::from_f32(acc[rg][mt][i]);
        }
    }
  } else if (storer) {
#pragma unroll
    for (int rg = 0; rg < T64_RG; ++rg) {
      const int row = r0 + 16 * rg + n;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int t = 16 * mt + 4 * g + i;
          const bool go = (ABL & 32) ? acc[rg][mt][i] == 1.2345e30f : true;
          if (go && t < M && row < N) {
            if (ksplit > 1 && wt != 0) t64_store_dev(wsr, ((uint32_t)sp * (uint32_t)M + t) * (uint32_t)N + row, acc[rg][mt][i]);
            else if (ksplit > 1) ws[((long long)sp * M + t) * N + row] = acc[rg][mt][i];
            else out[(long long)t * ldc + row] = Io<T>::from_f32(acc[rg][mt][i]);
          }
        }
    }
  }

  if constexpr (TL) {
    tl[6] = t64_now();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tl[7] = t64_now();
    if (lane == 0 && g_t64_tl != nullptr)
#pragma unroll
      for (int i = 0; i < 8; ++i) g_t64_tl[((long long)blockIdx.x * (NT / 64) + wave) * 8 + i] = tl[i];
  }

  // ---- split-K combine by the row tile's last workgroup to finish.  Hand-off (the condition the round-2
  // combine missed): the partials are device-scope stores (sc1: coherent across the XCDs' L2s without a cache-wide
  // write-back), every wave waits for its own to complete (vmcnt(0)), a barrier, then one device-scope ticket per
  // workgroup; the last arriver reads the partials with device-scope loads.  No workgroup waits for another (nothing
  // spins), and no L2 write-back / invalidate runs (those, as agent fences, cost 35-55 us here: every wave's write-back
  // plus the invalidate evicting the tokens of the workgroups still running).  The last arriver resets the ticket.
  if (tickets != nullptr && ksplit > 1 && (ABL & 32) == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    volatile uint32_t* last = reinterpret_cast<volatile uint32_t*>(sm);   // the table: no DMA is in flight any more
    // (the ticket is acquire-release at agent scope and the last arriver's waves take an agent acquire before reading:
    // the hand-off then rests on the memory model, not only on the sc1 cache policy of the partial stores and loads --
    // ADVICE r4; opt-in path, so its cost (a cache-wide write-back / invalidate per workgroup) is accepted)
    if (tid == 0)
      last[0] = __hip_atomic_fetch_add(&tickets[rt], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                (uint32_t)(ksplit - 1) ? 1u : 0u;
    __syncthreads();
    if (last[0] == 0u) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    t64_combine<T, NT>(wsr, ksplit, M, N, rt * T64_ROWS, out, ldc, tid);
    if (tid == 0) __hip_atomic_store(&tickets[rt], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- The register-fed form (round 5, k_gemm_4bit_t64r): 48 weight rows per workgroup over the WHOLE K, its 4 waves
// splitting K (wave w: groups [w kc, (w + 1) kc)), every operand loaded straight into VGPRs.
// Why: the LDS-DMA form above is bound by its in-flight depth -- per CU ~40 KiB in flight in 2-slot LDS rings beside
// the 64 KiB pair table, a 4-wave barrier per half-group, a reduce launch for the split-K partials (per-wave timeline,
// profiles/lab/r05_t64_timeline.txt: 9.6 us of loop for 224 KiB per CU, then 5 us of reduce).  Here each wave keeps
// T64R_D blocks of tokens and weights in flight in its own registers (one wave per SIMD: 512 registers), no barrier
// runs in the loop, and the K-parts meet in LDS at the end ((p0 + p1) + p2 + p3 -- k_skinny_reduce's order: with the
// same group split the outputs equal the LDS-DMA form + reduce launch bit for bit).  The price: every workgroup reads
// all token rows (64 x K x 2 B from L2 per 48 weight rows), so the form needs ~one workgroup per CU from its row tiles
// alone (host rule).  Arithmetic per block as above: T(code) pairs from the bank-private table into the MFMA, the
// block's two MFMAs summed in fp32, scaled by the block absmax (one fma per output).
constexpr int T64R_RG = 3, T64R_ROWS = 16 * T64R_RG, T64R_D = 4;   // rows per workgroup, blocks in flight per wave
constexpr int T64R_PITCH = T64R_ROWS + 4;                  // combine: floats per token row (conflict-free writes)
constexpr int T64R_OFF_C2 = T64_TABLE;                      // nested code map (256 floats)
constexpr int T64R_LDS = T64R_OFF_C2 + 1024;
static_assert(4 * 64 * T64R_PITCH * 4 <= T64_TABLE, "the four K-part tiles fit the table region");

template <typename T, bool NESTED>
__global__ void __launch_bounds__(256, 1)
k_gemm_4bit_t64r(int N, int M, int K, const T* __restrict__ A, int lda, const uint8_t* __restrict__ B, int ldb,
                 SkStats st, const float* __restrict__ code, T* __restrict__ out, int ldc, int kc) {
  __shared__ __attribute__((aligned(16))) uint8_t sm[T64R_LDS];
  uint8_t* table = sm;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 15, g = lane >> 4;
  const int r0 = blockIdx.x * T64R_ROWS;
  const int ngr = K >> 8, gr0 = min(wave * kc, ngr), ng = min(kc, ngr - gr0);   // this wave's groups (0 for idle parts)
  const int parts = (ngr + kc - 1) / kc;                     // K-parts holding a partial sum
  const int nb = 4 * ng;                                     // this wave's blocks

  // tokens: tile mt, lane (n, g) -> token min(16 mt + n, M - 1), k 16 g + 8 s of each block (16 B per s)
  uint32_t toff[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) toff[mt] = (uint32_t)min(16 * mt + n, M - 1) * (uint32_t)lda * 2u + 32u * (uint32_t)g;
  // weights: row group rg, lane (n, g) -> row min(r0 + 16 rg + n, N - 1), bytes 8 g .. 8 g + 7 of each block's 32
  uint32_t woff[T64R_RG], sblk[T64R_RG];
#pragma unroll
  for (int rg = 0; rg < T64R_RG; ++rg) {
    const uint32_t row = (uint32_t)min(r0 + 16 * rg + n, N - 1);
    woff[rg] = row * (uint32_t)ldb + 8u * (uint32_t)g;
    sblk[rg] = (uint32_t)(((unsigned long long)row * (unsigned long long)ldb) >> 5);   // the row's first block
  }
  const uint8_t* Ab = reinterpret_cast<const uint8_t*>(A);
  uint4 tb[T64R_D][4][2];
  t64_u32x2 wb[T64R_D][T64R_RG];
  auto issue = [&](int bi, auto dtag) {                      // block bi (clamped) of this wave -> ring slot d
    constexpr int d = decltype(dtag)::value;
    const long long kb = 4LL * gr0 + min(bi, max(nb - 1, 0));
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int s = 0; s < 2; ++s) tb[d][mt][s] = *reinterpret_cast<const uint4*>(Ab + 128LL * kb + toff[mt] + 16 * s);
#pragma unroll
    for (int rg = 0; rg < T64R_RG; ++rg)
      wb[d][rg] = __builtin_nontemporal_load(reinterpret_cast<const t64_u32x2*>(B + 32LL * kb + woff[rg]));
  };
  // statistics of group gi (clamped): nested -- the 4 block codes (one dword) and the absmax2 of each row; plain -- the
  // 4 block absmax
  uint32_t q4[T64R_RG], q4n[T64R_RG];
  float a2[T64R_RG], a2n[T64R_RG];
  float4 am[T64R_RG], amn[T64R_RG];
  auto stats = [&](int gi, uint32_t* q, float* a2v, float4* amv) {
    const uint32_t G = (uint32_t)(gr0 + min(gi, max(ng - 1, 0)));
#pragma unroll
    for (int rg = 0; rg < T64R_RG; ++rg) {
      const uint32_t j0 = sblk[rg] + 4u * G;
      if constexpr (NESTED) {
        q[rg] = *reinterpret_cast<const uint32_t*>(st.q8 + j0);
        a2v[rg] = st.absmax2[j0 >> st.bs2_shift];
      } else {
        amv[rg] = *reinterpret_cast<const float4*>(st.absmax + j0);
      }
    }
  };

  // (the nested code map and offset first: loaded after the ring, their first use would wait for the whole ring)
  float offset = 0.f;
  if constexpr (NESTED) {
    offset = *st.offset;
    reinterpret_cast<float*>(sm + T64R_OFF_C2)[tid] = st.code2[tid];
  }
  static_assert(T64R_D == 4, "one ring slot per block of a 4-block group");
  if (nb > 0) {
    issue(0, std::integral_constant<int, 0>{});
    issue(1, std::integral_constant<int, 1>{});
    issue(2, std::integral_constant<int, 2>{});
    issue(3, std::integral_constant<int, 3>{});
    stats(0, q4, a2, am);
  }
  // the pair table {T(code[hi]), T(code[lo])} per packed byte, 32 bank-private copies (the LDS-DMA form's layout)
  {
    float dt[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) dt[j] = code[j];
    float hi = dt[0], lo = dt[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) {
      hi = (tid >> 4) == j ? dt[j] : hi;
      lo = (tid & 15) == j ? dt[j] : lo;
    }
    const uint32_t v = Dot2<T>::pair(hi, lo);
#pragma unroll
    for (int k = 0; k < 8; ++k) *reinterpret_cast<uint4*>(table + 256 * tid + 16 * ((k + tid) & 7)) = make_uint4(v, v, v, v);
  }
  __syncthreads();
  const float* code2s = reinterpret_cast<const float*>(sm + T64R_OFF_C2);

  f32x4_t acc[T64R_RG][4];
#pragma unroll
  for (int rg = 0; rg < T64R_RG; ++rg)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[rg][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const uint32_t lane4 = (uint32_t)(lane & 31) * 4;

  auto consume = [&](auto dtag) {                             // block d of the current group, from ring slot d
    constexpr int d = decltype(dtag)::value;
    float a[T64R_RG];
#pragma unroll
    for (int rg = 0; rg < T64R_RG; ++rg) {
      if constexpr (NESTED) a[rg] = __fadd_rn(__fmul_rn(code2s[(q4[rg] >> (8 * d)) & 0xFF], a2[rg]), offset);
      else a[rg] = d == 0 ? am[rg].x : d == 1 ? am[rg].y : d == 2 ? am[rg].z : am[rg].w;
    }
    uint4 bf[T64R_RG][2];
#pragma unroll
    for (int rg = 0; rg < T64R_RG; ++rg)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint32_t w = s ? wb[d][rg].y : wb[d][rg].x;
        uint32_t l[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          l[i] = *reinterpret_cast<const uint32_t*>(table + __builtin_amdgcn_perm(w, lane4, 0x0C0C0000u | ((4u + i) << 8)));
        bf[rg][s] = make_uint4(l[0], l[1], l[2], l[3]);
      }
#pragma unroll
    for (int rg = 0; rg < T64R_RG; ++rg) {
      f32x4_t blk[4];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          blk[mt] = T64Mfma<T>::mma(tb[d][mt][s], bf[rg][s], s ? blk[mt] : f32x4_t{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[rg][mt][i] = __builtin_fmaf(a[rg], blk[mt][i], acc[rg][mt][i]);
    }
  };

  for (int gi = 0; gi < ng; ++gi) {
    stats(gi + 1, q4n, a2n, amn);                              // the next group's statistics ride with this group
    const int b0 = 4 * gi + T64R_D;
    consume(std::integral_constant<int, 0>{});
    issue(b0 + 0, std::integral_constant<int, 0>{});
    consume(std::integral_constant<int, 1>{});
    issue(b0 + 1, std::integral_constant<int, 1>{});
    consume(std::integral_constant<int, 2>{});
    issue(b0 + 2, std::integral_constant<int, 2>{});
    consume(std::integral_constant<int, 3>{});
    issue(b0 + 3, std::integral_constant<int, 3>{});
#pragma unroll
    for (int rg = 0; rg < T64R_RG; ++rg) {
      q4[rg] = q4n[rg];
      a2[rg] = a2n[rg];
      am[rg] = amn[rg];
    }
  }

  // ---- the K-parts meet in LDS (the table region: every wave is past its last lookup), then ((p0 + p1) + p2) + p3
  __syncthreads();
  float* pb = reinterpret_cast<float*>(sm);
  if (wave < parts) {
    float* pw = pb + wave * 64 * T64R_PITCH;
#pragma unroll
    for (int rg = 0; rg < T64R_RG; ++rg)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) pw[(16 * mt + 4 * g + i) * T64R_PITCH + 16 * rg + n] = acc[rg][mt][i];
  }
  __syncthreads();
  constexpr int C4 = T64R_ROWS / 4;                           // float4 columns of a token row
  const bool vec = (((uintptr_t)out & 7) == 0) && (ldc & 3) == 0;
#pragma unroll
  for (int j = 0; j < (64 * C4) / 256; ++j) {
    const int e = tid + 256 * j, t = e / C4, c = e - t * C4;
    if (t >= M) continue;
    float4 s = *reinterpret_cast<const float4*>(pb + t * T64R_PITCH + 4 * c);
    for (int p = 1; p < parts; ++p) {
      const float4 v = *reinterpret_cast<const float4*>(pb + (p * 64 + t) * T64R_PITCH + 4 * c);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    const int row = r0 + 4 * c;
    T* dst = out + (long long)t * ldc + row;
    if (vec && row + 3 < N) {
      *reinterpret_cast<uint2*>(dst) = make_uint2(t64_cvt2<T>(s.x, s.y), t64_cvt2<T>(s.z, s.w));
    } else {
      if (row < N) dst[0] = Io<T>::from_f32(s.x);
      if (row + 1 < N) dst[1] = Io<T>::from_f32(s.y);
      if (row + 2 < N) dst[2] = Io<T>::from_f32(s.z);
      if (row + 3 < N) dst[3] = Io<T>::from_f32(s.w);
    }
  }
}

// One ticket per row tile, in T64_TICKET_SETS sets handed out round-robin to launches, so launches in flight on
// different streams at the same time do not share counters (every counter is back at zero when its launch ends).
constexpr int T64_MAX_TILES = 1024, T64_TICKET_SETS = 16;
__device__ uint32_t g_t64_tickets[T64_TICKET_SETS * T64_MAX_TILES];

// 0 = auto (33..64 tokens), 1 = off, 2 = forced wherever it applies (1..64 tokens; tests / A-B)
Knob<int> g_t64_mode{0};
Knob<int> g_t64_ks{0};                                            // lab: force the split count (0 = the rule)
// 1: in-kernel last-arriver combine, 0 (default): k_skinny_reduce.  Measured (tools/t64_time.py,
// profiles/lab/r04_t64.txt): 11008 x 4096 at 64 rows 25.7 us in-kernel vs 22.6 us with the reduce launch -- the combine
// of a row tile is one workgroup reading 192 KiB of device-scope partials (8.6 us of tail on 58 CUs), the reduce
// launch spreads the same reads over ~700 workgroups for 5.7 us
Knob<int> g_t64_combine{0};
// partial-store policy (cgemm_4bit_set_t64_pstore): 2 = write-through 16-B lines by default -- the reduce launch's
// boundary then has no dirty partials to write back (11008 x 4096 at 64 rows 22.9 -> 21.8 us, 4096 x 11008 24.7 ->
// 22.3, 4096^2 19.0 -> 15.5; write-through dwords within 0.2 us of the lines; profiles/lab/r04_t64.txt)
Knob<int> g_t64_pstore{2};
// waves per 48-row set (cgemm_4bit_set_t64_waves): 1 = the round-4 4-wave kernel, 2 = 8 waves, two per SIMD (round 5),
// 0 = auto: 8 waves up to 48 tokens or where K is not split, 4 otherwise (round 5, 11008 x 4096 nested, graph replay over
// 14 copies: 33 / 48 / 64 rows 20.13 / 21.37 / 21.77 us on 4 waves vs 18.92 / 20.47 / 22.28 on 8, profiles/lab/r05_ab.txt;
// unsplit 28672 x 8192 at 64 rows 76.4 -> 72.0 us, profiles/lab/r05_t64r_ab.txt)
Knob<int> g_t64_kp{0};

// this launch's ticket set on the current device (nullptr: use the reduce launch).  Never during HIP-graph capture: a
// captured launch would bake one ticket set into the graph, and its replays could then share counters with eager
// launches handed the same set -- captured work always takes the reduce launch.
static uint32_t* t64_tickets(int row_tiles, long long partial_bytes) {
  if (!g_t64_combine || row_tiles > T64_MAX_TILES || partial_bytes > 0x7FFFFFFFLL) return nullptr;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(current_stream(), &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return nullptr;
  }
  static uint32_t* base[64] = {};
  static unsigned next[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (base[dev] == nullptr) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_t64_tickets)) != hipSuccess) return nullptr;
    base[dev] = static_cast<uint32_t*>(p);
  }
  return base[dev] + (next[dev]++ % T64_TICKET_SETS) * T64_MAX_TILES;
}

struct T64Geom {
  int row_tiles, ksplit, kc;
};
static T64Geom t64_geometry(int m, int k) {
  const int rt = (m + T64_ROWS - 1) / T64_ROWS, ngr = k / 256;
  int cus = device_cu_count();
  if (cus <= 0) cus = 256;
  int ks = std::max(1, std::min(ngr, cus / std::max(1, rt)));   // one round of workgroups on the CUs
  if (g_t64_ks > 0) ks = std::min(ngr, g_t64_ks.load());
  const int kc = (ngr + ks - 1) / ks;
  ks = (ngr + kc - 1) / kc;
  return {rt, ks, kc};
}

bool t64_applicable(int m, int n, int k, int lda, int ldb, int blocksize, int blocksize2, bool nested, const void* A,
                    const void* B) {
  if (g_t64_mode == 1) return false;
  if (n < 1 || n > 64 || ((g_t64_mode == 0 || g_t64_mode >= 16) && n < 33)) return false;
  return m >= 1 && k >= 256 && k % 256 == 0 && blocksize == 64 && 2LL * ldb >= k && ldb % 128 == 0 &&
         lda % 8 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0 &&
         (!nested || (blocksize2 >= 4 && (blocksize2 & (blocksize2 - 1)) == 0)) &&
         (long long)(m - 1) * ldb + k / 2 < 0xFFFFFFFFLL && (long long)(n - 1) * lda * 2 + 2LL * k < 0x7FFFFFFFLL;
}

// the register-fed form (k_gemm_4bit_t64r): 1 (default) = off, 2 = wherever the 33..64-token kernel applies, 0 = auto
// (where its row tiles alone fill >= 3/4 of the CUs).  Off by default: measured 1.4-2.8x slower than the LDS-DMA form +
// reduce on every shape, growing with the token rows -- every workgroup pulls all 64 x K token values through its
// vector-memory path, 4x the LDS-DMA form's 64 x K/4 (profiles/lab/r05_t64r_ab.txt; a rotated group order per workgroup,
// against L2-channel camping of the 16 same-channel token rows of one load, changed nothing)
Knob<int> g_t64r{1};
static bool t64r_route(int m, int k, const SkStats& st, bool nested) {
  if (g_t64r == 1 || g_t64_mode >= 15) return false;         // (the LDS-DMA form's labs keep their kernel)
  if (nested ? ((uintptr_t)st.q8 & 3) != 0 : ((uintptr_t)st.absmax & 15) != 0) return false;
  if (g_t64r == 2) return true;
  int cus = device_cu_count();
  if (cus <= 0) cus = 256;
  return 4LL * ((m + T64R_ROWS - 1) / T64R_ROWS) >= 3LL * cus;
}

long long t64_workspace_bytes(int m, int n, int k) {
  if (n < 1 || n > 64 || k < 256 || k % 256) return 0;
  const T64Geom geo = t64_geometry(m, k);
  return geo.ksplit > 1 ? (long long)geo.ksplit * n * m * (long long)sizeof(float) : 0;
}

// m = out features (weight rows), n = tokens, k = in features.  False: not applicable (nothing launched).
template <typename T>
bool launch_gemm_4bit_t64(int m, int n, int k, const T* A, int lda, const uint8_t* B, int ldb, SkStats st,
                          int blocksize, int blocksize2, const float* code, T* out, int ldc, float* ws,
                          long long ws_bytes) {
  const bool nested = st.q8 != nullptr;
  if (!t64_applicable(m, n, k, lda, ldb, blocksize, blocksize2, nested, A, B)) return false;
  if (t64r_route(m, k, st, nested)) {
    const int kc = (k / 256 + 3) / 4;
    const dim3 grid((unsigned)((m + T64R_ROWS - 1) / T64R_ROWS));
    st.bs_shift = 6;
    st.bs2_shift = nested ? __builtin_ctz(blocksize2) : 0;
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, grid, dim3(256), 0, current_stream(), m, n, k, A, lda, B, ldb, st, code, out, ldc, kc);
    };
    if (nested) go(k_gemm_4bit_t64r<T, true>);
    else go(k_gemm_4bit_t64r<T, false>);
    return true;
  }
  const T64Geom geo = t64_geometry(m, k);
  if (geo.ksplit > 1 &&
      (ws == nullptr || ((uintptr_t)ws & 15) || (long long)geo.ksplit * n * m * (long long)sizeof(float) > ws_bytes))
    return false;
  st.bs_shift = 6;
  st.bs2_shift = nested ? __builtin_ctz(blocksize2) : 0;
  const dim3 grid((unsigned)(geo.row_tiles * geo.ksplit));
  uint32_t* tickets = geo.ksplit > 1 && g_t64_mode != 15 ? t64_tickets(geo.row_tiles, (long long)geo.ksplit * n * m * 4) : nullptr;
  const int pstore = (long long)geo.ksplit * n * m * 4 <= 0x7FFFFFFFLL ? g_t64_pstore.load() : 0;
  auto lab = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(T64_THREADS), 0, current_stream(), m, n, k, A, lda, B, ldb, st, code, out, ldc, ws,
                       geo.ksplit, geo.kc, tickets, pstore);
  };
#ifdef BNB_LAB
  if (g_t64_mode >= 16 && nested) {                          // lab ablations (nested bf16 / fp16 only)
    switch (g_t64_mode - 16) {
      case 1: lab(k_gemm_4bit_t64<T, true, 1>); break;
      case 2: lab(k_gemm_4bit_t64<T, true, 2>); break;
      case 4: lab(k_gemm_4bit_t64<T, true, 4>); break;
      case 6: lab(k_gemm_4bit_t64<T, true, 6>); break;
      case 8: lab(k_gemm_4bit_t64<T, true, 8>); break;
      case 16: lab(k_gemm_4bit_t64<T, true, 16>); break;
      case 24: lab(k_gemm_4bit_t64<T, true, 24>); break;
      case 30: lab(k_gemm_4bit_t64<T, true, 30>); break;
      case 32: lab(k_gemm_4bit_t64<T, true, 32>); break;
      case 15: lab(k_gemm_4bit_t64<T, true>); break;
      case 64: lab(k_gemm_4bit_t64<T, true, 64>); break;
      case 128: lab(k_gemm_4bit_t64<T, true, 128>); break;
      case 256: lab(k_gemm_4bit_t64<T, true, 256>); break;
      case 512: lab(k_gemm_4bit_t64<T, true, 512>); break;
      case 30 + 32 + 64 + 128 + 256: lab(k_gemm_4bit_t64<T, true, 30 + 32 + 64 + 128 + 256>); break;
      default: lab(k_gemm_4bit_t64<T, true>); break;
    }
  } else
#else
  (void)lab;
#endif
  if (g_t64_kp == 2 || (g_t64_kp == 0 && (n <= 48 || geo.ksplit == 1))) {
    if (nested)
      hipLaunchKernelGGL((k_gemm_4bit_t64<T, true, 0, 2>), grid, dim3(2 * T64_THREADS), 0, current_stream(), m, n, k, A,
                         lda, B, ldb, st, code, out, ldc, ws, geo.ksplit, geo.kc, tickets, pstore);
    else
      hipLaunchKernelGGL((k_gemm_4bit_t64<T, false, 0, 2>), grid, dim3(2 * T64_THREADS), 0, current_stream(), m, n, k, A,
                         lda, B, ldb, st, code, out, ldc, ws, geo.ksplit, geo.kc, tickets, pstore);
  } else if (nested)
    hipLaunchKernelGGL((k_gemm_4bit_t64<T, true>), grid, dim3(T64_THREADS), 0, current_stream(), m, n, k, A, lda, B, ldb,
                       st, code, out, ldc, ws, geo.ksplit, geo.kc, tickets, pstore);
  else
    hipLaunchKernelGGL((k_gemm_4bit_t64<T, false>), grid, dim3(T64_THREADS), 0, current_stream(), m, n, k, A, lda, B,
                       ldb, st, code, out, ldc, ws, geo.ksplit, geo.kc, tickets, pstore);
  if (geo.ksplit > 1 && g_t64_mode != 15 && tickets == nullptr)
    launch_splitk_rows_reduce<T>(ws, geo.ksplit, n, m, out, ldc);
  return true;
}

template bool launch_gemm_4bit_t64<bf16_t>(int, int, int, const bf16_t*, int, const uint8_t*, int, SkStats, int, int,
                                           const float*, bf16_t*, int, float*, long long);
template bool launch_gemm_4bit_t64<fp16_t>(int, int, int, const fp16_t*, int, const uint8_t*, int, SkStats, int, int,
                                           const float*, fp16_t*, int, float*, long long);

}  // namespace bnb

extern "C" {
// [additive, testing] the 33..64-token kernel's split-K count: ks > 0 forces it (tests of the combine and of ragged
// splits; same results within the GEMM tolerance, bit-identical across the combine forms), 0 = the rule; returns the
// previous setting
int cgemm_4bit_set_t64_splits(int ks) {
  const int prev = bnb::g_t64_ks;
  bnb::g_t64_ks = ks;
  return prev;
}
// [additive, testing] split-K combine of the 33..64-token kernel: 1 = in the kernel (last workgroup of each row tile),
// 0 (default) = the separate reduce launch; returns the previous setting
// [additive, testing] partial-store policy of that kernel's split-K: 0 plain, 1 write-through dwords, 2 (default)
// write-through 16-B lines staged through LDS; returns the previous setting
int cgemm_4bit_set_t64_pstore(int p) {
  const int prev = bnb::g_t64_pstore;
  bnb::g_t64_pstore = p;
  return prev;
}
// [additive, testing] waves per 48-row set of the 33..64-token kernel: 1 = 4 waves (one per SIMD), 2 = 8 waves (two per
// SIMD; round 5), 0 = auto (8 waves up to 48 tokens); returns the previous setting
int cgemm_4bit_set_t64_waves(int kp) {
  const int prev = bnb::g_t64_kp;
  bnb::g_t64_kp = kp == 2 ? 2 : kp == 1 ? 1 : 0;
  return prev;
}
#ifdef BNB_LAB
// [lab build only, not in the header] timeline buffer of the ABL-512 variant (mode 16 + 512): 8 stamps per wave
int cgemm_4bit_t64_timeline(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(bnb::g_t64_tl), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif
// [additive, testing] the register-fed 33..64-token form: 0 = auto, 1 = off, 2 = wherever the kernel applies; returns the
// previous setting
int cgemm_4bit_set_t64_regfed(int v) {
  const int prev = bnb::g_t64r;
  bnb::g_t64r = (v == 1 || v == 2) ? v : 0;
  return prev;
}
int cgemm_4bit_set_t64_combine(int on) {
  const int prev = bnb::g_t64_combine;
  bnb::g_t64_combine = on ? 1 : 0;
  return prev;
}
// [additive, testing] the 33..64-token kernel (gemm4bit_t64.hip): 0 = auto, 1 = off, 2 = wherever it applies (1..64
// tokens; other values: auto -- the lab build also takes its ablation modes >= 15); returns the previous setting
int cgemm_4bit_set_t64_mode(int mode) {
  BNB_RANGE("cgemm_4bit_set_t64_mode");
  const int prev = bnb::g_t64_mode;
#ifdef BNB_LAB
  bnb::g_t64_mode = mode;
#else
  bnb::g_t64_mode = (mode == 1 || mode == 2) ? mode : 0;
#endif
  return prev;
}
}
