// Few-token 4-bit weight GEMM, whole K per workgroup, one launch (batched decode / short prefill, 1..32 activation
// rows) for gfx950.
//
// Slot and semantics: the M > 1 path of cgemm_4bit_inference (ref:sycl/pythonInterface.cpp:377-378), i.e.
// dequantize_4bit + F.linear (ref:python_src_quants/autograd/_functions.py:491-507), in the reference GEMV's
// arithmetic (ref:sycl/sycl_code/kernel_gemm.cpp:1291-1294, 1336-1343: the 16 code values held in T, one absmax per
// block): each weight contributes T(code[q]) * x in the MFMA (exact fp32 products, fp32 sums over the block's 64 k),
// and the block sum is scaled by its fp32 absmax (one fp32 fma per output).  Tolerance class: the GEMV's.
//
// With a few tokens the product is a weight stream (0.5 B per weight, read once).  What sets the time here
// (profiles/lab/r03_fewtok32.txt, ablations of the first form of this kernel):
//   * weight reads in 32-byte pieces of 32 rows per instruction cost ~3 us at 11008 x 4096 against 8 rows x 128 B:
//     the weights therefore move by LDS-DMA in whole 128-B row segments (4 blocks of 64 k; 16-B slots XOR-swizzled
//     by (row >> 1) & 7 through the source address) into a per-wave LDS ring, and each lane reads its MFMA operand
//     bytes from there (ds_read_b64, conflict-free under the swizzle);
//   * every token / statistics load instruction costs time, so a wave covers TWO 16-row weight groups with each token
//     fragment (v_mfma_f32_16x16x32: lane (n, g) = (l & 15, l >> 4) holds k = 64b + 16g + 8s .. +7 of MFMA s = 0, 1,
//     so one 8-B operand read covers exactly one 64-element absmax block b and the block's two MFMAs sum unscaled
//     T(code) x products; the absmax scale is one fma per accumulator after them -- no per-weight multiply or cast);
//   * the table maps a packed byte straight to the MFMA operand dword {T(code[hi]), T(code[lo])} (32 bank-private
//     copies, entry e of copy c at byte 256 e + 4 c: one v_perm_b32 per lookup address);
//   * tokens are the MFMA A operand (rows = tokens) read straight into registers through a buffer resource over rows
//     0..M-1 (lanes of rows >= M get an out-of-range offset: zeros, no memory access, no branch).
// The workgroup (4 waves) owns 16 RG weight rows and all of K; its waves take K in quarters of whole 4-block groups
// (two groups in flight per wave) and the four partial sums meet in LDS in wave order: deterministic, one launch,
// no workspace.
#include "gemm_common.hpp"
#include "gemv_common.hpp"

#include <algorithm>
#include <type_traits>

namespace bnb {

// LDS-DMA of a streamed (read-once) 16-B piece per lane: non-temporal, like the GEMV's weight loads (M0 = the
// wave-uniform LDS base, saved and restored around the statement)
__device__ __forceinline__ void glds16_nt(const void* gsrc, void* lds_base) {
  unsigned keep;
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_base);
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(dst) : "memory");
}

// lab timeline (ABL 128): per wave 8 s_memrealtime stamps (10 ns ticks) at g_ft_tl[(block * 8 + wave) * 8 + i]
__device__ unsigned long long* g_ft_tl = nullptr;
__device__ __forceinline__ unsigned long long ft_now() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

[[maybe_unused]] constexpr int FT_THREADS = 256;
// pair table: entry e of bank-private copy c at byte 256 e + 4 c (32 copies, 64 KiB span) so that a lookup address is
// ONE v_perm_b32 of {packed dword, lane byte}; the nested code map sits in the entry rows' spare upper halves
constexpr int FT_TABLE = 256 * 256;
constexpr int FT_NG = 2;                // 4-block groups in flight per wave

template <typename T> struct FtMfma;
template <> struct FtMfma<bf16_t> {
  __device__ static __forceinline__ f32x4_t mma(const uint4& a, const uint4& b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                   0, 0, 0);
  }
};
template <> struct FtMfma<fp16_t> {
  __device__ static __forceinline__ f32x4_t mma(const uint4& a, const uint4& b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0,
                                                  0, 0);
  }
};

template <int RG, int WAVES> constexpr int ft_lds_bytes() { return FT_TABLE + WAVES * FT_NG * (16 * RG * 128); }
static_assert(ft_lds_bytes<3, 8>() <= 160 * 1024 && ft_lds_bytes<4, 4>() <= 160 * 1024, "LDS budget");

// RG: 16-row weight groups per workgroup (and per wave); MT: 16-token A tiles (1: <= 16 tokens, 2: <= 32).
// S4: blocksize 64 with K % 256 == 0 (and a nested group of >= 4 blocks): the four statistics of a row's group are
// contiguous and aligned, so they arrive as ONE load per row group (plain: float4; nested: 4 codes as a dword + one
// absmax2) instead of one or two per block -- per-block statistics loads were the largest cost of the first form
// (profiles/lab/r03_fewtok32.txt).
// ABL (lab ablations, wrong results, timing only): 1 = no token loads, 2 = no statistics loads, 4 = no table lookups;
// 32 = the weight DMA without the non-temporal hint (correct results); 64 = the weight pieces loaded into registers
// (non-temporal) instead of the ring (its reads see stale data); 128 = per-wave timeline stamps (g_ft_tl, lab).
// WAVES: the workgroup's waves, each a 1 / WAVES share of K (whole 4-block groups); one workgroup per CU.
// X8 (<= 8 tokens, MT 1): the A operand's rows 8..15 are dead, so ONE token load per lane fetches two blocks -- lanes
// t < 8 block b of row t, lanes t >= 8 block b + 1 of row t - 8 -- and block b + 1's fragment is brought down to
// lanes t < 8 by a DPP row rotate (4 v_mov_dpp): half the token load instructions, which the per-CU vector-memory
// issue rate makes worth more than the moves (profiles/lab/r03_fewtok32_timeline.txt).
template <typename T, int RG, int MT, bool NESTED, bool S4, int WAVES, bool X8 = false, int ABL = 0>
__global__ void __launch_bounds__(64 * WAVES, 1)
k_gemm_4bit_fewtok(int N, int M, int K, const T* __restrict__ A, int lda, const uint8_t* __restrict__ B, int ldb,
                   SkStats st, const float* __restrict__ code, T* __restrict__ out, int ldc) {
  constexpr int ROWS = 16 * RG;
  constexpr int GB = ROWS * 128;                            // LDS bytes of one group: ROWS rows x 4 blocks x 32 B
  constexpr int PIECES = ROWS / 8;                          // 1-KiB DMA pieces per group (8 rows x 128 B each)
  constexpr int NV = RG * MT;                               // accumulator tiles per lane
  // VMEM instructions of one group, in issue order: tokens, statistics, then the DMA pieces
  static_assert(!X8 || MT == 1, "X8: one 16-token tile");
  constexpr int GROUP_OPS =
      ((ABL & 1) ? 0 : (X8 ? 2 : 4) * MT * 2) + ((ABL & 2) ? 0 : (S4 ? 1 : 4 * RG) * (NESTED ? 2 : 1)) + PIECES;
  __shared__ __attribute__((aligned(16))) uint8_t sm[ft_lds_bytes<RG, WAVES>()];
  uint8_t* table = sm;
  auto code2s_at = [&](uint32_t t) -> float& { return *reinterpret_cast<float*>(table + 256 * (t >> 5) + 128 + 4 * (t & 31)); };
  uint8_t* ring = sm + FT_TABLE;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 15, g = lane >> 4;
  const int r0 = blockIdx.x * ROWS;
  const int nblk = K >> 6, ngr = (nblk + 3) >> 2;            // 64-k blocks; 4-block groups
  const int g0 = wave * ngr / WAVES, ng = (wave + 1) * ngr / WAVES - g0;   // this wave's groups (may be 0)
  const int rowbytes = K >> 1;
  unsigned long long tl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlw0 = 0, tlw1 = 0, tlw2 = 0;   // group 0 / 1 / 2 landed
  if constexpr ((ABL & 128) != 0) tl[0] = ft_now();

  // ---- table values first (the VMEM counter retires in order)
  const int te = tid & 255;                                 // table entry of this thread (tid < 256 stores it)
  const float code_hi = code[te >> 4], code_lo = code[te & 15];
  float offset = 0.0f, c2v = 0.0f;
  if constexpr (NESTED) {
    c2v = st.code2[te];
    offset = *st.offset;
  }
  asm volatile("" ::: "memory");

  // ---- per-lane sources
  // tokens: A tile mt, lane (t = n, g): row 16 mt + n, elements 64 b + 16 g + 8 s .. +7 (s = 0, 1: 32 contiguous bytes)
  const uint32_t xbytes = (uint32_t)(((long long)(M - 1) * lda + K) * sizeof(T));
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(A), (short)0, (int)xbytes, 0x00020000);
  uint32_t xoff[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    if constexpr (X8) {
      const int t = n & 7;
      xoff[mt] = t < M ? (uint32_t)(((long long)t * lda + 16 * g + 64 * (n >> 3)) * sizeof(T)) : 0x80000000u;
    } else {
      const int t = 16 * mt + n;
      xoff[mt] = t < M ? (uint32_t)(((long long)t * lda + 16 * g) * sizeof(T)) : 0x80000000u;
    }
  }
  // statistics: weight row r0 + 16 rg + n (clamped), element index of block b = 2 ldb row + 64 b
  long long sbase[RG];
#pragma unroll
  for (int rg = 0; rg < RG; ++rg) sbase[rg] = 2LL * ldb * min(r0 + 16 * rg + n, N - 1);
  const long long sbase_l = 2LL * ldb * min(r0 + 16 * min(g, RG - 1) + n, N - 1);   // S4: this lane's row group
  // DMA: piece j of a group = rows 8j .. 8j+7; lane l -> row 8j + (l >> 3), LDS slot l & 7 holding source slot
  // (l & 7) ^ ((row >> 1) & 7); slots past the row's end (the last, partial group) re-read its last slot (never used)
  const uint8_t* wsrc[PIECES];
  int wslot[PIECES];
#pragma unroll
  for (int j = 0; j < PIECES; ++j) {
    const int rr = 8 * j + (lane >> 3);
    wslot[j] = 16 * ((lane & 7) ^ ((rr >> 1) & 7));
    wsrc[j] = B + (long long)min(r0 + rr, N - 1) * ldb;
  }
  uint8_t* my_ring = ring + wave * FT_NG * GB;

  struct Group {
    uint4 x[4][MT][2];
    float am[S4 ? 1 : 4][RG];
    uint32_t q8[S4 ? 1 : 4][RG];
    float a2[S4 ? 1 : 4][RG];
    uint4 wd[(ABL & 64) ? PIECES : 1];                      // (lab ABL 64: the weight pieces in registers)
    // S4: the 4 statistics of row group min(g, RG - 1), row n -- one load per lane for ALL row groups of the wave
    // (lanes g = 0 .. RG-1 each fetch one row group); consume() hands them to the other lanes by ds_bpermute
    float4 am4;
    uint32_t q4;
    float a2g;
  };
  Group gr[FT_NG];
  auto issue = [&](Group& R, int gi, int slot) {            // this wave's group gi into ring slot `slot`
    const int ga = g0 + gi;
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      const int b = min(4 * ga + bb, nblk - 1);
      if constexpr ((ABL & 1) == 0 && X8) {
        if ((bb & 1) == 0) {                               // blocks bb, bb + 1 in one load (rows 0..7 / lanes 8..15)
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(xr, (int)(xoff[0] + (uint32_t)(128 * b + 16 * s)), 0, 0);
            R.x[bb][0][s] = make_uint4(v[0], v[1], v[2], v[3]);
          }
        }
      } else if constexpr ((ABL & 1) == 0) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(xr, (int)(xoff[mt] + (uint32_t)(128 * b + 16 * s)), 0, 0);
            R.x[bb][mt][s] = make_uint4(v[0], v[1], v[2], v[3]);
          }
      } else {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) R.x[bb][mt][0] = R.x[bb][mt][1] = make_uint4(b, mt, 0, 0);
      }
      if constexpr ((ABL & 2) == 0 && !S4) {
#pragma unroll
        for (int rg = 0; rg < RG; ++rg) {
          const long long j = (sbase[rg] + 64LL * b) >> st.bs_shift;
          if constexpr (NESTED) {
            R.q8[bb][rg] = st.q8[j];
            R.a2[bb][rg] = st.absmax2[j >> st.bs2_shift];
          } else {
            R.am[bb][rg] = st.absmax[j];
          }
        }
      } else if constexpr ((ABL & 2) != 0 && !S4) {
#pragma unroll
        for (int rg = 0; rg < RG; ++rg) { R.q8[bb][rg] = 1; R.a2[bb][rg] = 1.f; R.am[bb][rg] = 1.f; }
      }
    }
    if constexpr ((ABL & 2) != 0 && S4) {
      R.q4 = 0x01010101u; R.a2g = 1.f; R.am4 = make_float4(1.f, 1.f, 1.f, 1.f);
    }
    if constexpr ((ABL & 2) == 0 && S4) {                  // the group's 4 statistics of row group min(g, RG-1)
      const long long j0 = (sbase_l >> 6) + 4LL * min(ga, ngr - 1);
      if constexpr (NESTED) {
        R.q4 = *reinterpret_cast<const uint32_t*>(st.q8 + j0);
        R.a2g = st.absmax2[j0 >> st.bs2_shift];
      } else {
        R.am4 = *reinterpret_cast<const float4*>(st.absmax + j0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");      // this slot's previous ring reads are done (WAR)
    const int col = 128 * ga;
#pragma unroll
    for (int j = 0; j < PIECES; ++j) {
      if constexpr ((ABL & 64) != 0) {
        const u32x4_t v = __builtin_nontemporal_load((gvec_p)(wsrc[j] + min(col + wslot[j], rowbytes - 16)));
        R.wd[j] = make_uint4(v.x, v.y, v.z, v.w);
      } else if constexpr ((ABL & 32) != 0) glds16(wsrc[j] + min(col + wslot[j], rowbytes - 16), my_ring + slot * GB + 1024 * j);
      else glds16_nt(wsrc[j] + min(col + wslot[j], rowbytes - 16), my_ring + slot * GB + 1024 * j);
    }
  };
  int nwait = 0;
  auto wait_group = [&](bool next_issued) {                 // the oldest group in flight has landed (DMA included)
    if (next_issued) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GROUP_OPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr ((ABL & 128) != 0) {
      // constant indices only: a dynamic one puts tl[] in scratch, and scratch waves launch late (skews the stamps)
      const unsigned long long now = ft_now();
      tlw0 = nwait == 0 ? now : tlw0;
      tlw1 = nwait == 1 ? now : tlw1;
      tlw2 = nwait == 2 ? now : tlw2;
      ++nwait;
    }
  };

  // both prologue groups unconditionally (clamped: a wave with fewer groups re-reads its last one, never consumed) --
  // a branch here would make hipcc's wait for the table values above conservative (vmcnt(0) behind the stream)
  issue(gr[0], 0, 0);
  issue(gr[1], min(1, max(ng - 1, 0)), 1);
  if constexpr ((ABL & 128) != 0) tl[1] = ft_now();

  // ---- table: thread t writes entry t = {T(code[t >> 4]), T(code[t & 15])} into its 32 copies
  if (tid < 256) {
    const int t = tid;
    const uint32_t v = Dot2<T>::pair(code_hi, code_lo);
#pragma unroll
    for (int k = 0; k < 8; ++k) *reinterpret_cast<uint4*>(table + 256 * t + 16 * ((k + t) & 7)) = make_uint4(v, v, v, v);
    if constexpr (NESTED) code2s_at(t) = c2v;
  }
  __syncthreads();
  if constexpr ((ABL & 128) != 0) tl[2] = ft_now();

  const uint32_t lane4 = (uint32_t)(lane & 31) * 4;
  f32x4_t acc[RG][MT];
#pragma unroll
  for (int rg = 0; rg < RG; ++rg)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[rg][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto consume = [&](Group& R, int gi, int slot) {
    const uint8_t* gs = my_ring + slot * GB;
    // pin this group's register loads here, behind wait_group: otherwise hipcc hoists their first uses (the statistics
    // ds_bpermute) into the previous group's consume, and its wait for them -- the newest loads it can see -- is
    // vmcnt(0), which also drains the DMA pieces issued after them (one group in flight instead of two)
    if constexpr ((ABL & 1) == 0) {
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            if (!X8 || (bb & 1) == 0)
              asm volatile("" : "+v"(R.x[bb][mt][s].x), "+v"(R.x[bb][mt][s].y), "+v"(R.x[bb][mt][s].z), "+v"(R.x[bb][mt][s].w));
    }
    if constexpr ((ABL & 2) == 0 && S4) {
      if constexpr (NESTED) asm volatile("" : "+v"(R.q4), "+v"(R.a2g));
      else asm volatile("" : "+v"(R.am4.x), "+v"(R.am4.y), "+v"(R.am4.z), "+v"(R.am4.w));
    }
    if constexpr ((ABL & 2) == 0 && !S4) {
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
#pragma unroll
        for (int rg = 0; rg < RG; ++rg) {
          if constexpr (NESTED) asm volatile("" : "+v"(R.q8[bb][rg]), "+v"(R.a2[bb][rg]));
          else asm volatile("" : "+v"(R.am[bb][rg]));
        }
    }
    // S4: row group rg's statistics come from lane 16 rg + n (ds_bpermute, one per dword)
    uint32_t q4[S4 ? RG : 1];
    float a2g[S4 ? RG : 1];
    float4 am4[S4 ? RG : 1];
    if constexpr (S4) {
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) {
        const int src = 4 * (16 * rg + n);
        if constexpr (NESTED) {
          q4[rg] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)R.q4);
          a2g[rg] = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, R.a2g)));
        } else {
          am4[rg] = make_float4(__builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, R.am4.x))),
                                __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, R.am4.y))),
                                __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, R.am4.z))),
                                __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, R.am4.w))));
        }
      }
    }
    // this lane's 8 packed bytes of block bb: row 16 rg + n, bytes 32 bb + 8 g .. +7 = 16-B slot 2 bb + (g >> 1);
    // all four blocks' reads up front (S4: the group is always whole, so one basic block and no LDS drain per block)
    uint2 wvg[4][RG];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) {
        const int rr = 16 * rg + n;
        const int slot16 = (2 * bb + (g >> 1)) ^ ((rr >> 1) & 7);
        if (S4 || bb == 0) wvg[bb][rg] = *reinterpret_cast<const uint2*>(gs + rr * 128 + 16 * slot16 + 8 * (g & 1));
      }
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      if (!S4 && 4 * (g0 + gi) + bb >= nblk) break;          // (wave-uniform) the partial last group
      uint2 wv[RG];
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) {
        if constexpr (S4) {
          wv[rg] = wvg[bb][rg];
        } else if (bb == 0) {
          wv[rg] = wvg[0][rg];
        } else {
          const int rr = 16 * rg + n;
          const int slot16 = (2 * bb + (g >> 1)) ^ ((rr >> 1) & 7);
          wv[rg] = *reinterpret_cast<const uint2*>(gs + rr * 128 + 16 * slot16 + 8 * (g & 1));
        }
      }
      // this block's token fragments (X8, odd block: rotated down from the lanes 8..15 of the pair's load)
      uint4 xf[MT][2];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if constexpr (X8 && (ABL & 1) == 0) {
            if (bb & 1) {
              const uint4 u = R.x[bb - 1][mt][s];
              xf[mt][s] = make_uint4(__builtin_amdgcn_mov_dpp(u.x, 0x128, 0xF, 0xF, false),
                                     __builtin_amdgcn_mov_dpp(u.y, 0x128, 0xF, 0xF, false),
                                     __builtin_amdgcn_mov_dpp(u.z, 0x128, 0xF, 0xF, false),
                                     __builtin_amdgcn_mov_dpp(u.w, 0x128, 0xF, 0xF, false));
            } else {
              xf[mt][s] = R.x[bb][mt][s];
            }
          } else {
            xf[mt][s] = R.x[bb][mt][s];
          }
        }
      f32x4_t blk[RG][MT];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int rg = 0; rg < RG; ++rg) {
          uint32_t d = s ? wv[rg].y : wv[rg].x;
          if constexpr ((ABL & 64) != 0) d ^= R.wd[(rg * 2 + s + bb) % PIECES].x;
          uint32_t l[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {                      // byte i -> entry, lane copy -> bank
            if constexpr ((ABL & 4) != 0) l[i] = d + i;
            else l[i] = *reinterpret_cast<const uint32_t*>(table + __builtin_amdgcn_perm(d, lane4, 0x0C0C0000u | ((4u + i) << 8)));
          }
          const uint4 bf = make_uint4(l[0], l[1], l[2], l[3]);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
            blk[rg][mt] = FtMfma<T>::mma(xf[mt][s], bf, s ? blk[rg][mt] : f32x4_t{0.f, 0.f, 0.f, 0.f});
        }
      }
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) {
        float a;
        if constexpr (S4) {
          if constexpr (NESTED) a = __fadd_rn(__fmul_rn(code2s_at((q4[rg] >> (8 * bb)) & 0xFF), a2g[rg]), offset);
          else a = bb == 0 ? am4[rg].x : bb == 1 ? am4[rg].y : bb == 2 ? am4[rg].z : am4[rg].w;
        } else {
          if constexpr (NESTED) a = __fadd_rn(__fmul_rn(code2s_at(R.q8[bb][rg]), R.a2[bb][rg]), offset);
          else a = R.am[bb][rg];
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[rg][mt][i] = __builtin_fmaf(a, blk[rg][mt][i], acc[rg][mt][i]);
      }
    }
  };

  // ---- main loop: group gi in slot gi & 1; group gi + 2 refills that slot once gi is consumed
  int gi = 0;
  for (; gi + 3 < ng; gi += 2) {                            // steady state: both refills in range, no branches
    wait_group(true);
    consume(gr[0], gi, 0);
    issue(gr[0], gi + 2, 0);
    wait_group(true);
    consume(gr[1], gi + 1, 1);
    issue(gr[1], gi + 3, 1);
  }
  // tail: groups gi .. ng - 1 (at most 3), wave-uniform branches
  if (gi < ng) {
    wait_group(gi + 1 < ng);
    consume(gr[0], gi, 0);
    if (gi + 2 < ng) issue(gr[0], gi + 2, 0);
  }
  if (gi + 1 < ng) {
    wait_group(gi + 2 < ng);
    consume(gr[1], gi + 1, 1);
  }
  if (gi + 2 < ng) {
    wait_group(false);
    consume(gr[0], gi + 2, 0);
  }

  if constexpr ((ABL & 128) != 0) tl[6] = ft_now();
  // ---- the WAVES K shares meet in LDS, summed in wave order
  __syncthreads();                                          // every wave is done with the table and its ring
  float* red = reinterpret_cast<float*>(sm);
#pragma unroll
  for (int rg = 0; rg < RG; ++rg)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[((wave * NV + rg * MT + mt) * 4 + i) * 64 + lane] = acc[rg][mt][i];
  __syncthreads();
  // D[4 g + i][n] of tile (rg, mt): token 16 mt + 4 g + i, weight row r0 + 16 rg + n
  for (int v = wave; v < NV * 4; v += WAVES) {
    const int tile = v >> 2, i = v & 3, rg = tile / MT, mt = tile - rg * MT;
    float s = red[v * 64 + lane];
#pragma unroll
    for (int w = 1; w < WAVES; ++w) s += red[(w * NV * 4 + v) * 64 + lane];
    const int t = 16 * mt + 4 * g + i, col = r0 + 16 * rg + n;
    if (t < M && col < N) out[(long long)t * ldc + col] = Io<T>::from_f32(s);
  }
  if constexpr ((ABL & 128) != 0) {
    tl[7] = ft_now();
    tl[3] = tlw0;
    tl[4] = tlw1;
    tl[5] = tlw2;
    if (lane == 0 && g_ft_tl != nullptr)
#pragma unroll
      for (int i = 0; i < 8; ++i) g_ft_tl[((long long)blockIdx.x * WAVES + wave) * 8 + i] = tl[i];
  }
}

// 0 = auto, 1 = off, 2 = forced wherever it fits (A/B knob; tests); >= 16: lab ablations
Knob<int> g_fewtok_mode{0};
extern Knob<int> g_fewtoken_kernel;   // gemm4bit_wk.hip: != 0 selects one of the older few-token kernels
int skinny_cfg_knob();          // gemm4bit_skinny.hip: >= 0 forces a split-K geometry (lab A/B)

bool fewtok_applicable(int m, int n, int k, int lda, int ldb, int blocksize, const void* A, const void* B) {
  return g_fewtok_mode != 1 && n >= 1 && n <= 32 && m >= 1 && k >= 64 && k % 64 == 0 && 2LL * ldb >= k &&
         blocksize >= 64 && (blocksize & (blocksize - 1)) == 0 && lda % 8 == 0 && ldb % 16 == 0 &&
         ((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0 &&
         (long long)(n - 1) * lda * 2 + 2LL * k < 0x7FFFFFFFLL;
}

int fewtok_rows_groups(int m) {                           // RG: 16-row groups per workgroup (one workgroup per CU)
  const int cus = device_cu_count();
  return std::min(4, std::max(1, (m + 16 * cus - 1) / (16 * cus)));
}

// The auto rule (tools/fewtok32_ab.py, profiles/lab/r03_fewtok32.txt; 11008 x 4096 at 8 tokens 17.2 -> 10.2 us,
// 4096 x 4096 10.5 -> 5.9 us, 2..4 rows ahead of the multi-row GEMV): weights of >= 3/4 of a 16-row group per CU;
// at 17..32 tokens only with >= 2 row groups per workgroup (one 16-row group re-reads each token fragment for too few
// weights: 4096 x 11008 at 32 tokens 24.7 vs 21.8 us split-K); at 2..4 tokens not on the 4-wave 64-row form
// (14336 x 4096 at 2 tokens 15.0 vs 12.0 us multi-row GEMV).
bool fewtok_auto_takes(int m, int n, int k) {
  const int cus = device_cu_count(), rg = fewtok_rows_groups(m);
  if (4 * ((m + 15) / 16) < 3 * cus) return false;
  if (n > 16 && rg < 2) return false;
  if (n <= 4 && rg >= 4) return false;
  return true;
}

// m = out features (weight rows), n = tokens, k = in features.  False: not applicable (nothing launched).
template <typename T>
bool launch_gemm_4bit_fewtok(int m, int n, int k, const T* A, int lda, const uint8_t* B, int ldb, SkStats st,
                             int blocksize, int blocksize2, const float* code, T* out, int ldc) {
  if (!fewtok_applicable(m, n, k, lda, ldb, blocksize, A, B)) return false;
  const bool nested = st.q8 != nullptr;
  if (nested && (blocksize2 <= 0 || (blocksize2 & (blocksize2 - 1)))) return false;
  if (g_fewtok_mode == 0 && !fewtok_auto_takes(m, n, k)) return false;
  // one workgroup per CU: RG 16-row groups each, as few as cover the rows in one round (11008 rows: 3 -> 230
  // workgroups); 8 waves (two per SIMD) where the LDS ring allows it, else 4
  const int rg = fewtok_rows_groups(m);
  st.bs_shift = __builtin_ctz(blocksize);
  st.bs2_shift = nested ? __builtin_ctz(blocksize2) : 0;
  const dim3 grid((unsigned)((m + 16 * rg - 1) / (16 * rg)));
  // the 4-statistics-per-load form: blocksize 64, whole 4-block groups per row (K % 256 == 0, so every row's first
  // statistic is 4-aligned), a nested group of >= 4 blocks
  const bool s4 = blocksize == 64 && k % 256 == 0 && (2LL * ldb) % 256 == 0 && (!nested || blocksize2 >= 4);
  auto go = [&](auto kern, int waves) {
    hipLaunchKernelGGL(kern, grid, dim3(64 * waves), 0, current_stream(), m, n, k, A, lda, B, ldb, st, code, out, ldc);
  };
#ifndef BNB_LAB
  if (g_fewtok_mode >= 16) return false;                    // (the ablation kernels exist in the lab build only)
#else
  if (g_fewtok_mode >= 16) {                                // lab ablations: nested, <= 8 tokens, 48-row workgroups
    if (nested && s4 && rg == 3 && n > 16 && n <= 32) {     // (round 6: 17..32 tokens, timeline + ablations)
      switch (g_fewtok_mode - 16) {
        case 128: go(k_gemm_4bit_fewtok<T, 3, 2, true, true, 8, false, 128>, 8); return true;
        case 129: go(k_gemm_4bit_fewtok<T, 3, 2, true, true, 8, false, 129>, 8); return true;
        case 130: go(k_gemm_4bit_fewtok<T, 3, 2, true, true, 8, false, 130>, 8); return true;
        case 132: go(k_gemm_4bit_fewtok<T, 3, 2, true, true, 8, false, 132>, 8); return true;
        case 135: go(k_gemm_4bit_fewtok<T, 3, 2, true, true, 8, false, 135>, 8); return true;
        default: return false;
      }
    }
    if (!nested || n > 8 || !s4) return false;
    constexpr bool X8L = true;
    if (rg == 1) {                                          // (timeline of the 16-row form)
      if (g_fewtok_mode - 16 != 128) return false;
      go(k_gemm_4bit_fewtok<T, 1, 1, true, true, 8, X8L, 128>, 8);
      return true;
    }
    if (rg != 3) return false;
    switch (g_fewtok_mode - 16) {
      case 1: go(k_gemm_4bit_fewtok<T, 3, 1, true, true, 8, X8L, 1>, 8); break;
      case 2: go(k_gemm_4bit_fewtok<T, 3, 1, true, true, 8, X8L, 2>, 8); break;
      case 3: go(k_gemm_4bit_fewtok<T, 3, 1, true, true, 8, X8L, 3>, 8); break;
      case 4: go(k_gemm_4bit_fewtok<T, 3, 1, true, true, 8, X8L, 4>, 8); break;
      case 7: go(k_gemm_4bit_fewtok<T, 3, 1, true, true, 8, X8L, 7>, 8); break;
      case 32: go(k_gemm_4bit_fewtok<T, 3, 1, true, true, 8, X8L, 32>, 8); break;
      case 39: go(k_gemm_4bit_fewtok<T, 3, 1, true, true, 8, X8L, 39>, 8); break;
      case 64: go(k_gemm_4bit_fewtok<T, 3, 1, true, true, 8, X8L, 64>, 8); break;
      case 71: go(k_gemm_4bit_fewtok<T, 3, 1, true, true, 8, X8L, 71>, 8); break;
      case 128: go(k_gemm_4bit_fewtok<T, 3, 1, true, true, 8, X8L, 128>, 8); break;
      case 135: go(k_gemm_4bit_fewtok<T, 3, 1, true, true, 8, X8L, 135>, 8); break;
      case 132: go(k_gemm_4bit_fewtok<T, 3, 1, true, true, 8, X8L, 132>, 8); break;
      case 192: go(k_gemm_4bit_fewtok<T, 3, 1, true, true, 8, X8L, 192>, 8); break;
      case 129: go(k_gemm_4bit_fewtok<T, 3, 1, true, true, 8, X8L, 129>, 8); break;
      default: return false;
    }
    return true;
  }
#endif
  const bool x8 = n <= 8;
  auto by_rg = [&](auto mt_tag, auto nested_tag, auto s4_tag) {
    constexpr int MT = decltype(mt_tag)::value;
    constexpr bool NS = decltype(nested_tag)::value, S = decltype(s4_tag)::value;
    auto go_x8 = [&](auto rg_tag, auto waves_tag) {
      constexpr int R = decltype(rg_tag)::value, W = decltype(waves_tag)::value;
      if constexpr (MT == 1) {
        if (x8) { go(k_gemm_4bit_fewtok<T, R, MT, NS, S, W, true>, W); return; }
      }
      go(k_gemm_4bit_fewtok<T, R, MT, NS, S, W, false>, W);
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    using I8 = std::integral_constant<int, 8>;
    switch (rg) {
      case 1: go_x8(I1{}, I8{}); break;
      case 2: go_x8(I2{}, I8{}); break;
      case 3:   // (17..32 tokens with per-block statistics: 4 waves, 8 would spill)
        if constexpr (MT == 2 && !S) go_x8(I3{}, I4{});
        else go_x8(I3{}, I8{});
        break;
      default: go_x8(I4{}, I4{}); break;
    }
  };
  auto by_s4 = [&](auto mt_tag, auto nested_tag) {
    if (s4) by_rg(mt_tag, nested_tag, std::true_type{});
    else by_rg(mt_tag, nested_tag, std::false_type{});
  };
  auto by_tokens = [&](auto nested_tag) {
    if (n <= 16) by_s4(std::integral_constant<int, 1>{}, nested_tag);
    else by_s4(std::integral_constant<int, 2>{}, nested_tag);
  };
  if (nested) by_tokens(std::true_type{});
  else by_tokens(std::false_type{});
  return true;
}

template bool launch_gemm_4bit_fewtok<bf16_t>(int, int, int, const bf16_t*, int, const uint8_t*, int, SkStats, int, int,
                                              const float*, bf16_t*, int);
template bool launch_gemm_4bit_fewtok<fp16_t>(int, int, int, const fp16_t*, int, const uint8_t*, int, SkStats, int, int,
                                              const float*, fp16_t*, int);

}  // namespace bnb

extern "C" {
#ifdef BNB_LAB
// [lab build only, not in the header] timeline buffer of the ABL-128 variants (mode 16 + 128): 8 stamps per wave
int cgemm_4bit_fewtok_timeline(unsigned long long* buf) {
  BNB_RANGE("cgemm_4bit_fewtok_timeline");
  return hipMemcpyToSymbol(HIP_SYMBOL(bnb::g_ft_tl), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif
// [additive, testing] whole-K few-token kernel: 0 = auto, 1 = off, 2 = wherever it fits (other values: auto; the lab
// build also takes its ablation modes >= 16)
void cgemm_4bit_set_fewtok_mode(int mode) {
#ifdef BNB_LAB
  bnb::g_fewtok_mode = mode;
#else
  bnb::g_fewtok_mode = (mode == 1 || mode == 2) ? mode : 0;
#endif
}
// [additive] 1 when the 4-bit GEMM entry points run the whole-K few-token kernel for out features m, n activation rows,
// in features k and this blocksize (the auto rule above, or the forced mode), else 0 -- the Python layer asks before
// it sends 2..4 rows to the multi-row GEMV
// (the launch's own conditions: a lab mode (>= 16), an older few-token kernel (g_fewtoken_kernel) or a forced split-K
// geometry (g_skinny_cfg) each keep the launch off this kernel, so the answer is 0 for them too)
int cgemm_4bit_fewtok_takes(int m, int n, int k, int blocksize) {
  BNB_RANGE("cgemm_4bit_set_fewtok_mode");
  if (bnb::g_fewtok_mode == 1 || bnb::g_fewtok_mode >= 16 || bnb::g_fewtoken_kernel != 0 || bnb::skinny_cfg_knob() >= 0 ||
      n < 1 || n > 32 || k < 64 || k % 64 || blocksize < 64 || (blocksize & (blocksize - 1)))
    return 0;
  return (bnb::g_fewtok_mode >= 2 || bnb::fewtok_auto_takes(m, n, k)) ? 1 : 0;
}
}
