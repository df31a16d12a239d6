// Hand-written bf16 / fp16 GEMM for gfx950, C[m][n] = sum_k A[m][k] * B[n][k] (both operands k-contiguous,
// the F.linear shape).  It is the GEMM half of the large-prefill NF4 path: the reference dequantises the
// 4-bit weight and calls F.linear (ref:python_src_quants/autograd/_functions.py:507, MatMul4Bit.forward);
// here k_dequantize_4bit_stream writes the weight once and this kernel multiplies it (no vendor GEMM).
//
// Geometry (the shape a tuned library GEMM uses on this chip): 256 x 256 output tile, BK = 64, FOUR waves
// (256 threads, one wave per SIMD, one workgroup per CU), each wave 128 x 128 outputs = 8 x 8 accumulators of
// v_mfma_f32_16x16x32 (256 accumulator registers).  Every fragment read from LDS feeds 8 MFMAs, so a k32 step
// is 16 ds_read_b128 per 64 MFMAs -- a third fewer LDS bytes per MFMA than the 8-wave 128 x 64 split
// (MI355X_MICROARCH.md 'DVFS give-back': LDS read bytes cost clock).
//
// Pipeline (round 4 default, V & 8192: see tile3 below -- three barriers per k-tile, each operand's DMA issued as soon
// as its rows of the stage are free; the two-half form described next is the round-3 schedule, kept as an A/B arm):
// two LDS stages of 64 KiB (A and B tiles [256][64], 16-B slots XOR-swizzled by (row >> 1) & 7 through
// the DMA source address, conflict-free for the fragment reads).  Both operands move by LDS-DMA
// (global_load_lds_dwordx4, scalar base + one 32-bit lane offset per piece, so ragged edges are clamped once in
// the offsets and a k-step advances only the scalar base).  Per k-tile t, two halves:
//   half 1: the 64 MFMAs of k32 step 0 (fragments already in registers) while this wave reads step 1's fragments;
//           lgkmcnt(0) + barrier: every wave is done with stage t & 1;
//   half 2: DMA of tile t+2 into that stage, interleaved with step 1's MFMAs; vmcnt(16) (tile t+1 landed) +
//           barrier; tile t+1's step-0 fragments read under the remaining MFMAs.
// The DMA of a tile is therefore in flight for a whole k-tile (~2k MFMA cycles), and no vmcnt(0) drain sits in
// the loop (cdna_hip_programming.md §5 'Pipelining across barriers').
#include "gemm_common.hpp"
#include "int8_common.hpp"

#include <algorithm>
#include <type_traits>
#include <utility>

namespace bnb {

constexpr int HG_BM = 256, HG_BN = 256, HG_BK = 64, HG_THREADS = 256;
constexpr int HG_TILE = HG_BM * HG_BK * 2;        // 32 KiB per operand per stage
constexpr int HG_STAGE = 2 * HG_TILE;             // A + B
constexpr int HG_LDS_MAIN = 2 * HG_STAGE;         // 128 KiB
// epilogue staging of 16-bit outputs: per wave 128 rows x 256 B, rows padded to 272 B (16-B aligned; the 8-B
// fragment writes of 16 consecutive rows then hit 2 banks each, 2-way at most)
constexpr int HG_EPI_PITCH = 272;
constexpr int HG_LDS_EPI = 4 * 128 * HG_EPI_PITCH;   // 136 KiB
[[maybe_unused]] constexpr int HG_LDS = HG_LDS_MAIN > HG_LDS_EPI ? HG_LDS_MAIN : HG_LDS_EPI;

// LDS-DMA with a scalar base: lane address = sbase + voff (unsigned 32-bit), 16 B per lane to lds + 16 * lane.
// M0 (the LDS destination) is written and restored inside the statement (it is compiler-reserved).
__device__ __forceinline__ void glds16_sv(const void* sbase, uint32_t voff, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds)
               : "memory");
}

typedef float hg_f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 hg_bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 hg_f16x2_t __attribute__((ext_vector_type(2)));
// {T(lo), T(hi)}: one RNE conversion each (v_cvt_pk_bf16_f32 / v_cvt_pkrtz is NOT used for fp16: RNE per element)
template <typename T> __device__ __forceinline__ uint32_t cvt_pk(float lo, float hi);
template <> __device__ __forceinline__ uint32_t cvt_pk<bf16_t>(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((hg_f32x2_t){lo, hi}, hg_bf16x2_t));
}
template <> __device__ __forceinline__ uint32_t cvt_pk<fp16_t>(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((hg_f32x2_t){lo, hi}, hg_f16x2_t));
}

// The MFMA is issued from inline asm with the accumulator pinned to AGPRs ("+a") and the fragments to VGPRs ("v"):
// with the builtin, hipcc's allocator treats both as either-file operands and, at 256 accumulator registers, shuffles
// them between the files every iteration (v_accvgpr_read/write/mov).  What the asm hides from hipcc is handled here:
// the fragment reads are ordinary LDS loads (hipcc waits on lgkmcnt before the statement that reads them), each
// accumulator is re-read 63 MFMAs after it was written, and the epilogue pads the MFMA -> accvgpr_read hazard itself.
//
// Operation kinds (one kernel body; the tile is 128 BYTES of k per row either way, and both MFMA shapes take 16
// consecutive bytes of k per lane: A[row l & 15][bytes 16 (l >> 4) ..] -- 8 bf16 / fp16 or 16 int8):
//   HG_BF16, HG_FP16   v_mfma_f32_16x16x32_{bf16,f16}, fp32 accumulators, one RNE rounding to T at the end
//   HG_I8_DEQ          v_mfma_i32_16x16x64_i8, exact int32, the fused mm_dequant epilogue to fp16
//                      (igemmlt + dequant_mm_int32_fp16, ref:sycl/sycl_code/kernel_quant.cpp:3969 order)
//   HG_I8_I32          the same product stored as int32 (igemmlt's row-major int32 C)
enum HgOp { HG_BF16 = 0, HG_FP16 = 1, HG_I8_DEQ = 2, HG_I8_I32 = 3 };
typedef unsigned hg_u32x4_t __attribute__((ext_vector_type(4)));
typedef int hg_i32x4_t __attribute__((ext_vector_type(4)));
template <int OP> struct HgOpT;
template <> struct HgOpT<HG_BF16> {
  typedef f32x4_t acc_t;
  static constexpr int ELEM = 2;
  __device__ static __forceinline__ acc_t mma(const hg_u32x4_t& a, const hg_u32x4_t& b, acc_t c) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
    return c;
  }
  __device__ static __forceinline__ acc_t mma0(const hg_u32x4_t& a, const hg_u32x4_t& b) {
    acc_t c;
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
    return c;
  }
};
template <> struct HgOpT<HG_FP16> {
  typedef f32x4_t acc_t;
  static constexpr int ELEM = 2;
  __device__ static __forceinline__ acc_t mma(const hg_u32x4_t& a, const hg_u32x4_t& b, acc_t c) {
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
    return c;
  }
  __device__ static __forceinline__ acc_t mma0(const hg_u32x4_t& a, const hg_u32x4_t& b) {
    acc_t c;
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
    return c;
  }
};
struct HgOpI8 {
  typedef hg_i32x4_t acc_t;
  static constexpr int ELEM = 1;
  __device__ static __forceinline__ acc_t mma(const hg_u32x4_t& a, const hg_u32x4_t& b, acc_t c) {
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
    return c;
  }
  __device__ static __forceinline__ acc_t mma0(const hg_u32x4_t& a, const hg_u32x4_t& b) {
    acc_t c;
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
    return c;
  }
};
template <> struct HgOpT<HG_I8_DEQ> : HgOpI8 {};
template <> struct HgOpT<HG_I8_I32> : HgOpI8 {};

// The same without saving / restoring M0: valid only in a kernel whose code uses M0 for nothing else (k_hgemm: no
// LDS-DMA builtin, no s_sendmsg / movrel / LDS-parameter access -- `grep m0` of its .s shows only these statements).
// The s_nop 0 is the M0-write -> LDS-DMA wait state.
__device__ __forceinline__ void glds16_sv_m0(const void* sbase, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" : : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}

// Chained form: M0 already holds this piece's LDS address (set >= 1 instruction earlier); afterwards it is advanced by
// `step` for the next piece, which must follow at least one other instruction later (the M0 -> LDS-DMA wait state).
template <int STEP>
__device__ __forceinline__ void glds16_chain(const void* sbase, uint32_t voff) {
  asm volatile("global_load_lds_dwordx4 %0, %1\n\ts_add_u32 m0, m0, %2" : : "v"(voff), "s"(sbase), "i"(STEP) : "memory");
}
__device__ __forceinline__ void hg_set_m0(uint32_t lds) { asm volatile("s_mov_b32 m0, %0" : : "s"(lds) : "memory"); }

// HG_DMA_BUF (round-6 A/B build switch): the LDS-DMA pieces as MUBUF `buffer_load_dwordx4 ... offen lds` (a buffer
// resource over the operand, the k-tile's byte offset in soffset, the same per-piece VGPR offsets) instead of the
// FLAT-encoded `global_load_lds_dwordx4`.  Same bytes to the same LDS slots, bit-identical outputs -- and 2.5-3.4 %
// slower (metric shape 230.0 -> 237.1 us, 4096^3 90.4 -> 93.5, int8 121.9 -> 124.9; tools/r06_hg_variant.sh,
// profiles/lab/r06_hg_dma_buf_ab.json), so the library keeps the FLAT form (0).
#ifndef HG_DMA_BUF
#define HG_DMA_BUF 0
#endif
typedef int hg_rsrc_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ hg_rsrc_t hg_rsrc(const void* base) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  // dword1: base[47:32], stride 0; dword2: num_records (no range check in practice: the offsets stay < 4 GiB);
  // dword3: the raw-buffer word of common.hpp's loads (DATA_FORMAT 32)
  hg_rsrc_t r = {(int)(uint32_t)a, (int)((uint32_t)(a >> 32) & 0xFFFFu), -1, 0x00020000};
  r[0] = __builtin_amdgcn_readfirstlane(r[0]);
  r[1] = __builtin_amdgcn_readfirstlane(r[1]);
  return r;
}
template <int STEP>
__device__ __forceinline__ void glds16_chain_buf(hg_rsrc_t rsrc, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds\n\ts_add_u32 m0, m0, %3" : : "v"(voff), "s"(rsrc), "s"(soff), "i"(STEP)
               : "memory");
}
__device__ __forceinline__ void glds16_buf_m0(hg_rsrc_t rsrc, uint32_t voff, uint32_t soff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" : : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds)
               : "memory");
}

__device__ __forceinline__ int hg_swz(int r, int s) { return r * 128 + ((s ^ ((r >> 1) & 7)) << 4); }

// one dword per lane by LDS-DMA (lane l -> lds + 4 l), scalar base + 32-bit lane offset, M0 written here
__device__ __forceinline__ void glds4_sv_m0(const void* sbase, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1" : : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}

// mm_dequant of two adjacent outputs of one row on packed fp32 (v_pk_mul_f32 / v_pk_add_f32: each lane's two
// elements rounded exactly as mm_dequant_value's scalar ops -- same operation order, one RNE per op), then one packed
// RNE cast to fp16: {fp16(lo), fp16(hi)}
__device__ __forceinline__ uint32_t mm_dequant_pair(int32_t a0, int32_t a1, float rs, float cs0, float cs1, float b0,
                                                    float b1) {
  hg_f32x2_t v = {(float)a0, (float)a1};
  v = v * (hg_f32x2_t){6.200012e-05f, 6.200012e-05f};
  v = v * (hg_f32x2_t){rs, rs};
  v = v * (hg_f32x2_t){cs0, cs1};
  asm volatile("" : "+v"(v));                          // (no fma / fma_mix folding across the barriers)
  v = v + (hg_f32x2_t){b0, b1};
  asm volatile("" : "+v"(v));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, hg_f16x2_t));
}

// V: schedule variant bits (A/B arms of tools/hgemm_lab.hip; HG_V is the launched one):
//   1 = step-1 fragment reads all after half 1's MFMAs, 2 = no sched_barrier fences in half 2,
//   4 = next-step fragments read in MFMA-need order, 8 = DMA spread (8 pieces before the wait, 8 after, one per
//   4 MFMAs; 1.6 PFLOP/s vs 1.44 for 0 at 4096 x 4096 x 11008, profiles/lab/r03_hgemm_variants.txt), 16 = LDS-DMA
//   without the M0 save / restore (another 2-3 %, profiles/lab/r03_hgemm_dma_variants.txt), 32 = 12 pieces before
//   the wait (no gain), 4096 = M0 chained from piece to piece (one s_add per piece instead of s_add + s_mov + s_nop:
//   another 2-3 %, profiles/lab/r03_hgemm_m0_chain.txt).  Lab-only ablations (wrong results, timing only): 64 = no
//   vmcnt wait, 128 / 256 = no barrier B2 / B1, 512 = register-staged copies (slower: 256 vs 242 us), 1024 = no
//   copies, 2048 = no fragment re-reads (profiles/lab/r03_hgemm_ablation.txt).  Launched: 8 + 16 + 4096.
// Round 4: the three-barrier operand-split schedule (V & 8192, tile3 below) is the launched one: bit-identical to the
// two-half schedule and 0.8-1.5 % faster at 4096 x 4096 x 11008 (bf16 234.6-235.3 vs 236.6-238.6 us; int8 4-wave
// 127.3-129.3 vs 128.7-129.3 us; tools/hgemm_variant_ab.py, profiles/lab/r04_hgemm_variants.txt).  The round-3
// two-half schedule is no longer launched (round 6): its compiled loop carried accumulator copies between the asm MFMAs
// (the note "The round-3 two-half schedule ..." below); the code stays for tools/hgemm_lab.hip.
constexpr int HG_V = 16 + 8192;
// variant bit: the full-tile 16-bit epilogue stores C write-through (sc1), so the launch ends with no dirty L2 lines for
// the next kernel's boundary to write back (chgemm_set_c_store; on by default: int8 igemmlt+dequant at the metric shape
// 126.3 -> 124.8 us, config 3 52.7 -> 51.7 us, the NF4 step unchanged to -1 us, C4 unchanged;
// profiles/lab/r04_store_policy.txt)
constexpr int HG_V_CWT = 32768;
static Knob<int> g_hg_cwt{1};
// variant bit: the 16-bit full-tile epilogue interleaved per 16-row group -- group i's outputs are converted (the bf16 /
// fp16 casts, or int8's mm_dequant) and staged while group i - 1's rows are read back and stored, so the VALU of the
// conversion overlaps the store stream instead of preceding all of it (chgemm_set_epilogue; round 5)
constexpr int HG_V_EPI = 65536;
static Knob<int> g_hg_epi{1};
// variant bit (with HG_V_EPI only): the interleaved epilogue's C stores carry the non-temporal hint (nt), so the output
// (not re-read by this step) does not displace the operands in the last-level cache (chgemm_set_c_store(2); A/B arm)
constexpr int HG_V_CNT = 131072;
// variant bit (lab): per-wave s_memrealtime stamps (10 ns ticks) at g_hg_tl[(blockIdx.x * 4 + wave) * 8 + i]: kernel
// start, prologue done (tile 0 landed, first barrier), k-loop done (DMA drained), epilogue's stores issued, stores
// complete, the workgroup's tile id, its XCD (chgemm_timeline; tools/hgemm_timeline.py)
constexpr int HG_V_TL = 262144;
__device__ unsigned long long* g_hg_tl = nullptr;
__device__ int g_hg_tl_nswap = 0;      // lab, HG_V_TL only: 1 = each XCD takes the other half of the N-tiles
__device__ int g_hg_tl_nostore = 0;    // lab, HG_V_TL only: 1 = the interleaved epilogue's C stores are dropped
[[maybe_unused]] static int g_hg_tl_on = 0;     // (lab build: chgemm_timeline)
__device__ __forceinline__ unsigned long long hg_now() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
// The round-3 two-half schedule (V = 8 + 16 + 4096) was the run-time A/B arm chgemm_set_variant(1) until round 6, when
// the cause of its int8 non-determinism (round 5, profiles/lab/r05_diag_int8_variant.txt) was found in the ISA, not in
// the waits: hipcc's register allocator, which sees an asm MFMA as an opaque statement, rotated accumulators through the
// two-half loop with v_accvgpr_read / v_accvgpr_mov (192-208 of them between the MFMAs of the V = 4120 kernels, e.g.
// `v_accvgpr_read_b32 v167, a55` six MFMAs after the asm MFMA that writes a[52:55]), without the MFMA -> AGPR-read wait
// states that its hazard recognizer inserts only for MFMAs it knows -- so a copy could read an accumulator before the
// MFMA wrote it, and which value it read depended on timing (only element 0 of acc[3][*] in the int8 kernel: one copied
// register of the rotation).  The bf16 / fp16 arms carried the same copies and passed by timing alone.  The arm is
// gone; tests/test_kernel_resources.py now checks that no k_hgemm kernel has an accumulator read, write or move between
// its first and last MFMA.
// lda / ldb / ldc in elements of the operand / output type.  rowStats / colStats / bias: HG_I8_DEQ only.
// SPLIT (bf16 / fp16 only): the split-K form -- its epilogue stores fp32 partials only.  A separate instantiation, so
// that each kernel has ONE epilogue reading the accumulators (two in one kernel made the allocator spill).
// Compile-time positions of the three-barrier schedule per tile shape (MFMA index q of the k-tile after which each
// event is issued; -1 = none).  256 x 256 (8, 8): 128 MFMAs, 16 pieces, vmcnt(13) at B3.  256 x 128 (8, 4) and
// 128 x 256 (4, 8): 64 MFMAs, 12 pieces -- the same order scaled: the stage's B rows are read first (w1), then B1; the
// B pieces go in while x1 is read; B2; the A pieces; B3 with the pieces issued so far left in flight; the next
// tile's step-0 fragments one per 2 MFMAs to the end, beside the last A pieces.
// compile-time loop: f(std::integral_constant<int, 0>) ... f(std::integral_constant<int, N - 1>)
template <class F, int... Q>
__device__ __forceinline__ void hg_static_for_impl(F&& f, std::integer_sequence<int, Q...>) {
  (f(std::integral_constant<int, Q>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void hg_static_for(F&& f) {
  hg_static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int WI, int WJ> struct HgPlan3;
// (lab: tools/hgemm_plan_sweep.sh builds the lab with these positions moved -- HG_P3_DB1 / DB2 / DB3 shift barrier B1 /
// B2 / B3 and everything keyed to it; the library is built with all three 0)
#ifndef HG_P3_DB1
#define HG_P3_DB1 0
#endif
#ifndef HG_P3_DB2
#define HG_P3_DB2 0
#endif
#ifndef HG_P3_DB3
#define HG_P3_DB3 0
#endif
#ifndef HG_P3_ABL
#define HG_P3_ABL 0
#endif
#ifndef HG_P3_AEARLY
#define HG_P3_AEARLY 0
#endif
template <> struct HgPlan3<8, 8> {
  static constexpr int D1 = HG_P3_DB1, D2 = HG_P3_DB2, D3 = HG_P3_DB3;
  // HG_P3_AEARLY (lab): the last 3 A pieces before B3 too (q B2 + 32, 34, 36), so B3 waits vmcnt(16) and the next
  // tile's fragment-read burst carries no DMA
  static constexpr int AE = HG_P3_AEARLY;
  static constexpr int B1 = 21 + D1, B2 = 50 + D2, B3 = 88 + D3, SETB = 22 + D1, SETA = 61 + D2, VM = AE ? 16 : 13,
                       SIDEQ = 120;
  __host__ __device__ static constexpr int wread(int q) { return q < 16 && (q & 1) == 0 ? q >> 1 : -1; }
  __host__ __device__ static constexpr int xread(int q) {
    return q >= 23 + D1 && q <= 44 + D1 && (q - 23 - D1) % 3 == 0 ? (q - 23 - D1) / 3 : -1;
  }
  __host__ __device__ static constexpr int bpiece(int q) {
    return q == 24 + D1 ? 0 : q == 28 + D1 ? 1 : q == 32 + D1 ? 2 : q == 36 + D1 ? 3 : q == 40 + D1 ? 4
         : q == 52 + D2 ? 5 : q == 56 + D2 ? 6 : q == 60 + D2 ? 7 : -1;
  }
  __host__ __device__ static constexpr int apiece(int q) {
    return q == 64 + D2 ? 0 : q == 68 + D2 ? 1 : q == 72 + D2 ? 2 : q == 76 + D2 ? 3 : q == 80 + D2 ? 4
         : AE ? (q == 82 + D2 ? 5 : q == 84 + D2 ? 6 : q == 86 + D2 ? 7 : -1)
              : (q == 97 + D3 ? 5 : q == 107 + D3 ? 6 : q == 117 + D3 ? 7 : -1);
  }
  __host__ __device__ static constexpr int nread(int q) { return q > B3 && q <= B3 + 31 && ((q - B3 - 1) & 1) == 0 ? (q - B3 - 1) >> 1 : -1; }
};
template <> struct HgPlan3<8, 4> {                      // 256 x 128: 4 B pieces, 8 A pieces per wave
  static constexpr int B1 = 9, B2 = 27, B3 = 38, SETB = 10, SETA = 22, VM = 9, SIDEQ = 58;
  __host__ __device__ static constexpr int wread(int q) { return q < 8 && (q & 1) == 0 ? q >> 1 : -1; }
  __host__ __device__ static constexpr int xread(int q) { return q >= 11 && q <= 25 && (q - 11) % 2 == 0 ? (q - 11) / 2 : -1; }
  __host__ __device__ static constexpr int bpiece(int q) { return q == 12 ? 0 : q == 15 ? 1 : q == 18 ? 2 : q == 21 ? 3 : -1; }
  __host__ __device__ static constexpr int apiece(int q) {
    return q == 28 ? 0 : q == 30 ? 1 : q == 32 ? 2 : q == 34 ? 3 : q == 36 ? 4 : q == 44 ? 5 : q == 50 ? 6 : q == 56 ? 7 : -1;
  }
  __host__ __device__ static constexpr int nread(int q) { return q > B3 && q <= B3 + 23 && ((q - B3 - 1) & 1) == 0 ? (q - B3 - 1) >> 1 : -1; }
};
template <> struct HgPlan3<4, 4> {                      // 128 x 128 (round 5): 32 MFMAs, 4 B + 4 A pieces per wave
  // step-1 fragments w1 at q 0..3 (B region of the stage), B1 at 5; the 4 B pieces at 6..9 beside x1 at 6..9, B2 at 11;
  // A pieces at 12, 13; B3 at 14 (vmcnt(6): the previous k-tile's 2 tail A pieces and this k-tile's 4 B + 2 A may
  // fly); the next tile's step-0 fragments one per 2 MFMAs from 15 to 29 (w0[0] last used at q 3, x0[i] at 12 + i,
  // w0[j] at 4 j + 3); the last 2 A pieces at 18 and 24.  M0 is set right after a barrier, one MFMA before its piece.
  static constexpr int B1 = 5, B2 = 11, B3 = 14, SETB = 5, SETA = 11, VM = 6, SIDEQ = 28;
  __host__ __device__ static constexpr int wread(int q) { return q < 4 ? q : -1; }
  __host__ __device__ static constexpr int xread(int q) { return q >= 6 && q <= 9 ? q - 6 : -1; }
  __host__ __device__ static constexpr int bpiece(int q) { return q >= 6 && q <= 9 ? q - 6 : -1; }
  __host__ __device__ static constexpr int apiece(int q) { return q == 12 ? 0 : q == 13 ? 1 : q == 18 ? 2 : q == 24 ? 3 : -1; }
  __host__ __device__ static constexpr int nread(int q) { return q > B3 && q <= B3 + 15 && ((q - B3 - 1) & 1) == 0 ? (q - B3 - 1) >> 1 : -1; }
};
template <> struct HgPlan3<4, 8> {                      // 128 x 256: 8 B pieces, 4 A pieces per wave
  static constexpr int B1 = 17, B2 = 27, B3 = 38, SETB = 17, SETA = 33, VM = 10, SIDEQ = 58;
  __host__ __device__ static constexpr int wread(int q) { return q < 16 && (q & 1) == 0 ? q >> 1 : -1; }
  __host__ __device__ static constexpr int xread(int q) { return q >= 19 && q <= 25 && (q - 19) % 2 == 0 ? (q - 19) / 2 : -1; }
  __host__ __device__ static constexpr int bpiece(int q) {
    return q == 18 ? 0 : q == 20 ? 1 : q == 22 ? 2 : q == 24 ? 3 : q == 26 ? 4 : q == 28 ? 5 : q == 30 ? 6 : q == 32 ? 7 : -1;
  }
  __host__ __device__ static constexpr int apiece(int q) { return q == 34 ? 0 : q == 36 ? 1 : q == 46 ? 2 : q == 54 ? 3 : -1; }
  __host__ __device__ static constexpr int nread(int q) { return q > B3 && q <= B3 + 23 && ((q - B3 - 1) & 1) == 0 ? (q - B3 - 1) >> 1 : -1; }
};

// Side dequantise (SIDE = true, bf16 / fp16 only): while it multiplies, the kernel also dequantises the NEXT 4-bit
// weight (the next projection of the layer, or the next layer's) into a second weight buffer -- the cdequantize_blockwise
// / dequantize_4bit_nested work of the following gemm_4bit call, software-pipelined one weight ahead so that the
// HBM-bound dequantise runs in the MFMA-bound GEMM's shadow instead of as its own launch (the same values as
// k_dequantize_4bit_stream, quant.hip: fp32 code * fp32 absmax, one RNE cast; nested statistics decoded as
// code2[q8] * absmax2 + offset).  Workgroup w owns packed dwords [w * per_wg, (w + 1) * per_wg), 1024 per
// "iteration" (4 dwords = 32 weights per lane, coalesced).  In the main loop one iteration runs every `every` k-tiles, right after
// barrier B3: its loads are issued then and consumed one side step later, after that step's B3 wait -- the loads sit
// before the next k-tile's DMA pieces, so vmcnt(VM) at the next B3 already covers them and the DMA counts stay exact
// (the loads and the 16-B stores are inline asm, invisible to hipcc's wait insertion, like the DMA).  Iterations
// left when the loop ends (few k-tiles) run after it.
struct HgSide {
  const uint8_t* packed;     // next weight, packed 4-bit (16-B aligned)
  const float* absmax;       // fp32 block statistics (nested == 0)
  const uint8_t* q8;         // nested: 8-bit codes of the statistics
  const float* code2;        // nested: their 256-entry code
  const float* absmax2;      // nested: second-level scales
  const float* offset;       // nested: the statistics' offset
  void* out;                 // ndw * 8 outputs of the GEMM's type (16-B aligned)
  long long ndw;             // packed dwords (elements / 8)
  int per_wg, iters, every, bs_shift, bs2_shift, nested, fp4;
  int mode;                  // A/B bits (chgemm_set_side_mode): 1 = non-temporal packed loads / output stores; 128 =
                             // the round-4 in-loop form instead of the tail form (below); lab ablations (timing only,
                             // wrong weights): 2 = no side stores, 8 = no consumption, 16 = no side loads, 32 = no side
                             // step in the loop, 64 = no tail
};
static Knob<int> g_side_mode{1};

// Tail form of the side dequantise (round 6, V & HG_V_TAIL, the default of chgemm_tn_pf_*): no side work inside the
// k-loop at all -- each wave, once its tile's epilogue has issued its C stores, dequantises its share of the next
// weight.  The in-loop form (round 4) paid for its side work in MFMA issue slots (+40-50 us at the metric shape); the
// tail form takes no issue slot from any MFMA, and the pipelined step costs what the unpipelined pair does
// (profiles/lab/r06_tail_ab.txt: 258.9 vs 257.8 us; C4 18.08 vs 18.03 ms).  It was built to spend the XCD slack (the
// k-loop ends up to ~8 % apart between the fastest and the slowest XCD on identical work) on the next
// weight by work stealing; that lost (below).  Values: exactly k_dequantize_4bit_stream's (code * absmax in fp32, one RNE cast;
// nested: code2[q8] * absmax2 + offset) -- the same helper arithmetic as the in-loop form, whatever wave does a chunk.
// Chunk c (64 lanes x HG_TAIL_U packed dwords) goes to wave c mod waves (static; work stealing measured slower, below).
constexpr int HG_V_TAIL = 524288;
constexpr int HG_TAIL_U = 16;                              // packed dwords per lane per wave chunk

// one wave's chunk c: 64 x HG_TAIL_U packed dwords, lane l taking dwords 64 j + l (the k_dequantize_4bit_stream layout:
// every load and every 16-B output store of the wave is one contiguous, whole-line run -- a lane-contiguous 16-B load
// per lane made each store instruction write 16 B of every 64 and ran the tail ~3x slower)
struct HgTailRegs {
  uint32_t w[HG_TAIL_U];
  uint32_t q[HG_TAIL_U];     // nested: the statistic's 8-bit code (decoded at store time, not at load time)
  float a[HG_TAIL_U];        // nested: its second-level scale; plain: the fp32 absmax
};
// issue the chunk's loads only -- nothing here consumes them, so the wave goes on to convert and store the previous
// chunk while these are in flight (a statistic decoded here would make the wave wait for its load first)
__device__ __forceinline__ void hg_tail_load(const HgSide& side, uint32_t c, int lane, HgTailRegs& r) {
  const uint32_t base = c * (64u * HG_TAIL_U);
  const uint32_t* Aw = reinterpret_cast<const uint32_t*>(side.packed);
#pragma unroll
  for (int j = 0; j < HG_TAIL_U; ++j) {
    const uint32_t d = min(base + 64u * j + (uint32_t)lane, (uint32_t)side.ndw - 1u);
    r.w[j] = __builtin_nontemporal_load(Aw + d);
    const uint32_t blk = (d * 8u) >> side.bs_shift;
    if (side.nested) {
      r.q[j] = side.q8[blk];
      r.a[j] = side.absmax2[blk >> side.bs2_shift];
    } else {
      r.a[j] = side.absmax[blk];
    }
  }
}
template <typename T16>
__device__ __forceinline__ void hg_tail_store(const HgSide& side, const float2* s_pair, const float* s_c2, float off,
                                              uint32_t c, int lane, const HgTailRegs& r) {
  const uint32_t base = c * (64u * HG_TAIL_U);
#pragma unroll
  for (int j = 0; j < HG_TAIL_U; ++j) {
    const uint32_t d = base + 64u * j + (uint32_t)lane;
    const float am = side.nested ? __fadd_rn(__fmul_rn(s_c2[r.q[j] & 0xFF], r.a[j]), off) : r.a[j];
    hg_u32x4_t o;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float2 p = s_pair[(r.w[j] >> (8 * i)) & 0xFF];
      o[i] = cvt_pk<T16>(__fmul_rn(p.x, am), __fmul_rn(p.y, am));
    }
    // device-scope write-through (sc1), as k_dequantize_4bit_stream's default store policy: the next launch reads it
    if (d < (uint32_t)side.ndw)
      asm volatile("global_store_dwordx4 %0, %1, %2 sc1\n\ts_nop 1" : : "v"(d * 16u), "v"(o), "s"(side.out) : "memory");
  }
}

// The tail form's loop, run by every wave on its own after the epilogue: no workgroup barrier (a barrier's release
// fence would wait for every store issued so far), the wave's own LDS copy of the code-pair table (2 KiB) and nested
// code map (1 KiB) in its own epilogue staging rows (`ep`, which it has finished reading: LDS operations of one wave
// run in order), its first chunk by its wave index and the rest from the counter, and each chunk's loads issued before
// the previous chunk is converted and stored (two register sets).
template <typename T16>
__device__ __forceinline__ void hg_side_tail(const HgSide& side, uint8_t* ep, int lane, uint32_t wave_id,
                                             uint32_t waves) {
  float2* s_pair = reinterpret_cast<float2*>(ep);
  float* s_c2 = reinterpret_cast<float*>(ep + 2048);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = lane + 64 * q;
    s_pair[e] = side.fp4 ? make_float2(code4_value<FP4>(e >> 4), code4_value<FP4>(e & 15))
                         : make_float2(code4_value<NF4>(e >> 4), code4_value<NF4>(e & 15));
    if (side.nested) s_c2[e] = side.code2[e];
  }
  const float off = side.nested ? *side.offset : 0.0f;
  const uint32_t nchunks = (uint32_t)((side.ndw + 64 * HG_TAIL_U - 1) / (64 * HG_TAIL_U));
  // static assignment: chunk c to wave c mod waves.  Work stealing was measured and dropped (profiles/lab/r06_tail_ab.txt):
  // a wave that waits for a counter's return also waits for its previous chunk's stores (vmcnt counts both, in order),
  // and that cost more than the XCD slack it recovered (one counter +40 us, eight per-XCD counters +12 us at the metric
  // shape, against +1 us static)
  // (the next chunk's loads are issued before this one is converted and stored: two register sets in rotation)
  HgTailRegs r0, r1;
  uint32_t c = wave_id;
  if (c < nchunks) {
    hg_tail_load(side, c, lane, r0);
    while (true) {
      const uint32_t n = c + waves;
      if (n < nchunks) hg_tail_load(side, n, lane, r1);
      hg_tail_store<T16>(side, s_pair, s_c2, off, c, lane, r0);
      if (n >= nchunks) break;
      const uint32_t n2 = n + waves;
      if (n2 < nchunks) hg_tail_load(side, n2, lane, r0);
      hg_tail_store<T16>(side, s_pair, s_c2, off, n, lane, r1);
      if (n2 >= nchunks) break;
      c = n2;
    }
  }
}

template <int OP, int V = 0, bool SPLIT = false, int WI = 8, int WJ = 8, bool SIDE = false>
__global__ void __launch_bounds__(HG_THREADS, 1)
k_hgemm(int M, int N, int K, const void* __restrict__ Av, long long lda, const void* __restrict__ Bv, long long ldb,
        void* __restrict__ Cv, long long ldc, const float* __restrict__ rowStats, const float* __restrict__ colStats,
        const fp16_t* __restrict__ bias, float* __restrict__ ws, int ksplit, int kchunk, HgSide side) {
  using Op = HgOpT<OP>;
  using acc_t = typename Op::acc_t;
  constexpr int E = Op::ELEM;
  static_assert(!SIDE || ((OP == HG_BF16 || OP == HG_FP16) && (V & 8192) != 0), "side dequantise: 16-bit, tile3");
  // tile shape: 2 x 2 waves of (16 WI) x (16 WJ) outputs -- 256 x 256 (8, 8), 256 x 128 (8, 4), 128 x 256 (4, 8)
  static_assert((WI == 8 && WJ == 8) || (V & 8192) != 0, "tile shapes other than 256 x 256 run the three-barrier schedule");
  constexpr int BM = 32 * WI, BN = 32 * WJ;
  constexpr int TA = BM * 128, STG = TA + BN * 128;     // A tile, then B tile, per stage
  constexpr int EPI_PITCH = 32 * WJ + 16;               // 16-bit output staging row per wave (16 B of padding)
  constexpr int LDS_BYTES = 2 * STG > 4 * 16 * WI * EPI_PITCH ? 2 * STG : 4 * 16 * WI * EPI_PITCH;
  // split-K (ksplit > 1, small tile grids): workgroup = (tile, split s); split s multiplies k-tiles
  // [s * kchunk, min((s + 1) * kchunk, all)) and stores fp32 partials ws[s][M][N] (summed in split order afterwards)
  const int tiles_all = ((N + BN - 1) / BN) * ((M + BM - 1) / BM);
  // (readfirstlane: the divisions by the runtime ksplit run on the VALU; their wave-uniform results must live in SGPRs,
  // not in two of the main loop's 256 VGPRs -- that spilled)
  const int wgs = xcd_remap(blockIdx.x, tiles_all * (SPLIT ? ksplit : 1));
  const int split = SPLIT ? __builtin_amdgcn_readfirstlane(wgs % ksplit) : 0;
  const int kt0 = split * kchunk;
  const uint8_t* A = reinterpret_cast<const uint8_t*>(Av) + (long long)kt0 * 128;
  const uint8_t* B = reinterpret_cast<const uint8_t*>(Bv) + (long long)kt0 * 128;
  // side dequantise (SIDE): pair table (2 KiB) + code2 (1 KiB) + two buffers of LDS-DMA landing slots for one
  // iteration (per wave: 64 x 16 B of packed weights, 64 x 4 B statistic codes, 64 x 4 B second-level scales)
  constexpr int SIDE_WAVE = 1536, SIDE_BUF = 4 * SIDE_WAVE;
  constexpr int SIDE_LDS = SIDE ? 3072 + 2 * SIDE_BUF : 0;
  // HG_I8_DEQ: the tile's row scales (BM floats), column scales (BN floats) and bias (BN halves), brought in by LDS-DMA
  // in the prologue so that the epilogue reads them from LDS instead of waiting on global loads
  constexpr int STATS_LDS = (OP == HG_I8_DEQ) ? 4 * BM + 4 * BN + 2 * BN : 0;
  __shared__ __attribute__((aligned(16))) uint8_t smem[LDS_BYTES + SIDE_LDS + STATS_LDS];
  constexpr bool TL = (V & HG_V_TL) != 0;
  unsigned long long tl0 = 0, tl1 = 0, tl2 = 0;
  if constexpr (TL) tl0 = hg_now();
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  using T16 = typename std::conditional<OP == HG_FP16, fp16_t, bf16_t>::type;
  // Side dequantise state.  One iteration = 4 packed dwords (32 weights, one statistics block) per lane, 1024 dwords
  // per workgroup.  Its words travel by LDS-DMA into landing slots (global_load_lds_*, M0 = this wave's slot row),
  // never into registers: an asm load's destination register is written when the load returns, and hipcc, which sees
  // the asm as writing it at issue, may copy it before then (it did: a loop phi move of the absmax2 register right
  // behind the load).  An iteration issued in k-tile t (after its last A piece, 3 loads) may stay in flight across B3
  // of t+1 (that wait is vmcnt(VM + 3) then) and is consumed after B3 of t+2, whose wait covers it -- two k-tiles for
  // loads that miss to HBM.  sd_i0 / i1 / i2: the iteration issued in this / the previous / the one-before k-tile (-1:
  // none); landing buffer = iteration & 1.  Counters are uniform; dword indices fit 32 bits (host: ndw < 2^28).
  float2* const s_pair = reinterpret_cast<float2*>(smem + LDS_BYTES);
  float* const s_c2 = reinterpret_cast<float*>(smem + LDS_BYTES + 2048);
  const uint8_t* const s_land = smem + LDS_BYTES + 3072 + wave * SIDE_WAVE;
  const uint32_t land0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(smem + LDS_BYTES + 3072)) + wave * SIDE_WAVE;
  uint32_t sd_base = 0;
  int sd_it = 0, sd_i0 = -1, sd_i1 = -1, sd_i2 = -1;
  float sd_off = 0.0f;
  if constexpr (SIDE) {
    // (before any DMA is issued: hipcc's vmcnt wait for the code2 load then waits for that load alone)
    s_pair[tid] = side.fp4 ? make_float2(code4_value<FP4>(tid >> 4), code4_value<FP4>(tid & 15))
                           : make_float2(code4_value<NF4>(tid >> 4), code4_value<NF4>(tid & 15));
    if (side.nested) {
      s_c2[tid] = side.code2[tid];
      sd_off = *side.offset;
    }
    sd_base = (uint32_t)blockIdx.x * (uint32_t)side.per_wg;
  }
  // the lane's first dword of iteration `it` (clamped for the loads; the stores check the unclamped one)
  auto side_gd = [&](int it) -> uint32_t { return sd_base + (uint32_t)it * 1024u + 4u * (uint32_t)tid; };
  // issue the next iteration's loads, always exactly three (the B3 wait counts them): 16 B of packed weights -> row 0,
  // statistic word -> row 1 (q8 byte or fp32 absmax), absmax2 -> row 2 (plain statistics: the absmax again).  Only
  // where nothing else holds M0 (after a k-tile's last A piece; the next SETB re-sets it).
  auto side_issue = [&]() {
    const uint32_t gd = min(side_gd(sd_it), (uint32_t)side.ndw - 4u);
    const uint32_t blk = (gd * 8u) >> side.bs_shift;
    const uint32_t lb = land0 + (sd_it & 1) * SIDE_BUF;
    if (side.mode & 16) {                                // lab: no loads (the wait count is then wrong: timing only)
      sd_i0 = sd_it++;
      return;
    }
    if (side.mode & 1)
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 nt"
                   : : "v"(gd * 4u), "s"(side.packed), "s"(lb) : "memory");
    else
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                   : : "v"(gd * 4u), "s"(side.packed), "s"(lb) : "memory");
    if (side.nested) {
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_ubyte %0, %1"
                   : : "v"(blk), "s"(side.q8), "s"(lb + 1024) : "memory");
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1"
                   : : "v"((blk >> side.bs2_shift) * 4u), "s"(side.absmax2), "s"(lb + 1280) : "memory");
    } else {
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1"
                   : : "v"(blk * 4u), "s"(side.absmax), "s"(lb + 1024) : "memory");
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1"
                   : : "v"(blk * 4u), "s"(side.absmax), "s"(lb + 1280) : "memory");
    }
    sd_i0 = sd_it++;
  };
  // consume iteration `it` in parts spread over MFMAs (after a wait covering its DMA): the landed words; the statistic;
  // then per packed dword j its 4 table lookups, and (a part later) fp32 code * absmax, one RNE cast each, one 16-B store
  hg_u32x4_t sd_w = {0u, 0u, 0u, 0u};
  uint32_t sd_q = 0, sd_a2 = 0;
  float sd_am = 0.0f;
  float2 sd_p[4];
  auto side_words = [&](int it) {
    const uint8_t* l = s_land + (it & 1) * SIDE_BUF;
    sd_w = *reinterpret_cast<const hg_u32x4_t*>(l + 16 * lane);
    sd_q = *reinterpret_cast<const uint32_t*>(l + 1024 + 4 * lane);
    sd_a2 = *reinterpret_cast<const uint32_t*>(l + 1280 + 4 * lane);
  };
  auto side_stat = [&]() {
    sd_am = side.nested ? __fadd_rn(__fmul_rn(s_c2[sd_q & 0xFF], __uint_as_float(sd_a2)), sd_off) : __uint_as_float(sd_q);
  };
  auto side_lookup = [&](int j) {
#pragma unroll
    for (int i = 0; i < 4; ++i) sd_p[i] = s_pair[(sd_w[j] >> (8 * i)) & 0xFF];
  };
  auto side_store = [&](int it, int j) {
    const uint32_t gd = side_gd(it) + (uint32_t)j;
    hg_u32x4_t o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = cvt_pk<T16>(__fmul_rn(sd_p[i].x, sd_am), __fmul_rn(sd_p[i].y, sd_am));
    // (s_nop 1: the store-data -> VALU overwrite wait state hipcc does not see through the asm)
    if (gd < (uint32_t)side.ndw && !(side.mode & 2)) {
      if (side.mode & 1)
        asm volatile("global_store_dwordx4 %0, %1, %2 nt\n\ts_nop 1" : : "v"(gd * 16u), "v"(o), "s"(side.out) : "memory");
      else
        asm volatile("global_store_dwordx4 %0, %1, %2\n\ts_nop 1" : : "v"(gd * 16u), "v"(o), "s"(side.out) : "memory");
    }
  };

  // ---- tile order: XCD-contiguous ids; groups of 4 M-tiles x all N-tiles (an XCD's 32 tiles share A / B rows)
  const int tilesN = (N + BN - 1) / BN, tilesM = (M + BM - 1) / BM;
  const int wg = SPLIT ? __builtin_amdgcn_readfirstlane(wgs / ksplit) : wgs;
  constexpr int GROUP = 4;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  int tn = (wg % group_span) / gsize;
  if constexpr (TL) {
    if (g_hg_tl_nswap) tn = (tn + tilesN / 2) % tilesN;
  }
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- DMA: wave w fills A pieces p = WI w + i and B pieces p = WJ w + i (tile rows 8p .. 8p+7); lane -> (row,
  // slot).  (32-bit arithmetic: the host keeps every offset below 4 GiB; 64-bit products made hipcc park each offset
  // in a 4-register tuple)
  uint32_t aoff[WI], boff[WJ];
  const uint32_t lda2 = (uint32_t)lda * E, ldb2 = (uint32_t)ldb * E;   // row strides in bytes
#pragma unroll
  for (int i = 0; i < WI; ++i) {
    const int row = 8 * (WI * wave + i) + (lane >> 3);
    const uint32_t slot = (uint32_t)((lane & 7) ^ ((row >> 1) & 7));
    aoff[i] = (uint32_t)min(m0 + row, M - 1) * lda2 + 16u * slot;
  }
#pragma unroll
  for (int i = 0; i < WJ; ++i) {
    const int row = 8 * (WJ * wave + i) + (lane >> 3);
    const uint32_t slot = (uint32_t)((lane & 7) ^ ((row >> 1) & 7));
    boff[i] = (uint32_t)min(n0 + row, N - 1) * ldb2 + 16u * slot;
  }
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
  const uint32_t ldsA0 = lds_base + wave * WI * 1024, ldsB0 = lds_base + TA + wave * WJ * 1024;
  [[maybe_unused]] const hg_rsrc_t rsA = hg_rsrc(A), rsB = hg_rsrc(B);
  auto dma_a = [&](int kt, int st, int i) {
    if constexpr (HG_DMA_BUF && (V & 16) != 0) glds16_buf_m0(rsA, aoff[i], (uint32_t)kt * 128u, ldsA0 + st * STG + i * 1024);
    else if constexpr ((V & 16) != 0) glds16_sv_m0(A + (long long)kt * 128, aoff[i], ldsA0 + st * STG + i * 1024);
    else glds16_sv(A + (long long)kt * 128, aoff[i], ldsA0 + st * STG + i * 1024);
  };
  auto dma_b = [&](int kt, int st, int i) {
    if constexpr (HG_DMA_BUF && (V & 16) != 0) glds16_buf_m0(rsB, boff[i], (uint32_t)kt * 128u, ldsB0 + st * STG + i * 1024);
    else if constexpr ((V & 16) != 0) glds16_sv_m0(B + (long long)kt * 128, boff[i], ldsB0 + st * STG + i * 1024);
    else glds16_sv(B + (long long)kt * 128, boff[i], ldsB0 + st * STG + i * 1024);
  };

  // ---- fragments: MFMA A operand = B rows (n), MFMA B operand = A rows (m), so D[n][m] and a lane's 4 results
  // are 4 consecutive n of one m: one 8-B store per accumulator.  Row keys ((row >> 1) & 7) do not depend on the
  // fragment index, so each operand needs one lane offset per k32 step.
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fg = lane >> 4, key = (fr >> 1) & 7;
  const int xo0 = (16 * WI * wm + fr) * 128 + ((fg ^ key) << 4);
  const int xo1 = (16 * WI * wm + fr) * 128 + (((4 + fg) ^ key) << 4);
  const int wo0 = TA + (16 * WJ * wn + fr) * 128 + ((fg ^ key) << 4);
  const int wo1 = TA + (16 * WJ * wn + fr) * 128 + (((4 + fg) ^ key) << 4);
  using frag_t = hg_u32x4_t;
  auto rd = [&](int st, int off, int f) -> frag_t {
    return *reinterpret_cast<const frag_t*>(smem + st * STG + off + f * 2048);
  };

  acc_t acc[WJ][WI];
  frag_t w0[WJ], x0[WI], w1[WJ], x1[WI];
  const int nk = min(kchunk, K * E / 128 - kt0);   // k-tiles of 128 bytes in this split (>= 1 by the host rule)

  // V & 512 (lab): register-staged copies instead of LDS-DMA -- ordinary 16-B global loads into 16 staging registers
  // (same swizzled source offsets), written to the same LDS slots one k-tile later by ds_write_b128.  The writes of
  // tile t+1 finish before half 1's barrier, so that barrier alone orders them against the reads: one barrier per
  // k-tile, no vmcnt bookkeeping of ours (hipcc counts the ordinary loads).
  constexpr bool RS = (V & 512) != 0;
  frag_t sg[RS ? 16 : 1];
  auto rs_load = [&](int kt, int q) {
    if constexpr (RS) {
      const uint8_t* base = (q < 8 ? A : B) + (long long)kt * 128;
      sg[q] = *reinterpret_cast<const frag_t*>(base + (q < 8 ? aoff[q] : boff[q - 8]));
    }
  };
  auto rs_write = [&](int st, int q) {
    if constexpr (RS)
      *reinterpret_cast<frag_t*>(smem + st * STG + (q < 8 ? 0 : TA) + wave * 8192 + (q & 7) * 1024 +
                                 16 * lane) = sg[q];
  };

  // half 1 of k-tile t (stage st): the 64 MFMAs of k32 step 0, step 1's fragments of the stage read underneath (one
  // read per 4 MFMAs); then this wave's reads are retired and the barrier says every wave is done with the stage.
  // FIRST: tile 0 starts the accumulators (SrcC = 0, so no zero-fill of the AGPRs is needed).
  auto half1 = [&](auto first, int t) {
    const int st = t & 1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (decltype(first)::value) acc[j][i] = Op::mma0(w0[j], x0[i]);
        else acc[j][i] = Op::mma(w0[j], x0[i], acc[j][i]);
        if constexpr (RS) {
          // register staging: piece q of tile t+1 into stage st ^ 1, then tile t+2's piece q into the same registers
          const int q = 2 * j + (i >> 2);
          if ((i & 3) == 0) rs_write(st ^ 1, q);
          if ((i & 3) == 1) rs_load(min(t + 2, nk - 1), q);
        }
        if (!(V & 1) && !(V & 2048) && (i & 3) == 3) {   // (V & 2048: lab ablation, no fragment re-reads)
          const int q = 2 * j + (i >> 2);               // 0..15
          if (q < 8) w1[q] = rd(st, wo1, q);
          else x1[q - 8] = rd(st, xo1, q - 8);
        }
      }
      if (!(V & 1)) __builtin_amdgcn_sched_barrier(0);
    }
    if (V & 1) {
#pragma unroll
      for (int f = 0; f < 8; ++f) { w1[f] = rd(st, wo1, f); x1[f] = rd(st, xo1, f); }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);                   // lgkmcnt(0): this wave's reads of stage st are done
    if constexpr ((V & 256) == 0) __builtin_amdgcn_s_barrier();   // ... and every other wave's (V & 256: lab ablation)
    __builtin_amdgcn_sched_barrier(0);
  };
  // half 2 of k-tile t: the 64 MFMAs of step 1.  Unless LAST: tile t+2's DMA into stage st under the first 32 (one
  // piece per 2 MFMAs; past the end the last tile is re-loaded into a stage nobody reads again, so the body stays
  // branch-free), vmcnt(16) = tile t+1 landed for this wave + barrier = for every wave, and tile t+1's step-0
  // fragments read under the last 32.
  auto half2 = [&](auto last, int t, int st) {
    constexpr bool L = decltype(last)::value;
    // PRE of the 16 DMA pieces go in before the wait for tile t+1, spread over the first 32 MFMAs; the rest after it,
    // spread over the last 32 (V & 8: 8 / 8; V & 32: 12 / 4; neither: 16 / 0, one per 2 MFMAs)
    constexpr int PRE = (V & 32) ? 12 : (V & 8) ? 8 : 16;
    const int kn = min(t + 2, nk - 1);
    auto dma = [&](int q) {
      if constexpr ((V & 1024) != 0) return;            // lab ablation: no copies at all (timing only)
      if constexpr ((V & 4096) != 0) {                   // M0 chained from piece to piece (pieces issued in order)
        if (q < 7) glds16_chain<1024>(A + (long long)kn * 128, aoff[q]);
        else if (q == 7) glds16_chain<TA - 7 * 1024>(A + (long long)kn * 128, aoff[7]);
        else glds16_chain<1024>(B + (long long)kn * 128, boff[q - 8]);
        return;
      }
      if (q < 8) dma_a(kn, st, q);
      else dma_b(kn, st, q - 8);
    };
    if constexpr (!L && (V & 4096) != 0) hg_set_m0(ldsA0 + st * STG);
    // fragment q of the next step 0, in the order its MFMAs need them (w0[0], x0[0..7], w0[1..7]) unless V & 4 == 0
    auto rdn = [&](int q) {
      if constexpr ((V & 4) != 0) {
        if (q == 0) w0[0] = rd(st ^ 1, wo0, 0);
        else if (q <= 8) x0[q - 1] = rd(st ^ 1, xo0, q - 1);
        else w0[q - 8] = rd(st ^ 1, wo0, q - 8);
      } else {
        if (q < 8) w0[q] = rd(st ^ 1, wo0, q);
        else x0[q - 8] = rd(st ^ 1, xo0, q - 8);
      }
    };
    // DMA piece issued after MFMA `mi` (0..31) of a part holding `cnt` pieces: pieces land on MFMAs
    // (q + 1) * 32 / cnt - 1, q = 0 .. cnt - 1 (evenly spread, the last one on the part's last MFMA)
    auto piece_at = [](int mi, int cnt) -> int {
      for (int q = 0; q < cnt; ++q)
        if (((q + 1) * 32) / cnt - 1 == mi) return q;
      return -1;
    };
    if constexpr (RS) {
      // register staging: tile t+1 is already in stage st ^ 1 for every wave (half 1's barrier); its step-0
      // fragments are read under all 64 MFMAs, one per 4
#pragma unroll
      for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          acc[j][i] = Op::mma(w1[j], x1[i], acc[j][i]);
          if constexpr (!L) if ((i & 3) == 3) rdn(2 * j + (i >> 2));
        }
        if (!(V & 2)) __builtin_amdgcn_sched_barrier(0);
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[j][i] = Op::mma(w1[j], x1[i], acc[j][i]);
        if constexpr (!L) {
          const int q = piece_at(8 * j + i, PRE);
          if (q >= 0) dma(q);
        }
      }
      if (!(V & 2)) __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (!L) {
      // (V & 64 / V & 128: lab ablations that drop the wait / the barrier -- wrong results, timing only)
      if constexpr ((V & 64) != 0) {
      } else if constexpr (PRE == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // tile t+1 landed (this wave)
      else if constexpr (PRE == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      if constexpr ((V & 128) == 0) __builtin_amdgcn_s_barrier();      // ... every wave's pieces
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = 4; j < 8; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[j][i] = Op::mma(w1[j], x1[i], acc[j][i]);
        if constexpr (!L) {
          if (!(V & 2048) && (i & 1) == 1) rdn(4 * (j - 4) + (i >> 1));       // fragments 0..15
          const int q = piece_at(8 * (j - 4) + i, 16 - PRE);
          if (q >= 0) dma(PRE + q);
        }
      }
      if (!(V & 2)) __builtin_amdgcn_sched_barrier(0);
    }
  };

  // V & 8192: the operand-split schedule, three barriers per k-tile.  For the 256 x 256 tile (WI = WJ = 8, 128 MFMAs per
  // k-tile), MFMA index q:
  //   q 0..14   this wave reads step 1's B fragments (w1) of the stage, one per 2 MFMAs;
  //   q 21      lgkmcnt(0) + barrier B1: every wave is done with the stage's B rows, so tile t+2's B pieces go into
  //             them from q 24 on (5 before B2, 3 after), while this wave reads step 1's A fragments (x1, q 23..44);
  //   q 50      lgkmcnt(0) + barrier B2: the stage's A rows are free too; tile t+2's A pieces from q 64 on;
  //   q 88      vmcnt(13) (the 13 pieces issued so far in this k-tile may still fly: tile t+1, issued one k-tile
  //             earlier, has landed for this wave) + barrier B3 (... for every wave); tile t+1's step-0 fragments are
  //             read under the remaining 39 MFMAs (one per 2), beside the last 3 A pieces.
  // So a piece is issued as soon as its rows are free (from MFMA 24 instead of 64) and 13 of 16 stay in flight across
  // the tile boundary; the fragment reads of a k-tile never share an MFMA gap with more than one DMA issue.  The
  // half-width tiles (64 MFMAs per k-tile, 12 pieces) follow the same order on the HgPlan3 positions below.
  using P3 = HgPlan3<WI, WJ>;
  int sd_cd = 0;                                          // k-tiles until the next side step
  auto tile3 = [&](auto first, auto last, int t) {
    constexpr bool FIRST = decltype(first)::value, L = decltype(last)::value;
    constexpr int S = WI * WJ;                           // MFMAs per k32 step
    const int st = t & 1;
    const int kn = min(t + 2, nk - 1);
    bool sd_go = false;                                  // side issue in this k-tile (not the last)
    if constexpr (SIDE) {
      sd_i2 = sd_i1;
      sd_i1 = sd_i0;
      sd_i0 = -1;
      if constexpr (!L) {
        sd_go = sd_cd == 0 && !(side.mode & 32);         // (mode 32, lab: no side step in the loop)
        sd_cd = sd_go ? side.every - 1 : sd_cd - 1;
      }
    }
    // (unrolled at compile time -- hg_static_for hands the body a constant q: with a runtime loop of 2 S iterations
    // the unroller gave up on the 256 x 256 tile and left the accumulator and fragment arrays in scratch)
    hg_static_for<2 * S>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      constexpr int qq = q % S, j = qq / WI, i = qq % WI;
      if constexpr (q < S) {
        if constexpr (FIRST) acc[j][i] = Op::mma0(w0[j], x0[i]);
        else acc[j][i] = Op::mma(w0[j], x0[i], acc[j][i]);
      } else {
        acc[j][i] = Op::mma(w1[j], x1[i], acc[j][i]);
      }
      // (HG_P3_ABL lab bits, timing only: 16 = no LDS-DMA pieces in the loop, 32 = no fragment reads in the loop)
      if constexpr ((HG_P3_ABL & 32) == 0) {
        if constexpr (P3::wread(q) >= 0) w1[P3::wread(q)] = rd(st, wo1, P3::wread(q));
        if constexpr (P3::xread(q) >= 0) x1[P3::xread(q)] = rd(st, xo1, P3::xread(q));
      }
      if constexpr (q == P3::B1 || q == P3::B2) {
        // (HG_P3_ABL, lab builds only -- races, wrong results, timing only: 1 = no barrier at B1 / B2, 2 = no wait)
        if constexpr ((HG_P3_ABL & 2) == 0) __builtin_amdgcn_s_waitcnt(0xC07F);            // lgkmcnt(0)
        if constexpr (!L && (HG_P3_ABL & 1) == 0) __builtin_amdgcn_s_barrier();
      }
      if constexpr (!L) {
        if constexpr (q == P3::SETB) hg_set_m0(ldsB0 + st * STG);
        if constexpr (P3::bpiece(q) >= 0 && (HG_P3_ABL & 16) == 0) {
          if constexpr (HG_DMA_BUF) glds16_chain_buf<1024>(rsB, boff[P3::bpiece(q)], (uint32_t)kn * 128u);
          else glds16_chain<1024>(B + (long long)kn * 128, boff[P3::bpiece(q)]);
        }
        if constexpr (q == P3::SETA) hg_set_m0(ldsA0 + st * STG);
        if constexpr (P3::apiece(q) >= 0 && (HG_P3_ABL & 16) == 0) {
          if constexpr (HG_DMA_BUF) glds16_chain_buf<1024>(rsA, aoff[P3::apiece(q)], (uint32_t)kn * 128u);
          else glds16_chain<1024>(A + (long long)kn * 128, aoff[P3::apiece(q)]);
        }
        if constexpr (q == P3::B3) {
          // (HG_P3_ABL lab bits: 4 = no vmcnt wait at B3, 8 = no barrier at B3 -- timing only)
          if constexpr ((HG_P3_ABL & 4) == 0) {
            if (SIDE && sd_i1 >= 0) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(P3::VM + 3) : "memory");  // (+ its 3 loads)
            else asm volatile("s_waitcnt vmcnt(%0)" ::"i"(P3::VM) : "memory");
          }
          if constexpr ((HG_P3_ABL & 8) == 0) __builtin_amdgcn_s_barrier();
          if constexpr (SIDE) if (sd_i2 >= 0 && !(side.mode & 8)) side_words(sd_i2);   // issued two k-tiles ago:
        }                                                                                 // covered by this wait
        if constexpr (SIDE) {                            // (3 MFMAs between the dependent LDS reads and their use)
          constexpr int d = q - P3::B3;
          if constexpr (d == 3) {
            if (sd_i2 >= 0 && !(side.mode & 8)) {
              side_stat();
              side_lookup(0);
            }
          }
          if constexpr (d == 6 || d == 9 || d == 12 || d == 15) {
            if (sd_i2 >= 0 && !(side.mode & 8)) {
              side_store(sd_i2, d / 3 - 2);
              if constexpr (d < 15) side_lookup(d / 3 - 1);
            }
          }
          if constexpr (q == P3::SIDEQ) if (sd_go && sd_it < side.iters) side_issue();
        }
        constexpr int r = (HG_P3_ABL & 32) ? -1 : P3::nread(q);   // w0[0], x0[0..WI-1], w0[1..WJ-1]: their use order
        if constexpr (r == 0) w0[0] = rd(st ^ 1, wo0, 0);
        else if constexpr (r > 0 && r <= WI) x0[r - 1] = rd(st ^ 1, xo0, r - 1);
        else if constexpr (r > WI) w0[r - WI] = rd(st ^ 1, wo0, r - WI);
      }
      if constexpr ((q & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    });
  };

  // ---- prologue: tiles 0 and 1 in flight, tile 0 landed, its step-0 fragments in registers
  if constexpr (RS) {
#pragma unroll
    for (int q = 0; q < 16; ++q) rs_load(0, q);
#pragma unroll
    for (int q = 0; q < 16; ++q) rs_write(0, q);
#pragma unroll
    for (int q = 0; q < 16; ++q) rs_load(min(1, nk - 1), q);
    __syncthreads();
  } else {
    if constexpr (OP == HG_I8_DEQ) {
      // the statistics first (older than tile 0's pieces: the prologue's vmcnt below covers them); lanes past the
      // matrix edge fetch the last row / column (those slots are read only by the edge path, which does not use them)
      const uint32_t sb = lds_base + LDS_BYTES + SIDE_LDS;
      for (int c = wave; c < BM / 64; c += 4)
        glds4_sv_m0(rowStats, 4u * (uint32_t)min(m0 + 64 * c + lane, M - 1), sb + 256 * c);
      for (int c = wave; c < BN / 64; c += 4)
        glds4_sv_m0(colStats, 4u * (uint32_t)min(n0 + 64 * c + lane, N - 1), sb + 4 * BM + 256 * c);
      if (bias != nullptr && (N & 1) == 0)                 // bias as fp16 pairs (whole dwords: N even)
        for (int c = wave; c < BN / 128; c += 4)
          glds4_sv_m0(bias, 4u * (uint32_t)min(n0 / 2 + 64 * c + lane, N / 2 - 1), sb + 4 * BM + 4 * BN + 256 * c);
    }
#pragma unroll
    for (int i = 0; i < WI; ++i) dma_a(0, 0, i);
#pragma unroll
    for (int i = 0; i < WJ; ++i) dma_b(0, 0, i);
    const int k1 = min(1, nk - 1);
#pragma unroll
    for (int i = 0; i < WI; ++i) dma_a(k1, 1, i);
#pragma unroll
    for (int i = 0; i < WJ; ++i) dma_b(k1, 1, i);
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(WI + WJ) : "memory");   // tile 0 landed; tile 1 in flight
    if constexpr (SIDE) __builtin_amdgcn_s_waitcnt(0xC07F);          // (the side tables' LDS writes)
    __builtin_amdgcn_s_barrier();
  }
  if constexpr (TL) tl1 = hg_now();
#pragma unroll
  for (int f = 0; f < WJ; ++f) w0[f] = rd(0, wo0, f);
#pragma unroll
  for (int f = 0; f < WI; ++f) x0[f] = rd(0, xo0, f);

  if constexpr ((V & 8192) != 0) {
    if (nk == 1) {
      tile3(std::true_type{}, std::true_type{}, 0);
    } else {
      tile3(std::true_type{}, std::false_type{}, 0);
      for (int t = 1; t + 1 < nk; ++t) tile3(std::false_type{}, std::false_type{}, t);
      tile3(std::false_type{}, std::true_type{}, nk - 1);
    }
  } else {
    half1(std::true_type{}, 0);
    for (int t = 0; t + 1 < nk; ++t) {
      half2(std::false_type{}, t, t & 1);
      half1(std::false_type{}, t + 1);
    }
    half2(std::true_type{}, nk - 1, (nk - 1) & 1);
  }
  wait_vmcnt0();                                          // no LDS-DMA may outlive the workgroup
  if constexpr (TL) tl2 = hg_now();
  // MFMA (asm, invisible to hipcc's hazard recognizer) -> v_accvgpr_read: pad the wait states by hand
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (SIDE) {
    // the pending side iteration (its loads are covered by the vmcnt(0) above) and the ones the loop had no room for
    // (the last k-tile shifted its predecessors' iterations into sd_i2 / sd_i1 and consumed neither)
    auto consume = [&](int it) {
      side_words(it);
      side_stat();
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        side_lookup(j);
        side_store(it, j);
      }
    };
    if (sd_i2 >= 0) consume(sd_i2);
    if (sd_i1 >= 0) consume(sd_i1);
    for (; sd_it < side.iters && !(side.mode & 64); ++sd_it) {     // (mode 64, lab: no tail)
      const uint32_t gd0 = side_gd(sd_it);
      if (gd0 >= (uint32_t)side.ndw) continue;
      const uint32_t blk = (gd0 * 8u) >> side.bs_shift;
      const hg_u32x4_t w = *reinterpret_cast<const hg_u32x4_t*>(side.packed + 4ull * gd0);
      const float am = side.nested ? __fadd_rn(__fmul_rn(s_c2[side.q8[blk]], side.absmax2[blk >> side.bs2_shift]), sd_off)
                                   : side.absmax[blk];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float2 p = s_pair[(w[j] >> (8 * i)) & 0xFF];
          v[2 * i] = __fmul_rn(p.x, am);
          v[2 * i + 1] = __fmul_rn(p.y, am);
        }
        reinterpret_cast<uint4*>(side.out)[gd0 + j] =
            make_uint4(cvt_pk<T16>(v[0], v[1]), cvt_pk<T16>(v[2], v[3]), cvt_pk<T16>(v[4], v[5]), cvt_pk<T16>(v[6], v[7]));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- epilogue: acc[j][i][r] = C[m0 + 128 wm + 16 i + fr][n0 + 128 wn + 16 j + 4 fg + r] -- four consecutive
  // columns of one row per accumulator: one 8-B store (16-bit outputs) or 16-B store (int32).  Full tiles (the common
  // case) store unconditionally; edge tiles check every row / column.
  // (the lane's fragment row / group recomputed from mbcnt, not kept live from the prologue: at 256 VGPRs the main
  // loop has no register to spare for them)
  const int lane_e = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int mb = m0 + 16 * WI * wm + (lane_e & 15), nb = n0 + 16 * WJ * wn + 4 * (lane_e >> 4);
  constexpr int OUT = (OP == HG_I8_I32) ? 4 : 2;
  const bool full = (m0 + BM <= M) && (n0 + BN <= N) && (((ldc * OUT) & 15) == 0) &&
                    (((uintptr_t)Cv & 15) == 0);
  auto value = [&](int j, int i, int r, int n, float rs) -> float {   // HG_I8_DEQ: mm_dequant of one element
    return (float)Io<fp16_t>::to_f32(mm_dequant_value(acc[j][i][r], rs, colStats[n], bias ? (float)bias[n] : 0.0f));
  };
  if constexpr (SPLIT) {
    // fp32 partials of this split: acc[j][i] = C[mb + 16 i][nb + 16 j .. +3], one 16-B store each (N % 4 == 0 on the
    // host rule), rows / columns past the edge skipped
    // Buffer stores (SGPR base, one 32-bit lane offset) of the accumulator AGPRs themselves: a 64-bit address and 4
    // data VGPRs per store need registers the main loop does not leave (the int32 form of this epilogue spilled, and
    // the builtin 8-B store form miscompiled to copies of element 0); edge elements go out of range (offset past
    // num_records: the store is dropped).  After the MFMA -> read pad above, like every other accumulator read.
    if constexpr (OP == HG_BF16 || OP == HG_FP16) {
      const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(ws + (long long)split * M * N, (short)0,
                                                                          (int)((long long)M * N * 4), 0x00020000);
#pragma unroll
      for (int i = 0; i < WI; ++i) {
        const int m = mb + 16 * i;
        const uint32_t rowoff = (uint32_t)m * (uint32_t)N * 4u;
#pragma unroll
        for (int j = 0; j < WJ; ++j) {
          const int n = nb + 16 * j;
          const uint32_t off = (m < M && n < N) ? rowoff + 4u * (uint32_t)n : 0x80000000u;
          // straight from the accumulator AGPRs (stores take AGPR data on gfx950): no VGPRs, no reads to schedule
          if constexpr ((V & HG_V_CWT) != 0)             // write-through: no dirty partials for the reduce's boundary
            asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen sc1" : : "a"(acc[j][i]), "v"(off), "s"(wr) : "memory");
          else
            asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen" : : "a"(acc[j][i]), "v"(off), "s"(wr) : "memory");
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  } else if (full && OUT == 2) {
    // 16-bit outputs of a full tile: staged through LDS so every global store writes whole 256-B row segments
    // (direct 8-B fragment stores put 16 rows x 32 B in one instruction: +4 us of epilogue per launch at 4096^2)
    __syncthreads();                                   // every wave is past its last stage read
    uint8_t* ep = smem + wave * (16 * WI * EPI_PITCH);
    // HG_I8_DEQ: the lane's row / column statistics and bias loaded once, up front (the fragment registers are free
    // now): 8 row scales, 8 x 4 column scales (16-B loads: nb % 4 == 0) and 8 x 4 bias halves.  Loading them per
    // accumulator (256 dependent L1 loads per lane) cost ~24 us of fixed epilogue per launch.
    // (round 4: from the LDS copy the prologue's DMA made, not from global memory at this point)
    float rsv[WI];
    f32x4_t csv[WJ];
    uint2 bsv[WJ];
    if constexpr (OP == HG_I8_DEQ) {
      const uint8_t* sst = smem + LDS_BYTES + SIDE_LDS;
      const int rl = 16 * WI * wm + (lane_e & 15), cl = 16 * WJ * wn + 4 * (lane_e >> 4);
#pragma unroll
      for (int i = 0; i < WI; ++i) rsv[i] = *reinterpret_cast<const float*>(sst + 4 * (rl + 16 * i));
#pragma unroll
      for (int j = 0; j < WJ; ++j) {
        csv[j] = *reinterpret_cast<const f32x4_t*>(sst + 4 * BM + 4 * (cl + 16 * j));
        if ((N & 1) == 0)
          bsv[j] = bias ? *reinterpret_cast<const uint2*>(sst + 4 * BM + 4 * BN + 2 * (cl + 16 * j)) : make_uint2(0u, 0u);
        else
          bsv[j] = bias ? *reinterpret_cast<const uint2*>(bias + nb + 16 * j) : make_uint2(0u, 0u);
      }
    }
    auto convert = [&](int i, int j) {                   // accumulator (j, i) -> its 8 B of the wave's staging rows
      uint2 v;
      if constexpr (OP == HG_BF16 || OP == HG_FP16) {
        using T = typename std::conditional<OP == HG_BF16, bf16_t, fp16_t>::type;
        v.x = cvt_pk<T>(acc[j][i][0], acc[j][i][1]);
        v.y = cvt_pk<T>(acc[j][i][2], acc[j][i][3]);
      } else if constexpr (OP == HG_I8_DEQ) {
        auto bf = [&](uint32_t w, int hi) { return (float)__builtin_bit_cast(fp16_t, (uint16_t)(w >> (16 * hi))); };
        v.x = mm_dequant_pair(acc[j][i][0], acc[j][i][1], rsv[i], csv[j][0], csv[j][1], bf(bsv[j].x, 0), bf(bsv[j].x, 1));
        v.y = mm_dequant_pair(acc[j][i][2], acc[j][i][3], rsv[i], csv[j][2], csv[j][3], bf(bsv[j].y, 0), bf(bsv[j].y, 1));
      }
      *reinterpret_cast<uint2*>(ep + (16 * i + (lane_e & 15)) * EPI_PITCH + 2 * (16 * j + 4 * (lane_e >> 4))) = v;
    };
    uint8_t* cbase = reinterpret_cast<uint8_t*>(Cv) + ((long long)(m0 + 16 * WI * wm) * ldc + n0 + 16 * WJ * wn) * 2;
    constexpr int CPR = 2 * WJ, RPI = 64 / CPR;          // 16-B chunks per output row, rows per wave instruction
    auto store_rows = [&](int it) {                      // store instruction `it`: rows RPI it .. RPI it + RPI - 1
      const int row = RPI * it + lane_e / CPR, c16 = lane_e % CPR;
      const uint4 v = *reinterpret_cast<const uint4*>(ep + row * EPI_PITCH + 16 * c16);
      uint8_t* dst = cbase + (long long)row * ldc * 2 + 16 * c16;
      if constexpr ((V & HG_V_CWT) != 0)                 // device-scope write-through: C leaves no dirty L2 lines
        asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(dst), "v"((hg_u32x4_t){v.x, v.y, v.z, v.w}) : "memory");
      else
        *reinterpret_cast<uint4*>(dst) = v;
    };
    if ((V & HG_V_EPI) != 0 && (long long)ldc * 2 * 16 * WI < 0x7FFFFFFFLL) {
      // per 16-row group i: convert + stage its WJ accumulators; group i - 1 (staged and drained by lgkmcnt(0) after its
      // last write) is read back and stored in SPG instructions spread over group i's conversions.  The stores go through a
      // buffer resource on the wave's output corner: one lane-offset VGPR for all of them, the row step in an SGPR (a
      // 64-bit address per store made the 256 x 256 bf16 kind spill here)
      constexpr int SPG = 16 / RPI, EVERY = WJ / SPG;
      // (TL lab ablation g_hg_tl_nostore: zero records -- every C store is issued and dropped, no memory write)
      const int crec = (TL && g_hg_tl_nostore) ? 0 : 0x7FFFFFFF;
      const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(cbase, (short)0, crec, 0x00020000);
      const uint32_t ldc2 = (uint32_t)ldc * 2u;
      const uint32_t loff = (uint32_t)(lane_e / CPR) * ldc2 + 16u * (uint32_t)(lane_e % CPR);
      // store instruction `it` = rows RPI it .. + RPI - 1 of the wave's region; its read-back is issued one slot ahead of
      // its store, so the store finds the data landed (no LDS round trip exposed per store)
      auto read_rows = [&](int it) -> hg_u32x4_t {
        return *reinterpret_cast<const hg_u32x4_t*>(ep + (RPI * it + lane_e / CPR) * EPI_PITCH + 16 * (lane_e % CPR));
      };
      auto store_rows_v = [&](const hg_u32x4_t& v, int it) {
        const int soff = (int)((uint32_t)(RPI * it) * ldc2);
        // device-scope write-through (sc1, 16): no dirty C lines left; nt (2): streaming hint
        constexpr int AUX = ((V & HG_V_CWT) != 0 ? 16 : 0) | ((V & HG_V_CNT) != 0 ? 2 : 0);
        __builtin_amdgcn_raw_buffer_store_b128(v, cr, (int)loff, soff, AUX);
      };
      hg_u32x4_t pv = {0u, 0u, 0u, 0u};
      int pk = -1;
      auto slot = [&](int it) {                          // store the pending rows, read `it` (-1: only store)
        if (pk >= 0) store_rows_v(pv, pk);
        if (it >= 0) pv = read_rows(it);
        pk = it;
      };
#pragma unroll
      for (int i = 0; i < WI; ++i) {
#pragma unroll
        for (int j = 0; j < WJ; ++j) {
          convert(i, j);
          __builtin_amdgcn_sched_barrier(0);             // one accumulator at a time: no VGPR burst that displaces AGPRs
          if (i > 0 && j % EVERY == EVERY - 1) {
            slot(SPG * (i - 1) + j / EVERY);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);              // lgkmcnt(0): group i staged (the wave reads back only its own rows)
      }
#pragma unroll
      for (int s = 0; s < SPG; ++s) slot(SPG * (WI - 1) + s);
      slot(-1);
    } else {
#pragma unroll
      for (int i = 0; i < WI; ++i) {
#pragma unroll
        for (int j = 0; j < WJ; ++j) {
          convert(i, j);
          __builtin_amdgcn_sched_barrier(0);             // one accumulator at a time: no VGPR burst that displaces AGPRs
        }
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);                // lgkmcnt(0): the wave reads back only its own region
#pragma unroll 8
      for (int it = 0; it < 16 * WI / RPI; ++it) store_rows(it);
    }
  } else if (full) {
    if constexpr (OP == HG_I8_I32) {                   // int32: one 16-B store per accumulator already
#pragma unroll
      for (int i = 0; i < WI; ++i) {
        const long long m = mb + 16 * i;
#pragma unroll
        for (int j = 0; j < WJ; ++j) {
          const int n = nb + 16 * j;
          *reinterpret_cast<hg_i32x4_t*>(reinterpret_cast<int32_t*>(Cv) + m * ldc + n) = acc[j][i];
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      const int m = mb + 16 * i;
      const long long mc = min(m, M - 1);
      float rs = 0.f;
      if constexpr (OP == HG_I8_DEQ) rs = rowStats[mc];
#pragma unroll
      for (int j = 0; j < WJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = nb + 16 * j + r;
          if (m < M && n < N) {
            if constexpr (OP == HG_BF16) reinterpret_cast<bf16_t*>(Cv)[mc * ldc + n] = Io<bf16_t>::from_f32(acc[j][i][r]);
            else if constexpr (OP == HG_FP16) reinterpret_cast<fp16_t*>(Cv)[mc * ldc + n] = Io<fp16_t>::from_f32(acc[j][i][r]);
            else if constexpr (OP == HG_I8_DEQ)
              reinterpret_cast<fp16_t*>(Cv)[mc * ldc + n] =
                  mm_dequant_value(acc[j][i][r], rs, colStats[n], bias ? (float)bias[n] : 0.0f);
            else reinterpret_cast<int32_t*>(Cv)[mc * ldc + n] = acc[j][i][r];
          }
          __builtin_amdgcn_sched_barrier(0);
        }
    }
  }
  (void)value;
  if constexpr ((V & HG_V_TAIL) != 0) {
    // (a bare s_barrier, no fence: every wave is past its last LDS read -- the last k-tile's fragments fed its MFMAs,
    // its staging rows fed its stores -- before any wave writes its table over stage / staging bytes; a __syncthreads
    // release fence would also wait for the C stores)
    __builtin_amdgcn_s_barrier();
    hg_side_tail<T16>(side, smem + wave * (16 * WI * EPI_PITCH), lane_e, blockIdx.x * 4u + (uint32_t)wave,
                      gridDim.x * 4u);
  }
  if constexpr (TL) {
    const unsigned long long tl3 = hg_now();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long tl4 = hg_now();
    if (lane == 0 && g_hg_tl != nullptr) {
      unsigned long long* o = g_hg_tl + ((long long)blockIdx.x * 4 + wave) * 8;
      o[0] = tl0; o[1] = tl1; o[2] = tl2; o[3] = tl3; o[4] = tl4; o[5] = (unsigned long long)wgs;
      o[6] = (unsigned long long)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15);   // HW_REG_XCC_ID: the physical XCD
    }
  }
}

// Host rule: k bytes (k * element size) % 128 == 0, 16-B aligned rows and bases, and every lane offset
// (row * ld * element size bytes) below 4 GiB.
bool hgemm_fits(int m, int n, int k, long long lda, long long ldb, const void* A, const void* B, int elem) {
  if (m <= 0 || n <= 0 || k <= 0 || ((long long)k * elem) % 128 != 0) return false;
  if (((lda * elem) & 15) || ((ldb * elem) & 15) || lda < k || ldb < k) return false;
  if (((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return false;
  if ((long long)(m - 1) * lda * elem + (long long)k * elem > 0xFFFFFFFFLL) return false;
  if ((long long)(n - 1) * ldb * elem + (long long)k * elem > 0xFFFFFFFFLL) return false;
  return true;
}

long long hgemm_tiles(int m, int n) { return (long long)((m + HG_BM - 1) / HG_BM) * ((n + HG_BN - 1) / HG_BN); }

// Launch plan: tile shape (256 x 256, 256 x 128 or 128 x 256) and split-K, chosen by cost in units of one 256 x 256
// k-tile time (~1.37 us): rounds of workgroups on the CUs x k-tiles per workgroup x the shape's k-tile time (a half-width
// tile does half the MFMAs per k-tile with relatively more copies and fragment reads: HG_HALF_KT), plus, per split, the
// fp32 partials it writes and the reduce reads back (8 bytes per output at ~5 TB/s).  Grids of >= HG_SPLIT_TILES tiles
// are not split.  The full 256 x 256 tile wins wherever its grid fills the chip (the metric shape: 256 tiles, one
// round); the half-width tiles fill the chip where the 256 x 256 grid would be half empty (2048 x 4096: 128 tiles ->
// 256 tiles of 256 x 128, no split-K) or where fewer than 256 rows waste half a 256-row tile (96..128 tokens).
// Round 3's split rule (splits = CUs / tiles) could also overshoot the CU count by a few workgroups -- 43 tiles x 6 =
// 258 workgroups, a second round for 2 of them (256 x 11008 x 4096: 89 us against 58 on the library GEMM,
// tools/route_probe3.py, profiles/lab/r04_routes_before.txt).
constexpr int HG_SPLIT_TILES = 192, HG_SPLIT_MIN_KT = 8, HG_SPLIT_MAX = 8;
constexpr double HG_HALF_KT = 0.6;
// the 128 x 128 tile (round 5, 16-bit kinds, no side dequantise): a quarter of the 256 x 256 tile's MFMAs per k-tile with
// twice its copies and fragment reads per MFMA; its k-tile time in 256 x 256 k-tile units (lab-calibrated,
// chgemm_set_quarter_tile)
static Knob<double> g_hg_quarter_kt{0.40};
static Knob<int> g_hg_quarter{1};             // 0 = never, 1 = by cost (default), 2 = forced where allowed (tests / A-B)
struct HgPlan {
  int wi, wj, splits, kchunk;
};
int device_cu_count();   // CUs of the current device (cached; gemv4bit.hip)
static HgPlan hgemm_plan(int m, int n, int k, int elem, bool allow_split, bool full_tiles_only,
                         bool allow_quarter = false) {
  const int nkt = (int)((long long)k * elem / 128);
  int cus = device_cu_count();
  if (cus <= 0) cus = 256;
  const double part_kt = (double)m * n * 8.0 / 5.0e12 / 1.37e-6;   // one split's partial traffic, in k-tile times
  static const int shapes[4][2] = {{8, 8}, {8, 4}, {4, 8}, {4, 4}};
  const bool quarter = allow_quarter && !full_tiles_only && g_hg_quarter != 0;
  const bool forced = quarter && g_hg_quarter == 2;
  HgPlan best{8, 8, 1, nkt};
  double best_cost = 1e300;
  for (int si = forced ? 3 : 0; si < (full_tiles_only ? 1 : quarter ? 4 : 3); ++si) {
    const int wi = shapes[si][0], wj = shapes[si][1];
    const double tkt = (wi == 8 && wj == 8) ? 1.0 : (wi == 4 && wj == 4) ? g_hg_quarter_kt.load() : HG_HALF_KT;
    const long long tiles = (long long)((m + 32 * wi - 1) / (32 * wi)) * ((n + 32 * wj - 1) / (32 * wj));
    double cost = (double)((tiles + cus - 1) / cus) * nkt * tkt;
    if (cost < best_cost) {
      best_cost = cost;
      best = HgPlan{wi, wj, 1, nkt};
    }
    if (!allow_split || tiles >= HG_SPLIT_TILES || n % 4) continue;
    for (int sp = 2; sp <= HG_SPLIT_MAX; ++sp) {
      const int kchunk = (nkt + sp - 1) / sp;
      if (kchunk < HG_SPLIT_MIN_KT) break;
      const int splits = (nkt + kchunk - 1) / kchunk;
      cost = (double)((tiles * splits + cus - 1) / cus) * kchunk * tkt + part_kt * splits;
      if (cost < best_cost) {
        best_cost = cost;
        best = HgPlan{wi, wj, splits, kchunk};
      }
    }
  }
  return best;
}
long long hgemm_workspace_bytes(int m, int n, int k, int elem) {
  // the larger of the plans with and without the 128 x 128 tile: a side-dequantise launch (chgemm_tn_pf_*) plans
  // without it and must find its partials' room too
  const HgPlan pq = hgemm_plan(m, n, k, elem, true, false, elem == 2), pn = hgemm_plan(m, n, k, elem, true, false, false);
  const int splits = std::max(pq.splits, pn.splits);
  return splits > 1 ? (long long)splits * m * n * (long long)sizeof(float) : 0;
}

// side: the next weight's dequantise to run inside this launch (nullptr: none); its per-workgroup share and step spacing
// are set here from the grid
template <int OP, int V, int WI, int WJ, bool SIDE>
static void hgemm_launch_side(const HgPlan& pl, int m, int n, int k, const void* A, long long lda, const void* B,
                              long long ldb, void* C, long long ldc, const float* rowStats, const float* colStats,
                              const fp16_t* bias, float* ws, const HgSide& sd) {
  const unsigned tiles = (unsigned)(((m + 32 * WI - 1) / (32 * WI)) * ((n + 32 * WJ - 1) / (32 * WJ)));
  if (pl.splits > 1) {
    if constexpr (OP == HG_BF16 || OP == HG_FP16)
      hipLaunchKernelGGL((k_hgemm<OP, V, true, WI, WJ, SIDE>), dim3(tiles * pl.splits), dim3(HG_THREADS), 0,
                         current_stream(), m, n, k, A, lda, B, ldb, C, ldc, rowStats, colStats, bias, ws, pl.splits,
                         pl.kchunk, sd);
  } else {
    hipLaunchKernelGGL((k_hgemm<OP, V, false, WI, WJ, SIDE>), dim3(tiles), dim3(HG_THREADS), 0, current_stream(), m, n,
                       k, A, lda, B, ldb, C, ldc, rowStats, colStats, bias, nullptr, 1, pl.kchunk, sd);
  }
}

// false: a side dequantise was asked for that this kind / shape does not run (nothing launched)
template <int OP, int V, int WI, int WJ>
static bool hgemm_launch_shape(const HgPlan& pl, int m, int n, int k, const void* A, long long lda, const void* B,
                               long long ldb, void* C, long long ldc, const float* rowStats, const float* colStats,
                               const fp16_t* bias, float* ws, const HgSide* side) {
  // the tail form (default, round 6): the launched 16-bit kind, every tile shape; chgemm_set_side_mode(128 | ...) keeps
  // the round-4 in-loop form below
  if constexpr ((OP == HG_BF16 || OP == HG_FP16) && V == (HG_V | HG_V_CWT | HG_V_EPI)) {
    if (side && !(g_side_mode & 128)) {
      HgSide sd = *side;
      sd.mode = g_side_mode;
      hgemm_launch_side<OP, V | HG_V_TAIL, WI, WJ, false>(pl, m, n, k, A, lda, B, ldb, C, ldc, rowStats, colStats, bias,
                                                          ws, sd);
      return true;
    }
  }
  if constexpr ((OP == HG_BF16 || OP == HG_FP16) && (V & 8192) != 0 && !(WI == 4 && WJ == 4)) {
    if (side) {
      const long long wgs = (long long)((m + 32 * WI - 1) / (32 * WI)) * ((n + 32 * WJ - 1) / (32 * WJ)) * pl.splits;
      HgSide sd = *side;
      sd.mode = g_side_mode;
      const long long per = (sd.ndw + wgs - 1) / wgs;
      sd.iters = (int)((per + 4 * HG_THREADS - 1) / (4 * HG_THREADS));   // 4 dwords per lane per iteration
      sd.per_wg = sd.iters * 4 * HG_THREADS;
      // one side step every `every` k-tiles of the k-tiles that have a B3 (all but a workgroup's last)
      const int steps = pl.kchunk - 1;
      sd.every = steps > 0 ? std::max(1, (steps + sd.iters - 1) / sd.iters) : 1;
      // (the side form keeps the round-4 epilogue: with the side's state live the interleaved one spills)
      hgemm_launch_side<OP, (V & ~(HG_V_EPI | HG_V_CNT | HG_V_TL)), WI, WJ, true>(pl, m, n, k, A, lda, B, ldb, C, ldc, rowStats, colStats, bias,
                                                           ws, sd);
      return true;
    }
  }
  if (side) return false;           // (never launch the GEMM without the side dequantise the caller counts on)
  hgemm_launch_side<OP, V, WI, WJ, false>(pl, m, n, k, A, lda, B, ldb, C, ldc, rowStats, colStats, bias, ws, HgSide{});
  return true;
}

template <int OP>
int hgemm_launch(int m, int n, int k, const void* A, long long lda, const void* B, long long ldb, void* C, long long ldc,
                 const float* rowStats = nullptr, const float* colStats = nullptr, const fp16_t* bias = nullptr,
                 float* ws = nullptr, long long ws_bytes = 0, const HgSide* side = nullptr) {
  if (!hgemm_fits(m, n, k, lda, ldb, A, B, HgOpT<OP>::ELEM) || ldc < n) return 1;
  // the dequant epilogue reads 4 column scales / 4 bias halves per 16-B / 8-B load
  if (OP == HG_I8_DEQ && (((uintptr_t)colStats & 15) || ((uintptr_t)bias & 7))) return 1;
  constexpr bool FP = OP == HG_BF16 || OP == HG_FP16;
  // int8 (HG_I8_DEQ) runs the 256 x 256 tile only
  const bool full_only = !FP;
  if (side && !FP) return 1;
  // (the 128 x 128 tile: 16-bit kinds without a side dequantise or with its tail form -- the in-loop form is not built
  // for it)
  const bool quarter = FP && (side == nullptr || (!(g_side_mode & 128) && g_hg_cwt == 1 && g_hg_epi));
  HgPlan pl = hgemm_plan(m, n, k, HgOpT<OP>::ELEM, FP, full_only, quarter);
  if (pl.splits > 1 && (ws == nullptr || ((uintptr_t)ws & 15) ||
                        ws_bytes < (long long)pl.splits * m * n * (long long)sizeof(float)))
    pl = hgemm_plan(m, n, k, HgOpT<OP>::ELEM, false, full_only, quarter);   // no (large enough) workspace: no split
  // variant bits of the launched kernel: write-through C (g_hg_cwt) and the interleaved epilogue (g_hg_epi, with it)
  auto by_shape = [&](auto vtag) {
    constexpr int VV = decltype(vtag)::value;
    if (pl.wi == 8 && pl.wj == 8)
      return hgemm_launch_shape<OP, VV, 8, 8>(pl, m, n, k, A, lda, B, ldb, C, ldc, rowStats, colStats, bias, ws, side);
    if constexpr (FP) {
      if (pl.wi == 8) return hgemm_launch_shape<OP, VV, 8, 4>(pl, m, n, k, A, lda, B, ldb, C, ldc, rowStats, colStats, bias, ws, side);
      if (pl.wj == 8) return hgemm_launch_shape<OP, VV, 4, 8>(pl, m, n, k, A, lda, B, ldb, C, ldc, rowStats, colStats, bias, ws, side);
      return hgemm_launch_shape<OP, VV, 4, 4>(pl, m, n, k, A, lda, B, ldb, C, ldc, rowStats, colStats, bias, ws, side);
    }
    return false;
  };
  bool launched = true;
#ifdef BNB_LAB
  if (FP && g_hg_tl_on && g_hg_cwt == 1 && g_hg_epi && pl.wi == 8 && pl.wj == 8 && !side) {   // lab timeline
    // (16-bit kinds only: on the int8 body the stamps' registers spilled)
    if constexpr (FP)
      launched = hgemm_launch_shape<OP, HG_V | HG_V_CWT | HG_V_EPI | HG_V_TL, 8, 8>(pl, m, n, k, A, lda, B, ldb, C, ldc,
                                                                                  rowStats, colStats, bias, ws, nullptr);
  } else
#endif
  if (g_hg_cwt == 2 && g_hg_epi && pl.wi == 8 && pl.wj == 8) {   // the lab's nt arm: full tile only
    launched = hgemm_launch_shape<OP, HG_V | HG_V_CWT | HG_V_EPI | HG_V_CNT, 8, 8>(pl, m, n, k, A, lda, B, ldb, C, ldc,
                                                                                 rowStats, colStats, bias, ws, side);
  } else if (g_hg_cwt && g_hg_epi) {
    launched = by_shape(std::integral_constant<int, HG_V | HG_V_CWT | HG_V_EPI>{});
  } else if (g_hg_cwt) {
    launched = by_shape(std::integral_constant<int, HG_V | HG_V_CWT>{});
  } else {
    launched = by_shape(std::integral_constant<int, HG_V>{});
  }
  if (!launched) return 1;          // (a side dequantise this kind / shape does not run: nothing launched)
  if constexpr (FP) {
    using T = typename std::conditional<OP == HG_BF16, bf16_t, fp16_t>::type;
    if (pl.splits > 1) launch_splitk_rows_reduce<T>(ws, pl.splits, m, n, reinterpret_cast<T*>(C), (int)ldc);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error((int)e, "k_hgemm launch");
    return 2;
  }
  return 0;
}

// int8 row-major igemmlt on the 4-wave kernel (int8.hip's launch_igemm takes it for large tile grids): 0 = launched,
// 1 = not covered (the caller's kernels run), 2 = launch error
int igemm_4wave(int m, int n, int k, const int8_t* A, long long lda, const int8_t* B, long long ldb, void* C,
                long long ldc, bool dequant, const float* rowStats, const float* colStats, const fp16_t* bias) {
  // HG_I8_I32 is not launched: its epilogue needs spill registers, and a spill the allocator places between the last
  // (inline-asm, hazard-invisible) MFMAs and the wait-state pad reads accumulators before they are written (wrong
  // int32 at ragged shapes, caught by tests/test_hgemm_gpu.py).  The launched kinds compile spill-free.
  if (!dequant) return 1;
  return hgemm_launch<HG_I8_DEQ>(m, n, k, A, lda, B, ldb, C, ldc, rowStats, colStats, bias);
}

}  // namespace bnb

extern "C" {

// [additive] C[m, n] = A[m, k] . W[n, k]^T, row-major, bf16 / fp16 in and out, fp32 accumulation, on the hand-written
// k_hgemm (the GEMM of the large-prefill 4-bit path after cdequantize_blockwise_* into W; replaces the F.linear of
// ref:python_src_quants/autograd/_functions.py:507).  Returns 0 = launched, 1 = shape / alignment not supported
// (k % 64, 16-B aligned rows; nothing launched), 2 = launch error (cget_last_error*).
int chgemm_tn_bf16(int m, int n, int k, const bf16_t* A, int lda, const bf16_t* W, int ldw, bf16_t* C, int ldc) {
  BNB_RANGE("chgemm_tn_bf16");
  return bnb::hgemm_launch<bnb::HG_BF16>(m, n, k, A, lda, W, ldw, C, ldc);
}
int chgemm_tn_fp16(int m, int n, int k, const fp16_t* A, int lda, const fp16_t* W, int ldw, fp16_t* C, int ldc) {
  BNB_RANGE("chgemm_tn_fp16");
  return bnb::hgemm_launch<bnb::HG_FP16>(m, n, k, A, lda, W, ldw, C, ldc);
}
// [additive] the same with a caller workspace for split-K on small tile grids (< 192 tiles of 256 x 256: fp32
// partials, summed in split order by one more launch; same bits on every call).  chgemm_tn_workspace_bytes gives the
// bytes the shape needs (0: no split); a smaller workspace runs the unsplit kernel.
int chgemm_tn_ws_bf16(int m, int n, int k, const bf16_t* A, int lda, const bf16_t* W, int ldw, bf16_t* C, int ldc,
                      float* ws, long long ws_bytes) {
  BNB_RANGE("chgemm_tn_ws_bf16");
  return bnb::hgemm_launch<bnb::HG_BF16>(m, n, k, A, lda, W, ldw, C, ldc, nullptr, nullptr, nullptr, ws, ws_bytes);
}
int chgemm_tn_ws_fp16(int m, int n, int k, const fp16_t* A, int lda, const fp16_t* W, int ldw, fp16_t* C, int ldc,
                      float* ws, long long ws_bytes) {
  BNB_RANGE("chgemm_tn_ws_fp16");
  return bnb::hgemm_launch<bnb::HG_FP16>(m, n, k, A, lda, W, ldw, C, ldc, nullptr, nullptr, nullptr, ws, ws_bytes);
}
// [additive] chgemm_tn_ws_* that also dequantises the NEXT 4-bit weight inside the same launch (see HgSide): next_n
// elements (% 32 == 0, below 2^31) of packed 4-bit `next_packed` (16-B aligned; fp4 = 1: FP4 code, else NF4) with fp32
// block statistics `next_absmax` (next_q8 == NULL), or nested ones (next_q8 / next_code2 / next_absmax2 / next_offset,
// blocksize2), into `next_out` (16-B aligned, the GEMM's element type) -- exactly cdequantize_blockwise_*_{nf4,fp4} /
// the nested dequantise of that weight, run in the GEMM's shadow (the reference's dequantize_4bit of the following
// layer, ref:python_src_quants/functional.py:1329).  Returns 0 = launched, 1 = not supported (nothing launched: run the
// dequantise and the plain GEMM), 2 = launch error.
static int hgemm_pf(int op, int m, int n, int k, const void* A, int lda, const void* W, int ldw, void* C, int ldc,
                    float* ws, long long ws_bytes, const uint8_t* next_packed, const float* next_absmax,
                    const uint8_t* next_q8, const float* next_code2, const float* next_absmax2, const float* next_offset,
                    int fp4, int blocksize, int blocksize2, long long next_n, void* next_out) {
  const bool nested = next_q8 != nullptr;
  // (whole 32-weight groups, 16-B aligned operands, statistics blocks of >= 32: each lane's 4 packed dwords share one)
  if (next_n <= 0 || next_n % 32 || next_n >= (1LL << 31) || !next_packed || !next_out || ((uintptr_t)next_packed & 15) ||
      ((uintptr_t)next_out & 15) || blocksize < 32 || (blocksize & (blocksize - 1)))
    return 1;
  if (nested ? (!next_code2 || !next_absmax2 || !next_offset || blocksize2 <= 0 || (blocksize2 & (blocksize2 - 1)))
             : !next_absmax)
    return 1;
  bnb::HgSide sd{next_packed, next_absmax, next_q8, next_code2, next_absmax2, next_offset, next_out, next_n / 8,
                 0, 0, 1, __builtin_ctz(blocksize), nested ? __builtin_ctz(blocksize2) : 0, nested ? 1 : 0, fp4 ? 1 : 0,
                 0};
  return op == bnb::HG_BF16
             ? bnb::hgemm_launch<bnb::HG_BF16>(m, n, k, A, lda, W, ldw, C, ldc, nullptr, nullptr, nullptr, ws, ws_bytes, &sd)
             : bnb::hgemm_launch<bnb::HG_FP16>(m, n, k, A, lda, W, ldw, C, ldc, nullptr, nullptr, nullptr, ws, ws_bytes, &sd);
}
int chgemm_tn_pf_bf16(int m, int n, int k, const bf16_t* A, int lda, const bf16_t* W, int ldw, bf16_t* C, int ldc,
                      float* ws, long long ws_bytes, const uint8_t* next_packed, const float* next_absmax,
                      const uint8_t* next_q8, const float* next_code2, const float* next_absmax2,
                      const float* next_offset, int fp4, int blocksize, int blocksize2, long long next_n,
                      bf16_t* next_out) {
  BNB_RANGE("chgemm_tn_pf_bf16");
  return hgemm_pf(bnb::HG_BF16, m, n, k, A, lda, W, ldw, C, ldc, ws, ws_bytes, next_packed, next_absmax, next_q8,
                  next_code2, next_absmax2, next_offset, fp4, blocksize, blocksize2, next_n, next_out);
}
int chgemm_tn_pf_fp16(int m, int n, int k, const fp16_t* A, int lda, const fp16_t* W, int ldw, fp16_t* C, int ldc,
                      float* ws, long long ws_bytes, const uint8_t* next_packed, const float* next_absmax,
                      const uint8_t* next_q8, const float* next_code2, const float* next_absmax2,
                      const float* next_offset, int fp4, int blocksize, int blocksize2, long long next_n,
                      fp16_t* next_out) {
  BNB_RANGE("chgemm_tn_pf_fp16");
  return hgemm_pf(bnb::HG_FP16, m, n, k, A, lda, W, ldw, C, ldc, ws, ws_bytes, next_packed, next_absmax, next_q8,
                  next_code2, next_absmax2, next_offset, fp4, blocksize, blocksize2, next_n, next_out);
}
long long chgemm_tn_workspace_bytes(int m, int n, int k) { return bnb::hgemm_workspace_bytes(m, n, k, 2); }
// [additive, testing] the launch plan of chgemm_tn_ws_* for (m, n, k) with enough workspace: out = {WI, WJ, splits,
// k-tiles per split}; the output tile is 32 WI x 32 WJ (256 x 256, 256 x 128 or 128 x 256)
void chgemm_tn_plan(int m, int n, int k, int* out) {
  BNB_RANGE("chgemm_tn_plan");
  const bnb::HgPlan pl = bnb::hgemm_plan(m, n, k, 2, true, false, true);
  out[0] = pl.wi;
  out[1] = pl.wj;
  out[2] = pl.splits;
  out[3] = pl.kchunk;
}
// [additive, testing] the side dequantise's A/B bits (HgSide::mode); returns the previous setting
// [additive, testing] 1 (default): k_hgemm stores C and its split-K partials write-through (sc1), 0: write-back;
// 2: write-through + non-temporal (the 256 x 256 tile's interleaved epilogue; others as 1); returns the previous setting
int chgemm_set_c_store(int wt) {
  const int prev = bnb::g_hg_cwt;
  bnb::g_hg_cwt = (wt >= 0 && wt <= 2) ? wt : 1;
  return prev;
}
// [additive, testing] the 128 x 128 tile of the 16-bit k_hgemm: mode 0 = never, 1 = by the plan's cost (default), 2 = forced
// wherever allowed; kt_x1000 > 0 sets its k-tile time in 256 x 256 k-tile units x 1000 (the cost model); returns the
// previous mode
int chgemm_set_quarter_tile(int mode, int kt_x1000) {
  const int prev = bnb::g_hg_quarter;
  bnb::g_hg_quarter = (mode >= 0 && mode <= 2) ? mode : 1;
  if (kt_x1000 > 0) bnb::g_hg_quarter_kt = kt_x1000 / 1000.0;
  return prev;
}
#ifdef BNB_LAB
// [lab build only (make lab), not in the header] per-wave timeline of the 256 x 256 k_hgemm (HG_V_TL): buf = 8 u64 per
// wave (nullptr: off); _nswap / _nostore: the XCD N-tile swap and the dropped-store ablation (wrong results: lab only)
int chgemm_timeline_nswap(int v) {
  return hipMemcpyToSymbol(HIP_SYMBOL(bnb::g_hg_tl_nswap), &v, sizeof(v)) == hipSuccess ? 0 : 1;
}
int chgemm_timeline_nostore(int v) {
  return hipMemcpyToSymbol(HIP_SYMBOL(bnb::g_hg_tl_nostore), &v, sizeof(v)) == hipSuccess ? 0 : 1;
}
int chgemm_timeline(unsigned long long* buf) {
  bnb::g_hg_tl_on = buf != nullptr;
  return hipMemcpyToSymbol(HIP_SYMBOL(bnb::g_hg_tl), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif
// [additive, testing] 1 (default): the interleaved 16-bit epilogue (HG_V_EPI, with write-through C), 0: the round-4 one
// (convert and stage everything, then store); returns the previous setting
int chgemm_set_epilogue(int v) {
  const int prev = bnb::g_hg_epi;
  bnb::g_hg_epi = v ? 1 : 0;
  return prev;
}
// [additive, testing] the side dequantise's load / store hint: bit 1 = non-temporal (default); the lab build also takes
// its ablation bits (2 / 8 / 16 / 32 / 64: wrong weights, timing only), the product library masks them off
int chgemm_set_side_mode(int v) {
  BNB_RANGE("chgemm_set_side_mode");
  const int prev = bnb::g_side_mode;
#ifdef BNB_LAB
  bnb::g_side_mode = v;
#else
  bnb::g_side_mode = v & (1 | 128);
#endif
  return prev;
}

}  // extern "C"
