// 4-bit GEMV (decode path, M == 1) for gfx950.
//
// Replaces cgemm_4bit_inference_naive_{fp16,bf16,fp32}   ref:sycl/pythonInterface.cpp:408-415
//   -> gemm_4bit_inference_naive<T,BITS>                ref:sycl/sycl_code/op_gemm.cpp:893-929
//   -> kgemm_4bit_inference_naive<T,128,BITS>           ref:sycl/sycl_code/kernel_gemm.cpp:1271-1388
// Called by gemv_4bit (ref:python_src_quants/functional.py:1961-2060):
//   out[r] = sum_k A[k] * datatype[q(r,k)] * absmax[(2*ldb*r + k) / blocksize]
//   m = rows of W (out_features), k = in_features, B rows are ldb bytes apart.
// Numerics: the reference forms the weight in T precision (Q8, kernel_gemm.cpp:1336-1343);
// here every product is fp32 and each 32-element chunk is scaled once by its absmax
// (sum_k a_k*code_k)*absmax, accumulated in fp32.
//
// Design (MI355X, HBM-bound: 0.5 B of weights per MAC): one wave owns R output rows;
// lane l streams 16-B packed chunks c = l, l+64, ... of each row (1 KiB contiguous per wave
// instruction, non-temporal: weights are read exactly once), keeps the matching 32 activations
// in registers (shared by the R rows), looks bytes up in a 256-entry LDS pair table
// (byte -> {code[hi], code[lo]}), and reduces the R partial sums across the wave at the end.
#include "common.hpp"
#include "gemm_common.hpp"
#include "gemv_common.hpp"

namespace bnb {

template <typename T> struct XChunk;   // 32 activations of one chunk -> fp32 registers
template <> struct XChunk<bf16_t> {
  __device__ static __forceinline__ void load(const bf16_t* p, float (&x)[32]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint4 u = reinterpret_cast<const uint4*>(p)[i];
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[8 * i + 2 * j] = __uint_as_float(w[j] << 16);
        x[8 * i + 2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u);
      }
    }
  }
};
template <> struct XChunk<fp16_t> {
  __device__ static __forceinline__ void load(const fp16_t* p, float (&x)[32]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint4 u = reinterpret_cast<const uint4*>(p)[i];
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[8 * i + 2 * j] = (float)__builtin_bit_cast(fp16_t, (uint16_t)(w[j] & 0xFFFF));
        x[8 * i + 2 * j + 1] = (float)__builtin_bit_cast(fp16_t, (uint16_t)(w[j] >> 16));
      }
    }
  }
};
template <> struct XChunk<float> {
  __device__ static __forceinline__ void load(const float* p, float (&x)[32]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 u = reinterpret_cast<const float4*>(p)[i];
      x[4 * i] = u.x; x[4 * i + 1] = u.y; x[4 * i + 2] = u.z; x[4 * i + 3] = u.w;
    }
  }
};

__device__ __forceinline__ float chunk_dot(const float2* __restrict__ lut, const uint4& b, const float (&x)[32]) {
  const uint32_t w[4] = {b.x, b.y, b.z, b.w};
  float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float2 c = lut[(w[i >> 2] >> (8 * (i & 3))) & 0xFF];
    s0 = fmaf(x[2 * i], c.x, s0);
    s1 = fmaf(x[2 * i + 1], c.y, s1);
  }
  return s0 + s1;
}

// Fast path: K % 32 == 0, ldb % 16 == 0, A and B 16-B aligned.
template <typename T, int R>
__global__ void __launch_bounds__(256)
k_gemv_4bit(int M, int K, const T* __restrict__ A, const uint8_t* __restrict__ B, const float* __restrict__ absmax,
            const float* __restrict__ datatype, T* __restrict__ out, int ldb, int blocksize) {
  __shared__ float2 s_lut[256];
  s_lut[threadIdx.x] = make_float2(datatype[threadIdx.x >> 4], datatype[threadIdx.x & 15]);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= M) return;
  const int nchunks = K >> 5;   // 32 elements per 16-B chunk
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0f;
  const long long two_ldb = 2LL * ldb;
  for (int c = lane; c < nchunks; c += 64) {
    uint4 b[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = min(row0 + r, M - 1);
      b[r] = ld_nt16(B + (long long)row * ldb + 16LL * c);
    }
    float x[32];
    XChunk<T>::load(A + 32 * c, x);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = min(row0 + r, M - 1);
      const float am = absmax[(two_ldb * row + 32LL * c) / blocksize];
      acc[r] = fmaf(chunk_dot(s_lut, b[r], x), am, acc[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (row0 + r < M) out[row0 + r] = Io<T>::from_f32(acc[r]);
  }
}

// bf16 / fp16 fast path (K <= 16384).  Per packed byte: one conflict-free ds_read_b32 from a table of T
// pairs {T(code[hi]), T(code[lo])} and one v_dot2c_f32_{bf16,f16} against the matching activation pair.
// Codes are rounded to T as in the reference's T-precision quant_map (kernel_gemm.cpp:1294); products
// and sums are fp32, each 32-element chunk is scaled once by its fp32 absmax.
//
// Schedule per workgroup (4 waves, R rows per wave, every lane owns U chunks of 16 B per row):
//   1. absmax loads, then the activation vector by LDS-DMA, then all R*U weight loads (non-temporal);
//   2. the pair table is written while the weights are in flight: 32 copies, entry e of copy j at byte
//      128*e + 4*j, so lane l reads copy l&31 and a ds_read_b32 never conflicts;
//   3. s_waitcnt vmcnt(R*U) (activations landed, weights still in flight), barrier, then each chunk is
//      consumed as soon as its load returns.
// NESTED fuses the compressed-statistics decode (functional.py:1982-1984):
//   absmax[j] = code2[q8[j]] * absmax2[j >> log2(bs2)] + offset, fp32, the dequantize_blockwise order.
template <typename T, int R, int U, bool NESTED>
__global__ void __launch_bounds__(GV_THREADS)
k_gemv_4bit_dot(int M, int K, const T* __restrict__ A, const uint8_t* __restrict__ B, GemvStats st,
                const float* __restrict__ datatype, T* __restrict__ out, int ldb) {
  extern __shared__ __attribute__((aligned(16))) uint8_t gsm[];
  uint8_t* table = gsm;                               // GV_TABLE_BYTES
  uint8_t* xs = gsm + GV_TABLE_BYTES;                 // K * 2 bytes
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row0 = (blockIdx.x * (GV_THREADS / 64) + wave) * R;
  const int nch = K >> 5;
  const long long two_ldb = 2LL * ldb;

  // (1a) block statistics and the table values, oldest in the VMEM queue
  constexpr int NT = 256 * 8 / GV_THREADS;            // 16-B table stores per thread
  // the 16 code values arrive by scalar loads (lgkm queue), so nothing here waits on the VMEM queue
  float dt[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) dt[j] = datatype[j];
  float am[U][R];
  uint32_t q8[U][R];
  float a2[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = min(lane + 64 * u, nch - 1);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const long long j = (two_ldb * min(row0 + r, M - 1) + 32LL * c) >> st.bs_shift;
      if constexpr (NESTED) {
        q8[u][r] = st.q8[j];
        a2[u][r] = st.absmax2[j >> st.bs2_shift];
      } else {
        am[u][r] = st.absmax[j];
      }
    }
  }
  float offset = 0.0f, c2 = 0.0f;
  if constexpr (NESTED) { offset = *st.offset; c2 = st.code2[threadIdx.x]; }
  // (1b) activations by LDS-DMA
  const int nx = K >> 3;
  for (int j = 0; j * GV_THREADS < nx; ++j) {
    const int idx = (j * (GV_THREADS / 64) + wave) * 64 + lane;
    if (idx < nx) glds16(A + 8 * idx, xs + (j * (GV_THREADS / 64) + wave) * 1024);
  }
  // (1c) weights: the laundered pointer keeps these loads behind the DMA and ahead of the wait
  uintptr_t bp = (uintptr_t)B;
  asm volatile("" : "+s"(bp)::"memory");
  uint4 b[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = min(lane + 64 * u, nch - 1);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = min(row0 + r, M - 1);
      const u32x4_t v = __builtin_nontemporal_load((gvec_p)((gbyte_p)bp + (long long)row * ldb + 16LL * c));
      b[u][r] = make_uint4(v.x, v.y, v.z, v.w);
    }
  }
  // (2) bank-private table copies (+ the nested code map)
  float lo = dt[0];                                    // code[e & 15], e & 15 = (tid >> 3) & 15 for every k
#pragma unroll
  for (int j = 1; j < 16; ++j) lo = ((threadIdx.x >> 3) & 15) == j ? dt[j] : lo;
  static_assert(GV_THREADS == 256, "table fill assumes 256 threads");
#pragma unroll
  for (int k = 0; k < NT; ++k) {
    const int i = threadIdx.x + k * GV_THREADS;
    const float hi = (threadIdx.x >> 7) ? dt[2 * k + 1] : dt[2 * k];   // code[e >> 4], e >> 4 = 2k + (tid >> 7)
    const uint32_t v = Dot2<T>::pair(hi, lo);
    *reinterpret_cast<uint4*>(table + (i >> 3) * 128 + 16 * (i & 7)) = make_uint4(v, v, v, v);
  }
  float* code2s = reinterpret_cast<float*>(xs + 2 * K);
  if constexpr (NESTED) code2s[threadIdx.x] = c2;
  // (3) x landed (only the R*U weight loads may still be outstanding), table visible
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R * U) : "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  if (row0 >= M) return;
  if constexpr (NESTED) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < R; ++r) am[u][r] = __fadd_rn(__fmul_rn(code2s[q8[u][r]], a2[u][r]), offset);
  }
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0f;
  const uint32_t lane4 = (lane & 31) * 4;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool valid = lane + 64 * u < nch;           // tail lanes recompute a clamped chunk, then drop it
    const int c = min(lane + 64 * u, nch - 1);
    uint32_t x[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(xs + 64 * c)[q];
      x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t w[4] = {b[u][r].x, b[u][r].y, b[u][r].z, b[u][r].w};
      uint32_t l[16];
#pragma unroll
      for (int i = 0; i < 16; ++i)
        l[i] = *reinterpret_cast<const uint32_t*>(table + ((((w[i >> 2] >> (8 * (i & 3))) & 0xFF) << 7) | lane4));
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        s0 = Dot2<T>::dot(x[i], l[i], s0);
        s1 = Dot2<T>::dot(x[i + 1], l[i + 1], s1);
      }
      const float part = (s0 + s1) * am[u][r];
      acc[r] += valid ? part : 0.0f;
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (row0 + r < M) out[row0 + r] = Io<T>::from_f32(acc[r]);
  }
}

// Balanced-range GEMV (default where it fits, K <= 7680).  Measured at 11008 x 4096 (profiles/lab/
// r02_gemv_floor.txt): k_gemv_4bit_dot spends ~1/4 of its time before its first dot (its workgroups wait for
// activations and statistics queued behind other workgroups' weight requests) and is then bound by the
// table lookups' LDS and VALU issue.  This kernel changes four things, arithmetic unchanged (bit-identical):
//   * G = 2 x CUs workgroups, workgroup g owns M / G rows, one more for g < M % G (21-22 at 11008): every CU gets the same
//     work, NW = ceil(rows / R) waves take rows r0 + w + NW*j (j < R);
//   * the table lookup address is ONE v_perm_b32 of {packed dword, lane byte}: entry e of copy c at byte
//     256 e + 4 c (32 copies over a 64 KiB span; lanes l and l+32 share copy l & 31, different 32-lane groups),
//     against shift + mask + or for the 128-B-stride table;
//   * activations are stored swizzled, 16-B piece q of chunk c at 64 c + 16 ((q + (c >> 2)) & 3), so the
//     ds_read_b128 of chunks lane + 64u is conflict-free (4-way on the plain layout);
//   * every wave issues its statistics and activation loads, then a barrier, then its weights: the CU's
//     request queue holds all of the former ahead of any weight request.
// LDS: 64 KiB table + 2K activations (the nested code map sits in the table's spare halves): two workgroups per CU
// up to K = 8192 (exactly half the CU's LDS each), one workgroup of up to 16 waves per CU above that (K <= 16384).
constexpr int GB_TABLE_BYTES = 65536;
// nested statistics decoded where each chunk is consumed (LAZY, round 5) or all up front (the round-4 form, default; A/B
// knob cgemv_4bit_set_lazy_nested).  Measured and rejected: bit-identical, +0.2..+1.9 % (11008 x 4096 8.25 -> 8.34 us;
// tools/r05_gemv_lazy_ab.py, profiles/lab/r05_gemv_lazy_ab.txt)
static Knob<int> g_gv_lazy{0};
constexpr int GB_MAX_WAVES = 16;
// two workgroups per CU up to 79 KiB (K <= 7680), and at exactly half the CU's 160 KiB (K = 8192) from 2048 rows:
// 3584 / 4096 / 8192 x 8192 6.20 / 6.79 / 10.77 -> 6.00 / 6.34 / 10.43 us, but 1024 x 8192 4.00 -> 5.04 us, where
// two table fills per CU outweigh the gain (profiles/lab/r02_gemv_wide.txt).  Lab knob: cgemv_4bit_set_two_per_cu_lds.
static Knob<size_t> g_gb_two_per_cu_lds{79 * 1024};
constexpr size_t GB_HALF_CU_LDS = 80 * 1024;
constexpr int GB_HALF_CU_MIN_ROWS = 2048;

#ifdef BNB_LAB
// lab build only (make lab): per-wave s_memrealtime stamps (10 ns ticks) of k_gemv_4bit_bal at
// g_gv_tl[(blockIdx.x * GB_MAX_WAVES + wave) * 8 + i]: 0 start, 1 statistics / activation loads issued (first barrier),
// 2 weight loads issued, 3 statistics + activations landed and the table built (second barrier), 4 last chunk's dots
// done, 5 row stored, 6 the wave's XCD (HW_REG_XCC_ID), 7 block id (cgemv_4bit_timeline; tools/r06_gemv_timeline.py)
__device__ unsigned long long* g_gv_tl = nullptr;
__device__ int g_gv_abl = 0;   // lab A/B bits (cgemv_4bit_lab_bits): 1 = no barrier between the statistics / activation
                               // issue and the weight issue
__device__ __forceinline__ unsigned long long gv_now() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
#define GV_TL(i) tl[i] = gv_now()
#else
#define GV_TL(i) ((void)0)
#endif

template <typename T, int R, int U, bool NESTED, bool LAZY = true>
__global__ void __launch_bounds__(GB_MAX_WAVES * 64)
k_gemv_4bit_bal(const uint8_t* __restrict__ B, const T* __restrict__ A, const float* __restrict__ datatype,
                T* __restrict__ out, int q, int rem, int ldb, int K, int NW, GemvStats st) {
  extern __shared__ __attribute__((aligned(16))) uint8_t gsm[];
#ifdef BNB_LAB
  unsigned long long tl[6] = {0, 0, 0, 0, 0, 0};
#endif
  GV_TL(0);
  uint8_t* table = gsm;                               // GB_TABLE_BYTES
  uint8_t* xs = gsm + GB_TABLE_BYTES;                 // K * 2 bytes, swizzled
  // nested code map entry t in the unused upper half of table row t >> 5 (the copies fill bytes 0..127 of each
  // 256-B entry row), so the map costs no LDS of its own
  auto code2s_at = [&](uint32_t t) -> float& {
    return *reinterpret_cast<float*>(table + 256 * (t >> 5) + 128 + 4 * (t & 31));
  };
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // rows [r0, r1): q + 1 rows for the first `rem` workgroups, q for the rest (no division in the kernel)
  const int bid = blockIdx.x;
  const int r0 = bid * q + min(bid, rem), r1 = r0 + q + (bid < rem ? 1 : 0);
  const int nch = K >> 5;
  const long long two_ldb = 2LL * ldb;
  auto row_of = [&](int j) { return min(r0 + wave + NW * j, r1 - 1); };
  auto chunk_of = [&](int u) { return min(lane + 64 * u, nch - 1); };
  // this wave's weights, non-temporal, consumption order
  uint4 b[U][R];
  auto issue_weights = [&]() {
    uintptr_t bp = (uintptr_t)B;
    asm volatile("" : "+s"(bp)::"memory");
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const u32x4_t v =
            __builtin_nontemporal_load((gvec_p)((gbyte_p)bp + (long long)row_of(j) * ldb + 16LL * chunk_of(u)));
        b[u][j] = make_uint4(v.x, v.y, v.z, v.w);
      }
  };
#if defined(BNB_LAB)
  const bool wfirst = (g_gv_abl & 2) != 0;            // lab A/B: the weights before the statistics and activations
#elif defined(BNB_GV_WFIRST)
  constexpr bool wfirst = BNB_GV_WFIRST != 0;
#else
  constexpr bool wfirst = false;
#endif
  if (wfirst) {
    issue_weights();
    asm volatile("" ::: "memory");
  }

  // (1) code values (scalar), block statistics, activations by LDS-DMA (lane i of the instruction for LDS
  //     slot i = 16 B fetches the piece that belongs there under the swizzle)
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
  const int nx = K >> 3;
  for (int p = wave; p * 64 < nx; p += NW) {
    const int i = p * 64 + lane, c = i >> 2;
    if (i < nx) glds16(A + 8 * (4 * c + (((i & 3) - (c >> 2)) & 3)), xs + p * 1024);
  }
  if (wfirst) {
    GV_TL(1);
  } else {
#ifdef BNB_LAB
    if (!(g_gv_abl & 1))
#endif
    __builtin_amdgcn_s_barrier();                     // all statistics / activation requests are out
    GV_TL(1);
    issue_weights();                                  // (2)
  }
  GV_TL(2);
  // (3) table: thread t < 256 writes entry t (32 copies, 16-B stores rotated by t to spread the banks)
  for (int t = threadIdx.x; t < 256; t += NW * 64) {
    float hi = dt[0], lo = dt[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) {
      hi = (t >> 4) == j ? dt[j] : hi;
      lo = (t & 15) == j ? dt[j] : lo;
    }
    const uint32_t v = Dot2<T>::pair(hi, lo);
#pragma unroll
    for (int k = 0; k < 8; ++k) *reinterpret_cast<uint4*>(table + 256 * t + 16 * ((k + t) & 7)) = make_uint4(v, v, v, v);
  }
  if constexpr (NESTED) {
    if (threadIdx.x < 256) code2s_at(threadIdx.x) = c2;
    for (int t = threadIdx.x + NW * 64; t < 256; t += NW * 64) code2s_at(t) = st.code2[t];   // < 4 waves
  }
  if (wfirst) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R * U) : "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  GV_TL(3);
  // (nested, LAZY: each block's absmax is decoded where its chunk is consumed, so the code-map reads and the decode of
  // later chunks overlap the lookups of earlier ones instead of all preceding the first dot)
  if constexpr (NESTED && !LAZY) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < R; ++j) am[u][j] = __fadd_rn(__fmul_rn(code2s_at(q8[u][j]), a2[u][j]), offset);
  }
  float acc[R];
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = 0.0f;
  const uint32_t lane4 = (lane & 31) * 4;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool valid = lane + 64 * u < nch;
    const int c = chunk_of(u);
    uint32_t x[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(xs + 64 * c)[(q + (c >> 2)) & 3];
      x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t w[4] = {b[u][j].x, b[u][j].y, b[u][j].z, b[u][j].w};
      uint32_t l[16];
#pragma unroll
      for (int i = 0; i < 16; ++i)   // byte i & 3 of w[i >> 2] -> address byte 1, lane offset -> address byte 0
        l[i] = *reinterpret_cast<const uint32_t*>(
            table + __builtin_amdgcn_perm(w[i >> 2], lane4, 0x0C0C0000u | ((4u + (i & 3)) << 8)));
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        s0 = Dot2<T>::dot(x[i], l[i], s0);
        s1 = Dot2<T>::dot(x[i + 1], l[i + 1], s1);
      }
      if constexpr (NESTED && LAZY) am[u][j] = __fadd_rn(__fmul_rn(code2s_at(q8[u][j]), a2[u][j]), offset);
      const float part = (s0 + s1) * am[u][j];
      acc[j] += valid ? part : 0.0f;
    }
  }
  GV_TL(4);
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = wave_sum(acc[j]);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int row = r0 + wave + NW * j;
      if (row < r1) out[row] = Io<T>::from_f32(acc[j]);
    }
  }
#ifdef BNB_LAB
  if (g_gv_tl != nullptr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    GV_TL(5);
    if (lane == 0) {
      unsigned long long* o = g_gv_tl + ((long long)blockIdx.x * GB_MAX_WAVES + wave) * 8;
      for (int i = 0; i < 6; ++i) o[i] = tl[i];
      o[6] = (unsigned long long)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15);
      o[7] = blockIdx.x;
    }
  }
#endif
}

// Wide GEMV (narrow or long-K weights: the 70B shards, e.g. 1024 x 28672 and 128 x 8192): one workgroup per weight
// row, its NW waves split K (lane t of the workgroup takes chunks t + 64 NW u, u < U), summed across waves in LDS in
// wave order.  The balanced kernel gives a workgroup whole rows, so a few hundred rows leave most of the chip idle, and
// K > GV_MAX_K does not fit its LDS activation copy; here the activations come from L2 (each workgroup reads all
// of x) and only the pair table sits in LDS (the 128-B-stride copies of k_gemv_4bit_dot, conflict-free).  Same
// per-chunk arithmetic as the other table kernels; the chunk-to-lane grouping, and so the fp32 summation order, differs.
// R > 1 (round 3): R rows per workgroup (at most 4 waves), sharing one activation load and one table fill -- each
// workgroup reads all of x from L2, so one row per workgroup moved 4x the weight bytes again as activations at
// 1024 x 28672; every row's chunk grouping and summation order is unchanged (bit-identical to R = 1).
constexpr int GW_MAX_WAVES = 16;
constexpr int GW_MAX_WAVES_R = 4;                                   // (R > 1)

template <typename T, int U, bool NESTED, int R = 1>
__global__ void __launch_bounds__((R > 1 ? GW_MAX_WAVES_R : GW_MAX_WAVES) * 64)
k_gemv_4bit_wide(int M, int K, const T* __restrict__ A, const uint8_t* __restrict__ B, GemvStats st,
                 const float* __restrict__ datatype, T* __restrict__ out, int ldb) {
  extern __shared__ __attribute__((aligned(16))) uint8_t gsm[];
  uint8_t* table = gsm;                                           // GV_TABLE_BYTES
  float* code2s = reinterpret_cast<float*>(gsm + GV_TABLE_BYTES); // 256 (nested)
  float* red = code2s + 256;                                      // one partial per wave
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int NT = blockDim.x, NW = NT >> 6;
  const int row0 = blockIdx.x * R;
  const int nch = K >> 5;
  const long long two_ldb = 2LL * ldb;
  auto chunk_of = [&](int u) { return min(tid + NT * u, nch - 1); };
  auto row_of = [&](int j) { return min(row0 + j, M - 1); };
  // (1) code values (scalar) and the nested code map first: loaded later, inside the table fill, they queued behind
  //     the whole weight stream (1024 x 28672: 10.1 us); then statistics, activations (L2), the weights (non-temporal)
  float dt[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) dt[j] = datatype[j];
  float c2p[4] = {0.f, 0.f, 0.f, 0.f};                   // code2[tid + NT q], q < 256 / NT (NT >= 64)
  if constexpr (NESTED) {
#pragma unroll
    for (int q = 0; q < 4; ++q) c2p[q] = st.code2[min(tid + NT * q, 255)];
  }
  float am[R][U];
  uint32_t q8[R][U];
  float a2[R][U];
#pragma unroll
  for (int j = 0; j < R; ++j)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long blk = (two_ldb * row_of(j) + 32LL * chunk_of(u)) >> st.bs_shift;
      if constexpr (NESTED) {
        q8[j][u] = st.q8[blk];
        a2[j][u] = st.absmax2[blk >> st.bs2_shift];
      } else {
        am[j][u] = st.absmax[blk];
      }
    }
  float offset = 0.0f;
  if constexpr (NESTED) offset = *st.offset;
  uint4 xv[U][4];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int q = 0; q < 4; ++q) xv[u][q] = reinterpret_cast<const uint4*>(A + 32 * chunk_of(u))[q];
  uintptr_t bp = (uintptr_t)B;
  asm volatile("" : "+s"(bp)::"memory");
  uint4 b[R][U];
#pragma unroll
  for (int j = 0; j < R; ++j)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const u32x4_t v = __builtin_nontemporal_load((gvec_p)((gbyte_p)bp + (long long)row_of(j) * ldb + 16LL * chunk_of(u)));
      b[j][u] = make_uint4(v.x, v.y, v.z, v.w);
    }
  // (2) table: 16-B store i holds entry i >> 3 for copies 4 (i & 7) .. 4 (i & 7) + 3 (entry e of copy j at 128 e + 4 j)
  for (int i = tid; i < GV_TABLE_BYTES / 16; i += NT) {
    const int e = i >> 3;
    float hi = dt[0], lo = dt[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) {
      hi = (e >> 4) == j ? dt[j] : hi;
      lo = (e & 15) == j ? dt[j] : lo;
    }
    const uint32_t v = Dot2<T>::pair(hi, lo);
    *reinterpret_cast<uint4*>(table + 16 * i) = make_uint4(v, v, v, v);
  }
  if constexpr (NESTED) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (tid + NT * q < 256) code2s[tid + NT * q] = c2p[q];
  }
  __syncthreads();
  if constexpr (NESTED) {
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
      for (int u = 0; u < U; ++u) am[j][u] = __fadd_rn(__fmul_rn(code2s[q8[j][u]], a2[j][u]), offset);
  }
  // (3) dot: per chunk s0 / s1 chains of v_dot2 over 16 packed bytes, scaled by the chunk's absmax
  const uint32_t lane4 = (lane & 31) * 4;
  float accs[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
  float acc = 0.0f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t x[16] = {xv[u][0].x, xv[u][0].y, xv[u][0].z, xv[u][0].w, xv[u][1].x, xv[u][1].y, xv[u][1].z,
                            xv[u][1].w, xv[u][2].x, xv[u][2].y, xv[u][2].z, xv[u][2].w, xv[u][3].x, xv[u][3].y,
                            xv[u][3].z, xv[u][3].w};
    const uint32_t w[4] = {b[j][u].x, b[j][u].y, b[j][u].z, b[j][u].w};
    uint32_t l[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
      l[i] = *reinterpret_cast<const uint32_t*>(table + ((((w[i >> 2] >> (8 * (i & 3))) & 0xFF) << 7) | lane4));
    float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      s0 = Dot2<T>::dot(x[i], l[i], s0);
      s1 = Dot2<T>::dot(x[i + 1], l[i + 1], s1);
    }
    const float part = (s0 + s1) * am[j][u];
    acc += (tid + NT * u < nch) ? part : 0.0f;
  }
  accs[j] = wave_sum(acc);
  }
  if (lane == 0)
#pragma unroll
    for (int j = 0; j < R; ++j) red[wave * R + j] = accs[j];
  __syncthreads();
  if (tid < R && row0 + tid < M) {
    float s = red[tid];
    for (int w2 = 1; w2 < NW; ++w2) s += red[w2 * R + tid];
    out[row0 + tid] = Io<T>::from_f32(s);
  }
}

// General path (any K, ldb, alignment): one wave per row, one element per lane step.
template <typename T>
__global__ void __launch_bounds__(256)
k_gemv_4bit_generic(int M, int K, const T* __restrict__ A, const uint8_t* __restrict__ B, const float* __restrict__ absmax,
                    const float* __restrict__ datatype, T* __restrict__ out, int ldb, int blocksize) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float acc = 0.0f;
  const long long two_ldb = 2LL * ldb;
  for (int k = lane; k < K; k += 64) {
    const uint32_t byte = B[(long long)row * ldb + (k >> 1)];
    const uint32_t q = (k & 1) ? (byte & 15) : (byte >> 4);
    acc = fmaf(Io<T>::to_f32(A[k]), __fmul_rn(datatype[q], absmax[(two_ldb * row + k) / blocksize]), acc);
  }
  acc = wave_sum(acc);
  if (lane == 0) out[row] = Io<T>::from_f32(acc);
}

// 0 = auto (k_gemv_4bit_wide on narrow / long-K weights, k_gemv_4bit_bal where it fits, else k_gemv_4bit_dot),
// 1 = k_gemv_4bit_dot only, 2 = k_gemv_4bit_wide wherever it applies, 3 = auto without the wide kernel (A/B, tests);
// 20 + U: the wide kernel with U chunks per lane (lab)
Knob<int> g_gemv_kernel{0};
Knob<int> g_gemv_wide_rows{0};   // 1: the wide kernel one row per workgroup (A/B, tests)

int device_cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cus = n;
  }
  return cus;
}

// k_gemv_4bit_bal for this shape; false when it does not fit (K > GV_MAX_K, or more than 8 weight loads per
// lane would be needed to cover the rows).  When two workgroups of NW waves share a CU, an instance above 85
// VGPRs (R * U > 4: 88-98) is limited to NW <= 8 (4 waves per SIMD, 128 VGPRs).
// A/B knob: g_gemv_kernel = 10 + R forces at least R rows per wave.
template <typename T, bool NESTED>
static bool launch_gemv_bal(int m, int k, const T* A, const uint8_t* B, const GemvStats& st, const float* datatype,
                            T* out, int ldb) {
  const size_t lds = GB_TABLE_BYTES + 2 * (size_t)k;     // (+ the nested code map inside the table's spare halves)
  if (k > GV_MAX_K) return false;
  const bool two = lds <= g_gb_two_per_cu_lds || (lds <= GB_HALF_CU_LDS && m >= GB_HALF_CU_MIN_ROWS);
  const int G = min((two ? 2 : 1) * device_cu_count(), m);
  const int rows = (m + G - 1) / G;
  int U = ((k >> 5) + 63) / 64;
  if (U > 4) U = U <= 6 ? 6 : 8;
  // measured (tools/gemv_sweep.py): two per CU, plain statistics up to 12 waves; nested up to 8 (at 11008 x 4096
  // nested, 11 waves x 2 rows runs 9.4 us, 8 waves x 3 rows 8.3 us, the 4-waves-x-R-rows kernel 8.8 us)
  int max_waves = 16;
  if (two) max_waves = (NESTED || U * ((rows + 11) / 12) > 4) ? 8 : 12;
  int R = (rows + max_waves - 1) / max_waves;
  if (g_gemv_kernel >= 10) R = max(R, g_gemv_kernel - 10);   // A/B: more rows per wave
  if (R > 4 || R * U > 8) return false;
  // one workgroup per CU pays off for one row per wave (4096 x 11008: 9.9 vs 12.4 us, 4096 x 14336: 12.3 vs
  // 13.5) but not for two (8192 x 8192: 12.8 vs 11.5 us for the 4-waves-x-R-rows kernel)
  if (!two && R > 1) return false;
  const int nw = (rows + R - 1) / R;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(G), dim3(64 * nw), lds, current_stream(), B, A, datatype, out, m / G, m % G, ldb, k,
                       nw, st);
    return true;
  };
  auto pick = [&](auto lz) {
    constexpr bool LZ = decltype(lz)::value;
    switch (R * 8 + U) {
      case 8 + 1: return go(k_gemv_4bit_bal<T, 1, 1, NESTED, LZ>);
      case 8 + 2: return go(k_gemv_4bit_bal<T, 1, 2, NESTED, LZ>);
      case 8 + 3: return go(k_gemv_4bit_bal<T, 1, 3, NESTED, LZ>);
      case 8 + 4: return go(k_gemv_4bit_bal<T, 1, 4, NESTED, LZ>);
      case 8 + 6: return go(k_gemv_4bit_bal<T, 1, 6, NESTED, LZ>);
      case 8 + 8: return go(k_gemv_4bit_bal<T, 1, 8, NESTED, LZ>);
      case 16 + 1: return go(k_gemv_4bit_bal<T, 2, 1, NESTED, LZ>);
      case 16 + 2: return go(k_gemv_4bit_bal<T, 2, 2, NESTED, LZ>);
      case 16 + 3: return go(k_gemv_4bit_bal<T, 2, 3, NESTED, LZ>);
      case 16 + 4: return go(k_gemv_4bit_bal<T, 2, 4, NESTED, LZ>);
      case 24 + 1: return go(k_gemv_4bit_bal<T, 3, 1, NESTED, LZ>);
      case 24 + 2: return go(k_gemv_4bit_bal<T, 3, 2, NESTED, LZ>);
      case 32 + 1: return go(k_gemv_4bit_bal<T, 4, 1, NESTED, LZ>);
      case 32 + 2: return go(k_gemv_4bit_bal<T, 4, 2, NESTED, LZ>);
      default: return false;
    }
  };
  if constexpr (NESTED) {
    if (!g_gv_lazy) return pick(std::false_type{});
  }
  return pick(std::true_type{});
}


// k_gemv_4bit_wide: NW waves per row such that each lane holds U chunks; false when K needs more than 16 waves x 4
// chunks (K > 131072)
template <typename T, bool NESTED>
static bool launch_gemv_wide(int m, int k, const T* A, const uint8_t* B, const GemvStats& st, const float* datatype,
                             T* out, int ldb) {
  const int nch = k >> 5;
  // measured (tools/gemv_shape_probe.py, profiles/lab/r02_gemv_wide.txt): 4 chunks per lane on long K (1024 x 28672:
  // 13.3 / 11.6 / 12.0 / 10.3 us at U = 1..4), 1 on short K (128 x 8192: 3.8 / 4.5 / 4.9 / 6.5 us)
  int U = g_gemv_kernel >= 21 && g_gemv_kernel <= 24 ? g_gemv_kernel - 20 : (k > GV_MAX_K ? 4 : 1);
  int nw = (nch + 64 * U - 1) / (64 * U);
  if (nw > GW_MAX_WAVES) {
    nw = GW_MAX_WAVES;
    U = (nch + 64 * nw - 1) / (64 * nw);
  }
  if (U > 4) return false;
  nw = (nch + 64 * U - 1) / (64 * U);
  // rows per workgroup: as many as keep >= one workgroup per CU (at most 4, and only with <= 4 waves)
  int R = std::max(1, std::min(4, m / device_cu_count()));
  if (nw > GW_MAX_WAVES_R || g_gemv_wide_rows == 1 || (U != 1 && U != 4)) R = 1;
  const size_t lds = GV_TABLE_BYTES + 256 * sizeof(float) + GW_MAX_WAVES * 4 * sizeof(float);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)((m + R - 1) / R)), dim3(64 * nw), lds, current_stream(), m, k, A, B, st,
                       datatype, out, ldb);
    return true;
  };
  if (R > 1 && U == 4) {
    switch (R) {
      case 2: return go(k_gemv_4bit_wide<T, 4, NESTED, 2>);
      case 3: return go(k_gemv_4bit_wide<T, 4, NESTED, 3>);
      default: return go(k_gemv_4bit_wide<T, 4, NESTED, 4>);
    }
  }
  if (R > 1 && U == 1) {
    switch (R) {
      case 2: return go(k_gemv_4bit_wide<T, 1, NESTED, 2>);
      case 3: return go(k_gemv_4bit_wide<T, 1, NESTED, 3>);
      default: return go(k_gemv_4bit_wide<T, 1, NESTED, 4>);
    }
  }
  switch (U) {
    case 1: return go(k_gemv_4bit_wide<T, 1, NESTED>);
    case 2: return go(k_gemv_4bit_wide<T, 2, NESTED>);
    case 3: return go(k_gemv_4bit_wide<T, 3, NESTED>);
    default: return go(k_gemv_4bit_wide<T, 4, NESTED>);
  }
}

// the wide kernel by default: K beyond the balanced kernel's LDS (1024 x 28672, the 70B down-projection shard: 26.9
// -> 10.3 us), or fewer rows than CUs (128 x 8192, the 70B k/v shard: 5.2 -> 3.8 us).  From a few hundred rows
// its per-row table fill loses to the balanced kernel (1024 x 8192 4.0 vs 5.1 us, 11008 x 4096 8.1 vs 41 us).
static bool gemv_wide_preferred(int m, int k) {
  if (g_gemv_kernel == 2 || (g_gemv_kernel >= 21 && g_gemv_kernel <= 24)) return true;
  if (g_gemv_kernel != 0) return false;
  return k > GV_MAX_K || m < device_cu_count();
}

// Launch the table/dot kernel when the shape fits it; false -> caller uses another kernel.
template <typename T>
bool launch_gemv_dot(int m, int k, const T* A, const uint8_t* B, GemvStats st, const float* datatype, T* out, int ldb,
                     int blocksize, int blocksize2) {
  const bool nested = st.q8 != nullptr;
  if (k % 32 || ldb % 16 || ((uintptr_t)A & 15) || ((uintptr_t)B & 15) || blocksize < 32) return false;
  if ((blocksize & (blocksize - 1)) || (nested && (blocksize2 <= 0 || (blocksize2 & (blocksize2 - 1))))) return false;
  st.bs_shift = __builtin_ctz(blocksize);
  st.bs2_shift = nested ? __builtin_ctz(blocksize2) : 0;
  if (gemv_wide_preferred(m, k)) {
    const bool ok = nested ? launch_gemv_wide<T, true>(m, k, A, B, st, datatype, out, ldb)
                           : launch_gemv_wide<T, false>(m, k, A, B, st, datatype, out, ldb);
    if (ok) return true;
  }
  const size_t lds = GV_TABLE_BYTES + 2 * (size_t)k + (nested ? 1024 : 0);
  if (k > GV_MAX_K || lds > 65536) return false;
  if (g_gemv_kernel != 1) {
    const bool ok = nested ? launch_gemv_bal<T, true>(m, k, A, B, st, datatype, out, ldb)
                           : launch_gemv_bal<T, false>(m, k, A, B, st, datatype, out, ldb);
    if (ok) return true;
  }
  const int nch = k >> 5;
  auto go = [&](auto kern, int R) {
    const int waves = (m + R - 1) / R;
    hipLaunchKernelGGL(kern, dim3((waves + GV_THREADS / 64 - 1) / (GV_THREADS / 64)), dim3(GV_THREADS), lds,
                       current_stream(), m, k, A, B, st, datatype, out, ldb);
  };
  // 8 x 16 B weight loads in flight per lane: R rows x U chunk groups of 64 lanes
  if (nested) {
    if (nch <= 64) go(k_gemv_4bit_dot<T, 8, 1, true>, 8);
    else if (nch <= 128) go(k_gemv_4bit_dot<T, 4, 2, true>, 4);
    else if (nch <= 256) go(k_gemv_4bit_dot<T, 2, 4, true>, 2);
    else go(k_gemv_4bit_dot<T, 1, 8, true>, 1);
  } else {
    if (nch <= 64) go(k_gemv_4bit_dot<T, 8, 1, false>, 8);
    else if (nch <= 128) go(k_gemv_4bit_dot<T, 4, 2, false>, 4);
    else if (nch <= 256) go(k_gemv_4bit_dot<T, 2, 4, false>, 2);
    else go(k_gemv_4bit_dot<T, 1, 8, false>, 1);
  }
  return true;
}

template <typename T>
void gemv_4bit(int m, int n, int k, const T* A, const uint8_t* B, const float* absmax, const float* datatype, T* out,
               int lda, int ldb, int ldc, int blocksize) {
  (void)n; (void)lda; (void)ldc;
  if (m <= 0) return;
  if (k <= 0 || blocksize <= 0) { set_error(1, "gemv_4bit: bad k/blocksize"); return; }
  const bool fast = (k % 32 == 0) && (ldb % 16 == 0) && (((uintptr_t)A & 15) == 0) && (((uintptr_t)B & 15) == 0) &&
                    (blocksize % 32 == 0);
  if constexpr (sizeof(T) == 2) {
    GemvStats st{};
    st.absmax = absmax;
    if (fast && launch_gemv_dot<T>(m, k, A, B, st, datatype, out, ldb, blocksize, 0)) {
      BNB_LAUNCH_CHECK("gemv_4bit");
      return;
    }
  }
  if (fast) {
    constexpr int R = 4;
    const int waves = (m + R - 1) / R;
    hipLaunchKernelGGL((k_gemv_4bit<T, R>), dim3((waves + 3) / 4), dim3(256), 0, current_stream(), m, k, A, B, absmax,
                       datatype, out, ldb, blocksize);
  } else {
    hipLaunchKernelGGL((k_gemv_4bit_generic<T>), dim3((m + 3) / 4), dim3(256), 0, current_stream(), m, k, A, B, absmax,
                       datatype, out, ldb, blocksize);
  }
  BNB_LAUNCH_CHECK("gemv_4bit");
}

}  // namespace bnb

using namespace bnb;

extern "C" {

// [additive, testing] 0 = auto (k_gemv_4bit_bal where it fits), 1 = the 4-waves-x-R-rows kernel only
void cgemv_4bit_set_kernel(int which) { bnb::g_gemv_kernel = which; }
// [additive, testing] 1 = the wide GEMV one row per workgroup (the round-2 form); 0 = rows per workgroup by the rule
void cgemv_4bit_set_wide_rows(int mode) { bnb::g_gemv_wide_rows = mode; }
// [lab, not in the header] LDS bytes up to which the balanced GEMV runs two workgroups per CU (default 80 KiB)
#ifdef BNB_LAB
int cgemv_4bit_timeline(unsigned long long* buf) {   // [lab build only] k_gemv_4bit_bal stamps (nullptr: off)
  return hipMemcpyToSymbol(HIP_SYMBOL(bnb::g_gv_tl), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
int cgemv_4bit_lab_bits(int v) {                      // [lab build only] g_gv_abl
  return hipMemcpyToSymbol(HIP_SYMBOL(bnb::g_gv_abl), &v, sizeof(v)) == hipSuccess ? 0 : 1;
}
void cgemv_4bit_set_two_per_cu_lds(int bytes) { bnb::g_gb_two_per_cu_lds = (size_t)bytes; }   // [lab build only]
#endif
// [additive, testing] nested statistics of the balanced GEMV decoded where each chunk is consumed (1) or all before the
// first dot (0, default: measured faster); bit-identical; returns the previous setting
int cgemv_4bit_set_lazy_nested(int on) {
  const int prev = bnb::g_gv_lazy;
  bnb::g_gv_lazy = on ? 1 : 0;
  return prev;
}

void cgemm_4bit_inference_naive_fp16(int m, int n, int k, fp16_t* A, unsigned char* B, float* absmax, float* datatype,
                                     fp16_t* out, int lda, int ldb, int ldc, int blocksize) {
  BNB_RANGE("cgemm_4bit_inference_naive_fp16");
  gemv_4bit<fp16_t>(m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize);
}
void cgemm_4bit_inference_naive_bf16(int m, int n, int k, bf16_t* A, unsigned char* B, float* absmax, float* datatype,
                                     bf16_t* out, int lda, int ldb, int ldc, int blocksize) {
  BNB_RANGE("cgemm_4bit_inference_naive_bf16");
  gemv_4bit<bf16_t>(m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize);
}
void cgemm_4bit_inference_naive_fp32(int m, int n, int k, float* A, unsigned char* B, float* absmax, float* datatype,
                                     float* out, int lda, int ldb, int ldc, int blocksize) {
  BNB_RANGE("cgemm_4bit_inference_naive_fp32");
  gemv_4bit<float>(m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize);
}

// Decode GEMV with compressed statistics decoded in-kernel (replaces the dequantize_blockwise launch of
// functional.py:1982-1984 + the gemv).  Returns 0 when launched, 1 when the shape needs the two-step path, 2 when
// the launch failed (also recorded for cget_last_error), so a caller may skip the error query on 0.
int cgemm_4bit_inference_naive_nested_fp16(int m, int n, int k, fp16_t* A, unsigned char* B, unsigned char* absmax_q,
                                           float* code2, float* absmax2, float* offset, float* datatype, fp16_t* out,
                                           int lda, int ldb, int ldc, int blocksize, int blocksize2) {
  BNB_RANGE("cgemm_4bit_inference_naive_nested_fp16");
  (void)n; (void)lda; (void)ldc;
  GemvStats st{nullptr, absmax_q, code2, absmax2, offset, 0, 0};
  if (m <= 0) return 0;
  if (!launch_gemv_dot<fp16_t>(m, k, A, B, st, datatype, out, ldb, blocksize, blocksize2)) return 1;
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_error((int)e, "gemv_4bit_nested"); return 2; }
  return 0;
}
int cgemm_4bit_inference_naive_nested_bf16(int m, int n, int k, bf16_t* A, unsigned char* B, unsigned char* absmax_q,
                                           float* code2, float* absmax2, float* offset, float* datatype, bf16_t* out,
                                           int lda, int ldb, int ldc, int blocksize, int blocksize2) {
  BNB_RANGE("cgemm_4bit_inference_naive_nested_bf16");
  (void)n; (void)lda; (void)ldc;
  GemvStats st{nullptr, absmax_q, code2, absmax2, offset, 0, 0};
  if (m <= 0) return 0;
  if (!launch_gemv_dot<bf16_t>(m, k, A, B, st, datatype, out, ldb, blocksize, blocksize2)) return 1;
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { set_error((int)e, "gemv_4bit_nested"); return 2; }
  return 0;
}

}  // extern "C"
