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
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(1))) uint8_t* gbyte_p;
typedef const __attribute__((address_space(1))) u32x4_t* gvec_p;

template <typename T> struct Dot2;
template <> struct Dot2<bf16_t> {
  __device__ static __forceinline__ float dot(uint32_t a, uint32_t b, float c) {
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), c, false);
  }
  __device__ static __forceinline__ uint32_t pair(float lo, float hi) { return pack_bf16x2(lo, hi); }
};
template <> struct Dot2<fp16_t> {
  __device__ static __forceinline__ float dot(uint32_t a, uint32_t b, float c) {
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2_t, a), __builtin_bit_cast(f16x2_t, b), c, false);
  }
  __device__ static __forceinline__ uint32_t pair(float lo, float hi) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (fp16_t)lo) | ((uint32_t)__builtin_bit_cast(uint16_t, (fp16_t)hi) << 16);
  }
};

constexpr int GV_THREADS = 256;
constexpr int GV_TABLE_BYTES = 256 * 128;    // 32 bank-private copies of the 256-entry pair table
constexpr int GV_MAX_K = 16384;              // table + K/2 pairs of T within 64 KiB

struct GemvStats {
  const float* absmax;      // plain: fp32 per block
  const uint8_t* q8;        // nested: 8-bit codes per block
  const float* code2;       //         256-entry dynamic map
  const float* absmax2;     //         fp32 per group of bs2 blocks
  const float* offset;      //         scalar (device)
  int bs_shift, bs2_shift;
};

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

// One workgroup per CU (the decode weights of one layer fit in flight at once, <= 16 x 16 B per lane).
// k_gemv_4bit_dot gives every workgroup 4 waves x R rows, so at 11008 rows the 688 workgroups land 2, 3 or 4
// per CU and the kernel ends with the most loaded CU; here workgroup g of G = min(256, M) owns the balanced
// row range [g*M/G, (g+1)*M/G) (43 rows at 11008), so every CU streams the same bytes.
// Wave w takes rows r0 + w + 8j (j < RMAX), clamped to the range: a clamped row re-reads the range's last row,
// which the owning wave of the same CU is loading at the same moment (an L2 hit, no extra HBM bytes), and its
// sum is dropped.  Each lane takes chunks lane + 64u (u < U), clamped the same way.  All RMAX x U weight loads
// are issued before any is consumed, in consumption order (u outer, rows inner), so the compiler's counted
// waits retire them one by one.  Same table / dot / statistics arithmetic as k_gemv_4bit_dot (bit-identical).
constexpr int GC_THREADS = 512, GC_WAVES = GC_THREADS / 64;

template <typename T, int U, int RMAX, bool NESTED>
__global__ void __launch_bounds__(GC_THREADS, 1)
k_gemv_4bit_cu(int M, int K, const T* __restrict__ A, const uint8_t* __restrict__ B, GemvStats st,
               const float* __restrict__ datatype, T* __restrict__ out, int ldb, int G) {
  extern __shared__ __attribute__((aligned(16))) uint8_t gsm[];
  uint8_t* table = gsm;                               // GV_TABLE_BYTES
  uint8_t* xs = gsm + GV_TABLE_BYTES;                 // K * 2 bytes
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r0 = (int)((long long)blockIdx.x * M / G), r1 = (int)((long long)(blockIdx.x + 1) * M / G);
  const int nch = K >> 5;
  const long long two_ldb = 2LL * ldb;
  auto row_of = [&](int j) { return min(r0 + wave + GC_WAVES * j, r1 - 1); };
  auto chunk_of = [&](int u) { return min(lane + 64 * u, nch - 1); };

  // (1a) block statistics; the 16 code values by scalar loads
  float dt[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) dt[j] = datatype[j];
  float am[U][RMAX];
  uint32_t q8[U][RMAX];
  float a2[U][RMAX];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < RMAX; ++j) {
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
    c2 = st.code2[threadIdx.x & 255];
  }
  // (1b) activations by LDS-DMA (1 KiB per wave-instruction)
  const int nx = K >> 3;
  for (int p = wave; p * 64 < nx; p += GC_WAVES) {
    const int idx = p * 64 + lane;
    if (idx < nx) glds16(A + 8 * idx, xs + p * 1024);
  }
  // (1c) every weight chunk of this wave, non-temporal, behind the DMA (laundered pointer)
  uintptr_t bp = (uintptr_t)B;
  asm volatile("" : "+s"(bp)::"memory");
  uint4 b[U][RMAX];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < RMAX; ++j) {
      const u32x4_t v =
          __builtin_nontemporal_load((gvec_p)((gbyte_p)bp + (long long)row_of(j) * ldb + 16LL * chunk_of(u)));
      b[u][j] = make_uint4(v.x, v.y, v.z, v.w);
    }
  // (2) 32 bank-private copies of the pair table: entry e of copy c at byte 128 e + 4 c (512 threads x 4 stores)
  static_assert(GC_THREADS == 512, "table fill assumes 512 threads");
  {
    const int e_lo = (threadIdx.x >> 3) & 15;         // e & 15 for every store of this thread
    float lo = dt[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) lo = e_lo == j ? dt[j] : lo;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = threadIdx.x + k * GC_THREADS;     // 16-B store index: entry i >> 3, copies 4 (i & 7) ..
      const int e_hi = (i >> 3) >> 4;                 // = 4 k + (tid >> 7)
      float hi = dt[0];
#pragma unroll
      for (int j = 1; j < 16; ++j) hi = e_hi == j ? dt[j] : hi;
      const uint32_t v = Dot2<T>::pair(hi, lo);
      *reinterpret_cast<uint4*>(table + (i >> 3) * 128 + 16 * (i & 7)) = make_uint4(v, v, v, v);
    }
  }
  float* code2s = reinterpret_cast<float*>(xs + 2 * K);
  if constexpr (NESTED) {
    if (threadIdx.x < 256) code2s[threadIdx.x] = c2;
  }
  // (3) activations landed (only this wave's RMAX * U weight loads may be outstanding), table visible
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U * RMAX) : "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  if constexpr (NESTED) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < RMAX; ++j) am[u][j] = __fadd_rn(__fmul_rn(code2s[q8[u][j]], a2[u][j]), offset);
  }
  float acc[RMAX];
#pragma unroll
  for (int j = 0; j < RMAX; ++j) acc[j] = 0.0f;
  const uint32_t lane4 = (lane & 31) * 4;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool valid = lane + 64 * u < nch;
    const int c = chunk_of(u);
    uint32_t x[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(xs + 64 * c)[q];
      x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < RMAX; ++j) {
      const uint32_t w[4] = {b[u][j].x, b[u][j].y, b[u][j].z, b[u][j].w};
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
      const float part = (s0 + s1) * am[u][j];
      acc[j] += valid ? part : 0.0f;
    }
  }
#pragma unroll
  for (int j = 0; j < RMAX; ++j) acc[j] = wave_sum(acc[j]);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < RMAX; ++j) {
      const int row = r0 + wave + GC_WAVES * j;
      if (row < r1) out[row] = Io<T>::from_f32(acc[j]);
    }
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

// k_gemv_4bit_cu instance for (U, RMAX) rounded up to an instantiated pair; false when none fits.
template <typename T, int U, bool NESTED>
static bool launch_gemv_cu_r(int rmax, int m, int k, const T* A, const uint8_t* B, const GemvStats& st,
                             const float* datatype, T* out, int ldb, int G, size_t lds) {
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(G), dim3(GC_THREADS), lds, current_stream(), m, k, A, B, st, datatype, out, ldb, G);
    return true;
  };
  if (rmax <= 1) return go(k_gemv_4bit_cu<T, U, 1, NESTED>);
  if (rmax <= 2) return go(k_gemv_4bit_cu<T, U, 2, NESTED>);
  if constexpr (U <= 4) {
    if (rmax <= 3) return go(k_gemv_4bit_cu<T, U, 3, NESTED>);
    if (rmax <= 4) return go(k_gemv_4bit_cu<T, U, 4, NESTED>);
  }
  if constexpr (U <= 2) {
    if (rmax <= 6) return go(k_gemv_4bit_cu<T, U, 6, NESTED>);
    if (rmax <= 8) return go(k_gemv_4bit_cu<T, U, 8, NESTED>);
  }
  if constexpr (U == 1) {
    if (rmax <= 12) return go(k_gemv_4bit_cu<T, U, 12, NESTED>);
    if (rmax <= 16) return go(k_gemv_4bit_cu<T, U, 16, NESTED>);
  }
  return false;
}

template <typename T, bool NESTED>
static bool launch_gemv_cu(int m, int k, const T* A, const uint8_t* B, const GemvStats& st, const float* datatype,
                           T* out, int ldb, size_t lds) {
  const int G = m < 256 ? m : 256;                    // one workgroup per CU
  const int rows_max = (m + G - 1) / G;
  const int rmax = (rows_max + GC_WAVES - 1) / GC_WAVES;
  const int u = ((k >> 5) + 63) / 64;
  switch (u) {
    case 1: return launch_gemv_cu_r<T, 1, NESTED>(rmax, m, k, A, B, st, datatype, out, ldb, G, lds);
    case 2: return launch_gemv_cu_r<T, 2, NESTED>(rmax, m, k, A, B, st, datatype, out, ldb, G, lds);
    case 3: return launch_gemv_cu_r<T, 3, NESTED>(rmax, m, k, A, B, st, datatype, out, ldb, G, lds);
    case 4: return launch_gemv_cu_r<T, 4, NESTED>(rmax, m, k, A, B, st, datatype, out, ldb, G, lds);
    case 5: case 6: return launch_gemv_cu_r<T, 6, NESTED>(rmax, m, k, A, B, st, datatype, out, ldb, G, lds);
    case 7: case 8: return launch_gemv_cu_r<T, 8, NESTED>(rmax, m, k, A, B, st, datatype, out, ldb, G, lds);
    default: return false;
  }
}

int g_gemv_kernel = 0;   // 0 = auto (k_gemv_4bit_dot), 2 = k_gemv_4bit_cu (A/B benchmarks, tests)

// Launch the table/dot kernel when the shape fits it; false -> caller uses another kernel.
template <typename T>
bool launch_gemv_dot(int m, int k, const T* A, const uint8_t* B, GemvStats st, const float* datatype, T* out, int ldb,
                     int blocksize, int blocksize2) {
  const bool nested = st.q8 != nullptr;
  if (k % 32 || ldb % 16 || ((uintptr_t)A & 15) || ((uintptr_t)B & 15) || blocksize < 32) return false;
  if ((blocksize & (blocksize - 1)) || (nested && (blocksize2 <= 0 || (blocksize2 & (blocksize2 - 1))))) return false;
  const size_t lds = GV_TABLE_BYTES + 2 * (size_t)k + (nested ? 1024 : 0);
  if (k > GV_MAX_K || lds > 65536) return false;
  st.bs_shift = __builtin_ctz(blocksize);
  st.bs2_shift = nested ? __builtin_ctz(blocksize2) : 0;
  if (g_gemv_kernel == 2) {   // one workgroup per CU: measured slower at 11008 x 4096 (10.4 vs 8.8 us)
    const bool ok = nested ? launch_gemv_cu<T, true>(m, k, A, B, st, datatype, out, ldb, lds)
                           : launch_gemv_cu<T, false>(m, k, A, B, st, datatype, out, ldb, lds);
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

// [additive, testing] 0 = auto (the 4-waves-x-R-rows kernel), 2 = the one-workgroup-per-CU kernel
void cgemv_4bit_set_kernel(int which) { bnb::g_gemv_kernel = which; }

void cgemm_4bit_inference_naive_fp16(int m, int n, int k, fp16_t* A, unsigned char* B, float* absmax, float* datatype,
                                     fp16_t* out, int lda, int ldb, int ldc, int blocksize) {
  gemv_4bit<fp16_t>(m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize);
}
void cgemm_4bit_inference_naive_bf16(int m, int n, int k, bf16_t* A, unsigned char* B, float* absmax, float* datatype,
                                     bf16_t* out, int lda, int ldb, int ldc, int blocksize) {
  gemv_4bit<bf16_t>(m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize);
}
void cgemm_4bit_inference_naive_fp32(int m, int n, int k, float* A, unsigned char* B, float* absmax, float* datatype,
                                     float* out, int lda, int ldb, int ldc, int blocksize) {
  gemv_4bit<float>(m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize);
}

// Decode GEMV with compressed statistics decoded in-kernel (replaces the dequantize_blockwise launch of
// functional.py:1982-1984 + the gemv).  Returns 0 when launched, 1 when the shape needs the two-step path.
int cgemm_4bit_inference_naive_nested_fp16(int m, int n, int k, fp16_t* A, unsigned char* B, unsigned char* absmax_q,
                                           float* code2, float* absmax2, float* offset, float* datatype, fp16_t* out,
                                           int lda, int ldb, int ldc, int blocksize, int blocksize2) {
  (void)n; (void)lda; (void)ldc;
  GemvStats st{nullptr, absmax_q, code2, absmax2, offset, 0, 0};
  if (m <= 0) return 0;
  if (!launch_gemv_dot<fp16_t>(m, k, A, B, st, datatype, out, ldb, blocksize, blocksize2)) return 1;
  BNB_LAUNCH_CHECK("gemv_4bit_nested");
  return 0;
}
int cgemm_4bit_inference_naive_nested_bf16(int m, int n, int k, bf16_t* A, unsigned char* B, unsigned char* absmax_q,
                                           float* code2, float* absmax2, float* offset, float* datatype, bf16_t* out,
                                           int lda, int ldb, int ldc, int blocksize, int blocksize2) {
  (void)n; (void)lda; (void)ldc;
  GemvStats st{nullptr, absmax_q, code2, absmax2, offset, 0, 0};
  if (m <= 0) return 0;
  if (!launch_gemv_dot<bf16_t>(m, k, A, B, st, datatype, out, ldb, blocksize, blocksize2)) return 1;
  BNB_LAUNCH_CHECK("gemv_4bit_nested");
  return 0;
}

}  // extern "C"
