// Blockwise quantize / dequantize for gfx950.
//
// Replaces (same C-ABI names, argument order and meaning):
//   cquantize_blockwise_{fp16,bf16,fp32}{,_fp4,_nf4}     ref:sycl/pythonInterface.cpp:203-217
//   cdequantize_blockwise_{fp16,bf16,fp32}{,_fp4,_nf4}   ref:sycl/pythonInterface.cpp:199-221
//   cquantize_blockwise_cpu_fp32 / cdequantize_blockwise_cpu_fp32   ref:sycl/pythonInterface.cpp:419-420
// Semantics: kQuantizeBlockwise ref:sycl/sycl_code/kernel_quant.cpp:1229-1365 and
// kDequantizeBlockwise 1370-1471 with the intended full-size behaviour.
//
// Layout in HBM: A is n contiguous elements; absmax is fp32[ceil(n/bs)]; 4-bit output is
// ceil(n/2) bytes (high nibble = even element), 8-bit output is n bytes.
//
// Design (MI355X): quantize is one pass, 8 elements per lane, one quantisation block per
// 8..512 contiguous lanes; the per-block absmax is a wave64 xor-shuffle reduction (plus an
// LDS combine across waves for bs >= 1024).  Dequantize streams 16 packed bytes per lane
// (one 16-B load) through a 256-entry LDS pair table (byte -> two code values) and writes
// 16-B vector stores: it is HBM-bound (roofline: 0.5 B in + 2 B out per bf16 element).
#include "common.hpp"

#include <type_traits>

namespace bnb {

// ============================================================================ quantize

template <typename T> struct Load8;
template <> struct Load8<float> {
  __device__ static __forceinline__ void load(const float* p, float (&v)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
};
template <> struct Load8<fp16_t> {
  __device__ static __forceinline__ void load(const fp16_t* p, float (&v)[8]) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = (float)__builtin_bit_cast(fp16_t, (uint16_t)(w[i] & 0xFFFF));
      v[2 * i + 1] = (float)__builtin_bit_cast(fp16_t, (uint16_t)(w[i] >> 16));
    }
  }
};
template <> struct Load8<bf16_t> {
  __device__ static __forceinline__ void load(const bf16_t* p, float (&v)[8]) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
    }
  }
};

// THREADS lanes per CTA, 8 elements per lane; a quantisation block spans BS/8 lanes.
template <typename T, int BS, int DT, bool VEC>
__global__ void __launch_bounds__((BS / 8 > 256 ? BS / 8 : 256))
k_quantize_blockwise(const float* __restrict__ code, const T* __restrict__ A, float* __restrict__ absmax,
                     uint8_t* __restrict__ out, long long n) {
  constexpr int THREADS = (BS / 8 > 256 ? BS / 8 : 256);
  constexpr int G = BS / 8;                         // lanes per quantisation block
  constexpr int PER_CTA = THREADS * 8;
  __shared__ float s_code[256];
  __shared__ float s_wmax[THREADS / 64];
  if constexpr (DT == GENERAL8BIT) {
    for (int i = threadIdx.x; i < 256; i += THREADS) s_code[i] = code[i];
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  for (long long base = (long long)blockIdx.x * PER_CTA; base < n; base += (long long)gridDim.x * PER_CTA) {
    const long long e0 = base + (long long)threadIdx.x * 8;
    float v[8];
    if (VEC && e0 + 8 <= n) {
      Load8<T>::load(A + e0, v);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (e0 + j < n) ? Io<T>::to_f32(A[e0 + j]) : 0.0f;  // fill 0
    }
    float m = -3.402823466e+38f;
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
    if constexpr (G <= 64) {
      m = wave_max_xor(m, G);
    } else {
      m = wave_max_xor(m, 64);
      if (lane == 0) s_wmax[wave] = m;
      __syncthreads();
      constexpr int WPB = G / 64;                    // waves per quantisation block
      const int first = (wave / WPB) * WPB;
      m = s_wmax[first];
#pragma unroll
      for (int w = 1; w < WPB; ++w) m = fmaxf(m, s_wmax[first + w]);
      __syncthreads();
    }
    const long long blk = e0 / BS;
    if ((threadIdx.x % G) == 0 && e0 < n) absmax[blk] = m;
    const float r = 1.0f / m;                        // IEEE reciprocal (kernel_quant.cpp:1304)
    if constexpr (DT == GENERAL8BIT) {
      uint32_t q[8];
      float x[8], cq[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = __fmul_rn(v[j], r);
      quantize_dynamic8_n<8>(s_code, x, q, cq);      // the 8 searches interleaved (common.hpp)
      if (VEC && e0 + 8 <= n) {
        uint2 w;
        w.x = q[0] | (q[1] << 8) | (q[2] << 16) | (q[3] << 24);
        w.y = q[4] | (q[5] << 8) | (q[6] << 16) | (q[7] << 24);
        *reinterpret_cast<uint2*>(out + e0) = w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (e0 + j < n) out[e0 + j] = (uint8_t)q[j];
      }
    } else {
      uint32_t packed = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t hi = quant4<DT>(__fmul_rn(v[2 * j], r));
        const uint32_t lo = quant4<DT>(__fmul_rn(v[2 * j + 1], r));
        packed |= ((hi << 4) | lo) << (8 * j);
      }
      const long long b0 = e0 / 2;
      const long long nbytes = (n + 1) / 2;
      if (VEC && b0 + 4 <= nbytes) {
        *reinterpret_cast<uint32_t*>(out + b0) = packed;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (b0 + j < nbytes) out[b0 + j] = (uint8_t)(packed >> (8 * j));
      }
    }
  }
}

// ============================================================================ dequantize

template <typename T> struct Store;
template <> struct Store<bf16_t> {
  // 16 values -> 32 bytes
  __device__ static __forceinline__ void store16(bf16_t* p, const float (&v)[16]) {
    uint4 a, b;
    a.x = pack_bf16x2(v[0], v[1]);   a.y = pack_bf16x2(v[2], v[3]);
    a.z = pack_bf16x2(v[4], v[5]);   a.w = pack_bf16x2(v[6], v[7]);
    b.x = pack_bf16x2(v[8], v[9]);   b.y = pack_bf16x2(v[10], v[11]);
    b.z = pack_bf16x2(v[12], v[13]); b.w = pack_bf16x2(v[14], v[15]);
    reinterpret_cast<uint4*>(p)[0] = a;
    reinterpret_cast<uint4*>(p)[1] = b;
  }
};
template <> struct Store<fp16_t> {
  __device__ static __forceinline__ uint32_t pk(float a, float b) {
    return (uint32_t)__builtin_bit_cast(uint16_t, Io<fp16_t>::from_f32(a)) |
           ((uint32_t)__builtin_bit_cast(uint16_t, Io<fp16_t>::from_f32(b)) << 16);
  }
  __device__ static __forceinline__ void store16(fp16_t* p, const float (&v)[16]) {
    uint4 a, b;
    a.x = pk(v[0], v[1]);   a.y = pk(v[2], v[3]);   a.z = pk(v[4], v[5]);   a.w = pk(v[6], v[7]);
    b.x = pk(v[8], v[9]);   b.y = pk(v[10], v[11]); b.z = pk(v[12], v[13]); b.w = pk(v[14], v[15]);
    reinterpret_cast<uint4*>(p)[0] = a;
    reinterpret_cast<uint4*>(p)[1] = b;
  }
};
template <> struct Store<float> {
  __device__ static __forceinline__ void store16(float* p, const float (&v)[16]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      reinterpret_cast<float4*>(p)[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
  }
};

// Each lane owns 16 packed bytes.  4-bit: 32 elements; 8-bit: 16 elements.  bs >= 64
// guarantees one absmax per lane chunk.  The LDS table maps a byte to its code value(s).
template <typename T, int DT, bool VEC>
__global__ void __launch_bounds__(256)
k_dequantize_blockwise(const float* __restrict__ code, const uint8_t* __restrict__ A,
                       const float* __restrict__ absmax, T* __restrict__ out, int bs_shift, long long n) {
  __shared__ float2 s_pair[256];
  __shared__ float s_code[256];
  {
    const int b = threadIdx.x;
    if constexpr (DT == GENERAL8BIT) {
      s_code[b] = code[b];
    } else {
      s_pair[b] = make_float2(code4_value<DT>((uint32_t)b >> 4), code4_value<DT>((uint32_t)b & 15));
    }
  }
  __syncthreads();
  constexpr int EPL = (DT == GENERAL8BIT) ? 16 : 32;   // elements per lane
  const long long nbytes = (DT == GENERAL8BIT) ? n : (n + 1) / 2;
  const long long stride = (long long)gridDim.x * 256;
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t * 16 < nbytes; t += stride) {
    const long long byte0 = t * 16;
    const long long e0 = t * EPL;
    const float am = absmax[e0 >> bs_shift];
    if (VEC && e0 + EPL <= n) {
      const uint4 u = *reinterpret_cast<const uint4*>(A + byte0);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
      if constexpr (DT == GENERAL8BIT) {
        float v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = __fmul_rn(s_code[(w[i >> 2] >> (8 * (i & 3))) & 0xFF], am);
        Store<T>::store16(out + e0, v);
      } else {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float v[16];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float2 p = s_pair[(w[2 * h + (i >> 2)] >> (8 * (i & 3))) & 0xFF];
            v[2 * i] = __fmul_rn(p.x, am);
            v[2 * i + 1] = __fmul_rn(p.y, am);
          }
          Store<T>::store16(out + e0 + 16 * h, v);
        }
      }
    } else {
      for (int i = 0; i < 16; ++i) {
        const long long bi = byte0 + i;
        if (bi >= nbytes) break;
        const uint32_t byte = A[bi];
        if constexpr (DT == GENERAL8BIT) {
          out[bi] = Io<T>::from_f32(__fmul_rn(s_code[byte], absmax[bi >> bs_shift]));
        } else {
          const long long e = 2 * bi;
          const float2 p = s_pair[byte];
          out[e] = Io<T>::from_f32(__fmul_rn(p.x, absmax[e >> bs_shift]));
          if (e + 1 < n) out[e + 1] = Io<T>::from_f32(__fmul_rn(p.y, absmax[(e + 1) >> bs_shift]));
        }
      }
    }
  }
}

template <typename T> struct Pack2;
template <> struct Pack2<bf16_t> {
  __device__ static __forceinline__ uint32_t pk(float a, float b) { return pack_bf16x2(a, b); }
};
template <> struct Pack2<fp16_t> {
  __device__ static __forceinline__ uint32_t pk(float a, float b) { return Store<fp16_t>::pk(a, b); }
};

// 4-bit -> bf16/fp16 streaming dequantize (n % 8 == 0, 4-B aligned input, 16-B aligned output).
// Lane l of wave w owns packed dwords base + 64*(P*w + j) + l, j < P: every load instruction reads
// 256 contiguous bytes and every store instruction writes 1 KiB contiguous (8 outputs per lane).
// All P loads (+ their absmax) are issued before any is consumed.  Values are fp32 code*absmax,
// then one RNE cast -- identical to k_dequantize_blockwise.
// NESTED: the block statistics arrive compressed (compress_statistics=True) and are decoded in the
// kernel, absmax = code2[q8[b]] * absmax2[b >> bs2_shift] + offset in fp32 (the dequantize_blockwise
// product, then functional.py:1346-1350's `absmax += offset`), instead of a separate decode launch.
struct NestedStats {
  const uint8_t* q8;
  const float* code2;
  const float* absmax2;
  const float* offset;
  int bs2_shift;
};

// STP: store policy of the 16-B output stores -- 0 default (write-back L2), 1 non-temporal (nt), 2 device-scope
// write-through (sc1, through a buffer resource: the output below 2 GiB)
typedef uint32_t dq_u32x4 __attribute__((ext_vector_type(4)));
// SQ (round 5; NESTED, P = 8, blocksize 64, blocksize2 >= 64): a wave's pass covers 512 packed dwords = 64 statistics
// blocks, whose 64 codes are one aligned 64-B run and whose second-level scale is ONE value -- they come by two scalar
// loads per wave (s_load_dwordx16 + s_load_dword) instead of 8 + 8 per-lane vector loads (lanes 8 i .. 8 i + 7 share a
// block), leaving the vector-memory pipe the packed loads and the stores only.  Same values, same fp32 operations.
typedef const __attribute__((address_space(4))) uint32_t* dq_cu32_p;
typedef const __attribute__((address_space(4))) float* dq_cf32_p;
template <typename T, int DT, int P, bool NESTED = false, int STP = 0, bool SQ = false>
__global__ void __launch_bounds__(256)
k_dequantize_4bit_stream(const uint8_t* __restrict__ A, const float* __restrict__ absmax, T* __restrict__ out,
                         int bs_shift, long long ndw, NestedStats ns = {}) {
  static_assert(!SQ || (NESTED && P == 8), "scalar statistics: nested, 8 dwords per lane");
  __shared__ float2 s_pair[256];
  __shared__ float s_code2[NESTED ? 256 : 1];
  s_pair[threadIdx.x] = make_float2(code4_value<DT>(threadIdx.x >> 4), code4_value<DT>(threadIdx.x & 15));
  float off = 0.0f;
  if constexpr (NESTED) {
    s_code2[threadIdx.x] = ns.code2[threadIdx.x];
    off = *ns.offset;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t* Aw = reinterpret_cast<const uint32_t*>(A);
  const long long nblk = (ndw + 7) >> 3;                    // (SQ: blocksize 64 = 8 packed dwords per block)
  for (long long base = (long long)blockIdx.x * 256 * P; base < ndw; base += (long long)gridDim.x * 256 * P) {
    uint32_t w[P];
    float am[P];
    const long long blk0 = (base + 64LL * P * wave) >> 3;   // SQ: the wave's first block (wave-uniform, % 64 == 0)
    if (SQ && blk0 + 64 <= nblk) {
#pragma unroll
      for (int j = 0; j < P; ++j) w[j] = __builtin_nontemporal_load(Aw + min(base + 64LL * (P * wave + j) + lane, ndw - 1));
      uint32_t qv[16];
      const dq_cu32_p qc = (dq_cu32_p)(ns.q8 + blk0);
#pragma unroll
      for (int i = 0; i < 16; ++i) qv[i] = qc[i];
      const float a2 = *(dq_cf32_p)(ns.absmax2 + (blk0 >> ns.bs2_shift));
      // dword j of the lane is in block blk0 + 8 j + (lane >> 3): code byte (lane >> 3) & 3 of qv[2 j + (lane >> 5)]
      const int sh = 8 * ((lane >> 3) & 3);
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const uint32_t qw = (lane & 32) ? qv[2 * j + 1] : qv[2 * j];
        am[j] = __fadd_rn(__fmul_rn(s_code2[(qw >> sh) & 0xFF], a2), off);
      }
    } else {
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const long long d = min(base + 64LL * (P * wave + j) + lane, ndw - 1);
        w[j] = __builtin_nontemporal_load(Aw + d);
        if constexpr (NESTED) {
          const long long blk = (8 * d) >> bs_shift;
          am[j] = __fadd_rn(__fmul_rn(s_code2[ns.q8[blk]], ns.absmax2[blk >> ns.bs2_shift]), off);
        } else {
          am[j] = absmax[(8 * d) >> bs_shift];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const long long d = base + 64LL * (P * wave + j) + lane;
      float v[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float2 p = s_pair[(w[j] >> (8 * i)) & 0xFF];
        v[2 * i] = __fmul_rn(p.x, am[j]);
        v[2 * i + 1] = __fmul_rn(p.y, am[j]);
      }
      if (d < ndw) {
        uint4 o;
        o.x = Pack2<T>::pk(v[0], v[1]); o.y = Pack2<T>::pk(v[2], v[3]);
        o.z = Pack2<T>::pk(v[4], v[5]); o.w = Pack2<T>::pk(v[6], v[7]);
        if constexpr (STP == 1) {
          __builtin_nontemporal_store((dq_u32x4){o.x, o.y, o.z, o.w}, reinterpret_cast<dq_u32x4*>(out) + d);
        } else if constexpr (STP == 2) {
          const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0x7FFFFFFF, 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128((dq_u32x4){o.x, o.y, o.z, o.w}, r, (int)(16 * d), 0, 16);
        } else {
          reinterpret_cast<uint4*>(out)[d] = o;
        }
      }
    }
  }
}

// ============================================================================ CPU-path semantics
// The reference's host-pointer functions (cpu_ops.cpp).  Here they are executed on the GPU:
// host buffers are staged into HBM, processed by the kernels below, and copied back.

__global__ void k_quantize_cpu_semantics(const float* __restrict__ code, const float* __restrict__ A,
                                         float* __restrict__ absmax, uint8_t* __restrict__ out,
                                         long long blocksize, long long n) {
  // one workgroup per quantisation block (any blocksize): absmax = fmax over |A| from -FLT_MAX;
  // z = A / absmax (division: common.cpp:21); left neighbour + strictly-closer-right rule.
  __shared__ float s_code[256];
  __shared__ float s_red[4];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_code[i] = code[i];
  if (threadIdx.x == 0) s_code[0] = -1.0f;   // cpu_ops.cpp:20
  const long long b0 = (long long)blockIdx.x * blocksize;
  const long long b1 = (b0 + blocksize < n) ? b0 + blocksize : n;
  float m = -3.402823466e+38f;
  for (long long i = b0 + threadIdx.x; i < b1; i += blockDim.x) m = fmaxf(m, fabsf(A[i]));
  m = wave_max_xor(m, 64);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(s_red[0], s_red[1]), fmaxf(s_red[2], s_red[3]));
  if (threadIdx.x == 0) absmax[blockIdx.x] = m;
  for (long long i = b0 + threadIdx.x; i < b1; i += blockDim.x) {
    const float z = __fdiv_rn(A[i], m);
    int lo = 0, hi = 256;   // upper_bound
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s_code[mid] <= z) lo = mid + 1; else hi = mid;
    }
    int idx = lo - 1;
    if (idx < 0 || z != z) idx = 0;
    if (idx < 255) {
      const float dl = fabsf(__fsub_rn(z, s_code[idx]));
      const float dr = fabsf(__fsub_rn(z, s_code[idx + 1]));
      if (dr < dl) idx += 1;
    }
    out[i] = (uint8_t)idx;
  }
}

__global__ void k_dequantize_cpu_semantics(const float* __restrict__ code, const uint8_t* __restrict__ A,
                                           const float* __restrict__ absmax, float* __restrict__ out,
                                           long long blocksize, long long n) {
  __shared__ float s_code[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_code[i] = code[i];
  __syncthreads();
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = __fmul_rn(s_code[A[i]], absmax[i / blocksize]);
}

// ============================================================================ launchers

static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static inline int stream_grid(long long work_items, int threads) {
  long long g = (work_items + threads - 1) / threads;
  if (g < 1) g = 1;
  if (g > 8192) g = 8192;
  return (int)g;
}

template <typename T, int DT, int BS>
static void launch_quant_bs(const float* code, const T* A, float* absmax, uint8_t* out, long long n, bool vec) {
  constexpr int THREADS = (BS / 8 > 256 ? BS / 8 : 256);
  const int grid = stream_grid((n + 7) / 8, THREADS);
  if (vec)
    hipLaunchKernelGGL((k_quantize_blockwise<T, BS, DT, true>), dim3(grid), dim3(THREADS), 0, current_stream(), code, A, absmax, out, n);
  else
    hipLaunchKernelGGL((k_quantize_blockwise<T, BS, DT, false>), dim3(grid), dim3(THREADS), 0, current_stream(), code, A, absmax, out, n);
}

template <typename T, int DT>
void quantize_blockwise(const float* code, const T* A, float* absmax, uint8_t* out, int blocksize, long long n) {
  if (n <= 0) return;
  const bool vec = aligned16(A) && ((uintptr_t)out & 7) == 0;
  switch (blocksize) {
    case 4096: launch_quant_bs<T, DT, 4096>(code, A, absmax, out, n, vec); break;
    case 2048: launch_quant_bs<T, DT, 2048>(code, A, absmax, out, n, vec); break;
    case 1024: launch_quant_bs<T, DT, 1024>(code, A, absmax, out, n, vec); break;
    case 512: launch_quant_bs<T, DT, 512>(code, A, absmax, out, n, vec); break;
    case 256: launch_quant_bs<T, DT, 256>(code, A, absmax, out, n, vec); break;
    case 128: launch_quant_bs<T, DT, 128>(code, A, absmax, out, n, vec); break;
    case 64: launch_quant_bs<T, DT, 64>(code, A, absmax, out, n, vec); break;
    default: set_error(1, "quantize_blockwise: unsupported blocksize"); return;
  }
  BNB_LAUNCH_CHECK("quantize_blockwise");
}

// Launch shape of k_dequantize_4bit_stream (A/B knob cdequantize_set_stream_cfg): dwords per lane per pass (4, 8 or 16)
// and a cap on the grid (0: one pass per workgroup; else at most that many workgroups, grid-stride passes)
// store policy (cdequantize_set_store_policy): 2 = write-through by default.  The 90 MB bf16 weight of the metric step
// then leaves no dirty L2 lines for the kernel end / boundary to write back: the dequantise alone 23.1 -> 14.9 us, the
// metric step 263.3 -> 260.2 us, C1 8.85 -> 8.6 us; non-temporal stores 20.8 us alone but a slower step (266.0)
// (tools/dequant_store_ab.py, tools/bench_knobs.py; profiles/lab/r04_store_policy.txt)
static Knob<int> g_dq_p{8}, g_dq_grid_cap{0}, g_dq_store{2};
// scalar-loaded nested statistics (SQ above; cdequantize_set_nested_scalar): 1 = where they apply, 0 = off (default).
// Measured and rejected (round 5, tools/r05_epi_ab.py, profiles/lab/r05_ab.txt): bit-identical, but the metric weight's
// dequantise takes 30.6 us against 15.1 us with the per-lane loads (back to back), the metric step 265.5 vs 258.0 us --
// each wave waits on its scalar loads before any of its math, where the per-lane loads overlap across waves.
static Knob<int> g_dq_sq{0};
template <typename T, int DT, bool NESTED>
static void launch_dq_stream(const uint8_t* A, const float* absmax, T* out, int bs_shift, long long ndw,
                             const NestedStats& ns) {
  auto go = [&](auto pc) {
    constexpr int P = decltype(pc)::value;
    long long wgs = (ndw + 256 * P - 1) / (256 * P);
    if (wgs > 65536) wgs = 65536;
    if (g_dq_grid_cap > 0 && wgs > g_dq_grid_cap) wgs = g_dq_grid_cap;
    auto launch = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((int)wgs), dim3(256), 0, current_stream(), A, absmax, out, bs_shift, ndw, ns);
    };
    if constexpr (P == 8 && sizeof(T) == 2) {               // store-policy variants (the default shape only)
      if constexpr (NESTED) {
        // (64-B aligned codes: each wave's 64-code run is one aligned scalar load; every run read lies inside the codes)
        if (g_dq_sq && g_dq_store == 2 && ndw * 16 <= 0x7FFFFFFFLL && bs_shift == 6 && ns.bs2_shift >= 6 &&
            ((uintptr_t)ns.q8 & 63) == 0 && ((uintptr_t)ns.absmax2 & 3) == 0)
          return launch(k_dequantize_4bit_stream<T, DT, P, NESTED, 2, true>);
      }
      if (g_dq_store == 1) return launch(k_dequantize_4bit_stream<T, DT, P, NESTED, 1>);
      if (g_dq_store == 2 && ndw * 16 <= 0x7FFFFFFFLL) return launch(k_dequantize_4bit_stream<T, DT, P, NESTED, 2>);
    }
    launch(k_dequantize_4bit_stream<T, DT, P, NESTED>);
  };
  if (g_dq_p == 4) go(std::integral_constant<int, 4>{});
  else if (g_dq_p == 16) go(std::integral_constant<int, 16>{});
  else go(std::integral_constant<int, 8>{});
}

template <typename T, int DT>
void dequantize_blockwise(const float* code, const uint8_t* A, const float* absmax, T* out, int blocksize, long long n) {
  if (n <= 0) return;
  if (blocksize < 64 || (blocksize & (blocksize - 1))) { set_error(1, "dequantize_blockwise: unsupported blocksize"); return; }
  if constexpr (DT != GENERAL8BIT && sizeof(T) == 2) {
    if (n % 8 == 0 && ((uintptr_t)A & 3) == 0 && aligned16(out)) {
      launch_dq_stream<T, DT, false>(A, absmax, out, __builtin_ctz(blocksize), n / 8, NestedStats{});
      BNB_LAUNCH_CHECK("dequantize_blockwise");
      return;
    }
  }
  const long long nbytes = (DT == GENERAL8BIT) ? n : (n + 1) / 2;
  const int grid = stream_grid((nbytes + 15) / 16, 256);
  const bool vec = aligned16(A) && aligned16(out);
  if (vec)
    hipLaunchKernelGGL((k_dequantize_blockwise<T, DT, true>), dim3(grid), dim3(256), 0, current_stream(), code, A, absmax, out, __builtin_ctz(blocksize), n);
  else
    hipLaunchKernelGGL((k_dequantize_blockwise<T, DT, false>), dim3(grid), dim3(256), 0, current_stream(), code, A, absmax, out, __builtin_ctz(blocksize), n);
  BNB_LAUNCH_CHECK("dequantize_blockwise");
}

// 4-bit dequantise with compressed statistics in one launch; false when the shape needs the two-step path
template <typename T, int DT>
bool dequantize_4bit_nested(const uint8_t* A, const uint8_t* q8, const float* code2, const float* absmax2,
                            const float* offset, T* out, int blocksize, int blocksize2, long long n) {
  if (n <= 0) return true;
  if (blocksize < 64 || (blocksize & (blocksize - 1)) || blocksize2 <= 0 || (blocksize2 & (blocksize2 - 1)) ||
      n % 8 != 0 || ((uintptr_t)A & 3) != 0 || !aligned16(out))
    return false;
  const NestedStats ns{q8, code2, absmax2, offset, __builtin_ctz(blocksize2)};
  launch_dq_stream<T, DT, true>(A, nullptr, out, __builtin_ctz(blocksize), n / 8, ns);
  BNB_LAUNCH_CHECK("dequantize_4bit_nested");
  return true;
}

// Nested statistics -> fp32 absmax in one pass: out[i] = code2[q[i]] * absmax2[i >> bs2_shift] + offset,
// the fp32 product of dequantize_blockwise (kernel_quant.cpp:1430-1435) then the fp32 `absmax += offset`
// of functional.py:1346-1350 (two roundings, as the two-step path).  16 codes per thread.
__global__ void __launch_bounds__(256)
k_dequantize_nested_absmax(const float* __restrict__ code2, const uint8_t* __restrict__ q, const float* __restrict__ absmax2,
                           const float* __restrict__ offset, float* __restrict__ out, int bs2_shift, long long n) {
  __shared__ float c2[256];
  c2[threadIdx.x] = code2[threadIdx.x];
  const float off = *offset;
  __syncthreads();
  const long long i0 = 16 * ((long long)blockIdx.x * 256 + threadIdx.x);
  if (i0 >= n) return;
  if (i0 + 16 <= n && (((uintptr_t)(q + i0)) & 15) == 0 && (((uintptr_t)(out + i0)) & 15) == 0) {
    const uint4 v = *reinterpret_cast<const uint4*>(q + i0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      float r[4];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const long long i = i0 + 4 * d + b;
        r[b] = __fadd_rn(__fmul_rn(c2[(w[d] >> (8 * b)) & 0xFF], absmax2[i >> bs2_shift]), off);
      }
      reinterpret_cast<float4*>(out + i0)[d] = make_float4(r[0], r[1], r[2], r[3]);
    }
  } else {
    for (long long i = i0; i < i0 + 16 && i < n; ++i) out[i] = __fadd_rn(__fmul_rn(c2[q[i]], absmax2[i >> bs2_shift]), off);
  }
}

}  // namespace bnb

using namespace bnb;

// ============================================================================ C-ABI
extern "C" {

// [additive, testing] k_dequantize_4bit_stream launch shape: p = packed dwords per lane per pass (4, 8, 16), grid_cap =
// at most this many workgroups (0: none); returns the previous p
int cdequantize_set_stream_cfg(int p, int grid_cap) {
  const int prev = g_dq_p;
  g_dq_p = p;
  g_dq_grid_cap = grid_cap;
  return prev;
}
// [additive, testing] nested statistics of k_dequantize_4bit_stream by scalar loads (1, where they apply) or per lane
// (0, default: the scalar form measured 2x slower); bit-identical; returns the previous setting
int cdequantize_set_nested_scalar(int on) {
  const int prev = g_dq_sq;
  g_dq_sq = on ? 1 : 0;
  return prev;
}
// [additive, testing] store policy of k_dequantize_4bit_stream's 16-bit outputs (default launch shape): 0 = write-back,
// 1 = non-temporal, 2 (default) = device-scope write-through; returns the previous setting
int cdequantize_set_store_policy(int policy) {
  const int prev = g_dq_store;
  g_dq_store = policy;
  return prev;
}

#define BNB_QUANT_ABI(fname, T, DT)                                                                   \
  void fname(float* code, T* A, float* absmax, unsigned char* out, int blocksize, const int n) {     \
    BNB_RANGE(#fname);                                                                                \
    quantize_blockwise<T, DT>(code, A, absmax, out, blocksize, n);                                    \
  }
#define BNB_DEQUANT_ABI(fname, T, DT)                                                                 \
  void fname(float* code, unsigned char* A, float* absmax, T* out, int blocksize, const int n) {     \
    BNB_RANGE(#fname);                                                                                \
    dequantize_blockwise<T, DT>(code, A, absmax, out, blocksize, n);                                  \
  }

BNB_QUANT_ABI(cquantize_blockwise_fp16, fp16_t, GENERAL8BIT)
BNB_QUANT_ABI(cquantize_blockwise_fp16_fp4, fp16_t, FP4)
BNB_QUANT_ABI(cquantize_blockwise_fp16_nf4, fp16_t, NF4)
BNB_QUANT_ABI(cquantize_blockwise_bf16, bf16_t, GENERAL8BIT)
BNB_QUANT_ABI(cquantize_blockwise_bf16_fp4, bf16_t, FP4)
BNB_QUANT_ABI(cquantize_blockwise_bf16_nf4, bf16_t, NF4)
BNB_QUANT_ABI(cquantize_blockwise_fp32, float, GENERAL8BIT)
BNB_QUANT_ABI(cquantize_blockwise_fp32_fp4, float, FP4)
BNB_QUANT_ABI(cquantize_blockwise_fp32_nf4, float, NF4)

BNB_DEQUANT_ABI(cdequantize_blockwise_fp16, fp16_t, GENERAL8BIT)
BNB_DEQUANT_ABI(cdequantize_blockwise_fp16_fp4, fp16_t, FP4)
BNB_DEQUANT_ABI(cdequantize_blockwise_fp16_nf4, fp16_t, NF4)
BNB_DEQUANT_ABI(cdequantize_blockwise_bf16, bf16_t, GENERAL8BIT)
BNB_DEQUANT_ABI(cdequantize_blockwise_bf16_fp4, bf16_t, FP4)
BNB_DEQUANT_ABI(cdequantize_blockwise_bf16_nf4, bf16_t, NF4)
BNB_DEQUANT_ABI(cdequantize_blockwise_fp32, float, GENERAL8BIT)
BNB_DEQUANT_ABI(cdequantize_blockwise_fp32_fp4, float, FP4)
BNB_DEQUANT_ABI(cdequantize_blockwise_fp32_nf4, float, NF4)

// [additive] 4-bit dequantise with compressed statistics decoded in the kernel (one launch instead of
// the dequantize_blockwise of the absmax + the 4-bit dequantise, functional.py:1342-1350).  Returns 0 when
// launched, 1 when the shape needs the two-step path.
#define BNB_DEQUANT_NESTED_ABI(fname, T, DT)                                                                    \
  int fname(unsigned char* A, unsigned char* absmax_q, float* code2, float* absmax2, float* offset, T* out,      \
            int blocksize, int blocksize2, long long n) {                                                        \
    BNB_RANGE(#fname);                                                                                            \
    return dequantize_4bit_nested<T, DT>(A, absmax_q, code2, absmax2, offset, out, blocksize, blocksize2, n) ? 0  \
                                                                                                             : 1; \
  }
BNB_DEQUANT_NESTED_ABI(cdequantize_blockwise_nested_fp16_fp4, fp16_t, FP4)
BNB_DEQUANT_NESTED_ABI(cdequantize_blockwise_nested_fp16_nf4, fp16_t, NF4)
BNB_DEQUANT_NESTED_ABI(cdequantize_blockwise_nested_bf16_fp4, bf16_t, FP4)
BNB_DEQUANT_NESTED_ABI(cdequantize_blockwise_nested_bf16_nf4, bf16_t, NF4)

// The host-pointer entry points cquantize_blockwise_cpu_fp32 / cdequantize_blockwise_cpu_fp32
// (ref:sycl/pythonInterface.cpp:419-420) run on the host cores: cpu_ops.cpp.

// [additive] device-pointer form of the CPU-path quantize (the same division / nearest-code semantics,
// one byte per element, any blocksize) executed on the GPU; `code` is a device pointer and is NOT
// rewritten (the kernel uses code[0] = -1 internally).
void cquantize_blockwise_bytes_fp32(float* code, float* A, float* absmax, unsigned char* out, long long blocksize,
                                    long long n) {
  BNB_RANGE("cquantize_blockwise_bytes_fp32");
  if (n <= 0 || blocksize <= 0) return;
  const long long nb = (n + blocksize - 1) / blocksize;
  if (nb > 0x7fffffffLL) { set_error(1, "quantize_bytes: too many blocks"); return; }
  hipLaunchKernelGGL(k_quantize_cpu_semantics, dim3((unsigned)nb), dim3(256), 0, current_stream(), code, A, absmax,
                     out, blocksize, n);
  BNB_LAUNCH_CHECK("quantize_bytes");
}

// [additive] nested statistics -> fp32 absmax in one launch (replaces dequantize_blockwise + the
// offset add of functional.py:1346-1350); blocksize2 must be a power of two.
void cdequantize_nested_absmax_fp32(float* code2, unsigned char* q, float* absmax2, float* offset, float* out,
                                    int blocksize2, long long n) {
  BNB_RANGE("cdequantize_nested_absmax_fp32");
  if (n <= 0) return;
  if (blocksize2 <= 0 || (blocksize2 & (blocksize2 - 1))) {
    set_error(1, "dequantize_nested_absmax: blocksize2 must be a power of two");
    return;
  }
  const unsigned grid = (unsigned)((n + 16 * 256 - 1) / (16 * 256));
  hipLaunchKernelGGL(k_dequantize_nested_absmax, dim3(grid), dim3(256), 0, current_stream(), code2, q, absmax2, offset,
                     out, __builtin_ctz(blocksize2), n);
  BNB_LAUNCH_CHECK("dequantize_nested_absmax");
}

// Device-resident variant of the CPU-path dequantize (one byte per element, any blocksize);
// used by the config-1 GPU measurement.  Not in the reference ABI.
void cdequantize_blockwise_bytes_fp32(float* code, unsigned char* A, float* absmax, float* out, long long blocksize,
                                      long long n) {
  BNB_RANGE("cdequantize_blockwise_bytes_fp32");
  if (n <= 0 || blocksize <= 0) return;
  hipLaunchKernelGGL(k_dequantize_cpu_semantics, dim3(stream_grid(n, 256)), dim3(256), 0, current_stream(), code, A,
                     absmax, out, blocksize, n);
  BNB_LAUNCH_CHECK("dequantize_bytes");
}

}  // extern "C"
