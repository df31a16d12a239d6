// Optimizer updates: 8-bit blockwise states and 32-bit states, gfx950.
//
//   8-bit blockwise  kOptimizerStatic8bit2StateBlockwise  ref:sycl/sycl_code/kernel_quant.cpp:2715-2972
//                    kOptimizerStatic8bit1StateBlockwise  ref:sycl/sycl_code/kernel_quant.cpp:2977-3208
//                    launcher optimizerStatic8bitBlockwise ref:sycl/sycl_code/op_quant.cpp:1135-1240
//                    C-ABI c<name>_8bit_blockwise_grad_<T> ref:sycl/pythonInterface.cpp:264-284
//   32-bit           kOptimizer32bit2State / 1State       ref:sycl/sycl_code/kernel_quant.cpp:1614-2060
//                    C-ABI c<name>32bit_grad_<T>          ref:sycl/pythonInterface.cpp:223-241
//
// Semantics are the reference's formulas, op for op in fp32 (build: -ffp-contract=off), with the
// intended behaviour where the reference is defective:
//   * the state re-quantiser is the dynamic-map binary search with midpoint rounding that
//     quantize_2D performs upstream (kernel_quant.cpp:840-888 compares against 0 instead of the code
//     after the first step, Q21); with code[255] == 1 it equals dQuantize<0>, quantize_dynamic8 here;
//   * 1-state optimizers are selected by the enum of ops.h:68-76 (MOMENTUM 1, RMSPROP 2, ADAGRAD 4,
//     LION 5); the reference's kernel switches on 1/2/3/4, so ADAGRAD runs the Lion update and LION
//     runs none (Q22);
//   * tail elements of the last 2048-block are loaded as the upstream defaults (g = 0, state1 code
//     128, state2 code 0) and never stored; the reference loads past n (Q2-style, Q23).
// sqrt is __builtin_sqrtf, which hipcc lowers to the correctly rounded sequence (v_sqrt_f32 + two fma
// residual checks); __fsqrt_rn lowers to the bare 1-ulp v_sqrt_f32 on ROCm 7.2.
// The bias corrections are computed once on the host in double (the reference's pow(float, int)
// promotes to double) and rounded to fp32, as the oracle does.
//
// MI355X design: 16 B/element of HBM traffic for Adam fp32 8-bit (g, p read+write, two state bytes
// read+write), but VALU-bound in practice (a wave64 VALU op issues over 4 cycles; ~1450 per
// wave-block in the first version).  A 256-thread workgroup walks 2048-element blocks (grid = 4x the
// resident workgroups) with the next block's loads in flight; 8 contiguous elements per thread
// (16/32-B vector loads); the maps in LDS in the search layout of common.hpp DynMapView (branch-free,
// level-synchronous Eytzinger search, 3 VALU per level); the re-quantisation quotient via an fp64
// reciprocal product (exact, see requant8); one barrier per block for both absmax reductions.
// Lab (tools/optim_lab.hip, 2^27 fp32 elements): 920 us -> 676-689 us, bit-identical to the scalar form.
#include "common.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>

namespace bnb {

enum OptimizerKind { ADAM = 0, MOMENTUM = 1, RMSPROP = 2, LARS = 3, ADAGRAD = 4, LION = 5 };   // ref ops.h:68-76

constexpr int OPT_BLOCK = 2048, OPT_THREADS = 256, OPT_NPT = 8;

struct OptScalars {
  float beta1, beta2, eps, lr, weight_decay, gnorm_scale;
  float step_size;      // (-lr * correction2) / correction1
  float c2eps;          // correction2 * eps
  float decay;          // 1 - lr * weight_decay
  int step;
  bool skip_zeros;
};

__device__ __forceinline__ float sgnf(float x) { return (float)((x > 0.0f) - (x < 0.0f)); }

// 8 contiguous elements of T <-> fp32 (vector accesses when the whole group is in range and aligned)
template <typename T>
__device__ __forceinline__ void load8(const T* __restrict__ src, long long i, int n, float (&v)[8], float fill) {
  if (i + 8 <= n && (((uintptr_t)(src + i)) & 15) == 0) {
    if constexpr (sizeof(T) == 4) {
      const float4 a = reinterpret_cast<const float4*>(src + i)[0], b = reinterpret_cast<const float4*>(src + i)[1];
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
      const uint4 u = *reinterpret_cast<const uint4*>(src + i);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[2 * j] = Io<T>::to_f32(__builtin_bit_cast(T, (uint16_t)(w[j] & 0xFFFF)));
        v[2 * j + 1] = Io<T>::to_f32(__builtin_bit_cast(T, (uint16_t)(w[j] >> 16)));
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (i + j < n) ? Io<T>::to_f32(src[i + j]) : fill;
  }
}
template <typename T>
__device__ __forceinline__ void store8(T* __restrict__ dst, long long i, int n, const T (&v)[8]) {
  if (i + 8 <= n && (((uintptr_t)(dst + i)) & 15) == 0) {
    if constexpr (sizeof(T) == 4) {
      reinterpret_cast<float4*>(dst + i)[0] = make_float4(v[0], v[1], v[2], v[3]);
      reinterpret_cast<float4*>(dst + i)[1] = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        w[j] = (uint32_t)__builtin_bit_cast(uint16_t, v[2 * j]) | ((uint32_t)__builtin_bit_cast(uint16_t, v[2 * j + 1]) << 16);
      *reinterpret_cast<uint4*>(dst + i) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (i + j < n) dst[i + j] = v[j];
  }
}
__device__ __forceinline__ void load8u(const uint8_t* __restrict__ src, long long i, int n, uint32_t (&c)[8], uint32_t fill) {
  if (i + 8 <= n && (((uintptr_t)(src + i)) & 7) == 0) {
    const uint2 u = *reinterpret_cast<const uint2*>(src + i);
#pragma unroll
    for (int j = 0; j < 4; ++j) { c[j] = (u.x >> (8 * j)) & 0xFF; c[4 + j] = (u.y >> (8 * j)) & 0xFF; }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = (i + j < n) ? src[i + j] : fill;
  }
}
// 8 state bytes packed little-endian in a uint2 (tail bytes = fill)
__device__ __forceinline__ uint2 load8u_packed(const uint8_t* __restrict__ src, long long i, int n, uint32_t fill) {
  if (i + 8 <= n && (((uintptr_t)(src + i)) & 7) == 0) return *reinterpret_cast<const uint2*>(src + i);
  uint32_t w[2] = {0, 0};
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j >> 2] |= ((i + j < n) ? (uint32_t)src[i + j] : fill) << (8 * (j & 3));
  return make_uint2(w[0], w[1]);
}
__device__ __forceinline__ void store8u(uint8_t* __restrict__ dst, long long i, int n, const uint32_t (&c)[8]) {
  if (i + 8 <= n && (((uintptr_t)(dst + i)) & 7) == 0) {
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) { lo |= (c[j] & 0xFF) << (8 * j); hi |= (c[4 + j] & 0xFF) << (8 * j); }
    *reinterpret_cast<uint2*>(dst + i) = make_uint2(lo, hi);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (i + j < n) dst[i + j] = (uint8_t)c[j];
  }
}

// re-quantise a state value against its block absmax; the signed map keeps the sign of the value
// (kernel_quant.cpp:2930-2941)
template <bool SIGNED, class Code>
__device__ __forceinline__ uint32_t requant(Code code, float s, float absmax) {
  uint32_t c = quantize_dynamic8(code, __fdiv_rn(s, absmax));
  if (SIGNED && ((__float_as_uint(code[c]) ^ __float_as_uint(s)) >> 31)) c = (s > 0.0f) ? ((c + 1) & 0xFF) : ((c - 1) & 0xFF);
  return c;
}

// the same for the 8 values of a thread, searches interleaved (common.hpp dynmap_quantize_n)
template <bool SIGNED>
__device__ __forceinline__ void requant8(DynMapView code, const float (&s)[8], float absmax, uint32_t (&c)[8]) {
  // x = RN32(s / absmax) as (float)(s * RN64(1 / absmax)): 3 VALU instead of the ~11 of the fp32
  // division.  Exact: the fp64 product is within 2^-52 (relative) of s / absmax, while a quotient of
  // two 24-bit floats that is not itself a rounding midpoint lies at least 2^-49 from every midpoint
  // (s - m * absmax is a non-zero multiple of 2^(e_m + e_absmax) against |m * absmax| < 2^(49 + e_m +
  // e_absmax)), and an exact midpoint would need a 25-bit odd significand times a 24-bit one to fit in
  // 24 bits.  So the final rounding to fp32 lands where the IEEE division does (0/0 and x/inf alike).
  const double r64 = 1.0 / (double)absmax;
  float x[8], cq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (float)((double)s[j] * r64);
  dynmap_quantize_n<8, SIGNED>(code, x, c, cq);
  if (SIGNED) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if ((__float_as_uint(cq[j]) ^ __float_as_uint(s[j])) >> 31) c[j] = (s[j] > 0.0f) ? ((c[j] + 1) & 0xFF) : ((c[j] - 1) & 0xFF);
  }
}

// The maps live in LDS in the search layout of common.hpp DynMapView (breadth-first pivots, the
// final pick's records, the plain map for dequantisation).
template <bool TWO>
struct OptLds {
  float map1[DYNMAP_FLOATS], map2[TWO ? DYNMAP_FLOATS : 1];
  float xch[2][8];                               // double-buffered by block parity
};

// block max of two values over the workgroup with one barrier: xch alternates between two buffers
// by block parity, so the reads of block i finish (every wave passes block i+1's barrier) before
// block i+2 writes the same buffer
__device__ __forceinline__ void block_max256x2(float& a, float& b, float* xch) {
  a = wave_max_xor(a, 64);
  b = wave_max_xor(b, 64);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { xch[wave] = a; xch[4 + wave] = b; }
  __syncthreads();
  a = fmaxf(fmaxf(xch[0], xch[1]), fmaxf(xch[2], xch[3]));
  b = fmaxf(fmaxf(xch[4], xch[5]), fmaxf(xch[6], xch[7]));
}

// one thread's inputs of a 2048-block, kept packed while in flight (the prefetch of the next block)
template <typename T>
struct Opt2InT {
  float gv[8], pv[8];
  uint2 c1, c2;
  float am1, am2;
  __device__ __forceinline__ void load(const T* __restrict__ g, const T* __restrict__ p, const uint8_t* __restrict__ s1,
                                       const uint8_t* __restrict__ s2, const float* __restrict__ a1,
                                       const float* __restrict__ a2, long long blk, int n) {
    const long long i0 = blk * OPT_BLOCK + (long long)threadIdx.x * OPT_NPT;
    load8(g, i0, n, gv, 0.0f);
    c1 = load8u_packed(s1, i0, n, 0x80u);
    if (s2) c2 = load8u_packed(s2, i0, n, 0u);
    load8(p, i0, n, pv, 0.0f);
    am1 = a1[blk];
    am2 = a2 ? a2[blk] : 0.0f;
  }
  __device__ __forceinline__ void unpack(float (&g)[8], float (&p)[8], uint32_t (&q1)[8], uint32_t (&q2)[8]) const {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      g[j] = gv[j];
      p[j] = pv[j];
      q1[j] = ((j < 4 ? c1.x : c1.y) >> (8 * (j & 3))) & 0xFF;
      q2[j] = ((j < 4 ? c2.x : c2.y) >> (8 * (j & 3))) & 0xFF;
    }
  }
};

// ---------------------------------------------------------------- 8-bit blockwise, two states (Adam)
// FL (design lab only; 0 in the library): 1 = no re-quantisation, 2 = division only (timings of the
// parts), 8 = the scalar one-search-at-a-time re-quantiser
template <typename T, int OPT, int FL = 0>
__global__ void __launch_bounds__(OPT_THREADS)
k_optimizer_8bit_blockwise_2state(T* __restrict__ p, const T* __restrict__ g, uint8_t* __restrict__ state1,
                                  uint8_t* __restrict__ state2, const float* __restrict__ qmap1,
                                  const float* __restrict__ qmap2, float* __restrict__ absmax1,
                                  float* __restrict__ absmax2, OptScalars k, int n) {
  __shared__ __attribute__((aligned(16))) OptLds<true> L;
  dynmap_stage(L.map1, qmap1);
  dynmap_stage(L.map2, qmap2);
  __syncthreads();
  const DynMapView code1{reinterpret_cast<const char*>(L.map1)}, code2{reinterpret_cast<const char*>(L.map2)};
  const long long nb = (n + OPT_BLOCK - 1) / OPT_BLOCK;
  // software pipeline over the grid-stride loop: the next block's inputs are in flight while this
  // block's search runs (without it the HBM stream idles during the search, ~2x the HBM time)
  Opt2InT<T> in;
  long long blk = blockIdx.x;
  if (blk < nb) in.load(g, p, state1, state2, absmax1, absmax2, blk, n);
  for (int par = 0; blk < nb; blk += gridDim.x, par ^= 1) {
    const long long i0 = blk * OPT_BLOCK + (long long)threadIdx.x * OPT_NPT;
    float gv[8], pv[8], s1[8], s2[8];
    uint32_t c1[8], c2[8];
    in.unpack(gv, pv, c1, c2);
    const float am1 = in.am1, am2 = in.am2;
    if (blk + gridDim.x < nb) in.load(g, p, state1, state2, absmax1, absmax2, blk + gridDim.x, n);
    float m1 = -FLT_MAX, m2 = -FLT_MAX;
    bool ok[8];
    const float omb1 = __fsub_rn(1.0f, k.beta1), omb2 = __fsub_rn(1.0f, k.beta2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {                // branch-free: non-finite gradients select 0 states
      ok[j] = __builtin_isfinite(gv[j]);
      const float gs = __fmul_rn(gv[j], k.gnorm_scale);
      const float d2 = __fmul_rn(code2[c2[j]], am2), d1 = __fmul_rn(code1[c1[j]], am1);
      s2[j] = ok[j] ? __fadd_rn(__fmul_rn(d2, k.beta2), __fmul_rn(__fmul_rn(omb2, gs), gs)) : 0.0f;
      s1[j] = ok[j] ? __fadd_rn(__fmul_rn(d1, k.beta1), __fmul_rn(omb1, gs)) : 0.0f;
      m1 = fmaxf(m1, fabsf(s1[j]));
      m2 = fmaxf(m2, fabsf(s2[j]));
    }
    block_max256x2(m1, m2, L.xch[par]);
    if (threadIdx.x == 0) { absmax1[blk] = m1; absmax2[blk] = m2; }
    T po[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float upd = __fmul_rn(k.step_size, __fdiv_rn(s1[j], __fadd_rn(__builtin_sqrtf(s2[j]), k.c2eps)));
      T pt = Io<T>::from_f32(__fadd_rn(pv[j], upd));
      if (k.weight_decay > 0.0f) pt = Io<T>::from_f32(__fmul_rn(Io<T>::to_f32(pt), k.decay));
      po[j] = ok[j] ? pt : Io<T>::from_f32(pv[j]);
    }
    store8(p, i0, n, po);
    if constexpr (FL == 0) {
      requant8<true>(code1, s1, m1, c1);
      requant8<false>(code2, s2, m2, c2);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (FL & 1) {
          c1[j] = __float_as_uint(s1[j]) >> 24;
          c2[j] = __float_as_uint(s2[j]) >> 24;
        } else if (FL & 2) {                     // division only
          c1[j] = __float_as_uint(__fdiv_rn(s1[j], m1)) >> 24;
          c2[j] = __float_as_uint(__fdiv_rn(s2[j], m2)) >> 24;
        } else {                                 // FL 8: one search at a time (the scalar form)
          c1[j] = requant<true>(code1, s1[j], m1);
          c2[j] = requant<false>(code2, s2[j], m2);
        }
      }
    }
    store8u(state1, i0, n, c1);
    store8u(state2, i0, n, c2);
  }
}

// ---------------------------------------------------------------- 8-bit blockwise, one state
template <typename T, int OPT>
__global__ void __launch_bounds__(OPT_THREADS)
k_optimizer_8bit_blockwise_1state(T* __restrict__ p, const T* __restrict__ g, uint8_t* __restrict__ state1,
                                  const float* __restrict__ qmap1, float* __restrict__ absmax1, OptScalars k, int n) {
  __shared__ __attribute__((aligned(16))) OptLds<false> L;
  dynmap_stage(L.map1, qmap1);
  __syncthreads();
  const DynMapView code1{reinterpret_cast<const char*>(L.map1)};
  const long long nb = (n + OPT_BLOCK - 1) / OPT_BLOCK;
  Opt2InT<T> in;                                 // software pipeline, as the 2-state kernel
  long long blk = blockIdx.x;
  if (blk < nb) in.load(g, p, state1, nullptr, absmax1, nullptr, blk, n);
  for (int par = 0; blk < nb; blk += gridDim.x, par ^= 1) {
    const long long i0 = blk * OPT_BLOCK + (long long)threadIdx.x * OPT_NPT;
    float gv[8], pv[8], s1[8], gl[8];
    uint32_t c1[8], c2[8];
    in.unpack(gv, pv, c1, c2);
    const float am1 = in.am1;
    if (blk + gridDim.x < nb) in.load(g, p, state1, nullptr, absmax1, nullptr, blk + gridDim.x, n);
    float m1 = -FLT_MAX, m2 = 0.0f;
    bool upd[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float gs = __fmul_rn(gv[j], k.gnorm_scale);
      upd[j] = !k.skip_zeros || gv[j] != 0.0f;
      s1[j] = __fmul_rn(code1[c1[j]], am1);        // skipped elements keep their dequantised state
      gl[j] = gv[j];
      if (upd[j]) {
        if (k.weight_decay > 0.0f) {
          if (OPT == LION) pv[j] = Io<T>::to_f32(Io<T>::from_f32(__fmul_rn(pv[j], k.decay)));
          else gs = __fadd_rn(gs, __fmul_rn(pv[j], k.weight_decay));
        }
        if (OPT == MOMENTUM) {
          s1[j] = (k.step == 1) ? gs : __fadd_rn(__fmul_rn(s1[j], k.beta1), gs);
        } else if (OPT == LION) {
          // the smoothed sign is kept in T, as the reference stores it in g_vals (kernel_quant.cpp:3095)
          gl[j] = Io<T>::to_f32(Io<T>::from_f32(
              __fmul_rn(k.lr, sgnf(__fadd_rn(__fmul_rn(s1[j], k.beta1), __fmul_rn(__fsub_rn(1.0f, k.beta1), gs))))));
          s1[j] = __fadd_rn(__fmul_rn(s1[j], k.beta2), __fmul_rn(__fsub_rn(1.0f, k.beta2), gs));
        } else if (OPT == RMSPROP) {
          s1[j] = __fadd_rn(__fmul_rn(s1[j], k.beta1), __fmul_rn(__fsub_rn(1.0f, k.beta1), __fmul_rn(gs, gs)));
        } else {   // ADAGRAD
          s1[j] = __fadd_rn(s1[j], __fmul_rn(gs, gs));
        }
      }
      m1 = fmaxf(m1, fabsf(s1[j]));
    }
    block_max256x2(m1, m2, L.xch[par]);
    if (threadIdx.x == 0) absmax1[blk] = m1;
    T po[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float pn = pv[j];
      if (upd[j]) {
        if (OPT == MOMENTUM) pn = __fsub_rn(pv[j], __fmul_rn(k.lr, s1[j]));
        else if (OPT == LION) pn = __fsub_rn(pv[j], gl[j]);
        else pn = __fsub_rn(pv[j], __fmul_rn(k.lr, __fdiv_rn(gl[j], __fadd_rn(__builtin_sqrtf(s1[j]), k.eps))));
      }
      po[j] = Io<T>::from_f32(pn);
    }
    store8(p, i0, n, po);
    requant8<true>(code1, s1, m1, c1);
    store8u(state1, i0, n, c1);
  }
}

// ---------------------------------------------------------------- 32-bit states
// kOptimizer32bit2State / 1State with max_unorm == 0 (update_scale == 1); gradients are rounded to
// T after scaling (and after weight decay for one state), as the reference keeps them in g_vals.
template <typename T, int OPT>
__global__ void __launch_bounds__(OPT_THREADS)
k_optimizer_32bit(T* __restrict__ p, const T* __restrict__ g, float* __restrict__ state1, float* __restrict__ state2,
                  OptScalars k, int n) {
  const long long i0 = ((long long)blockIdx.x * OPT_THREADS + threadIdx.x) * OPT_NPT;
  if (i0 >= n) return;
  float gv[8], pv[8], s1[8], s2[8];
  load8(g, i0, n, gv, 0.0f);
  load8(p, i0, n, pv, 0.0f);
  load8(state1, i0, n, s1, 0.0f);
  if (OPT == ADAM) load8(state2, i0, n, s2, 0.0f);
  T po[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float gt = Io<T>::to_f32(Io<T>::from_f32(__fmul_rn(k.gnorm_scale, gv[j])));
    if (OPT != ADAM && k.weight_decay > 0.0f) gt = Io<T>::to_f32(Io<T>::from_f32(__fadd_rn(gt, __fmul_rn(pv[j], k.weight_decay))));
    float pn = pv[j];
    if (!k.skip_zeros || gt != 0.0f) {
      if (OPT == ADAM) {
        s1[j] = __fadd_rn(__fmul_rn(s1[j], k.beta1), __fmul_rn(__fsub_rn(1.0f, k.beta1), gt));
        s2[j] = __fadd_rn(__fmul_rn(s2[j], k.beta2), __fmul_rn(__fsub_rn(1.0f, k.beta2), __fmul_rn(gt, gt)));
        pn = Io<T>::to_f32(Io<T>::from_f32(
            __fadd_rn(pv[j], __fmul_rn(k.step_size, __fdiv_rn(s1[j], __fadd_rn(__builtin_sqrtf(s2[j]), k.c2eps))))));
        if (k.weight_decay > 0.0f) pn = __fmul_rn(pn, k.decay);
      } else if (OPT == MOMENTUM) {
        s1[j] = (k.step == 1) ? gt : __fadd_rn(__fmul_rn(s1[j], k.beta1), gt);
        pn = __fadd_rn(pv[j], -__fmul_rn(k.lr, s1[j]));
      } else if (OPT == LION) {
        pn = __fsub_rn(pv[j], __fmul_rn(k.lr, sgnf(__fadd_rn(__fmul_rn(s1[j], k.beta1), __fmul_rn(__fsub_rn(1.0f, k.beta1), gt)))));
        s1[j] = __fadd_rn(__fmul_rn(s1[j], k.beta2), __fmul_rn(__fsub_rn(1.0f, k.beta2), gt));
      } else if (OPT == RMSPROP) {
        s1[j] = __fadd_rn(__fmul_rn(s1[j], k.beta1), __fmul_rn(__fmul_rn(__fsub_rn(1.0f, k.beta1), gt), gt));
        pn = __fsub_rn(pv[j], __fdiv_rn(__fmul_rn(k.lr, gt), __fadd_rn(__builtin_sqrtf(s1[j]), k.eps)));
      } else {   // ADAGRAD
        s1[j] = __fadd_rn(s1[j], __fmul_rn(gt, gt));
        pn = __fsub_rn(pv[j], __fdiv_rn(__fmul_rn(k.lr, gt), __fadd_rn(__builtin_sqrtf(s1[j]), k.eps)));
      }
    }
    po[j] = Io<T>::from_f32(pn);
  }
  store8(p, i0, n, po);
  store8(state1, i0, n, s1);
  if (OPT == ADAM) store8(state2, i0, n, s2);
}

// ---------------------------------------------------------------- host side
static OptScalars make_scalars(float beta1, float beta2, float eps, int step, float lr, float weight_decay,
                               float gnorm_scale, bool skip_zeros) {
  OptScalars k{};
  k.beta1 = beta1; k.beta2 = beta2; k.eps = eps; k.lr = lr; k.weight_decay = weight_decay;
  k.gnorm_scale = gnorm_scale; k.step = step; k.skip_zeros = skip_zeros;
  // pow(float, int) in the reference promotes to double (kernel_quant.cpp:2740-2741)
  const float correction1 = (float)(1.0 - std::pow((double)beta1, (double)step));
  const float correction2 = (float)std::sqrt(1.0 - std::pow((double)beta2, (double)step));
  const float neg_lr_c2 = -lr * correction2;     // fp32, as the kernel's (-lr*correction2) / correction1
  k.step_size = neg_lr_c2 / correction1;
  k.c2eps = correction2 * eps;
  const float lr_wd = lr * weight_decay;
  k.decay = 1.0f - lr_wd;
  return k;
}

// grid of the pipelined 8-bit kernels: every workgroup resident at once (CUs x occupancy, queried once
// per kernel and device), each walking its blocks with the next one's loads in flight
template <class K>
static unsigned resident_grid(K kernel, long long nb) {
  static int cached[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  int& slots = cached[dev & 63];
  if (slots == 0) {
    int cus = 0, per_cu = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, OPT_THREADS, 0);
    slots = 4 * std::max(cus, 1) * std::max(per_cu, 1);   // 4 waves of workgroups: even tails (lab: 722 vs 752 us at 1x)
  }
  return (unsigned)std::min<long long>(nb, slots);
}

template <typename T, int OPT>
void optimizer_8bit_blockwise(T* p, T* g, uint8_t* state1, uint8_t* state2, float beta1, float beta2, float eps, int step,
                              float lr, float* qmap1, float* qmap2, float* absmax1, float* absmax2, float weight_decay,
                              float gnorm_scale, bool skip_zeros, int n) {
  if (n <= 0) return;
  const OptScalars k = make_scalars(beta1, beta2, eps, step, lr, weight_decay, gnorm_scale, skip_zeros);
  const long long nb = (n + OPT_BLOCK - 1) / OPT_BLOCK;
  if constexpr (OPT == ADAM) {
    const auto kern = k_optimizer_8bit_blockwise_2state<T, OPT>;
    hipLaunchKernelGGL(kern, dim3(resident_grid(kern, nb)), dim3(OPT_THREADS), 0, current_stream(), p, g, state1,
                       state2, qmap1, qmap2, absmax1, absmax2, k, n);
  } else {
    const auto kern = k_optimizer_8bit_blockwise_1state<T, OPT>;
    hipLaunchKernelGGL(kern, dim3(resident_grid(kern, nb)), dim3(OPT_THREADS), 0, current_stream(), p, g, state1,
                       qmap1, absmax1, k, n);
  }
  BNB_LAUNCH_CHECK("optimizer_8bit_blockwise");
}

template <typename T, int OPT>
void optimizer_32bit(T* g, T* p, float* state1, float* state2, float* unorm, float max_unorm, float param_norm,
                     float beta1, float beta2, float eps, float weight_decay, int step, float lr, float gnorm_scale,
                     bool skip_zeros, int n) {
  (void)unorm; (void)param_norm;
  if (n <= 0) return;
  if (max_unorm > 0.0f) {
    set_error(1, "optimizer32bit: max_unorm > 0 (update-norm clipping) is not supported by this build");
    return;
  }
  const OptScalars k = make_scalars(beta1, beta2, eps, step, lr, weight_decay, gnorm_scale, skip_zeros);
  const unsigned blocks = (unsigned)((n + OPT_THREADS * OPT_NPT - 1) / (OPT_THREADS * OPT_NPT));
  hipLaunchKernelGGL((k_optimizer_32bit<T, OPT>), dim3(blocks), dim3(OPT_THREADS), 0, current_stream(), p, g, state1,
                     state2, k, n);
  BNB_LAUNCH_CHECK("optimizer_32bit");
}

}  // namespace bnb

using namespace bnb;

extern "C" {

#define BNB_BLOCKWISE8(fname, OPT, gtype, gbits)                                                                   \
  void c##fname##_8bit_blockwise_grad_##gbits(gtype* p, gtype* g, unsigned char* state1, unsigned char* state2,    \
                                              float beta1, float beta2, float eps, int step, float lr,             \
                                              float* quantiles1, float* quantiles2, float* absmax1, float* absmax2, \
                                              float weight_decay, const float gnorm_scale, bool skip_zeros, int n) { \
    BNB_RANGE("c" #fname "_8bit_blockwise_grad_" #gbits);                                                         \
    optimizer_8bit_blockwise<gtype, OPT>(p, g, state1, state2, beta1, beta2, eps, step, lr, quantiles1, quantiles2, \
                                         absmax1, absmax2, weight_decay, gnorm_scale, skip_zeros, n);              \
  }
// ref:sycl/pythonInterface.cpp:271-284 (+ the dtypes it leaves out, additive)
BNB_BLOCKWISE8(adam, ADAM, float, fp32)
BNB_BLOCKWISE8(adam, ADAM, fp16_t, fp16)
BNB_BLOCKWISE8(adam, ADAM, bf16_t, bf16)
BNB_BLOCKWISE8(momentum, MOMENTUM, float, fp32)
BNB_BLOCKWISE8(momentum, MOMENTUM, fp16_t, fp16)
BNB_BLOCKWISE8(momentum, MOMENTUM, bf16_t, bf16)
BNB_BLOCKWISE8(rmsprop, RMSPROP, float, fp32)
BNB_BLOCKWISE8(rmsprop, RMSPROP, fp16_t, fp16)
BNB_BLOCKWISE8(rmsprop, RMSPROP, bf16_t, bf16)
BNB_BLOCKWISE8(adagrad, ADAGRAD, float, fp32)
BNB_BLOCKWISE8(adagrad, ADAGRAD, fp16_t, fp16)
BNB_BLOCKWISE8(adagrad, ADAGRAD, bf16_t, bf16)
BNB_BLOCKWISE8(lion, LION, float, fp32)
BNB_BLOCKWISE8(lion, LION, fp16_t, fp16)
BNB_BLOCKWISE8(lion, LION, bf16_t, bf16)

#define BNB_FUNC32(fname, OPT, gtype, gbits)                                                                    \
  void c##fname##32bit_grad_##gbits(gtype* g, gtype* p, float* state1, float* state2, float* unorm,             \
                                    float max_unorm, float param_norm, const float beta1, const float beta2,    \
                                    const float eps, const float weight_decay, const int step, const float lr,  \
                                    const float gnorm_scale, bool skip_zeros, const int n) {                    \
    BNB_RANGE("c" #fname "32bit_grad_" #gbits);                                                              \
    optimizer_32bit<gtype, OPT>(g, p, state1, state2, unorm, max_unorm, param_norm, beta1, beta2, eps,          \
                                weight_decay, step, lr, gnorm_scale, skip_zeros, n);                            \
  }
// ref:sycl/pythonInterface.cpp:230-241 (names as the reference spells them) + bf16 siblings (additive)
BNB_FUNC32(adam, ADAM, float, fp32)
BNB_FUNC32(adam, ADAM, fp16_t, fp16)
BNB_FUNC32(adam, ADAM, bf16_t, bf16)
BNB_FUNC32(momentum, MOMENTUM, float, 32)
BNB_FUNC32(momentum, MOMENTUM, fp16_t, 16)
BNB_FUNC32(momentum, MOMENTUM, bf16_t, bf16)
BNB_FUNC32(rmsprop, RMSPROP, float, 32)
BNB_FUNC32(rmsprop, RMSPROP, fp16_t, 16)
BNB_FUNC32(rmsprop, RMSPROP, bf16_t, bf16)
BNB_FUNC32(lion, LION, float, fp32)
BNB_FUNC32(lion, LION, fp16_t, fp16)
BNB_FUNC32(lion, LION, bf16_t, bf16)
BNB_FUNC32(adagrad, ADAGRAD, float, 32)
BNB_FUNC32(adagrad, ADAGRAD, fp16_t, 16)
BNB_FUNC32(adagrad, ADAGRAD, bf16_t, bf16)

}  // extern "C"
