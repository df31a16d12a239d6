// Shared device helpers for the gfx950 (MI355X / CDNA4) quantized-matmul backend.
//
// Codec constants follow the reference decision trees exactly (float literals,
// strict '>' comparisons):
//   NF4  quantise  ref:sycl/sycl_code/kernel_quant.cpp:705-756
//   NF4  values    ref:sycl/sycl_code/kernel_quant.cpp:650-703
//   FP4  quantise  ref:sycl/sycl_code/kernel_quant.cpp:547-594
//   FP4  values    ref:sycl/sycl_code/kernel_quant.cpp:520-545
//   8-bit dynamic  ref:sycl/sycl_code/kernel_quant.cpp:765-819 (dQuantize<0>)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint16_t bf16_t;   // bfloat16 bit pattern
typedef _Float16 fp16_t;   // IEEE binary16

namespace bnb {

enum DataType { GENERAL8BIT = 0, FP4 = 1, NF4 = 2 };

// ---------------------------------------------------------------- runtime state
hipStream_t current_stream();
void set_error(int code, const char* what);
#define BNB_LAUNCH_CHECK(name)                                              \
  do {                                                                      \
    hipError_t e_ = hipGetLastError();                                      \
    if (e_ != hipSuccess) ::bnb::set_error((int)e_, name);                  \
  } while (0)

// ---------------------------------------------------------------- dtype traits
template <typename T> struct Io;
template <> struct Io<float> {
  __device__ static __forceinline__ float to_f32(float v) { return v; }
  __device__ static __forceinline__ float from_f32(float v) { return v; }
};
// Opaque register barrier: stops the gfx950 backend from folding a preceding fmul/fadd into a
// v_fma_mix*_f16 with the f32->f16 conversion.  That fold (fmul -> fma(x, y, +0)) turns a -0.0
// product into +0.0 and fuses mul+add even under -ffp-contract=off; the reference rounds the fp32
// result once, so every f32 -> f16 conversion of a computed value goes through this barrier.
__device__ __forceinline__ float opaque(float v) {
  asm volatile("" : "+v"(v));
  return v;
}

template <> struct Io<fp16_t> {
  __device__ static __forceinline__ float to_f32(fp16_t v) { return (float)v; }
  __device__ static __forceinline__ fp16_t from_f32(float v) { return (fp16_t)opaque(v); }
};
template <> struct Io<bf16_t> {
  __device__ static __forceinline__ float to_f32(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
  // one round-to-nearest-even cast; hipcc lowers this to v_cvt_pk_bf16_f32 on gfx950
  __device__ static __forceinline__ bf16_t from_f32(float v) { return __builtin_bit_cast(bf16_t, (__bf16)v); }
};

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)Io<bf16_t>::from_f32(lo) | ((uint32_t)Io<bf16_t>::from_f32(hi) << 16);
}

// ---------------------------------------------------------------- codecs
// NF4 values, ref:kernel_quant.cpp:650-703 (table form of the same tree)
static __constant__ float kNF4Values[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
    -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
    0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f, 0.33791524171829224f,
    0.44070982933044434f, 0.5626170039176941f, 0.7229568362236023f, 1.0f};
// FP4 magnitudes by low 3 bits, ref:kernel_quant.cpp:520-545
static __constant__ float kFP4Mag[8] = {0.00000000f, 5.208333333e-03f, 0.66666667f, 1.00000000f,
                                        0.33333333f, 0.50000000f, 0.16666667f, 0.25000000f};

__device__ __forceinline__ float nf4_value(uint32_t q) { return kNF4Values[q & 15]; }

__device__ __forceinline__ uint32_t quantize_nf4(float x) {
  // count of thresholds strictly exceeded == the reference's balanced tree (NaN -> 0)
  uint32_t q = 0;
  q += x > -0.8480964004993439f;
  q += x > -0.6106329262256622f;
  q += x > -0.4599952697753906f;
  q += x > -0.33967943489551544f;
  q += x > -0.23460740596055984f;
  q += x > -0.13791173323988914f;
  q += x > -0.045525018125772476f;
  q += x > 0.03979014977812767f;
  q += x > 0.1202552504837513f;
  q += x > 0.2035212516784668f;
  q += x > 0.2920137718319893f;
  q += x > 0.3893125355243683f;
  q += x > 0.5016634166240692f;
  q += x > 0.6427869200706482f;
  q += x > 0.8614784181118011f;
  return q;
}

__device__ __forceinline__ uint32_t quantize_fp4(float x) {
  const uint32_t sign = x < 0.0f ? 8u : 0u;
  const float a = fabsf(x);
  uint32_t c = 0;
  c += a > 0.00260417f;
  c += a > 0.0859375f;
  c += a > 0.20833333f;
  c += a > 0.29166667f;
  c += a > 0.4166667f;
  c += a > 0.583333f;
  c += a > 0.8333333f;
  // count -> code: 0,1,6,7,4,5,2,3  (packed 4 bits per entry)
  const uint32_t code = (0x32547610u >> (4 * c)) & 7u;
  return code | sign;
}

__device__ __forceinline__ float fp4_magnitude(uint32_t q) { return kFP4Mag[q & 7]; }

// signed 4-bit code value (table entry) such that value*absmax == the reference's
// dequantised value bit-exactly: NF4 v*absmax; FP4 (m*absmax)*sign == (sign*m)*absmax.
template <int DT> __device__ __forceinline__ float code4_value(uint32_t q) {
  if constexpr (DT == NF4) return nf4_value(q);
  else return (q & 8) ? -fp4_magnitude(q) : fp4_magnitude(q);
}

// value * absmax in fp32 for the 4-bit codes (one rounding), sign applied after (exact)
template <int DT> __device__ __forceinline__ float dequant4(uint32_t q, float absmax) {
  if constexpr (DT == NF4) {
    return nf4_value(q) * absmax;
  } else {
    const float v = fp4_magnitude(q) * absmax;
    return (q & 8) ? -v : v;
  }
}

template <int DT> __device__ __forceinline__ uint32_t quant4(float x) {
  if constexpr (DT == NF4) return quantize_nf4(x);
  else return quantize_fp4(x);
}

// dQuantize<0>: binary search + midpoint rounding over a 256-entry code held in LDS
__device__ __forceinline__ uint32_t quantize_dynamic8(const float* __restrict__ code, float x) {
  int pivot = 127, upper_pivot = 255, lower_pivot = 0;
  float lower = -1.0f, upper = 1.0f;
  float val = code[pivot];
#pragma unroll
  for (int i = 64; i > 0; i >>= 1) {
    if (x > val) {
      lower_pivot = pivot;
      lower = val;
      pivot += i;
    } else {
      upper_pivot = pivot;
      upper = val;
      pivot -= i;
    }
    val = code[pivot];
  }
  if (upper_pivot == 255) upper = code[upper_pivot];
  if (lower_pivot == 0) lower = code[lower_pivot];
  if (x > val) {
    const float mid = __fmul_rn(__fadd_rn(upper, val), 0.5f);
    return x > mid ? upper_pivot : pivot;
  } else {
    const float mid = __fmul_rn(__fadd_rn(lower, val), 0.5f);
    return x < mid ? lower_pivot : pivot;
  }
}

// ---------------------------------------------------------------- memory helpers
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
// 16-B non-temporal load (streamed-once data, e.g. packed weights of a decode GEMV)
__device__ __forceinline__ uint4 ld_nt16(const void* p) {
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// ---------------------------------------------------------------- wave helpers (wave64)
__device__ __forceinline__ float wave_max_xor(float v, int width) {
  for (int o = 1; o < width; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace bnb
