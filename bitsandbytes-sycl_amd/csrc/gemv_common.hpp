// Shared pieces of the 4-bit GEMV kernels (gemv4bit.hip: one activation row; gemv4bit_tok.hip: 2..8 rows).
#pragma once

#include "common.hpp"

namespace bnb {

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

int device_cu_count();   // CUs of the current device (cached; gemv4bit.hip)

}  // namespace bnb
