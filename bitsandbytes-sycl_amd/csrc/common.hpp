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
#include <atomic>
#include <stdint.h>
#include <stdio.h>

typedef uint16_t bf16_t;   // bfloat16 bit pattern
typedef _Float16 fp16_t;   // IEEE binary16

namespace bnb {

// A process-global A/B or testing knob of the C-ABI setters (c*_set_*): an atomic, so a setter on one host thread and a
// launch on another never race; a launch reads each knob once when it plans.  Knobs are per process, not per device.
template <typename T> using Knob = std::atomic<T>;

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

// dQuantize<0>: binary search + midpoint rounding over a 256-entry code held in LDS.  Code is a
// plain pointer or a view with operator[] (e.g. DynMapView below).
template <class Code>
__device__ __forceinline__ uint32_t quantize_dynamic8(Code code, float x) {
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

// quantize_dynamic8 for N independent values, branch-free and level-synchronous: the N searches issue
// their LDS reads of one level together (one lgkmcnt wait per level, not one per read; the scalar
// form compiles to exec-masked branches with a full wait after every read).  Identical results: after
// the last step (+-1) on the even pivot p the bracketing pivots are p + 1 and max(p - 1, 0), so the
// midpoint pick reads code[p - 1], code[p], code[p + 1] once at the end and the search itself carries
// only the pivot.  The first step's pivots (127, then 63 / 191) come from registers.
// q[j] = code index; cq[j] = code[q[j]] (callers keep the sign of the value with it).
template <int N, class Code>
__device__ __forceinline__ void quantize_dynamic8_n(Code code, const float (&x)[N], uint32_t (&q)[N], float (&cq)[N]) {
  const float c127 = code[127], c63 = code[63], c191 = code[191];
  int pv[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const bool gt0 = x[j] > c127;
    const bool gt1 = x[j] > (gt0 ? c191 : c63);
    pv[j] = (gt0 ? 191 : 63) + (gt1 ? 32 : -32);
  }
#pragma unroll
  for (int i = 16; i > 0; i >>= 1) {
    float val[N];
#pragma unroll
    for (int j = 0; j < N; ++j) val[j] = code[pv[j]];
#pragma unroll
    for (int j = 0; j < N; ++j) pv[j] += x[j] > val[j] ? i : -i;
  }
  float lo[N], mid[N], hi[N];
#pragma unroll
  for (int j = 0; j < N; ++j) { lo[j] = code[max(pv[j] - 1, 0)]; mid[j] = code[pv[j]]; hi[j] = code[pv[j] + 1]; }
#pragma unroll
  for (int j = 0; j < N; ++j) {                 // branch-free pick between p and its neighbour on x's side
    const bool above = x[j] > mid[j];
    const float nb = above ? hi[j] : lo[j];
    const float m = __fmul_rn(__fadd_rn(nb, mid[j]), 0.5f);
    const bool move = above ? (x[j] > m) : (x[j] < m);
    q[j] = move ? (uint32_t)(above ? pv[j] + 1 : max(pv[j] - 1, 0)) : (uint32_t)pv[j];
    cq[j] = move ? nb : mid[j];
  }
}

// A 256-entry dynamic map laid out in LDS for the branch-free dQuantize<0> search (quantize_dynamic8
// semantics for any sorted map: the same pivots and comparisons in the same order, stored differently).
// 1024 floats (4 KiB), byte offsets:
//      0  tree[i], i = 1..127: the search pivots in breadth-first (Eytzinger) order, tree[1] = code[127],
//         children of node i at 2i and 2i + 1.  A level is a = 2a + (x > v ? 4 : 0) on the byte offset
//         a = 4i (v_cmp, v_cndmask, v_lshl_or); one level's nodes are contiguous, so levels of <= 32
//         nodes never bank-conflict.  After 7 levels a = 4 (128 + L) and the even pivot is p = 2L.
//    512  code[2L]                             at byte a    (the final pick's records share the offset
//   1024  code[max(2L - 1, 0)]                 at a + 512    a of the search: immediate ds_read
//   1536  code[2L + 1]                         at a + 1024   offsets, no address arithmetic)
//   2048  (code[2L-1] + code[2L]) * 0.5        at a + 1536   the two midpoints of quantize_dynamic8,
//   2560  (code[2L+1] + code[2L]) * 0.5        at a + 2048   rounded as it rounds them (-inf at L = 0)
//   3072  code[c], c = 0..255                  (dequantisation)
constexpr int DYNMAP_FLOATS = 1024;

struct DynMapView {
  const char* base;
  __device__ __forceinline__ float at(int byte_off) const { return *reinterpret_cast<const float*>(base + byte_off); }
  __device__ __forceinline__ float operator[](uint32_t c) const { return at(3072 + 4 * (int)c); }
};

// build the layout from a 256-entry global map (256 threads, 4 entries each; consecutive lanes write
// consecutive dwords)
__device__ __forceinline__ void dynmap_stage(float* table, const float* __restrict__ code) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int f = it * 256 + threadIdx.x, part = f >> 7, L = f & 127;
    float v;
    if (part == 0) {                             // tree node L (slot 0 unused)
      const int i = max(L, 1), d = 31 - __builtin_clz(i);
      v = code[((2 * (i - (1 << d)) + 1) << (7 - d)) - 1];
    } else if (part == 1) {
      v = code[2 * L];
    } else if (part == 2) {
      v = code[max(2 * L - 1, 0)];
    } else if (part == 3) {
      v = code[2 * L + 1];
    } else if (part == 4) {   // -inf for p = 0: nothing lies below code[0]'s pick (q would clamp to 0)
      v = L == 0 ? -__builtin_inff() : __fmul_rn(__fadd_rn(code[2 * L - 1], code[2 * L]), 0.5f);
    } else if (part == 5) {
      v = __fmul_rn(__fadd_rn(code[2 * L + 1], code[2 * L]), 0.5f);
    } else {
      v = code[f - 768];
    }
    table[f] = v;
  }
}

// dQuantize<0> of N independent values, level-synchronous: q[j] = code index; with CQ, cq[j] = code[q[j]]
template <int N, bool CQ>
__device__ __forceinline__ void dynmap_quantize_n(DynMapView m, const float (&x)[N], uint32_t (&q)[N],
                                                  float (&cq)[N]) {
  const float root = m.at(4);
  int a[N];
#pragma unroll
  for (int j = 0; j < N; ++j) a[j] = x[j] > root ? 12 : 8;
#pragma unroll
  for (int d = 1; d < 7; ++d) {
    float v[N];
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] = m.at(a[j]);
#pragma unroll
    for (int j = 0; j < N; ++j) a[j] = 2 * a[j] + (x[j] > v[j] ? 4 : 0);
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    // quantize_dynamic8's tail, branch-free: with mlo <= code[p] <= mhi (midpoints of a sorted map),
    // "x > code[p] ? (x > mhi ? p+1 : p) : (x < mlo ? p-1 : p)" is p + (x > mhi) - (x < mlo)
    const float mlo = m.at(a[j] + 1536), mhi = m.at(a[j] + 2048);
    const bool up = x[j] > mhi, dn = x[j] < mlo;
    const int p = (a[j] - 512) >> 1;
    q[j] = (uint32_t)(p + (up ? 1 : 0) - (dn ? 1 : 0));
    if constexpr (CQ) cq[j] = up ? m.at(a[j] + 1024) : (dn ? m.at(a[j] + 512) : m.at(a[j]));
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

// roctx ranges around the C-ABI entry points (SURVEY §5's tracing plan: the only tracing hook a user of the drop-in
// library gets).  Off unless BNB_ROCTX=1 is set when the library first checks: then libroctx64 is opened once
// (dlopen, no link-time dependency) and every entry point pushes a range named after itself for the duration of the
// call (host side: the launch, not the kernel; rocprofv3 --marker-trace records them).  Off, a range costs one load and
// one branch.
struct BnbRange {
  bool on;
  explicit BnbRange(const char* name);
  ~BnbRange();
};
#define BNB_RANGE(name) ::bnb::BnbRange bnb_range_guard_(name)

}  // namespace bnb
