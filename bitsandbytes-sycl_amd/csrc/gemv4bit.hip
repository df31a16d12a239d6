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

template <typename T>
void gemv_4bit(int m, int n, int k, const T* A, const uint8_t* B, const float* absmax, const float* datatype, T* out,
               int lda, int ldb, int ldc, int blocksize) {
  (void)n; (void)lda; (void)ldc;
  if (m <= 0) return;
  if (k <= 0 || blocksize <= 0) { set_error(1, "gemv_4bit: bad k/blocksize"); return; }
  const bool fast = (k % 32 == 0) && (ldb % 16 == 0) && (((uintptr_t)A & 15) == 0) && (((uintptr_t)B & 15) == 0) &&
                    (blocksize % 32 == 0);
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

}  // extern "C"
