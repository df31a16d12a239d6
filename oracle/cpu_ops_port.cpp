// CPU baseline port — TEST / BENCH INFRASTRUCTURE ONLY (see oracle/__init__.py).
//
// A fresh C++ restatement of the reference's CPU path for blockwise 8-bit-code
// quantisation, used as bench.py's `cpu_baseline` (kind "port") and as a
// second CPU check in tests.  It keeps the reference's execution structure:
//   * dequantize: ONE thread, out[i] = code[A[i]] * absmax[i / blocksize]
//     (ref:sycl/cpu_ops.cpp:7-14);
//   * quantize: one std::thread per block, launched in waves of 256
//     (ref:sycl/cpu_ops.cpp:16-63); per block: absmax = fmax over |A| seeded
//     with -FLT_MAX, z = A / absmax (division, not reciprocal), left neighbour
//     by binary search, move right iff strictly closer (ref:sycl/common.cpp:4-35);
//     code[0] is forced to -1.0f in place (ref:sycl/cpu_ops.cpp:20).
// The reference's own BinSearch/Direct2 SIMD helper (ref:sycl/include/*) is
// replaced by std::upper_bound, which returns the same left neighbour for the
// sorted 256-entry codes used here.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

namespace {

struct BlockJob {
  const float* code;
  const float* A;
  float* absmax;
  uint8_t* out;
  long long begin, end, blocksize;
};

void quantize_one_block(const BlockJob& j) {
  float amax = -FLT_MAX;
  for (long long i = j.begin; i < j.end; ++i) amax = std::fmax(amax, std::fabs(j.A[i]));
  j.absmax[j.begin / j.blocksize] = amax;
  for (long long i = j.begin; i < j.end; ++i) {
    const float z = j.A[i] / amax;
    long long idx = (long long)(std::upper_bound(j.code, j.code + 256, z) - j.code) - 1;
    if (idx < 0) idx = 0;
    if (std::isnan(z)) idx = 0;
    if (idx < 255) {
      const float dl = std::fabs(z - j.code[idx]);
      const float dr = std::fabs(z - j.code[idx + 1]);
      if (dr < dl) idx += 1;
    }
    j.out[i] = (uint8_t)idx;
  }
}

}  // namespace

extern "C" {

void port_dequantize_cpu(const float* code, const uint8_t* A, const float* absmax, float* out,
                         long long blocksize, long long n) {
  for (long long b = 0; b < n; b += blocksize) {
    const long long e = std::min(n, b + blocksize);
    const float s = absmax[b / blocksize];
    for (long long i = b; i < e; ++i) out[i] = code[A[i]] * s;
  }
}

void port_quantize_cpu(float* code, const float* A, float* absmax, uint8_t* out, long long blocksize,
                       long long n) {
  code[0] = -1.0f;
  const long long nblocks = (n + blocksize - 1) / blocksize;
  const long long wave = 256;
  for (long long first = 0; first < nblocks; first += wave) {
    const long long cnt = std::min(wave, nblocks - first);
    std::vector<std::thread> threads;
    threads.reserve(cnt);
    for (long long t = 0; t < cnt; ++t) {
      const long long b = (first + t) * blocksize;
      BlockJob job{code, A, absmax, out, b, std::min(n, b + blocksize), blocksize};
      threads.emplace_back([job] { quantize_one_block(job); });
    }
    for (auto& th : threads) th.join();
  }
}

}  // extern "C"
