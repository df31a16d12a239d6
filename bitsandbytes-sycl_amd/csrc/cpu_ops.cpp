// Host (CPU) path of the blockwise 8-bit-code quantizer: the reference's cpu_ops.cpp entry points
// (ref:sycl/pythonInterface.cpp:419-420 -> ref:sycl/cpu_ops.cpp:7-63, ref:sycl/common.cpp:4-35).
//
// These run on the host cores with host pointers and never touch HIP, so they work on a machine
// without a GPU (config 1 of BASELINE.json).  Semantics are the reference's:
//   quantize   code[0] := -1.0f in place (cpu_ops.cpp:20); per block absmax = fmax over |A| seeded with
//              -FLT_MAX (common.cpp:12-14); z = A / absmax (a division, common.cpp:21 -- the GPU kernels
//              multiply by the reciprocal instead); the left neighbour of z in the sorted 256-entry code
//              (BinAlgo<Direct2>::scalar, include/Algo-Direct2.h:21-33), then one step right iff that
//              neighbour is strictly closer (common.cpp:26-30); NaN -> index 0.
//   dequantize out[i] = code[A[i]] * absmax[i / blocksize] (cpu_ops.cpp:7-14), one byte per element.
// Execution differs (results do not): instead of one OS thread per block in waves of 256
// (cpu_ops.cpp:31-61; 262,144 thread creations at config 1) and a single-threaded dequantize, blocks are
// split into contiguous ranges over a bounded number of worker threads (cset_cpu_threads, else BNB_CPU_THREADS,
// else OMP_NUM_THREADS, else the hardware threads, at most 64).  Every element's value depends only on
// its own block, so the split cannot change a result.
#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <thread>
#include <vector>

namespace {

std::atomic<int> g_cpu_threads{0};

int cpu_threads() {
  int t = g_cpu_threads.load();
  if (t > 0) return t;
  for (const char* var : {"BNB_CPU_THREADS", "OMP_NUM_THREADS"}) {   // the job's CPU share, when the host says
    if (const char* e = std::getenv(var)) {
      t = std::atoi(e);
      if (t > 0) return t;
    }
  }
  t = (int)std::thread::hardware_concurrency();
  if (t <= 0) t = 1;
  return t > 64 ? 64 : t;
}

// fn(first_block, end_block) over [0, nblocks) split into contiguous ranges; small jobs stay inline.
template <typename Fn>
void parallel_blocks(long long nblocks, long long elems_per_block, Fn fn) {
  int threads = cpu_threads();
  const long long min_elems_per_thread = 1 << 16;
  const long long total = nblocks * elems_per_block;
  long long cap = total / min_elems_per_thread;
  if (cap < 1) cap = 1;
  if (threads > cap) threads = (int)cap;
  if (threads > nblocks) threads = (int)nblocks;
  if (threads <= 1) {
    fn(0LL, nblocks);
    return;
  }
  std::vector<std::thread> pool;
  pool.reserve(threads - 1);
  const long long per = nblocks / threads, rem = nblocks % threads;
  long long b = 0;
  long long first_end = 0;
  for (int t = 0; t < threads; ++t) {
    const long long e = b + per + (t < rem ? 1 : 0);
    if (t == 0) {
      first_end = e;
    } else {
      pool.emplace_back([=] { fn(b, e); });
    }
    b = e;
  }
  fn(0LL, first_end);
  for (auto& th : pool) th.join();
}

// Largest i with code[i] <= z (the left neighbour); 0 when z < code[0] or z is NaN.  `code` is sorted
// ascending with 256 entries; `code[j] <= z` is true then false along j, and 8 halving steps find the
// last true (indices reached: 128, then i + 64, ..., at most 255).  NaN compares false everywhere -> 0.
inline int left_neighbour(const float* code, float z) {
  int i = 0;
  for (int half = 128; half >= 1; half >>= 1)
    if (code[i + half] <= z) i += half;
  return i;
}

void quantize_range(const float* code, const float* A, float* absmax, uint8_t* out, long long blocksize, long long n,
                    long long b0, long long b1) {
  for (long long blk = b0; blk < b1; ++blk) {
    const long long s = blk * blocksize;
    const long long e = std::min(n, s + blocksize);
    float amax = -FLT_MAX;
    for (long long i = s; i < e; ++i) amax = std::fmax(amax, std::fabs(A[i]));
    absmax[blk] = amax;
    for (long long i = s; i < e; ++i) {
      const float z = A[i] / amax;
      int idx = left_neighbour(code, z);
      if (idx < 255) {
        const float dl = std::fabs(z - code[idx]);
        const float dr = std::fabs(z - code[idx + 1]);
        if (dr < dl) idx += 1;
      }
      out[i] = (uint8_t)idx;
    }
  }
}

}  // namespace

extern "C" {

// ref:sycl/pythonInterface.cpp:419 -> quantize_cpu (cpu_ops.cpp:16-63).  Host pointers.
void cquantize_blockwise_cpu_fp32(float* code, float* A, float* absmax, unsigned char* out, long long blocksize,
                                  long long n) {
  if (n <= 0 || blocksize <= 0) return;
  code[0] = -1.0f;   // in-place side effect of the reference (cpu_ops.cpp:20)
  const long long nblocks = (n + blocksize - 1) / blocksize;
  parallel_blocks(nblocks, blocksize, [&](long long b0, long long b1) {
    quantize_range(code, A, absmax, out, blocksize, n, b0, b1);
  });
}

// ref:sycl/pythonInterface.cpp:420 -> dequantize_cpu (cpu_ops.cpp:7-14).  Host pointers.
void cdequantize_blockwise_cpu_fp32(float* code, unsigned char* A, float* absmax, float* out, long long blocksize,
                                    long long n) {
  if (n <= 0 || blocksize <= 0) return;
  const long long nblocks = (n + blocksize - 1) / blocksize;
  parallel_blocks(nblocks, blocksize, [&](long long b0, long long b1) {
    for (long long blk = b0; blk < b1; ++blk) {
      const long long s = blk * blocksize;
      const long long e = std::min(n, s + blocksize);
      const float m = absmax[blk];
      for (long long i = s; i < e; ++i) out[i] = code[A[i]] * m;
    }
  });
}

// [additive] worker threads of the two host entry points (0 = default); returns the count in effect.
int cset_cpu_threads(int threads) {
  g_cpu_threads.store(threads > 0 ? threads : 0);
  return cpu_threads();
}

}  // extern "C"
