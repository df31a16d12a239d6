// Library GEMM with a per-shape solution search: the F.linear half of the large-prefill pair (the reference's
// M > 1 algorithm, dequantize_4bit + F.linear, ref:autograd/_functions.py:491-507), C[M, N] = A[M, K] . W[N, K]^T,
// bf16 / fp16 in and out, fp32 accumulation.
//
// Why (profiles/lab/r02_rocblas_solutions.txt): the default solution the libraries pick is far off for some of these
// shapes -- 4096 x 11008 x 4096 (the gate/up projection at 4096 tokens) runs 407 us on torch's hipBLASLt default and
// 411 us on rocBLAS's standard algorithm, while one of the 230 solutions rocBLAS lists for it takes 250 us.  So the
// first call of a shape (>= 10 GFLOP) times the standard algorithm and every listed solution on its own operands (one
// warm and one timed call each, the best three re-timed, within a time budget) and keeps a solution only when it beats
// the standard one by more than 5 %.  The plan is cached per device, dtype, leading dimensions, N, K and quarter-octave bucket of M (variable
// prefill lengths share a plan); a solution that rejects a later size in its bucket falls back to the standard
// algorithm.  No search during HIP-graph capture (the standard algorithm, or the cached plan, is used).
#define ROCBLAS_BETA_FEATURES_API          // rocblas_gemm_ex_get_solutions (a beta, "deprecated"-tagged API)
#pragma clang diagnostic ignored "-Wdeprecated-declarations"
#include <rocblas/rocblas.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "common.hpp"

namespace bnb {

namespace {

struct PlanKey {
  int dev, dtype, mb, n, k, lda, ldw, ldc;
  bool operator<(const PlanKey& o) const {
    return std::tie(dev, dtype, mb, n, k, lda, ldw, ldc) < std::tie(o.dev, o.dtype, o.mb, o.n, o.k, o.lda, o.ldw, o.ldc);
  }
};

std::mutex g_mu;
std::map<PlanKey, int> g_plans;                 // solution index (rocBLAS lists negative ones too); 0 = standard
std::map<int, rocblas_handle> g_handles;        // per device
Knob<int> g_search{1};                               // 0: never search (standard algorithm only)
Knob<double> g_budget_ms{2000.0};                    // search time per shape (230 solutions at 4096 x 11008 x 4096: ~1 s)
constexpr double kSearchMinFlop = 1e10;         // smaller problems keep the standard algorithm (nothing to win)

int rows_bucket(int m) {
  int bits = 0;
  while ((1 << bits) <= m) ++bits;              // bit length of m
  const int step = 1 << (bits > 3 ? bits - 3 : 0);
  return m / step * step;
}

rocblas_handle handle_for(int dev) {
  auto it = g_handles.find(dev);
  if (it != g_handles.end()) return it->second;
  rocblas_handle h = nullptr;
  if (rocblas_create_handle(&h) != rocblas_status_success) return nullptr;
  g_handles[dev] = h;
  return h;
}

// C (row-major [m, n], ldc) = A (row-major [m, k], lda) x W (row-major [n, k], ldw)^T.  In rocBLAS's column-major
// terms: C^T [n, m] = op(W^T [k, n])^T x A^T [k, m], i.e. transA = T on W, transB = N on A.
rocblas_status call(rocblas_handle h, rocblas_datatype t, int m, int n, int k, const void* A, int lda, const void* W,
                    int ldw, void* C, int ldc, int sol) {
  const float alpha = 1.0f, beta = 0.0f;
  return rocblas_gemm_ex(h, rocblas_operation_transpose, rocblas_operation_none, n, m, k, &alpha, W, t, ldw, A, t, lda,
                         &beta, C, t, ldc, C, t, ldc, rocblas_datatype_f32_r,
                         sol != 0 ? rocblas_gemm_algo_solution_index : rocblas_gemm_algo_standard, sol, 0);
}

// time one call of solution `sol` on the stream (ms); < 0 when the solution rejects the problem
float time_call(rocblas_handle h, rocblas_datatype t, int m, int n, int k, const void* A, int lda, const void* W,
                int ldw, void* C, int ldc, int sol, hipStream_t s, hipEvent_t e0, hipEvent_t e1, int reps) {
  hipEventRecord(e0, s);
  for (int r = 0; r < reps; ++r)
    if (call(h, t, m, n, k, A, lda, W, ldw, C, ldc, sol) != rocblas_status_success) return -1.0f;
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms = 0.0f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int search(rocblas_handle h, rocblas_datatype t, int m, int n, int k, const void* A, int lda, const void* W, int ldw,
           void* C, int ldc, hipStream_t s) {
  const auto start = std::chrono::steady_clock::now();
  auto elapsed_ms = [&] {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - start).count();
  };
  const float alpha = 1.0f, beta = 0.0f;
  rocblas_int count = 0;
  if (rocblas_gemm_ex_get_solutions(h, rocblas_operation_transpose, rocblas_operation_none, n, m, k, &alpha, W, t, ldw,
                                    A, t, lda, &beta, C, t, ldc, C, t, ldc, rocblas_datatype_f32_r,
                                    rocblas_gemm_algo_solution_index, 0, nullptr, &count) != rocblas_status_success ||
      count <= 0)
    return 0;
  std::vector<rocblas_int> sols(count);
  if (rocblas_gemm_ex_get_solutions(h, rocblas_operation_transpose, rocblas_operation_none, n, m, k, &alpha, W, t, ldw,
                                    A, t, lda, &beta, C, t, ldc, C, t, ldc, rocblas_datatype_f32_r,
                                    rocblas_gemm_algo_solution_index, 0, sols.data(), &count) != rocblas_status_success)
    return 0;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  time_call(h, t, m, n, k, A, lda, W, ldw, C, ldc, 0, s, e0, e1, 1);                 // warm
  const float t_std = time_call(h, t, m, n, k, A, lda, W, ldw, C, ldc, 0, s, e0, e1, 2);
  std::vector<std::pair<float, int>> cand;
  for (int i = 0; i < count && elapsed_ms() < g_budget_ms; ++i) {
    // the first call of a solution also loads its code object: one untimed call, then one timed
    if (time_call(h, t, m, n, k, A, lda, W, ldw, C, ldc, sols[i], s, e0, e1, 1) < 0.0f) continue;
    const float ms = time_call(h, t, m, n, k, A, lda, W, ldw, C, ldc, sols[i], s, e0, e1, 1);
    if (ms > 0.0f) cand.emplace_back(ms, sols[i]);
  }
  std::sort(cand.begin(), cand.end());
  int best = 0;
  float t_best = t_std;
  for (size_t i = 0; i < cand.size() && i < 3; ++i) {
    const float ms = time_call(h, t, m, n, k, A, lda, W, ldw, C, ldc, cand[i].second, s, e0, e1, 2);
    if (ms > 0.0f && ms < t_best) {
      t_best = ms;
      best = cand[i].second;
    }
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return (best != 0 && t_best < 0.95f * t_std) ? best : 0;
}

template <rocblas_datatype DT>
int gemm_tn(int m, int n, int k, const void* A, int lda, const void* W, int ldw, void* C, int ldc) {
  if (m <= 0 || n <= 0) return 0;
  if (k <= 0 || lda < k || ldw < k || ldc < n) {
    set_error(1, "gemm_tn: needs k > 0, lda >= k, ldw >= k, ldc >= n");
    return 1;
  }
  int dev = 0;
  hipGetDevice(&dev);
  const hipStream_t s = current_stream();
  std::lock_guard<std::mutex> lock(g_mu);
  rocblas_handle h = handle_for(dev);
  if (h == nullptr || rocblas_set_stream(h, s) != rocblas_status_success) {
    set_error(1, "gemm_tn: rocBLAS handle");
    return 1;
  }
  const PlanKey key{dev, (int)DT, rows_bucket(m), n, k, lda, ldw, ldc};
  auto it = g_plans.find(key);
  int sol = 0;
  if (it != g_plans.end()) {
    sol = it->second;
  } else {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hipStreamIsCapturing(s, &cs);
    if (cs == hipStreamCaptureStatusNone) {
      const bool big = 2.0 * m * n * k >= kSearchMinFlop;
      sol = (g_search && big) ? search(h, DT, m, n, k, A, lda, W, ldw, C, ldc, s) : 0;
      g_plans[key] = sol;
    }
  }
  rocblas_status st = call(h, DT, m, n, k, A, lda, W, ldw, C, ldc, sol);
  if (st != rocblas_status_success && sol != 0) st = call(h, DT, m, n, k, A, lda, W, ldw, C, ldc, 0);
  if (st != rocblas_status_success) {
    set_error((int)st, "gemm_tn: rocblas_gemm_ex");
    return 1;
  }
  return 0;
}

}  // namespace

}  // namespace bnb

extern "C" {

// [additive] C[m, n] = A[m, k] . W[n, k]^T (row-major, bf16 / fp16 in and out, fp32 accumulation): the library GEMM of
// the large-prefill 4-bit path (after cdequantize_blockwise_* / cdequantize_blockwise_nested_* into W), with the
// per-shape solution search above.  Returns 0 on success, 1 on error (cget_last_error*).
int cgemm_tn_bf16(int m, int n, int k, const bf16_t* A, int lda, const bf16_t* W, int ldw, bf16_t* C, int ldc) {
  BNB_RANGE("cgemm_tn_bf16");
  return bnb::gemm_tn<rocblas_datatype_bf16_r>(m, n, k, A, lda, W, ldw, C, ldc);
}
int cgemm_tn_fp16(int m, int n, int k, const fp16_t* A, int lda, const fp16_t* W, int ldw, fp16_t* C, int ldc) {
  BNB_RANGE("cgemm_tn_fp16");
  return bnb::gemm_tn<rocblas_datatype_f16_r>(m, n, k, A, lda, W, ldw, C, ldc);
}
// [additive] solution search: on = 0 -> the standard algorithm only; budget_ms > 0 sets the per-shape search time;
// clear != 0 forgets every cached plan.  Returns the number of cached plans.
int cgemm_tn_set_search(int on, double budget_ms, int clear) {
  BNB_RANGE("cgemm_tn_set_search");
  std::lock_guard<std::mutex> lock(bnb::g_mu);
  bnb::g_search = on;
  if (budget_ms > 0.0) bnb::g_budget_ms = budget_ms;
  if (clear) bnb::g_plans.clear();
  return (int)bnb::g_plans.size();
}
// [additive] the cached plan for (m, n, k, dtype 0 = bf16 / 1 = fp16, lda, ldw, ldc) on the current device: 1 = a
// searched rocBLAS solution, 0 = the standard algorithm, -1 = not searched yet
int cgemm_tn_plan(int m, int n, int k, int dtype, int lda, int ldw, int ldc) {
  BNB_RANGE("cgemm_tn_plan");
  int dev = 0;
  hipGetDevice(&dev);
  std::lock_guard<std::mutex> lock(bnb::g_mu);
  const bnb::PlanKey key{dev, dtype == 0 ? (int)rocblas_datatype_bf16_r : (int)rocblas_datatype_f16_r,
                         bnb::rows_bucket(m), n, k, lda, ldw, ldc};
  auto it = bnb::g_plans.find(key);
  return it == bnb::g_plans.end() ? -1 : (it->second != 0 ? 1 : 0);
}

}  // extern "C"
