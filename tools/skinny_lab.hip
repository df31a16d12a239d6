// Few-token NF4 GEMM lab (csrc/gemm4bit_skinny.hip) at 8 tokens x 11008 x 4096 (and argv shapes): the kernel
// with parts switched off (ABL: 1 no weight loads, 2 no activation DMA, 4 no MFMA), plain fp32 absmax,
// 14 rotating weight copies (past the 256 MB MALL), event timing of the main kernel only (no reduce).
#include "gemm4bit_skinny.hip"
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>
namespace bnb {
hipStream_t current_stream() { return nullptr; }
void set_error(int, const char* what) { printf("error: %s\n", what); }
}  // namespace bnb
using namespace bnb;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 11008, K = argc > 2 ? atoi(argv[2]) : 4096, M = argc > 3 ? atoi(argv[3]) : 8;
  const int COPIES = 14, BS = 64;
  std::vector<uint8_t*> W(COPIES);
  std::vector<float*> AM(COPIES);
  for (int c = 0; c < COPIES; ++c) { CK(hipMalloc(&W[c], (size_t)N * K / 2)); CK(hipMalloc(&AM[c], (size_t)N * K / BS * 4)); }
  uint16_t *X, *Y; float *code, *ws;
  CK(hipMalloc(&X, (size_t)M * K * 2)); CK(hipMalloc(&Y, (size_t)M * N * 2)); CK(hipMalloc(&code, 64));
  CK(hipMalloc(&ws, (size_t)64 * M * N * 4));
  {
    std::vector<uint8_t> h((size_t)N * K / 2); uint32_t r = 7;
    for (auto& v : h) { r = r * 1664525u + 1013904223u; v = (uint8_t)(r >> 24); }
    std::vector<float> a((size_t)N * K / BS); for (auto& v : a) { r = r * 1664525u + 1013904223u; v = 0.01f + (r >> 8) / 16777216.0f * 0.05f; }
    for (int c = 0; c < COPIES; ++c) { CK(hipMemcpy(W[c], h.data(), h.size(), hipMemcpyHostToDevice)); CK(hipMemcpy(AM[c], a.data(), a.size() * 4, hipMemcpyHostToDevice)); }
    std::vector<uint16_t> hx((size_t)M * K); for (auto& v : hx) { r = r * 1664525u + 1013904223u; v = (uint16_t)(0x3c00 + (r >> 28)); }
    CK(hipMemcpy(X, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
    float hc[16]; for (int i = 0; i < 16; ++i) hc[i] = (i - 7.5f) / 8; CK(hipMemcpy(code, hc, 64, hipMemcpyHostToDevice));
  }
  const int s = skinny_geometry(N, M, K).splits;   // base form at these token counts
  const int grid = ((N + SK_ROWS - 1) / SK_ROWS) * s;
  printf("N=%d K=%d M=%d: %d splits, %d workgroups, weights %.1f MB\n", N, K, M, s, grid, N * (double)K / 2e6);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto mk = [&](auto kern) {
    return [=](int i) {
      SkStats st{AM[i % COPIES], nullptr, nullptr, nullptr, nullptr, __builtin_ctz(BS), 0};
      hipLaunchKernelGGL(kern, dim3(grid), dim3(SK_THREADS), 0, 0, N, M, K, (const bf16_t*)X, K, W[i % COPIES], K / 2, st,
                         code, ws, (bf16_t*)Y, N, s);
    };
  };
  struct V { const char* name; std::function<void(int)> fn; std::vector<double> us; };
  std::vector<V> vs;
  vs.push_back({"full", mk(k_gemm_4bit_skinny<bf16_t, 1, 10, false, 0>), {}});
  vs.push_back({"no MFMA", mk(k_gemm_4bit_skinny<bf16_t, 1, 10, false, 4>), {}});
  vs.push_back({"no X DMA", mk(k_gemm_4bit_skinny<bf16_t, 1, 10, false, 2>), {}});
  vs.push_back({"no W loads", mk(k_gemm_4bit_skinny<bf16_t, 1, 10, false, 1>), {}});
  vs.push_back({"loads only (no MFMA, no X)", mk(k_gemm_4bit_skinny<bf16_t, 1, 10, false, 6>), {}});
  vs.push_back({"nothing loaded", mk(k_gemm_4bit_skinny<bf16_t, 1, 10, false, 7>), {}});
  for (int i = 0; i < 50; ++i) for (auto& v : vs) v.fn(i);
  CK(hipDeviceSynchronize());
  for (int rep = 0; rep < 10; ++rep)
    for (auto& v : vs) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 28; ++i) v.fn(i);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1e3 / 28);
    }
  for (auto& v : vs) {
    std::sort(v.us.begin(), v.us.end());
    printf("%-28s median %7.2f us (incl. launch gaps)\n", v.name, v.us[v.us.size() / 2]);
  }
  return 0;
}
