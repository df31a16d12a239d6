// Fused NF4 GEMM: the cross-barrier fragment pipeline (k_gemm_4bit_256<.., XB = true>) against the
// launched M16 schedule, interleaved timing on random data, outputs compared bit for bit.
// Usage: gemm_xb_lab [M N K]
#include "gemm4bit_256.hip"
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>
namespace bnb {
hipStream_t current_stream() { return nullptr; }
void set_error(int, const char* what) { printf("error: %s\n", what); }
int g_tile_override = 0;
}  // namespace bnb
using namespace bnb;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 4096, K = argc > 3 ? atoi(argv[3]) : 11008;
  const int BS = 64;
  uint16_t *X, *Y0, *Y1; uint8_t* W; float *am, *code;
  CK(hipMalloc(&X, (size_t)M * K * 2)); CK(hipMalloc(&Y0, (size_t)M * N * 2)); CK(hipMalloc(&Y1, (size_t)M * N * 2));
  CK(hipMalloc(&W, (size_t)N * K / 2)); CK(hipMalloc(&am, (size_t)N * K / BS * 4)); CK(hipMalloc(&code, 64));
  {
    std::vector<uint16_t> hx((size_t)M * K); srand(3);
    for (auto& v : hx) { float f = ((rand() & 0xFFFF) - 32768) / 16384.0f; uint32_t u; memcpy(&u, &f, 4); v = (uint16_t)(u >> 16); }
    CK(hipMemcpy(X, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
    std::vector<uint8_t> hw((size_t)N * K / 2); for (auto& v : hw) v = rand() & 0xFF;
    CK(hipMemcpy(W, hw.data(), hw.size(), hipMemcpyHostToDevice));
    std::vector<float> ha((size_t)N * (K / BS)); for (auto& v : ha) v = 0.005f + 0.045f * (rand() & 0xFFFF) / 65536.0f;
    CK(hipMemcpy(am, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
    float hc[16]; for (int i = 0; i < 16; ++i) hc[i] = (i - 7.5f) / 8; CK(hipMemcpy(code, hc, 64, hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  auto mk = [&](auto kern, uint16_t* Y) {
    return [=]() { hipLaunchKernelGGL(kern, dim3(tiles), dim3(512), 0, 0, N, M, K, (const bf16_t*)X, W, am, code, (bf16_t*)Y, K, K / 2, N, BS, (float*)nullptr, 1); };
  };
  struct V { const char* name; std::function<void()> fn; std::vector<double> us; };
  std::vector<V> vs;
  vs.push_back({"M16 (library)", mk(k_gemm_4bit_256<bf16_t, false, true, 4, false>, Y0), {}});
  vs.push_back({"M16 cross-barrier", mk(k_gemm_4bit_256<bf16_t, false, true, 4, true>, Y1), {}});
  for (int i = 0; i < 50; ++i) for (auto& v : vs) v.fn();
  CK(hipDeviceSynchronize());
  {
    std::vector<uint16_t> a((size_t)M * N), b((size_t)M * N);
    CK(hipMemcpy(a.data(), Y0, a.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), Y1, b.size() * 2, hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (size_t i = 0; i < a.size(); ++i) diff += a[i] != b[i];
    printf("cross-barrier vs library: %s (%zu differ)\n", diff ? "DIFFER" : "bit-identical", diff);
  }
  const double flop = 2.0 * M * N * K;
  for (int rep = 0; rep < 12; ++rep)
    for (auto& v : vs) {
      for (int i = 0; i < 2; ++i) v.fn();
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) v.fn();
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1e3 / 10);
    }
  for (auto& v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double med = v.us[v.us.size() / 2];
    printf("%-22s median %7.1f us  min %7.1f  max %7.1f  %7.1f TFLOP/s\n", v.name, med, v.us.front(), v.us.back(), flop / med / 1e6);
  }
  return 0;
}
