// A/B of the current 256-tile NF4 GEMM (csrc/gemm4bit_256.hip) against a saved copy of an earlier
// revision (tools/_bin/gemm4bit_256_old.hip, namespace bnbold), alternating in one process.
#include "gemm4bit_256.hip"
#include "_bin/gemm4bit_256_old.hip"
#include <vector>
#include <cstring>
#include <cstdlib>
namespace bnb {
hipStream_t current_stream() { return nullptr; }
void set_error(int, const char* what) { printf("error: %s\n", what); }
int g_tile_override = 0;
}  // namespace bnb
using namespace bnb;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
int main() {
  const int M = 4096, N = 4096, K = 11008, BS = 64;
  uint16_t *X, *Y; uint8_t* W; float *am, *code;
  CK(hipMalloc(&X, (size_t)M * K * 2)); CK(hipMalloc(&Y, (size_t)M * N * 2));
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
  const int tiles = (M / 256) * (N / 256);
  auto launch_new = [&]() { hipLaunchKernelGGL((k_gemm_4bit_256<bf16_t, false>), dim3(tiles), dim3(512), 0, 0, N, M, K, (const bf16_t*)X, W, am, code, (bf16_t*)Y, K, K / 2, N, BS, (float*)nullptr, 1); };
  auto launch_old = [&]() { hipLaunchKernelGGL((bnbold::k_gemm_4bit_256<bf16_t>), dim3(tiles), dim3(512), 0, 0, N, M, K, (const bf16_t*)X, W, am, code, (bf16_t*)Y, K, K / 2, N, BS); };
  for (int i = 0; i < 300; ++i) launch_new();
  CK(hipDeviceSynchronize());
  for (int rep = 0; rep < 4; ++rep) {
    for (int which = 0; which < 2; ++which) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 30; ++i) { if (which) launch_old(); else launch_new(); }
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      printf("%s %8.1f us\n", which ? "old" : "new", ms * 1e3 / 30);
    }
  }
  return 0;
}
