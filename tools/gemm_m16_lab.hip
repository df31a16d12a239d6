// Fused NF4 GEMM: the 32x32x16 MFMA schedule against the 16x16x32 one (k_gemm_4bit_256<.., M16>), same
// tile, same LDS layout, alternating in one process on random data (the chip's clock under load depends on
// the MFMA shape, MI355X_MICROARCH.md 'DVFS give-back' item 7).  Usage: gemm_m16_lab [M N K]
#include "gemm4bit_256.hip"
#include <cmath>
#include <cstdlib>
#include <cstring>
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
  auto l32 = [&]() { hipLaunchKernelGGL((k_gemm_4bit_256<bf16_t, false, false, 1>), dim3(tiles), dim3(512), 0, 0, N, M, K, (const bf16_t*)X, W, am, code, (bf16_t*)Y0, K, K / 2, N, BS, (float*)nullptr, 1); };
  auto l16 = [&]() { hipLaunchKernelGGL((k_gemm_4bit_256<bf16_t, false, true, 1>), dim3(tiles), dim3(512), 0, 0, N, M, K, (const bf16_t*)X, W, am, code, (bf16_t*)Y1, K, K / 2, N, BS, (float*)nullptr, 1); };
  auto l16c = [&]() { hipLaunchKernelGGL((k_gemm_4bit_256<bf16_t, false, true, 4>), dim3(tiles), dim3(512), 0, 0, N, M, K, (const bf16_t*)X, W, am, code, (bf16_t*)Y1, K, K / 2, N, BS, (float*)nullptr, 1); };
  for (int i = 0; i < 200; ++i) { l32(); l16(); }
  CK(hipDeviceSynchronize());
  {
    std::vector<uint16_t> a((size_t)M * N), b((size_t)M * N);
    CK(hipMemcpy(a.data(), Y0, a.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), Y1, b.size() * 2, hipMemcpyDeviceToHost));
    double md = 0, mr = 0; size_t bad = 0;
    for (size_t i = 0; i < a.size(); ++i) {
      uint32_t ua = (uint32_t)a[i] << 16, ub = (uint32_t)b[i] << 16; float fa, fb; memcpy(&fa, &ua, 4); memcpy(&fb, &ub, 4);
      const double d = fabs((double)fa - fb); md = std::max(md, d); mr = std::max(mr, (double)fabsf(fa));
      bad += d > 0.02 * fabs((double)fa) + 0.05;
    }
    printf("agreement: max|d| %.4g  max|y| %.4g  outside tol %zu / %zu\n", md, mr, bad, a.size());
  }
  const double flop = 2.0 * M * N * K;
  for (int i = 0; i < 50; ++i) l16c();
  CK(hipDeviceSynchronize());
  {
    std::vector<uint16_t> a((size_t)M * N), b((size_t)M * N);
    CK(hipMemcpy(a.data(), Y0, a.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), Y1, b.size() * 2, hipMemcpyDeviceToHost));
    printf("LUT x4 vs 32x32: %s\n", memcmp(a.data(), b.data(), a.size() * 2) ? "DIFFER" : "bit-identical");
  }
  const char* names[3] = {"32x32x16 LUTx1", "16x16x32 LUTx1", "16x16x32 LUTx4"};
  for (int rep = 0; rep < 4; ++rep) {
    for (int which = 0; which < 3; ++which) {
      auto go = [&]() { if (which == 0) l32(); else if (which == 1) l16(); else l16c(); };
      for (int i = 0; i < 20; ++i) go();
      CK(hipEventRecord(e0));
      for (int i = 0; i < 30; ++i) go();
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / 30;
      printf("%s %8.1f us  %7.1f TFLOP/s\n", names[which], us, flop / us / 1e6);
    }
  }
  return 0;
}
