// NF4 GEMM lab 2: the register-dequant kernel (tools/gemm4bit_rd_lab.hip) against the LDS-dequant
// 256-tile kernel (csrc/gemm4bit_256.hip) at M=4096, N=4096, K=11008: agreement and timing, plus
// ablations (FL 1: no activation DMA, 2: no dequant; results garbage for FL != 0).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I bitsandbytes-sycl_amd/csrc tools/gemm_lab2.hip
#include "gemm4bit_256.hip"
#include "gemm4bit_rd_lab.hip"
#include "gemm4bit_w4_lab.hip"
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <type_traits>

namespace bnb {
hipStream_t current_stream() { return nullptr; }
void set_error(int, const char* what) { printf("error: %s\n", what); }
int g_tile_override = 0;
}  // namespace bnb
using namespace bnb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static float bf2f(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 4096, K = argc > 3 ? atoi(argv[3]) : 11008;
  const int BS = 64;
  uint16_t *X, *Y0, *Y1; uint8_t* W; float *am, *code;
  CK(hipMalloc(&X, (size_t)M * K * 2)); CK(hipMalloc(&Y0, (size_t)M * N * 2)); CK(hipMalloc(&Y1, (size_t)M * N * 2));
  CK(hipMalloc(&W, (size_t)N * K / 2)); CK(hipMalloc(&am, (size_t)N * K / BS * 4)); CK(hipMalloc(&code, 64));
  {
    std::vector<uint16_t> hx((size_t)M * K);
    srand(3);
    for (auto& v : hx) { float f = ((rand() & 0xFFFF) - 32768) / 16384.0f; uint32_t u; memcpy(&u, &f, 4); v = (uint16_t)(u >> 16); }
    CK(hipMemcpy(X, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
    std::vector<uint8_t> hw((size_t)N * K / 2);
    for (auto& v : hw) v = rand() & 0xFF;
    CK(hipMemcpy(W, hw.data(), hw.size(), hipMemcpyHostToDevice));
    std::vector<float> ha((size_t)N * (K / BS));
    for (auto& v : ha) v = 0.005f + 0.045f * (rand() & 0xFFFF) / 65536.0f;
    CK(hipMemcpy(am, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
  }
  const float hc[16] = {-1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
                        -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
                        0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f, 0.33791524171829224f,
                        0.44070982933044434f, 0.5626170039176941f, 0.7229568362236023f, 1.0f};
  CK(hipMemcpy(code, hc, 64, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  auto launch = [&](auto kern, uint16_t* Y) {
    hipLaunchKernelGGL(kern, dim3(tiles), dim3(512), 0, 0, N, M, K, (const bf16_t*)X, W, am, code, (bf16_t*)Y, K, K / 2, N, BS);
  };
  // the library kernel takes (ws, ksplit) as well
  auto launch256 = [&](uint16_t* Y) {
    hipLaunchKernelGGL((k_gemm_4bit_256<bf16_t, false>), dim3(tiles), dim3(512), 0, 0, N, M, K, (const bf16_t*)X, W, am,
                       code, (bf16_t*)Y, K, K / 2, N, BS, (float*)nullptr, 1);
  };
  auto launchw4 = [&](auto kern, uint16_t* Y) {
    hipLaunchKernelGGL(kern, dim3(tiles), dim3(256), 0, 0, N, M, K, (const bf16_t*)X, W, am, code, (bf16_t*)Y, K, K / 2, N, BS);
  };
  auto run = [&](const char* name, auto kern, uint16_t* Y, bool w4 = false) {
    auto go = [&]() {
      if constexpr (std::is_same_v<decltype(kern), int>) launch256(Y);
      else if (w4) launchw4(kern, Y);
      else launch(kern, Y);
    };
    for (int i = 0; i < 3; ++i) go();
    CK(hipDeviceSynchronize());
    const int R = 30;
    CK(hipEventRecord(e0));
    for (int i = 0; i < R; ++i) go();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / R;
    printf("%-24s %8.1f us  %7.1f TFLOP/s\n", name, us, 2.0 * M * N * K / us / 1e6);
    fflush(stdout);
  };
  // warm the clocks
  for (int i = 0; i < 200; ++i) launch256(Y0);
  CK(hipDeviceSynchronize());
  auto agree = [&]() {
    std::vector<uint16_t> a((size_t)M * N), b((size_t)M * N);
    CK(hipMemcpy(a.data(), Y0, a.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), Y1, b.size() * 2, hipMemcpyDeviceToHost));
    double maxd = 0, maxa = 0, sumd = 0;
    size_t nbad = 0;
    for (size_t i = 0; i < a.size(); ++i) {
      const double x = bf2f(a[i]), y = bf2f(b[i]);
      const double d = fabs(x - y);
      maxd = fmax(maxd, d); maxa = fmax(maxa, fabs(x)); sumd += d;
      if (!(d <= 0.02 * fabs(x) + 0.05)) ++nbad;
    }
    printf("agreement: max|d| %.4g  max|ref| %.4g  mean|d| %.4g  bad %zu / %zu\n", maxd, maxa, sumd / a.size(), nbad, a.size());
  };
  run("256 (LDS dequant)", 0, Y0);
  run("w4 (1 wave/SIMD)", k_gemm_4bit_w4<bf16_t, 0>, Y1, true);
  agree();
  run("w4 setprio", k_gemm_4bit_w4<bf16_t, 4>, Y1, true);
  agree();
  run("w4 no-dma", k_gemm_4bit_w4<bf16_t, 1>, Y1, true);
  run("w4 no-dequant", k_gemm_4bit_w4<bf16_t, 2>, Y1, true);
  run("w4 no-dma no-deq", k_gemm_4bit_w4<bf16_t, 3>, Y1, true);
  run("256 (LDS dequant)", 0, Y0);
  run("w4 (1 wave/SIMD)", k_gemm_4bit_w4<bf16_t, 0>, Y1, true);
  run("rd (reg dequant)", k_gemm_4bit_rd<bf16_t, 0>, Y1);
  return 0;
}
