// LAB (not built into the library): csrc/hgemm.hip (hand-written 4-wave 256x256 bf16 GEMM) against rocBLAS's
// standard algorithm on the same operands: agreement (fp32-accumulated references, bf16 outputs) and timing,
// interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).  Operands uniform [-1, 1) random.
// Usage: hgemm_lab [M N K] [rounds]
#define ROCBLAS_BETA_FEATURES_API
#pragma clang diagnostic ignored "-Wdeprecated-declarations"
#include <rocblas/rocblas.h>

#include "hgemm.hip"

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace bnb {
hipStream_t current_stream() { return nullptr; }
void set_error(int, const char* what) { printf("error: %s\n", what); }
int g_tile_override = 0;
BnbRange::BnbRange(const char*) : on(false) {}
BnbRange::~BnbRange() {}
int device_cu_count() { return 256; }
template <typename T> void launch_splitk_rows_reduce(const float*, int, int, int, T*, int) {}   // split-K unused here
template void launch_splitk_rows_reduce<bf16_t>(const float*, int, int, int, bf16_t*, int);
template void launch_splitk_rows_reduce<fp16_t>(const float*, int, int, int, fp16_t*, int);
}  // namespace bnb
using namespace bnb;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static float bf2f(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }

// the k_hgemm schedule variants compared (HG_V bits, csrc/hgemm.hip)
template <int... Vs> struct Variants {
  template <class F> static void each(F f) { (f(std::integral_constant<int, Vs>{}), ...); }
};
using LabV = Variants<16 + 8192, 8 + 16 + 4096>;

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 4096, K = argc > 3 ? atoi(argv[3]) : 11008;
  const int rounds = argc > 4 ? atoi(argv[4]) : 5;
  uint16_t *X, *W, *Y0, *Y1;
  CK(hipMalloc(&X, (size_t)M * K * 2)); CK(hipMalloc(&W, (size_t)N * K * 2));
  CK(hipMalloc(&Y0, (size_t)M * N * 2)); CK(hipMalloc(&Y1, (size_t)M * N * 2));
  const int data = argc > 5 ? atoi(argv[5]) : 0;   // 0: uniform [-1, 1); 1: X ~ N(0,1), W = NF4 values x absmax ~ 0.02-0.06
  {
    std::vector<uint16_t> h((size_t)std::max(M, N) * K);
    srand(3);
    auto bf = [](float f) { uint32_t u; memcpy(&u, &f, 4); return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16); };
    auto gauss = [] {
      const float u1 = (rand() + 1.0f) / (RAND_MAX + 2.0f), u2 = (rand() + 1.0f) / (RAND_MAX + 2.0f);
      return sqrtf(-2.0f * logf(u1)) * cosf(6.2831853f * u2);
    };
    static const float nf4[16] = {-1.0f, -0.6961928f, -0.5250731f, -0.3949175f, -0.2844414f, -0.1847734f, -0.0910500f, 0.0f,
                                  0.0795803f, 0.1609302f, 0.2461123f, 0.3379152f, 0.4407098f, 0.5626170f, 0.7229568f, 1.0f};
    for (size_t i = 0; i < (size_t)M * K; ++i)
      h[i] = data ? bf(gauss()) : bf(((rand() & 0xFFFF) - 32768) / 32768.0f);
    CK(hipMemcpy(X, h.data(), (size_t)M * K * 2, hipMemcpyHostToDevice));
    float am = 0.04f;
    for (size_t i = 0; i < (size_t)N * K; ++i) {
      if (data && i % 64 == 0) am = 0.02f + 0.04f * (rand() & 0xFFFF) / 65536.0f;
      h[i] = data ? bf(nf4[rand() & 15] * am) : bf(((rand() & 0xFFFF) - 32768) / 32768.0f);
    }
    CK(hipMemcpy(W, h.data(), (size_t)N * K * 2, hipMemcpyHostToDevice));
  }
  rocblas_handle h;
  rocblas_create_handle(&h);
  const float alpha = 1.0f, beta = 0.0f;
  auto lib = [&]() {
    rocblas_gemm_ex(h, rocblas_operation_transpose, rocblas_operation_none, N, M, K, &alpha, W, rocblas_datatype_bf16_r, K, X,
                    rocblas_datatype_bf16_r, K, &beta, Y0, rocblas_datatype_bf16_r, N, Y0, rocblas_datatype_bf16_r, N,
                    rocblas_datatype_f32_r, rocblas_gemm_algo_standard, 0, 0);
  };
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  auto mine = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(tiles), dim3(HG_THREADS), 0, 0, M, N, K, (const void*)X, (long long)K, (const void*)W,
                       (long long)K, (void*)Y1, (long long)N, nullptr, nullptr, nullptr, nullptr, 1, K * 2 / 128,
                       bnb::HgSide{});
  };
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](auto go, int R) {
    CK(hipEventRecord(e0));
    for (int i = 0; i < R; ++i) go();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / R;
  };
  auto agree = [&](const char* name) {
    std::vector<uint16_t> a((size_t)M * N), b((size_t)M * N);
    CK(hipMemcpy(a.data(), Y0, a.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), Y1, b.size() * 2, hipMemcpyDeviceToHost));
    double maxd = 0, maxa = 0, sumd = 0;
    size_t nbad = 0;
    for (size_t i = 0; i < a.size(); ++i) {
      const double x = bf2f(a[i]), y = bf2f(b[i]);
      const double d = fabs(x - y);
      maxd = fmax(maxd, d); maxa = fmax(maxa, fabs(x)); sumd += d;
      if (!(d <= 0.01 * fabs(x) + 0.02 * sqrt((double)K / 3.0) * 0.05)) ++nbad;
    }
    printf("%-12s agreement: max|d| %.4g  max|ref| %.4g  mean|d| %.4g  bad %zu / %zu\n", name, maxd, maxa, sumd / a.size(), nbad,
           a.size());
  };
  const double flop = 2.0 * M * N * K;
  // warm the clocks on the library, then correctness, then interleaved rounds
  for (int i = 0; i < 100; ++i) lib();
  CK(hipDeviceSynchronize());
  auto check = [&](auto kern, const char* name) {
    CK(hipMemset(Y1, 0xFF, (size_t)M * N * 2));
    mine(kern);
    CK(hipDeviceSynchronize());
    agree(name);
  };
  LabV::each([&](auto v) {
    char name[32];
    snprintf(name, sizeof name, "hgemm v%d", (int)decltype(v)::value);
    check(k_hgemm<HG_BF16, decltype(v)::value>, name);
  });
  const int R = 20;
  for (int r = 0; r < rounds; ++r) {
    const double t_lib = timeit(lib, R);
    printf("round %d  rocblas %7.1f us %6.0f TF |", r, t_lib, flop / t_lib / 1e6);
    LabV::each([&](auto v) {
      const double t = timeit([&] { mine(k_hgemm<HG_BF16, decltype(v)::value>); }, R);
      printf(" v%d %7.1f us %6.0f TF |", (int)decltype(v)::value, t, flop / t / 1e6);
    });
    printf("\n");
    fflush(stdout);
  }
  return 0;
}
