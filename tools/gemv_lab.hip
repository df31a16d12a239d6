// Decode GEMV lab (11008 x 4096 NF4, bf16 activations, plain fp32 absmax): the library table/dot kernel
// at several (R rows per wave, U chunk groups per lane) schedules, over 14 rotating weight copies (past
// the 256 MB MALL).  Run under `rocprofv3 --kernel-trace --stats` for per-kernel durations; outputs are
// checked against the library configuration (fp32 sums in a different order: tolerance, not bits).
#include "gemv4bit.hip"
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <vector>

namespace bnb {
hipStream_t current_stream() { return nullptr; }
void set_error(int, const char* what) { printf("error: %s\n", what); }
}  // namespace bnb
using namespace bnb;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
  const int M = 11008, K = 4096, BS = 64, COPIES = 14;
  const size_t wbytes = (size_t)M * K / 2, nabs = (size_t)M * K / BS;
  std::vector<uint8_t*> W(COPIES);
  std::vector<float*> AM(COPIES);
  bf16_t *x, *y0, *y1;
  float* code;
  for (int c = 0; c < COPIES; ++c) { CK(hipMalloc(&W[c], wbytes)); CK(hipMalloc(&AM[c], nabs * 4)); }
  CK(hipMalloc(&x, K * 2)); CK(hipMalloc(&y0, M * 2)); CK(hipMalloc(&y1, M * 2)); CK(hipMalloc(&code, 64));
  {
    std::vector<uint8_t> h(wbytes);
    uint32_t r = 7;
    for (auto& v : h) { r = r * 1664525u + 1013904223u; v = (uint8_t)(r >> 24); }
    std::vector<float> a(nabs);
    for (auto& v : a) { r = r * 1664525u + 1013904223u; v = 0.01f + (r >> 8) / 16777216.0f * 0.05f; }
    for (int c = 0; c < COPIES; ++c) {
      CK(hipMemcpy(W[c], h.data(), wbytes, hipMemcpyHostToDevice));
      CK(hipMemcpy(AM[c], a.data(), nabs * 4, hipMemcpyHostToDevice));
    }
    std::vector<uint16_t> hx(K);
    for (auto& v : hx) { r = r * 1664525u + 1013904223u; float f = ((r >> 8) / 16777216.0f - 0.5f); uint32_t u; memcpy(&u, &f, 4); v = (uint16_t)(u >> 16); }
    CK(hipMemcpy(x, hx.data(), K * 2, hipMemcpyHostToDevice));
    const float nf4[16] = {-1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f, -0.28444138169288635f,
                           -0.18477343022823334f, -0.09105003625154495f, 0.0f, 0.07958029955625534f, 0.16093020141124725f,
                           0.24611230194568634f, 0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
                           0.7229568362236023f, 1.0f};
    CK(hipMemcpy(code, nf4, 64, hipMemcpyHostToDevice));
  }
  const size_t lds = GV_TABLE_BYTES + 2 * (size_t)K;
  auto run = [&](const char* name, auto kern, int R, bf16_t* y, int reps) {
    const int waves = (M + R - 1) / R;
    const int grid = (waves + 3) / 4;
    for (int i = 0; i < reps; ++i) {
      const int c = i % COPIES;
      GemvStats st{};
      st.absmax = AM[c];
      st.bs_shift = __builtin_ctz(BS);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, M, K, x, W[c], st, code, y, K / 2);
    }
    CK(hipDeviceSynchronize());
    printf("%s done\n", name);
  };
  auto check = [&](const char* name) {
    std::vector<uint16_t> a(M), b(M);
    CK(hipMemcpy(a.data(), y0, M * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), y1, M * 2, hipMemcpyDeviceToHost));
    double md = 0, mr = 0;
    for (int i = 0; i < M; ++i) {
      uint32_t ua = (uint32_t)a[i] << 16, ub = (uint32_t)b[i] << 16;
      float fa, fb; memcpy(&fa, &ua, 4); memcpy(&fb, &ub, 4);
      md = std::max(md, (double)fabsf(fa - fb)); mr = std::max(mr, (double)fabsf(fa));
    }
    printf("  %s: max|d| %.4g of max|y| %.4g\n", name, md, mr);
  };
  for (int rep = 0; rep < 2; ++rep) {
    run("R4U2 (library)", k_gemv_4bit_dot<bf16_t, 4, 2, false>, 4, y0, 200);
    run("R2U4", k_gemv_4bit_dot<bf16_t, 2, 4, false>, 2, y1, 200); check("R2U4");
    run("R8U1", k_gemv_4bit_dot<bf16_t, 8, 1, false>, 8, y1, 200); check("R8U1");
    run("R4U4", k_gemv_4bit_dot<bf16_t, 4, 4, false>, 4, y1, 200); check("R4U4");
    run("R8U2", k_gemv_4bit_dot<bf16_t, 8, 2, false>, 8, y1, 200); check("R8U2");
    run("R2U8", k_gemv_4bit_dot<bf16_t, 2, 8, false>, 2, y1, 200); check("R2U8");
  }
  return 0;
}
