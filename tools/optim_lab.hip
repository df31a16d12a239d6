// Optimizer kernel lab: Adam 8-bit blockwise (fp32) at 2^27 elements with the dynamic maps in the
// search layout (common.hpp DynMapView) at several grid sizes, against the scalar one-search-at-a-time
// form, plus the no-requant / division-only parts.
// Every variant starts from the same state and must produce bit-identical p, states and absmax.
#include "optim.hip"
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>
namespace bnb {
hipStream_t current_stream() { return nullptr; }
void set_error(int, const char* what) { printf("error: %s\n", what); }
}  // namespace bnb
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// create_dynamic_map(signed, 7, 8) (functional.create_dynamic_map), float32 arithmetic
static std::vector<float> dynamic_map(bool sign) {
  std::vector<float> d;
  for (int i = 0; i < 7; ++i) {
    const int items = sign ? (1 << i) + 1 : (1 << (i + 1)) + 1;
    std::vector<float> b(items);
    for (int j = 0; j < items; ++j) b[j] = 0.1f + (0.9f * j) / (items - 1);
    for (int j = 0; j + 1 < items; ++j) {
      const float v = (float)std::pow(10.0, -6 + i) * ((b[j] + b[j + 1]) / 2.0f);
      d.push_back(v);
      if (sign) d.push_back(-v);
    }
  }
  d.push_back(0.0f);
  d.push_back(1.0f);
  while (d.size() < 256) d.push_back(0.0f);
  std::sort(d.begin(), d.end());
  return d;
}

int main() {
  const int n = 1 << 27, nb = n / 2048;
  float *p, *g, *q1, *q2, *a1, *a2; uint8_t *s1, *s2;
  CK(hipMalloc(&p, n * 4LL)); CK(hipMalloc(&g, n * 4LL)); CK(hipMalloc(&s1, n)); CK(hipMalloc(&s2, n));
  CK(hipMalloc(&q1, 1024)); CK(hipMalloc(&q2, 1024)); CK(hipMalloc(&a1, nb * 4)); CK(hipMalloc(&a2, nb * 4));
  std::vector<float> hp(n), hg(n), ha1(nb), ha2(nb);
  std::vector<uint8_t> hs1(n), hs2(n);
  uint32_t r = 12345;
  auto rnd = [&]() { r = r * 1664525u + 1013904223u; return r >> 8; };
  for (int i = 0; i < n; ++i) {
    hg[i] = (rnd() / 16777216.0f - 0.5f) * 0.02f;
    hp[i] = (rnd() / 16777216.0f - 0.5f);
    hs1[i] = (uint8_t)(rnd() & 0xFF);
    hs2[i] = (uint8_t)(128 + (rnd() & 0x7F));
  }
  for (int b = 0; b < nb; ++b) { ha1[b] = 0.005f + (rnd() & 0xFF) * 1e-5f; ha2[b] = 1e-5f + (rnd() & 0xFF) * 1e-7f; }
  const std::vector<float> c1 = dynamic_map(true), c2 = dynamic_map(false);
  CK(hipMemcpy(q1, c1.data(), 1024, hipMemcpyHostToDevice));
  CK(hipMemcpy(q2, c2.data(), 1024, hipMemcpyHostToDevice));
  auto reset = [&]() {
    CK(hipMemcpy(g, hg.data(), n * 4LL, hipMemcpyHostToDevice)); CK(hipMemcpy(p, hp.data(), n * 4LL, hipMemcpyHostToDevice));
    CK(hipMemcpy(s1, hs1.data(), n, hipMemcpyHostToDevice)); CK(hipMemcpy(s2, hs2.data(), n, hipMemcpyHostToDevice));
    CK(hipMemcpy(a1, ha1.data(), nb * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(a2, ha2.data(), nb * 4, hipMemcpyHostToDevice));
  };
  bnb::OptScalars k{};
  k.beta1 = 0.9f; k.beta2 = 0.999f; k.eps = 1e-8f; k.lr = 1e-3f; k.gnorm_scale = 1.0f; k.step_size = -1e-3f; k.c2eps = 1e-8f; k.decay = 1.0f; k.step = 5;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> rp(n), ra(2 * nb);
  std::vector<uint8_t> rs(2LL * n);
  bool have_ref = false;
  auto run = [&](const char* name, auto kern, bool check, int grid = 0) {
    if (grid == 0) grid = nb;
    auto launch = [&]() { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, p, (const float*)g, s1, s2, (const float*)q1, (const float*)q2, a1, a2, k, n); };
    if (check) {
      reset();
      launch();
      CK(hipDeviceSynchronize());
      std::vector<float> op(n), oa(2 * nb);
      std::vector<uint8_t> os(2LL * n);
      CK(hipMemcpy(op.data(), p, n * 4LL, hipMemcpyDeviceToHost));
      CK(hipMemcpy(os.data(), s1, n, hipMemcpyDeviceToHost)); CK(hipMemcpy(os.data() + n, s2, n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(oa.data(), a1, nb * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(oa.data() + nb, a2, nb * 4, hipMemcpyDeviceToHost));
      if (!have_ref) { rp = op; rs = os; ra = oa; have_ref = true; }
      const bool same = !memcmp(op.data(), rp.data(), n * 4LL) && os == rs && !memcmp(oa.data(), ra.data(), nb * 8LL);
      long hist[4] = {0, 0, 0, 0};
      for (int i = 0; i < n; ++i) hist[std::min(3, std::abs((int)os[i] - 127) / 32)]++;
      printf("  %s: identical to scalar: %s  (state1 |code-127|/32 histogram %ld %ld %ld %ld)\n", name, same ? "yes" : "NO",
             hist[0], hist[1], hist[2], hist[3]);
    }
    reset();
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; ++i) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / 10, bytes = n * 16.0 + nb * 16.0;
    printf("%-26s %8.1f us  %7.0f GB/s\n", name, us, bytes / us / 1e3);
    fflush(stdout);
  };
  for (int rr = 0; rr < 2; ++rr) {
    run("adam8 fp32 scalar", bnb::k_optimizer_8bit_blockwise_2state<float, bnb::ADAM, 8>, rr == 0);
    for (int gr : {1024, 2048, 4096, nb}) {
      char nm[64];
      snprintf(nm, sizeof nm, "adam8 fp32 grid %d", gr);
      run(nm, bnb::k_optimizer_8bit_blockwise_2state<float, bnb::ADAM, 0>, rr == 0, gr);
    }
    run("adam8 fp32 no-requant g1024", bnb::k_optimizer_8bit_blockwise_2state<float, bnb::ADAM, 1>, false, 1024);
    run("adam8 fp32 div only g1024", bnb::k_optimizer_8bit_blockwise_2state<float, bnb::ADAM, 2>, false, 1024);
  }
  return 0;
}
