// Decode-GEMV floor lab (round 2): how fast can the 25.4 MB of a 11008 x 4096 NF4 layer (packed bytes + fp32
// absmax) be streamed at all, back to back over 14 rotating copies (past the 256 MB MALL), against the library
// GEMV on the same buffers.  k_stream: every lane issues all of its 16-B non-temporal loads at once and folds
// them into one value per wave (kept live by a store), i.e. the GEMV's memory pattern with no table/dot work.
#include "gemv4bit.hip"
#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <functional>
#include <vector>

namespace bnb {
hipStream_t current_stream() { return nullptr; }
void set_error(int, const char* what) { printf("error: %s\n", what); }
}  // namespace bnb
using namespace bnb;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int U, int THREADS>
__global__ void __launch_bounds__(THREADS) k_stream(const uint4* __restrict__ src, long long n16, uint32_t* __restrict__ sink) {
  const long long base = (long long)blockIdx.x * THREADS * U + threadIdx.x;
  uint4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = min(base + (long long)u * THREADS, n16 - 1);
    const u32x4_t t = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(src + i));
    v[u] = make_uint4(t.x, t.y, t.z, t.w);
  }
  uint32_t s = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) s ^= v[u].x + v[u].y + v[u].z + v[u].w;
  if (s == 0x12345678u) sink[blockIdx.x] = s;
}

int main() {
  const int M = 11008, K = 4096, BS = 64, COPIES = 14;
  const size_t wbytes = (size_t)M * K / 2, nabs = (size_t)M * K / BS;
  std::vector<uint8_t*> W(COPIES);
  std::vector<float*> AM(COPIES);
  bf16_t *x, *y;
  float* code;
  uint32_t* sink;
  for (int c = 0; c < COPIES; ++c) { CK(hipMalloc(&W[c], wbytes + nabs * 4)); AM[c] = (float*)(W[c] + wbytes); }
  CK(hipMalloc(&x, K * 2)); CK(hipMalloc(&y, M * 2)); CK(hipMalloc(&code, 64)); CK(hipMalloc(&sink, 1 << 20));
  {
    std::vector<uint8_t> h(wbytes + nabs * 4);
    uint32_t r = 7;
    for (size_t i = 0; i < wbytes; ++i) { r = r * 1664525u + 1013904223u; h[i] = (uint8_t)(r >> 24); }
    float* a = (float*)(h.data() + wbytes);
    for (size_t i = 0; i < nabs; ++i) { r = r * 1664525u + 1013904223u; a[i] = 0.01f + (r >> 8) / 16777216.0f * 0.05f; }
    for (int c = 0; c < COPIES; ++c) CK(hipMemcpy(W[c], h.data(), h.size(), hipMemcpyHostToDevice));
    std::vector<uint16_t> hx(K, 0x3f80);
    CK(hipMemcpy(x, hx.data(), K * 2, hipMemcpyHostToDevice));
    float nf4[16];
    for (int i = 0; i < 16; ++i) nf4[i] = (i - 7.5f) / 7.5f;
    CK(hipMemcpy(code, nf4, 64, hipMemcpyHostToDevice));
  }
  const long long n16 = (long long)(wbytes + nabs * 4) / 16;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  struct V { const char* name; std::function<void(int)> fn; std::vector<double> us; };
  std::vector<V> vs;
  auto stream = [&](auto kern, int U, int T) {
    return [=](int c) {
      const long long g = (n16 + (long long)U * T - 1) / ((long long)U * T);
      hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3(T), 0, 0, (const uint4*)W[c], n16, sink);
    };
  };
  vs.push_back({"stream U8 x256 (6.2k WG)", stream(k_stream<8, 256>, 8, 256), {}});
  vs.push_back({"stream U16 x256 (3.1k WG)", stream(k_stream<16, 256>, 16, 256), {}});
  vs.push_back({"stream U4 x512", stream(k_stream<4, 512>, 4, 512), {}});
  vs.push_back({"stream U2 x256 (25k WG)", stream(k_stream<2, 256>, 2, 256), {}});
  vs.push_back({"GEMV library (plain)", [&](int c) {
                  GemvStats st{};
                  st.absmax = AM[c];
                  launch_gemv_dot<bf16_t>(M, K, x, W[c], st, code, y, K / 2, BS, 0);
                }, {}});
  for (auto& v : vs)
    for (int i = 0; i < 28; ++i) v.fn(i % COPIES);
  CK(hipDeviceSynchronize());
  for (int rep = 0; rep < 15; ++rep)
    for (auto& v : vs) {
      for (int i = 0; i < 14; ++i) v.fn(i);
      CK(hipEventRecord(e0));
      for (int i = 0; i < 28; ++i) v.fn(i % COPIES);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1e3 / 28);
    }
  const double bytes = (double)(wbytes + nabs * 4);
  for (auto& v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double med = v.us[v.us.size() / 2];
    printf("%-28s median %6.2f us  %6.0f GB/s  (min %6.2f)\n", v.name, med, bytes / med / 1e3, v.us.front());
  }
  return 0;
}
