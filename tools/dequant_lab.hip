// 4-bit dequantise lab at the metric weight (4096 x 11008 NF4 -> bf16, nested statistics): the library
// stream kernel at P = 4 / 8 / 16 packed dwords per lane against a 16-B-per-lane variant (one 16-B load ->
// 32 outputs -> four 16-B stores).  Outputs must be bit-identical.
#include "quant.hip"
#include <cstdlib>
#include <cstring>
#include <vector>

namespace bnb {
hipStream_t current_stream() { return nullptr; }
void set_error(int, const char* what) { printf("error: %s\n", what); }

template <typename T, int DT, int P>
__global__ void __launch_bounds__(256)
k_dq16(const uint8_t* __restrict__ A, T* __restrict__ out, int bs_shift, long long nq, NestedStats ns) {
  __shared__ float2 s_pair[256];
  __shared__ float s_code2[256];
  s_pair[threadIdx.x] = make_float2(code4_value<DT>(threadIdx.x >> 4), code4_value<DT>(threadIdx.x & 15));
  s_code2[threadIdx.x] = ns.code2[threadIdx.x];
  const float off = *ns.offset;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint4* Aq = reinterpret_cast<const uint4*>(A);
  for (long long base = (long long)blockIdx.x * 256 * P; base < nq; base += (long long)gridDim.x * 256 * P) {
    uint4 w[P];
    float am[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const long long d = min(base + 64LL * (P * wave + j) + lane, nq - 1);
      const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(Aq + d));
      w[j] = make_uint4(v[0], v[1], v[2], v[3]);
      const long long blk = (32 * d) >> bs_shift;
      am[j] = __fadd_rn(__fmul_rn(s_code2[ns.q8[blk]], ns.absmax2[blk >> ns.bs2_shift]), off);
    }
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const long long d = base + 64LL * (P * wave + j) + lane;
      if (d >= nq) continue;
      const uint32_t ww[4] = {w[j].x, w[j].y, w[j].z, w[j].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float2 p = s_pair[(ww[q] >> (8 * i)) & 0xFF];
          v[2 * i] = __fmul_rn(p.x, am[j]);
          v[2 * i + 1] = __fmul_rn(p.y, am[j]);
        }
        uint4 o;
        o.x = Pack2<T>::pk(v[0], v[1]); o.y = Pack2<T>::pk(v[2], v[3]);
        o.z = Pack2<T>::pk(v[4], v[5]); o.w = Pack2<T>::pk(v[6], v[7]);
        reinterpret_cast<uint4*>(out)[4 * d + q] = o;
      }
    }
  }
}
}  // namespace bnb
using namespace bnb;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
  const long long n = 4096LL * 11008;
  const int bs = 64, bs2 = 256;
  const long long nb = n / bs, nb2 = (nb + bs2 - 1) / bs2;
  uint8_t *A, *q8;
  float *code2, *a2, *off;
  bf16_t *o0, *o1;
  CK(hipMalloc(&A, n / 2)); CK(hipMalloc(&q8, nb)); CK(hipMalloc(&code2, 1024)); CK(hipMalloc(&a2, nb2 * 4));
  CK(hipMalloc(&off, 4)); CK(hipMalloc(&o0, n * 2)); CK(hipMalloc(&o1, n * 2));
  {
    std::vector<uint8_t> h(n / 2);
    uint32_t r = 1;
    for (auto& v : h) { r = r * 1664525u + 1013904223u; v = (uint8_t)(r >> 24); }
    CK(hipMemcpy(A, h.data(), n / 2, hipMemcpyHostToDevice));
    std::vector<uint8_t> hq(nb);
    for (auto& v : hq) { r = r * 1664525u + 1013904223u; v = (uint8_t)(r >> 24); }
    CK(hipMemcpy(q8, hq.data(), nb, hipMemcpyHostToDevice));
    std::vector<float> c(256), ha(nb2);
    for (int i = 0; i < 256; ++i) c[i] = -1.0f + 2.0f * i / 255.0f;
    for (auto& v : ha) { r = r * 1664525u + 1013904223u; v = 0.01f + (r >> 8) / 16777216.0f; }
    CK(hipMemcpy(code2, c.data(), 1024, hipMemcpyHostToDevice));
    CK(hipMemcpy(a2, ha.data(), nb2 * 4, hipMemcpyHostToDevice));
    const float fo = 0.02f;
    CK(hipMemcpy(off, &fo, 4, hipMemcpyHostToDevice));
  }
  const NestedStats ns{q8, code2, a2, off, __builtin_ctz(bs2)};
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto time = [&](const char* name, auto fn) {
    for (int i = 0; i < 5; ++i) fn();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 50; ++i) fn();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / 50, bytes = n / 2 + nb + nb2 * 4 + n * 2.0;
    printf("%-28s %8.2f us  %7.0f GB/s\n", name, us, bytes / us / 1e3);
    fflush(stdout);
  };
  auto check = [&]() {
    std::vector<uint16_t> a(n), b(n);
    CK(hipMemcpy(a.data(), o0, n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), o1, n * 2, hipMemcpyDeviceToHost));
    printf("  identical: %s\n", memcmp(a.data(), b.data(), n * 2) ? "NO" : "yes");
    CK(hipMemset(o1, 0, n * 2));
  };
  const long long ndw = n / 8, nq = n / 32;
  auto lib = [&](auto kern, int P, bf16_t* o) {
    return [=]() {
      const long long wgs = (ndw + 256LL * P - 1) / (256LL * P);
      hipLaunchKernelGGL(kern, dim3((int)std::min(wgs, 65536LL)), dim3(256), 0, 0, A, nullptr, o, __builtin_ctz(bs), ndw, ns);
    };
  };
  auto v16 = [&](auto kern, int P, int cap) {
    return [=]() {
      const long long wgs = (nq + 256LL * P - 1) / (256LL * P);
      hipLaunchKernelGGL(kern, dim3((int)std::min(wgs, (long long)cap)), dim3(256), 0, 0, A, o1, __builtin_ctz(bs), nq, ns);
    };
  };
  for (int rep = 0; rep < 2; ++rep) {
    time("stream P=8 (library)", lib(k_dequantize_4bit_stream<bf16_t, NF4, 8, true>, 8, o0));
    time("stream P=4", lib(k_dequantize_4bit_stream<bf16_t, NF4, 4, true>, 4, o1)); check();
    time("stream P=16", lib(k_dequantize_4bit_stream<bf16_t, NF4, 16, true>, 16, o1)); check();
    time("16B/lane P=2", v16(k_dq16<bf16_t, NF4, 2>, 2, 65536)); check();
    time("16B/lane P=4", v16(k_dq16<bf16_t, NF4, 4>, 4, 65536)); check();
    time("16B/lane P=2 grid 2048", v16(k_dq16<bf16_t, NF4, 2>, 2, 2048)); check();
  }
  return 0;
}
