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

// Ablations of k_gemv_4bit_dot (plain statistics): MODE bit 0 = no table fill, bit 1 = no table lookups (the
// packed dwords go straight into the dot), bit 2 = no activation DMA, bit 3 = no compute at all (xor-fold).
__device__ unsigned long long* g_tl;
__device__ __forceinline__ unsigned long long now() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
template <int R, int U, int MODE>
__global__ void __launch_bounds__(GV_THREADS)
k_ablate(int M, int K, const bf16_t* __restrict__ A, const uint8_t* __restrict__ B, const float* __restrict__ absmax,
         const float* __restrict__ datatype, bf16_t* __restrict__ out, int ldb) {
  extern __shared__ __attribute__((aligned(16))) uint8_t gsm[];
  uint8_t* table = gsm;
  uint8_t* xs = gsm + GV_TABLE_BYTES;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row0 = (blockIdx.x * (GV_THREADS / 64) + wave) * R;
  const int nch = K >> 5;
  const long long two_ldb = 2LL * ldb;
  unsigned long long ts[2 + 2 * U * R];
  if (MODE & 16) ts[0] = now();
  float dt[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) dt[j] = datatype[j];
  float am[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = min(lane + 64 * u, nch - 1);
#pragma unroll
    for (int r = 0; r < R; ++r) am[u][r] = absmax[(two_ldb * min(row0 + r, M - 1) + 32LL * c) >> 6];
  }
  const int nx = K >> 3;
  if (!(MODE & 4))
    for (int j = 0; j * GV_THREADS < nx; ++j) {
      const int idx = (j * (GV_THREADS / 64) + wave) * 64 + lane;
      if (idx < nx) glds16(A + 8 * idx, xs + (j * (GV_THREADS / 64) + wave) * 1024);
    }
  uintptr_t bp = (uintptr_t)B;
  asm volatile("" : "+s"(bp)::"memory");
  uint4 b[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = min(lane + 64 * u, nch - 1);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = min(row0 + r, M - 1);
      const u32x4_t v = __builtin_nontemporal_load((gvec_p)((gbyte_p)bp + (long long)row * ldb + 16LL * c));
      b[u][r] = make_uint4(v.x, v.y, v.z, v.w);
    }
  }
  if (!(MODE & 1)) {
    float lo = dt[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) lo = ((threadIdx.x >> 3) & 15) == j ? dt[j] : lo;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = threadIdx.x + k * GV_THREADS;
      const float hi = (threadIdx.x >> 7) ? dt[2 * k + 1] : dt[2 * k];
      const uint32_t v = Dot2<bf16_t>::pair(hi, lo);
      *reinterpret_cast<uint4*>(table + (i >> 3) * 128 + 16 * (i & 7)) = make_uint4(v, v, v, v);
    }
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R * U) : "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  if (MODE & 16) ts[1] = now();
  if (row0 >= M) return;
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0f;
  const uint32_t lane4 = (lane & 31) * 4;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = min(lane + 64 * u, nch - 1);
    uint32_t x[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(xs + 64 * c)[q];
      x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (MODE & 16) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U * R - 1 - (u * R + r)) : "memory");
        asm volatile("" : "+v"(b[u][r].x), "+v"(b[u][r].y), "+v"(b[u][r].z), "+v"(b[u][r].w));
        ts[2 + U * R + u * R + r] = now();
      }
      const uint32_t w[4] = {b[u][r].x, b[u][r].y, b[u][r].z, b[u][r].w};
      if (MODE & 8) { acc[r] += __uint_as_float((w[0] ^ w[1] ^ w[2] ^ w[3]) & 0x3fffffff); continue; }
      uint32_t l[16];
#pragma unroll
      for (int i = 0; i < 16; ++i)
        l[i] = (MODE & 2) ? w[i >> 2] : *reinterpret_cast<const uint32_t*>(table + ((((w[i >> 2] >> (8 * (i & 3))) & 0xFF) << 7) | lane4));
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        s0 = Dot2<bf16_t>::dot(x[i], l[i], s0);
        s1 = Dot2<bf16_t>::dot(x[i + 1], l[i + 1], s1);
      }
      acc[r] += (s0 + s1) * am[u][r];
      if (MODE & 16) { asm volatile("" : "+v"(acc[r])); ts[2 + u * R + r] = now(); }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (row0 + r < M) out[row0 + r] = Io<bf16_t>::from_f32(acc[r]);
  }
  if ((MODE & 16) && lane == 0) {
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    unsigned long long* o = g_tl + 32 * (blockIdx.x * 4 + wave);
    for (int i = 0; i < 2 + 2 * U * R; ++i) o[i] = ts[i];
    o[30] = hw;
    o[31] = xcc;
  }
}

// Perm-addressed table: entry e of copy j at byte 256*e + 4*j (32 copies, 64 KiB span), so the LDS address of
// byte k of a packed dword w is one v_perm_b32 of {w, lane4}: byte0 = 4*(lane&31), byte1 = byte k of w.
// Activations by LDS-DMA at 64 KiB.  LATE: absmax loads go out after the weights and scale the raw chunk sums
// at the end (same fp32 order as k_gemv_4bit_dot: acc[r] += part[u][r] * am[u][r], u ascending).
constexpr int PT_BYTES = 65536;
template <int R, int U, bool LATE>
__global__ void __launch_bounds__(GV_THREADS)
k_perm(int M, int K, const bf16_t* __restrict__ A, const uint8_t* __restrict__ B, const float* __restrict__ absmax,
       const float* __restrict__ datatype, bf16_t* __restrict__ out, int ldb) {
  extern __shared__ __attribute__((aligned(16))) uint8_t gsm[];
  uint8_t* table = gsm;
  uint8_t* xs = gsm + PT_BYTES;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row0 = (blockIdx.x * (GV_THREADS / 64) + wave) * R;
  const int nch = K >> 5;
  const long long two_ldb = 2LL * ldb;
  float dt[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) dt[j] = datatype[j];
  float am[U][R];
  if (!LATE) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = min(lane + 64 * u, nch - 1);
#pragma unroll
      for (int r = 0; r < R; ++r) am[u][r] = absmax[(two_ldb * min(row0 + r, M - 1) + 32LL * c) >> 6];
    }
  }
  const int nx = K >> 3;
  for (int j = 0; j * GV_THREADS < nx; ++j) {
    const int idx = (j * (GV_THREADS / 64) + wave) * 64 + lane;
    if (idx < nx) glds16(A + 8 * idx, xs + (j * (GV_THREADS / 64) + wave) * 1024);
  }
  uintptr_t bp = (uintptr_t)B;
  asm volatile("" : "+s"(bp)::"memory");
  uint4 b[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = min(lane + 64 * u, nch - 1);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = min(row0 + r, M - 1);
      const u32x4_t v = __builtin_nontemporal_load((gvec_p)((gbyte_p)bp + (long long)row * ldb + 16LL * c));
      b[u][r] = make_uint4(v.x, v.y, v.z, v.w);
    }
  }
  if (LATE) {
    uintptr_t ap = (uintptr_t)absmax;
    asm volatile("" : "+s"(ap)::"memory");
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = min(lane + 64 * u, nch - 1);
#pragma unroll
      for (int r = 0; r < R; ++r) am[u][r] = ((const float*)ap)[(two_ldb * min(row0 + r, M - 1) + 32LL * c) >> 6];
    }
  }
  {   // thread t fills entry t: 32 copies of pair(code[t >> 4], code[t & 15]), 16-B stores rotated by t
    const int t = threadIdx.x;
    float hi = dt[0], lo = dt[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) { hi = (t >> 4) == j ? dt[j] : hi; lo = (t & 15) == j ? dt[j] : lo; }
    const uint32_t v = Dot2<bf16_t>::pair(hi, lo);
#pragma unroll
    for (int k = 0; k < 8; ++k) *reinterpret_cast<uint4*>(table + 256 * t + 16 * ((k + t) & 7)) = make_uint4(v, v, v, v);
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LATE ? 2 * R * U : R * U) : "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  if (row0 >= M) return;
  float part[U][R];
  const uint32_t lane4 = (lane & 31) * 4;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = min(lane + 64 * u, nch - 1);
    uint32_t x[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(xs + 64 * c)[q];
      x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t w[4] = {b[u][r].x, b[u][r].y, b[u][r].z, b[u][r].w};
      uint32_t l[16];
#pragma unroll
      for (int i = 0; i < 16; ++i)
        l[i] = *reinterpret_cast<const uint32_t*>(table + __builtin_amdgcn_perm(w[i >> 2], lane4, 0x0C0C0000u | ((4u + (i & 3)) << 8)));
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        s0 = Dot2<bf16_t>::dot(x[i], l[i], s0);
        s1 = Dot2<bf16_t>::dot(x[i + 1], l[i + 1], s1);
      }
      part[u][r] = (s0 + s1);
    }
  }
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    acc[r] = 0.0f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool valid = lane + 64 * u < nch;
      const float p = part[u][r] * am[u][r];
      acc[r] += valid ? p : 0.0f;
    }
    acc[r] = wave_sum(acc[r]);
  }
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (row0 + r < M) out[row0 + r] = Io<bf16_t>::from_f32(acc[r]);
  }
}

// One workgroup per CU with the perm-addressed table (64 KiB) + activations at 64 KiB; NW waves, rows
// r0 + w + NW*j (j < R) of the balanced range [g*M/G, (g+1)*M/G), clamped; chunks lane + 64u (u < U).
template <int R, int U, int NW, bool TL = false>
__global__ void __launch_bounds__(NW * 64, 1)
k_cuperm(int M, int K, const bf16_t* __restrict__ A, const uint8_t* __restrict__ B, const float* __restrict__ absmax,
         const float* __restrict__ datatype, bf16_t* __restrict__ out, int ldb, int G) {
  extern __shared__ __attribute__((aligned(16))) uint8_t gsm[];
  uint8_t* table = gsm;
  uint8_t* xs = gsm + PT_BYTES;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r0 = (int)((long long)blockIdx.x * M / G), r1 = (int)((long long)(blockIdx.x + 1) * M / G);
  const int nch = K >> 5;
  const long long two_ldb = 2LL * ldb;
  unsigned long long ts[2 + 2 * R * U];
  if (TL) ts[0] = now();
  auto row_of = [&](int j) { return min(r0 + wave + NW * j, r1 - 1); };
  auto chunk_of = [&](int u) { return min(lane + 64 * u, nch - 1); };
  float dt[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) dt[j] = datatype[j];
  float am[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < R; ++j) am[u][j] = absmax[(two_ldb * row_of(j) + 32LL * chunk_of(u)) >> 6];
  const int nx = K >> 3;
  for (int p = wave; p * 64 < nx; p += NW) {
    const int idx = p * 64 + lane;
    if (idx < nx) glds16(A + 8 * idx, xs + p * 1024);
  }
  uintptr_t bp = (uintptr_t)B;
  asm volatile("" : "+s"(bp)::"memory");
  uint4 b[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const u32x4_t v = __builtin_nontemporal_load((gvec_p)((gbyte_p)bp + (long long)row_of(j) * ldb + 16LL * chunk_of(u)));
      b[u][j] = make_uint4(v.x, v.y, v.z, v.w);
    }
  if (threadIdx.x < 256) {
    const int t = threadIdx.x;
    float hi = dt[0], lo = dt[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) { hi = (t >> 4) == j ? dt[j] : hi; lo = (t & 15) == j ? dt[j] : lo; }
    const uint32_t v = Dot2<bf16_t>::pair(hi, lo);
#pragma unroll
    for (int k = 0; k < 8; ++k) *reinterpret_cast<uint4*>(table + 256 * t + 16 * ((k + t) & 7)) = make_uint4(v, v, v, v);
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R * U) : "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  if (TL) ts[1] = now();
  float acc[R];
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = 0.0f;
  const uint32_t lane4 = (lane & 31) * 4;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool valid = lane + 64 * u < nch;
    const int c = chunk_of(u);
    uint32_t x[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(xs + 64 * c)[q];
      x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (TL) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U * R - 1 - (u * R + j)) : "memory");
        asm volatile("" : "+v"(b[u][j].x), "+v"(b[u][j].y), "+v"(b[u][j].z), "+v"(b[u][j].w));
        ts[2 + U * R + u * R + j] = now();
      }
      const uint32_t w[4] = {b[u][j].x, b[u][j].y, b[u][j].z, b[u][j].w};
      uint32_t l[16];
#pragma unroll
      for (int i = 0; i < 16; ++i)
        l[i] = *reinterpret_cast<const uint32_t*>(table + __builtin_amdgcn_perm(w[i >> 2], lane4, 0x0C0C0000u | ((4u + (i & 3)) << 8)));
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        s0 = Dot2<bf16_t>::dot(x[i], l[i], s0);
        s1 = Dot2<bf16_t>::dot(x[i + 1], l[i + 1], s1);
      }
      const float part = (s0 + s1) * am[u][j];
      acc[j] += valid ? part : 0.0f;
      if (TL) { asm volatile("" : "+v"(acc[j])); ts[2 + u * R + j] = now(); }
    }
  }
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = wave_sum(acc[j]);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int row = r0 + wave + NW * j;
      if (row < r1) out[row] = Io<bf16_t>::from_f32(acc[j]);
    }
  }
  if (TL && lane == 0) {
    unsigned long long* o = g_tl + 32 * (blockIdx.x * NW + wave);
    for (int i = 0; i < 2 + 2 * U * R; ++i) o[i] = ts[i];
  }
}

// Flexible variant: PERM (perm-addressed 64 KiB table) / SWZ (activation chunks swizzled so the ds_read_b128
// of chunk c = lane + 64u is bank-conflict-free: piece q of chunk c at 64c + 16((q + (c >> 2)) & 3)) /
// PREBAR (statistics and activations are issued by every wave, then a barrier, then the weights, so a CU's
// queue holds all of them ahead of any weight request) / CU (balanced row range per workgroup).
template <int R, int U, int NW, bool PERM, bool SWZ, bool PREBAR, bool CU, bool XREG = false, bool TL = false>
__global__ void __launch_bounds__(NW * 64)
k_gv(int M, int K, const bf16_t* __restrict__ A, const uint8_t* __restrict__ B, const float* __restrict__ absmax,
     const float* __restrict__ datatype, bf16_t* __restrict__ out, int ldb, int G) {
  extern __shared__ __attribute__((aligned(16))) uint8_t gsm[];
  constexpr int TB = PERM ? PT_BYTES : GV_TABLE_BYTES;
  uint8_t* table = gsm;
  uint8_t* xs = gsm + TB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int r0, r1;
  if (CU) { r0 = (int)((long long)blockIdx.x * M / G); r1 = (int)((long long)(blockIdx.x + 1) * M / G); }
  else { r0 = (blockIdx.x * NW + wave) * R; r1 = min(r0 + R, M); }
  const int nch = K >> 5;
  const long long two_ldb = 2LL * ldb;
  unsigned long long ts[2 + 2 * R * U];
  if (TL) ts[0] = now();
  auto row_of = [&](int j) { return CU ? min(r0 + wave + NW * j, r1 - 1) : min(r0 + j, M - 1); };
  auto row_real = [&](int j) { return CU ? r0 + wave + NW * j : r0 + j; };
  auto chunk_of = [&](int u) { return min(lane + 64 * u, nch - 1); };
  float dt[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) dt[j] = datatype[j];
  uint4 xr[U][4];
  if (XREG) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) xr[u][q] = reinterpret_cast<const uint4*>(A + 32 * chunk_of(u))[q];
  }
  float am[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < R; ++j) am[u][j] = absmax[(two_ldb * row_of(j) + 32LL * chunk_of(u)) >> 6];
  const int nx = K >> 3;
  for (int p = wave; !XREG && p * 64 < nx; p += NW) {
    const int i = p * 64 + lane;                         // LDS slot (16 B)
    int src = i;
    if (SWZ) { const int c = i >> 2; src = 4 * c + (((i & 3) - (c >> 2)) & 3); }
    if (i < nx) glds16(A + 8 * src, xs + p * 1024);
  }
  if (PREBAR) __builtin_amdgcn_s_barrier();
  uintptr_t bp = (uintptr_t)B;
  asm volatile("" : "+s"(bp)::"memory");
  uint4 b[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const u32x4_t v = __builtin_nontemporal_load((gvec_p)((gbyte_p)bp + (long long)row_of(j) * ldb + 16LL * chunk_of(u)));
      b[u][j] = make_uint4(v.x, v.y, v.z, v.w);
    }
  if (PERM) {
    for (int t = threadIdx.x; t < 256; t += NW * 64) {
      float hi = dt[0], lo = dt[0];
#pragma unroll
      for (int j = 1; j < 16; ++j) { hi = (t >> 4) == j ? dt[j] : hi; lo = (t & 15) == j ? dt[j] : lo; }
      const uint32_t v = Dot2<bf16_t>::pair(hi, lo);
#pragma unroll
      for (int k = 0; k < 8; ++k) *reinterpret_cast<uint4*>(table + 256 * t + 16 * ((k + t) & 7)) = make_uint4(v, v, v, v);
    }
  } else {
    for (int i = threadIdx.x; i < 2048; i += NW * 64) {
      const int e = i >> 3;
      float hi = dt[0], lo = dt[0];
#pragma unroll
      for (int j = 1; j < 16; ++j) { hi = (e >> 4) == j ? dt[j] : hi; lo = (e & 15) == j ? dt[j] : lo; }
      const uint32_t v = Dot2<bf16_t>::pair(hi, lo);
      *reinterpret_cast<uint4*>(table + e * 128 + 16 * (i & 7)) = make_uint4(v, v, v, v);
    }
  }
  if (!XREG) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R * U) : "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (TL) ts[1] = now();
  if (!CU && r0 >= M) return;
  float acc[R];
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = 0.0f;
  const uint32_t lane4 = (lane & 31) * 4;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool valid = lane + 64 * u < nch;
    const int c = chunk_of(u);
    uint32_t x[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int slot = SWZ ? ((q + (c >> 2)) & 3) : q;
      const uint4 v = XREG ? xr[u][q] : reinterpret_cast<const uint4*>(xs + 64 * c)[slot];
      x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (TL) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U * R - 1 - (u * R + j)) : "memory");
        asm volatile("" : "+v"(b[u][j].x), "+v"(b[u][j].y), "+v"(b[u][j].z), "+v"(b[u][j].w));
        ts[2 + U * R + u * R + j] = now();
      }
      const uint32_t w[4] = {b[u][j].x, b[u][j].y, b[u][j].z, b[u][j].w};
      uint32_t l[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t a = PERM ? __builtin_amdgcn_perm(w[i >> 2], lane4, 0x0C0C0000u | ((4u + (i & 3)) << 8))
                                : ((((w[i >> 2] >> (8 * (i & 3))) & 0xFF) << 7) | lane4);
        l[i] = *reinterpret_cast<const uint32_t*>(table + a);
      }
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        s0 = Dot2<bf16_t>::dot(x[i], l[i], s0);
        s1 = Dot2<bf16_t>::dot(x[i + 1], l[i + 1], s1);
      }
      const float part = (s0 + s1) * am[u][j];
      acc[j] += valid ? part : 0.0f;
      if (TL) { asm volatile("" : "+v"(acc[j])); ts[2 + u * R + j] = now(); }
    }
  }
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = wave_sum(acc[j]);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int row = row_real(j);
      if (row < r1) out[row] = Io<bf16_t>::from_f32(acc[j]);
    }
  }
  if (TL && lane == 0) {
    unsigned long long* o = g_tl + 32 * (blockIdx.x * NW + wave);
    for (int i = 0; i < 2 + 2 * U * R; ++i) o[i] = ts[i];
  }
}

// Weights first, then activations (registers) and statistics: every table lookup proceeds as its weights land
// (the in-order counter never makes a lookup wait for the activations), the dots follow once x is in.
template <int R, int U, int NW>
__global__ void __launch_bounds__(NW * 64)
k_latex(int M, int K, const bf16_t* __restrict__ A, const uint8_t* __restrict__ B, const float* __restrict__ absmax,
        const float* __restrict__ datatype, bf16_t* __restrict__ out, int ldb, int G) {
  extern __shared__ __attribute__((aligned(16))) uint8_t gsm[];
  uint8_t* table = gsm;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r0 = (int)((long long)blockIdx.x * M / G), r1 = (int)((long long)(blockIdx.x + 1) * M / G);
  const int nch = K >> 5;
  const long long two_ldb = 2LL * ldb;
  auto row_of = [&](int j) { return min(r0 + wave + NW * j, r1 - 1); };
  auto chunk_of = [&](int u) { return min(lane + 64 * u, nch - 1); };
  float dt[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) dt[j] = datatype[j];
  uint4 b[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const u32x4_t v = __builtin_nontemporal_load((gvec_p)((gbyte_p)B + (long long)row_of(j) * ldb + 16LL * chunk_of(u)));
      b[u][j] = make_uint4(v.x, v.y, v.z, v.w);
    }
  uint4 xr[U][4];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int q = 0; q < 4; ++q) xr[u][q] = reinterpret_cast<const uint4*>(A + 32 * chunk_of(u))[q];
  float am[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < R; ++j) am[u][j] = absmax[(two_ldb * row_of(j) + 32LL * chunk_of(u)) >> 6];
  for (int t = threadIdx.x; t < 256; t += NW * 64) {
    float hi = dt[0], lo = dt[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) { hi = (t >> 4) == j ? dt[j] : hi; lo = (t & 15) == j ? dt[j] : lo; }
    const uint32_t v = Dot2<bf16_t>::pair(hi, lo);
#pragma unroll
    for (int k = 0; k < 8; ++k) *reinterpret_cast<uint4*>(table + 256 * t + 16 * ((k + t) & 7)) = make_uint4(v, v, v, v);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  const uint32_t lane4 = (lane & 31) * 4;
  uint32_t l[U][R][16];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t w[4] = {b[u][j].x, b[u][j].y, b[u][j].z, b[u][j].w};
#pragma unroll
      for (int i = 0; i < 16; ++i)
        l[u][j][i] = *reinterpret_cast<const uint32_t*>(table + __builtin_amdgcn_perm(w[i >> 2], lane4, 0x0C0C0000u | ((4u + (i & 3)) << 8)));
    }
  float acc[R];
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = 0.0f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool valid = lane + 64 * u < nch;
    const uint32_t x[16] = {xr[u][0].x, xr[u][0].y, xr[u][0].z, xr[u][0].w, xr[u][1].x, xr[u][1].y, xr[u][1].z, xr[u][1].w,
                            xr[u][2].x, xr[u][2].y, xr[u][2].z, xr[u][2].w, xr[u][3].x, xr[u][3].y, xr[u][3].z, xr[u][3].w};
#pragma unroll
    for (int j = 0; j < R; ++j) {
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        s0 = Dot2<bf16_t>::dot(x[i], l[u][j][i], s0);
        s1 = Dot2<bf16_t>::dot(x[i + 1], l[u][j][i + 1], s1);
      }
      const float part = (s0 + s1) * am[u][j];
      acc[j] += valid ? part : 0.0f;
    }
  }
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = wave_sum(acc[j]);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int row = r0 + wave + NW * j;
      if (row < r1) out[row] = Io<bf16_t>::from_f32(acc[j]);
    }
  }
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
  auto ablate = [&](auto kern, int R) {
    return [=](int c) {
      const int waves = (M + R - 1) / R;
      hipLaunchKernelGGL(kern, dim3((waves + 3) / 4), dim3(GV_THREADS), GV_TABLE_BYTES + 2 * K, 0, M, K, x, W[c], AM[c],
                         code, y, K / 2);
    };
  };
  vs.push_back({"ablate R4U2 full", ablate(k_ablate<4, 2, 0>, 4), {}});
  vs.push_back({"ablate R4U2 no table fill", ablate(k_ablate<4, 2, 1>, 4), {}});
  vs.push_back({"ablate R4U2 no lookups", ablate(k_ablate<4, 2, 2>, 4), {}});
  vs.push_back({"ablate R4U2 no x DMA", ablate(k_ablate<4, 2, 4>, 4), {}});
  vs.push_back({"ablate R4U2 fill+x only", ablate(k_ablate<4, 2, 8>, 4), {}});
  vs.push_back({"ablate R4U2 loads only", ablate(k_ablate<4, 2, 13>, 4), {}});
  vs.push_back({"ablate R2U2 full", ablate(k_ablate<2, 2, 0>, 2), {}});
  vs.push_back({"ablate R2U2 loads only", ablate(k_ablate<2, 2, 13>, 2), {}});
  vs.push_back({"ablate R1U2 full", ablate(k_ablate<1, 2, 0>, 1), {}});
  vs.push_back({"ablate R8U2 full", ablate(k_ablate<8, 2, 0>, 8), {}});
  auto permk = [&](auto kern, int R) {
    return [=](int c) {
      const int waves = (M + R - 1) / R;
      hipLaunchKernelGGL(kern, dim3((waves + 3) / 4), dim3(GV_THREADS), PT_BYTES + 2 * K, 0, M, K, x, W[c], AM[c],
                         code, y, K / 2);
    };
  };
  {   // bit-exactness of the perm kernels against the library GEMV on copy 0
    std::vector<uint16_t> ref(M), got(M);
    vs[4].fn(0);
    CK(hipMemcpy(ref.data(), y, M * 2, hipMemcpyDeviceToHost));
    const std::pair<const char*, std::function<void(int)>> checks[] = {
        {"perm R4", permk(k_perm<4, 2, false>, 4)}, {"perm R6 late", permk(k_perm<6, 2, true>, 6)},
        {"perm R8", permk(k_perm<8, 2, false>, 8)}};
    for (auto& ck : checks) {
      CK(hipMemset(y, 0xFF, M * 2));
      ck.second(0);
      CK(hipMemcpy(got.data(), y, M * 2, hipMemcpyDeviceToHost));
      printf("%s bit-identical: %s\n", ck.first, memcmp(ref.data(), got.data(), M * 2) ? "NO" : "yes");
    }
  }
  vs.push_back({"perm R4U2", permk(k_perm<4, 2, false>, 4), {}});
  vs.push_back({"perm R4U2 late", permk(k_perm<4, 2, true>, 4), {}});
  vs.push_back({"perm R6U2", permk(k_perm<6, 2, false>, 6), {}});
  vs.push_back({"perm R6U2 late", permk(k_perm<6, 2, true>, 6), {}});
  vs.push_back({"perm R8U2", permk(k_perm<8, 2, false>, 8), {}});
  vs.push_back({"perm R8U2 late", permk(k_perm<8, 2, true>, 8), {}});
  auto cuperm = [&](auto kern, int NW, int G) {
    return [=](int c) {
      hipLaunchKernelGGL(kern, dim3(G), dim3(NW * 64), PT_BYTES + 2 * K, 0, M, K, x, W[c], AM[c], code, y, K / 2, G);
    };
  };
  {
    std::vector<uint16_t> ref(M), got(M);
    vs[4].fn(0);
    CK(hipMemcpy(ref.data(), y, M * 2, hipMemcpyDeviceToHost));
    const std::pair<const char*, std::function<void(int)>> checks[] = {
        {"cuperm 12w", cuperm(k_cuperm<4, 2, 12>, 12, 256)}, {"cuperm 16w", cuperm(k_cuperm<3, 2, 16>, 16, 256)},
        {"cuperm 8w", cuperm(k_cuperm<6, 2, 8>, 8, 256)}};
    for (auto& ck : checks) {
      CK(hipMemset(y, 0xFF, M * 2));
      ck.second(0);
      CK(hipMemcpy(got.data(), y, M * 2, hipMemcpyDeviceToHost));
      printf("%s bit-identical: %s\n", ck.first, memcmp(ref.data(), got.data(), M * 2) ? "NO" : "yes");
    }
  }
  vs.push_back({"cuperm 12 waves R4", cuperm(k_cuperm<4, 2, 12>, 12, 256), {}});
  vs.push_back({"cuperm 16 waves R3", cuperm(k_cuperm<3, 2, 16>, 16, 256), {}});
  vs.push_back({"cuperm 8 waves R6", cuperm(k_cuperm<6, 2, 8>, 8, 256), {}});
  vs.push_back({"cuperm 12 waves R2 G512", cuperm(k_cuperm<2, 2, 12>, 12, 512), {}});
  vs.push_back({"cuperm 8 waves R3 G512", cuperm(k_cuperm<3, 2, 8>, 8, 512), {}});
  std::vector<std::pair<const char*, std::function<void(int)>>> gvs;
#define GVX(NAME, R, U, NW, P, S, PB, CUM, G, XR)                                                                     \
  gvs.push_back({NAME, [&](int c) {                                                                                 \
    const int g = CUM ? (G) : (M + (NW) * (R) - 1) / ((NW) * (R));                                                  \
    hipLaunchKernelGGL((k_gv<R, U, NW, P, S, PB, CUM, XR>), dim3(g), dim3((NW) * 64), (P ? PT_BYTES : GV_TABLE_BYTES) + (XR ? 0 : 2 * K), 0, \
                       M, K, x, W[c], AM[c], code, y, K / 2, g);                                                    \
  }});
#define GV(NAME, R, U, NW, P, S, PB, CUM, G) GVX(NAME, R, U, NW, P, S, PB, CUM, G, false)
  GV("gv cuperm12 R2 swz prebar G512", 2, 2, 12, true, true, true, true, 512)
  GV("gv cuperm11 R2 swz prebar G512", 2, 2, 11, true, true, true, true, 512)
  GV("gv cuperm6 R4 swz prebar G512", 4, 2, 6, true, true, true, true, 512)
#define LX(NAME, R, U, NW, G)                                                                                     \
  gvs.push_back({NAME, [&](int c) {                                                                             \
    hipLaunchKernelGGL((k_latex<R, U, NW>), dim3(G), dim3((NW) * 64), PT_BYTES, 0, M, K, x, W[c], AM[c], code, y, K / 2, G); \
  }});
  LX("latex NW12 R2 G512", 2, 2, 12, 512)
  LX("latex NW8 R3 G512", 3, 2, 8, 512)
  LX("latex NW6 R4 G512", 4, 2, 6, 512)
  LX("latex NW11 R2 G512", 2, 2, 11, 512)
  {
    std::vector<uint16_t> ref(M), got(M);
    vs[4].fn(0);
    CK(hipMemcpy(ref.data(), y, M * 2, hipMemcpyDeviceToHost));
    for (auto& ck : gvs) {
      CK(hipMemset(y, 0xFF, M * 2));
      ck.second(0);
      CK(hipMemcpy(got.data(), y, M * 2, hipMemcpyDeviceToHost));
      printf("%s bit-identical: %s\n", ck.first, memcmp(ref.data(), got.data(), M * 2) ? "NO" : "yes");
      vs.push_back({ck.first, ck.second, {}});
    }
  }
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
  {   // one timeline launch of the full kernel in the middle of a back-to-back stream
    const int waves = (M + 3) / 4, nwg = (waves + 3) / 4;
    unsigned long long* tl;
    CK(hipMalloc(&tl, (size_t)8192 * 32 * 8));
    CK(hipMemset(tl, 0, (size_t)8192 * 32 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_tl), &tl, sizeof(tl)));
    auto full = ablate(k_ablate<4, 2, 0>, 4);
    for (int rep = 0; rep < 3; ++rep) {
      for (int i = 0; i < 14; ++i) full(i);
      if (getenv("TL_GV"))
        hipLaunchKernelGGL((k_gv<2, 2, 12, true, true, true, true, false, true>), dim3(512), dim3(768), PT_BYTES + 2 * K, 0, M, K, x, W[0], AM[0], code, y, K / 2, 512);
      else if (getenv("TL_CUPERM"))
        hipLaunchKernelGGL((k_cuperm<4, 2, 12, true>), dim3(256), dim3(768), PT_BYTES + 2 * K, 0, M, K, x, W[0], AM[0], code, y, K / 2, 256);
      else
      hipLaunchKernelGGL((k_ablate<4, 2, 16>), dim3(nwg), dim3(GV_THREADS), GV_TABLE_BYTES + 2 * K, 0, M, K, x, W[0], AM[0], code, y, K / 2);
      for (int i = 1; i < 4; ++i) full(i);
      CK(hipDeviceSynchronize());
    }
    std::vector<unsigned long long> h((size_t)8192 * 32);
    CK(hipMemcpy(h.data(), tl, h.size() * 8, hipMemcpyDeviceToHost));
    FILE* f = fopen("gpurun_out/gemv_timeline.bin", "wb");
    if (f) { fwrite(h.data(), 8, h.size(), f); fclose(f); }
  }
  const double bytes = (double)(wbytes + nabs * 4);
  for (auto& v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double med = v.us[v.us.size() / 2];
    printf("%-28s median %6.2f us  %6.0f GB/s  (min %6.2f)\n", v.name, med, bytes / med / 1e3, v.us.front());
  }
  return 0;
}
