// Lab (GPU): how fast does the chip start the waves of a one-shot streaming grid?  Each wave stamps s_memrealtime
// (10 ns ticks) at entry, then optionally streams `per_wave` 16-byte vectors per lane from a contiguous chunk and
// stamps again.  The stamps separate the dispatch ramp (entry times) from the memory ramp (landing times) for the
// grid shapes the few-token kernel uses (8 waves x 160 KiB LDS) and the alternatives (4 waves, smaller LDS).
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/launch_lab.hip -o tools/_launch_lab.so
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ unsigned long long lab_now() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__global__ __launch_bounds__(512, 1) void k_launch_lab(const uint4* __restrict__ src, int per_wave,
                                                       unsigned long long* __restrict__ stamps, uint4* sink) {
  unsigned long long t0 = lab_now();
  extern __shared__ uint4 lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long gw = (long long)blockIdx.x * (blockDim.x >> 6) + wave;
  unsigned hwid = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID, 32 bits
  uint4 acc = {0, 0, 0, 0};
  const uint4* p = src + gw * (long long)per_wave * 64 + lane;
  unsigned long long t1 = 0;
  if (per_wave > 0) {
    for (int i = 0; i < per_wave; i += 4) {
      typedef unsigned v4u __attribute__((ext_vector_type(4)));
      v4u v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = __builtin_nontemporal_load((const v4u*)(p + (long long)(i + j) * 64));
      if (i == 0) t1 = lab_now();
#pragma unroll
      for (int j = 0; j < 4; ++j) { acc.x ^= v[j].x; acc.y ^= v[j].y; acc.z ^= v[j].z; acc.w ^= v[j].w; }
    }
  }
  lds[threadIdx.x] = acc;
  __syncthreads();
  unsigned long long t2 = lab_now();
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = acc;
  if (lane == 0) {
    stamps[gw * 4 + 0] = t0;
    stamps[gw * 4 + 1] = t1;
    stamps[gw * 4 + 2] = t2;
    stamps[gw * 4 + 3] = hwid;
  }
}

// The few-token kernel's stream without its arithmetic: 48-row workgroups x 8 waves over a 2048-B-row weight, each wave
// 12 x 1 KiB instructions issued up front.  MODE bit 0: LDS-DMA (global_load_lds_dwordx4 nt) instead of register
// loads; bit 1: the few-token pattern (instruction = 8 rows x 128 B of the wave's k-eighth) instead of 1 KiB contiguous
// per instruction (wave = 12 KiB contiguous); bit 2: no nt hint.
template <int MODE>
__global__ __launch_bounds__(512, 1) void k_stream_lab(const uint8_t* __restrict__ src, int rows,
                                                       unsigned long long* __restrict__ stamps, uint4* sink) {
  unsigned long long t0 = lab_now();
  extern __shared__ uint4 lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long gw = (long long)blockIdx.x * 8 + wave;
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  v4u v[12];
  const uint8_t* ptr[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    if constexpr ((MODE & 16) != 0) {       // bit 4: 16 rows x 64 B per instruction (lane l: row l & 15, chunk l >> 4)
      const int gi = j / 6, pj = j % 6;
      const int row = min(48 * (int)blockIdx.x + 16 * (pj % 3) + (lane & 15), rows - 1);
      ptr[j] = src + (long long)row * 2048 + 128 * (2 * wave + gi) + 64 * (pj / 3) + 16 * (lane >> 4);
    } else if constexpr ((MODE & 2) != 0) {
      const int gi = j / 6, pj = j % 6;
      const int row = min(48 * (int)blockIdx.x + 8 * pj + (lane >> 3), rows - 1);
      ptr[j] = src + (long long)row * 2048 + 128 * (2 * wave + gi) + 16 * (lane & 7);
    } else {
      ptr[j] = src + gw * 12288 + 1024 * j + 16 * lane;
    }
  }
  v4u tok[8];
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    if constexpr ((MODE & 8) != 0) {       // bit 3: "token" loads, 4 x 1 KiB before each group's 6 pieces, from a
      if (j % 6 == 0) {                    // 64-KiB L2-resident matrix (wave w: its own 8-KiB k-eighth)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          tok[(j / 6) * 4 + q] = *(const v4u*)(src + (long long)rows * 2048 + 8192 * wave + 4096 * (j / 6) + 1024 * q + 16 * lane);
      }
    }
    if constexpr ((MODE & 1) != 0) {
      const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds + wave * 768 + 64 * j));
      unsigned keep;
      if constexpr ((MODE & 4) != 0)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(ptr[j]), "s"(dst) : "memory");
      else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(ptr[j]), "s"(dst) : "memory");
    } else if constexpr ((MODE & 4) != 0) {
      v[j] = *(const v4u*)ptr[j];
    } else {
      v[j] = __builtin_nontemporal_load((const v4u*)ptr[j]);
    }
  }
  const unsigned long long t1 = lab_now();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  v4u acc = {0, 0, 0, 0};
  if constexpr ((MODE & 1) != 0) {
#pragma unroll
    for (int j = 0; j < 12; ++j) acc ^= *(volatile v4u*)(lds + wave * 768 + 64 * j + lane);
  } else {
#pragma unroll
    for (int j = 0; j < 12; ++j) acc ^= v[j];
  }
  if constexpr ((MODE & 8) != 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) acc ^= tok[q];
  }
  const unsigned long long t2 = lab_now();
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = make_uint4(acc.x, acc.y, acc.z, acc.w);
  if (lane == 0) {
    stamps[gw * 4 + 0] = t0;
    stamps[gw * 4 + 1] = t1;
    stamps[gw * 4 + 2] = t2;
    stamps[gw * 4 + 3] = 0;
  }
}

extern "C" int stream_lab(const void* src, int rows, void* stamps, void* sink, int mode, void* stream) {
  const int blocks = (rows + 47) / 48;
  auto go = [&](auto kern) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(512), 160 * 1024, (hipStream_t)stream, (const uint8_t*)src, rows,
                       (unsigned long long*)stamps, (uint4*)sink);
  };
  switch (mode) {
    case 0: go(k_stream_lab<0>); break;
    case 1: go(k_stream_lab<1>); break;
    case 2: go(k_stream_lab<2>); break;
    case 3: go(k_stream_lab<3>); break;
    case 4: go(k_stream_lab<4>); break;
    case 5: go(k_stream_lab<5>); break;
    case 6: go(k_stream_lab<6>); break;
    case 7: go(k_stream_lab<7>); break;
    case 11: go(k_stream_lab<11>); break;
    case 16: go(k_stream_lab<16>); break;
    case 24: go(k_stream_lab<24>); break;
    case 17: go(k_stream_lab<17>); break;
    case 9: go(k_stream_lab<9>); break;
    case 10: go(k_stream_lab<10>); break;
    default: return 3;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int launch_lab(const void* src, int per_wave, void* stamps, void* sink, int blocks, int waves, int lds_bytes,
                          void* stream) {
  if (hipFuncSetAttribute((const void*)k_launch_lab, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
      hipSuccess)
    return 1;
  hipLaunchKernelGGL(k_launch_lab, dim3(blocks), dim3(64 * waves), lds_bytes, (hipStream_t)stream,
                     (const uint4*)src, per_wave, (unsigned long long*)stamps, (uint4*)sink);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
