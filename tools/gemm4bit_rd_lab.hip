// DESIGN LAB (not built into the library): 256 x 256-tile fused 4-bit weight GEMM with the weights
// dequantised straight into MFMA B operands (register dequant).  Round-1 result at 4096x4096x11008
// (tools/gemm_lab2.hip, warm clocks): 343-352 us against 346-350 us for the LDS-dequant kernel in
// csrc/gemm4bit_256.hip -- a tie.  PMC: 8 % more wave-cycles (LDS command-FIFO-full issue stalls from
// 8 A-fragment reads per 8 MFMAs) at a ~8 % higher clock (far fewer LDS bank conflicts); the chip is
// power/clock-limited at this point, so the library keeps gemm4bit_256.hip.  Semantics and ABI: gemm4bit.hip (ref:sycl/pythonInterface.cpp:377-378,
// the M>1 slot of kernel_gemm.cpp:1015 / dequantize_4bit + F.linear, autograd/_functions.py:507).
//
// Geometry: 512 threads = 8 waves side by side along the out-features: wave w owns output columns
// n0 + 32w .. +31 for all 256 token rows (8 x v_mfma_f32_32x32x16 accumulators, 128 VGPRs).
// Because no two waves share a weight column, every packed weight byte is dequantised exactly once
// per workgroup, and it is dequantised in the lane that feeds it to the MFMA:
//   * lane (c, h) = (lane & 31, lane >> 5) loads 16 packed bytes of weight row n0 + 32w + c per k-step
//     (one global_load_dwordx4; bytes 16h .. 16h+15 of the row's 32-byte k-step chunk) and the
//     row's absmax for that k-step (bs >= 64, so one value per k-step);
//   * sub-step ks uses dword ks of those bytes: elements k = 32h + 8ks .. +7 of the k-step, i.e.
//     exactly the 8 k of a 32x32x16 B operand; the A operand of the same lane reads the same k
//     (16-B slot 4h + ks of the activation row).
// Each packed byte goes through a 256-entry {code[hi], code[lo]} pair table, two fp32 multiplies
// by absmax and one RNE cast: the reference's dequantised values (kernel_quant.cpp:1428-1453).
// The table has 32 bank-private copies (entry e of copy j at byte 256e + 8j, lane uses copy
// lane & 31), so the ds_read_b64 lookups never conflict, and its address is one v_perm_b32:
// byte 1 = the packed byte, byte 0 = 8 * (lane & 31).
//
// LDS (128 KiB, one workgroup per CU): [0, 64K) the pair table, [64K, 128K) two 32-KiB activation
// stages [256 rows][128 B] filled by LDS-DMA, 16-B slots XOR-swizzled by (row >> 1) & 7 on the
// source address (conflict-free 32-row fragment reads).  The epilogue reuses all 128 KiB.
#include "gemm_common.hpp"

namespace bnb {

constexpr int R_BM = 256, R_BN = 256, R_BK = 64, R_THREADS = 512;
constexpr int R_LUT = 256 * 32 * 8;             // 64 KiB
constexpr int R_XT = R_BM * R_BK * 2;           // 32 KiB per stage
constexpr int R_WT = R_BN * R_BK / 2;           // 8 KiB packed weights per stage
constexpr int R_AT = 8 * 256;                   // 2 KiB absmax per stage (one 256-B piece per wave)
constexpr int R_OFF_X = R_LUT;
constexpr int R_OFF_W = R_OFF_X + 2 * R_XT;     // 3 weight stages
constexpr int R_OFF_AM = R_OFF_W + 3 * R_WT;    // 3 absmax stages
constexpr int R_LDS = R_OFF_AM + 3 * R_AT;      // 161,792 B

typedef float f32x2r_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2r_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int rd_swz(int r, int s) { return r * 128 + ((s ^ ((r >> 1) & 7)) << 4); }

// scalar v_mul_f32: hipcc would otherwise SLP-pack pairs into v_pk_mul_f32, which costs ~4x the
// issue slots beside MFMAs on gfx950 (MI355X_MICROARCH.md, price of one filler)
__device__ __forceinline__ float rd_mul(float a, float b) {
  float r;
  asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

template <typename T> __device__ __forceinline__ uint32_t rd_cvt2(float lo, float hi);
template <> __device__ __forceinline__ uint32_t rd_cvt2<bf16_t>(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2r_t){lo, hi}, bf16x2r_t));
}
template <> __device__ __forceinline__ uint32_t rd_cvt2<fp16_t>(float lo, float hi) {
  return Mfma<fp16_t>::pack2(lo, hi);
}

// FL (design lab only; 0 in the library): 1 = no activation DMA in the k-loop, 2 = no dequant,
// 4 = s_setprio(1) around the MFMA groups, 8 = plain C++ multiplies (build with -fno-slp-vectorize),
// 16 = one LDS read after every MFMA instead of bursts
template <typename T, int FL = 0>
__global__ void __launch_bounds__(R_THREADS, 1)
k_gemm_4bit_rd(int N, int M, int K, const T* __restrict__ A, const uint8_t* __restrict__ B,
               const float* __restrict__ absmax, const float* __restrict__ datatype, T* __restrict__ out,
               int lda, int ldb, int ldc, int blocksize) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[R_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 31, h = lane >> 5;

  // ---- pair table: thread (j = tid & 31, hi = tid >> 5) writes entries 16hi .. 16hi+15 of copy j
  {
    const int j = tid & 31, hi = tid >> 5;
    const float vhi = datatype[hi];
    float2* dst = reinterpret_cast<float2*>(smem + 256 * 16 * hi + 8 * j);
#pragma unroll
    for (int lo = 0; lo < 16; ++lo) dst[32 * lo] = make_float2(vhi, datatype[lo]);
  }

  // ---- tile order: XCD-contiguous ids, grouped 4 token-tiles x all feature-tiles
  const int tilesN = (N + R_BN - 1) / R_BN, tilesM = (M + R_BM - 1) / R_BM;
  const int wg = xcd_remap(blockIdx.x, tilesN * tilesM);
  constexpr int GROUP = 4;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * R_BM, n0 = tn * R_BN;

  // ---- activation DMA: wave-instruction i of wave w fills rows 8(4w+i) .. +7 (1 KiB, lane-linear)
  const T* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wave + i) + (lane >> 3);
    xsrc[i] = A + (long long)min(m0 + row, M - 1) * lda + 8 * ((lane & 7) ^ ((row >> 1) & 7));
  }
  // ---- weight DMA: wave w fills its own 32 rows (one 1-KiB piece: lane l -> row l >> 1, half l & 1)
  // and their absmax (one dword piece: lane l -> row l & 31; lanes 32-63 repeat, branch-free)
  const uint8_t* wsrc = B + (long long)min(n0 + 32 * wave + (lane >> 1), N - 1) * ldb + 16 * (lane & 1);
  const long long abase = 2LL * ldb * min(n0 + 32 * wave + c, N - 1);   // element index of (row, k = 0)
  const int bs_shift = __builtin_ctz(blocksize);                          // blocksize: power of two >= 64
  const uint32_t lanebase = 8u * c;
  const int nk = K / R_BK;

  auto dma_w = [&](int kt) {
    const int st = kt % 3;
    glds16(wsrc + (long long)kt * (R_BK / 2), smem + R_OFF_W + st * R_WT + wave * 1024);
    glds4(absmax + ((abase + (long long)kt * R_BK) >> bs_shift), smem + R_OFF_AM + st * R_AT + wave * 256);
  };
  auto dma_x = [&](int kt, int buf, int i) {
    glds16(xsrc[i] + (long long)kt * R_BK, smem + R_OFF_X + buf * R_XT + (4 * wave + i) * 1024);
  };
  // this lane's 16 packed bytes (row n0 + 32w + c, elements 32h .. 32h+31 of the k-step) + absmax
  auto read_w = [&](int kt, uint32_t (&wd)[4], float& am) {
    const int st = kt % 3;
    const uint4 v = *reinterpret_cast<const uint4*>(smem + R_OFF_W + st * R_WT + wave * 1024 + 32 * c + 16 * h);
    wd[0] = v.x; wd[1] = v.y; wd[2] = v.z; wd[3] = v.w;
    am = *reinterpret_cast<const float*>(smem + R_OFF_AM + st * R_AT + wave * 256 + 4 * c);
  };
  // pair-table lookups for one packed dword (4 bytes = 8 k of this lane's column); the finish
  // multiplies by absmax and rounds once to T, giving the B operand of one 32x32x16 MFMA
  auto lut_read = [&](uint32_t wd, float2 (&cv)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t addr = __builtin_amdgcn_perm(wd, lanebase, 0x0C0C0000u | ((4u + j) << 8));
      cv[j] = *reinterpret_cast<const float2*>(smem + addr);
    }
  };
  auto finish = [&](const float2 (&cv)[4], float am) -> uint4 {
    uint32_t p[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (FL & 8) p[j] = rd_cvt2<T>(cv[j].x * am, cv[j].y * am);
      else p[j] = rd_cvt2<T>(rd_mul(cv[j].x, am), rd_mul(cv[j].y, am));
    }
    return make_uint4(p[0], p[1], p[2], p[3]);
  };
  auto fake_b = [&](uint32_t wd) { return make_uint4(wd, wd ^ 0x11111111u, wd >> 1, wd + 7u); };
  auto read_a = [&](const uint8_t* xs, int ks, uint4 (&a)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const uint4*>(xs + rd_swz(32 * i + c, 4 * h + ks));
  };

  f32x16_t acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;

  // ---- prologue: X(0), W(0), W(1) in flight; the pair table is published by the same barrier
#pragma unroll
  for (int i = 0; i < 4; ++i) dma_x(0, 0, i);
  dma_w(0);
  dma_w(min(1, nk - 1));
  wait_vmcnt0();
  __syncthreads();

  uint32_t wd[4];
  float am;
  uint4 b0;
  float2 cv[4];
  read_w(0, wd, am);
  if (FL & 2) b0 = fake_b(wd[0]);
  else { lut_read(wd[0], cv); b0 = finish(cv, am); }

  // ---- k-loop.  Step t computes on X(t) (stage t & 1) and W(t) (stage t % 3, landed one step ago).
  // It issues X(t+1) and W(t+2) first thing, so the DMA has the whole step to land before the
  // closing vmcnt(0) + barrier.  Sub-steps are software-pipelined: while the 8 MFMAs of ks run, the
  // A fragments and table lookups of ks+1 are in flight and B(ks+1) is finished between the MFMA
  // halves; the last sub-step prepares B(0) of step t+1 (its weights landed a step ago).
  // sched_barriers pin the order (hipcc would otherwise sink the reads next to their uses).
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    const uint8_t* xs = smem + R_OFF_X + s * R_XT;
    uint4 a[2][8], b[2];
    b[0] = b0;
    read_a(xs, 0, a[0]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int cur = ks & 1, nxt = cur ^ 1;
      uint32_t wn[4];
      float amn = am;
      if (FL & 16) {
        // fine interleave: one LDS read (A fragment or table lookup of ks+1) after every MFMA
        if (ks == 3 && t + 1 < nk) read_w(t + 1, wn, amn);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          acc[i] = Mfma32<T>::mma(a[cur][i], b[cur], acc[i]);
          if (ks < 3) {
            a[nxt][i] = *reinterpret_cast<const uint4*>(xs + rd_swz(32 * i + c, 4 * h + ks + 1));
            if (i < 4 && !(FL & 2)) {
              const uint32_t addr = __builtin_amdgcn_perm(wd[ks + 1], lanebase, 0x0C0C0000u | ((4u + i) << 8));
              cv[i] = *reinterpret_cast<const float2*>(smem + addr);
            }
          }
          if (i == 1 && ks == 0) {
            if (!(FL & 1)) {
#pragma unroll
              for (int q = 0; q < 4; ++q) dma_x(min(t + 1, nk - 1), s ^ 1, q);
            }
            dma_w(min(t + 2, nk - 1));
          }
          if (i == 5) {
            if (ks < 3) {
              b[nxt] = (FL & 2) ? fake_b(wd[ks + 1]) : finish(cv, am);
            } else if (t + 1 < nk) {
              wd[0] = wn[0]; wd[1] = wn[1]; wd[2] = wn[2]; wd[3] = wn[3];
              am = amn;
              if (FL & 2) b0 = fake_b(wd[0]);
              else { lut_read(wd[0], cv); b0 = finish(cv, am); }
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        continue;
      }
      if (ks < 3) {
        if (!(FL & 2)) lut_read(wd[ks + 1], cv);
        read_a(xs, ks + 1, a[nxt]);
      } else if (t + 1 < nk) {
        read_w(t + 1, wn, amn);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (FL & 4) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = Mfma32<T>::mma(a[cur][i], b[cur], acc[i]);
      if (FL & 4) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if (ks == 0) {
        if (!(FL & 1)) {
#pragma unroll
          for (int i = 0; i < 4; ++i) dma_x(min(t + 1, nk - 1), s ^ 1, i);
        }
        dma_w(min(t + 2, nk - 1));
      }
      if (ks < 3) {
        b[nxt] = (FL & 2) ? fake_b(wd[ks + 1]) : finish(cv, am);
      } else if (t + 1 < nk) {
        wd[0] = wn[0]; wd[1] = wn[1]; wd[2] = wn[2]; wd[3] = wn[3];
        am = amn;
        if (FL & 2) b0 = fake_b(wd[0]);
        else { lut_read(wd[0], cv); b0 = finish(cv, am); }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (FL & 4) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 4; i < 8; ++i) acc[i] = Mfma32<T>::mma(a[cur][i], b[cur], acc[i]);
      if (FL & 4) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
    wait_vmcnt0();
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- epilogue: acc -> LDS (per-wave [256][32] T, 64-B rows) -> 16-B stores, 64 B per row
  uint8_t* ep = smem + wave * (256 * 64);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * i + 8 * (r >> 2) + 4 * h + (r & 3);
      *reinterpret_cast<T*>(ep + row * 64 + 2 * c) = Io<T>::from_f32(acc[i][r]);
    }
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the wave reads back only its own region
  const int gcol0 = n0 + 32 * wave;
  const bool vec_ok = ((ldc & 7) == 0) && (((uintptr_t)out & 15) == 0);
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = lane + 64 * it;
    const int row = id >> 2, part = id & 3;
    const int grow = m0 + row, gcol = gcol0 + 8 * part;
    if (grow >= M) continue;
    const uint4 v = *reinterpret_cast<const uint4*>(ep + row * 64 + 16 * part);
    T* dst = out + (long long)grow * ldc + gcol;
    if (vec_ok && gcol + 8 <= N) {
      *reinterpret_cast<uint4*>(dst) = v;
    } else {
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      for (int e = 0; e < 8 && gcol + e < N; ++e) dst[e] = __builtin_bit_cast(T, (uint16_t)(w4[e >> 1] >> (16 * (e & 1))));
    }
  }
}

template <typename T>
void launch_gemm_4bit_rd(int m, int n, int k, const T* A, const uint8_t* B, const float* absmax, const float* datatype,
                         T* out, int lda, int ldb, int ldc, int blocksize) {
  const long long tiles = (long long)((m + R_BN - 1) / R_BN) * ((n + R_BM - 1) / R_BM);
  hipLaunchKernelGGL((k_gemm_4bit_rd<T, 0>), dim3((unsigned)tiles), dim3(R_THREADS), 0, current_stream(), m, n, k, A,
                     B, absmax, datatype, out, lda, ldb, ldc, blocksize);
}

template void launch_gemm_4bit_rd<bf16_t>(int, int, int, const bf16_t*, const uint8_t*, const float*, const float*,
                                          bf16_t*, int, int, int, int);
template void launch_gemm_4bit_rd<fp16_t>(int, int, int, const fp16_t*, const uint8_t*, const float*, const float*,
                                          fp16_t*, int, int, int, int);

}  // namespace bnb
