// 256 x 256-tile int8 GEMM on v_mfma_i32_16x16x64_i8 (gfx950): the large-problem kernel behind
// igemmlt (ref:sycl/sycl_code/op_gemm.cpp:541-655, C = A @ B^T exact int32) and the fused
// igemmlt + dequant_mm_int32_fp16 path (ref:sycl/sycl_code/kernel_quant.cpp:3846-3987).
//
// Geometry: 512 threads = 8 waves (2 along M x 4 along N), 128 x 64 outputs per wave (8 x 4 tiles of
// 16x16), BK = 128 bytes, two LDS stages (2 x (32 + 32) KiB), one barrier per k-step, fragments register-
// pipelined across it.  Both operands
// arrive by LDS-DMA (16 B per lane, XOR-swizzled through the source address) from any layout whose
// 16-k runs are contiguous: row-major, col32 (A) and col_ampere (B); col_turing B (4-k runs, the reference's
// formatB, ref:functional.py:410-418) is copied by whole 8-row groups and its fragments gathered as 4 dwords.  Fragment convention: lane l
// holds 16 consecutive k of row l&15, k-chunk l>>4 -- identical for A and B, so the int32 result is
// exact whatever order the instruction sums k in.  Epilogues: int32 row-major / col32, int8 col32
// (alpha = 1 or per-row scale) and the fused mm_dequant to fp16, staged through LDS for 16-B stores.
#include "gemm_common.hpp"
#include "int8_common.hpp"

#include <algorithm>

namespace bnb {

typedef __attribute__((ext_vector_type(4))) int i32x4_t;

constexpr int J_BM = 256, J_BN = 256, J_BK = 128, J_THREADS = 512;
constexpr int J_TILE = J_BM * J_BK;                     // 32 KiB
constexpr int J_EPI_STRIDE = 136;                       // fp16 staging row: 128 B + 8 B pad
constexpr int J_LDS_MAIN = 4 * J_TILE;                  // 128 KiB
constexpr int J_LDS_EPI = 8 * 128 * J_EPI_STRIDE;       // 136 KiB
constexpr int J_LDS = J_LDS_MAIN > J_LDS_EPI ? J_LDS_MAIN : J_LDS_EPI;

template <int F>
__device__ __forceinline__ const int8_t* chunk_ptr(const int8_t* P, long long ld, long long r, long long k) {
  return P + fmt_offset<F>(r, k, ld);    // 16 contiguous bytes for ROW / COL32 / AMPERE when k % 16 == 0
}

// SPLIT (row-major A and B only): the grid is tiles x ksplit, workgroup `split` sums k-tiles [kb, kb + nk) of K / 128
// and stores its int32 tile to ws[split][M][N]; k_igemm_splitk_reduce adds the splits (exact integer sums, so any
// order gives the unsplit kernel's int32) and applies the epilogue.  For small tile grids: the column shards of the
// multi-GPU step (N / 8 = 512 features: 16-32 tiles on 256 CUs).
template <int AF, int BF, int EPI, bool SPLIT = false>
__global__ void __launch_bounds__(J_THREADS, 1)
k_igemm_256(int M, int N, int K, const int8_t* __restrict__ A, const int8_t* __restrict__ B, void* __restrict__ Cout,
            const float* __restrict__ row_scale, long long lda, long long ldb, long long ldc,
            const float* __restrict__ rowStats, const float* __restrict__ colStats, const fp16_t* __restrict__ bias,
            int32_t* __restrict__ ws = nullptr, int ksplit_arg = 1) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[J_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int tilesN = (N + J_BN - 1) / J_BN, tilesM = (M + J_BM - 1) / J_BM;
  const int ksplit = SPLIT ? ksplit_arg : 1;
  const int ntiles = tilesN * tilesM;
  // with split-K the split is the outer index, so an XCD's workgroups share one K range
  const int wg_all = xcd_remap(blockIdx.x, ntiles * ksplit);
  const int split = SPLIT ? wg_all / ntiles : 0;
  const int wg = SPLIT ? wg_all - split * ntiles : wg_all;
  constexpr int GROUP = 4;
  const int group_span = GROUP * tilesN;
  const int first_m = (wg / group_span) * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * J_BM, n0 = tn * J_BN;

  // DMA roles: wave-instruction i covers tile rows 8*(4*wave+i) .. +7, lane -> (row, 16-B slot)
  long long arow[4], brow[4];
  int kslot[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wave + i) + (lane >> 3);
    arow[i] = min(m0 + row, M - 1);
    brow[i] = min(n0 + row, N - 1);
    kslot[i] = 16 * ((lane & 7) ^ (row & 7));
  }
  // col_turing B (col4_4r2_8c, ldb = 32 * pad8(rows)): within a 32-column block the 256 tile rows are 32 groups of
  // 8 rows x 32 bytes = 8 KiB contiguous, and a 16-B chunk holds 4 bytes (4 consecutive k) of 4 rows.  The tile's
  // 4 column blocks are copied as they lie (4 x 8 KiB); slot s of (group g, row parity par) receives source chunk
  // s ^ (2 (g & 1) + par), which makes the fragment reads below conflict-free.  Rows past pad8(n) re-read the last
  // group (their outputs are not stored).
  // One lane offset (the lane's group, parity and swizzled chunk; gl & 1 = (lane >> 4) & 1 for every piece); the
  // piece's column block and 1-KiB slice are wave-uniform.  Offsets are clamped to the buffer (K / 32 column
  // blocks of ldb bytes, < 4 GiB), so rows past pad8(n) read valid bytes.
  const unsigned t_lane = ((n0 >> 3) + (lane >> 4)) * 256 + ((lane >> 3) & 1) * 128 +
                          16 * ((lane & 7) ^ (2 * ((lane >> 4) & 1) + ((lane >> 3) & 1)));
  const unsigned t_last = (unsigned)((long long)(K >> 5) * ldb - 16);
  auto dma_b_turing = [&](int kt, int buf, int i) {
    const int p = 4 * wave + i, cb = p >> 3, j = p & 7;
    const unsigned off = min(t_lane + (unsigned)(((long long)kt * 4 + cb) * ldb) + 1024u * j, t_last);
    glds16(B + off, smem + 2 * J_TILE + buf * J_TILE + cb * 8192 + j * 1024);
  };
  const int nk_all = K / J_BK;
  const int kb = SPLIT ? (int)((long long)split * nk_all / ksplit) : 0;   // this split's first k-tile
  auto dma = [&](int kt, int buf) {
    const long long k0 = (long long)(kb + kt) * J_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      glds16(chunk_ptr<AF>(A, lda, arow[i], k0 + kslot[i]), smem + buf * J_TILE + (4 * wave + i) * 1024);
      if constexpr (BF == TURING) dma_b_turing(kt, buf, i);
      else glds16(chunk_ptr<BF>(B, ldb, brow[i], k0 + kslot[i]), smem + 2 * J_TILE + buf * J_TILE + (4 * wave + i) * 1024);
    }
  };

  const int wm = wave >> 2, wn = wave & 3;
  i32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = i32x4_t{0, 0, 0, 0};

  // Cross-barrier pipeline: tile t's ks = 1 fragments are read into registers before its ks = 0 MFMAs,
  // so after the barrier the wave reads tile t+1's ks = 0 fragments under tile t's ks = 1 MFMAs; the
  // barrier and a tile's first LDS latency hide behind 32 MFMAs (tools/igemm_lab.hip: 5-8 % over
  // reading each k-half after the barrier, outputs bit-identical).
  // col_turing fragment offsets: row r = 64 wn + 16 j + (lane & 15) lies in group 8 wn + 2 j + ((lane >> 3) & 1) at
  // parity lane & 1 and pair (lane & 7) >> 1; k-chunk (lane >> 4) -> column block (lane >> 5), half (lane >> 4) & 1
  int tb[4] = {0, 0, 0, 0};
  if constexpr (BF == TURING) {
    const int f = 2 * ((lane >> 3) & 1) + (lane & 1);
    const int base = (8 * wn + ((lane >> 3) & 1)) * 256 + (lane & 1) * 128 + 4 * ((lane & 7) >> 1) +
                     8192 * (lane >> 5) + 64 * ((lane >> 4) & 1);
#pragma unroll
    for (int u = 0; u < 4; ++u) tb[u] = base + 16 * (u ^ f);
  }
  uint4 fa[2][8], fb[2][4];
  auto frag = [&](int buf, int ks, uint4 (&a)[8], uint4 (&b)[4]) {
    const uint8_t* as = smem + buf * J_TILE;
    const uint8_t* bs = smem + 2 * J_TILE + buf * J_TILE;
    const int slot = 4 * ks + (lane >> 4);
    if constexpr (BF == TURING) {
      // 16 consecutive k of one row = 4 dwords from the 4 chunks of its (group, parity) half-row, read in k order;
      // the lane's offsets tb[u] are loop-invariant, k-half ks adds 2 column blocks and fragment j 2 groups
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t d[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) d[u] = *reinterpret_cast<const uint32_t*>(bs + tb[u] + ks * 16384 + j * 512);
        b[j] = make_uint4(d[0], d[1], d[2], d[3]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const uint4*>(bs + swz(64 * wn + 16 * j + (lane & 15), slot));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const uint4*>(as + swz(128 * wm + 16 * i + (lane & 15), slot));
  };
  auto mma = [&](const uint4 (&a)[8], const uint4 (&b)[4]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4_t, a[i]), __builtin_bit_cast(i32x4_t, b[j]),
                                                          acc[i][j], 0, 0, 0);
  };
  const int nk = SPLIT ? (int)((long long)(split + 1) * nk_all / ksplit) - kb : nk_all;
  dma(0, 0);
  if (nk > 1) {
    dma(1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile 0 landed; tile 1 stays in flight
  } else {
    wait_vmcnt0();
  }
  __syncthreads();
  frag(0, 0, fa[0], fb[0]);
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    frag(s, 1, fa[1], fb[1]);
    mma(fa[0], fb[0]);
    wait_vmcnt0();                                     // this wave's part of tile t+1 landed
    __builtin_amdgcn_s_waitcnt(0xC07F);                // and its reads of tile t are done
    __builtin_amdgcn_s_barrier();
    if (t + 2 < nk) dma(t + 2, s);                     // every wave is past tile t: reuse its stage
    if (t + 1 < nk) frag(s ^ 1, 0, fa[0], fb[0]);
    mma(fa[1], fb[1]);
  }
  __syncthreads();                                     // epilogue staging reuses the stages

  // ---- epilogues (C/D: col = lane&15, row = 4*(lane>>4) + r)
  const int grow0 = m0 + 128 * wm, gcol0 = n0 + 64 * wn;
  if constexpr (SPLIT) {
    int32_t* wsp = ws + (long long)split * M * N;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = grow0 + 16 * i + 4 * (lane >> 4) + r;
        if (row >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = gcol0 + 16 * j + (lane & 15);
          if (col < N) wsp[(long long)row * N + col] = acc[i][j][r];
        }
      }
    return;
  }
  if constexpr (EPI == EPI_F16_ROW_DEQUANT) {
    uint8_t* ep = smem + wave * (128 * J_EPI_STRIDE);
    float cs[4], bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = min(gcol0 + 16 * j + (lane & 15), N - 1);
      cs[j] = colStats[col];
      bv[j] = bias ? (float)bias[col] : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * i + 4 * (lane >> 4) + r;
        const float rs = rowStats[min(grow0 + row, M - 1)];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<fp16_t*>(ep + row * J_EPI_STRIDE + 2 * (16 * j + (lane & 15))) =
              mm_dequant_value(acc[i][j][r], rs, cs[j], bv[j]);
      }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    fp16_t* out = reinterpret_cast<fp16_t*>(Cout);
    const bool vec_ok = ((ldc & 7) == 0) && (((uintptr_t)out & 15) == 0);
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int id = lane + 64 * it;
      const int row = id >> 3, c8 = id & 7;
      const int grow = grow0 + row, gcol = gcol0 + 8 * c8;
      if (grow >= M) continue;
      const uint2 lo = *reinterpret_cast<const uint2*>(ep + row * J_EPI_STRIDE + 16 * c8);
      const uint2 hi = *reinterpret_cast<const uint2*>(ep + row * J_EPI_STRIDE + 16 * c8 + 8);
      fp16_t* dst = out + (long long)grow * ldc + gcol;
      if (vec_ok && gcol + 8 <= N) {
        *reinterpret_cast<uint4*>(dst) = make_uint4(lo.x, lo.y, hi.x, hi.y);
      } else {
        const uint32_t w4[4] = {lo.x, lo.y, hi.x, hi.y};
        for (int e = 0; e < 8 && gcol + e < N; ++e) dst[e] = __builtin_bit_cast(fp16_t, (uint16_t)(w4[e >> 1] >> (16 * (e & 1))));
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = grow0 + 16 * i + 4 * (lane >> 4) + r;
        if (row >= M) continue;
        float rsc = 1.0f;
        if constexpr (EPI == EPI_I8_COL32_ROWSCALE) rsc = row_scale[row];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = gcol0 + 16 * j + (lane & 15);
          if (col >= N) continue;
          const int32_t v = acc[i][j][r];
          if constexpr (EPI == EPI_I32_ROW) reinterpret_cast<int32_t*>(Cout)[(long long)row * ldc + col] = v;
          else if constexpr (EPI == EPI_I32_COL32) reinterpret_cast<int32_t*>(Cout)[fmt_offset<COL32>(row, col, ldc)] = v;
          else if constexpr (EPI == EPI_I8_COL32) reinterpret_cast<int8_t*>(Cout)[fmt_offset<COL32>(row, col, ldc)] = rint_i8((float)v);
          else reinterpret_cast<int8_t*>(Cout)[fmt_offset<COL32>(row, col, ldc)] = rint_i8(__fmul_rn((float)v, rsc));
        }
      }
  }
}

// out[r, c] = EPI(sum_s ws[s][r][c]): int32 sums (exact), then the fused mm_dequant to fp16 or the int32 store.
// 4 columns per thread (N % 4 == 0: 16-B loads), else one.
template <int EPI>
__global__ void __launch_bounds__(256)
k_igemm_splitk_reduce(const int32_t* __restrict__ ws, int ksplit, int M, int N, void* __restrict__ Cout, long long ldc,
                      const float* __restrict__ rowStats, const float* __restrict__ colStats,
                      const fp16_t* __restrict__ bias) {
  const long long mn = (long long)M * N;
  const int V = (N & 3) == 0 ? 4 : 1;
  const long long i0 = (long long)V * ((long long)blockIdx.x * 256 + threadIdx.x);
  if (i0 >= mn) return;
  int32_t v[4] = {0, 0, 0, 0};
  if (V == 4) {
    for (int s = 0; s < ksplit; ++s) {
      const int4 p = *reinterpret_cast<const int4*>(ws + s * mn + i0);
      v[0] += p.x; v[1] += p.y; v[2] += p.z; v[3] += p.w;
    }
  } else {
    for (int s = 0; s < ksplit; ++s) v[0] += ws[s * mn + i0];
  }
  const long long r = i0 / N, c0 = i0 - r * N;
  for (int e = 0; e < V; ++e) {
    const long long c = c0 + e;
    if constexpr (EPI == EPI_F16_ROW_DEQUANT) {
      reinterpret_cast<fp16_t*>(Cout)[r * ldc + c] =
          mm_dequant_value(v[e], rowStats[r], colStats[c], bias ? (float)bias[c] : 0.0f);
    } else {
      reinterpret_cast<int32_t*>(Cout)[r * ldc + c] = v[e];
    }
  }
}

static Knob<int> g_igemm_splitk{-1};   // < 0: auto; 1 = never split; >= 2: force that factor where it applies (tests)

// Split-K factor for a row-major 256-tile problem: enough workgroups for the 256 CUs when the output has fewer
// than ~200 tiles, with at least 8 k-tiles (1024 k) per split -- 2 below 256 rows (few-token forwards, where the
// weight stream is the work) -- at most 16 splits.
int igemm_splitk_factor(int m, int n, int k) {
  if (k % J_BK != 0 || m < 1 || n < 256) return 1;
  const long long tiles = (long long)((m + J_BM - 1) / J_BM) * ((n + J_BN - 1) / J_BN);
  int ks;
  if (g_igemm_splitk >= 1) {
    ks = g_igemm_splitk;
  } else {
    if (tiles >= 200) return 1;
    ks = (int)((256 + tiles / 2) / tiles);
  }
  ks = std::min(ks, std::max(1, (k / J_BK) / (m < 256 ? 2 : 8)));
  return std::max(1, std::min(ks, 16));
}

long long igemm_workspace_bytes(int m, int n, int k) {
  const int ks = igemm_splitk_factor(m, n, k);
  return ks > 1 ? (long long)ks * m * n * (long long)sizeof(int32_t) : 0;
}

template <int AF, int BF, int EPI>
bool launch_igemm_256(int m, int n, int k, const int8_t* A, const int8_t* B, void* C, const float* row_scale,
                      long long lda, long long ldb, long long ldc, const float* rowStats, const float* colStats,
                      const fp16_t* bias, int32_t* ws, long long ws_bytes) {
  if constexpr (AF == TURING) {
    return false;                                                  // A in 4-byte runs: register-staged kernel
  } else {
    // below 256 rows only the split-K form (row-major operands, a workspace), which fills the chip from the
    // weight side; otherwise the 128-tile kernel
    if (k % J_BK != 0 || n < 256 || m < 1) return false;
    if ((AF == ROW && lda % 16) || (BF == ROW && ldb % 16) || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return false;
    if (BF == TURING && (ldb % 256 || ldb < 32LL * n || (long long)(k / 32) * ldb >= (1LL << 32))) return false;
    const long long tiles = (long long)((m + J_BM - 1) / J_BM) * ((n + J_BN - 1) / J_BN);
    if constexpr (AF == ROW && BF == ROW && (EPI == EPI_F16_ROW_DEQUANT || EPI == EPI_I32_ROW)) {
      const int ks = igemm_splitk_factor(m, n, k);
      if (ks > 1 && ws != nullptr && ((uintptr_t)ws & 15) == 0 &&
          (long long)ks * m * n * (long long)sizeof(int32_t) <= ws_bytes) {
        hipLaunchKernelGGL((k_igemm_256<AF, BF, EPI, true>), dim3((unsigned)(tiles * ks)), dim3(J_THREADS), 0,
                           current_stream(), m, n, k, A, B, C, row_scale, lda, ldb, ldc, rowStats, colStats, bias, ws,
                           ks);
        const long long mn = (long long)m * n;
        const long long threads = (n % 4 == 0) ? mn / 4 : mn;
        hipLaunchKernelGGL((k_igemm_splitk_reduce<EPI>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                           current_stream(), ws, ks, m, n, C, ldc, rowStats, colStats, bias);
        return true;
      }
    }
    if (m < 256) return false;
    hipLaunchKernelGGL((k_igemm_256<AF, BF, EPI>), dim3((unsigned)tiles), dim3(J_THREADS), 0, current_stream(), m, n,
                       k, A, B, C, row_scale, lda, ldb, ldc, rowStats, colStats, bias, nullptr, 1);
    return true;
  }
}

#define BNB_INST(AF, BF, EPI)                                                                                      \
  template bool launch_igemm_256<AF, BF, EPI>(int, int, int, const int8_t*, const int8_t*, void*, const float*,    \
                                              long long, long long, long long, const float*, const float*,         \
                                              const fp16_t*, int32_t*, long long);
BNB_INST(ROW, ROW, EPI_F16_ROW_DEQUANT)
BNB_INST(ROW, ROW, EPI_I32_ROW)
BNB_INST(COL32, AMPERE, EPI_I32_COL32)
BNB_INST(COL32, AMPERE, EPI_I8_COL32)
BNB_INST(COL32, AMPERE, EPI_I8_COL32_ROWSCALE)
BNB_INST(COL32, TURING, EPI_I32_COL32)
BNB_INST(COL32, TURING, EPI_I8_COL32)
BNB_INST(COL32, TURING, EPI_I8_COL32_ROWSCALE)
#undef BNB_INST

}  // namespace bnb

extern "C" {
// [additive, testing] int8 split-K factor: -1 = auto, 1 = never split, >= 2 = force where it applies
void cigemm_set_splitk(int ks) { bnb::g_igemm_splitk = ks; }
}
