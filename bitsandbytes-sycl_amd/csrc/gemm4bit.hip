// Fused 4-bit (NF4/FP4) weight GEMM for M > 1 (prefill) on gfx950 MFMA.
//
// Slot in the reference: cgemm_4bit_inference          ref:sycl/pythonInterface.cpp:377-378
//   -> gemm_4bit_inference<T>                          ref:sycl/sycl_code/op_gemm.cpp:843-889
//   -> kgemm_4bit_inference<T,96> (broken, Q7)         ref:sycl/sycl_code/kernel_gemm.cpp:1015-1265
// and the path it replaces for M > 1: MatMul4Bit.forward = dequantize_4bit + F.linear
//   ref:python_src_quants/autograd/_functions.py:491-507, functional.py:1291-1424.
//
// Argument convention (same as the gemv ABI, functional.py:1992-1997): m = out_features
// (rows of the packed weight W), n = activation rows (tokens), k = in_features;
//   out[t, r] = sum_k A[t*lda + k] * code[q(r,k)] * absmax[(2*ldb*r + k) / blocksize]
// A is [n, k] (row stride lda), out is [n, m] (row stride ldc), W rows are ldb bytes apart.
// Numerics = the reference M>1 path: each weight element is dequantised in fp32 and rounded
// once to T (bf16/fp16) exactly like dequantize_4bit, then multiplied on the bf16/fp16 MFMA
// with fp32 accumulation.
//
// Design (MI355X): 128x128 output tile per 256-thread workgroup (4 waves, 2x2, 64x64 per wave,
// v_mfma_f32_16x16x32_{bf16,f16}), BK = 64, two LDS stages.  Activations are staged by
// global_load_lds (16 B per lane, XOR-swizzled via the source address); the packed weight
// tile (4 KiB per stage: a quarter of the bf16 bytes) is loaded to registers, dequantised once
// per workgroup through a 256-entry LDS pair table and written to LDS as T in the same
// swizzled layout, so both MFMA operands are read with conflict-free ds_read_b128.
// XCD-aware tile order keeps the tiles that share activation panels on one XCD's L2.
#include "gemm_common.hpp"

#include <algorithm>

namespace bnb {

constexpr int G_BM = 128, G_BN = 128, G_BK = 64, G_THREADS = 256;
constexpr int G_TILE_BYTES = G_BM * G_BK * 2;        // 16 KiB per operand per stage
constexpr int G_LDS_BYTES = 4 * G_TILE_BYTES + 256 * 8;

template <typename T>
__global__ void __launch_bounds__(G_THREADS, 2)
k_gemm_4bit(int N, int M, int K, const T* __restrict__ A, const uint8_t* __restrict__ B,
            const float* __restrict__ absmax, const float* __restrict__ datatype, T* __restrict__ out,
            int lda, int ldb, int ldc, int blocksize) {
  // here: M = tokens (rows of A/out), N = out features (rows of W)
  __shared__ __attribute__((aligned(16))) uint8_t smem[G_LDS_BYTES];
  uint8_t* Xs = smem;                                  // [2][128][64] T
  uint8_t* Ws = smem + 2 * G_TILE_BYTES;               // [2][128][64] T
  float2* lut = reinterpret_cast<float2*>(smem + 4 * G_TILE_BYTES);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  lut[tid] = make_float2(datatype[tid >> 4], datatype[tid & 15]);

  // ---- XCD-aware tile mapping (bijective for any grid size)
  const int tilesN = (N + G_BN - 1) / G_BN;
  const int tilesM = (M + G_BM - 1) / G_BM;
  const int nwg = tilesN * tilesM;
  int wg = blockIdx.x;
  {
    const int xcd = wg & 7, q = nwg >> 3, r = nwg & 7;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (wg >> 3);
  }
  // group 8 token-tiles together so an XCD's consecutive tiles share weight panels too
  constexpr int GROUP = 8;
  const int group_span = GROUP * tilesN;
  const int gidx = wg / group_span;
  const int first_m = gidx * GROUP;
  const int gsize = min(tilesM - first_m, GROUP);
  const int tm = first_m + (wg % group_span) % gsize;
  const int tn = (wg % group_span) / gsize;
  const int m0 = tm * G_BM, n0 = tn * G_BN;

  // ---- per-thread staging roles
  // activations: 4 glds per wave per stage; wave-instruction i covers rows 8*(4*wave+i) .. +7
  const T* xsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (4 * wave + i) + (lane >> 3);
    const int grow = min(m0 + row, M - 1);
    const int gslot = (lane & 7) ^ (row & 7);
    xsrc[i] = A + (long long)grow * lda + 8 * gslot;
  }
  // weights: thread t -> row t>>1, half h (32 elements = 16 packed bytes)
  const int wrow = tid >> 1, wh = tid & 1;
  const int gwrow = min(n0 + wrow, N - 1);
  const uint8_t* wsrc = B + (long long)gwrow * ldb + 16 * wh;
  const long long am_base = 2LL * ldb * gwrow + 32 * wh;

  const int wm = wave >> 1, wn = wave & 1;
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = K / G_BK;

  // prologue: stage 0 activations, weights of k-tile 0 to registers
#pragma unroll
  for (int i = 0; i < 4; ++i) glds16(xsrc[i], Xs + (4 * wave + i) * 1024);
  uint4 wq = ld_nt16(wsrc);
  float wam = absmax[am_base / blocksize];
  __syncthreads();   // lut ready

  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    uint8_t* xs = Xs + cur * G_TILE_BYTES;
    uint8_t* ws = Ws + cur * G_TILE_BYTES;
    // dequantise this k-tile's weights into LDS (each element once per workgroup)
    {
      const uint32_t w[4] = {wq.x, wq.y, wq.z, wq.w};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        uint32_t pk[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float2 c = lut[(w[s] >> (8 * j)) & 0xFF];
          pk[j] = Mfma<T>::pack2(__fmul_rn(c.x, wam), __fmul_rn(c.y, wam));
        }
        *reinterpret_cast<uint4*>(ws + swz(wrow, 4 * wh + s)) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 1 < nk) {
      const int k1 = (t + 1) * G_BK;
      uint8_t* xn = Xs + (cur ^ 1) * G_TILE_BYTES;
#pragma unroll
      for (int i = 0; i < 4; ++i) glds16(xsrc[i] + k1, xn + (4 * wave + i) * 1024);
      wq = ld_nt16(wsrc + k1 / 2);
      wam = absmax[(am_base + k1) / blocksize];
    }
    // MFMA on the current stage
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 a[4], b[4];
      const int slot = 4 * ks + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const uint4*>(xs + swz(64 * wm + 16 * i + (lane & 15), slot));
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const uint4*>(ws + swz(64 * wn + 16 * j + (lane & 15), slot));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = Mfma<T>::mma(a[i], b[j], acc[i][j]);
    }
  }

  // epilogue: C/D map of 16x16x32: col = lane&15, row = 4*(lane>>4) + r
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + 64 * wn + 16 * j + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + 64 * wm + 16 * i + 4 * (lane >> 4) + r;
        if (row < M && col < N) out[(long long)row * ldc + col] = Io<T>::from_f32(acc[i][j][r]);
      }
    }
  }
}

Knob<int> g_tile_override{0};

// Split-K factor for the 256-tile kernel: enough workgroups to cover the 256 CUs when the output has
// fewer than ~200 256x256 tiles (narrow column shards, e.g. N/8 = 512 features at M = 4096, or few
// tokens: 16 x 4096 x 11008 ran 176 us on the 32-workgroup 128-tile grid), with at least 8 k-tiles
// per split.  Below 256 weight rows (the 70B k/v shard 128 x 8192 at 4096 tokens: 16 half-empty tiles) the split
// form still beats the 128-tile kernel's 32 whole-K workgroups (151 us there; profiles/lab/r02_narrow_weight.txt).
// Needs a caller-supplied fp32 workspace of ksplit * m * n floats.
static int splitk_factor(int m, int n, int k) {
  if (m < 64) return 1;
  const long long tiles = (long long)((m + 255) / 256) * ((n + 255) / 256);
  if (tiles >= 200) return 1;
  int ks = (int)((256 + tiles / 2) / tiles);
  ks = std::min(ks, std::max(1, (k / G_BK) / 8));
  return std::max(1, std::min(ks, 16));
}

long long gemm_4bit_workspace_bytes(int m, int n, int k) {
  const int ks = splitk_factor(m, n, k);
  return std::max(ks > 1 ? (long long)ks * m * n * (long long)sizeof(float) : 0LL, skinny_workspace_bytes(m, n, k));
}

template <typename T>
void gemm_4bit(int m, int n, int k, const T* A, const uint8_t* B, const float* absmax, const float* datatype, T* out,
               int lda, int ldb, int ldc, int blocksize, float* ws = nullptr, long long ws_bytes = 0) {
  if (m <= 0 || n <= 0) return;
  if (k <= 0 || k % G_BK != 0 || lda % 8 != 0 || ldb % 16 != 0 || blocksize < 64 || blocksize % 32 != 0 ||
      ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) {
    set_error(1, "gemm_4bit: requires k % 64 == 0, lda % 8 == 0, ldb % 16 == 0, 16-B aligned A/B, blocksize >= 64");
    return;
  }
  // few tokens (<= 64, SK_MAX_TOKENS): the weight-streaming kernels (gemm4bit_skinny.hip, gemm4bit_wk.hip)
  if (g_tile_override == 0) {
    const SkStats st{absmax, nullptr, nullptr, nullptr, nullptr, 0, 0};
    if (launch_gemm_4bit_skinny<T>(m, n, k, A, lda, B, ldb, st, blocksize, 0, datatype, out, ldc, ws, ws_bytes)) {
      BNB_LAUNCH_CHECK("gemm_4bit");
      return;
    }
  }
  // m = out features (weight rows), n = tokens.  Large problems: 256x256 tiles (split-K when the
  // tile grid is too small and a workspace is given); small: 128x128.
  const long long tiles256 = (long long)((m + 255) / 256) * ((n + 255) / 256);
  const bool pow2_bs = (blocksize & (blocksize - 1)) == 0;
  int ks = splitk_factor(m, n, k);
  if (ws == nullptr || ((uintptr_t)ws & 15) || (long long)ks * m * n * (long long)sizeof(float) > ws_bytes) ks = 1;
  // 256x256 (with split-K) when its grid fills the chip (>= 128 workgroups), and also when it still has at
  // least half the workgroups of the 128x128 grid, which then run the full K each (e.g. 512 features x
  // 256 tokens: 8 workgroups of 128x128 took 174 us where 2 x 16-way split 256x256 tiles take ~25)
  const long long tiles128 = (long long)((m + G_BN - 1) / G_BN) * ((n + G_BM - 1) / G_BM);
  const bool use256 = pow2_bs && (g_tile_override == 256 ||
                                  (g_tile_override != 128 && (m >= 256 || ks > 1) &&
                                   (tiles256 * ks >= 128 || 2 * tiles256 * ks >= tiles128)));
  if (use256) {
    launch_gemm_4bit_256<T>(m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize, ws, ks);
  } else {
    const int tiles = ((m + G_BN - 1) / G_BN) * ((n + G_BM - 1) / G_BM);
    hipLaunchKernelGGL((k_gemm_4bit<T>), dim3(tiles), dim3(G_THREADS), 0, current_stream(), m, n, k, A, B, absmax,
                       datatype, out, lda, ldb, ldc, blocksize);
  }
  BNB_LAUNCH_CHECK("gemm_4bit");
}

static __device__ float g_nf4_table[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
    -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
    0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f, 0.33791524171829224f,
    0.44070982933044434f, 0.5626170039176941f, 0.7229568362236023f, 1.0f};

static const float* nf4_table_device() {
  void* p = nullptr;
  hipGetSymbolAddress(&p, HIP_SYMBOL(g_nf4_table));
  return (const float*)p;
}

}  // namespace bnb

using namespace bnb;

extern "C" {

// Reference ABI slot (NF4 hard-coded, fp16), ref:sycl/pythonInterface.cpp:377-378.
void cgemm_4bit_inference(int m, int n, int k, fp16_t* A, unsigned char* B, float* absmax, fp16_t* out, int lda,
                          int ldb, int ldc, int blocksize) {
  BNB_RANGE("cgemm_4bit_inference");
  gemm_4bit<fp16_t>(m, n, k, A, B, absmax, nf4_table_device(), out, lda, ldb, ldc, blocksize);
}
// bf16 sibling and table-driven variants (any 16-entry code: NF4/FP4).
void cgemm_4bit_inference_bf16(int m, int n, int k, bf16_t* A, unsigned char* B, float* absmax, bf16_t* out, int lda,
                               int ldb, int ldc, int blocksize) {
  BNB_RANGE("cgemm_4bit_inference_bf16");
  gemm_4bit<bf16_t>(m, n, k, A, B, absmax, nf4_table_device(), out, lda, ldb, ldc, blocksize);
}
void cgemm_4bit_inference_code_fp16(int m, int n, int k, fp16_t* A, unsigned char* B, float* absmax, float* datatype,
                                    fp16_t* out, int lda, int ldb, int ldc, int blocksize) {
  BNB_RANGE("cgemm_4bit_inference_code_fp16");
  gemm_4bit<fp16_t>(m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize);
}
void cgemm_4bit_inference_code_bf16(int m, int n, int k, bf16_t* A, unsigned char* B, float* absmax, float* datatype,
                                    bf16_t* out, int lda, int ldb, int ldc, int blocksize) {
  BNB_RANGE("cgemm_4bit_inference_code_bf16");
  gemm_4bit<bf16_t>(m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize);
}
// [additive] the same with a caller-owned fp32 workspace that enables split-K for small tile grids
// (size it with cgemm_4bit_workspace_bytes; a smaller or NULL workspace just disables split-K).
void cgemm_4bit_inference_code_ws_fp16(int m, int n, int k, fp16_t* A, unsigned char* B, float* absmax,
                                       float* datatype, fp16_t* out, int lda, int ldb, int ldc, int blocksize,
                                       float* workspace, long long workspace_bytes) {
  BNB_RANGE("cgemm_4bit_inference_code_ws_fp16");
  gemm_4bit<fp16_t>(m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize, workspace, workspace_bytes);
}
void cgemm_4bit_inference_code_ws_bf16(int m, int n, int k, bf16_t* A, unsigned char* B, float* absmax,
                                       float* datatype, bf16_t* out, int lda, int ldb, int ldc, int blocksize,
                                       float* workspace, long long workspace_bytes) {
  BNB_RANGE("cgemm_4bit_inference_code_ws_bf16");
  gemm_4bit<bf16_t>(m, n, k, A, B, absmax, datatype, out, lda, ldb, ldc, blocksize, workspace, workspace_bytes);
}
long long cgemm_4bit_workspace_bytes(int m, int n, int k) { return gemm_4bit_workspace_bytes(m, n, k); }

}  // extern "C"

extern "C" {
// [additive, testing] force the tile kernel used by the 4-bit GEMM (0 = auto, 128 = 128x128 kernel)
void cgemm_4bit_set_tile(int tile) { bnb::g_tile_override = tile; }
}
