"""numpy restatement of the reference hot-path algorithm (TEST INFRASTRUCTURE ONLY).

See oracle/__init__.py for who may import this and how it is pinned.
All arithmetic that the reference performs in fp32 is performed here in
numpy float32 (IEEE, correctly rounded, no FMA contraction), so integer/byte
outputs (codes, absmax, int8, layouts) are expected to match the GPU
bit-exactly.  ``ref:`` below means ``/root/reference/``.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
FLT_MAX = np.finfo(np.float32).max

# ---------------------------------------------------------------------------
# Codebooks and thresholds (Appendix B of SURVEY.md)
# ---------------------------------------------------------------------------

# NF4 values returned by the dequantisation tree, ref:sycl/sycl_code/kernel_quant.cpp:650-703
NF4_TREE_VALUES = np.array(
    [-1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453,
     -0.28444138169288635, -0.18477343022823334, -0.09105003625154495, 0.0,
     0.07958029955625534, 0.16093020141124725, 0.24611230194568634, 0.33791524171829224,
     0.44070982933044434, 0.5626170039176941, 0.7229568362236023, 1.0], dtype=F32)

# the same table as the Python layer builds it, ref:python_src_quants/functional.py:1035-1052
NF4_PY_TABLE = [-1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453,
                -0.28444138169288635, -0.18477343022823334, -0.09105003625154495, 0.0,
                0.07958029955625534, 0.16093020141124725, 0.24611230194568634,
                0.33791524171829224, 0.44070982933044434, 0.5626170039176941,
                0.7229568362236023, 1.0]

# NF4 quantisation thresholds (float literals of the decision tree), ascending,
# ref:sycl/sycl_code/kernel_quant.cpp:705-756.  index = #{t : x > t}.
NF4_THRESHOLDS = np.array(
    [-0.8480964004993439, -0.6106329262256622, -0.4599952697753906, -0.33967943489551544,
     -0.23460740596055984, -0.13791173323988914, -0.045525018125772476, 0.03979014977812767,
     0.1202552504837513, 0.2035212516784668, 0.2920137718319893, 0.3893125355243683,
     0.5016634166240692, 0.6427869200706482, 0.8614784181118011], dtype=F32)

# FP4 quantiser tree, ref:sycl/sycl_code/kernel_quant.cpp:547-594.  Restated as a
# count over the sorted magnitude thresholds followed by a count->code map:
# |x|>0.29166667 ? (|x|>0.583333 ? (|x|>0.8333333 ? 3 : 2) : (|x|>0.4166667 ? 5 : 4))
#                : (|x|>0.0859375 ? (|x|>0.20833333 ? 7 : 6) : (|x|>0.00260417 ? 1 : 0))
FP4_MAG_THRESHOLDS = np.array(
    [0.00260417, 0.0859375, 0.20833333, 0.29166667, 0.4166667, 0.583333, 0.8333333], dtype=F32)
FP4_COUNT_TO_CODE = np.array([0b000, 0b001, 0b110, 0b111, 0b100, 0b101, 0b010, 0b011], dtype=np.uint8)

# FP4 dequantisation tree magnitudes indexed by the low 3 bits,
# ref:sycl/sycl_code/kernel_quant.cpp:520-545 (value = c*absmax*sign)
FP4_TREE_MAG = np.array(
    [0.00000000, 5.208333333e-03, 0.66666667, 1.00000000,
     0.33333333, 0.50000000, 0.16666667, 0.25000000], dtype=F32)

# FP4 table of the Python layer (used by gemv as `datatype`), ref:python_src_quants/functional.py:1063
FP4_PY_TABLE = [0, 0.0625, 8.0, 12.0, 4.0, 6.0, 2.0, 3.0, -0, -0.0625, -8.0, -12.0, -4.0, -6.0, -2.0, -3.0]

# LLM.int8 constants, ref:sycl/sycl_code/kernel_quant.cpp:3846 and functional.py:2413-2415
MM_DEQUANT_CONST = F32(6.200012e-05)
STATS_INIT = F32(-50000.0)


def fp4_table() -> np.ndarray:
    """get_4bit_type('fp4') restated: table / max|table| in float32 (functional.py:1063, 1096)."""
    t = np.array(FP4_PY_TABLE, dtype=F32)
    return (t / np.abs(t).max()).astype(F32)


def nf4_table() -> np.ndarray:
    t = np.array(NF4_PY_TABLE, dtype=F32)
    return (t / np.abs(t).max()).astype(F32)


# ---------------------------------------------------------------------------
# dtype helpers (bf16 has no numpy dtype: carried as uint16 bit patterns)
# ---------------------------------------------------------------------------

def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """float32 -> bf16 bits, round-to-nearest-even, NaN kept NaN (quiet)."""
    x = np.ascontiguousarray(x, dtype=F32)
    u = x.view(np.uint32).astype(np.uint64)
    rnd = ((u >> 16) & 1) + 0x7FFF
    out = ((u + rnd) >> 16).astype(np.uint16)
    nan = np.isnan(x)
    out[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return out


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(F32)


def cast_out(v: np.ndarray, out_dtype: str) -> np.ndarray:
    """fp32 -> output dtype with a single round-to-nearest-even cast (kernel_quant.cpp:1428-1453)."""
    v = v.astype(F32)
    if out_dtype == "fp32":
        return v
    if out_dtype == "fp16":
        with np.errstate(over="ignore"):
            return v.astype(np.float16)
    if out_dtype == "bf16":
        return f32_to_bf16_bits(v)
    raise ValueError(out_dtype)


def as_f32(a: np.ndarray, in_dtype: str) -> np.ndarray:
    """Input element -> fp32 (exact for every input dtype)."""
    if in_dtype == "bf16":
        return bf16_bits_to_f32(a)
    return np.asarray(a).astype(F32)


# ---------------------------------------------------------------------------
# scalar codecs (vectorised)
# ---------------------------------------------------------------------------

def quantize_nf4(x: np.ndarray) -> np.ndarray:
    """dQuantizeNF4, kernel_quant.cpp:705-756: strict '>' tree == count of thresholds exceeded; NaN -> 0."""
    x = np.asarray(x, dtype=F32)
    return (x[..., None] > NF4_THRESHOLDS).sum(-1).astype(np.uint8)


def quantize_fp4(x: np.ndarray) -> np.ndarray:
    """dQuantizeFP4, kernel_quant.cpp:547-594: sign bit only for x<0 (NaN, -0.0 -> sign 0)."""
    x = np.asarray(x, dtype=F32)
    sign = np.where(x < 0, 8, 0).astype(np.uint8)
    mag = np.abs(x)
    cnt = (mag[..., None] > FP4_MAG_THRESHOLDS).sum(-1)
    return (FP4_COUNT_TO_CODE[cnt] + sign).astype(np.uint8)


def dequant_fp4_value(q: np.ndarray, absmax: np.ndarray) -> np.ndarray:
    """dDequantizeFP4Tree, kernel_quant.cpp:520-545: (c*absmax)*sign in fp32."""
    q = np.asarray(q, dtype=np.uint8)
    v = (FP4_TREE_MAG[q & 7] * np.asarray(absmax, dtype=F32)).astype(F32)
    return np.where((q & 8) != 0, -v, v).astype(F32)


def dequant_nf4_value(q: np.ndarray, absmax: np.ndarray) -> np.ndarray:
    """dDequantizeNF4(q)*absmax, kernel_quant.cpp:1449-1450."""
    return (NF4_TREE_VALUES[np.asarray(q, dtype=np.uint8)] * np.asarray(absmax, dtype=F32)).astype(F32)


def quantize_8bit_dynamic(code: np.ndarray, x: np.ndarray) -> np.ndarray:
    """dQuantize<STOCHASTIC=0>, kernel_quant.cpp:765-819, restated lane-parallel.

    Binary search over the 256-entry code with pivot 127 and steps 64..1, then
    midpoint rounding against the bracketing pivots (strict comparisons).
    """
    code = np.asarray(code, dtype=F32)
    x = np.asarray(x, dtype=F32)
    shp = x.shape
    x = x.reshape(-1)
    pivot = np.full(x.shape, 127, dtype=np.int64)
    upper_pivot = np.full(x.shape, 255, dtype=np.int64)
    lower_pivot = np.zeros(x.shape, dtype=np.int64)
    lower = np.full(x.shape, -1.0, dtype=F32)
    upper = np.full(x.shape, 1.0, dtype=F32)
    val = code[pivot]
    i = 64
    while i > 0:
        gt = x > val
        lower_pivot = np.where(gt, pivot, lower_pivot)
        lower = np.where(gt, val, lower)
        upper_pivot = np.where(gt, upper_pivot, pivot)
        upper = np.where(gt, upper, val)
        pivot = np.where(gt, pivot + i, pivot - i)
        val = code[pivot]
        i >>= 1
    upper = np.where(upper_pivot == 255, code[255], upper)
    lower = np.where(lower_pivot == 0, code[0], lower)
    gt = x > val
    mid_up = ((upper + val) * F32(0.5)).astype(F32)
    mid_lo = ((lower + val) * F32(0.5)).astype(F32)
    res = np.where(gt,
                   np.where(x > mid_up, upper_pivot, pivot),
                   np.where(x < mid_lo, lower_pivot, pivot))
    return res.astype(np.uint8).reshape(shp)


# ---------------------------------------------------------------------------
# blockwise quantize / dequantize (GPU semantics)
# ---------------------------------------------------------------------------

def block_absmax(x: np.ndarray, blocksize: int) -> np.ndarray:
    """Per-block max|x| in fp32, kernel_quant.cpp:1285-1298.

    fmax-reduction seeded with -FLT_MAX (NaN elements are ignored by fmax); a
    partial tail block is zero-filled (upstream BlockLoad fill value 0.0f), so
    its absmax is max(0, ...).
    """
    n = x.size
    nb = (n + blocksize - 1) // blocksize
    pad = nb * blocksize - n
    xa = np.abs(x.astype(F32))
    if pad:
        xa = np.concatenate([xa, np.zeros(pad, dtype=F32)])
    xa = xa.reshape(nb, blocksize)
    m = np.fmax.reduce(xa, axis=1, initial=-FLT_MAX)
    return m.astype(F32)


def quantize_blockwise(x: np.ndarray, blocksize: int, qtype: str, code: np.ndarray | None = None):
    """kQuantizeBlockwise<T,BS,NPT,0,DT> (kernel_quant.cpp:1229-1365) with the intended
    full-size semantics.

    x: fp32 values (already converted from the input dtype).  Returns (absmax fp32[nb],
    packed uint8): 4-bit -> ceil(n/2) bytes, byte j = q(x[2j])<<4 | q(x[2j+1]);
    8-bit -> n bytes.
    """
    x = np.asarray(x, dtype=F32).reshape(-1)
    n = x.size
    absmax = block_absmax(x, blocksize)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = (F32(1.0) / absmax).astype(F32)               # kernel_quant.cpp:1304 (IEEE reciprocal)
        rr = np.repeat(r, blocksize)[:n]
        xn = (x * rr).astype(F32)                         # kernel_quant.cpp:1328/1337/1346
    if qtype == "8bit":
        assert code is not None
        return absmax, quantize_8bit_dynamic(code, xn)
    if n % 2:
        # the zero fill element of the tail block: 0 * r
        with np.errstate(invalid="ignore"):
            xn = np.concatenate([xn, (F32(0.0) * rr[-1:]).astype(F32)])
    q = quantize_nf4(xn) if qtype == "nf4" else quantize_fp4(xn)
    packed = ((q[0::2] << 4) | q[1::2]).astype(np.uint8)
    return absmax, packed


def dequantize_blockwise(packed: np.ndarray, absmax: np.ndarray, blocksize: int, n: int,
                         qtype: str, out_dtype: str, code: np.ndarray | None = None) -> np.ndarray:
    """kDequantizeBlockwise (kernel_quant.cpp:1370-1471) + launcher (op_quant.cpp:659-703):
    element i uses absmax[i // blocksize]; value computed in fp32 then one RNE cast."""
    absmax = np.asarray(absmax, dtype=F32)
    am = np.repeat(absmax, blocksize)[:n]
    if qtype == "8bit":
        v = (np.asarray(code, dtype=F32)[np.asarray(packed, dtype=np.uint8)[:n]] * am).astype(F32)
    else:
        p = np.asarray(packed, dtype=np.uint8)
        q = np.empty(p.size * 2, dtype=np.uint8)
        q[0::2] = p >> 4          # high nibble = even element (kernel_quant.cpp:1441, 1449)
        q[1::2] = p & 0x0F
        q = q[:n]
        v = dequant_nf4_value(q, am) if qtype == "nf4" else dequant_fp4_value(q, am)
    return cast_out(v, out_dtype)


def unpack_4bit(packed: np.ndarray, n: int) -> np.ndarray:
    p = np.asarray(packed, dtype=np.uint8).reshape(-1)
    q = np.empty(p.size * 2, dtype=np.uint8)
    q[0::2] = p >> 4
    q[1::2] = p & 0x0F
    return q[:n]


def nested_absmax(qabsmax: np.ndarray, absmax2: np.ndarray, code: np.ndarray, offset: np.float32,
                  blocksize2: int = 256) -> np.ndarray:
    """Nested statistics (functional.py:1243-1257, 1346-1350, 1982-1984):
    absmax = dequantize_blockwise(qabsmax, state2) + offset, all fp32."""
    n = qabsmax.size
    a = dequantize_blockwise(qabsmax, absmax2, blocksize2, n, "8bit", "fp32", code=code)
    return (a + F32(offset)).astype(F32)


# ---------------------------------------------------------------------------
# 4-bit GEMV / GEMM (floating point: tolerance-based parity)
# ---------------------------------------------------------------------------

def dequant_weight_f32(packed: np.ndarray, absmax: np.ndarray, N: int, K: int, blocksize: int,
                       table: np.ndarray) -> np.ndarray:
    """W[n,k] = table[q]*absmax[(n*K+k)//blocksize] in fp32, the per-element weight the
    gemv kernel forms (kernel_gemm.cpp:1299-1381, with the Q8 T-precision quirk removed)."""
    q = unpack_4bit(packed, N * K).reshape(N, K)
    am = np.repeat(np.asarray(absmax, dtype=F32), blocksize)[: N * K].reshape(N, K)
    return (np.asarray(table, dtype=F32)[q] * am).astype(F32)


def gemv_4bit(x: np.ndarray, packed: np.ndarray, absmax: np.ndarray, N: int, K: int,
              blocksize: int, table: np.ndarray) -> np.ndarray:
    """out[n] = sum_k x[k] * W[n,k], fp64 accumulation (kgemm_4bit_inference_naive semantics)."""
    W = dequant_weight_f32(packed, absmax, N, K, blocksize, table).astype(np.float64)
    return W @ np.asarray(x, dtype=np.float64).reshape(K)


def round_to(x: np.ndarray, dtype: str) -> np.ndarray:
    """fp32 -> T -> fp32 with one round-to-nearest-even (T = bf16 or fp16)."""
    x = np.asarray(x, dtype=F32)
    if dtype == "bf16":
        return bf16_bits_to_f32(f32_to_bf16_bits(x))
    if dtype == "fp16":
        return x.astype(np.float16).astype(F32)
    return x


def gemv_4bit_ref_faithful(x: np.ndarray, packed: np.ndarray, absmax: np.ndarray, N: int, K: int,
                           blocksize: int, table: np.ndarray, dtype: str) -> np.ndarray:
    """The reference GEMV WITH its T-precision arithmetic: kgemm_4bit_inference_naive
    (ref:sycl/sycl_code/kernel_gemm.cpp:1291-1294, 1305, 1336-1343, DPCT_COMPATIBILITY_TEMP >= 800 branch) holds the
    16-entry code table and the block absmax in T (`quant_map[i] = T(datatype[i])`, `T local_absmax`), forms each
    weight as a T product (`local_B = quant_map[q] * local_absmax`, rounded to T) and each activation x weight product
    in T (`(float)(local_A[k] * local_B[k])`), accumulating those in fp32.  Here: the same roundings, the sum of the
    T-rounded products in fp64 (the kernel's per-lane fp32 order differs from any fixed order by far less than the
    T roundings).  x is given as its T values."""
    q = unpack_4bit(packed, N * K).reshape(N, K)
    tab = round_to(np.asarray(table, dtype=F32), dtype)
    am = round_to(np.repeat(np.asarray(absmax, dtype=F32), blocksize)[: N * K].reshape(N, K), dtype)
    w = round_to(tab[q] * am, dtype)
    prod = round_to(w * round_to(np.asarray(x, dtype=F32).reshape(1, K), dtype), dtype)
    return prod.astype(np.float64).sum(axis=1)


def gemm_4bit_dequant_ref(X: np.ndarray, packed: np.ndarray, absmax: np.ndarray, N: int, K: int,
                          blocksize: int, table: np.ndarray, weight_dtype: str = "bf16") -> np.ndarray:
    """Reference M>1 path (autograd/_functions.py:507): W = dequantize_4bit (one RNE cast to the
    compute dtype), then linear; accumulated in fp64 here."""
    W = dequant_weight_f32(packed, absmax, N, K, blocksize, table)
    if weight_dtype == "bf16":
        W = bf16_bits_to_f32(f32_to_bf16_bits(W))
    elif weight_dtype == "fp16":
        W = W.astype(np.float16).astype(F32)
    return np.asarray(X, dtype=np.float64) @ W.astype(np.float64).T


# ---------------------------------------------------------------------------
# LLM.int8: statistics, double quant, igemmlt, mm_dequant
# ---------------------------------------------------------------------------

def colrow_absmax(A: np.ndarray, threshold: float = 0.0):
    """get_colrow_absmax (functional.py:2400-2435) + kgetColRowStats (kernel_quant.cpp:3214-3379),
    intended semantics (Q6: max over all items).  With threshold>0 the SPARSE_DECOMP branch
    (3292-3301): |a| >= threshold is excluded (zeroed) and counted per row."""
    a = np.abs(np.asarray(A, dtype=np.float16).astype(F32))
    nnz_rows = None
    if threshold > 0.0:
        mask = a >= F32(threshold)
        nnz_rows = mask.sum(1).astype(np.int32)
        a = np.where(mask, F32(0.0), a)
    row = np.maximum(STATS_INIT, np.fmax.reduce(a, axis=1, initial=-FLT_MAX)).astype(F32)
    col = np.maximum(STATS_INIT, np.fmax.reduce(a, axis=0, initial=-FLT_MAX)).astype(F32)
    return row, col, nnz_rows


def _rint_to_int8(v: np.ndarray) -> np.ndarray:
    """(char)rint(v): round-half-even; NaN -> 0 (GPU cvt semantics); saturate to int8."""
    r = np.rint(v)
    r = np.where(np.isnan(r), 0, r)
    r = np.clip(r, -128, 127)
    return r.astype(np.int8)


def double_quant(A: np.ndarray, row_stats: np.ndarray, col_stats: np.ndarray, threshold: float = 0.0):
    """kDoubleRowColQuant, kernel_quant.cpp:3424, 3453-3496:
    out_row = (int8)rint(a * (127.0f/rowStats[r])); out_col = (int8)rint(a * (127.0f/colStats[c])).
    With threshold>0, |a|>=threshold gives 0 in out_row (outliers go to COO)."""
    a = np.asarray(A, dtype=np.float16).astype(F32)
    with np.errstate(divide="ignore", invalid="ignore"):
        rs = (F32(127.0) / np.asarray(row_stats, dtype=F32)).astype(F32)
        cs = (F32(127.0) / np.asarray(col_stats, dtype=F32)).astype(F32)
        out_row = _rint_to_int8((a * rs[:, None]).astype(F32))
        out_col = _rint_to_int8((a * cs[None, :]).astype(F32))
    if threshold > 0.0:
        out_row = np.where(np.abs(a) >= F32(threshold), np.int8(0), out_row).astype(np.int8)
    return out_row, out_col


def igemmlt(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    """C = A @ B^T exact int32 (op_gemm.cpp:541-655 contract; test_matmulqlt.py:194-204 exactness)."""
    return (np.asarray(A, dtype=np.int64) @ np.asarray(B, dtype=np.int64).T).astype(np.int32)


def igemmlt_int8_out(A, B, row_scale=None):
    """int8-output variants (cigemmlt_*_8 / _8_rowscale): sat_int8(rint(acc * alpha)), alpha=1 or per-row."""
    acc = igemmlt(A, B).astype(F32)
    if row_scale is not None:
        acc = (acc * np.asarray(row_scale, dtype=F32)[:, None]).astype(F32)
    return _rint_to_int8(acc)


def mm_dequant(C: np.ndarray, row_stats: np.ndarray, col_stats: np.ndarray, bias=None) -> np.ndarray:
    """kdequant_mm_int32_fp16, kernel_quant.cpp:3969 operation order, fp32, no contraction:
    half( ((float(C) * 6.200012e-05f) * rowStat) * colStat + bias )."""
    c = np.asarray(C, dtype=np.int32).astype(F32)
    v = (c * MM_DEQUANT_CONST).astype(F32)
    v = (v * np.asarray(row_stats, dtype=F32)[:, None]).astype(F32)
    v = (v * np.asarray(col_stats, dtype=F32)[None, :]).astype(F32)
    if bias is not None:
        v = (v + np.asarray(bias, dtype=np.float16).astype(F32)[None, :]).astype(F32)
    with np.errstate(over="ignore"):
        return v.astype(np.float16)


# ---------------------------------------------------------------------------
# Tile layouts (blas_utils.h:244-346; kernel_quant.cpp:3640-3835; functional.py:482-518)
# ---------------------------------------------------------------------------

def _pad(v, m):
    return (v + m - 1) // m * m


def layout_shape(rows: int, cols: int, fmt: str):
    if fmt == "col32":
        return rows, _pad(cols, 32)
    if fmt == "col_turing":
        return _pad(rows, 8), _pad(cols, 32)
    if fmt == "col_ampere":
        return _pad(rows, 32), _pad(cols, 32)
    raise ValueError(fmt)


def layout_offsets(rows: int, cols: int, fmt: str) -> np.ndarray:
    """Linear offset of element (r, c) of a [rows, cols] matrix in format `fmt`.

    col32      : (c//32)*(32*rows) + 32*r + c%32                                (kernel_quant.cpp:3675-3676)
    col_turing : (c//32)*(32*R8) + (r//8)*256 + 128*(r%2) + 16*(c//4 % 8) + 4*((r%8)//2) + c%4
                 (blas_utils.h:283-300 col4_4r2_8c; == kernel_quant.cpp:3729-3745)
    col_ampere : (c//32)*(32*R32) + (r//32)*1024 + 32*ampere_row(r%32) + c%32,
                 ampere_row(x) = 8*((x%8)//2) + 2*(x//8) + x%2   (blas_utils.h:318-330; kernel_quant.cpp:3808-3829)
    """
    r = np.arange(rows, dtype=np.int64)[:, None]
    c = np.arange(cols, dtype=np.int64)[None, :]
    if fmt == "col32":
        return (c // 32) * (32 * rows) + 32 * r + c % 32
    if fmt == "col_turing":
        R8 = _pad(rows, 8)
        rr, cc = r % 8, c % 32
        to_row = 4 * (rr % 2) + cc // 8
        to_col = 16 * ((cc // 4) % 2) + 4 * (rr // 2) + cc % 4
        return (c // 32) * (32 * R8) + (r // 8) * 256 + to_row * 32 + to_col
    if fmt == "col_ampere":
        R32 = _pad(rows, 32)
        rr = r % 32
        to_row = 8 * ((rr % 8) // 2) + (rr // 8) * 2 + rr % 2
        return (c // 32) * (32 * R32) + (r // 32) * 1024 + to_row * 32 + c % 32
    raise ValueError(fmt)


def layout_offsets_kernel_form(rows: int, cols: int, fmt: str) -> np.ndarray:
    """Same maps written the way the SYCL kernel writes them (kernel_quant.cpp:3670-3835,
    non-transposed branches) — used to cross-check the blas_utils form above."""
    off = np.zeros((rows, cols), dtype=np.int64)
    for r in range(rows):
        for c in range(cols):
            if fmt == "col32":
                off[r, c] = (c // 32) * (32 * rows) + r * 32 + c % 32
            elif fmt == "col_turing":
                outRows = _pad(rows, 8)
                o = (c // 32) * outRows * 32 + (r // 8) * 256
                sub, subcol = r % 8, c % 32
                if sub % 2 == 1:
                    o += 128 + (subcol // 4) * 16 + (subcol % 4) + ((sub % 8) - 1) * 2
                else:
                    o += (subcol // 4) * 16 + (subcol % 4) + (sub % 8) * 2
                off[r, c] = o
            else:
                outRows = _pad(rows, 32)
                o = (c // 32) * outRows * 32 + (r // 32) * 1024
                sub = r % 32
                local_row = ((sub % 8) // 2) * 8 + (sub // 8) * 2 + (sub % 2)
                off[r, c] = o + local_row * 32 + c % 32
    return off


def transform(A: np.ndarray, fmt: str, transpose: bool = False) -> np.ndarray:
    """ctransform_row2{col32,turing,ampere}{,T}: row-major int8 [rows, cols] -> fmt buffer of A
    (or of A^T when transpose), zero padded (get_transform_buffer uses torch.zeros)."""
    A = np.asarray(A)
    if transpose:
        A = A.T
    rows, cols = A.shape
    R, C = layout_shape(rows, cols, fmt)
    out = np.zeros(R * C, dtype=A.dtype)
    out[layout_offsets(rows, cols, fmt).reshape(-1)] = A.reshape(-1)
    return out.reshape(R, C)


def untransform(buf: np.ndarray, rows: int, cols: int, fmt: str) -> np.ndarray:
    return np.asarray(buf).reshape(-1)[layout_offsets(rows, cols, fmt)]


# ---------------------------------------------------------------------------
# CPU path (config 1 baseline semantics): cpu_ops.cpp + common.cpp
# ---------------------------------------------------------------------------

def dequantize_cpu(code: np.ndarray, A: np.ndarray, absmax: np.ndarray, blocksize: int) -> np.ndarray:
    """dequantize_cpu, ref:sycl/cpu_ops.cpp:7-14: out[i] = code[A[i]] * absmax[i/bs] (fp32)."""
    n = A.size
    am = np.repeat(np.asarray(absmax, dtype=F32), blocksize)[:n]
    return (np.asarray(code, dtype=F32)[A] * am).astype(F32)


def quantize_cpu(code: np.ndarray, A: np.ndarray, blocksize: int):
    """quantize_cpu/quantize_block, ref:sycl/cpu_ops.cpp:16-63, common.cpp:4-35.

    code[0] is forced to -1.0 (in place in the reference, Q15); absmax = fmax over |A|
    from -FLT_MAX; z = A/absmax (division, Q16); idx = largest i with code[i] <= z
    (BinAlgo Direct2 left neighbour, clamped to [0,255]); move right iff strictly closer."""
    code = np.array(code, dtype=F32, copy=True)
    code[0] = F32(-1.0)
    A = np.asarray(A, dtype=F32).reshape(-1)
    n = A.size
    nb = (n + blocksize - 1) // blocksize
    absmax = np.empty(nb, dtype=F32)
    out = np.empty(n, dtype=np.uint8)
    for b in range(nb):
        blk = A[b * blocksize:(b + 1) * blocksize]
        m = np.fmax.reduce(np.abs(blk), initial=-FLT_MAX).astype(F32)
        absmax[b] = m
        with np.errstate(divide="ignore", invalid="ignore"):
            z = (blk / m).astype(F32)
        idx = np.searchsorted(code, z, side="right") - 1
        idx = np.clip(idx, 0, 255)
        idx = np.where(np.isnan(z), 0, idx)
        nxt = np.minimum(idx + 1, 255)
        dl = np.abs((z - code[idx]).astype(F32))
        dr = np.abs((z - code[nxt]).astype(F32))
        idx = np.where((idx < 255) & (dr < dl), idx + 1, idx)
        out[b * blocksize:(b + 1) * blocksize] = idx
    return absmax, out, code
