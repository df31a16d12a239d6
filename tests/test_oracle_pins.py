"""Pin the CPU oracle against the reference's own source constants (no GPU needed).

The reference has no golden vectors; each check below cross-validates two places in the
reference source that must agree, or a property the reference's constants imply.
"""
import numpy as np

from oracle import ref
from oracle.maps import create_dynamic_map

F32 = np.float32


def test_nf4_tree_equals_python_table():
    # kernel_quant.cpp:650-703 (dequant tree) == functional.py:1035-1052 (get_4bit_type('nf4'))
    assert np.array_equal(ref.NF4_TREE_VALUES, ref.nf4_table())
    assert np.all(np.diff(ref.NF4_TREE_VALUES) > 0)


def test_nf4_thresholds_are_midpoints():
    # kernel_quant.cpp:705-756 thresholds are the midpoints of consecutive NF4 values (nearest rounding)
    mids = ((ref.NF4_TREE_VALUES[:-1].astype(np.float64) + ref.NF4_TREE_VALUES[1:]) / 2).astype(F32)
    assert np.max(np.abs(mids - ref.NF4_THRESHOLDS)) < 2e-7


def test_nf4_quantize_table_roundtrip_and_ties():
    q = ref.quantize_nf4(ref.NF4_TREE_VALUES)
    assert np.array_equal(q, np.arange(16))
    # strict '>' : a value exactly at a threshold goes to the lower code
    assert np.array_equal(ref.quantize_nf4(ref.NF4_THRESHOLDS), np.arange(15))
    assert np.array_equal(ref.quantize_nf4(np.nextafter(ref.NF4_THRESHOLDS, F32(2))), np.arange(1, 16))
    assert ref.quantize_nf4(np.array([np.nan], F32))[0] == 0


def test_fp4_tree_matches_python_table():
    # dDequantizeFP4Tree values (kernel_quant.cpp:520-545) == get_4bit_type('fp4') / 12 (functional.py:1063)
    t = ref.fp4_table()
    codes = np.arange(16, dtype=np.uint8)
    tree = ref.dequant_fp4_value(codes, F32(1.0))
    assert np.array_equal(tree, t)   # == also equates the tree's -0.0 (code 8) with the table's int `-0` -> +0.0
    nz = t != 0
    assert np.array_equal(np.signbit(tree[nz]), np.signbit(t[nz]))
    assert np.signbit(tree[8]) and not np.signbit(t[8])


def test_fp4_quantizer_is_nearest_magnitude():
    # every tree threshold lies between the two magnitudes it separates (kernel_quant.cpp:547-594)
    mags = ref.FP4_TREE_MAG[ref.FP4_COUNT_TO_CODE]        # magnitudes in count order
    assert np.all(np.diff(mags) > 0)
    th = ref.FP4_MAG_THRESHOLDS
    assert np.all((th > mags[:-1]) & (th < mags[1:]))
    # quantising each magnitude returns its own code, with and without sign
    q = ref.quantize_fp4(mags)
    assert np.array_equal(q, ref.FP4_COUNT_TO_CODE)
    qn = ref.quantize_fp4(-mags[1:])
    assert np.array_equal(qn, ref.FP4_COUNT_TO_CODE[1:] | 8)
    assert ref.quantize_fp4(np.array([-0.0, np.nan], F32)).tolist() == [0, 0]


def test_dynamic_map_properties():
    code = create_dynamic_map()
    assert code.dtype == np.float32 and code.shape == (256,)
    assert np.all(np.diff(code) >= 0)
    assert code[-1] == 1.0 and 0.0 in code
    # quantising the code's own values returns their index (dQuantize<0>, kernel_quant.cpp:765-819)
    idx = ref.quantize_8bit_dynamic(code, code)
    assert np.array_equal(code[idx], code)


def test_mm_dequant_constant():
    # kernel_quant.cpp:3846: 6.200012e-05f ~= 1/(127*127)
    assert abs(float(ref.MM_DEQUANT_CONST) - 1 / (127 * 127)) < 1e-10


def test_layout_maps_two_forms_agree():
    # blas_utils.h:244-346 index maps == kernel_quant.cpp:3640-3835 kernel arithmetic
    for rows, cols in ((8, 32), (40, 96), (33, 70)):
        for fmt in ("col32", "col_turing", "col_ampere"):
            a = ref.layout_offsets(rows, cols, fmt)
            b = ref.layout_offsets_kernel_form(rows, cols, fmt)
            assert np.array_equal(a, b), fmt
            R, C = ref.layout_shape(rows, cols, fmt)
            assert len(np.unique(a)) == rows * cols and a.max() < R * C


def test_transform_roundtrip():
    rng = np.random.default_rng(0)
    A = rng.integers(-127, 128, size=(37, 75), dtype=np.int8)
    for fmt in ("col32", "col_turing", "col_ampere"):
        buf = ref.transform(A, fmt)
        assert np.array_equal(ref.untransform(buf, 37, 75, fmt), A)
        bufT = ref.transform(A, fmt, transpose=True)
        assert np.array_equal(ref.untransform(bufT, 75, 37, fmt), A.T)


def test_blockwise_roundtrip_error_bounds():
    # dequant(quant(x)) error bounded by half the largest code gap times absmax
    rng = np.random.default_rng(3)
    x = rng.standard_normal(64 * 50).astype(F32)
    gap_nf4 = float(np.diff(ref.NF4_TREE_VALUES).max())
    gap_fp4 = float(np.diff(np.sort(ref.FP4_TREE_MAG)).max())
    for qtype, gap in (("nf4", gap_nf4), ("fp4", gap_fp4)):
        absmax, q = ref.quantize_blockwise(x, 64, qtype)
        y = ref.dequantize_blockwise(q, absmax, 64, x.size, qtype, "fp32")
        err = np.abs(y - x) / np.repeat(absmax, 64)
        assert err.max() <= gap / 2 + 1e-6


def test_zero_block_semantics():
    # absmax 0 -> 1/0 = inf -> 0*inf = NaN -> code 0 (NF4 -1.0) -> dequant -1*0 = -0.0
    x = np.zeros(64, F32)
    absmax, q = ref.quantize_blockwise(x, 64, "nf4")
    assert absmax[0] == 0 and np.all(q == 0)
    y = ref.dequantize_blockwise(q, absmax, 64, 64, "nf4", "fp32")
    assert np.all(y == 0) and np.all(np.signbit(y))


def test_double_quant_and_stats_semantics():
    A = np.array([[1.0, -2.0, 0.5], [0.0, 0.0, 0.0], [127.0, 3.0, -64.0]], np.float16)
    rs, cs, _ = ref.colrow_absmax(A)
    assert rs.tolist() == [2.0, 0.0, 127.0] and cs.tolist() == [127.0, 3.0, 64.0]
    orow, ocol = ref.double_quant(A, rs, cs)
    assert orow[0].tolist() == [64, -127, 32]       # rint(63.5)=64 (half-even), 127/2*-2, 31.75->32
    assert orow[1].tolist() == [0, 0, 0]            # 0 * inf = NaN -> 0
    assert ocol[2].tolist() == [127, 127, -127]


def test_igemm_exact_and_mm_dequant_order():
    rng = np.random.default_rng(1)
    A = rng.integers(-127, 128, size=(8, 64), dtype=np.int8)
    B = rng.integers(-127, 128, size=(5, 64), dtype=np.int8)
    C = ref.igemmlt(A, B)
    assert np.array_equal(C, A.astype(np.int64) @ B.astype(np.int64).T)
    rs = np.full(8, 2.0, F32)
    cs = np.full(5, 0.5, F32)
    D = ref.mm_dequant(C, rs, cs)
    assert np.allclose(D.astype(np.float64), C / (127.0 * 127.0), rtol=2e-3, atol=1e-3)


def test_cpu_path_semantics():
    code = create_dynamic_map()
    A = np.array([0.5, -1.0, 0.25, 0.0], F32)
    absmax, q, code2 = ref.quantize_cpu(code, A, 4)
    assert code2[0] == -1.0 and absmax[0] == 1.0
    assert q[1] == 0                   # -1 -> forced code[0]
    y = ref.dequantize_cpu(code2, q, absmax, 4)
    assert np.abs(y - A).max() < 0.02


def test_gemv_tolerance_covers_ref_faithful_variant():
    """Q8 on the CPU: the reference GEMV's T-precision arithmetic (oracle.ref.gemv_4bit_ref_faithful, table / absmax /
    weights / products rounded to T, ref:sycl/sycl_code/kernel_gemm.cpp:1291-1294, 1336-1343) stays inside the stated
    GEMV tolerance of the fp64 oracle (2e-2 bf16, 1e-2 fp16 of rms + |ref|), so the tolerance covers both the
    reference's rounding and this build's fp32 weights.  The GPU test at config 2 is
    test_matmul4bit_gpu.py::test_gemv_c2_tolerance_covers_ref_faithful_variant."""
    rng = np.random.default_rng(8)
    N, K = 1024, 4096
    W = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    for qt in ("nf4", "fp4"):
        am, q = ref.quantize_blockwise(W.reshape(-1), 64, qt)
        table = ref.nf4_table() if qt == "nf4" else ref.fp4_table()
        for dt, tol in (("bf16", 2e-2), ("fp16", 1e-2)):
            x = ref.round_to(rng.standard_normal(K).astype(np.float32), dt)
            exp = ref.gemv_4bit(x, q, am, N, K, 64, table)
            got = ref.gemv_4bit_ref_faithful(x, q, am, N, K, 64, table, dt)
            rms = np.sqrt(np.mean(exp ** 2))
            assert np.all(np.abs(got - exp) <= tol * rms + tol * np.abs(exp)), (qt, dt)
            assert not np.array_equal(got, exp)      # the variant does round differently
