"""GPU parity: 4-bit GEMV (decode) and the fused 4-bit GEMM (prefill) vs the CPU oracle.

Floating point, so parity is a tolerance: rtol = 2e-2 and
atol = 2e-2 * rms(out) for bf16 outputs (fp16: 1e-2), against an fp64 restatement; plus the
reference test's own bound mean|out - out_fp| < 0.115 (tests_pvc/autograd.py:388-391).
"""
import ctypes as ct

import numpy as np
import pytest
import torch

from helpers import to_numpy, to_torch
from oracle import ref

pytestmark = pytest.mark.gpu


def _F():
    import python_src_quants.functional as F
    return F


@pytest.fixture(autouse=True)
def _static_route(monkeypatch):
    """These are kernel tests: pin the static route rule, so a shape above the few-token range reaches the kernel under
    test instead of whichever route the measurement (functional.GEMM_4BIT_ROUTE_TUNING) found faster on this box.
    The measured route itself is tested in test_configs_gpu.py."""
    monkeypatch.setattr(_F(), "GEMM_4BIT_ROUTE_TUNING", False)


def _lib_matmul(F, X, Wd):
    """X @ Wd^T through the library GEMM the product's large-prefill route uses (cgemm_tn_*, gemm_lib.hip) with the
    plan cached for this shape: the reference's F.linear on the dequantised weight."""
    m, k = X.shape
    n = Wd.shape[0]
    out = torch.empty(m, n, device=X.device, dtype=X.dtype)
    fn = F.lib.cgemm_tn_bf16 if X.dtype == torch.bfloat16 else F.lib.cgemm_tn_fp16
    F.pre_call(X.device)
    assert fn(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k), F.get_ptr(X), ct.c_int32(k), F.get_ptr(Wd), ct.c_int32(k),
              F.get_ptr(out), ct.c_int32(n)) == 0
    return out


def _close(got, exp, rtol, arel):
    got = np.asarray(got, np.float64)
    exp = np.asarray(exp, np.float64)
    atol = arel * np.sqrt(np.mean(exp**2)) + 1e-30
    bad = np.abs(got - exp) > atol + rtol * np.abs(exp)
    return bad.mean(), np.abs(got - exp).max()


def test_gemv_golden(golden, dev):
    F = _F()
    N, K, bs = golden["gemv_meta"].tolist()
    x = to_torch(golden["gemv_x"], "bf16", dev)
    q = torch.from_numpy(golden["gemv_q"]).to(dev)
    absmax = torch.from_numpy(golden["gemv_absmax"]).to(dev)
    code = torch.from_numpy(ref.nf4_table()).to(dev)
    out = torch.empty(N, dtype=torch.bfloat16, device=dev)
    F.lib.cgemm_4bit_inference_naive_bf16(ct.c_int32(N), ct.c_int32(1), ct.c_int32(K), F.get_ptr(x), F.get_ptr(q),
                                          F.get_ptr(absmax), F.get_ptr(code), F.get_ptr(out), ct.c_int32(N),
                                          ct.c_int32(K // 2), ct.c_int32(N), ct.c_int32(bs))
    torch.cuda.synchronize()
    frac, _ = _close(ref.bf16_bits_to_f32(to_numpy(out, "bf16")), golden["gemv_y"], 2e-2, 2e-2)
    assert frac == 0.0


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("qt", ["nf4", "fp4"])
@pytest.mark.parametrize("shape", [(11008, 4096), (4096, 11008), (1000, 192), (77, 64 * 33), (300, 6144),
                                   (37, 40960)])
def test_gemv_functional(dev, dtype, qt, shape):
    F = _F()
    N, K = shape
    torch.manual_seed(N + K)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    for nested in (False, True):
        q, st = F.quantize_4bit(W, blocksize=64, quant_type=qt, compress_statistics=nested)
        x = torch.randn(1, K, device=dev, dtype=dtype)
        y = F.gemv_4bit(x, q.t(), state=st)
        assert y.shape == (1, N) and y.dtype == dtype
        absmax = F._absmax_fp32(st).cpu().numpy()
        exp = ref.gemv_4bit(x.float().cpu().numpy()[0], q.cpu().numpy(), absmax, N, K, 64, st.code.cpu().numpy())
        tol = {torch.bfloat16: 2e-2, torch.float16: 1e-2, torch.float32: 1e-4}[dtype]
        frac, err = _close(y.float().cpu().numpy()[0], exp, tol, tol)
        assert frac == 0.0, (nested, err)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("qt", ["nf4", "fp4"])
def test_gemv_c2_tolerance_covers_ref_faithful_variant(dev, dtype, nested, qt):
    """Q8: the reference's GEMV holds the code table and absmax in T and rounds every weight and
    every x * w product to T (ref:sycl/sycl_code/kernel_gemm.cpp:1291-1294, 1305, 1336-1343); this build computes
    the weight in fp32 and accumulates fp32 dot products.  At config 2 (11008 x 4096) both the HIP output and the
    ref-faithful restatement (oracle.ref.gemv_4bit_ref_faithful) sit within the stated tolerance of the fp64 oracle
    (|d| <= tol * rms + tol * |ref|, tol 2e-2 bf16 / 1e-2 fp16), and within twice it of each other."""
    F = _F()
    N, K = 11008, 4096
    torch.manual_seed(41 + nested)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type=qt, compress_statistics=nested)
    del W
    x = torch.randn(1, K, device=dev, dtype=dtype)
    y = F.gemv_4bit(x, q.t(), state=st).float().cpu().numpy()[0]
    absmax = F._absmax_fp32(st).cpu().numpy()
    xn, qn, code = x.float().cpu().numpy()[0], q.cpu().numpy(), st.code.cpu().numpy()
    exp = ref.gemv_4bit(xn, qn, absmax, N, K, 64, code)
    faithful = ref.gemv_4bit_ref_faithful(xn, qn, absmax, N, K, 64, code, "bf16" if dtype == torch.bfloat16 else "fp16")
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-2
    frac, err = _close(y, exp, tol, tol)
    assert frac == 0.0, ("hip", err)
    frac, err = _close(faithful, exp, tol, tol)
    assert frac == 0.0, ("ref-faithful", err)
    frac, err = _close(y, faithful, 2 * tol, 2 * tol)
    assert frac == 0.0, ("hip vs ref-faithful", err)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(11008, 4096), (513, 6144), (4096, 11008), (64, 192)])
def test_gemv_nested_fused_matches_two_step(dev, dtype, shape):
    """The in-kernel decode of compressed statistics is bit-identical to dequantize_blockwise(absmax) +
    offset (ref:functional.py:1982-1984) followed by the plain GEMV."""
    F = _F()
    N, K = shape
    torch.manual_seed(7)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    x = torch.randn(1, K, device=dev, dtype=dtype)
    fused = F.gemv_4bit(x, q.t(), state=st)
    absmax = F._absmax_fp32(st)
    ref_out = torch.empty_like(fused)
    name = {torch.bfloat16: "bf16", torch.float16: "fp16"}[dtype]
    getattr(F.lib, f"cgemm_4bit_inference_naive_{name}")(
        ct.c_int32(N), ct.c_int32(1), ct.c_int32(K), F.get_ptr(x), F.get_ptr(q), F.get_ptr(absmax),
        F.get_ptr(st.code), F.get_ptr(ref_out), ct.c_int32(N), ct.c_int32(K // 2), ct.c_int32(N), ct.c_int32(64))
    torch.cuda.synchronize()
    assert torch.equal(fused.view(torch.int16), ref_out.view(torch.int16))


def test_gemv_generic_path(dev):
    """K not a multiple of 32 / unaligned B -> the general kernel path."""
    F = _F()
    N, K, bs = 50, 64 * 3 + 30, 64
    rng = np.random.default_rng(2)
    w = (rng.standard_normal(N * K) * 0.1).astype(np.float32)
    absmax, q = ref.quantize_blockwise(w, bs, "nf4")      # flat blocks straddle rows: (r*K + k)/bs
    ldb = (K + 1) // 2
    x = rng.standard_normal(K).astype(np.float32)
    X = torch.from_numpy(x).to(dev)
    Q = torch.from_numpy(q).to(dev)
    AM = torch.from_numpy(absmax).to(dev)
    code = torch.from_numpy(ref.nf4_table()).to(dev)
    out = torch.empty(N, device=dev)
    F.lib.cgemm_4bit_inference_naive_fp32(ct.c_int32(N), ct.c_int32(1), ct.c_int32(K), F.get_ptr(X), F.get_ptr(Q),
                                          F.get_ptr(AM), F.get_ptr(code), F.get_ptr(out), ct.c_int32(N),
                                          ct.c_int32(ldb), ct.c_int32(N), ct.c_int32(bs))
    torch.cuda.synchronize()
    exp = ref.gemv_4bit(x, q, absmax, N, K, bs, ref.nf4_table())
    assert np.allclose(out.cpu().numpy(), exp, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("qt", ["nf4", "fp4"])
@pytest.mark.parametrize("mnk", [(1, 256, 128), (130, 300, 320), (256, 384, 1024), (64, 128, 64), (333, 1000, 576)])
def test_gemm_4bit_vs_oracle(dev, dtype, qt, mnk):
    F = _F()
    M, N, K = mnk
    torch.manual_seed(M * 31 + N)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    X = torch.randn(M, K, device=dev, dtype=dtype)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type=qt)
    Y = F.gemm_4bit(X, q, st)
    assert Y.shape == (M, N) and Y.dtype == dtype
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), st.absmax.cpu().numpy(), N, K, 64,
                                    st.code.cpu().numpy(), "bf16" if dtype == torch.bfloat16 else "fp16")
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-2
    frac, err = _close(Y.float().cpu().numpy(), exp, tol, tol)
    assert frac == 0.0, err
    # the reference path for M>1 (dequantize_4bit + linear) agrees too
    Wd = F.dequantize_4bit(q, st)
    Yref = torch.nn.functional.linear(X.float(), Wd.float())
    assert (Y.float() - Yref).abs().mean().item() < 0.115


@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("mnk", [(1024, 128, 2048), (2000, 100, 4096), (4096, 200, 1024), (700, 64, 8192)])
def test_gemm_4bit_narrow_weight_split_k(dev, nested, mnk):
    """Fewer than 256 weight rows at prefill sizes (the 70B k/v shard, 128 x 8192): the 256-tile kernel in its
    split-K form (half-empty tiles, clamped loads, guarded stores) instead of 32 whole-K 128-tile workgroups --
    within the oracle tolerance on every output, and equal to the 128-tile kernel up to fp32 summation order."""
    F = _F()
    M, N, K = mnk
    torch.manual_seed(M + N + K)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=nested)
    Y = F.gemm_4bit(X, q, st)
    torch.cuda.synchronize()
    assert F.lib.cget_last_error() == 0
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), F._absmax_fp32(st).cpu().numpy(), N, K,
                                    64, st.code.cpu().numpy(), "bf16")
    frac, err = _close(Y.float().cpu().numpy(), exp, 2e-2, 2e-2)
    assert frac == 0.0, err
    F.lib.cgemm_4bit_set_tile(128)
    try:
        Y128 = F.gemm_4bit(X, q, st)
    finally:
        F.lib.cgemm_4bit_set_tile(0)
    rms = Y128.float().pow(2).mean().sqrt().item()
    assert (Y.float() - Y128.float()).abs().max().item() < 1e-2 * rms + 1e-2 * Y128.float().abs().max().item()


@pytest.mark.parametrize("tile", [128, 256])
@pytest.mark.parametrize("mnk", [(256, 256, 128), (300, 520, 640), (1000, 384, 256)])
def test_gemm_4bit_each_tile_kernel(dev, tile, mnk):
    """Force each tile kernel (128x128 / 256x256) on shapes with ragged M/N tails."""
    F = _F()
    M, N, K = mnk
    torch.manual_seed(M + N + K)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4")
    F.lib.cgemm_4bit_set_tile(tile)
    try:
        Y = F.gemm_4bit(X, q, st)
    finally:
        F.lib.cgemm_4bit_set_tile(0)
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), st.absmax.cpu().numpy(), N, K, 64,
                                    st.code.cpu().numpy(), "bf16")
    frac, err = _close(Y.float().cpu().numpy(), exp, 2e-2, 2e-2)
    assert frac == 0.0, err


def test_gemm_4bit_tile_kernels_agree_large(dev, monkeypatch):
    """Metric shape class: the 256x256 kernel (auto) equals the 128x128 kernel up to fp32 summation order
    (the fused kernel forced: at this size gemm_4bit would take the dequantise + library GEMM path)."""
    F = _F()
    monkeypatch.setattr(F, "GEMM_4BIT_DEQUANT_MIN_ROWS", 1 << 30)
    monkeypatch.setattr(F, "GEMM_4BIT_ROUTE_TUNING", False)
    M, N, K = 2048, 2048, 11008
    torch.manual_seed(11)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    Y = F.gemm_4bit(X, q, st)
    F.lib.cgemm_4bit_set_tile(128)
    try:
        Y1 = F.gemm_4bit(X, q, st)
    finally:
        F.lib.cgemm_4bit_set_tile(0)
    Wd = F.dequantize_4bit(q, st)
    Yref = X.float() @ Wd.float().t()
    rms = Yref.pow(2).mean().sqrt().item()
    assert (Y.float() - Yref).abs().max().item() < 2e-2 * rms + 2e-2 * Yref.abs().max().item()
    assert (Y.float() - Y1.float()).abs().max().item() < 1e-2 * rms + 1e-2 * Yref.abs().max().item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mnk,ks", [((1024, 512, 4096), 8), ((300, 264, 1088), 2), ((256, 384, 1024), 2),
                                    ((16, 1024, 2048), 4), ((3, 512, 1024), 2)])
def test_gemm_4bit_split_k_vs_oracle(dev, dtype, mnk, ks):
    """Split-K on the 256x256 kernel (small tile grids, e.g. narrow column shards): fp32 partials in a
    caller workspace, summed in split order, one cast.  Same tolerance as the unsplit kernel."""
    F = _F()
    M, N, K = mnk
    # (few-token shapes run the weight-streaming kernel by default: force the 256x256 kernel here)
    few = M <= F.GEMM_4BIT_FEW_TOKENS
    assert F.lib.cgemm_4bit_workspace_bytes(N, M, K) >= ks * M * N * 4
    if not few:
        assert F.lib.cgemm_4bit_workspace_bytes(N, M, K) == ks * M * N * 4
    torch.manual_seed(M + 7 * N)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    X = torch.randn(M, K, device=dev, dtype=dtype)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4")
    F.lib.cgemm_4bit_set_tile(256 if few else 0)
    try:
        Y = F.gemm_4bit(X, q, st)
    finally:
        F.lib.cgemm_4bit_set_tile(0)
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), st.absmax.cpu().numpy(), N, K, 64,
                                    st.code.cpu().numpy(), "bf16" if dtype == torch.bfloat16 else "fp16")
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-2
    frac, err = _close(Y.float().cpu().numpy(), exp, tol, tol)
    assert frac == 0.0, err
    # without a workspace the dispatcher falls back to an unsplit kernel: same result up to fp32 order
    out = torch.empty_like(Y)
    fn = F.lib.cgemm_4bit_inference_code_bf16 if dtype == torch.bfloat16 else F.lib.cgemm_4bit_inference_code_fp16
    F.lib.cgemm_4bit_set_tile(256 if few else 0)
    try:
        fn(ct.c_int32(N), ct.c_int32(M), ct.c_int32(K), F.get_ptr(X), F.get_ptr(q), F.get_ptr(st.absmax),
           F.get_ptr(st.code), F.get_ptr(out), ct.c_int32(K), ct.c_int32(K // 2), ct.c_int32(N), ct.c_int32(64))
        torch.cuda.synchronize()
    finally:
        F.lib.cgemm_4bit_set_tile(0)
    rms = Y.float().pow(2).mean().sqrt().item()
    assert (Y.float() - out.float()).abs().max().item() < 1e-2 * rms + 1e-2 * Y.float().abs().max().item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("qt", ["nf4", "fp4"])
def test_gemm_4bit_library_path(dev, dtype, qt, monkeypatch):
    """From GEMM_4BIT_DEQUANT_MIN_ROWS x GEMM_4BIT_DEQUANT_MIN_FEATURES gemm_4bit runs the reference's M > 1
    algorithm on the GPU: the HIP dequantise kernel into a workspace, then one library GEMM.  Bit-equal to
    dequantize_4bit + torch.matmul (the static rule's library GEMM), within the GEMM tolerance of the oracle, and close
    to the fused kernel.
    (The static rule: the measured route is switched off here.)"""
    F = _F()
    monkeypatch.setattr(F, "GEMM_4BIT_ROUTE_TUNING", False)
    M, N, K = 2048, 1024, 2048
    assert M >= F.GEMM_4BIT_DEQUANT_MIN_ROWS and N >= F.GEMM_4BIT_DEQUANT_MIN_FEATURES
    torch.manual_seed(17)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    X = torch.randn(M, K, device=dev, dtype=dtype)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type=qt, compress_statistics=True)
    # round 4: the static rule sends this shape to the hand-written k_hgemm (split-K: 32 tiles); the library pair is
    # still selectable (_route="library") and stays bit-equal to dequantize_4bit + torch.matmul
    assert F.gemm_4bit_static_route(M, N, K) == "hgemm"
    Yl = F.gemm_4bit(X, q, st, _route="library")
    assert torch.equal(Yl, torch.matmul(X, F.dequantize_4bit(q, st).t()))
    Y = F.gemm_4bit(X, q, st)
    absmax = F._absmax_fp32(st).cpu().numpy()
    for got in (Yl, Y):
        frac, err = _close(got.float().cpu().numpy(), ref.gemm_4bit_dequant_ref(
            X.float().cpu().numpy(), q.cpu().numpy(), absmax, N, K, 64, st.code.cpu().numpy(),
            "bf16" if dtype == torch.bfloat16 else "fp16"), 2e-2 if dtype == torch.bfloat16 else 1e-2,
            2e-2 if dtype == torch.bfloat16 else 1e-2)
        assert frac == 0.0, err
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), absmax, N, K, 64,
                                    st.code.cpu().numpy(), "bf16" if dtype == torch.bfloat16 else "fp16")
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-2
    frac, err = _close(Y.float().cpu().numpy(), exp, tol, tol)
    assert frac == 0.0, err
    F.GEMM_4BIT_DEQUANT_MIN_ROWS, saved = 1 << 30, F.GEMM_4BIT_DEQUANT_MIN_ROWS
    try:
        Yf = F.gemm_4bit(X, q, st)
    finally:
        F.GEMM_4BIT_DEQUANT_MIN_ROWS = saved
    rms = Y.float().pow(2).mean().sqrt().item()
    assert (Y.float() - Yf.float()).abs().max().item() < 1e-2 * rms + 1e-2 * Y.float().abs().max().item()


def test_gemm_4bit_split_k_metric_shard(dev):
    """The 8-way column shard of the metric shape (M=4096, N/8=512, K=11008): split-K result vs the
    dequantize_4bit + fp32 matmul reference path."""
    F = _F()
    M, N, K = 4096, 512, 11008
    assert F.lib.cgemm_4bit_workspace_bytes(N, M, K) > 0
    torch.manual_seed(5)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    Y = F.gemm_4bit(X, q, st)
    Yref = X.float() @ F.dequantize_4bit(q, st).float().t()
    rms = Yref.pow(2).mean().sqrt().item()
    assert (Y.float() - Yref).abs().max().item() < 2e-2 * rms + 2e-2 * Yref.abs().max().item()
    assert (Y.float() - Yref).abs().mean().item() < 0.115


def test_gemm_4bit_legacy_abi_nf4_fp16(dev):
    """cgemm_4bit_inference (ref ABI slot, fp16, NF4 hard-coded)."""
    F = _F()
    M, N, K = 96, 256, 512
    torch.manual_seed(3)
    W = torch.randn(N, K, device=dev, dtype=torch.float16) * 0.05
    X = torch.randn(M, K, device=dev, dtype=torch.float16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4")
    out = torch.empty(M, N, device=dev, dtype=torch.float16)
    F.lib.cgemm_4bit_inference(ct.c_int32(N), ct.c_int32(M), ct.c_int32(K), F.get_ptr(X), F.get_ptr(q),
                               F.get_ptr(st.absmax), F.get_ptr(out), ct.c_int32(K), ct.c_int32(K // 2), ct.c_int32(N),
                               ct.c_int32(64))
    torch.cuda.synchronize()
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), st.absmax.cpu().numpy(), N, K, 64,
                                    ref.nf4_table(), "fp16")
    frac, err = _close(out.float().cpu().numpy(), exp, 1e-2, 1e-2)
    assert frac == 0.0, err


def test_gemm_4bit_asymmetric_identity(dev):
    """A = I and asymmetric W: catches a transposed C write (guide §3)."""
    F = _F()
    K = N = 128
    X = torch.eye(K, device=dev, dtype=torch.bfloat16)
    W = torch.arange(N * K, device=dev, dtype=torch.float32).reshape(N, K).remainder(7).sub(3).div(3).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4")
    Y = F.gemm_4bit(X, q, st)
    Wd = F.dequantize_4bit(q, st)
    assert torch.equal(Y, Wd.t().contiguous())


def test_gemm_4bit_reuse_weight_chunks(dev, monkeypatch):
    """Chunked forward on the dequantise + GEMM path: chunks after the first reuse the dequantised weight
    (reuse_weight); each chunk equals its own unchunked call bit for bit, the whole product equals the unchunked call
    within the GEMM tolerance (NOT bit for bit: k_hgemm's launch plan -- tile shape and split-K -- follows the row count,
    so outputs are not row-split invariant), and a different weight is never reused."""
    monkeypatch.setattr(_F(), "GEMM_4BIT_ROUTE_TUNING", False)
    F = _F()
    from python_src_quants.parallel import ColumnShardedLinear4bit
    M, N, K = 4096, 1024, 2048
    torch.manual_seed(23)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    lin = ColumnShardedLinear4bit(W, world=1, rank=0, device=dev)
    full = F.gemm_4bit(X, lin.qweight, lin.quant_state)
    chunked = lin.forward(X, chunks=2)
    # each chunk equals its own unchunked call bit for bit (the GEMM's split-K factor follows the row count, so the
    # whole product is compared within the GEMM tolerance)
    per_chunk = torch.cat([F.gemm_4bit(X[:2048], lin.qweight, lin.quant_state),
                           F.gemm_4bit(X[2048:], lin.qweight, lin.quant_state)])
    assert torch.equal(chunked, per_chunk)
    rms = full.float().pow(2).mean().sqrt().item()
    assert (chunked.float() - full.float()).abs().max().item() <= 1e-2 * rms + 1e-2 * full.float().abs().max().item()
    # a second weight through the same workspace: reuse_weight must not hand back the first one
    W2 = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    q2, st2 = F.quantize_4bit(W2, blocksize=64, quant_type="nf4", compress_statistics=True)
    y2 = F.gemm_4bit(X[:2048], q2, st2, reuse_weight=True)
    assert torch.equal(y2, F.gemm_4bit(X[:2048], q2, st2))


def test_gemm_4bit_library_path_two_streams(dev, monkeypatch):
    """Two streams running the dequantise + library GEMM path concurrently on different weights each use
    their own weight workspace (keyed by stream): both results equal their single-stream values."""
    monkeypatch.setattr(_F(), "GEMM_4BIT_ROUTE_TUNING", False)
    F = _F()
    M, N, K = 2048, 2048, 1024
    torch.manual_seed(29)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    qs = [F.quantize_4bit((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16), blocksize=64,
                          quant_type="nf4", compress_statistics=True) for _ in range(2)]
    ref_out = [F.gemm_4bit(X, q, st) for q, st in qs]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    outs = [None, None]
    for _ in range(3):
        for i, s in enumerate(streams):
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                outs[i] = F.gemm_4bit(X, qs[i][0], qs[i][1])
        torch.cuda.synchronize()
        for i in range(2):
            assert torch.equal(outs[i], ref_out[i])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("mnk", [(2, 11008, 4096), (3, 300, 1152), (16, 4096, 11008), (17, 1000, 2048),
                                 (33, 64, 128), (48, 520, 640), (64, 4096, 4096), (64, 11008, 4096)])
def test_gemm_4bit_few_tokens_vs_oracle(dev, dtype, nested, mnk):
    """1..64 activation rows (batched decode, short prefill) run the weight-streaming kernel (gemm4bit_skinny.hip;
    33..64 rows on its 4-tile instance): same dequantised weights, fp32 sums split over K in split order.  Nested
    statistics are decoded in the kernel.  Same tolerance as the tile kernels; ragged rows, one-block K,
    a tail chunk (K = 11008 = 86 blocks) and single-split shapes."""
    F = _F()
    M, N, K = mnk
    torch.manual_seed(M * 7 + N)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    X = torch.randn(M, K, device=dev, dtype=dtype)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=nested)
    Y = F.gemm_4bit(X, q, st)
    assert Y.shape == (M, N) and Y.dtype == dtype
    absmax = F._absmax_fp32(st).cpu().numpy()
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), absmax, N, K, 64,
                                    st.code.cpu().numpy(), "bf16" if dtype == torch.bfloat16 else "fp16")
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-2
    frac, err = _close(Y.float().cpu().numpy(), exp, tol, tol)
    assert frac == 0.0, err
    # the tile kernels (forced; the multi-row GEMV for 2..4 rows switched off) agree up to fp32 summation order
    F.lib.cgemm_4bit_set_tile(128)
    saved = F.GEMM_4BIT_GEMV_TOKENS
    F.GEMM_4BIT_GEMV_TOKENS = 1
    try:
        Yt = F.gemm_4bit(X, q, st, absmax=F._absmax_fp32(st))
    finally:
        F.lib.cgemm_4bit_set_tile(0)
        F.GEMM_4BIT_GEMV_TOKENS = saved
    rms = Yt.float().pow(2).mean().sqrt().item()
    assert (Y.float() - Yt.float()).abs().max().item() < 1e-2 * rms + 1e-2 * Yt.float().abs().max().item()


def test_gemm_4bit_few_tokens_nested_matches_plain(dev):
    """In-kernel decode of compressed statistics = the decoded fp32 absmax passed in: bit-identical."""
    F = _F()
    M, N, K = 24, 4096, 11008
    torch.manual_seed(5)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    Yn = F.gemm_4bit(X, q, st)
    Yp = F.gemm_4bit(X, q, st, absmax=F._absmax_fp32(st))
    assert torch.equal(Yn, Yp)
    # deterministic: the split partials are summed in a fixed order
    assert torch.equal(Yn, F.gemm_4bit(X, q, st))


def test_gemm_4bit_few_tokens_entry_point_declines(dev):
    """The one-launch entry point returns 1 (nothing launched) when the shape does not fit it."""
    F = _F()
    M, N, K = 65, 256, 1024                     # > 64 tokens (SK_MAX_TOKENS)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    q, st = F.quantize_4bit((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16), blocksize=64,
                            quant_type="nf4", compress_statistics=True)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    s2 = st.state2
    off = st.offset.reshape(1).float()
    rc = F.lib.cgemm_4bit_inference_nested_ws_bf16(
        ct.c_int32(N), ct.c_int32(M), ct.c_int32(K), F.get_ptr(X), F.get_ptr(q), F.get_ptr(st.absmax),
        F.get_ptr(s2.code), F.get_ptr(s2.absmax), F.get_ptr(off), F.get_ptr(st.code), F.get_ptr(out),
        ct.c_int32(K), ct.c_int32(K // 2), ct.c_int32(N), ct.c_int32(64), ct.c_int32(s2.blocksize), None,
        ct.c_longlong(0))
    assert rc == 1
    Y = F.gemm_4bit(X, q, st)                  # routed to the tile kernels
    Wd = F.dequantize_4bit(q, st)
    Yref = X.float() @ Wd.float().t()
    rms = Yref.pow(2).mean().sqrt().item()
    assert (Y.float() - Yref).abs().max().item() < 2e-2 * rms + 2e-2 * Yref.abs().max().item()


@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("qt,bs", [("nf4", 64), ("fp4", 64), ("nf4", 128), ("fp4", 256)])
@pytest.mark.parametrize("mnk", [(5, 1001, 2048), (24, 4099, 4096), (3, 63, 128), (32, 1, 256)])
def test_gemm_4bit_few_tokens_ragged_n(dev, nested, qt, bs, mnk):
    """Few-token kernel on out_features not a multiple of 4 (the scalar partial-store and reduce tails), split-K
    shapes, FP4 and blocksizes 128 / 256, nested and plain statistics -- against the fp64 oracle."""
    F = _F()
    M, N, K = mnk
    torch.manual_seed(M + N + bs)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=bs, quant_type=qt, compress_statistics=nested)
    Y = F.gemm_4bit(X, q, st)
    assert Y.shape == (M, N)
    absmax = F._absmax_fp32(st).cpu().numpy()
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), absmax, N, K, bs,
                                    st.code.cpu().numpy(), "bf16")
    frac, err = _close(Y.float().cpu().numpy(), exp, 2e-2, 2e-2)
    assert frac == 0.0, err


def test_gemm_4bit_library_knob_covers_few_tokens(dev, monkeypatch):
    """GEMM_4BIT_DEQUANT_MIN_ROWS = 1 and GEMM_4BIT_FEW_TOKENS = 0 force the dequantise + GEMM pair for few tokens too
    (the few-token branch is not taken): since round 4 the pair's GEMM is k_hgemm, so the result equals the forced "hgemm" route bit for bit and
    dequantize_4bit + torch.matmul within the GEMM tolerance; the library GEMM stays reachable (_route="library")."""
    monkeypatch.setattr(_F(), "GEMM_4BIT_ROUTE_TUNING", False)
    F = _F()
    monkeypatch.setattr(F, "GEMM_4BIT_DEQUANT_MIN_ROWS", 1)
    monkeypatch.setattr(F, "GEMM_4BIT_FEW_TOKENS", 0)
    M, N, K = 8, 2048, 1024
    torch.manual_seed(31)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    assert F.gemm_4bit_static_route(M, N, K) == "hgemm"
    Y = F.gemm_4bit(X, q, st)
    assert torch.equal(Y, F.gemm_4bit(X, q, st, _route="hgemm"))
    E = torch.matmul(X, F.dequantize_4bit(q, st).t())
    assert torch.equal(F.gemm_4bit(X, q, st, _route="library"), E)
    rms = E.float().pow(2).mean().sqrt().item()
    assert (Y.float() - E.float()).abs().max().item() <= 1e-2 * rms + 1e-2 * E.float().abs().max().item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("shape", [(11008, 4096), (4096, 11008), (4096, 4096), (1024, 8192), (3584, 8192),
                                   (14336, 4096), (28672, 4096), (5000, 7680), (7, 64), (300, 6144), (257, 16384),
                                   (12345, 128), (1, 4096), (513, 2048), (40000, 1024)])
@pytest.mark.parametrize("quant", [("nf4", 64), ("fp4", 128), ("nf4", 256)])
def test_gemv_balanced_kernel_matches_dot_kernel(dev, dtype, nested, shape, quant):
    """The balanced-range GEMV (k_gemv_4bit_bal: 2 workgroups per CU, perm-addressed table, swizzled activations,
    clamped duplicate rows) gives the bits of the 4-waves-x-R-rows kernel on every decode shape it takes
    (Llama-2-7B / Llama-3-8B / 70B-shard projections, ragged and tiny M) and falls back where it does not fit."""
    F = _F()
    N, K = shape
    qt, bs = quant
    torch.manual_seed(N + K)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    q, st = F.quantize_4bit(W, blocksize=bs, quant_type=qt, compress_statistics=nested)
    x = torch.randn(1, K, device=dev, dtype=dtype)
    try:
        F.lib.cgemv_4bit_set_kernel(3)          # the automatic choice without the wide kernel
        y_auto = F.gemv_4bit(x, q.t(), state=st)
        F.lib.cgemv_4bit_set_kernel(1)
        y_dot = F.gemv_4bit(x, q.t(), state=st)
    finally:
        F.lib.cgemv_4bit_set_kernel(0)
    assert torch.equal(y_auto.view(torch.int16), y_dot.view(torch.int16))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(1024, 28672), (128, 8192), (37, 40960), (7, 64), (200, 2080), (3, 131072),
                                   (1000, 4096)])
@pytest.mark.parametrize("quant", [("nf4", 64), ("fp4", 128)])
def test_gemv_wide_kernel(dev, dtype, shape, quant):
    """k_gemv_4bit_wide (1..4 rows per workgroup, K split over its waves, summed in wave order): the default for K
    beyond the balanced kernel's LDS and for fewer rows than CUs, forced here on every shape (1000 x 4096 would take
    the balanced kernel).  Within the oracle tolerance for plain and compressed statistics, the in-kernel decode
    bit-identical to the decoded-absmax call, and the default route equal to the forced one where it is taken."""
    F = _F()
    N, K = shape
    qt, bs = quant
    torch.manual_seed(N + K + bs)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    x = torch.randn(1, K, device=dev, dtype=dtype)
    name = {torch.bfloat16: "bf16", torch.float16: "fp16"}[dtype]
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-2
    for nested in (False, True):
        q, st = F.quantize_4bit(W, blocksize=bs, quant_type=qt, compress_statistics=nested)
        absmax = F._absmax_fp32(st)
        exp = ref.gemv_4bit(x.float().cpu().numpy()[0], q.cpu().numpy(), absmax.cpu().numpy(), N, K, bs,
                            st.code.cpu().numpy())
        y_default = F.gemv_4bit(x, q.t(), state=st)
        F.lib.cgemv_4bit_set_kernel(2)
        try:
            y = F.gemv_4bit(x, q.t(), state=st)
            F.lib.cgemv_4bit_set_wide_rows(1)       # one row per workgroup: the rows-per-workgroup form is bit-equal
            try:
                y_r1 = F.gemv_4bit(x, q.t(), state=st)
            finally:
                F.lib.cgemv_4bit_set_wide_rows(0)
            two_step = torch.empty_like(y)
            getattr(F.lib, f"cgemm_4bit_inference_naive_{name}")(
                ct.c_int32(N), ct.c_int32(1), ct.c_int32(K), F.get_ptr(x), F.get_ptr(q), F.get_ptr(absmax),
                F.get_ptr(st.code), F.get_ptr(two_step), ct.c_int32(N), ct.c_int32(K // 2), ct.c_int32(N), ct.c_int32(bs))
            torch.cuda.synchronize()
        finally:
            F.lib.cgemv_4bit_set_kernel(0)
        assert F.lib.cget_last_error() == 0
        frac, err = _close(y.float().cpu().numpy()[0], exp, tol, tol)
        assert frac == 0.0, (nested, err)
        assert torch.equal(y.view(torch.int16), two_step.view(torch.int16))
        assert torch.equal(y.view(torch.int16), y_r1.view(torch.int16))
        if K > 16384 or N < 256:
            assert torch.equal(y_default.view(torch.int16), y.view(torch.int16))


@pytest.mark.parametrize("nested", [False, True])
def test_gemv_plan_cache_follows_state_changes(dev, nested):
    """gemv_4bit's cached per-weight call plan: repeated calls give identical bits, and replacing the state's
    statistics (absmax, nested offset) or calling with another dtype is seen on the next call."""
    F = _F()
    torch.manual_seed(5)
    N, K = 1024, 2048
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=nested)
    x = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
    y0 = F.gemv_4bit(x, q.t(), state=st)
    assert torch.equal(F.gemv_4bit(x, q.t(), state=st), y0)
    if nested:
        st.offset = st.offset * 2 if torch.is_tensor(st.offset) else st.offset * 2
        F.lib.cgemv_4bit_set_kernel(1)
        try:
            exp = F.gemv_4bit(x, q.t(), state=st)
        finally:
            F.lib.cgemv_4bit_set_kernel(0)
        y1 = F.gemv_4bit(x, q.t(), state=st)
        assert torch.equal(y1, exp) and not torch.equal(y1, y0)
    else:
        st.absmax = st.absmax * 2
        y1 = F.gemv_4bit(x, q.t(), state=st)
        assert torch.equal(y1.float(), (y0.float() * 2).to(torch.bfloat16).float()) or \
            torch.allclose(y1.float(), y0.float() * 2, rtol=1e-2, atol=1e-3)
    yh = F.gemv_4bit(x.half(), q.t(), state=st)
    assert yh.dtype == torch.float16 and torch.allclose(yh.float(), y1.float(), rtol=2e-2, atol=2e-2)
    out = torch.empty(1, N, device=dev, dtype=torch.bfloat16)
    assert F.gemv_4bit(x, q.t(), state=st, out=out) is out and torch.equal(out, y1)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("rows", [2, 3, 4])
@pytest.mark.parametrize("shape", [(11008, 4096), (4096, 11008), (4096, 4096), (1001, 2048), (63, 128), (28672, 1024),
                                   (3584, 8192), (40000, 4096)])
def test_gemm_4bit_multirow_gemv_matches_gemv(dev, dtype, nested, rows, shape):
    """2..4 activation rows run the multi-row GEMV (gemv4bit_tok.hip): every row of the result is bit-identical to
    gemv_4bit on that row alone (same lookups, chains and wave reduction), plain and compressed statistics."""
    F = _F()
    N, K = shape
    torch.manual_seed(N + K + rows)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    X = torch.randn(rows, K, device=dev, dtype=dtype)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=nested)
    F.set_fewtok_mode(1)                       # the multi-row GEMV itself (the whole-K MFMA kernel takes these by default)
    try:
        Y = F.gemm_4bit(X, q, st)
    finally:
        F.set_fewtok_mode(0)
    assert Y.shape == (rows, N)
    F.lib.cgemv_4bit_set_kernel(3)              # the balanced / dot GEMV family (not the wide kernel of narrow weights)
    try:
        for t in range(rows):
            y = F.gemv_4bit(X[t:t + 1], q.t(), state=st)
            if N < 256:   # fewer weight rows than CUs: the multi-row GEMV declines, the split-K kernel runs
                rms = y.float().pow(2).mean().sqrt().item()
                assert (Y[t].float() - y.reshape(-1).float()).abs().max().item() < 2e-2 * rms + 2e-2 * y.float().abs().max().item()
            else:
                assert torch.equal(Y[t], y.reshape(-1)), f"row {t} differs from gemv_4bit"
    finally:
        F.lib.cgemv_4bit_set_kernel(0)


@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("qt,bs", [("nf4", 64), ("fp4", 64), ("nf4", 128), ("fp4", 256)])
@pytest.mark.parametrize("mnk", [(2, 11008, 4096), (3, 1001, 2048), (4, 4099, 4096), (2, 1, 256)])
def test_gemm_4bit_multirow_gemv_vs_oracle(dev, nested, qt, bs, mnk):
    """The multi-row GEMV against the fp64 oracle of dequantize_4bit + matmul: FP4, blocksizes 64..256, ragged
    out_features, one-row weights -- the GEMV tolerance (codes in T, fp32 products)."""
    F = _F()
    M, N, K = mnk
    torch.manual_seed(M * 13 + N + bs)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=bs, quant_type=qt, compress_statistics=nested)
    F.set_fewtok_mode(1)                       # the multi-row GEMV itself
    try:
        Y = F.gemm_4bit(X, q, st)
    finally:
        F.set_fewtok_mode(0)
    absmax = F._absmax_fp32(st).cpu().numpy()
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), absmax, N, K, bs,
                                    st.code.cpu().numpy(), "bf16")
    frac, err = _close(Y.float().cpu().numpy(), exp, 2e-2, 2e-2)
    assert frac == 0.0, err


def test_gemm_4bit_multirow_gemv_entry_declines(dev):
    """The multi-row entry point launches nothing (returns 1) for 1 or 5 rows; gemm_4bit then
    takes the few-token kernel, which agrees with the multi-row GEMV up to summation order."""
    F = _F()
    N, K = 512, 1024
    torch.manual_seed(77)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=False)
    for M in (1, 5):
        X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        rc = F.lib.cgemm_4bit_inference_tokens_bf16(
            ct.c_int32(N), ct.c_int32(M), ct.c_int32(K), F.get_ptr(X), ct.c_int32(K), F.get_ptr(q), ct.c_int32(K // 2),
            F.get_ptr(st.absmax), None, None, None, None, F.get_ptr(st.code), F.get_ptr(out), ct.c_int32(N),
            ct.c_int32(64), ct.c_int32(0))
        assert rc == 1
    X = torch.randn(4, K, device=dev, dtype=torch.bfloat16)
    Yg = F.gemm_4bit(X, q, st)
    saved = F.GEMM_4BIT_GEMV_TOKENS
    F.GEMM_4BIT_GEMV_TOKENS = 1
    try:
        Ys = F.gemm_4bit(X, q, st)
    finally:
        F.GEMM_4BIT_GEMV_TOKENS = saved
    rms = Ys.float().pow(2).mean().sqrt().item()
    assert (Yg.float() - Ys.float()).abs().max().item() < 1e-2 * rms + 1e-2 * Ys.float().abs().max().item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("mnk", [(5, 1001, 2048), (8, 11008, 4096), (16, 4096, 11008), (24, 4099, 4096), (32, 1, 256),
                                 (7, 300, 128), (17, 4096, 4096), (12, 28672 // 8, 8192)])
def test_fewtoken_whole_k_and_split_k_kernels(dev, dtype, nested, mnk):
    """The two few-token kernels, each forced (cgemm_4bit_set_fewtoken_kernel 2 / 1): the whole-K kernel (K split
    over the workgroup's waves, summed in LDS in wave order, no workspace) and the split-K skinny kernel (+ ordered
    reduce launch) -- each within the oracle tolerance, and the whole-K one deterministic across calls.  Covers one-block K
    (fewer blocks than waves), ragged out_features, 1 and 2 token tiles, the 4- and 8-wave instances."""
    F = _F()
    M, N, K = mnk
    torch.manual_seed(M * 31 + N)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    X = torch.randn(M, K, device=dev, dtype=dtype)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=nested)
    absmax = F._absmax_fp32(st).cpu().numpy()
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), absmax, N, K, 64,
                                    st.code.cpu().numpy(), "bf16" if dtype == torch.bfloat16 else "fp16")
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-2
    saved = F.GEMM_4BIT_GEMV_TOKENS
    F.GEMM_4BIT_GEMV_TOKENS = 1
    outs = []
    try:
        for kern in (2, 1):
            F.lib.cgemm_4bit_set_fewtoken_kernel(kern)
            Y = F.gemm_4bit(X, q, st)
            torch.cuda.synchronize()
            assert F.lib.cget_last_error() == 0
            frac, err = _close(Y.float().cpu().numpy(), exp, tol, tol)
            assert frac == 0.0, (kern, err)
            outs.append(Y)
        F.lib.cgemm_4bit_set_fewtoken_kernel(2)
        assert torch.equal(outs[0], F.gemm_4bit(X, q, st))      # the whole-K kernel again: deterministic
    finally:
        F.lib.cgemm_4bit_set_fewtoken_kernel(0)
        F.GEMM_4BIT_GEMV_TOKENS = saved


@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("mnk", [(40, 1001, 2048), (64, 4096, 11008), (33, 4099, 4096), (12, 300, 1152), (24, 130, 256),
                                 (64, 129, 128), (48, 1024, 8192)])
def test_fewtoken_split_k_geometries(dev, nested, mnk):
    """The split-K few-token kernel in each workgroup geometry (cgemm_4bit_set_skinny_config 0 / 1 / 2: 4 waves, 8
    waves with the same blocks per split, 8 waves with twice the blocks per split) and the default rule (-1): every
    form within the oracle tolerance; the forms with the same splits give the same bits (per-row summation order is
    unchanged).  Covers ragged out_features below and above one 128-row workgroup, one-split K and 1 / 2 / 4 token tiles."""
    F = _F()
    M, N, K = mnk
    torch.manual_seed(M * 7 + N)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=nested)
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), F._absmax_fp32(st).cpu().numpy(), N, K,
                                    64, st.code.cpu().numpy(), "bf16")
    saved = F.GEMM_4BIT_GEMV_TOKENS
    F.GEMM_4BIT_GEMV_TOKENS = 1
    outs = {}
    try:
        F.lib.cgemm_4bit_set_fewtoken_kernel(1)
        for cfg in (0, 1, 2, -1):
            F.lib.cgemm_4bit_set_skinny_config(cfg)
            Y = F.gemm_4bit(X, q, st)
            torch.cuda.synchronize()
            assert F.lib.cget_last_error() == 0
            frac, err = _close(Y.float().cpu().numpy(), exp, 2e-2, 2e-2)
            assert frac == 0.0, (cfg, err)
            outs[cfg] = Y
        assert torch.equal(outs[0], outs[1])
    finally:
        F.lib.cgemm_4bit_set_skinny_config(-1)
        F.lib.cgemm_4bit_set_fewtoken_kernel(0)
        F.GEMM_4BIT_GEMV_TOKENS = saved


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mnk", [(2048, 1024, 2048), (300, 520, 640), (4096, 11008, 4096), (1, 64, 64)])
def test_library_gemm_solution_search(dev, dtype, mnk):
    """cgemm_tn_* (gemm_lib.hip): C = A . W^T on rocBLAS with the per-shape solution search -- within the bf16/fp16
    GEMM tolerance of torch.matmul, a plan cached after the first call (>= 0), deterministic on the cached plan, the
    same bits with the search switched off when the plan is the standard algorithm, and replayable from a HIP graph."""
    F = _F()
    m, n, k = mnk
    torch.manual_seed(m + n)
    X = torch.randn(m, k, device=dev, dtype=dtype)
    Wd = (torch.randn(n, k, device=dev) * 0.02).to(dtype)
    ref_out = torch.matmul(X.float(), Wd.float().t())
    Y = _lib_matmul(F, X, Wd)
    err = (Y.float() - ref_out).abs().max().item()
    assert err <= 1e-2 * ref_out.abs().max().item() + 1e-3, err
    dt = 0 if dtype == torch.bfloat16 else 1
    plan = F.lib.cgemm_tn_plan(m, n, k, dt, k, k, n)
    assert plan >= 0
    assert torch.equal(_lib_matmul(F, X, Wd), Y)
    if plan == 0:
        F.lib.cgemm_tn_set_search(0, ct.c_double(0.0), 0)
        try:
            assert torch.equal(_lib_matmul(F, X, Wd), Y)
        finally:
            F.lib.cgemm_tn_set_search(1, ct.c_double(0.0), 0)
    # HIP-graph capture of the planned call (the plan and rocBLAS's workspace exist from the calls above), replayed
    X2 = torch.randn(m, k, device=dev, dtype=dtype)
    Y2 = torch.empty(m, n, device=dev, dtype=dtype)
    fn = F.lib.cgemm_tn_bf16 if dtype == torch.bfloat16 else F.lib.cgemm_tn_fp16
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            F.pre_call(X2.device)
            fn(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k), F.get_ptr(X2), ct.c_int32(k), F.get_ptr(Wd), ct.c_int32(k),
               F.get_ptr(Y2), ct.c_int32(n))
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(Y2, _lib_matmul(F, X2, Wd))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("qt,bs", [("nf4", 64), ("fp4", 64), ("nf4", 256)])
@pytest.mark.parametrize("mnk", [(1, 4096, 4096), (2, 11008, 4096), (5, 1001, 2048), (8, 4096, 11008),
                                 (13, 300, 1152), (16, 8192, 256), (17, 520, 640), (32, 11008, 4096), (31, 63, 11008),
                                 (3, 14336, 4096), (24, 14337, 1024), (9, 8200, 768)])
def test_fewtok32_kernel_vs_oracle(dev, dtype, nested, qt, bs, mnk):
    """The whole-K few-token kernel (gemm4bit_fewtok.hip), forced wherever it fits (set_fewtok_mode(2), the 2..4-row
    GEMV switched off): 1..4 row groups per workgroup (1001 .. 11008 out features), 4- and 8-wave forms, ragged out
    features, K shares of unequal length (K = 11008: 43 groups; 640: a partial 4-block group, waves without groups),
    the per-block and the 4-per-load statistics forms (blocksize 256 / 64), FP4, nested and plain statistics --
    against the fp64 oracle.  Its arithmetic is the reference GEMV's (T(code) * x summed per block, then * absmax), so
    the bar is the GEMV's / the tile kernels'."""
    F = _F()
    M, N, K = mnk
    torch.manual_seed(M * 13 + N + bs)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    X = torch.randn(M, K, device=dev, dtype=dtype)
    q, st = F.quantize_4bit(W, blocksize=bs, quant_type=qt, compress_statistics=nested)
    saved = F.GEMM_4BIT_GEMV_TOKENS
    F.GEMM_4BIT_GEMV_TOKENS = 1
    F.set_fewtok_mode(2)
    try:
        Y = F.gemm_4bit(X, q, st)
        Y2 = F.gemm_4bit(X, q, st)
        Yp = F.gemm_4bit(X, q, st, absmax=F._absmax_fp32(st))
    finally:
        F.set_fewtok_mode(0)
        F.GEMM_4BIT_GEMV_TOKENS = saved
    assert Y.shape == (M, N) and Y.dtype == dtype
    assert torch.equal(Y, Y2)                          # deterministic (the K quarters meet in wave order)
    assert torch.equal(Y, Yp)                          # in-kernel nested decode = the decoded absmax passed in
    absmax = F._absmax_fp32(st).cpu().numpy()
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), absmax, N, K, bs,
                                    st.code.cpu().numpy(), "bf16" if dtype == torch.bfloat16 else "fp16")
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-2
    frac, err = _close(Y.float().cpu().numpy(), exp, tol, tol)
    assert frac == 0.0, err


@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("rows", [2, 3, 4])
@pytest.mark.parametrize("shape", [(11008, 4096), (4096, 4096), (4096, 11008)])
def test_fewtok_default_rows_close_to_gemv_and_deterministic(dev, nested, rows, shape):
    """The DEFAULT route of 2..4 activation rows (round 3: the whole-K MFMA few-token kernel wherever
    cgemm_4bit_fewtok_takes says so, else the multi-row GEMV): each row within the GEMV tolerance of gemv_4bit on that
    row alone (|d| <= 2e-2 * rms + 2e-2 * |ref|; bit-identity is given up on the MFMA kernel), and the same bits on a
    second call (deterministic)."""
    F = _F()
    N, K = shape
    torch.manual_seed(N + 3 * K + rows)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    X = torch.randn(rows, K, device=dev, dtype=torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=nested)
    Y = F.gemm_4bit(X, q, st)
    Y2 = F.gemm_4bit(X, q, st)
    assert torch.equal(Y, Y2)
    for t in range(rows):
        y = F.gemv_4bit(X[t:t + 1], q.t(), state=st).reshape(-1).float()
        rms = y.pow(2).mean().sqrt().item()
        assert torch.all((Y[t].float() - y).abs() <= 2e-2 * rms + 2e-2 * y.abs()), f"row {t}"
