"""The hand-written gfx950 GEMM behind the large-prefill 4-bit route (csrc/hgemm.hip, C-ABI chgemm_tn_*): the
F.linear of ref:python_src_quants/autograd/_functions.py:507 after the dequantise, C[m, n] = A[m, k] . W[n, k]^T.

Floating-point contract (a floating-point kernel, so the check is against a plain torch fp32 product of the same
operands): fp32 accumulation, one RNE rounding to bf16 / fp16 at the end -- |C - C32| <= 2^-8 |C32| (bf16) or
2^-11 |C32| (fp16) plus 1e-4 of the output rms for the accumulation-order difference.  Plus: deterministic (same bits
on every call), edge tiles (ragged m, n), the unsupported-shape return code, HIP-graph replay, and the gemm_4bit
"hgemm" route against the oracle."""
import ctypes as ct

import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


def _F():
    import python_src_quants.functional as F
    return F


def _hgemm(F, X, W, out=None, lda=None, ldw=None):
    m, k = X.shape
    n = W.shape[0]
    if out is None:
        out = torch.empty(m, n, device=X.device, dtype=X.dtype)
    fn = F.lib.chgemm_tn_bf16 if X.dtype == torch.bfloat16 else F.lib.chgemm_tn_fp16
    F.pre_call(X.device)
    rc = fn(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k), F.get_ptr(X), ct.c_int32(lda or X.stride(0)), F.get_ptr(W),
            ct.c_int32(ldw or W.stride(0)), F.get_ptr(out), ct.c_int32(out.stride(0)))
    return rc, out


def _hgemm_ws(F, X, W):
    """chgemm_tn_ws_* with the workspace its rule asks for (split-K on small tile grids), as gemm_4bit calls it."""
    m, k = X.shape
    n = W.shape[0]
    out = torch.empty(m, n, device=X.device, dtype=X.dtype)
    nbytes = int(F.lib.chgemm_tn_workspace_bytes(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k)))
    ws = torch.empty(max(nbytes, 4) // 4, dtype=torch.float32, device=X.device)
    fn = F.lib.chgemm_tn_ws_bf16 if X.dtype == torch.bfloat16 else F.lib.chgemm_tn_ws_fp16
    F.pre_call(X.device)
    rc = fn(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k), F.get_ptr(X), ct.c_int32(k), F.get_ptr(W), ct.c_int32(k),
            F.get_ptr(out), ct.c_int32(n), F.get_ptr(ws), ct.c_longlong(nbytes))
    return rc, out


def _check(Y, X, W):
    exp = torch.matmul(X.float(), W.float().t())
    rel = 2.0 ** -8 if Y.dtype == torch.bfloat16 else 2.0 ** -11
    err = (Y.float() - exp).abs()
    bound = rel * exp.abs() + 1e-4 * exp.pow(2).mean().sqrt()
    bad = (err > bound).sum().item()
    assert bad == 0, (bad, err.max().item())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mnk", [(4096, 4096, 11008), (1000, 1100, 4096), (257, 513, 64), (4096, 11008, 4096),
                                 (3, 5, 128), (512, 256, 28672)])
def test_hgemm_against_fp32_product(dev, dtype, mnk):
    F = _F()
    m, n, k = mnk
    g = torch.Generator(device=dev).manual_seed(m * 7 + n)
    X = (torch.rand(m, k, device=dev, generator=g) * 2 - 1).to(dtype)
    W = (torch.rand(n, k, device=dev, generator=g) * 2 - 1).to(dtype)
    rc, Y = _hgemm(F, X, W)
    torch.cuda.synchronize()
    assert rc == 0
    _check(Y, X, W)
    rc2, Y2 = _hgemm(F, X, W)
    torch.cuda.synchronize()
    assert rc2 == 0 and torch.equal(Y, Y2)          # deterministic


def test_hgemm_strided_operands_and_output(dev):
    """Leading dimensions larger than k / n (row slices of wider buffers), output written into a strided view."""
    F = _F()
    m, n, k = 600, 700, 1024
    g = torch.Generator(device=dev).manual_seed(5)
    Xb = torch.randn(m, k + 64, device=dev, generator=g).to(torch.bfloat16)
    Wb = torch.randn(n, k + 128, device=dev, generator=g).to(torch.bfloat16)
    X, W = Xb[:, :k], Wb[:, :k]
    Ob = torch.full((m, n + 8), 7.0, device=dev, dtype=torch.bfloat16)
    rc, _ = _hgemm(F, X, W, out=Ob[:, :n], lda=k + 64, ldw=k + 128)
    torch.cuda.synchronize()
    assert rc == 0
    _check(Ob[:, :n], X, W)
    assert torch.all(Ob[:, n:] == 7.0)              # nothing written past n


def test_hgemm_declines_unsupported_shapes(dev):
    F = _F()
    X = torch.randn(256, 96, device=dev, dtype=torch.bfloat16)
    W = torch.randn(256, 96, device=dev, dtype=torch.bfloat16)
    rc, _ = _hgemm(F, X, W)                          # k % 64 != 0
    assert rc == 1
    X = torch.randn(256, 132, device=dev, dtype=torch.bfloat16)
    W = torch.randn(256, 132, device=dev, dtype=torch.bfloat16)
    rc, _ = _hgemm(F, X[:, :128], W[:, :128], lda=132, ldw=132)   # rows not 16-B aligned
    assert rc == 1


def test_hgemm_graph_replay(dev):
    F = _F()
    m, n, k = 2048, 2048, 2048
    X = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    W = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
    out = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    _hgemm(F, X, W, out=out)
    ref_out = out.clone()
    out.zero_()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            _hgemm(F, X, W, out=out)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref_out)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nested", [False, True])
def test_gemm_4bit_hgemm_route_vs_oracle(dev, dtype, nested):
    """gemm_4bit's "hgemm" route (dequantise into the weight workspace + k_hgemm) within the GEMM tolerance of the fp64
    oracle (the reference's M > 1 algorithm, ref:autograd/_functions.py:491-507), and equal to the dequantised weight
    multiplied by chgemm_tn directly."""
    F = _F()
    M, N, K = 1024, 1536, 2048
    torch.manual_seed(11 + nested)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    X = torch.randn(M, K, device=dev, dtype=dtype)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=nested)
    Y = F.gemm_4bit(X, q, st, _route="hgemm")
    _, Yd = _hgemm_ws(F, X, F.dequantize_4bit(q, st))     # (24 tiles: the route runs split-K)
    assert torch.equal(Y, Yd)
    absmax = F._absmax_fp32(st).cpu().numpy()
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), absmax, N, K, 64, st.code.cpu().numpy(),
                                    "bf16" if dtype == torch.bfloat16 else "fp16")
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-2
    got = Y.float().cpu().numpy().astype(np.float64)
    rms = np.sqrt(np.mean(exp ** 2))
    assert np.all(np.abs(got - exp) <= tol * rms + tol * np.abs(exp))


@pytest.mark.parametrize("mnk", [(4096, 4096, 4096), (700, 900, 1024), (256, 512, 128)])
def test_int8_on_the_4wave_kernel_is_bit_identical(dev, mnk):
    """The same kernel body for int8 (HG_I8_DEQ, forced by cigemm_set_tile(4); the default for full grids since round
    4): the fused mm_dequant bits equal the 8-wave igemm_256's (cigemm_set_tile(8)) / the 128-tile kernel's and the
    default route's -- all exact int32 sums then the same dequant.  The int32
    product itself (igemm_rowmajor) stays on the default kernels under the knob; checked exact here."""
    F = _F()
    m, n, k = mnk
    g = torch.Generator(device=dev).manual_seed(m + k)
    A = torch.randint(-127, 128, (m, k), device=dev, dtype=torch.int8, generator=g)
    B = torch.randint(-127, 128, (n, k), device=dev, dtype=torch.int8, generator=g)
    rs = torch.rand(m, device=dev, generator=g) * 2 + 0.5
    cs = torch.rand(n, device=dev, generator=g) * 2 + 0.5
    bias = torch.randn(n, device=dev, generator=g).half()
    outs = {}
    try:
        for tile in (4, 8, 0):
            F.lib.cigemm_set_tile(tile)
            outs[tile] = (F.igemmlt_dequant(A, B, rs, cs, bias=bias), F.igemm_rowmajor(A, B))
    finally:
        F.lib.cigemm_set_tile(0)
    torch.cuda.synchronize()
    assert torch.equal(outs[4][1], outs[8][1]) and torch.equal(outs[0][1], outs[8][1])
    assert torch.equal(outs[4][0], outs[8][0]) and torch.equal(outs[0][0], outs[8][0])
    exact = (A.double() @ B.double().t())
    assert torch.equal(outs[4][1].double(), exact)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mnk", [(4096, 1024, 8192), (4096, 1024, 28672), (1000, 1100, 4096), (512, 11008, 4096),
                                 (257, 516, 1024), (2048, 3584, 8192), (300, 260, 576)])
def test_hgemm_split_k_against_fp32_product(dev, dtype, mnk):
    """Small tile grids through chgemm_tn_ws_*: split-K (when the launch plan picks it) over fp32 partials in the
    caller's workspace, summed in split order -- within the same fp32-product bound as the unsplit kernel (the k order
    differs, the accumulation is fp32 either way), deterministic across calls, and the workspace query covers the
    plan; a too-small workspace runs the best unsplit plan."""
    F = _F()
    m, n, k = mnk
    g = torch.Generator(device=dev).manual_seed(m + n + k)
    X = (torch.rand(m, k, device=dev, generator=g) * 2 - 1).to(dtype)
    W = (torch.rand(n, k, device=dev, generator=g) * 2 - 1).to(dtype)
    nbytes = int(F.lib.chgemm_tn_workspace_bytes(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k)))
    plan = (ct.c_int * 4)()
    F.lib.chgemm_tn_plan(m, n, k, plan)
    # (the query covers the plan and, since round 5, the plan without the 128 x 128 tile that a side-dequantise launch
    # takes: at least the chosen plan's partials)
    assert nbytes >= (plan[2] * m * n * 4 if plan[2] > 1 else 0), (tuple(plan), nbytes)
    ws = torch.empty(max(nbytes, 4) // 4, dtype=torch.float32, device=dev)
    fn = F.lib.chgemm_tn_ws_bf16 if dtype == torch.bfloat16 else F.lib.chgemm_tn_ws_fp16
    outs = []
    for wsb in (nbytes, nbytes, 0):
        out = torch.empty(m, n, device=dev, dtype=dtype)
        F.pre_call(dev)
        rc = fn(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k), F.get_ptr(X), ct.c_int32(k), F.get_ptr(W), ct.c_int32(k),
                F.get_ptr(out), ct.c_int32(n), F.get_ptr(ws), ct.c_longlong(wsb))
        torch.cuda.synchronize()
        assert rc == 0
        _check(out, X, W)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])
    rc, Yu = _hgemm(F, X, W)                        # the plain entry point runs the unsplit kernel
    torch.cuda.synchronize()
    assert torch.equal(Yu, outs[2])


@pytest.mark.parametrize("mnk", [(4096, 4096, 11008), (1000, 1100, 4096), (257, 513, 64), (300, 260, 128),
                                 (512, 768, 192), (4096, 1024, 28672)])
def test_hgemm_deterministic_and_int8_tile_forms_equal(dev, mnk):
    """Run-to-run determinism of the launched k_hgemm kinds (the removed round-3 schedule arm was not
    deterministic on int8 -- compiler accumulator copies between its asm MFMAs; tests/test_kernel_resources.py
    guards the ISA), checked where that arm failed: three runs of the bf16 / fp16 split-K path and of the int8 4-wave
    igemmlt + dequant are bit-identical, and the 4-wave int8 kernel equals the independent 8-wave igemm_256 bit for bit
    (exact int32, the same per-element dequant)."""
    F = _F()
    m, n, k = mnk
    g = torch.Generator(device=dev).manual_seed(m + 3 * n + k)
    for dtype in (torch.bfloat16, torch.float16):
        X = (torch.rand(m, k, device=dev, generator=g) * 2 - 1).to(dtype)
        W = (torch.rand(n, k, device=dev, generator=g) * 2 - 1).to(dtype)
        outs = []
        for _ in range(3):
            rc, Y = _hgemm_ws(F, X, W)
            torch.cuda.synchronize()
            assert rc == 0
            outs.append(Y)
        _check(outs[0], X, W)
        assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    A = torch.randint(-127, 128, (m, k), device=dev, dtype=torch.int8, generator=g)
    B = torch.randint(-127, 128, (n, k), device=dev, dtype=torch.int8, generator=g)
    rs = torch.rand(m, device=dev, generator=g) * 2 + 0.5
    cs = torch.rand(n, device=dev, generator=g) * 2 + 0.5
    bias = torch.randn(n, device=dev, generator=g).half()
    res = []
    for tile in (8, 4, 4, 4):
        F.lib.cigemm_set_tile(tile)
        try:
            res.append(F.igemmlt_dequant(A, B, rs, cs, bias=bias))
            torch.cuda.synchronize()
        finally:
            F.lib.cigemm_set_tile(0)
    assert all(torch.equal(res[0], r) for r in res[1:])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mnk,plan", [((2048, 4096, 4096), (8, 4, 1)), ((96, 11008, 4096), (4, 8, 5)),
                                      ((4096, 1024, 8192), (8, 4, 2)), ((128, 8192, 8192), (4, 4, 4)),
                                      ((300, 700, 1024), None), ((2051, 1037, 640), None), ((4096, 4096, 2048), (8, 8, 1))])
def test_hgemm_tile_shapes_against_fp32_product(dev, dtype, mnk, plan):
    """The half-width tiles (256 x 128 and 128 x 256, picked by the launch plan for grids that a 256 x 256 tiling leaves
    half empty or rows that waste half a 256-row tile) and, since round 5, the 128 x 128 tile (128 x 8192 x 8192: 4
    splits of 64 tiles instead of 8 of 32), with and without split-K, ragged edges included: against the fp32 product
    (the module's contract) and deterministic; chgemm_tn_plan reports the plan the shape takes."""
    F = _F()
    m, n, k = mnk
    out4 = (ct.c_int * 4)()
    F.lib.chgemm_tn_plan(m, n, k, out4)
    if plan is not None:
        assert tuple(out4[:3]) == plan, tuple(out4)
    g = torch.Generator(device=dev).manual_seed(m + 7 * n + k)
    X = (torch.rand(m, k, device=dev, generator=g) * 2 - 1).to(dtype)
    W = (torch.rand(n, k, device=dev, generator=g) * 2 - 1).to(dtype)
    rc, Y = _hgemm_ws(F, X, W)
    torch.cuda.synchronize()
    assert rc == 0
    _check(Y, X, W)
    rc2, Y2 = _hgemm_ws(F, X, W)
    torch.cuda.synchronize()
    assert rc2 == 0 and torch.equal(Y, Y2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mnk", [(4096, 512, 11008), (4096, 128, 8192), (300, 260, 576), (2051, 1037, 640),
                                 (129, 130, 64), (4096, 1024, 8192), (1, 3, 128)])
def test_hgemm_quarter_tile_against_fp32_product(dev, dtype, mnk):
    """The 128 x 128 tile (round 5; chgemm_set_quarter_tile(2) forces it): with the workspace its plan asks for (split-K
    on small grids) and without (unsplit), ragged edges included, against the fp32 product and deterministic; unsplit it
    runs the same MFMA sequence per output block as the 256 x 256 kernel, so its bits equal chgemm_tn_*'s."""
    F = _F()
    m, n, k = mnk
    g = torch.Generator(device=dev).manual_seed(m + 3 * n + k)
    X = (torch.rand(m, k, device=dev, generator=g) * 2 - 1).to(dtype)
    W = (torch.rand(n, k, device=dev, generator=g) * 2 - 1).to(dtype)
    rc0, Yfull = _hgemm(F, X, W)                        # the unsplit 256 x 256 kernel
    prev = F.lib.chgemm_set_quarter_tile(ct.c_int(2), ct.c_int(0))
    try:
        plan = (ct.c_int * 4)()
        F.lib.chgemm_tn_plan(m, n, k, plan)
        assert tuple(plan[:2]) == (4, 4), tuple(plan)
        rc1, Y = _hgemm_ws(F, X, W)
        rc2, Y2 = _hgemm_ws(F, X, W)
        fn = F.lib.chgemm_tn_ws_bf16 if dtype == torch.bfloat16 else F.lib.chgemm_tn_ws_fp16
        Yu = torch.empty(m, n, device=dev, dtype=dtype)
        F.pre_call(dev)
        rc3 = fn(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k), F.get_ptr(X), ct.c_int32(k), F.get_ptr(W), ct.c_int32(k),
                 F.get_ptr(Yu), ct.c_int32(n), F.get_ptr(None), ct.c_longlong(0))   # no workspace: unsplit 128 x 128
        torch.cuda.synchronize()
    finally:
        F.lib.chgemm_set_quarter_tile(ct.c_int(prev), ct.c_int(0))
    assert rc0 == 0 and rc1 == 0 and rc2 == 0 and rc3 == 0
    _check(Y, X, W)
    assert torch.equal(Y, Y2)
    assert torch.equal(Yu, Yfull)
