"""GPU parity: LLM.int8 path — stats, double_quant, layouts, igemmlt, mm_dequant (bit-exact),
and the fused row-major igemmlt+dequant kernel."""
import ctypes as ct

import numpy as np
import pytest
import torch

from helpers import same_bits
from oracle import ref

pytestmark = pytest.mark.gpu


def _F():
    import python_src_quants.functional as F
    return F


def test_double_quant_golden(golden, dev):
    F = _F()
    A = torch.from_numpy(golden["dq_A"]).to(dev)
    orow, ocol, rs, cs, coo = F.double_quant(A)
    assert coo is None
    assert same_bits(rs.cpu().numpy(), golden["dq_rs"])
    assert same_bits(cs.cpu().numpy(), golden["dq_cs"])
    assert same_bits(orow.cpu().numpy(), golden["dq_row"])
    assert same_bits(ocol.cpu().numpy(), golden["dq_col"])


@pytest.mark.parametrize("shape", [(4096, 4096), (1, 7), (17, 300), (513, 1030), (2048, 11008), (33, 520), (100, 1032),
                                   (1, 8), (31, 4096)])
def test_double_quant_random(dev, shape):
    F = _F()
    torch.manual_seed(shape[0])
    A = (torch.randn(*shape, device=dev) * 4).half()
    A[0, : min(5, shape[1])] = 0
    orow, ocol, rs, cs, _ = F.double_quant(A)
    An = A.cpu().numpy()
    ers, ecs, _ = ref.colrow_absmax(An)
    assert same_bits(rs.cpu().numpy(), ers) and same_bits(cs.cpu().numpy(), ecs)
    er, ec = ref.double_quant(An, ers, ecs)
    assert same_bits(orow.cpu().numpy(), er) and same_bits(ocol.cpu().numpy(), ec)


def test_colrow_stats_threshold(dev):
    F = _F()
    torch.manual_seed(0)
    A = torch.randn(100, 600, device=dev).half()
    A[3, 10] = 20
    A[50, 599] = -30
    A[99, 0] = 7
    rs, cs, nnz = F.get_colrow_absmax(A, threshold=6.0)
    ers, ecs, enr = ref.colrow_absmax(A.cpu().numpy(), threshold=6.0)
    assert same_bits(rs.cpu().numpy(), ers) and same_bits(cs.cpu().numpy(), ecs)
    assert nnz[-1].item() == int(enr.sum()) == 3
    orow, ocol, rs2, cs2, coo = F.double_quant(A, threshold=6.0)
    assert coo is not None and coo.nnz == 3
    got = sorted(zip(coo.rowidx.tolist(), coo.colidx.tolist(), coo.values.float().tolist()))
    assert got == [(3, 10, 20.0), (50, 599, -30.0), (99, 0, 7.0)]
    assert orow[3, 10].item() == 0 and orow[50, 599].item() == 0


@pytest.mark.parametrize("fmt", ["col32", "col_turing", "col_ampere"])
@pytest.mark.parametrize("shape", [(64, 96), (33, 70), (4096, 4096), (1, 1), (130, 4000)])
def test_transforms(dev, fmt, shape):
    F = _F()
    rng = np.random.default_rng(shape[1])
    A = rng.integers(-128, 128, size=shape, dtype=np.int8)
    At = torch.from_numpy(A).to(dev)
    for transpose in (False, True):
        out, st = F.transform(At, fmt, transpose=transpose)
        assert same_bits(out.cpu().numpy(), ref.transform(A, fmt, transpose=transpose)), (fmt, transpose)
    if fmt != "col32":
        out, st = F.transform(At, fmt)
        back, _ = F.transform(out, "row", state=st)
        assert torch.equal(back, At)


def test_transforms_golden(golden, dev):
    F = _F()
    A = torch.from_numpy(golden["ig_A"]).to(dev)
    for fmt in ("col32", "col_turing", "col_ampere"):
        assert same_bits(F.transform(A, fmt)[0].cpu().numpy(), golden[f"tf_{fmt}"])
        assert same_bits(F.transform(A, fmt, transpose=True)[0].cpu().numpy(), golden[f"tfT_{fmt}"])


@pytest.mark.parametrize("formatB", ["col_turing", "col_ampere"])
@pytest.mark.parametrize("mnk", [(64, 40, 96), (4096, 4096, 4096), (1, 1, 1), (77, 300, 1000), (256, 129, 128),
                                 (300, 520, 256)])
def test_igemmlt_exact(dev, formatB, mnk):
    F = _F()
    m, n, k = mnk
    rng = np.random.default_rng(m + n + k)
    A = rng.integers(-127, 128, size=(m, k), dtype=np.int8)
    B = rng.integers(-127, 128, size=(n, k), dtype=np.int8)
    At, Bt = torch.from_numpy(A).to(dev), torch.from_numpy(B).to(dev)
    C32A, SA = F.transform(At, "col32")
    CxB, SB = F.transform(Bt, formatB)
    out32, Sout = F.igemmlt(C32A, CxB, SA, SB)
    got = ref.untransform(out32.cpu().numpy(), m, n, "col32")
    if m * n * k <= 2e8:
        exp = ref.igemmlt(A, B)
    else:
        exp = (torch.from_numpy(A).to(dev).double() @ torch.from_numpy(B).to(dev).double().T).cpu().numpy()
        exp = exp.astype(np.int64).astype(np.int32)
    assert np.array_equal(got, exp)


def test_igemmlt_golden_and_mm_dequant(golden, dev):
    F = _F()
    A = torch.from_numpy(golden["ig_A"]).to(dev)
    B = torch.from_numpy(golden["ig_B"]).to(dev)
    C32A, SA = F.transform(A, "col32")
    CxB, SB = F.transform(B, "col_turing")
    out32, Sout = F.igemmlt(C32A, CxB, SA, SB)
    m, n = golden["ig_C"].shape
    assert np.array_equal(ref.untransform(out32.cpu().numpy(), m, n, "col32"), golden["ig_C"])
    rs = torch.from_numpy(golden["ig_rstat"]).to(dev)
    cs = torch.from_numpy(golden["ig_cstat"]).to(dev)
    bias = torch.from_numpy(golden["ig_bias"]).to(dev)
    D = F.mm_dequant(out32, Sout, rs, cs, bias=bias)
    assert same_bits(D.cpu().numpy(), golden["ig_D"])


def test_igemmlt_int8_out(dev):
    F = _F()
    rng = np.random.default_rng(9)
    m, n, k = 70, 50, 64
    A = rng.integers(-4, 5, size=(m, k), dtype=np.int8)
    B = rng.integers(-4, 5, size=(n, k), dtype=np.int8)
    At, Bt = torch.from_numpy(A).to(dev), torch.from_numpy(B).to(dev)
    C32A, SA = F.transform(At, "col32")
    CxB, SB = F.transform(Bt, "col_ampere")
    out8, Sout = F.igemmlt(C32A, CxB, SA, SB, dtype=torch.int8)
    got = ref.untransform(out8.cpu().numpy(), m, n, "col32")
    assert np.array_equal(got, ref.igemmlt_int8_out(A, B))
    # row-scaled variant through the raw ABI
    scale = torch.from_numpy(rng.uniform(0.01, 0.2, m).astype(np.float32)).to(dev)
    out = torch.zeros_like(out8)
    F.lib.cigemmlt_ampere_8_rowscale(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k), F.get_ptr(C32A), F.get_ptr(CxB),
                                     F.get_ptr(out), F.get_ptr(scale), ct.c_int32(32 * m), ct.c_int32(32 * ((n + 31) // 32) * 32),
                                     ct.c_int32(32 * m))
    torch.cuda.synchronize()
    got = ref.untransform(out.cpu().numpy(), m, n, "col32")
    assert np.array_equal(got, ref.igemmlt_int8_out(A, B, scale.cpu().numpy()))


@pytest.mark.parametrize("mnk", [(4096, 4096, 4096), (300, 200, 448), (1, 64, 128), (129, 257, 1000),
                                 (520, 300, 384), (4096, 4096, 11008)])
def test_igemmlt_row_dequant_fused(dev, mnk):
    F = _F()
    m, n, k = mnk
    rng = np.random.default_rng(k)
    A = rng.integers(-127, 128, size=(m, k), dtype=np.int8)
    B = rng.integers(-127, 128, size=(n, k), dtype=np.int8)
    rs = rng.uniform(0.5, 2, m).astype(np.float32)
    cs = rng.uniform(0.5, 2, n).astype(np.float32)
    bias = rng.standard_normal(n).astype(np.float16)
    At, Bt = torch.from_numpy(A).to(dev), torch.from_numpy(B).to(dev)
    out = F.igemmlt_dequant(At, Bt, torch.from_numpy(rs).to(dev), torch.from_numpy(cs).to(dev),
                            bias=torch.from_numpy(bias).to(dev))
    C = F.igemm_rowmajor(At, Bt)
    if m * n * k <= 2e8:
        exact = ref.igemmlt(A, B)
    else:
        # at the benched sizes: an exact float64 product on the GPU (|sum| <= 127^2 * k < 2^53), an independent
        # check of the int32 result the fused epilogue consumes
        exact = (At.double() @ Bt.double().T).cpu().numpy().astype(np.int64).astype(np.int32)
    assert np.array_equal(C.cpu().numpy(), exact)
    exp = ref.mm_dequant(exact, rs, cs, bias)
    assert same_bits(out.cpu().numpy(), exp)


def test_extract_outliers(dev):
    F = _F()
    rng = np.random.default_rng(4)
    B = rng.integers(-127, 128, size=(40, 96), dtype=np.int8)
    idx = torch.tensor([0, 5, 31, 32, 95], dtype=torch.int32, device=dev)
    for fmt in ("col_turing", "col_ampere"):
        CxB, SB = F.transform(torch.from_numpy(B).to(dev), fmt)
        out = F.extract_outliers(CxB, SB, idx)
        assert np.array_equal(out.cpu().numpy(), B[:, idx.cpu().numpy()])


@pytest.mark.parametrize("shape", [(4096, 11008), (33, 520), (7, 16384), (5, 16392), (3, 8), (300, 1030)])
def test_int8_row_quant_matches_double_quant(dev, shape):
    """The one-pass row quantisation (inference forward) gives double_quant's CA and row stats bit for bit,
    including a zero row and an all-NaN row (row stat stays at the -50000 pre-fill)."""
    F = _F()
    torch.manual_seed(shape[1])
    A = (torch.randn(*shape, device=dev) * 3).half()
    A[0] = 0
    if shape[0] > 2:
        A[2] = float("nan")
    CA, SCA = F.int8_row_quant(A)
    orow, _, rs, _, _ = F.double_quant(A)
    assert same_bits(SCA.cpu().numpy(), rs.cpu().numpy())
    assert same_bits(CA.cpu().numpy(), orow.cpu().numpy())


def test_matmul8bitlt_inference_uses_row_quant(dev):
    """Linear8bitLt-style inference (no grad, threshold 0) through the one-pass quantisation equals the
    double_quant route (same CA, same fused GEMM)."""
    F = _F()
    from python_src_quants.autograd._functions import MatMul8bitLt, MatmulLtState
    torch.manual_seed(8)
    A = torch.randn(64, 512, device=dev).half()
    W = (torch.randn(256, 512, device=dev) * 0.05).half()
    st = MatmulLtState()
    st.has_fp16_weights = False
    st.CB, _, st.SCB, _, _ = F.double_quant(W)
    out = MatMul8bitLt.apply(A, W, None, None, st)
    CA, _, SCA, _, _ = F.double_quant(A)
    exp = F.igemmlt_dequant(CA, st.CB, SCA, st.SCB)
    assert torch.equal(out, exp)


@pytest.mark.parametrize("mnk", [(300, 520, 384), (512, 768, 1024), (257, 1000, 128)])
def test_igemmlt_turing_abi_all_epilogues(dev, mnk):
    """The reference ABI's own formatB (col_turing, ref:functional.py:410-418) at sizes that take the 256-tile
    kernel: cigemmlt_turing_32 / _8 / _8_rowscale against the exact oracle, ragged last tiles included."""
    F = _F()
    m, n, k = mnk
    rng = np.random.default_rng(m * 3 + n)
    A = rng.integers(-127, 128, size=(m, k), dtype=np.int8)
    B = rng.integers(-127, 128, size=(n, k), dtype=np.int8)
    At, Bt = torch.from_numpy(A).to(dev), torch.from_numpy(B).to(dev)
    C32A, SA = F.transform(At, "col32")
    CxB, SB = F.transform(Bt, "col_turing")
    out32, _ = F.igemmlt(C32A, CxB, SA, SB)
    assert np.array_equal(ref.untransform(out32.cpu().numpy(), m, n, "col32"), ref.igemmlt(A, B))
    small = rng.integers(-3, 4, size=(m, k), dtype=np.int8)
    C32s, SAs = F.transform(torch.from_numpy(small).to(dev), "col32")
    out8, _ = F.igemmlt(C32s, CxB, SAs, SB, dtype=torch.int8)
    assert np.array_equal(ref.untransform(out8.cpu().numpy(), m, n, "col32"), ref.igemmlt_int8_out(small, B))
    scale = torch.from_numpy(rng.uniform(0.001, 0.01, m).astype(np.float32)).to(dev)
    out = torch.zeros_like(out8)
    rc = F.lib.cigemmlt_turing_8_rowscale(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k), F.get_ptr(C32A), F.get_ptr(CxB),
                                          F.get_ptr(out), F.get_ptr(scale), ct.c_int32(32 * m),
                                          ct.c_int32(((n + 7) // 8) * 8 * 32), ct.c_int32(32 * m))
    torch.cuda.synchronize()
    assert rc == 0
    got = ref.untransform(out.cpu().numpy(), m, n, "col32")
    assert np.array_equal(got, ref.igemmlt_int8_out(A, B, scale.cpu().numpy()))


@pytest.mark.parametrize("mnk", [(4096, 512, 11008), (2048, 512, 11008), (2048, 1024, 4096), (4096, 2048, 11008),
                                 (300, 258, 2048), (513, 777, 3072), (8, 4096, 4096), (33, 1030, 2048), (1, 256, 1024)])
def test_igemm_split_k_exact(dev, mnk):
    """Split-K over a workspace for small 256-tile grids (the column shards of the multi-GPU step): the int32
    partials are summed exactly, so the int32 result equals the exact product (fp64 GPU matmul) and the fused
    dequant equals the unsplit kernel's bits; auto factor, forced factors and the unsplit kernel compared."""
    F = _F()
    m, n, k = mnk
    g = torch.Generator(device=dev).manual_seed(m + n)
    A = torch.randint(-127, 128, (m, k), device=dev, dtype=torch.int8, generator=g)
    B = torch.randint(-127, 128, (n, k), device=dev, dtype=torch.int8, generator=g)
    exp = (A.double() @ B.double().T).round().to(torch.int64).to(torch.int32)
    rs = torch.rand(m, device=dev, generator=g) * 2 + 0.5
    cs = torch.rand(n, device=dev, generator=g) * 2 + 0.5
    bias = torch.randn(n, device=dev, generator=g).half()
    outs32, outs16 = [], []
    try:
        for ks in (1, -1, 3, 16):
            F.lib.cigemm_set_splitk(ks)
            outs32.append(F.igemm_rowmajor(A, B))
            outs16.append(F.igemmlt_dequant(A, B, rs, cs, bias=bias))
            torch.cuda.synchronize()
            assert F.lib.cget_last_error() == 0
    finally:
        F.lib.cigemm_set_splitk(-1)
    for o in outs32:
        assert torch.equal(o, exp)
    for o in outs16[1:]:
        assert torch.equal(o.view(torch.int16), outs16[0].view(torch.int16))
    if n >= 256 and k % 128 == 0 and k >= 2 * 128 * (2 if m < 256 else 8):
        tiles = ((m + 255) // 256) * ((n + 255) // 256)
        assert (F.lib.cigemmlt_workspace_bytes(m, n, k) > 0) == (tiles < 200)
