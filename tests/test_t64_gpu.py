"""The 33..64-token kernel (gemm4bit_t64.hip): 192 weight rows x 64 tokens per workgroup, split-K with the ordered
reduce, every operand by LDS-DMA.  Its arithmetic is the whole-K few-token kernel's (T(code) x tokens summed per
64-element block on the MFMA, then x absmax), so the bar is the GEMV's / the tile kernels' against the fp64 oracle;
deterministic; the in-kernel nested decode equals passing the decoded absmax.  Auto at 33..64 rows; forced
(cgemm_4bit_set_t64_mode(2)) also at 1..32 rows; shapes it does not take (blocksize != 64, K % 256) fall back.  Both
forms of the kernel: 4 waves (one per SIMD) and 8 waves (two per SIMD, the two waves of a row set on alternate blocks,
their partial sums added in LDS; cgemm_4bit_set_t64_waves).  Round 5: the register-fed form (48 rows x whole K per
workgroup, its 4 waves splitting K, K-parts summed in LDS in split order; cgemm_4bit_set_t64_regfed) against the oracle,
and bit for bit against the LDS-DMA form + reduce launch where both split K the same way."""
import ctypes as ct

import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


def _F():
    import python_src_quants.functional as F
    return F


def _close(got, exp, rtol, atol_rel):
    rms = float(np.sqrt(np.mean(exp.astype(np.float64) ** 2))) + 1e-12
    bad = np.abs(got - exp) > atol_rel * rms + rtol * np.abs(exp)
    return float(bad.mean()), float(np.max(np.abs(got - exp)))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("qt,bs", [("nf4", 64), ("fp4", 64), ("nf4", 256)])
@pytest.mark.parametrize("mnk,mode", [((33, 11008, 4096), 0), ((64, 11008, 4096), 0), ((48, 4096, 11008), 0),
                                      ((64, 4096, 4096), 0), ((40, 1000, 2304), 0), ((64, 193, 256), 0),
                                      ((57, 3584, 8192), 0), ((1, 4096, 4096), 2), ((17, 520, 768), 2),
                                      ((64, 28672, 512), 0)])
@pytest.mark.parametrize("waves,regfed", [(1, 1), (2, 1), (1, 2)])
def test_t64_vs_oracle(dev, dtype, nested, qt, bs, mnk, mode, waves, regfed):
    F = _F()
    M, N, K = mnk
    torch.manual_seed(M * 7 + N + K + bs)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    X = torch.randn(M, K, device=dev, dtype=dtype)
    q, st = F.quantize_4bit(W, blocksize=bs, quant_type=qt, compress_statistics=nested)
    prev = F.lib.cgemm_4bit_set_t64_mode(ct.c_int(mode))
    prev_w = F.lib.cgemm_4bit_set_t64_waves(ct.c_int(waves))
    prev_r = F.lib.cgemm_4bit_set_t64_regfed(ct.c_int(regfed))
    saved = F.GEMM_4BIT_GEMV_TOKENS
    F.GEMM_4BIT_GEMV_TOKENS = 1
    F.set_fewtok_mode(1)                               # (forced rows <= 32: not the whole-K kernel)
    try:
        Y = F.gemm_4bit(X, q, st)
        Y2 = F.gemm_4bit(X, q, st)
        Yp = F.gemm_4bit(X, q, st, absmax=F._absmax_fp32(st))
    finally:
        F.lib.cgemm_4bit_set_t64_mode(ct.c_int(prev))
        F.lib.cgemm_4bit_set_t64_waves(ct.c_int(prev_w))
        F.lib.cgemm_4bit_set_t64_regfed(ct.c_int(prev_r))
        F.set_fewtok_mode(0)
        F.GEMM_4BIT_GEMV_TOKENS = saved
    assert Y.shape == (M, N) and Y.dtype == dtype
    assert torch.equal(Y, Y2)                          # deterministic (splits summed in order)
    assert torch.equal(Y, Yp)                          # in-kernel nested decode = the decoded absmax passed in
    absmax = F._absmax_fp32(st).cpu().numpy()
    exp = ref.gemm_4bit_dequant_ref(X.float().cpu().numpy(), q.cpu().numpy(), absmax, N, K, bs,
                                    st.code.cpu().numpy(), "bf16" if dtype == torch.bfloat16 else "fp16")
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-2
    frac, err = _close(Y.float().cpu().numpy(), exp, tol, tol)
    assert frac == 0.0, err


def test_t64_is_the_default_at_33_to_64_rows(dev):
    """At 33..64 rows with blocksize 64 and K % 256 == 0 the auto rule takes the new kernel, and its result differs
    from the split-K weight-stream kernel it replaced only within the tolerance (different block-sum association)."""
    F = _F()
    N, K, M = 11008, 4096, 64
    torch.manual_seed(3)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    Y = F.gemm_4bit(X, q, st)
    prev = F.lib.cgemm_4bit_set_t64_mode(ct.c_int(1))
    try:
        Yo = F.gemm_4bit(X, q, st)
    finally:
        F.lib.cgemm_4bit_set_t64_mode(ct.c_int(prev))
    assert not torch.equal(Y, Yo)                      # a different kernel ran
    e = Yo.float()
    rms = e.pow(2).mean().sqrt()
    assert bool(((Y.float() - e).abs() <= 2e-2 * rms + 2e-2 * e.abs()).all())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mnk", [(64, 11008, 4096), (33, 4096, 11008), (40, 1000, 2304), (64, 193, 4096),
                                 (57, 3584, 8192), (48, 520, 4096)])
@pytest.mark.parametrize("splits", [0, 3, 11])
@pytest.mark.parametrize("waves", [1, 2])
def test_t64_in_kernel_combine_matches_reduce_launch(dev, dtype, mnk, splits, waves):
    """Write-through partial stores (dwords, staged 16-B lines) equal plain ones bit for bit.  The split-K partials summed by each row tile's last workgroup to finish (agent-scope release / acquire
    hand-off, one ticket per row tile) equal the separate k_skinny_reduce launch bit for bit: same additions in split
    order; whole float4 rows (N % 4 == 0, partial last row tile) and the scalar form (N = 193); more than 8 splits
    (the batched loads' second round).  Ten launches in a row: every ticket is back at zero after its launch.  A
    captured launch takes the reduce launch (no ticket set is baked into a graph), so its replays give the same bits."""
    F = _F()
    M, N, K = mnk
    torch.manual_seed(N + K + M)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    X = torch.randn(M, K, device=dev, dtype=dtype)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    prev_ks = F.lib.cgemm_4bit_set_t64_splits(ct.c_int(splits))
    prev_mode = F.lib.cgemm_4bit_set_t64_mode(ct.c_int(2))
    prev_w = F.lib.cgemm_4bit_set_t64_waves(ct.c_int(waves))
    prev_ps = F.lib.cgemm_4bit_set_t64_pstore(ct.c_int(0))
    prev_r = F.lib.cgemm_4bit_set_t64_regfed(ct.c_int(1))
    try:
        F.lib.cgemm_4bit_set_t64_combine(ct.c_int(0))
        ref_out = F.gemm_4bit(X, q, st)                 # plain partials + the reduce launch
        outs = []
        for ps in (1, 2):                               # write-through partials (dwords / staged 16-B lines)
            F.lib.cgemm_4bit_set_t64_pstore(ct.c_int(ps))
            outs.append(F.gemm_4bit(X, q, st))
        F.lib.cgemm_4bit_set_t64_combine(ct.c_int(1))
        outs += [F.gemm_4bit(X, q, st) for _ in range(10)]
        out = torch.empty_like(ref_out)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            F.gemm_4bit(X, q, st, out=out)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                F.gemm_4bit(X, q, st, out=out)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        replays = []
        for _ in range(3):
            out.zero_()
            g.replay()
            torch.cuda.synchronize()
            replays.append(out.clone())
    finally:
        F.lib.cgemm_4bit_set_t64_combine(ct.c_int(0))
        F.lib.cgemm_4bit_set_t64_pstore(ct.c_int(prev_ps))
        F.lib.cgemm_4bit_set_t64_mode(ct.c_int(prev_mode))
        F.lib.cgemm_4bit_set_t64_splits(ct.c_int(prev_ks))
        F.lib.cgemm_4bit_set_t64_waves(ct.c_int(prev_w))
        F.lib.cgemm_4bit_set_t64_regfed(ct.c_int(prev_r))
    for o in outs + replays:
        assert torch.equal(o, ref_out)


@pytest.mark.parametrize("nested", [False, True])
def test_t64_eight_waves_close_to_four(dev, nested):
    """The 8-wave form sums each row set's blocks in two interleaved halves (then first + second): within the GEMM
    tolerance of the 4-wave form, deterministic, and the same under a HIP-graph replay."""
    F = _F()
    N, K, M = 11008, 4096, 64
    torch.manual_seed(5 + nested)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=nested)
    prev = F.lib.cgemm_4bit_set_t64_waves(ct.c_int(1))
    prev_r = F.lib.cgemm_4bit_set_t64_regfed(ct.c_int(1))
    try:
        Y4 = F.gemm_4bit(X, q, st)
        F.lib.cgemm_4bit_set_t64_waves(ct.c_int(2))
        Y8 = F.gemm_4bit(X, q, st)
        Y8b = F.gemm_4bit(X, q, st)
        out = torch.empty_like(Y8)
        F.gemm_4bit(X, q, st, out=out)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                F.gemm_4bit(X, q, st, out=out)
        torch.cuda.current_stream().wait_stream(s)
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
    finally:
        F.lib.cgemm_4bit_set_t64_waves(ct.c_int(prev))
        F.lib.cgemm_4bit_set_t64_regfed(ct.c_int(prev_r))
    assert torch.equal(Y8, Y8b) and torch.equal(out, Y8)
    e = Y4.float()
    rms = e.pow(2).mean().sqrt()
    assert bool(((Y8.float() - e).abs() <= 1e-2 * rms + 1e-2 * e.abs()).all())


def _regfed_run(F, X, q, st, regfed, splits=0, waves=1, out=None):
    prev = (F.lib.cgemm_4bit_set_t64_regfed(ct.c_int(regfed)), F.lib.cgemm_4bit_set_t64_splits(ct.c_int(splits)),
            F.lib.cgemm_4bit_set_t64_waves(ct.c_int(waves)), F.lib.cgemm_4bit_set_t64_mode(ct.c_int(2)))
    try:
        return F.gemm_4bit(X, q, st, out=out)
    finally:
        F.lib.cgemm_4bit_set_t64_regfed(ct.c_int(prev[0]))
        F.lib.cgemm_4bit_set_t64_splits(ct.c_int(prev[1]))
        F.lib.cgemm_4bit_set_t64_waves(ct.c_int(prev[2]))
        F.lib.cgemm_4bit_set_t64_mode(ct.c_int(prev[3]))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("mnk", [(64, 11008, 4096), (33, 11008, 4096), (48, 1000, 2304), (64, 193, 8192),
                                 (40, 4096, 11008), (64, 11008, 256)])
def test_t64r_equals_lds_form_plus_reduce(dev, dtype, nested, mnk):
    """Where both forms split K into the same groups (the LDS-DMA form forced to 4 splits: kc = ceil(groups / 4), the
    register-fed form's per-wave share), the register-fed form's in-LDS sum of its K-parts equals the LDS-DMA form's
    partials + k_skinny_reduce bit for bit ((p0 + p1) + p2 + p3, one RNE cast), at whole and ragged row tiles (N = 193,
    1000), 33 tokens, 3 parts (K = 2304: 9 groups), one part (K = 256)."""
    F = _F()
    M, N, K = mnk
    torch.manual_seed(M + N + K + nested)
    W = (torch.randn(N, K, device=dev) * 0.02).to(dtype)
    X = torch.randn(M, K, device=dev, dtype=dtype)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=nested)
    a = _regfed_run(F, X, q, st, 1, splits=4)
    b = _regfed_run(F, X, q, st, 2)
    c = _regfed_run(F, X, q, st, 2)
    assert torch.equal(b, c)
    assert torch.equal(a, b)


def test_t64r_auto_rule_and_graph_replay(dev):
    """Auto (cgemm_4bit_set_t64_regfed(0)): the register-fed form at 11008 out-features (230 row tiles of 48 fill the
    CUs), the LDS-DMA form at 4096 (86 would not); the default (off) is the LDS-DMA form.  Under HIP-graph capture the
    register-fed launch replays to the same bits."""
    F = _F()
    torch.manual_seed(11)
    for N, K, regfed_expected in [(11008, 4096, True), (4096, 4096, False)]:
        W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        X = torch.randn(64, K, device=dev, dtype=torch.bfloat16)
        q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
        default = F.gemm_4bit(X, q, st)
        auto = _regfed_run(F, X, q, st, 0)
        forced = _regfed_run(F, X, q, st, 2)
        off = _regfed_run(F, X, q, st, 1)
        assert torch.equal(default, off)
        if regfed_expected:
            assert torch.equal(auto, forced)
        else:
            assert torch.equal(auto, off)
    out = torch.empty_like(forced)
    prev = F.lib.cgemm_4bit_set_t64_regfed(ct.c_int(2))
    try:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            F.gemm_4bit(X, q, st, out=out)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                F.gemm_4bit(X, q, st, out=out)
        torch.cuda.current_stream().wait_stream(s)
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
    finally:
        F.lib.cgemm_4bit_set_t64_regfed(ct.c_int(prev))
    assert torch.equal(out, forced)
