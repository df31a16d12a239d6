"""LDS-DMA staging invariants of the production kernels, checked dynamically: before every launch the LDS of every CU is
filled with 0xFFFFFFFF (cprobe_lds_poison: a NaN in fp32, bf16 and fp16; LDS is not cleared between kernels -- the
positive control below proves the next kernel sees it), then the kernel runs on ragged / short-last-group shapes and
must return bit for bit what it returns without the poison.  A read of a staged slot before its LDS-DMA landed (a
vmcnt / barrier count one short), a slot that a short last group never writes, or a wrong M0 destination would read
the poison and change the result (round 3 dropped a GEMV variant that returned NaN this way).
Kernels covered: k_hgemm (bf16 / fp16, split-K, int8 4-wave), igemm_256 (8-wave), the whole-K few-token kernel, the
split-K few-token kernel, the decode GEMVs (balanced / dot / wide / multi-row), the fused NF4 GEMM, the dequantise and
k_hgemm with the side dequantise of the next weight (prefetch)."""
import ctypes as ct

import pytest
import torch

pytestmark = pytest.mark.gpu

POISON = 0xFFFFFFFF


def _F():
    import python_src_quants.functional as F
    return F


def _poison(F, dev):
    F.pre_call(dev)
    assert F.lib.cprobe_lds_poison(ct.c_uint(POISON), 4096) == 0


@pytest.fixture(scope="module")
def poison_visible(dev):
    """Positive control: after the poison launch, a kernel that reads LDS it never wrote sees the pattern."""
    F = _F()
    out = torch.zeros(256 * 256, dtype=torch.int32, device=dev)
    _poison(F, dev)
    F.pre_call(dev)
    assert F.lib.cprobe_lds_peek(F.get_ptr(out), 256) == 0
    torch.cuda.synchronize()
    seen = (out == -1).float().mean().item()
    if seen < 0.5:
        pytest.skip(f"LDS poison not observable on this stack ({seen:.2f} of the peeked words)")
    return True


def _same_under_poison(F, dev, fn, reps=3):
    torch.cuda.synchronize()
    ref = fn().clone()
    torch.cuda.synchronize()
    for _ in range(reps):
        _poison(F, dev)
        got = fn()
        torch.cuda.synchronize()
        assert torch.equal(got, ref), "result changed under LDS poisoning"
    if ref.is_floating_point():
        assert not torch.isnan(ref).any()


def test_control_sees_poison(dev, poison_visible):
    assert poison_visible


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mnk", [(257, 513, 64), (300, 260, 192), (1000, 1100, 4096), (512, 768, 4096),
                                 (4096, 1024, 8192)])
def test_hgemm_under_poison(dev, poison_visible, dtype, mnk):
    F = _F()
    m, n, k = mnk
    g = torch.Generator(device=dev).manual_seed(m + n + k)
    X = (torch.rand(m, k, device=dev, generator=g) * 2 - 1).to(dtype)
    W = (torch.rand(n, k, device=dev, generator=g) * 2 - 1).to(dtype)
    out = torch.empty(m, n, device=dev, dtype=dtype)
    nbytes = int(F.lib.chgemm_tn_workspace_bytes(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k)))
    ws = torch.empty(max(nbytes, 4) // 4, dtype=torch.float32, device=dev)
    fn_c = F.lib.chgemm_tn_ws_bf16 if dtype == torch.bfloat16 else F.lib.chgemm_tn_ws_fp16

    def run():
        F.pre_call(dev)
        assert fn_c(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k), F.get_ptr(X), ct.c_int32(k), F.get_ptr(W),
                    ct.c_int32(k), F.get_ptr(out), ct.c_int32(n), F.get_ptr(ws), ct.c_longlong(nbytes)) == 0
        return out
    _same_under_poison(F, dev, run)


@pytest.mark.parametrize("tile", [4, 8])
@pytest.mark.parametrize("mnk", [(700, 900, 1024), (4096, 4096, 256), (256, 512, 128)])
def test_int8_gemm_under_poison(dev, poison_visible, tile, mnk):
    F = _F()
    m, n, k = mnk
    g = torch.Generator(device=dev).manual_seed(m * 3 + k)
    A = torch.randint(-127, 128, (m, k), device=dev, dtype=torch.int8, generator=g)
    B = torch.randint(-127, 128, (n, k), device=dev, dtype=torch.int8, generator=g)
    rs = torch.rand(m, device=dev, generator=g) + 0.5
    cs = torch.rand(n, device=dev, generator=g) + 0.5
    out = torch.empty(m, n, device=dev, dtype=torch.float16)
    F.lib.cigemm_set_tile(tile)
    try:
        _same_under_poison(F, dev, lambda: F.igemmlt_dequant(A, B, rs, cs, out=out))
    finally:
        F.lib.cigemm_set_tile(0)


def _quantized(F, dev, N, K, nested, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    return F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=nested)


@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("rows,N,K,mode", [(3, 11008, 4096, 0), (8, 4096, 4096, 0), (17, 11008, 4096, 2),
                                           (32, 1001, 2048, 2), (5, 4099, 4096, 2), (40, 4096, 11008, 0),
                                           (64, 11008, 4096, 0), (2, 11008, 4096, 1), (4, 1000, 192, 1)])
def test_few_token_under_poison(dev, poison_visible, nested, rows, N, K, mode):
    """mode: the whole-K kernel auto (0) / off (1: multi-row GEMV and split-K) / forced wherever it fits (2)."""
    F = _F()
    q, st = _quantized(F, dev, N, K, nested, rows + N)
    X = torch.randn(rows, K, device=dev, dtype=torch.bfloat16, generator=torch.Generator(device=dev).manual_seed(3))
    out = torch.empty(rows, N, device=dev, dtype=torch.bfloat16)
    F.set_fewtok_mode(mode)
    try:
        _same_under_poison(F, dev, lambda: F.gemm_4bit(X, q, st, out=out))
    finally:
        F.set_fewtok_mode(0)


@pytest.mark.parametrize("nested", [False, True])
@pytest.mark.parametrize("N,K", [(11008, 4096), (4096, 11008), (1000, 192), (37, 40960), (1024, 28672), (77, 2112)])
def test_gemv_under_poison(dev, poison_visible, nested, N, K):
    F = _F()
    q, st = _quantized(F, dev, N, K, nested, N + K)
    x = torch.randn(1, K, device=dev, dtype=torch.bfloat16, generator=torch.Generator(device=dev).manual_seed(4))
    out = torch.empty(1, N, device=dev, dtype=torch.bfloat16)
    _same_under_poison(F, dev, lambda: F.gemv_4bit(x, q.t(), out=out, state=st))


@pytest.mark.parametrize("rows,N,K", [(300, 1024, 4096), (700, 512, 11008), (2048, 4096, 1024)])
def test_fused_and_dequant_under_poison(dev, poison_visible, rows, N, K):
    F = _F()
    q, st = _quantized(F, dev, N, K, True, rows)
    X = torch.randn(rows, K, device=dev, dtype=torch.bfloat16, generator=torch.Generator(device=dev).manual_seed(5))
    out = torch.empty(rows, N, device=dev, dtype=torch.bfloat16)
    _same_under_poison(F, dev, lambda: F.gemm_4bit(X, q, st, out=out, _route="fused"))
    _same_under_poison(F, dev, lambda: F.dequantize_4bit(q, st))


@pytest.mark.parametrize("mnk,nxt", [((300, 260, 192), (1003, 192)), ((4096, 1024, 8192), (11008, 4096)),
                                     ((1000, 1100, 4096), (64, 64))])
@pytest.mark.parametrize("nested", [True, False])
def test_prefetch_side_dequant_under_poison(dev, poison_visible, mnk, nxt, nested):
    """k_hgemm with the next weight's dequantise inside it (its landing slots, pair table and code2 copy in LDS): the
    GEMM output and the written weight must not change under the poison."""
    F = _F()
    m, n, k = mnk
    g = torch.Generator(device=dev).manual_seed(m + k)
    X = (torch.rand(m, k, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    W = (torch.rand(n, k, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    Wn = (torch.randn(*nxt, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(Wn, blocksize=64, quant_type="nf4", compress_statistics=nested)
    out = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    target = torch.empty(nxt[0] * nxt[1], device=dev, dtype=torch.bfloat16)
    nbytes = int(F.lib.chgemm_tn_workspace_bytes(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k)))
    ws = torch.empty(max(nbytes, 4) // 4, dtype=torch.float32, device=dev)

    def run():
        F.pre_call(dev)
        assert F._launch_prefetch_gemm(X, W, out, ws, nbytes, (q, st), target) == 0
        return torch.cat([out.view(-1), target])
    _same_under_poison(F, dev, run)
    torch.cuda.synchronize()
    assert torch.equal(target, F.dequantize_4bit(q, st).view(-1))
