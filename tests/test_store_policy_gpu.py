"""The store-policy knobs change where the bytes are cached, never the bytes: the 4-bit streaming dequantise's outputs
(cdequantize_set_store_policy 0 write-back / 1 non-temporal / 2 write-through, the default), k_hgemm's C and split-K
partials (chgemm_set_c_store 0 / 1, the default) and the int8 row quantise (cint8_set_row_quant_store) give
bit-identical results -- dequantise, the NF4 GEMM on the 256 x 256 / half-width / split-K plans, int8 igemmlt+dequant."""
import ctypes as ct

import pytest
import torch

pytestmark = pytest.mark.gpu

import python_src_quants.functional as F  # noqa: E402


def _knobs(dq, cs, rq):
    return (F.lib.cdequantize_set_store_policy(ct.c_int(dq)), F.lib.chgemm_set_c_store(ct.c_int(cs)),
            F.lib.cint8_set_row_quant_store(ct.c_int(rq)))


@pytest.mark.parametrize("mnk", [(4096, 4096, 2048), (2048, 1024, 4096), (4096, 512, 8192), (2048, 4096, 1152)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_store_policies_bit_identical(dev, mnk, dtype):
    M, N, K = mnk
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    X = torch.randn(M, K, device=dev, generator=g).to(dtype)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(dtype)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    A = (torch.randn(M, K, device=dev, generator=g) * 2).half()
    CB, _, SCB, _, _ = F.double_quant((W * 3).half())
    results = {}
    prev = _knobs(0, 0, 0)
    try:
        for dq, cs, rq in [(0, 0, 0), (1, 0, 0), (2, 1, 1), (2, 0, 0), (0, 1, 0)]:
            _knobs(dq, cs, rq)
            wd = F.dequantize_4bit(q, st)
            y = F.gemm_4bit(X, q, st, _route="hgemm")
            ca, sca = F.int8_row_quant(A)
            y8 = F.igemmlt_dequant(ca, CB, sca, SCB)
            torch.cuda.synchronize()
            results[(dq, cs, rq)] = (wd, y, ca, sca, y8)
    finally:
        _knobs(*prev)
    ref = results[(0, 0, 0)]
    for key, got in results.items():
        for a, b in zip(ref, got):
            assert torch.equal(a, b), key
