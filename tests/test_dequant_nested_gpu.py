"""Round 5: the streaming 4-bit dequantise with nested statistics can read each wave's 64 statistic codes and its
second-level scale by scalar loads (k_dequantize_4bit_stream SQ, cdequantize_set_nested_scalar(1); measured slower, so
off by default).  It must equal the per-lane form and the oracle bit for bit: whole and ragged tails (waves whose 64 blocks run past the end fall back to
the per-lane loads), a code array that is not 64-B aligned (the launch keeps the per-lane form), NF4 / FP4, bf16 / fp16,
and the metric weight through gemm_4bit's dequantise + k_hgemm route."""
import ctypes as ct

import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


def _F():
    import python_src_quants.functional as F
    return F


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("qt", ["nf4", "fp4"])
@pytest.mark.parametrize("shape", [(4096, 11008), (1000, 4096), (37, 320), (3, 64), (4096, 4096)])
def test_nested_scalar_stats_equal_per_lane_and_oracle(dev, dtype, qt, shape):
    F = _F()
    torch.manual_seed(shape[0] + shape[1])
    W = (torch.randn(*shape, device=dev) * 0.02).to(dtype)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type=qt, compress_statistics=True)
    prev = F.lib.cdequantize_set_nested_scalar(ct.c_int(1))
    try:
        a = F.dequantize_4bit(q, st)
        F.lib.cdequantize_set_nested_scalar(ct.c_int(0))
        b = F.dequantize_4bit(q, st)
    finally:
        F.lib.cdequantize_set_nested_scalar(ct.c_int(prev))
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    absmax = F._absmax_fp32(st).cpu().numpy()
    name = "bf16" if dtype == torch.bfloat16 else "fp16"
    exp = ref.dequantize_blockwise(q.cpu().numpy().reshape(-1), absmax, 64, W.numel(), qt, name)
    got = a.reshape(-1).cpu().view(torch.int16).numpy().view(np.uint16)
    assert np.array_equal(got, np.asarray(exp).view(np.uint16))


def test_nested_scalar_stats_unaligned_codes(dev):
    """Codes at a 16-B offset from a 64-B boundary (a sliced state): the launch keeps the per-lane loads, same bits."""
    F = _F()
    torch.manual_seed(7)
    W = (torch.randn(2048, 4096, device=dev) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    ref_out = F.dequantize_4bit(q, st)
    buf = torch.empty(st.absmax.numel() + 16, dtype=torch.uint8, device=dev)
    shifted = buf[16:16 + st.absmax.numel()]
    shifted.copy_(st.absmax)
    assert shifted.data_ptr() % 64 != 0
    st.absmax = shifted
    out = F.dequantize_4bit(q, st)
    assert torch.equal(out.view(torch.int16), ref_out.view(torch.int16))
