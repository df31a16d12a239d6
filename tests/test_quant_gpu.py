"""GPU parity: blockwise quantize/dequantize (HIP) vs the CPU oracle — bit-exact.

Covers cquantize_blockwise_* / cdequantize_blockwise_* (ref:sycl/pythonInterface.cpp:199-221)
for fp32/fp16/bf16 x {nf4, fp4, dynamic 8-bit} x blocksizes 64..4096, ragged tails (n not a
multiple of the blocksize, odd n), n == 1, all-zero blocks, NaN, and misaligned pointers.
"""
import ctypes as ct

import numpy as np
import pytest
import torch

from helpers import DTYPES, same_bits, to_numpy, to_torch
from oracle import ref
from oracle.maps import create_dynamic_map

pytestmark = pytest.mark.gpu


def _F():
    import python_src_quants.functional as F
    return F


def _quant_abi(F, dtype, qtype):
    suffix = "" if qtype == "8bit" else f"_{qtype}"
    return getattr(F.lib, f"cquantize_blockwise_{dtype}{suffix}"), getattr(F.lib, f"cdequantize_blockwise_{dtype}{suffix}")


def _run_quant(F, dev, a_np, dtype, qtype, bs, code_np):
    n = a_np.size
    A = to_torch(a_np, dtype, dev)
    nb = (n + bs - 1) // bs
    absmax = torch.zeros(nb, dtype=torch.float32, device=dev)
    out = torch.zeros(n if qtype == "8bit" else (n + 1) // 2, dtype=torch.uint8, device=dev)
    code = torch.from_numpy(code_np).to(dev)
    qfn, _ = _quant_abi(F, dtype, qtype)
    qfn(F.get_ptr(code if qtype == "8bit" else None), F.get_ptr(A), F.get_ptr(absmax), F.get_ptr(out), ct.c_int32(bs), ct.c_int(n))
    torch.cuda.synchronize()
    assert F.lib.cget_last_error() == 0
    return absmax.cpu().numpy(), out.cpu().numpy()


def _run_dequant(F, dev, q_np, absmax_np, n, qtype, bs, out_dtype, code_np):
    q = torch.from_numpy(q_np).to(dev)
    absmax = torch.from_numpy(absmax_np).to(dev)
    out = torch.empty(n, dtype=DTYPES[out_dtype], device=dev)
    code = torch.from_numpy(code_np).to(dev)
    _, dfn = _quant_abi(F, out_dtype, qtype)
    dfn(F.get_ptr(code if qtype == "8bit" else None), F.get_ptr(q), F.get_ptr(absmax), F.get_ptr(out), ct.c_int(bs), ct.c_int(n))
    torch.cuda.synchronize()
    assert F.lib.cget_last_error() == 0
    return to_numpy(out, out_dtype)


def test_golden_quant_dequant(golden, dev):
    F = _F()
    code = golden["dynamic_code"]
    for i in range(int(golden["n_quant_cases"])):
        di, qi, bs, n = golden[f"q{i}_meta"].tolist()
        dtype, qtype = ["fp32", "fp16", "bf16"][di], ["nf4", "fp4", "8bit"][qi]
        absmax, q = _run_quant(F, dev, golden[f"q{i}_in"], dtype, qtype, bs, code)
        assert same_bits(absmax, golden[f"q{i}_absmax"]), (i, dtype, qtype, bs, n, "absmax")
        assert same_bits(q, golden[f"q{i}_q"]), (i, dtype, qtype, bs, n, "codes")
        for od in ("fp32", "fp16", "bf16"):
            y = _run_dequant(F, dev, golden[f"q{i}_q"], golden[f"q{i}_absmax"], n, qtype, bs, od, code)
            assert same_bits(y, golden[f"q{i}_deq_{od}"]), (i, dtype, qtype, bs, n, od)


@pytest.mark.parametrize("qtype", ["nf4", "fp4", "8bit"])
@pytest.mark.parametrize("bs", [64, 128, 256, 512, 1024, 2048, 4096])
@pytest.mark.parametrize("dtype", ["bf16", "fp16", "fp32"])
def test_random_sizes_bit_exact(dev, qtype, bs, dtype):
    F = _F()
    code = create_dynamic_map()
    rng = np.random.default_rng(bs * 7 + len(qtype))
    for n in (bs * 37 + 3, bs - 1, 2 * bs, 1, 131071, 8 * 100003):
        x = (rng.standard_normal(n) * rng.uniform(0.1, 10)).astype(np.float32)
        if n > 3:
            x[rng.integers(0, n, 3)] = np.nan
        a = ref.f32_to_bf16_bits(x) if dtype == "bf16" else x.astype(np.float16 if dtype == "fp16" else np.float32)
        xf = ref.as_f32(a, dtype)
        ea, eq = ref.quantize_blockwise(xf, bs, qtype, code=code)
        absmax, q = _run_quant(F, dev, a, dtype, qtype, bs, code)
        assert same_bits(absmax, ea), (n, "absmax")
        assert same_bits(q, eq), (n, "codes", np.flatnonzero(q != eq)[:8])
        for od in ("bf16", "fp16", "fp32"):
            y = _run_dequant(F, dev, eq, ea, n, qtype, bs, od, code)
            assert same_bits(y, ref.dequantize_blockwise(eq, ea, bs, n, qtype, od, code=code)), (n, od)


def test_zero_block_and_misaligned(dev):
    F = _F()
    n, bs = 64 * 9, 64
    x = np.random.default_rng(0).standard_normal(n + 8).astype(np.float32)
    x[65:129] = 0                             # = elements 64..127 of the offset view below
    base = torch.from_numpy(x).to(dev)
    A = base[1:n + 1]                         # 4-byte offset: forces the unaligned (scalar) path
    a_np = x[1:n + 1]
    for qtype in ("nf4", "fp4"):
        absmax = torch.zeros(n // bs, device=dev)
        outbuf = torch.zeros((n + 1) // 2 + 1, dtype=torch.uint8, device=dev)
        out = outbuf[1:]                      # odd byte offset
        getattr(F.lib, f"cquantize_blockwise_fp32_{qtype}")(None, F.get_ptr(A), F.get_ptr(absmax), F.get_ptr(out),
                                                            ct.c_int32(bs), ct.c_int(n))
        ea, eq = ref.quantize_blockwise(a_np, bs, qtype)
        assert same_bits(absmax.cpu().numpy(), ea)
        assert same_bits(out.cpu().numpy(), eq)
        assert ea[1] == 0 and np.all(eq[32:64] == 0)


def test_functional_4bit_roundtrip(dev):
    F = _F()
    torch.manual_seed(0)
    for qt in ("nf4", "fp4"):
        for dt in (torch.bfloat16, torch.float16, torch.float32):
            w = torch.randn(512, 320, device=dev, dtype=dt)
            q, st = F.quantize_4bit(w, blocksize=64, quant_type=qt)
            assert q.shape == ((512 * 320 + 1) // 2, 1) and q.dtype == torch.uint8
            wd = F.dequantize_4bit(q, st)
            assert wd.shape == w.shape and wd.dtype == dt
            # reference's own error bound style (functional round trip)
            err = (wd.float() - w.float()).abs().mean().item()
            assert err < (0.12 if qt == "nf4" else 0.15)
            # nested statistics (compress_statistics=True, the Linear4bit default)
            q2, st2 = F.quantize_4bit(w, blocksize=64, quant_type=qt, compress_statistics=True)
            assert torch.equal(q2, q) and st2.nested
            wd2 = F.dequantize_4bit(q2, st2)
            assert (wd2.float() - wd.float()).abs().max().item() < 0.05 * w.abs().max().item()


def test_functional_nested_matches_oracle(dev):
    """quantize_4bit(compress_statistics=True): nested absmax bit-exact vs oracle given torch's offset."""
    F = _F()
    torch.manual_seed(1)
    w = torch.randn(256, 512, device=dev, dtype=torch.bfloat16)
    q, st = F.quantize_4bit(w, blocksize=64, quant_type="nf4", compress_statistics=True)
    xf = ref.as_f32(to_numpy(w.reshape(-1), "bf16"), "bf16")
    absmax, eq = ref.quantize_blockwise(xf, 64, "nf4")
    assert same_bits(q.cpu().numpy().reshape(-1), eq)
    off = np.float32(st.offset.item())
    ea2, eq2 = ref.quantize_blockwise((absmax - off).astype(np.float32), 256, "8bit", code=st.state2.code.cpu().numpy())
    assert same_bits(st.absmax.cpu().numpy(), eq2)
    assert same_bits(st.state2.absmax.cpu().numpy(), ea2)
    full = F.dequantize_blockwise(st.absmax, st.state2) + st.offset
    exp = ref.nested_absmax(eq2, ea2, st.state2.code.cpu().numpy(), off)
    assert same_bits(full.cpu().numpy(), exp)
    # the one-launch decode (cdequantize_nested_absmax_fp32) used by gemm_4bit gives the same bits
    assert same_bits(F._absmax_fp32(st).cpu().numpy(), exp)


@pytest.mark.parametrize("n", [1, 255, 4096 * 11008 // 64 + 3, 70001])
def test_nested_absmax_one_launch_ragged(dev, n):
    """cdequantize_nested_absmax_fp32 on ragged lengths and unaligned tails vs the oracle."""
    F = _F()
    rng = np.random.default_rng(n)
    q = rng.integers(0, 256, n, dtype=np.uint8)
    a2 = rng.uniform(0.01, 1.0, (n + 255) // 256).astype(np.float32)
    code = F.create_dynamic_map(signed=True)
    off = np.float32(0.0123)
    out = torch.empty(n, device=dev)
    tc, tq, ta2, toff = code.to(dev), torch.from_numpy(q).to(dev), torch.from_numpy(a2).to(dev), torch.tensor([off], device=dev)
    F.lib.cdequantize_nested_absmax_fp32(F.get_ptr(tc), F.get_ptr(tq), F.get_ptr(ta2), F.get_ptr(toff), F.get_ptr(out),
                                         ct.c_int32(256), ct.c_longlong(n))
    torch.cuda.synchronize()
    assert same_bits(out.cpu().numpy(), ref.nested_absmax(q, a2, code.numpy(), off))


def test_cpu_semantics_on_device(golden, dev):
    """[additive] cquantize_blockwise_bytes_fp32 / cdequantize_blockwise_bytes_fp32: the CPU path's semantics
    (division, nearest code, code[0] = -1) on device pointers, bit-exact against the CPU-path fixtures; the
    caller's device code table is not rewritten.  (The host entry points themselves: tests/test_cpu_path.py.)"""
    F = _F()
    A = torch.from_numpy(golden["cpu_A"].copy()).to(dev)
    code = torch.from_numpy(create_dynamic_map().copy()).to(dev)
    absmax = torch.zeros((A.numel() + 63) // 64, device=dev)
    out = torch.zeros(A.numel(), dtype=torch.uint8, device=dev)
    F.lib.cquantize_blockwise_bytes_fp32(F.get_ptr(code), F.get_ptr(A), F.get_ptr(absmax), F.get_ptr(out),
                                         ct.c_longlong(64), ct.c_longlong(A.numel()))
    torch.cuda.synchronize()
    assert F.lib.cget_last_error() == 0
    assert code[0].item() != -1.0
    assert same_bits(absmax.cpu().numpy(), golden["cpu_absmax"])
    assert same_bits(out.cpu().numpy(), golden["cpu_q"])
    code_after = torch.from_numpy(golden["cpu_code_after"]).to(dev)
    y = torch.zeros(A.numel(), device=dev)
    F.lib.cdequantize_blockwise_bytes_fp32(F.get_ptr(code_after), F.get_ptr(out), F.get_ptr(absmax), F.get_ptr(y),
                                           ct.c_longlong(64), ct.c_longlong(A.numel()))
    torch.cuda.synchronize()
    assert same_bits(y.cpu().numpy(), golden["cpu_deq"])
    # the functional CPU route (host cores) gives the same codes as the device form
    q2, st = F.quantize_blockwise(torch.from_numpy(golden["cpu_A"].copy()), blocksize=64)
    assert same_bits(q2.numpy(), golden["cpu_q"])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("qt", ["nf4", "fp4"])
@pytest.mark.parametrize("shape,bs", [((1024, 4096), 64), ((300, 640), 128), ((7, 64 * 9), 64)])
def test_dequantize_4bit_nested_one_launch(dev, dtype, qt, shape, bs):
    """dequantize_4bit with compressed statistics runs one launch (cdequantize_blockwise_nested_*, absmax
    decoded in the kernel) and gives the bits of the two-step path (fp32 absmax, then the 4-bit dequantise)."""
    F = _F()
    torch.manual_seed(shape[0] + bs)
    w = torch.randn(*shape, device=dev, dtype=dtype)
    q, st = F.quantize_4bit(w, blocksize=bs, quant_type=qt, compress_statistics=True)
    one = F.dequantize_4bit(q, st)
    am = F._absmax_fp32(st)
    two = torch.empty_like(one)
    getattr(F.lib, f"cdequantize_blockwise_{F._QB[dtype]}_{qt}")(F.get_ptr(None), F.get_ptr(q), F.get_ptr(am),
                                                                  F.get_ptr(two), ct.c_int(bs), ct.c_int(two.numel()))
    torch.cuda.synchronize()
    assert torch.equal(one.view(torch.int16), two.view(torch.int16))
