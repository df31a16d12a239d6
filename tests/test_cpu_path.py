"""The product's CPU path (config 1 of BASELINE.json): cquantize_blockwise_cpu_fp32 /
cdequantize_blockwise_cpu_fp32 run on the host cores (csrc/cpu_ops.cpp) with no GPU present.

Bit-exact against the golden fixtures, the numpy oracle (ref.quantize_cpu / ref.dequantize_cpu,
following ref:sycl/cpu_ops.cpp:7-63 and ref:sycl/common.cpp:4-35) and the C++ baseline port
(oracle/cpu_ops_port.cpp, the reference's thread-per-block structure), for several thread counts.
These tests never initialise HIP: they run here, in the GPU-less container."""
import ctypes as ct
import os

import numpy as np
import pytest
import torch

from oracle import ref
from oracle.maps import create_dynamic_map

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lib():
    import python_src_quants as bnb
    if not bnb.HIP_AVAILABLE:
        pytest.skip("library not built")
    return bnb.lib


def _port():
    path = os.path.join(ROOT, "oracle", "_build", "libcpu_ops_port.so")
    if not os.path.exists(path):
        pytest.skip("CPU port not built (run __graft_entry__.build())")
    return ct.CDLL(path)


def _p(a: np.ndarray):
    return a.ctypes.data_as(ct.c_void_p)


def _quant(lib, code, A, bs):
    absmax = np.zeros((A.size + bs - 1) // bs, np.float32)
    out = np.zeros(A.size, np.uint8)
    lib.cquantize_blockwise_cpu_fp32(_p(code), _p(A), _p(absmax), _p(out), ct.c_longlong(bs), ct.c_longlong(A.size))
    return absmax, out


def _dequant(lib, code, q, absmax, bs):
    y = np.zeros(q.size, np.float32)
    lib.cdequantize_blockwise_cpu_fp32(_p(code), _p(q), _p(absmax), _p(y), ct.c_longlong(bs), ct.c_longlong(q.size))
    return y


def test_cpu_path_golden(golden):
    lib = _lib()
    code = create_dynamic_map().copy()
    absmax, q = _quant(lib, code, golden["cpu_A"].copy(), 64)
    assert code[0] == -1.0                              # in-place side effect (cpu_ops.cpp:20)
    assert np.array_equal(code, golden["cpu_code_after"])
    assert np.array_equal(absmax, golden["cpu_absmax"]) and np.array_equal(q, golden["cpu_q"])
    assert np.array_equal(_dequant(lib, code, q, absmax, 64), golden["cpu_deq"])


@pytest.mark.parametrize("threads", [1, 3, 8])
@pytest.mark.parametrize("bs,n", [(64, 1), (64, 64 * 1000 + 17), (256, 300_001), (4096, 1 << 20), (100, 12_345)])
def test_cpu_path_vs_oracle_and_port(threads, bs, n):
    """Random inputs with edge values (zeros blocks, NaN, +-inf-free huge/tiny, exact code values)."""
    lib, port = _lib(), _port()
    lib.cset_cpu_threads(threads)
    try:
        rng = np.random.default_rng(n + bs)
        A = (rng.standard_normal(n) * 3).astype(np.float32)
        if n > 4 * bs:
            A[bs:2 * bs] = 0.0                          # all-zero block -> absmax 0 -> NaN -> index 0
            A[2 * bs] = np.nan
            A[3 * bs:3 * bs + 8] = [1e-30, -1e-30, 1e30, -1e30, 0.5, -0.5, 1.0, -1.0]
        code0 = create_dynamic_map().copy()
        code_a, code_b = code0.copy(), code0.copy()
        am, q = _quant(lib, code_a, A, bs)
        e_am, e_q, e_code = ref.quantize_cpu(code0.copy(), A, bs)
        assert np.array_equal(code_a, e_code)
        assert np.array_equal(am, e_am, equal_nan=True) and np.array_equal(q, e_q)
        p_am = np.zeros_like(am)
        p_q = np.zeros_like(q)
        port.port_quantize_cpu(_p(code_b), _p(A), _p(p_am), _p(p_q), ct.c_longlong(bs), ct.c_longlong(n))
        assert np.array_equal(am, p_am, equal_nan=True) and np.array_equal(q, p_q)
        y = _dequant(lib, code_a, q, am, bs)
        assert np.array_equal(y, ref.dequantize_cpu(code_a, q, am, bs), equal_nan=True)
    finally:
        lib.cset_cpu_threads(0)


def test_config1_nf4_bytes_dequant_matches_port():
    """Config 1 (BASELINE.json): NF4 4096 x 4096, bs = 64, through the CPU entry point -- the 16-entry NF4 table
    padded to 256 and one index byte per element -- bit-identical to the single-threaded port."""
    lib, port = _lib(), _port()
    n, bs = 4096 * 4096, 64
    rng = np.random.default_rng(0)
    q = rng.integers(0, 16, size=n, dtype=np.uint8)
    absmax = rng.uniform(0.01, 3.0, n // bs).astype(np.float32)
    code = np.zeros(256, np.float32)
    code[:16] = ref.nf4_table()
    y = _dequant(lib, code, q, absmax, bs)
    y_port = np.empty_like(y)
    port.port_dequantize_cpu(_p(code), _p(q), _p(absmax), _p(y_port), ct.c_longlong(bs), ct.c_longlong(n))
    assert np.array_equal(y, y_port)
    assert np.array_equal(y[:4096], ref.nf4_table()[q[:4096]] * np.repeat(absmax[:64], 64))


def test_functional_cpu_route():
    """functional.quantize_blockwise / dequantize_blockwise on CPU tensors take the host entry points (no GPU):
    plain and nested statistics, and a non-fp32 input converted first."""
    import python_src_quants.functional as F
    _lib()
    rng = np.random.default_rng(3)
    a = rng.standard_normal(64 * 513).astype(np.float32)
    q, st = F.quantize_blockwise(torch.from_numpy(a.copy()), blocksize=64)
    e_am, e_q, e_code = ref.quantize_cpu(create_dynamic_map().copy(), a, 64)
    assert np.array_equal(q.numpy(), e_q) and np.array_equal(st.absmax.numpy(), e_am)
    y = F.dequantize_blockwise(q, st)
    assert y.dtype == torch.float32
    assert np.array_equal(y.numpy(), ref.dequantize_cpu(e_code, e_q, e_am, 64))
    # nested statistics: the decoded fp32 absmax drives the dequantize (not the uint8 codes)
    qn, stn = F.quantize_blockwise(torch.from_numpy(a.copy()), blocksize=64, nested=True)
    assert np.array_equal(qn.numpy(), e_q)
    yn = F.dequantize_blockwise(qn, stn)
    am2 = F.dequantize_blockwise(stn.absmax, stn.state2) + stn.offset
    assert np.array_equal(yn.numpy(), ref.dequantize_cpu(e_code, e_q, am2.numpy(), 64))
    assert (yn - y).abs().max().item() < 0.05 * float(np.abs(a).max())
    # fp16 input on CPU: converted to fp32 before the host call
    qh, sth = F.quantize_blockwise(torch.from_numpy(a.copy()).half(), blocksize=64)
    e_am_h, e_q_h, _ = ref.quantize_cpu(create_dynamic_map().copy(), a.astype(np.float16).astype(np.float32), 64)
    assert np.array_equal(qh.numpy(), e_q_h)
