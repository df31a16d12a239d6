"""CPU-only checks: the C-ABI library loads and exports every symbol include/bnb_hip.h declares,
host-side Python logic (tables, QuantState serialisation, layout buffer shapes), and the CPU
baseline port against the numpy oracle.  No GPU compute is called here."""
import ctypes as ct
import os
import re

import numpy as np
import pytest
import torch

from oracle import ref
from oracle.maps import create_dynamic_map

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "bnb_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", txt)) - {"extern"})


def test_library_exports_every_header_symbol():
    import python_src_quants as bnb
    assert bnb.HIP_AVAILABLE, "libbitsandbytes_hip.so did not load"
    lib = ct.CDLL(str(bnb.cextension.get_hip_bnb_library_path()))
    syms = _header_symbols()
    assert len(syms) >= 60
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_library_exports_nothing_outside_the_header():
    """the product library's dynamic symbol table is exactly the header's functions (linker version
    script generated from include/bnb_hip.h, csrc/Makefile) -- no lab hook (per-wave timelines, ablation modes that drop
    work) and no C++ internal is reachable through it; those live in the lab build (`make lab`)."""
    import shutil
    import subprocess
    import python_src_quants as bnb
    nm = shutil.which("nm")
    if nm is None:
        pytest.skip("no nm")
    path = str(bnb.cextension.get_hip_bnb_library_path())
    out = subprocess.run([nm, "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if len(ln.split()) == 3 and ln.split()[1] in "TtWw"}
    assert exported == set(_header_symbols()), (sorted(exported - set(_header_symbols())),
                                                sorted(set(_header_symbols()) - exported))
    for lab_only in ("chgemm_timeline", "chgemm_timeline_nostore", "cgemm_4bit_t64_timeline",
                     "cgemm_4bit_fewtok_timeline", "chgemm_set_variant"):
        assert lab_only not in exported


def test_reference_abi_names_present():
    """The hot-path names of ref:sycl/pythonInterface.cpp:192-422 are all exported."""
    import python_src_quants as bnb
    lib = bnb.lib._lib
    names = ["get_context", "get_cusparse", "cget_managed_ptr", "cprefetch", "cgemm_4bit_inference",
             "cdequant_mm_int32_fp16", "cget_col_row_stats", "cdouble_rowcol_quant",
             "cquantize_blockwise_cpu_fp32", "cdequantize_blockwise_cpu_fp32",
             "cextractOutliers_turing", "cextractOutliers_ampere"]
    for t in ("fp16", "bf16", "fp32"):
        for q in ("", "_fp4", "_nf4"):
            names += [f"cquantize_blockwise_{t}{q}", f"cdequantize_blockwise_{t}{q}"]
        names.append(f"cgemm_4bit_inference_naive_{t}")
    for f in ("turing", "ampere"):
        names += [f"cigemmlt_{f}_32", f"cigemmlt_{f}_8", f"cigemmlt_{f}_8_rowscale"]
    for f in ("col32", "turing", "ampere"):
        names += [f"ctransform_row2{f}", f"ctransform_row2{f}T"]
    assert all(hasattr(lib, n) for n in names), [n for n in names if not hasattr(lib, n)]


def test_python_tables_match_oracle():
    import python_src_quants.functional as F
    assert np.array_equal(F.get_4bit_type("nf4", device="cpu").numpy(), ref.nf4_table())
    assert np.array_equal(F.get_4bit_type("fp4", device="cpu").numpy(), ref.fp4_table())
    assert np.array_equal(F.create_dynamic_map().numpy(), create_dynamic_map())
    lm = F.create_linear_map(signed=True)
    assert lm.numel() == 256
    nm = F.create_normal_map()
    assert nm.numel() == 256 and float(nm.max()) == 1.0


def test_quant_state_roundtrip_packed():
    import python_src_quants.functional as F
    absmax = torch.arange(8, dtype=torch.uint8)
    state2 = F.QuantState(absmax=torch.rand(1), blocksize=256, code=torch.rand(256), dtype=torch.float32)
    qs = F.QuantState(absmax=absmax, shape=torch.Size([16, 32]), code=torch.rand(16), blocksize=64,
                      quant_type="nf4", dtype=torch.bfloat16, offset=torch.tensor(0.25), state2=state2)
    d = qs.as_dict(packed=True)
    assert "quant_state.bitsandbytes__nf4" in d and d["quant_state.bitsandbytes__nf4"].dtype == torch.uint8
    back = F.QuantState.from_dict({"weight." + k: v for k, v in d.items()}, device="cpu")
    assert back == qs
    with pytest.raises(ValueError):
        F.QuantState.from_dict({"absmax": absmax}, device="cpu")


def test_transform_buffer_shapes():
    import python_src_quants.functional as F
    assert F.get_transform_buffer((33, 70), torch.int8, "cpu", "col32")[0].shape == (33, 96)
    assert F.get_transform_buffer((33, 70), torch.int8, "cpu", "col_turing")[0].shape == (40, 96)
    assert F.get_transform_buffer((33, 70), torch.int8, "cpu", "col_ampere")[0].shape == (64, 96)
    buf, st = F.get_transform_buffer((33, 70), torch.int8, "cpu", "col_turing", transpose=True)
    assert buf.shape == (72, 64) and st == ((70, 33), "col_turing")
    for fmt in ("col32", "col_turing", "col_ampere"):
        assert F.get_transform_buffer((33, 70), torch.int8, "cpu", fmt)[0].shape == ref.layout_shape(33, 70, fmt)


def test_gpu_ops_refuse_cpu_tensors():
    """No silent CPU fallback: 4-bit ops on CPU tensors raise like the reference (functional.py:1158)."""
    import python_src_quants.functional as F
    with pytest.raises(NotImplementedError):
        F.quantize_4bit(torch.randn(64, 64), quant_type="nf4")


def _port():
    path = os.path.join(ROOT, "oracle", "_build", "libcpu_ops_port.so")
    if not os.path.exists(path):
        pytest.skip("CPU port not built (run __graft_entry__.build())")
    return ct.CDLL(path)


def test_cpu_port_matches_oracle(golden):
    lib = _port()
    A = golden["cpu_A"].copy()
    code = create_dynamic_map().copy()
    absmax = np.zeros((A.size + 63) // 64, np.float32)
    out = np.zeros(A.size, np.uint8)
    lib.port_quantize_cpu(code.ctypes.data_as(ct.c_void_p), A.ctypes.data_as(ct.c_void_p),
                          absmax.ctypes.data_as(ct.c_void_p), out.ctypes.data_as(ct.c_void_p),
                          ct.c_longlong(64), ct.c_longlong(A.size))
    assert code[0] == -1.0
    assert np.array_equal(absmax, golden["cpu_absmax"]) and np.array_equal(out, golden["cpu_q"])
    y = np.zeros(A.size, np.float32)
    lib.port_dequantize_cpu(code.ctypes.data_as(ct.c_void_p), out.ctypes.data_as(ct.c_void_p),
                            absmax.ctypes.data_as(ct.c_void_p), y.ctypes.data_as(ct.c_void_p),
                            ct.c_longlong(64), ct.c_longlong(A.size))
    assert np.array_equal(y, golden["cpu_deq"])


def test_golden_fixtures_reproduce(golden):
    """The committed fixtures are exactly what the oracle produces (regression pin of the oracle)."""
    code = golden["dynamic_code"]
    assert np.array_equal(code, create_dynamic_map())
    for i in range(int(golden["n_quant_cases"])):
        di, qi, bs, n = golden[f"q{i}_meta"].tolist()
        dtype, qtype = ["fp32", "fp16", "bf16"][di], ["nf4", "fp4", "8bit"][qi]
        absmax, q = ref.quantize_blockwise(ref.as_f32(golden[f"q{i}_in"], dtype), bs, qtype, code=code)
        assert np.array_equal(absmax, golden[f"q{i}_absmax"]) and np.array_equal(q, golden[f"q{i}_q"])
    rs, cs, _ = ref.colrow_absmax(golden["dq_A"])
    assert np.array_equal(ref.double_quant(golden["dq_A"], rs, cs)[0], golden["dq_row"])
    assert np.array_equal(ref.igemmlt(golden["ig_A"], golden["ig_B"]), golden["ig_C"])


def test_route_rows_bucket():
    """The measured-route cache groups row counts in quarter-octave buckets (host logic, no GPU)."""
    import python_src_quants.functional as F
    assert [F._route_rows_bucket(r) for r in (2048, 2559, 2560, 4096, 4500, 5119, 5120, 65536, 70000)] == \
        [2048, 2048, 2560, 4096, 4096, 4096, 5120, 65536, 65536]
    for r in range(1, 5000, 7):
        b = F._route_rows_bucket(r)
        assert b <= r and r - b < max(1, r // 4 + 1)


def test_roctx_ranges_switch():
    """roctx ranges around the C-ABI entry points (SURVEY §5 tracing plan) are off by default and on with
    BNB_ROCTX=1 (libroctx64 opened at run time); checked in fresh processes, no GPU needed."""
    import subprocess
    import sys
    code = ("import sys; sys.path[:0] = [%r]; import python_src_quants.functional as F; "
            "print(F.lib.croctx_enabled())" % os.path.join(ROOT, "bitsandbytes-sycl_amd"))
    env = dict(os.environ)
    env.pop("BNB_ROCTX", None)
    off = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    env["BNB_ROCTX"] = "1"
    on = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert off.stdout.strip().splitlines()[-1] == "0", off.stderr[-500:]
    assert on.stdout.strip().splitlines()[-1] == "1", on.stderr[-500:]
