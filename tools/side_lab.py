"""A/B of the side dequantise inside k_hgemm (chgemm_tn_pf_bf16) at the metric shape: the plain GEMM, the dequantise
kernel alone, their sum, and the prefetching GEMM under each chgemm_set_side_mode setting (1 = non-temporal side loads
/ stores, 2 = no side stores, lab ablation, the weight is not written).  Interleaved rounds after a clock ramp."""
import ctypes as ct
import os
import sys
os.environ.setdefault("BNB_HIP_LIBRARY", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                   "bitsandbytes-sycl_amd", "build", "libbitsandbytes_hip_lab.so"))   # lab hooks: `make -C bitsandbytes-sycl_amd/csrc lab`
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import python_src_quants.functional as F  # noqa: E402
from python_src_quants.cextension import lib  # noqa: E402

M, N, K = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (4096, 4096, 11008)))
modes = [int(a) for a in os.environ.get("SIDE_MODES", "1,3,9,17,33,97").split(",")]
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
Wd = F.dequantize_4bit(q, st).view(N, K).contiguous()
out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
target = torch.empty(N * K, device=dev, dtype=torch.bfloat16)
wsb = int(lib.chgemm_tn_workspace_bytes(ct.c_int32(M), ct.c_int32(N), ct.c_int32(K)))
ws = F._gemm_workspace(dev, wsb)


def plain():
    lib.chgemm_tn_ws_bf16(ct.c_int32(M), ct.c_int32(N), ct.c_int32(K), F.get_ptr(X), ct.c_int32(K), F.get_ptr(Wd),
                          ct.c_int32(K), F.get_ptr(out), ct.c_int32(N), F.get_ptr(ws), ct.c_longlong(wsb))


def deq():
    F._dequant_4bit_nested(q, st, target)


def pf(mode):
    def run():
        lib.chgemm_set_side_mode(ct.c_int(mode))
        F._launch_prefetch_gemm(X, Wd, out, ws, wsb, (q, st), target)
    return run


cands = {"gemm": plain, "dequant": deq}
for m in modes:
    cands[f"pf mode {m}"] = pf(m)
t_end = time.perf_counter() + 0.5
while time.perf_counter() < t_end:
    plain()
    torch.cuda.synchronize()
best = {k: 1e9 for k in cands}
R = 20
for rnd in range(5):
    for name, fn in cands.items():
        fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(R):
            fn()
        e.record()
        e.synchronize()
        best[name] = min(best[name], s.elapsed_time(e) / R * 1e3)
lib.chgemm_set_side_mode(ct.c_int(1))
print(f"shape {M}x{N}x{K}")
for k, v in best.items():
    print(f"{k:14s} {v:8.1f} us")
print(f"{'gemm+dequant':14s} {best['gemm'] + best['dequant']:8.1f} us")
