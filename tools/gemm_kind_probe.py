"""Probe (GPU, for rocprofv3 PMC passes): 20 launches at 4096 x 4096 x 11008 of one GEMM kind --
i8_8w (k_igemm_256, the igemmlt+dequant default), i8_4w (k_hgemm HG_I8_DEQ, cigemm_set_tile(4)), bf16 (k_hgemm bf16).
Usage: python tools/gemm_kind_probe.py KIND"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import ctypes as ct  # noqa: E402

import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402

kind = sys.argv[1]
m, n, k = 4096, 4096, 11008
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
if kind.startswith("i8"):
    A = torch.randint(-127, 128, (m, k), device=dev, dtype=torch.int8, generator=g)
    B = torch.randint(-127, 128, (n, k), device=dev, dtype=torch.int8, generator=g)
    rs = torch.rand(m, device=dev, generator=g) * 2 + 0.5
    cs = torch.rand(n, device=dev, generator=g) * 2 + 0.5
    out = torch.empty(m, n, device=dev, dtype=torch.float16)
    F.lib.cigemm_set_tile(4 if kind == "i8_4w" else 0)
    call = lambda: F.igemmlt_dequant(A, B, rs, cs, out=out)  # noqa: E731
else:
    A = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
    B = torch.randn(n, k, device=dev, generator=g).to(torch.bfloat16)
    C = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    F.pre_call(dev)
    call = lambda: F.lib.chgemm_tn_bf16(m, n, k, F.get_ptr(A), k, F.get_ptr(B), k, F.get_ptr(C), n)  # noqa: E731
for _ in range(20):
    call()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20):
    call()
e.record()
e.synchronize()
print(kind, f"{s.elapsed_time(e) / 20 * 1e3:.1f} us")
F.lib.cigemm_set_tile(0)
