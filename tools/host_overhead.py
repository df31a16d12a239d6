"""Host-side cost per call of the Python entry points (wall time of a loop of calls, GPU work tiny)
and a cProfile of the decode GEMV call.  Usage: python tools/host_overhead.py"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402

dev = torch.device("cuda", 0)
K, N = 4096, 11008
W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
qp, stp = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=False)
x = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
X = torch.randn(64, K, device=dev, dtype=torch.bfloat16)
out1 = torch.empty(1, N, device=dev, dtype=torch.bfloat16)
calls = {
    "gemv_4bit nested": lambda: F.gemv_4bit(x, q.t(), state=st),
    "gemv_4bit nested out=": lambda: F.gemv_4bit(x, q.t(), state=st, out=out1),
    "gemv_4bit plain": lambda: F.gemv_4bit(x, qp.t(), state=stp),
    "gemm_4bit 64 rows": lambda: F.gemm_4bit(X, q, st),
    "dequantize_4bit nested": lambda: F.dequantize_4bit(q, st),
    "torch.empty (reference point)": lambda: torch.empty(1, N, device=dev, dtype=torch.bfloat16),
}
for name, fn in calls.items():
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    reps = 2000
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name:32s} host {1e6 * (t1 - t0) / reps:7.1f} us/call   incl. drain {1e6 * (t2 - t0) / reps:7.1f}", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(2000):
    F.gemv_4bit(x, q.t(), state=st)
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
