"""Few-token NF4 GEMM (batched decode / short prefill, M = 2..256 tokens): GPU time per call, replayed
from a HIP graph so the host cost is out of the measurement.  Routes: as routed (fused kernel),
forced library (dequantise + hipBLASLt), and the M = 1 GEMV x M for reference.  K, N from argv."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402

dev = torch.device("cuda", 0)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 11008
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
am = F._absmax_fp32(st)


def graph_time(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    return sorted(ts)[3]


print(f"N={N} K={K} (weights {N * K / 2 / 1e6:.1f} MB packed): tokens | fused (as routed) | library | GEMV x tokens  [us]")
x1 = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
y1 = torch.empty(1, N, device=dev, dtype=torch.bfloat16)
t_gemv = graph_time(lambda: F.gemv_4bit(x1, q.t(), state=st, out=y1))
for M in (2, 4, 8, 16, 32, 64, 128, 256):
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    t_f = graph_time(lambda: F.gemm_4bit(X, q, st, out=Y, absmax=am))
    r0, f0 = F.GEMM_4BIT_DEQUANT_MIN_ROWS, F.GEMM_4BIT_DEQUANT_MIN_FEATURES
    F.GEMM_4BIT_DEQUANT_MIN_ROWS, F.GEMM_4BIT_DEQUANT_MIN_FEATURES = 1, 1
    try:
        t_l = graph_time(lambda: F.gemm_4bit(X, q, st, out=Y))
    finally:
        F.GEMM_4BIT_DEQUANT_MIN_ROWS, F.GEMM_4BIT_DEQUANT_MIN_FEATURES = r0, f0
    print(f"{M:4d} | {t_f:8.1f} | {t_l:8.1f} | {t_gemv * M:8.1f}", flush=True)
