"""NF4 M>1 routing sweep at K = 11008 (nested statistics, bf16): the fused kernel (split-K as routed)
against the dequantise + hipBLASLt pair, with the dequantisation (first chunk) and without it (a later
chunk of the same weight, reuse_weight=True).  Decides GEMM_4BIT_DEQUANT_MIN_ROWS / _FEATURES and the
chunked-forward rule.  Usage: python tools/route_sweep.py [K]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402

dev = torch.device("cuda", 0)
K = int(sys.argv[1]) if len(sys.argv) > 1 else 11008
Xall = torch.randn(4096, K, device=dev, dtype=torch.bfloat16)
BIG = 1 << 30


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / reps)
    return sorted(ts)[len(ts) // 2]


print(f"K={K}  rows x features: fused | library (dequant+GEMM) | library GEMM only (reuse)   [us]", flush=True)
for M, n in ((512, 4096), (1024, 4096), (2048, 4096), (1024, 2048), (2048, 2048), (4096, 2048), (1024, 1024),
             (2048, 1024), (4096, 1024), (1024, 512), (2048, 512), (4096, 512)):
    X = Xall[:M]
    W = (torch.randn(n, K, device=dev) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    Y = torch.empty(M, n, device=dev, dtype=torch.bfloat16)
    r0, f0 = F.GEMM_4BIT_DEQUANT_MIN_ROWS, F.GEMM_4BIT_DEQUANT_MIN_FEATURES
    try:
        F.GEMM_4BIT_DEQUANT_MIN_ROWS, F.GEMM_4BIT_DEQUANT_MIN_FEATURES = BIG, BIG
        am = F._absmax_fp32(st)
        t_fused = timed(lambda: F.gemm_4bit(X, q, st, out=Y, absmax=am))
        F.GEMM_4BIT_DEQUANT_MIN_ROWS, F.GEMM_4BIT_DEQUANT_MIN_FEATURES = 1, 1
        t_lib = timed(lambda: F.gemm_4bit(X, q, st, out=Y))
        F.gemm_4bit(X, q, st, out=Y)
        t_reuse = timed(lambda: F.gemm_4bit(X, q, st, out=Y, reuse_weight=True))
    finally:
        F.GEMM_4BIT_DEQUANT_MIN_ROWS, F.GEMM_4BIT_DEQUANT_MIN_FEATURES = r0, f0
    print(f"{M:5d} x {n:5d}: {t_fused:8.1f} | {t_lib:8.1f} | {t_reuse:8.1f}", flush=True)
