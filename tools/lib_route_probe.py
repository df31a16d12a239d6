"""Probe (GPU): the M > 1 4-bit GEMM routes at prefill sizes, per shape (rows x out_features x in_features, bf16,
NF4 bs 64, nested statistics), interleaved over rounds:
  fused    : k_gemm_4bit_256 (the hand-written fused kernel, forced)
  lt       : our dequantise + torch.matmul on hipBLASLt (torch's default BLAS on ROCm)
  rocblas  : our dequantise + torch.matmul on rocBLAS (torch.backends.cuda.preferred_blas_library("cublas"))
  searched : our dequantise + cgemm_tn (rocBLAS with the per-shape solution search of gemm_lib.hip)
Usage: python tools/lib_route_probe.py [MxNxK ...]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402

SHAPES = [(4096, 11008, 4096), (2048, 11008, 4096), (8192, 11008, 4096), (4096, 4096, 11008), (4096, 4096, 4096),
          (16384, 11008, 4096)]
if len(sys.argv) > 1:
    SHAPES = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]]


def t_us(fn, it=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for (m, n, k) in SHAPES:
        X = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        W = (torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16)
        q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
        del W
        Y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)

        def fused():
            F.gemm_4bit(X, q, st, out=Y, _route="fused")

        def lib(name):
            def go():
                torch.backends.cuda.preferred_blas_library(name)
                try:
                    F.gemm_4bit(X, q, st, out=Y, _route="library")
                finally:
                    torch.backends.cuda.preferred_blas_library("cublaslt")
            return go
        def tn():
            F.gemm_4bit(X, q, st, out=Y, _route="library_tn")
        arms = {"fused": fused, "lt": lib("cublaslt"), "rocblas": lib("cublas"), "searched": tn}
        t_end = time.perf_counter() + 1.0
        while time.perf_counter() < t_end:
            fused()
            torch.cuda.synchronize()
        res = {a: [] for a in arms}
        for _ in range(5):
            for a, fn in arms.items():
                res[a].append(t_us(fn))
        f = 2.0 * m * n * k
        line = f"{m}x{n}x{k}:"
        for a, v in res.items():
            med = sorted(v)[2]
            line += f"  {a} {med:7.1f} us ({f / med / 1e6:5.0f} TF)"
        print(line, flush=True)
        del X, q, st, Y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
