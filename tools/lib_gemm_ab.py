"""A/B (GPU): the library bf16 GEMM of the metric step two ways on the same dequantised weight, interleaved rounds,
medians: torch.matmul (torch's hipBLASLt heuristic) and cgemm_tn_bf16 (gemm_lib.hip: rocBLAS with the per-shape
solution search).  Usage: python tools/lib_gemm_ab.py [MxNxK ...]"""
import ctypes as ct
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402

SHAPES = [(4096, 4096, 11008), (65536, 4096, 11008), (4096, 11008, 4096), (2048, 4096, 11008)]
if len(sys.argv) > 1:
    SHAPES = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]]


def t_us(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / it


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for (m, n, k) in SHAPES:
        X = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        W = (torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16)
        Y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)

        def lib():
            F.pre_call(dev)
            F.lib.cgemm_tn_bf16(ct.c_int32(m), ct.c_int32(n), ct.c_int32(k), F.get_ptr(X), ct.c_int32(k), F.get_ptr(W),
                                ct.c_int32(k), F.get_ptr(Y), ct.c_int32(n))
        arms = {"torch.matmul": lambda: torch.matmul(X, W.t(), out=Y), "cgemm_tn": lib}
        lib()
        t_end = time.perf_counter() + 1.0
        while time.perf_counter() < t_end:
            for fn in arms.values():
                fn()
            torch.cuda.synchronize()
        res = {a: [] for a in arms}
        for _ in range(7):
            for a, fn in arms.items():
                res[a].append(t_us(fn, 20 if m * n * k < 1e12 else 5))
        f = 2.0 * m * n * k
        line = f"{m}x{n}x{k}:"
        for a, v in res.items():
            med = sorted(v)[3]
            line += f"  {a} {med:8.1f} us ({f / med / 1e6:5.0f} TF)"
        print(line + f"  plan {F.lib.cgemm_tn_plan(m, n, k, 0, k, k, n)}", flush=True)
        del X, W, Y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
