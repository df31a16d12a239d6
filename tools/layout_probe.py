"""Probe (GPU): does the library bf16 GEMM of the metric step run faster on another weight layout?
X [M, K] @ W^T with W stored [N, K] (the dequantise's natural output, hipBLASLt 'TN') against W^T stored [K, N]
('NN'); metric shape and the Llama-2-7B prefill shapes; torch's default heuristic; interleaved rounds, medians.
Usage: python tools/layout_probe.py"""
import time

import torch

SHAPES = [(4096, 4096, 11008), (4096, 11008, 4096), (2048, 4096, 11008), (65536, 4096, 4096), (65536, 4096, 11008)]


def t_us(fn, it=10):
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
    torch.manual_seed(0)
    for (m, n, k) in SHAPES:
        X = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        W = torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02
        WT = W.t().contiguous()
        Y = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        arms = {"TN (W [N,K])": lambda: torch.matmul(X, W.t(), out=Y),
                "NN (W^T [K,N])": lambda: torch.matmul(X, WT, out=Y)}
        t_end = time.perf_counter() + 1.0
        while time.perf_counter() < t_end:
            for fn in arms.values():
                fn()
            torch.cuda.synchronize()
        res = {a: [] for a in arms}
        for _ in range(5):
            for a, fn in arms.items():
                res[a].append(t_us(fn))
        f = 2.0 * m * n * k
        line = f"{m}x{n}x{k}:"
        for a, v in res.items():
            med = sorted(v)[2]
            line += f"  {a} {med:8.1f} us ({f / med / 1e6:5.0f} TF)"
        print(line, flush=True)
        del X, W, WT, Y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
