"""A/B (GPU): the two few-token 4-bit GEMM kernels behind gemm_4bit at 5..32 activation rows -- the whole-K kernel
(gemm4bit_wk.hip, forced: cgemm_4bit_set_fewtoken_kernel(2)) and the split-K skinny kernel + its reduce launch
(1) -- on the Llama-2-7B weights (nested NF4 bs 64), 14 rotating weight copies per shape (> the 256 MB
MALL for the big ones), HIP-graph replay, interleaved rounds; medians.
Usage: python tools/fewtoken_ab.py [tokens ...]
       FEWTOKEN_ROUTE=1 python tools/fewtoken_ab.py 33 48 64   (instead: the split-K kernel's 33..64-row instance
       against the route gemm_4bit took there before it, GEMM_4BIT_FEW_TOKENS = 32)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402

TOKENS = [int(a) for a in sys.argv[1:]] or [5, 8, 16, 24, 32]
SHAPES = [(11008, 4096), (4096, 11008), (4096, 4096)]


def graph_time(calls, iters=20):
    for c in calls:
        c()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for c in calls:
            c()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters / len(calls)


def main():
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(3)
    F.GEMM_4BIT_GEMV_TOKENS = 1          # keep 2..4 rows off the multi-row GEMV (not measured here)
    for (n_out, k_in) in SHAPES:
        ws = []
        for _ in range(14):
            W = (torch.randn(n_out, k_in, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
            ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
            del W
        nbytes_w = n_out * k_in // 2 + n_out * k_in // 64 + n_out * k_in // 64 // 256 * 4
        for m in TOKENS:
            x = torch.randn(m, k_in, device=dev, dtype=torch.bfloat16, generator=gen)
            out = torch.empty(m, n_out, device=dev, dtype=torch.bfloat16)
            calls = [(lambda q=q, st=st: F.gemm_4bit(x, q, st, out=out)) for q, st in ws]
            route = os.environ.get("FEWTOKEN_ROUTE") == "1"
            arms = ((1, "split-K 64-row"), (0, "previous route")) if route else ((2, "whole-K"), (1, "split-K"))
            res = {a: [] for a, _ in arms}
            for _ in range(5):
                for kern, _ in arms:
                    if route:
                        F.GEMM_4BIT_FEW_TOKENS = 64 if kern == 1 else 32
                    else:
                        F.lib.cgemm_4bit_set_fewtoken_kernel(kern)
                    res[kern].append(graph_time(calls))
            F.lib.cgemm_4bit_set_fewtoken_kernel(0)
            nbytes = nbytes_w + m * k_in * 2 + m * n_out * 2
            line = f"{n_out}x{k_in} tokens {m:3d}:"
            for kern, name in arms:
                med = sorted(res[kern])[2]
                line += f"  {name} {med:6.2f} us ({nbytes / med / 1e3:6.0f} GB/s)"
            print(line, flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
