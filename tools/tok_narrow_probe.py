"""Probe (GPU): 2..8 activation rows on narrow / long-K weights (the Llama-2-70B 8-way shards) through gemm_4bit's
default route (multi-row GEMV at 2..4 rows, else the whole-K kernel at <= 6 rows on narrow weights, else
split-K), with the multi-row GEMV off ("no-tok") and with only the split-K kernel ("split-K"); nested NF4 bs 64, bf16, distinct weight copies, HIP-graph replay.
Usage: python tools/tok_narrow_probe.py [NxK ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402
from gemv_shape_probe import graph_us  # noqa: E402

SHAPES = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]] or [(128, 8192), (1024, 8192), (1024, 28672),
                                                                         (3584, 8192)]


def main():
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(2)
    for n, k in SHAPES:
        copies = max(2, min(64, int(400e6 // (n * k // 2))))
        ws = []
        for _ in range(copies):
            W = (torch.randn(n, k, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
            ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
            del W
        line = f"{n}x{k}:"
        for m in (2, 4, 8):
            x = torch.randn(m, k, device=dev, dtype=torch.bfloat16, generator=gen)
            out = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
            calls = [(lambda q=q, st=st: F.gemm_4bit(x, q, st, out=out)) for q, st in ws]
            t = {}
            saved = F.GEMM_4BIT_GEMV_TOKENS
            for arm, (gt, fk) in {"default": (saved, 0), "no-tok": (1, 0), "split-K": (1, 1)}.items():
                F.GEMM_4BIT_GEMV_TOKENS = gt
                F.lib.cgemm_4bit_set_fewtoken_kernel(fk)
                t[arm] = graph_us(calls)
            F.GEMM_4BIT_GEMV_TOKENS = saved
            F.lib.cgemm_4bit_set_fewtoken_kernel(0)
            line += f"  | {m} rows: " + " ".join(f"{a} {v:6.2f}" for a, v in t.items())
        print(line, flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
