"""A/B (GPU): the few-token split-K kernel's combine -- in-launch (last arriving workgroup of a row block sums the
slabs; cgemm_4bit_set_skinny_reduce(1)) vs the separate k_skinny_reduce launch (0) -- nested NF4 bs 64, bf16,
14 rotating weight copies, HIP-graph replay, medians of 5 interleaved rounds; outputs compared bit for bit.
Usage: [SKINNY_SHAPES=NxK,...] python tools/skinny_reduce_ab.py [tokens ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402
from fewtoken_ab import graph_time  # noqa: E402

TOKENS = [int(a) for a in sys.argv[1:]] or [5, 8, 16, 32, 48, 64]
SHAPES = [tuple(int(v) for v in a.split("x")) for a in
          os.environ.get("SKINNY_SHAPES", "11008x4096,4096x11008,4096x4096,1024x8192,3584x8192").split(",")]


def main():
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(5)
    F.GEMM_4BIT_GEMV_TOKENS = 1
    F.lib.cgemm_4bit_set_fewtoken_kernel(1)     # the split-K kernel at every token count
    for (n_out, k_in) in SHAPES:
        ws = []
        for _ in range(14):
            W = (torch.randn(n_out, k_in, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
            ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
            del W
        for m in TOKENS:
            x = torch.randn(m, k_in, device=dev, dtype=torch.bfloat16, generator=gen)
            out = torch.empty(m, n_out, device=dev, dtype=torch.bfloat16)
            calls = [(lambda q=q, st=st: F.gemm_4bit(x, q, st, out=out)) for q, st in ws]
            res, ys = {1: [], 0: []}, {}
            for _ in range(5):
                for mode in (1, 0):
                    F.lib.cgemm_4bit_set_skinny_reduce(mode)
                    res[mode].append(graph_time(calls))
                    ys[mode] = F.gemm_4bit(x, ws[0][0], ws[0][1]).clone()
            F.lib.cgemm_4bit_set_skinny_reduce(1)
            same = torch.equal(ys[0], ys[1])
            print(f"{n_out}x{k_in} tokens {m:3d}: in-launch combine {sorted(res[1])[2]:6.2f} us   reduce launch "
                  f"{sorted(res[0])[2]:6.2f} us   identical {same}", flush=True)
        del ws
        torch.cuda.empty_cache()
    F.lib.cgemm_4bit_set_fewtoken_kernel(0)


if __name__ == "__main__":
    main()
