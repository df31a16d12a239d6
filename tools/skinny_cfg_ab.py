"""A/B (GPU): geometry of the few-token split-K kernel (cgemm_4bit_set_skinny_config: 0 = 4 waves per workgroup,
1 = 8 waves, 2 = 8 waves with twice the blocks per split, -1 = the launcher's rule), nested NF4 bs 64 on the
Llama-2-7B weights (SKINNY_SHAPES=NxK,... for others), 14 rotating copies, HIP-graph replay, medians of 5 interleaved
rounds; max |difference| to configuration 0 relative to its rms.
Usage: [SKINNY_CFGS=0,1,2,-1] python tools/skinny_cfg_ab.py [tokens ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402
from fewtoken_ab import graph_time  # noqa: E402

TOKENS = [int(a) for a in sys.argv[1:]] or [8, 16, 32, 48, 64]
SHAPES = [tuple(int(v) for v in a.split("x")) for a in os.environ.get("SKINNY_SHAPES", "11008x4096,4096x11008,4096x4096").split(",")]
CFGS = [int(v) for v in os.environ.get("SKINNY_CFGS", "0,1,2").split(",")]


def main():
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(5)
    F.GEMM_4BIT_GEMV_TOKENS = 1
    F.lib.cgemm_4bit_set_fewtoken_kernel(1)     # split-K kernel only (no whole-K at <= 6 rows)
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
            res = {c: [] for c in CFGS}
            ref = {}
            for _ in range(5):
                for cfg in CFGS:
                    F.lib.cgemm_4bit_set_skinny_config(cfg)
                    res[cfg].append(graph_time(calls))
                    ref[cfg] = F.gemm_4bit(x, ws[0][0], ws[0][1]).float()
            F.lib.cgemm_4bit_set_skinny_config(-1)
            rms = ref[CFGS[0]].pow(2).mean().sqrt().item()
            line = f"{n_out}x{k_in} tokens {m:3d}:"
            for cfg in CFGS:
                d = (ref[cfg] - ref[CFGS[0]]).abs().max().item() / rms
                line += f"  cfg{cfg} {sorted(res[cfg])[2]:6.2f} us (diff {d:.1e})"
            print(line, flush=True)
        del ws
        torch.cuda.empty_cache()
    F.lib.cgemm_4bit_set_fewtoken_kernel(0)


if __name__ == "__main__":
    main()
