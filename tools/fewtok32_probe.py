"""Probe (GPU, for rocprofv3 PMC passes): launches the few-token kernel `reps` times on 14 rotating 11008 x 4096
nested NF4 weights at M tokens, mode from argv (cgemm_4bit_set_fewtok_mode).  Usage: fewtok32_probe.py MODE M"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitsandbytes-sycl_amd"))
from python_src_quants import functional as F  # noqa: E402

mode, m = int(sys.argv[1]), int(sys.argv[2])
n_out, k_in = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (11008, 4096)
dev = torch.device("cuda", 0)
gen = torch.Generator(device=dev).manual_seed(3)
ws = []
for _ in range(14):
    W = (torch.randn(n_out, k_in, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
    ws.append(F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True))
    del W
x = torch.randn(m, k_in, device=dev, dtype=torch.bfloat16, generator=gen)
out = torch.empty(m, n_out, device=dev, dtype=torch.bfloat16)
F.GEMM_4BIT_GEMV_TOKENS = 1
F.set_fewtok_mode(mode)
for _ in range(3):
    for q, st in ws:
        F.gemm_4bit(x, q, st, out=out)
torch.cuda.synchronize()
print("done")
