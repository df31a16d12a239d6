"""Run the 33..64-token kernel at 11008 x 4096 x 64 rows (NF4 nested, bf16) repeatedly, for rocprofv3 counter passes
(tools/lab_counters.sh t64 python3 tools/t64_driver.py [iters])."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import python_src_quants.functional as F  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
N, K, M = 11008, 4096, 64
W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
for _ in range(iters):
    F.gemm_4bit(X, q, st, out=Y)
torch.cuda.synchronize()
print("ok")
