"""Run the few-token NF4 GEMM (nested stats) a fixed number of times for a kernel trace.
Usage: python tools/skinny_probe.py N K M [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import python_src_quants.functional as F  # noqa: E402

N, K, M = (int(a) for a in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 200
dev = torch.device("cuda", 0)
W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
copies = [F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True) for _ in range(14)]
X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
for i in range(reps):
    q, st = copies[i % len(copies)]
    F.gemm_4bit(X, q, st, out=Y)
torch.cuda.synchronize()
print("done")
