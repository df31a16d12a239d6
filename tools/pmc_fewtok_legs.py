"""Run the bench's decode-GEMV and few-token legs once (the config-2 weight 11008 x 4096 NF4, 14 rotating copies),
for rocprofv3 PMC passes: tools/pmc_fewtok.sh."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda", 0)
print(bench.bench_decode_gemv(dev), flush=True)
print(bench.bench_few_token_gemm(dev), flush=True)
