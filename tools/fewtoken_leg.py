"""The bench's few-token leg on its own (11008 x 4096 NF4, nested statistics, 14 rotating copies, HIP-graph replay)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

print(json.dumps(bench.bench_few_token_gemm(bench.torch.device("cuda", 0))))
