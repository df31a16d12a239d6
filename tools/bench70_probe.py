"""Run bench.py's config-5 leg (bench_llama2_70b_shard) alone on the GPU: python tools/bench70_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.argv = ["bench.py"]
import bench  # noqa: E402

print(json.dumps(bench.bench_llama2_70b_shard(torch.device("cuda", 0))))
