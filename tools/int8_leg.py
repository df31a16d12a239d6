"""The bench's int8 legs on their own (metric shape and config 3): fused igemmlt+dequant, the inference forward with
one-pass row quantisation, and the reference ABI flow."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = bench.torch.device("cuda", 0)
print(json.dumps({"metric_shape": bench.bench_int8(dev, 4096, 4096, 11008), "config3": bench.bench_int8(dev, 4096, 4096, 4096)}))
