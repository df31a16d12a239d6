"""Print the bench's measured ceilings (bench.measure_peaks: MFMA bf16 / int8 at one and two waves per SIMD, HBM read)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

print(json.dumps(bench.measure_peaks(bench.torch.device("cuda", 0))))
