"""bench.py's token-row chunk rule for the sharded step (auto_chunks): one chunk on one GPU, two at 2 and 4 GPUs, one at
8 (profiles/lab/r04_shard_compute.txt), an explicit --chunks honoured when it divides M."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_auto_chunks():
    assert bench.auto_chunks(1) == 1 and bench.auto_chunks(1, 4) == 1
    assert bench.auto_chunks(2) == 2 and bench.auto_chunks(4) == 2 and bench.auto_chunks(8) == 1
    assert bench.auto_chunks(8, 2) == 2 and bench.auto_chunks(2, 4) == 4
    assert bench.auto_chunks(2, 3) == 1                  # 3 does not divide M = 4096
