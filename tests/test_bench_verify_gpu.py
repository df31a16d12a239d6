"""bench.py's output checks on the GPU at world 1 (the N > 1 path is covered over gloo in tests/test_bench_verify_cpu.py):
the NF4 world-1 sample accepts the product's own output and rejects a single corrupted element; the int8 sample is
bit-exact against the unsharded igemmlt + dequant (a shard's rows equal the full product's rows bit for bit) and rejects
a one-ulp change; verify_sharded_output flags a shard that differs from its block of the assembled output."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import python_src_quants.functional as F  # noqa: E402
from python_src_quants.parallel import ColumnShardedLinear8bitLt  # noqa: E402


def test_nf4_world1_sample_accepts_and_rejects():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    X = torch.randn(512, 1024, device=dev, dtype=torch.bfloat16, generator=g)
    W = (torch.randn(768, 1024, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q, st = F.quantize_4bit(W, blocksize=64, quant_type="nf4", compress_statistics=True)
    Y = F.gemm_4bit(X, q, st)
    rows = bench.sample_rows(512, 64)
    check = bench.nf4_world1_sample(X, q, st, rows)
    assert check(Y)["ok"]
    Yb = Y.clone()
    Yb[rows[3], 5] += 1.0
    assert not check(Yb)["ok"]
    res = bench.verify_sharded_output(Y, Y, 1, 0, dev, sample_fn=check)
    assert res["ok"] and res["shard_block_mismatches"] == 0


def test_int8_world1_sample_bitwise_and_shard_mismatch():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(8)
    A = (torch.randn(512, 1024, device=dev, generator=g) * 2).half()
    Wt = (torch.randn(768, 1024, device=dev, generator=g) * 0.05).half()
    CB, _, SCB, _, _ = F.double_quant(Wt)
    rows = bench.sample_rows(512, 64)
    check = bench.int8_world1_sample(A, CB, SCB, rows)
    for world in (1, 2, 3):
        parts = [ColumnShardedLinear8bitLt(CB, SCB, world, r).forward_local(A) for r in range(world)]
        assembled = torch.cat(parts, dim=1)
        assert check(assembled)["ok"], world             # shard rows = the full product's rows, bit for bit
    bad = assembled.clone()
    bad.view(torch.int16)[rows[7], 11] += 1                # one ulp
    assert not check(bad)["ok"]
    # a shard that is not what the assembled output holds in its block
    shard = parts[1].clone()
    shard[0, 0] += 1
    res = bench.verify_sharded_output(shard, assembled, 3, 1, dev)
    assert not res["ok"] and res["shard_block_mismatches"] == 1
