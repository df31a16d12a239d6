"""bench.py's N > 1 self-validation, rehearsed on CPU over gloo with two ranks: the real sharded-step
helper assembles a toy product, then bench.verify_sharded_output checks (a) each rank's shard against its block of the
assembled output bit for bit, (b) the assembled output identical on every rank, (c) rank 0's sampled rows against the
world-1 product.  A fault injected on one rank -- in each of the three places only one check can see -- must turn the
run into a non-zero exit with outputs_verified false on rank 0's line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(*extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--verify-check", *extra], env=env,
                       capture_output=True, text=True, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


def test_verify_clean_run_passes():
    r, rec = _run()
    assert r.returncode == 0, r.stderr[-3000:]
    assert rec["outputs_verified"] is True
    v = rec["verification"]
    assert v["shard_block_mismatches"] == 0 and v["assembled_identical_on_all_ranks"] and v["world1_sample_ok"]
    d = rec["distributed"]
    assert d["backend"] == "gloo" and d["world_size"] == 2
    assert sorted(x["rank"] for x in d["ranks"]) == [0, 1]


@pytest.mark.parametrize("mode,rank,field", [
    ("shard", 1, "shard_block_mismatches"),
    ("shard", 0, "shard_block_mismatches"),
    ("assembled", 1, "assembled_identical_on_all_ranks"),
    ("values", 1, "world1_sample_ok"),
])
def test_verify_fault_exits_nonzero(mode, rank, field):
    r, rec = _run("--corrupt", mode, "--corrupt-rank", str(rank))
    assert r.returncode != 0
    assert rec is not None, r.stderr[-3000:]
    assert rec["outputs_verified"] is False
    v = rec["verification"]
    if field == "shard_block_mismatches":
        assert v[field] == 1
    else:
        assert v[field] is False
