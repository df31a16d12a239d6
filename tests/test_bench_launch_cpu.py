"""bench.py's multi-GPU launch: `bench.py --gpus N` without a launcher starts N rank processes
itself (torch.distributed.run as one child process, before any GPU call), and a launcher whose WORLD_SIZE disagrees
with --gpus is refused with a non-zero exit instead of measuring (and reporting) a different world size."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(kw)
    return env


def test_rank_launch_cmd():
    cmd = bench.rank_launch_cmd(["--gpus", "4", "--steps", "7"], 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "7"]
    assert bench._gpus_arg(["--gpus=8"]) == 8 and bench._gpus_arg([]) == 1


def test_world_mismatch_message():
    assert bench.world_mismatch(["--gpus", "2"], {}) == ""
    assert bench.world_mismatch(["--gpus", "2"], {"WORLD_SIZE": "2"}) == ""
    assert "WORLD_SIZE=4" in bench.world_mismatch(["--gpus", "8"], {"WORLD_SIZE": "4"})
    assert bench.world_mismatch([], {"WORLD_SIZE": "2"})      # --gpus defaults to 1


def test_world_mismatch_exits_nonzero():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-check"], env=_env(WORLD_SIZE="2", RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stderr
    assert "WORLD_SIZE=2" in r.stderr and "--gpus 3" in r.stderr
    assert r.stdout.strip() == ""


def test_gpus_n_launches_n_ranks():
    """No launcher, --gpus 2: two rank processes, rank 0 reports n_gpus 2 (gloo, no GPU work)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["gpus_arg"] == 2
    assert sorted(x["rank"] for x in rec["ranks"]) == [0, 1]
    assert sorted(x["local_rank"] for x in rec["ranks"]) == [0, 1]
    assert len({x["pid"] for x in rec["ranks"]}) == 2
