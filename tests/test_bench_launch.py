"""CPU: bench.py's rank launch.  `bench.py --gpus N` without an external launcher must start N
ranks itself (the driver's 8-GPU run cannot silently degrade to one rank), forward rank 0's one
JSON line and fail loudly when WORLD_SIZE and --gpus disagree.  --launch-check stops right after
the process group is up, so no GPU is needed."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra)
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_its_ranks_without_a_launcher(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-check"], env=_env(),
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout          # exactly one JSON line, rank 0's
    doc = json.loads(lines[0])
    assert doc["n_gpus"] == n
    assert doc["process_group"] == {"world_size": n, "backend": "gloo"}


def test_bench_refuses_world_size_mismatch():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], env=_env(WORLD_SIZE="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert r.stdout.strip() == ""
    assert "WORLD_SIZE=1" in r.stderr


def test_bench_failing_rank_fails_the_launch():
    # a rank that dies must make the parent exit non-zero, with no result line
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"],
                       env=_env(LGX_LAUNCH_CHECK_FAIL_RANK="1"), capture_output=True, text=True, timeout=180)
    assert r.returncode != 0
    assert r.stdout.strip() == ""
