"""bench.py's rank launch on the CPU (no GPU call is made): `python bench.py --gpus N` starts N
ranks itself, a --gpus that disagrees with WORLD_SIZE is refused, and a failing rank ends the
whole command with a non-zero status instead of a hang."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", **kw)
    return env


def test_gpus_n_starts_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-check"], capture_output=True,
                       text=True, timeout=180, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0's line only
    d = json.loads(lines[0])
    assert d == {"launch_check": True, "n_gpus": 3, "ranks_reporting": 3}


def test_gpus_disagreeing_with_world_size_is_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], capture_output=True, text=True, timeout=120,
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), cwd=ROOT)
    assert r.returncode == 2
    assert "--gpus 2 but WORLD_SIZE=1" in r.stderr


def test_failing_rank_fails_the_command():
    t0 = time.time()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--fail-rank", "1", "--launch-check",
                        "--pg-timeout", "60"], capture_output=True, text=True, timeout=170, env=_env(), cwd=ROOT)
    assert r.returncode != 0
    assert "fails on request" in r.stderr
    assert time.time() - t0 < 150
