"""CPU: bench.py's N-rank launch contract (no GPU call is reached in these cases).

* a launcher-started rank whose WORLD_SIZE differs from ``--gpus`` fails before touching the
  GPU, instead of timing a different job than the one it names;
* ``--gpus 2`` without WORLD_SIZE starts two rank processes and returns a failing rank's exit
  status (here the ranks fail at device selection: this container has no GPU).
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = [sys.executable, os.path.join(REPO, "bench.py")]
QUIET = ["--steps", "1", "--warmup", "0", "--no-roofline", "--no-cpu-baseline", "--no-input-pipeline"]


def _env(**kv):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(kv)
    return env


def test_bench_rejects_world_mismatch():
    r = subprocess.run(BENCH + ["--gpus", "2"] + QUIET, env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                       cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in (r.stdout + r.stderr)


def test_bench_launcher_propagates_rank_failure():
    r = subprocess.run(BENCH + ["--gpus", "2", "--dist-backend", "gloo"] + QUIET, env=_env(HIP_VISIBLE_DEVICES=""),
                       cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0, r.stdout + r.stderr
    assert "{" not in r.stdout  # no bench line from a failed job
