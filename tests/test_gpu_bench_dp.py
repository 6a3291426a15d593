"""GPU: ``bench.py --gpus 2`` starts its two ranks itself.

The driver runs ``python bench.py --gpus N`` without a launcher; the bench must then start N
rank processes before any GPU call, join a process group of exactly N ranks and report
``n_gpus: N``.  On a one-GPU box the nccl (RCCL) path needs N devices, so the same code runs
here with ``--dist-backend gloo`` (both ranks on cuda:0; everything else -- the Trainer, the
bucketed all-reduce hooks, the max-over-ranks timing -- is the nccl path's).  Checks: one JSON
line with n_gpus 2, world_size 2 and global_batch 2 x bs, and bitwise-identical parameters on
both ranks after the timed steps (each rank trained on its own batch: only the gradient
all-reduce makes them agree).  Reference: trainer.py:96-97 (nn.DataParallel over the GPUs).
"""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_launches_two_ranks(tmp_path):
    dump = str(tmp_path / "state")
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--img", "256", "--batch", "2", "--steps", "3", "--warmup", "2", "--no-roofline",
           "--no-cpu-baseline", "--no-input-pipeline", "--dump-state", dump]
    r = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2
    assert res["config"]["world_size"] == 2
    assert res["config"]["dist_backend"] == "gloo"
    assert res["config"]["global_batch"] == 4
    assert res["config"]["parallelism"] == "dp2"
    assert res["value"] > 0 and res["steps"] == 3
    s0 = torch.load(dump + ".rank0.pt", weights_only=True)
    s1 = torch.load(dump + ".rank1.pt", weights_only=True)
    assert s0["world"] == s1["world"] == 2 and (s0["rank"], s1["rank"]) == (0, 1)
    for a, b in zip(s0["data"], s1["data"]):
        assert torch.equal(a, b), "ranks disagree after the all-reduced steps"
