"""Run the swinT224 Trainer twice per mode (eager / graph) and report whether the losses and
final states are bitwise identical run-to-run (nondeterministic library kernels or races
show up here).  python tools/determinism_check.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import test_gpu_graph as tg  # noqa: E402

for graph in (False, True):
    a, b = tg._run(graph, 1e-3), tg._run(graph, 1e-3)
    same_loss = a[0] == b[0]
    diffs = [(u - v).abs().max().item() for u, v in zip(a[1], b[1])]
    print(f"graph={graph}: losses identical {same_loss}; max state diff {max(diffs):.3e}")
    print("  ", a[0])
    print("  ", b[0])
