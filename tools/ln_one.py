"""LayerNorm forward / backward at the Swin-T 1024^2 bs 8 step's shapes (plain and residual-add
modes), a few times each, for rocprofv3 kernel-trace passes (kernel durations, not host time).
    python tools/ln_one.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
B = 8
with torch.autocast("cuda", dtype=torch.bfloat16):
    for rows, C in ((B * 65536, 96), (B * 16384, 192), (B * 4096, 384), (B * 1024, 768)):
        w = torch.nn.Parameter(torch.randn(C, device="cuda"))
        bb = torch.nn.Parameter(torch.randn(C, device="cuda"))
        x = torch.randn(rows, C, device="cuda", dtype=torch.bfloat16).requires_grad_(True)
        a = torch.randn(rows, C, device="cuda", dtype=torch.bfloat16).requires_grad_(True)
        for _ in range(reps):
            y = ops.layer_norm(x, w, bb)
            y.backward(torch.ones_like(y))
            s, y2 = ops.add_layer_norm(a, x, None, w, bb)
            torch.autograd.backward([y2, s], [torch.ones_like(y2), torch.ones_like(s)])
torch.cuda.synchronize()
print("ok")
