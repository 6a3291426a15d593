"""Run one window-attention forward (and optionally backward) shape repeatedly (rocprofv3).
    python tools/attn_one.py res nh shift [bwd 0|1] [reps] [p_drop]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import ops  # noqa: E402

res, nh, shift = (int(v) for v in sys.argv[1:4])
bwd = len(sys.argv) > 4 and sys.argv[4] == "1"
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
p_drop = float(sys.argv[6]) if len(sys.argv) > 6 else 0.0
C = 32 * nh
qkv = torch.randn(8, res, res, 3 * C, device="cuda", dtype=torch.bfloat16, requires_grad=bwd)
qb = torch.randn(3 * C, device="cuda")
tb = torch.randn(169, nh, device="cuda")
with torch.autocast("cuda", dtype=torch.bfloat16):
    for _ in range(reps):
        y = ops.window_attention(qkv, qb, tb, nh, shift, p_drop, 1)
        if bwd:
            y.backward(torch.ones_like(y))
torch.cuda.synchronize()
print("ok")
