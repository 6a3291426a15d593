"""Run the fused stage-0 attention unit (qkv Linear + window attention + proj, training forward
and its backward) repeatedly, for rocprofv3 counter / kernel-trace passes.
    python tools/attn_qkv_one.py [reps] [p_drop]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
p_drop = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
B, R, C, nh = 8, 256, 96, 3
torch.manual_seed(0)
x = (torch.randn(B, R, R, C, device="cuda") * 0.5).bfloat16().requires_grad_(True)
w = torch.nn.Parameter(torch.randn(3 * C, C, device="cuda") * 0.05)
b = torch.nn.Parameter(torch.randn(3 * C, device="cuda") * 0.05)
tb = torch.nn.Parameter(torch.randn(169, nh, device="cuda") * 0.02)
wp = torch.nn.Parameter(torch.randn(C, C, device="cuda") * 0.05)
bp = torch.nn.Parameter(torch.randn(C, device="cuda") * 0.05)
with torch.autocast("cuda", dtype=torch.bfloat16):
    for i in range(reps):
        y = ops.window_attention_qkv(x, w, b, tb, nh, 3, p_drop, seed=i, proj_weight=wp, proj_bias=bp)
        y.float().sum().backward()
torch.cuda.synchronize()
assert ops.fused_qkv_calls == reps, ops.fused_qkv_calls
print("ok")
