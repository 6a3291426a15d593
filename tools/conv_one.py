"""Run one refine-conv forward shape repeatedly (for rocprofv3 counter passes).
    python tools/conv_one.py [d2s 0|1] [reps] [fwd|bwd] [act]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import ops  # noqa: E402

d2s = len(sys.argv) > 1 and sys.argv[1] == "1"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
B, C, H = 8, 96, 1024
x = torch.randn((B, H // 4, H // 4, 16 * C) if d2s else (B, H, H, C), device="cuda", dtype=torch.bfloat16)
w = torch.randn(C, C, 3, 3, device="cuda") * 0.03
b = torch.randn(C, device="cuda")
a = torch.nn.functional.gelu(x)
bwd = len(sys.argv) > 3 and sys.argv[3] == "bwd"
act = len(sys.argv) > 4 and sys.argv[4] == "act"  # the model's path: activation precomputed
with torch.autocast("cuda", dtype=torch.bfloat16):
    if bwd:
        xq, wq = x.requires_grad_(True), w.requires_grad_(True)
        # act: the model's path (activation from the producer; the weight gradient reads it as is)
        z = ops.refine_conv_act(xq, a, wq, b, d2s, (H, H)) if act else ops.refine_conv(xq, wq, b, d2s, (H, H))
        dz = torch.randn_like(z)
    for _ in range(reps):
        if bwd:
            torch.autograd.grad(z, (xq, wq), dz, retain_graph=True)
        elif act:
            ops.refine_conv_act(x, a, w, b, d2s, (H, H))
        else:
            ops.refine_conv(x, w, b, d2s, (H, H))
torch.cuda.synchronize()
print("ok")
