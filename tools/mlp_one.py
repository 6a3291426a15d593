"""The stage-0 MLP without autograd (8 x 256^2 tokens, 96 -> 384 -> 96, bf16), a few times, for
rocprofv3 kernel-trace passes: the fused inference kernel, or with MSU_MLP_INFER=0 the
token-GEMM pair it replaces.
    python tools/mlp_one.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
g = torch.Generator().manual_seed(0)
w1 = torch.nn.Parameter((torch.randn(384, 96, generator=g) / 96 ** 0.5).cuda())
b1 = torch.nn.Parameter((torch.randn(384, generator=g) * 0.1).cuda())
w2 = torch.nn.Parameter((torch.randn(96, 384, generator=g) / 384 ** 0.5).cuda())
b2 = torch.nn.Parameter((torch.randn(96, generator=g) * 0.1).cuda())
x = torch.randn(8, 256, 256, 96, generator=g).cuda().bfloat16()
with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
    for _ in range(reps):
        y = ops.mlp(x, w1, b1, w2, b2)
torch.cuda.synchronize()
print("ok", ops.mlp_infer_calls)
