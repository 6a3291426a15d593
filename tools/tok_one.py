"""Run one token-GEMM shape repeatedly (for rocprofv3 counter passes).
    python tools/tok_one.py M N K [epi] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import ops  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
epi = int(sys.argv[4]) if len(sys.argv) > 4 else 0
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
b = torch.randn(N, device="cuda")
h = torch.randn(M, N, device="cuda", dtype=torch.bfloat16) if epi == 2 else None
for _ in range(reps):
    if epi == 2:
        ops.tok_gemm(a, w, None, 2, h=h)
    else:
        ops.tok_gemm(a, w, b, epi)
torch.cuda.synchronize()
print("ok")
