"""Time one tiled-NT-GEMM shape (also the program of rocprofv3 counter passes).
    python tools/nt_one.py M N K [reps] [epi]   -> average launch time (HIP events), TF/s, rel err"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import ops  # noqa: E402

M, N, K = (int(a) for a in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
g = torch.Generator(device="cpu").manual_seed(0)
a = (torch.rand(M, K, generator=g) * 2 - 1).to("cuda", torch.bfloat16)
w = ((torch.rand(N, K, generator=g) * 2 - 1) * 0.05).to("cuda", torch.bfloat16)
bias = torch.randn(N, generator=g).to("cuda")
y = ops.nt_gemm(a, w, bias)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    ops.nt_gemm(a, w, bias)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / reps * 1e3
ref = torch.nn.functional.linear(a.float(), w.float(), bias)
err = ((y.float() - ref).norm() / ref.norm()).item()
print(f"nt M={M} N={N} K={K}: {us:.1f} us/launch, {2.0 * M * N * K / us / 1e6:.1f} TF/s, rel err {err:.1e}")
