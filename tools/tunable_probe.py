"""Time the hipBLASLt/rocBLAS path of F.linear at the stage 1-3 shapes (run with and without
PYTORCH_TUNABLEOP_ENABLED=1 to compare TunableOp's pick against the default heuristic)."""
import os
import sys
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.kbench import timeit  # noqa: E402

shapes = [(131072, 576, 192), (131072, 192, 192), (131072, 768, 192), (131072, 192, 768),
          (32768, 1152, 384), (32768, 384, 384), (32768, 1536, 384), (32768, 384, 1536),
          (8192, 2304, 768), (8192, 768, 768), (8192, 3072, 768), (8192, 768, 3072),
          (32768, 384, 1152), (131072, 192, 576)]
tot = 0.0
for M, N, K in shapes:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    ms = timeit(lambda: torch.nn.functional.linear(a, w, b))
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    md = timeit(lambda: dy.matmul(w))
    tot += ms + md
    print(f"M={M} N={N} K={K}: fwd {ms*1e3:.1f} us ({2*M*N*K/ms/1e9:.0f} TF/s)  dgrad {md*1e3:.1f} us", flush=True)
print(f"total {tot*1e3:.1f} us")
