"""Time token-GEMM shapes: python tools/tok_time.py M,N,K[,epi] ..."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import ops  # noqa: E402


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for spec in sys.argv[1:]:
    v = [int(x) for x in spec.split(",")]
    M, N, K = v[:3]
    epi = v[3] if len(v) > 3 else 0
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device="cuda")
    h = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    if epi == 2:
        f = lambda: ops.tok_gemm(a, w, None, 2, h=h)
        byts = M * (K + 2 * N) * 2
    else:
        f = lambda: ops.tok_gemm(a, w, b, epi)
        byts = M * (K + N * (2 if epi == 1 else 1)) * 2
    ms = timeit(f)
    print(f"M={M} N={N} K={K} epi={epi}: {ms*1e3:.1f} us  {byts/ms/1e6:.0f} GB/s", flush=True)
