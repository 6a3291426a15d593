"""Kernel times of the NT GEMM over the stage 1-3 shapes of the Swin-T 8 x 1024^2 step, in one
process for whichever library is loaded (MSU_LIB_OVERRIDE selects another build), with the
relative error against fp32 PyTorch per shape.  Run it once per library, interleaved, for an A/B:
    python tools/nt_shapes.py [reps] [tag]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import ops  # noqa: E402

# (M, N, K, epi, kn): epi 0 plain + bias, 1 GELU dual, 2 GELU'; kn: weight read as [K][N]
SHAPES = [(131072, 576, 192, 0, 0), (131072, 192, 192, 0, 0), (131072, 768, 192, 1, 0), (131072, 192, 768, 0, 0),
          (131072, 768, 192, 2, 0), (32768, 1152, 384, 0, 0), (32768, 384, 384, 0, 0), (32768, 1536, 384, 1, 0),
          (32768, 384, 1536, 0, 0), (32768, 1536, 384, 2, 0), (32768, 768, 384, 0, 0), (32768, 384, 768, 0, 0),
          (8192, 2304, 768, 0, 0), (8192, 768, 768, 0, 0), (8192, 3072, 768, 1, 0), (8192, 768, 3072, 0, 0),
          (32768, 384, 1152, 0, 1), (131072, 192, 576, 0, 1)]
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
tag = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(os.environ.get("MSU_LIB_OVERRIDE", "") or "cur")
# NT_FORCE=1/2/3: a forced tile form (msu_nt_gemm_mode bits 1-2) for this run
force = int(os.environ.get("NT_FORCE", "0"))
a3 = int(os.environ.get("NT_A3", "-1"))
if force or a3 >= 0:
    from semantic_segmentation_of_stylegan2_artifacts_amd import _lib  # noqa: E402
    prev = _lib.lib().msu_nt_gemm_mode(0)
    a3 = (prev >> 3) & 1 if a3 < 0 else a3
    _lib.lib().msu_nt_gemm_mode((prev & 17) | (force << 1) | (a3 << 3))
    tag = f"F{force}A{a3}"
tot = 0.0
for M, N, K, epi, kn in SHAPES:
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = (torch.rand(M, K, generator=g) * 2 - 1).to("cuda", torch.bfloat16)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) * 0.05).to("cuda", torch.bfloat16)
    bias = torch.randn(N, generator=g).to("cuda") if epi != 2 and not kn else None
    h = torch.randn(M, N, generator=g).to("cuda", torch.bfloat16) if epi == 2 else None
    if kn:
        wk = w.t().contiguous()
        fn = lambda: ops.nt_gemm_kn(a, wk, epi, h=h)  # noqa: E731
    else:
        fn = lambda: ops.nt_gemm(a, w, bias, epi, h=h)  # noqa: E731
    y = fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps * 1e3)
    out = y[0] if isinstance(y, tuple) else y
    ref = torch.nn.functional.linear(a.float(), w.float(), bias)
    if epi == 2:
        hf = h.float().requires_grad_(True)
        torch.nn.functional.gelu(hf).backward(torch.ones_like(hf))
        ref = ref * hf.grad
    err = ((out.float() - ref).norm() / ref.norm()).item()
    us = statistics.median(ts)
    tot += us
    print(f"{tag} nt M={M} N={N} K={K} epi={epi} kn={kn}: {us:7.1f} us {2.0 * M * N * K / us / 1e6:6.0f} TF/s "
          f"rel err {err:.1e}", flush=True)
print(f"{tag} total {tot:.1f} us")
