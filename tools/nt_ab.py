"""Same-process A/B of the two NT GEMM kernels (msu_nt_gemm_mode 1 = ping-pong, 0 = persistent
2-barrier) over the stage 1-3 shapes of the Swin-T 8 x 1024^2 step, interleaved rounds on random
data (cdna_hip_programming.md 5.4 rules 24-25); prints per shape the median us and TF/s of each
kernel and the relative error of the ping-pong result against fp32.
    python tools/nt_ab.py [rounds] [reps]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import _lib, ops  # noqa: E402

SHAPES = [(131072, 576, 192, 0), (131072, 192, 192, 0), (131072, 768, 192, 1), (131072, 192, 768, 0),
          (131072, 768, 192, 2), (32768, 1152, 384, 0), (32768, 384, 384, 0), (32768, 1536, 384, 1),
          (32768, 384, 1536, 0), (32768, 1536, 384, 2), (32768, 768, 384, 0), (32768, 384, 768, 0)]
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
L = _lib.lib()
res = {}
for M, N, K, epi in SHAPES:
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = (torch.rand(M, K, generator=g) * 2 - 1).to("cuda", torch.bfloat16)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) * 0.05).to("cuda", torch.bfloat16)
    bias = torch.randn(N, generator=g).to("cuda") if epi != 2 else None
    h = torch.randn(M, N, generator=g).to("cuda", torch.bfloat16) if epi == 2 else None
    times = {0: [], 1: []}
    for r in range(rounds):
        for mode in (1, 0):
            L.msu_nt_gemm_mode(mode)
            y = ops.nt_gemm(a, w, bias, epi, h=h)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                ops.nt_gemm(a, w, bias, epi, h=h)
            e1.record()
            torch.cuda.synchronize()
            times[mode].append(e0.elapsed_time(e1) / reps * 1e3)
            if mode == 1 and r == 0:
                out = y[0] if isinstance(y, tuple) else y
                ref = torch.nn.functional.linear(a.float(), w.float(), bias)
                if epi == 2:
                    hf = h.float().requires_grad_(True)
                    torch.nn.functional.gelu(hf).backward(torch.ones_like(hf))
                    ref = ref * hf.grad
                err = ((out.float() - ref).norm() / ref.norm()).item()
    L.msu_nt_gemm_mode(1)
    pp = _lib.plan_nt(M, N)[2]
    t1, t0 = statistics.median(times[1]), statistics.median(times[0])
    f = 2.0 * M * N * K / 1e6
    print(f"M={M} N={N} K={K} epi={epi} pp={int(pp)}: pingpong {t1:.1f} us ({f / t1:.0f} TF/s) | "
          f"persistent {t0:.1f} us ({f / t0:.0f} TF/s) | x{t0 / t1:.2f} | rel err {err:.1e}", flush=True)
