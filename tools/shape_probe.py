"""Time one Linear shape on every hand-written GEMM form that covers it: the NT GEMM's cost-model
pick and each forced tile form (msu_nt_gemm_mode bits 1-2), and the token GEMM when supported.
    python tools/shape_probe.py M N K [reps]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import _lib, ops  # noqa: E402

M, N, K = (int(a) for a in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
g = torch.Generator(device="cpu").manual_seed(0)
a = (torch.rand(M, K, generator=g) * 2 - 1).to("cuda", torch.bfloat16)
w = ((torch.rand(N, K, generator=g) * 2 - 1) * 0.05).to("cuda", torch.bfloat16)
ref = torch.nn.functional.linear(a.float(), w.float())
L = _lib.lib()
prev = L.msu_nt_gemm_mode(0)


def timed(fn):
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
    err = ((y.float() - ref).norm() / ref.norm()).item()
    return statistics.median(ts), err


arms = [(f"nt F{f}", f) for f in (0, 1, 2, 3)]
for name, f in arms:
    L.msu_nt_gemm_mode((prev & 17) | (f << 1))
    us, err = timed(lambda: ops.nt_gemm(a, w, None))
    print(f"{name:8s} M={M} N={N} K={K}: {us:8.1f} us {2.0 * M * N * K / us / 1e6:7.1f} TF/s "
          f"{(M * K + N * K + M * N) * 2 / us / 1e3:7.1f} GB/s  rel err {err:.1e}", flush=True)
L.msu_nt_gemm_mode(prev)
if ops.tok_supported_epi(M, N, K, ops.TOK_PLAIN):
    us, err = timed(lambda: ops.tok_gemm(a, w, None))
    print(f"{'tok':8s} M={M} N={N} K={K}: {us:8.1f} us {2.0 * M * N * K / us / 1e6:7.1f} TF/s "
          f"{(M * K + N * K + M * N) * 2 / us / 1e3:7.1f} GB/s  rel err {err:.1e}", flush=True)
print("route:", ops.gemm_route(M, N, K), "plan:", _lib.plan_nt(M, N))
