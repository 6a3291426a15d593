"""Time the one-pass stage-0 Linear backward (msu_linear_bwd) against the two-kernel path
(token-GEMM input gradient + msu_linear_wgrad) at the bench's stage-0 shapes, alone on the GPU.

    python tools/linbwd_bench.py [K N [gg]]      (default: every stage-0 shape)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import _lib, ops  # noqa: E402

DEV = "cuda"
M = 8 * 65536


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    L = _lib.lib()
    s = torch.cuda.current_stream().cuda_stream
    shapes = [(96, 288, False), (96, 96, False), (96, 384, False), (384, 96, False), (384, 96, True)]
    if len(sys.argv) > 2:
        shapes = [(int(sys.argv[1]), int(sys.argv[2]), len(sys.argv) > 3 and sys.argv[3] == "1")]
    for K, N, gg in shapes:
        dy = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
        x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
        wt = w.t().contiguous()
        h = torch.randn(M, K, device=DEV, dtype=torch.bfloat16) if gg else None
        dx = torch.empty(M, K, device=DEV, dtype=torch.bfloat16)
        dw = torch.zeros(N, K, device=DEV)
        db = torch.zeros(N, device=DEV)
        ws = torch.empty(L.msu_linear_bwd_workspace(M, K, N), device=DEV)
        ws2 = torch.empty(L.msu_wgrad_workspace(M, N, K), device=DEV)
        hp = None if h is None else h.data_ptr()

        def fused():
            _lib.call("msu_linear_bwd", 1, dy.data_ptr(), x.data_ptr(), wt.data_ptr(), hp, dx.data_ptr(),
                      dw.data_ptr(), db.data_ptr(), ws.data_ptr(), M, K, N, 1, s)

        def dgrad():
            ops._gemm(dy, wt, None, ops.TOK_GELU_GRAD if gg else ops.TOK_PLAIN, h)

        def wgrad():
            _lib.call("msu_linear_wgrad", 1, dy.data_ptr(), x.data_ptr(), dw.data_ptr(), db.data_ptr(),
                      ws2.data_ptr(), M, N, K, 1, s)

        tf, td, tw = timeit(fused), timeit(dgrad), timeit(wgrad)
        byts = M * (N + 2 * K + (K if gg else 0)) * 2
        print(f"linbwd K={K:4d} N={N:4d} gg={int(gg)}: fused {tf*1e3:7.1f} us ({byts/tf/1e6:6.0f} GB/s)   "
              f"dgrad {td*1e3:7.1f} + wgrad {tw*1e3:7.1f} = {(td+tw)*1e3:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
