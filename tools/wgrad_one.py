"""Time one Linear weight-gradient shape (also the program of the rocprofv3 counter passes).
    python tools/wgrad_one.py M N K [reps]      -> prints the average launch time (HIP events)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import _lib  # noqa: E402

M, N, K = (int(a) for a in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
L = _lib.lib()
ws = torch.empty(L.msu_wgrad_workspace(M, N, K), device="cuda")
dw = torch.empty(N, K, device="cuda")
db = torch.empty(N, device="cuda")
s = torch.cuda.current_stream().cuda_stream


def launch():
    _lib.call("msu_linear_wgrad", 1, dy.data_ptr(), x.data_ptr(), dw.data_ptr(), db.data_ptr(), ws.data_ptr(),
              M, N, K, 0, s)


launch()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    launch()
e1.record()
torch.cuda.synchronize()
ref = dy.float().t() @ x.float()
err = (dw - ref).abs().max().item() / ref.abs().max().item()
print(f"wgrad M={M} N={N} K={K}: {e0.elapsed_time(e1) / reps * 1e3:.1f} us/launch (+colsum), rel err {err:.2e}")
