"""Time one Linear weight-gradient shape (for rocprofv3 counter passes).
    python tools/wgrad_one.py M N K [reps]"""
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
for _ in range(reps):
    _lib.call("msu_linear_wgrad", 1, dy.data_ptr(), x.data_ptr(), dw.data_ptr(), db.data_ptr(), ws.data_ptr(),
              M, N, K, 0, s)
torch.cuda.synchronize()
print("ok")
