"""Stage-1 MLP forward (8 x 128^2 tokens, 192 -> 768 -> 192, training form: H kept) on the fused
kernel (csrc/mlp_s1.hip) vs the GEMM pair, same process, HIP events; and the no-grad forms.
    python tools/mlp_s1_one.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
M, C, Hd = 8 * 128 * 128, 192, 768
g = torch.Generator().manual_seed(0)
x = torch.randn(M, C, generator=g).to("cuda", torch.bfloat16)
w1 = (torch.randn(Hd, C, generator=g) / C ** 0.5).to("cuda")
b1 = (0.1 * torch.randn(Hd, generator=g)).to("cuda")
w2 = (torch.randn(C, Hd, generator=g) / Hd ** 0.5).to("cuda")
b2 = (0.1 * torch.randn(C, generator=g)).to("cuda")
shapes = {"fused": ops.MLP_KERNEL_SHAPES, "pair": ops.MLP_KERNEL_SHAPES[:1]}
res = {}
for rnd in range(3):
    for name, sh in shapes.items():
        ops.MLP_FUSED_SHAPES = sh
        for keep in (True, False):
            fn = lambda: torch.ops.msunet.mlp(x, w1, b1, w2, b2, keep)  # noqa: E731
            with torch.autocast("cuda", dtype=torch.bfloat16):
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    fn()
                e1.record()
            torch.cuda.synchronize()
            res.setdefault((name, keep), []).append(e0.elapsed_time(e1) / reps * 1e3)
for (name, keep), v in res.items():
    print(f"mlp_s1 {name} keep={keep}: {min(v):.1f} us (min of {len(v)}; all {', '.join(f'{t:.1f}' for t in v)})")
