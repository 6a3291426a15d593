"""cProfile of the host side of the bench training step (GPU box): python tools/host_prof.py [steps]
Prints the top functions by own time, to find Python overhead per launch."""
import cProfile
import os
import pstats
import sys

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
from semantic_segmentation_of_stylegan2_artifacts_amd import load_config  # noqa: E402
from semantic_segmentation_of_stylegan2_artifacts_amd.network import MSUNet  # noqa: E402
from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer  # noqa: E402
from semantic_segmentation_of_stylegan2_artifacts_amd.data import batch_pool  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
backbone = sys.argv[2] if len(sys.argv) > 2 else "swin_t"
dev = torch.device("cuda", 0)
cfg = load_config(None, backbone, **{"DATA.IMG_SIZE": 1024, "DATA.BATCH_SIZE": 8})
torch.manual_seed(cfg.SEED)
model = MSUNet(cfg, img_size=1024, num_classes=1).to(dev)
tr = Trainer(model, cfg, dev)
pool = batch_pool(2, 8, 1024, dev, cfg.SEED)
for i in range(3):
    tr.step(*pool[i % 2])
torch.cuda.synchronize()
import time  # noqa: E402
for i in range(2):  # host time of forward / backward / rest, no sync inside a step
    t0 = time.perf_counter()
    loss = tr.forward_loss(*pool[i % 2])
    t1 = time.perf_counter()
    loss.backward()
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    print(f"host fwd {1e3*(t1-t0):.1f} ms  bwd {1e3*(t2-t1):.1f} ms  then GPU drain {1e3*(t3-t2):.1f} ms", flush=True)
for g in tr.groups:
    g.grad.zero_()
pr = cProfile.Profile()
pr.enable()
for i in range(steps):
    tr.step(*pool[i % 2])
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)
st.sort_stats("cumulative").print_stats(25)
