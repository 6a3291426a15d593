import os, sys, torch
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
from semantic_segmentation_of_stylegan2_artifacts_amd import load_config
from semantic_segmentation_of_stylegan2_artifacts_amd.network import MSUNet
from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer
from semantic_segmentation_of_stylegan2_artifacts_amd.data import batch_pool
from torch.profiler import profile, ProfilerActivity
dev = torch.device("cuda", 0)
cfg = load_config(None, "swin_t", **{"DATA.IMG_SIZE": 1024, "DATA.BATCH_SIZE": 8})
model = MSUNet(cfg, img_size=1024, num_classes=1).to(dev)
tr = Trainer(model, cfg, dev)
pool = batch_pool(1, 8, 1024, dev, 0)
for _ in range(2): tr.step(*pool[0])
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], record_shapes=True) as prof:
    tr.step(*pool[0]); torch.cuda.synchronize()
evs = prof.events()
from collections import Counter
c = Counter()
for e in evs:
    if e.name in ("aten::copy_", "aten::add", "aten::add_", "aten::clone", "aten::contiguous", "aten::to", "aten::_to_copy"):
        shapes = e.input_shapes
        big = any(len(s) > 0 and torch.Size(s).numel() > 10_000_000 for s in shapes if isinstance(s, list))
        if not big: continue
        p = e.cpu_parent
        chain = []
        while p is not None and len(chain) < 4:
            chain.append(p.name[:60]); p = p.cpu_parent
        c[(e.name, str(shapes)[:80], " <- ".join(chain))] += 1
for k, v in c.most_common(25): print(v, k)
