"""Graph capture of the trainer step with the bucketed RCCL all-reduce inside it.

One GPU, a one-rank "nccl" (RCCL) process group; the Trainer's GradBucketer is installed by
hand (world_size 1 has none) so that every bucket's all_reduce is issued from the side stream
during the captured backward, as on 8 GPUs.  Compares 5 steps (3 replays) with an eager run.

    python tools/graph_rccl_check.py
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))


def run(graph, pg):
    import cases
    from oracle.msunet import make_cfg
    from semantic_segmentation_of_stylegan2_artifacts_amd import load_config
    from semantic_segmentation_of_stylegan2_artifacts_amd.network.model_parts import MSUNetSys
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer, GradBucketer
    spec = cases.model_cases()["swinT224"]
    cfg = make_cfg(**spec["cfg"])
    m = MSUNetSys(img_size=224, embed_dim=96, depths=cfg["depths"], num_heads=cfg["num_heads"], drop_path_rate=0.0)
    m.load_state_dict(cases.model_params(cfg, spec["seed"]), strict=True)
    m = m.cuda().train()
    x, t = cases.model_inputs(cfg, 2, spec["seed"])
    x, t = x.cuda(), t.cuda()
    tr = Trainer(m, load_config(None, "swin_t", **{"TRAIN.BASE_LR": 1e-3}), "cuda", use_graph=graph)
    tr.reducer = GradBucketer(tr.groups, 1 << 20, pg)
    losses = [tr.step(x, t).item() for _ in range(5)]
    torch.cuda.synchronize()
    return losses, torch.cat([g.data for g in tr.groups]), tr._graph is not None


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    le, pe, _ = run(False, dist.group.WORLD)
    lg, pgr, captured = run(True, dist.group.WORLD)
    print("captured:", captured)
    print("eager:", le)
    print("graph:", lg)
    err = (pe - pgr).abs().max().item()
    print("max |param diff|:", err)
    dist.destroy_process_group()
    ok = captured and err < 1e-6 and all(abs(a - b) < 1e-6 for a, b in zip(le, lg))
    print("OK" if ok else "MISMATCH")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
