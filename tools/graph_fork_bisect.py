"""Bisect the run-to-run difference of the forked-stream HIP-graph step by side-stream use.

The step forks three kinds of work onto the side stream: Linear weight gradients
(ops._side_wgrad), the attention parameter-gradient tail (ops._side_attn_tail) and the
discarded reference branches (MSUNetSys.skip_dead_branches).  For each combination this
captures the swinT224 step with the side stream forked into the graph (MSU_GRAPH_SIDE=1),
twice, with lr = 0, and prints how many parameters' AdamW moments differ between the two
captures and the first parameter backward reached with a different gradient.

    python tools/graph_fork_bisect.py [steps]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

MODES = {  # name: (weight gradients, attention tail, dead branches) on the side stream
    "all": (True, True, True),
    "wgrad_only": (True, False, False),
    "tail_only": (False, True, False),
    "dead_only": (False, False, True),
    "wgrad_tail": (True, True, False),
}


def run(mode, steps):
    import cases
    from oracle.msunet import make_cfg
    from semantic_segmentation_of_stylegan2_artifacts_amd import load_config, ops
    from semantic_segmentation_of_stylegan2_artifacts_amd.network.model_parts import MSUNetSys
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer
    wg, tail, dead = MODES[mode]
    ops._side_wgrad, ops._side_attn_tail = wg, tail
    spec = cases.model_cases()["swinT224"]
    cfg = make_cfg(**spec["cfg"])
    m = MSUNetSys(img_size=224, embed_dim=96, depths=cfg["depths"], num_heads=cfg["num_heads"], drop_path_rate=0.0,
                  attn_drop_rate=0.0, drop_rate=0.0)
    m.load_state_dict(cases.model_params(cfg, spec["seed"]), strict=True)
    m.skip_dead_branches = not dead
    m = m.cuda().train()
    x, t = cases.model_inputs(cfg, 2, spec["seed"])
    x, t = x.cuda(), t.cuda()
    tr = Trainer(m, load_config(None, "swin_t", **{"TRAIN.BASE_LR": 0.0}), "cuda", use_graph=True, graph_warmup=2)
    for _ in range(steps):
        tr.step(x, t)
    torch.cuda.synchronize()
    assert tr._graph is not None
    per = {}
    for g in tr.groups:
        for n, p, off in zip(g.names, g.params, g.offsets):
            per[n] = g.exp_avg[off:off + p.numel()].clone()
    return {n: per[n] for n, _ in m.named_parameters() if n in per}


def main():
    os.environ["MSU_GRAPH_SIDE"] = "1"
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else list(MODES)
    for mode in modes:
        t0 = time.time()
        a, b = run(mode, steps), run(mode, steps)
        order = list(a.keys())
        bad = [n for n in order if not torch.equal(a[n], b[n])]
        mx = max((float((a[n] - b[n]).abs().max()) for n in bad), default=0.0)
        print(f"{mode}: {len(bad)} / {len(order)} params differ (max {mx:.2e}); first reached by backward: "
              f"{bad[-1] if bad else '-'}  [{time.time() - t0:.0f} s]", flush=True)


if __name__ == "__main__":
    main()
