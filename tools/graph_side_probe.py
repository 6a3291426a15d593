"""Which parameters' gradients differ between HIP-graph replays of the forked-stream step?

Runs the swinT224 Trainer (lr = 0: weights fixed, every step computes the same gradient into
the AdamW first moment) eagerly and with the captured step (MSU_GRAPH_SIDE=1: side stream
forked into the graph), twice each, and prints per parameter the max |exp_avg| difference of
each run against the first eager run.  A race in the forked graph shows up as parameters that
differ between the two graph runs.

    MSU_GRAPH_SIDE=1 python tools/graph_side_probe.py [steps]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def run(graph, steps):
    import cases
    from oracle.msunet import make_cfg
    from semantic_segmentation_of_stylegan2_artifacts_amd import load_config
    from semantic_segmentation_of_stylegan2_artifacts_amd.network.model_parts import MSUNetSys
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer
    spec = cases.model_cases()["swinT224"]
    cfg = make_cfg(**spec["cfg"])
    m = MSUNetSys(img_size=224, embed_dim=96, depths=cfg["depths"], num_heads=cfg["num_heads"], drop_path_rate=0.0,
                  attn_drop_rate=0.0, drop_rate=0.0)
    m.load_state_dict(cases.model_params(cfg, spec["seed"]), strict=True)
    m = m.cuda().train()
    x, t = cases.model_inputs(cfg, 2, spec["seed"])
    x, t = x.cuda(), t.cuda()
    tr = Trainer(m, load_config(None, "swin_t", **{"TRAIN.BASE_LR": 0.0}), "cuda", use_graph=graph, graph_warmup=2)
    losses = [tr.step(x, t).item() for _ in range(steps)]
    torch.cuda.synchronize()
    flat = {}
    for g in tr.groups:
        for n, p, off in zip(g.names, g.params, g.offsets):
            flat[n] = g.exp_avg[off:off + p.numel()].clone()
    per = {n: flat[n] for n, _ in m.named_parameters() if n in flat}  # forward (registration) order
    return losses, per, tr._graph is not None


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    print("MSU_GRAPH_SIDE =", os.environ.get("MSU_GRAPH_SIDE", "0"))
    runs = {"eager0": run(False, steps), "eager1": run(False, steps), "graph0": run(True, steps),
            "graph1": run(True, steps)}
    base = runs["eager0"][1]
    for k, (losses, per, cap) in runs.items():
        diffs = sorted(((float((per[n] - base[n]).abs().max()), n) for n in base), reverse=True)
        nz = [d for d in diffs if d[0] > 0]
        print(f"{k}: captured={cap} losses={losses}")
        print(f"   params differing from eager0: {len(nz)} / {len(diffs)}")
        for d, n in nz[:12]:
            print(f"     {d:.3e}  {n}")
    # the divergence point: in forward (registration) order, the LAST parameter that differs
    # between the two eager runs is the first one backward reached with a different gradient
    order = list(runs["eager0"][1].keys())
    e1 = runs["eager1"][1]
    bad = [n for n in order if not torch.equal(e1[n], base[n])]
    print("eager1 vs eager0, differing params in forward order (last = first reached by backward):")
    print("   " + ", ".join(bad))
    g0, g1 = runs["graph0"][1], runs["graph1"][1]
    badg = [n for n in order if not torch.equal(g0[n], g1[n])]
    print("graph1 vs graph0, differing params in forward order (last = first reached by backward):")
    print("   " + ", ".join(badg))
    diffs = sorted(((float((g0[n] - g1[n]).abs().max()), n) for n in g0), reverse=True)
    nz = [d for d in diffs if d[0] > 0]
    print(f"graph0 vs graph1: {len(nz)} params differ")
    for d, n in nz[:20]:
        print(f"     {d:.3e}  {n}")


if __name__ == "__main__":
    main()
