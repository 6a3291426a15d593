"""Run-to-run determinism of the eager training step under switches, in one process.

For each configuration (weight-gradient side stream on / off, GEMM route default / lib, conv
kernel v3 / v2 is a build-time env and not switched here) run the swinT224 Trainer N times from
the same weights (lr = 0: every step computes the same gradient into the AdamW moments) and
count the distinct final moment vectors; list the parameters that differ between runs.

    python tools/determinism_matrix.py [runs]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def run(steps=3, skip_dead=False):
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
    m.skip_dead_branches = skip_dead
    x, t = cases.model_inputs(cfg, 2, spec["seed"])
    x, t = x.cuda(), t.cuda()
    tr = Trainer(m, load_config(None, "swin_t", **{"TRAIN.BASE_LR": 0.0}), "cuda", use_graph=False)
    for _ in range(steps):
        tr.step(x, t)
    torch.cuda.synchronize()
    per = {}
    for g in tr.groups:
        for n, p, off in zip(g.names, g.params, g.offsets):
            per[n] = g.exp_avg[off:off + p.numel()].clone()
    return per


def configs():
    # (label, side stream, GEMM route, dead branches skipped, wgrad on side, attention tail on side)
    if len(sys.argv) > 2 and sys.argv[2] == "default":  # the default eager step only
        return [("side, all parts", True, "", False, True, True)]
    if len(sys.argv) > 2 and sys.argv[2] == "parts":
        return [("side, all parts", True, "", False, True, True),
                ("side, no dead branches", True, "", True, True, True),
                ("side, wgrad on main", True, "", False, False, True),
                ("side, attention tail on main", True, "", False, True, False),
                ("side, only dead branches", True, "", False, False, False)]
    return [(f"side={side} route={route or 'default'}", side, route, False, True, True)
            for side in (True, False) for route in ("", "lib")]


def main():
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    for label, side, route, skip_dead, wg, tail in configs():
        if True:
            ops._side_enabled = side
            ops._ROUTE_FORCE = route
            ops._side_wgrad = wg
            ops._side_attn_tail = tail
            ops._tok_cache.clear()
            res = [run(skip_dead=skip_dead) for _ in range(runs)]
            base = res[0]
            ndiff = [sum(1 for n in base if not torch.equal(r[n], base[n])) for r in res[1:]]
            print(f"{label}: params differing from run 0: {ndiff}", flush=True)
            for k, r in enumerate(res[1:]):
                d = sorted(((float((r[n] - base[n]).abs().max()), n) for n in base), reverse=True)
                d = [e for e in d if e[0] > 0]
                if d:
                    print(f"   run {k + 1}: " + ", ".join(f"{n} {v:.1e}" for v, n in sorted(d, key=lambda e: e[1])),
                          flush=True)


if __name__ == "__main__":
    main()
