"""GPU: the trainer's transposed bf16 weight shadow (msu_transpose16_multi).

The Linear input gradients dX = dY . W (the backward of model_parts.py:143-151's Linears,
the fused MLP, the skip fusions and PatchMerging's reduction) read W^T from a per-step
transposed shadow written by one batched transpose after AdamW, so both hand-written GEMMs
run their forward layout.  Checked here:

* the batched transpose itself over ragged shapes (partial 64 x 64 tiles, N != K, tiny and
  wide entries) is bitwise the transpose;
* inside the trainer the shadow equals the transpose of the bf16 shadow after every step;
* the training step with the transposed shadow computes the same step as without it (the
  NT GEMM's KN variant / per-call W^T copies): AdamW moments within bf16 rounding.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

import cases  # noqa: E402
from oracle.msunet import make_cfg  # noqa: E402

DEV = "cuda"


def test_transpose16_multi_ragged():
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    shapes = [(96, 288), (288, 96), (576, 192), (8, 8), (72, 136), (768, 3072), (200, 64)]
    g = torch.Generator(device="cpu").manual_seed(3)
    tab, srcs, soff, doff, tiles = [], [], 0, 0, 0
    for N, K in shapes:
        tab.append((soff, doff, N, K, tiles))
        srcs.append(torch.randn(N, K, generator=g))
        soff += N * K + 8  # gaps between entries stay untouched
        doff += N * K + 16
        tiles += -(-N // 64) * -(-K // 64)
    src = torch.zeros(soff, dtype=torch.bfloat16)
    for (so, _, N, K, _), s in zip(tab, srcs):
        src[so:so + N * K] = s.reshape(-1).to(torch.bfloat16)
    src = src.to(DEV)
    dst = torch.full((doff,), 7.0, device=DEV, dtype=torch.bfloat16)
    table = torch.tensor(tab, dtype=torch.int64).to(DEV)
    ops.transpose16_multi(src, dst, table, tiles)
    torch.cuda.synchronize()
    for (so, do, N, K, _), s in zip(tab, srcs):
        want = src[so:so + N * K].view(N, K).t()
        assert torch.equal(dst[do:do + N * K].view(K, N), want), (N, K)
        assert torch.all(dst[do + N * K:do + N * K + 16] == 7.0)


def _run(shadow_t, steps=3, lr=0.0):
    from semantic_segmentation_of_stylegan2_artifacts_amd import load_config, ops
    from semantic_segmentation_of_stylegan2_artifacts_amd.network.model_parts import MSUNetSys
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer
    prev = ops._SHADOW_T
    ops._SHADOW_T = shadow_t
    try:
        spec = cases.model_cases()["swinT224"]
        cfg = make_cfg(**spec["cfg"])
        m = MSUNetSys(img_size=cfg["img_size"], embed_dim=cfg["embed_dim"], depths=cfg["depths"],
                      num_heads=cfg["num_heads"], drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.0)
        m.load_state_dict(cases.model_params(cfg, spec["seed"]), strict=True)
        m = m.to(DEV).train()
        x, t = cases.model_inputs(cfg, 2, spec["seed"])
        x, t = x.to(DEV), t.to(DEV)
        tr = Trainer(m, load_config(None, "swin_t", **{"TRAIN.BASE_LR": lr}), DEV, use_graph=False)
        losses = [tr.step(x, t).item() for _ in range(steps)]
        torch.cuda.synchronize()
        if shadow_t:
            n = 0
            for g in tr.groups:
                for p in g.params:
                    st = getattr(p, "_msu_shadow_t", None)
                    if st is not None:
                        assert torch.equal(st, p._msu_shadow.t()), "stale transposed shadow"
                        n += 1
            assert n > 50
        moments = {n: g.exp_avg[o:o + p.numel()].clone()
                   for g in tr.groups for n, p, o in zip(g.names, g.params, g.offsets)}
        return losses, moments
    finally:
        ops._SHADOW_T = prev


def test_transposed_shadow_step_matches():
    la, ma = _run(True)
    lb, mb = _run(False)
    assert la == pytest.approx(lb, rel=1e-5)
    for n in ma:
        a, b = ma[n], mb[n]
        den = b.norm().item()
        if den == 0:
            assert a.norm().item() == 0, n
            continue
        assert (a - b).norm().item() <= 2e-2 * den, n


def test_transposed_shadow_follows_weight_updates():
    """lr > 0: the shadow is re-transposed after every AdamW (checked inside _run)."""
    _run(True, steps=3, lr=1e-3)
