"""GPU end-to-end parity: the HIP MS-UNet (fp32 activations) against the golden vectors
produced by the REFERENCE model_parts.py (torchvision block restated, see oracle/) and the
reference DynamicLoss.  Tolerance: 1e-3 relative on logits (north star), loss 1e-4,
per-parameter gradient norms 1e-3 relative."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import cases  # noqa: E402
from oracle.msunet import make_cfg, msunet_forward  # noqa: E402
from oracle.dynamic_loss import dynamic_loss as oracle_loss  # noqa: E402

DEV = "cuda"


def _build(cfg):
    from semantic_segmentation_of_stylegan2_artifacts_amd.network.model_parts import MSUNetSys
    return MSUNetSys(img_size=cfg["img_size"], patch_size=cfg["patch_size"], in_chans=cfg["in_chans"],
                     num_classes=cfg["num_classes"], embed_dim=cfg["embed_dim"], depths=cfg["depths"],
                     num_heads=cfg["num_heads"], window_size=cfg["window_size"], mlp_ratio=cfg["mlp_ratio"],
                     drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=cfg["drop_path_rate"])


@pytest.mark.parametrize("case", list(cases.model_cases().keys()))
def test_msunet_fp32_matches_reference_golden(golden_dir, case):
    from semantic_segmentation_of_stylegan2_artifacts_amd.loss import DynamicLoss
    z = np.load(os.path.join(golden_dir, f"msunet_{case}.npz"))
    spec = cases.model_cases()[case]
    cfg = make_cfg(**spec["cfg"])
    model = _build(cfg)
    model.load_state_dict(cases.model_params(cfg, spec["seed"]), strict=True)
    model = model.to(DEV).train()
    x, target = cases.model_inputs(cfg, spec["batch"], spec["seed"])
    logits = model(x.to(DEV))
    ref = torch.from_numpy(z["logits"])
    err = (logits.detach().cpu() - ref).abs().max().item()
    assert err <= 1e-3 * ref.abs().max().item(), err
    loss = DynamicLoss(alpha=0.2, beta=0.8, tversky_bce_mix=0.45)(logits, target.to(DEV))
    assert abs(loss.item() - float(z["loss"])) <= 1e-4 * max(1.0, abs(float(z["loss"])))
    loss.backward()
    params = dict(model.named_parameters())
    for k, n in zip(list(z["grad_names"]), z["grad_norm"]):
        g = params[k].grad
        assert g is not None, k
        assert abs(g.norm().item() - n) <= 2e-3 * abs(n) + 1e-6, (k, g.norm().item(), n)
    for k in z["no_grad_names"]:
        assert params[k].grad is None, k
    for k in cases.FULL_GRAD_KEYS:
        gr = torch.from_numpy(z["grad." + k])
        e = (params[k].grad.cpu() - gr).abs().max().item()
        assert e <= 2e-3 * gr.abs().max().item() + 1e-7, (k, e)


def test_msunet_bf16_close_to_fp32():
    """bf16 autocast training forward stays close to the fp32 oracle (Dice-level check)."""
    spec = cases.model_cases()["swinT224"]
    cfg = make_cfg(**spec["cfg"])
    params = cases.model_params(cfg, spec["seed"])
    model = _build(cfg)
    model.load_state_dict(params, strict=True)
    model = model.to(DEV).train()
    x, target = cases.model_inputs(cfg, spec["batch"], spec["seed"])
    ref = msunet_forward(params, cfg, x).detach()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = model(x.to(DEV)).float().cpu()
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < 5e-2, rel
    # Dice of the binarised predictions agree
    pb, rb = torch.sigmoid(out) > 0.5, torch.sigmoid(ref) > 0.5
    agree = (pb == rb).float().mean().item()
    assert agree > 0.98, agree


def test_msunet_input_channel_check():
    from semantic_segmentation_of_stylegan2_artifacts_amd.network import MSUNet
    from semantic_segmentation_of_stylegan2_artifacts_amd import load_config
    cfg = load_config(None, "swin_t")
    m = MSUNet(cfg, img_size=224).to(DEV)
    with pytest.raises(ValueError):
        m(torch.zeros(1, 4, 224, 224, device=DEV))


def test_side_stream_paths_are_exact():
    """The discarded branches on the side stream change nothing (same logits with them
    skipped), and the gradients with the side stream equal the single-stream ones (same
    kernels; only the qkv bias sums its two shares in the other order: f32 rounding)."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import FlatGroup
    spec = cases.model_cases()["swinT224"]
    cfg = make_cfg(**spec["cfg"])
    params = cases.model_params(cfg, spec["seed"])
    x, target = cases.model_inputs(cfg, spec["batch"], spec["seed"])
    grads = {}
    for side in (True, False):
        model = _build(cfg)
        model.load_state_dict(params, strict=True)
        model = model.to(DEV).train()
        named = [(n, p) for n, p in model.named_parameters()
                 if not any(p is q for m in model.dead_modules() for q in m.parameters())]
        grp = FlatGroup(named, 0.0, torch.device(DEV))
        old = ops._side_enabled
        ops._side_enabled = side
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(x.to(DEV))
                model.skip_dead_branches = True
                out_skip = model(x.to(DEV))
                model.skip_dead_branches = False
            assert torch.equal(out, out_skip)
            out.float().square().mean().backward()
            torch.cuda.synchronize()
        finally:
            ops._side_enabled = old
        grads[side] = grp.grad.clone()
    torch.testing.assert_close(grads[True], grads[False], rtol=1e-6, atol=1e-9)
