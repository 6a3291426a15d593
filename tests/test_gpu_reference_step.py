"""GPU: the reference's own training step runs UNCHANGED on this package's modules.

The body of ``reference_step`` is the per-batch sequence of the reference trainer, statement
for statement: the AdamW parameter groups of /root/reference/trainer.py:130-152, the
GradScaler of :182 and the step of :299-316 (``torch.amp.autocast('cuda', dtype=torch.float16)``
around forward, loss, ``zero_grad(set_to_none=True)``, ``scaler.scale(loss).backward()``,
``scaler.step(optimizer)``, ``scaler.update()``, then ``loss.item()``).  Only ``MSUNet`` /
``MSUNetSys`` and ``DynamicLoss`` come from this package; under the fp16 autocast every op
runs its f16 HIP kernels (torch.ops.msunet.*, f16 MFMA).

Checks against the fp32 golden fixture of the reference (swinT224: Swin-T widths/heads,
224^2, produced by importing the reference model_parts.py):
* fp16 logits within 1e-2 relative L2 of the golden logits, loss within 1e-2 relative;
* the gradients GradScaler hands to AdamW (unscaled in place by scaler.step) match the golden
  per-parameter gradient norms within 5e-2 relative (+1e-3 of the largest norm);
* the optimizer step happened (parameters moved) and no gradient was non-finite;
* GradScaler's overflow path: with an absurd initial scale the scaled f16 backward overflows,
  the step is skipped (parameters untouched) and the scale is backed off -- as in the
  reference, where GradScaler skips inf steps.
"""
import os

import numpy as np
import pytest
import torch
from torch import optim

pytestmark = pytest.mark.gpu

import cases  # noqa: E402
from oracle.msunet import make_cfg  # noqa: E402


def _model():
    from semantic_segmentation_of_stylegan2_artifacts_amd.network.model_parts import MSUNetSys
    spec = cases.model_cases()["swinT224"]
    cfg = make_cfg(**spec["cfg"])
    m = MSUNetSys(img_size=cfg["img_size"], patch_size=cfg["patch_size"], in_chans=cfg["in_chans"],
                  num_classes=cfg["num_classes"], embed_dim=cfg["embed_dim"], depths=cfg["depths"],
                  num_heads=cfg["num_heads"], window_size=cfg["window_size"], mlp_ratio=cfg["mlp_ratio"],
                  drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.0)
    m.load_state_dict(cases.model_params(cfg, spec["seed"]), strict=True)
    x, t = cases.model_inputs(cfg, spec["batch"], spec["seed"])
    return m, x, t


def make_optimizer(model, base_lr, weight_decay, betas, eps):
    """trainer.py:130-152 (decay split of :137)."""
    decay_params = []
    no_decay_params = []
    for name, param in model.named_parameters():
        if not param.requires_grad:
            continue
        if param.ndim == 1 or name.endswith(".bias") or "norm" in name.lower():
            no_decay_params.append(param)
        else:
            decay_params.append(param)
    return optim.AdamW([{"params": decay_params, "weight_decay": weight_decay},
                        {"params": no_decay_params, "weight_decay": 0.0}],
                       lr=base_lr, betas=betas, eps=eps, amsgrad=False)


def reference_step(model, dynamic_loss, optimizer, scaler, image_batch, label_batch, device, probe):
    """trainer.py:299-319, unchanged (probe: records what the test inspects)."""
    image_batch = image_batch.to(device)
    label_batch = label_batch.to(device)
    with torch.amp.autocast('cuda', dtype=torch.float16):
        outputs = model(image_batch)  # prediction
        loss = dynamic_loss(outputs, label_batch)  # loss
        optimizer.zero_grad(set_to_none=True)
        scaler.scale(loss).backward()
        probe(model, outputs, loss, scaler)
        scaler.step(optimizer)
        scaler.update()
    return loss.item()


def test_reference_fp16_autocast_gradscaler_step(golden_dir):
    from semantic_segmentation_of_stylegan2_artifacts_amd.loss import DynamicLoss
    z = np.load(os.path.join(golden_dir, "msunet_swinT224.npz"))
    model, x, t = _model()
    model = model.cuda().train()
    dynamic_loss = DynamicLoss(alpha=0.2, beta=0.8, tversky_bce_mix=0.45)
    optimizer = make_optimizer(model, 1e-4, 1e-3, (0.9, 0.999), 1e-8)
    scaler = torch.amp.GradScaler('cuda')
    before = {k: p.detach().clone() for k, p in model.named_parameters()}
    seen = {}

    def probe(m, outputs, loss, sc):
        seen["logits"] = outputs.detach().float().cpu()
        seen["loss"] = loss.item()
        s = sc.get_scale()
        seen["grads"] = {k: (p.grad.float() / s).cpu() for k, p in m.named_parameters() if p.grad is not None}
        seen["scale"] = s

    loss_val = reference_step(model, dynamic_loss, optimizer, scaler, x, t, "cuda", probe)
    ref = torch.from_numpy(z["logits"])
    rel = ((seen["logits"] - ref).norm() / ref.norm()).item()
    assert rel < 1e-2, rel
    assert abs(loss_val - float(z["loss"])) <= 1e-2 * abs(float(z["loss"])), (loss_val, float(z["loss"]))
    g = seen["grads"]
    assert all(torch.isfinite(v).all() for v in g.values()), "non-finite gradient at the default scale"
    norms = dict(zip(list(z["grad_names"]), z["grad_norm"]))
    gmax = max(norms.values())
    assert set(g) == set(norms)
    for k, n in norms.items():
        gn = g[k].norm().item()
        assert abs(gn - n) <= 5e-2 * n + 1e-3 * gmax, (k, gn, n)
    moved = sum(not torch.equal(before[k], p.detach()) for k, p in model.named_parameters() if k in norms)
    assert moved == len(norms)
    assert scaler.get_scale() == seen["scale"]  # no overflow: scale unchanged after one step


def test_reference_gradscaler_skips_overflowing_f16_step():
    from semantic_segmentation_of_stylegan2_artifacts_amd.loss import DynamicLoss
    model, x, t = _model()
    model = model.cuda().train()
    dynamic_loss = DynamicLoss(alpha=0.2, beta=0.8, tversky_bce_mix=0.45)
    optimizer = make_optimizer(model, 1e-4, 1e-3, (0.9, 0.999), 1e-8)
    scaler = torch.amp.GradScaler('cuda', init_scale=2.0 ** 40)
    before = {k: p.detach().clone() for k, p in model.named_parameters()}
    seen = {}

    def probe(m, outputs, loss, sc):
        seen["nonfinite"] = any(not torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)

    reference_step(model, dynamic_loss, optimizer, scaler, x, t, "cuda", probe)
    assert seen["nonfinite"], "the 2^40-scaled f16 backward should overflow"
    for k, p in model.named_parameters():
        assert torch.equal(before[k], p.detach()), k
    assert scaler.get_scale() < 2.0 ** 40
