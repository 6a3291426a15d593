"""GPU: the trainer's fast paths change nothing numerically.

trainer.FlatGroup re-homes parameters into flat buffers, marks them for direct gradient
accumulation (the backward kernels add into the preallocated .grad views instead of
returning a gradient for AccumulateGrad) and keeps a per-step bf16 shadow that the Linear
ops read instead of casting.  A bf16 forward+backward through the Trainer must give the
same parameter gradients as the plain autograd path on an identical model, and one
Trainer.step must equal torch.optim.AdamW (the reference's optimizer, trainer.py:130-152)
applied to those gradients."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

import cases  # noqa: E402
from oracle.msunet import make_cfg  # noqa: E402

DEV = "cuda"


def _setup():
    from semantic_segmentation_of_stylegan2_artifacts_amd import load_config
    from semantic_segmentation_of_stylegan2_artifacts_amd.network.model_parts import MSUNetSys
    spec = cases.model_cases()["swinT224"]
    cfg = make_cfg(**spec["cfg"])
    model = MSUNetSys(img_size=cfg["img_size"], patch_size=cfg["patch_size"], in_chans=cfg["in_chans"],
                      num_classes=cfg["num_classes"], embed_dim=cfg["embed_dim"], depths=cfg["depths"],
                      num_heads=cfg["num_heads"], window_size=cfg["window_size"], mlp_ratio=cfg["mlp_ratio"],
                      drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.0)
    model.load_state_dict(cases.model_params(cfg, spec["seed"]), strict=True)
    x, target = cases.model_inputs(cfg, 2, spec["seed"])
    conf = load_config(None, "swin_t", **{"TRAIN.BASE_LR": 1e-3})
    return model.to(DEV).train(), x.to(DEV), target.to(DEV), conf


def test_direct_grads_and_shadow_match_autograd():
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer
    model, x, target, conf = _setup()
    ref = copy.deepcopy(model)
    tr = Trainer(model, conf, DEV)
    for g in tr.groups:
        g.refresh_shadow()
    loss = tr.forward_loss(x, target)
    loss.backward()
    loss_ref = tr.loss_fn
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lr = loss_ref(ref(x), target)
    lr.backward()
    assert torch.equal(loss.detach(), lr.detach())
    rp = dict(ref.named_parameters())
    n_checked = 0
    for g in tr.groups:
        for name, p in zip(g.names, g.params):
            gr = rp[name].grad
            assert gr is not None, name
            torch.testing.assert_close(p.grad, gr, rtol=1e-6, atol=1e-7, msg=name)
            n_checked += 1
    assert n_checked == sum(len(g.params) for g in tr.groups)


def test_dead_branch_parameters_get_static_shadows():
    """The dead central-decoder branches' weights (never updated) get one 16-bit shadow at
    Trainer construction: ops._shadow returns it (no per-step cast), equal to the cast; a write
    through the parameter makes it stale (the op casts again)."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer
    model, x, target, conf = _setup()
    Trainer(model, conf, DEV)
    dead = [p for m in model.dead_modules() for p in m.parameters() if p.dim() >= 2]
    assert dead
    for p in dead:
        sh = ops._shadow(p, torch.bfloat16)
        assert sh is p._msu_shadow
        assert torch.equal(sh, p.detach().to(torch.bfloat16))
    with torch.no_grad():
        dead[0].mul_(2)
    assert ops._shadow(dead[0], torch.bfloat16) is not dead[0]._msu_shadow
    assert torch.equal(ops._shadow(dead[0], torch.bfloat16), dead[0].detach().to(torch.bfloat16))


def test_trainer_step_equals_torch_adamw():
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer, is_no_decay
    model, x, target, conf = _setup()
    ref = copy.deepcopy(model)
    tr = Trainer(model, conf, DEV)
    tr.step(x, target)
    # reference: same gradients through plain autograd, then torch AdamW with the two groups
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = tr.loss_fn(ref(x), target)
    loss.backward()
    live = {n for g in tr.groups for n in g.names}
    decay = [p for n, p in ref.named_parameters() if n in live and not is_no_decay(n, p)]
    nodecay = [p for n, p in ref.named_parameters() if n in live and is_no_decay(n, p)]
    opt = torch.optim.AdamW([{"params": decay, "weight_decay": conf.TRAIN.WEIGHT_DECAY},
                             {"params": nodecay, "weight_decay": 0.0}], lr=tr.lr,
                            betas=tuple(conf.TRAIN.OPTIMIZER.BETAS), eps=conf.TRAIN.OPTIMIZER.EPS)
    opt.step()
    rp = dict(ref.named_parameters())
    for g in tr.groups:
        for name, p in zip(g.names, g.params):
            torch.testing.assert_close(p.detach(), rp[name].detach(), rtol=1e-5, atol=1e-6, msg=name)
    # the shadow follows the update; a write through the parameter invalidates it
    p0 = tr.groups[0].params[0]
    assert torch.equal(p0._msu_shadow, p0.detach().to(torch.bfloat16))
    with torch.no_grad():
        p0.mul_(2.0)
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    assert ops._shadow(p0, torch.bfloat16) is not p0._msu_shadow


def test_nonfinite_gradient_skips_the_step():
    """GradScaler semantics (reference trainer.py:182, 315-316): a step whose gradients hold an
    inf / NaN changes neither the parameters nor the AdamW moments, and is not counted as an
    optimizer step (bias correction of the next step uses step 2, not 3)."""
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer
    model, x, target, conf = _setup()
    ref = copy.deepcopy(model)
    tr = Trainer(model, conf, DEV, use_graph=False)  # swaps loss_fn between steps (eager semantics)
    tr.step(x, target)
    snap = [(g.data.clone(), g.exp_avg.clone(), g.exp_avg_sq.clone()) for g in tr.groups]
    bad = x.clone()
    bad[0, 0, 5, 7] = float("nan")  # -> NaN logits -> NaN gradients everywhere
    loss = tr.step(bad, target)
    torch.cuda.synchronize()
    assert not torch.isfinite(loss).item()
    assert tr.found_inf.item() == 1.0
    for g, (d, m, v) in zip(tr.groups, snap):
        assert torch.equal(g.data, d)
        assert torch.equal(g.exp_avg, m)
        assert torch.equal(g.exp_avg_sq, v)
        assert not g.grad.any()  # zeroed for the next step
    assert tr.optimizer_steps() == 1
    # a gradient that is finite everywhere but one parameter: still skipped
    snap = [g.data.clone() for g in tr.groups]
    orig = tr.loss_fn

    class _Poison(torch.nn.Module):
        def forward(self, out, lab):
            loss = orig(out, lab)
            p = tr.groups[0].params[3]
            return loss + (p * float("inf")).sum() * 0.0  # d/dp = NaN for this parameter only

    tr.loss_fn = _Poison()
    tr.step(x, target)
    tr.loss_fn = orig
    torch.cuda.synchronize()
    for g, d in zip(tr.groups, snap):
        assert torch.equal(g.data, d)
    assert tr.optimizer_steps() == 1
    tr.step(x, target)
    assert tr.optimizer_steps() == 2


def test_nonfinite_input_skips_replayed_step():
    """The same GradScaler rule inside the HIP-graph replay: a NaN image in the replayed
    step's input buffer skips the captured AdamW, a finite one applies it."""
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer
    model, x, target, conf = _setup()
    tr = Trainer(model, conf, DEV, use_graph=True, graph_warmup=2)
    for _ in range(3):
        tr.step(x, target)
    assert tr._graph is not None and tr.optimizer_steps() == 3
    snap = [g.data.clone() for g in tr.groups]
    bad = x.clone()
    bad[0, 1, 3, 3] = float("inf")
    tr.step(bad, target)
    torch.cuda.synchronize()
    assert tr.found_inf.item() == 1.0 and tr.optimizer_steps() == 3
    for g, d in zip(tr.groups, snap):
        assert torch.equal(g.data, d)
    tr.step(x, target)
    assert tr.optimizer_steps() == 4
    assert not torch.equal(tr.groups[0].data, snap[0])


def test_adamw_dev_skip_matches_torch_adamw():
    """The device-hyper AdamW (lr / step read on the GPU) over three steps, the middle one
    flagged non-finite, equals torch.optim.AdamW run on the two finite steps only (the skipped
    step neither updates nor advances the bias-correction step)."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    g = torch.Generator().manual_seed(7)
    n = 10007
    p0 = torch.randn(n, generator=g)
    grads = [torch.randn(n, generator=g) * s for s in (1.0, 3.0, 0.5)]
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=1e-2, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.05)
    for k in (0, 2):
        ref.grad = grads[k].clone()
        opt.step()
    p = p0.to(DEV)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    hyper = torch.tensor([1e-2, 0.0], device=DEV, dtype=torch.float64)
    found = torch.zeros(1, device=DEV)
    for k in range(3):
        gd = grads[k].to(DEV)
        if k == 1:
            gd[17] = float("inf")
        found.zero_()
        ops.nonfinite_(gd, found)
        ops.step_advance_(hyper, found)
        ops.adamw_dev_(p, gd, m, v, hyper, 0.9, 0.999, 1e-8, 0.05, found_inf=found)
    assert hyper[1].item() == 2.0
    # same scalars and operation order as torch: a few ulp at most (CPU vs GPU rounding)
    torch.testing.assert_close(p.cpu(), ref.detach(), rtol=4e-7, atol=1e-8)
    torch.testing.assert_close(m.cpu(), opt.state[ref]["exp_avg"], rtol=4e-7, atol=2e-8)
    torch.testing.assert_close(v.cpu(), opt.state[ref]["exp_avg_sq"], rtol=4e-7, atol=1e-12)


@pytest.mark.parametrize("sdt", [torch.bfloat16, torch.float16, None], ids=["bf16", "f16", "noshadow"])
def test_adamw_dev2_equals_adamw_zero_and_cast(sdt):
    """msu_adamw_dev2 (the trainer's optimizer pass): bitwise msu_adamw_dev, then the gradient
    zeroed and the 16-bit shadow cast from the updated parameters -- the three launches it
    replaces; a skipped step (found_inf) still zeroes the gradient and leaves parameters and
    shadow as they were."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    g = torch.Generator().manual_seed(3)
    n = 100003
    p0 = torch.randn(n, generator=g).to(DEV)
    m0, v0 = (0.1 * torch.randn(n, generator=g)).to(DEV), torch.rand(n, generator=g).to(DEV)
    g0 = torch.randn(n, generator=g).to(DEV)
    for skip in (False, True):
        hyper = torch.tensor([1e-3, 5.0], device=DEV, dtype=torch.float64)
        found = torch.tensor([1.0 if skip else 0.0], device=DEV)
        pa, ma, va, ga = p0.clone(), m0.clone(), v0.clone(), g0.clone()
        ops.adamw_dev_(pa, ga, ma, va, hyper, 0.9, 0.999, 1e-8, 0.05, found_inf=found)
        pb, mb, vb, gb = p0.clone(), m0.clone(), v0.clone(), g0.clone()
        sh = p0.to(sdt) if sdt is not None else None
        ops.adamw_dev_(pb, gb, mb, vb, hyper, 0.9, 0.999, 1e-8, 0.05, found_inf=found, shadow=sh, zero_grad=True)
        torch.cuda.synchronize()
        assert torch.equal(pa, pb) and torch.equal(ma, mb) and torch.equal(va, vb)
        assert torch.count_nonzero(gb).item() == 0
        if sdt is not None:
            assert torch.equal(sh, pb.to(sdt))
