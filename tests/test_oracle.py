"""CPU: the oracle against the golden vectors produced by the reference code itself."""
import json
import os

import numpy as np
import pytest
import torch

import cases
from oracle import dynamic_loss as odl
from oracle.msunet import make_cfg, msunet_forward, param_spec, dead_prefixes, SWIN_B


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


@pytest.mark.parametrize("case", list(cases.loss_cases().keys()))
def test_dynamic_loss_matches_reference(golden_dir, case):
    z = _load(golden_dir, "dynamic_loss.npz")
    logits, target, kw = cases.loss_cases()[case]
    x = logits.clone().requires_grad_(True)
    loss = odl.dynamic_loss(x, target, **kw)
    loss.backward()
    assert abs(loss.item() - float(z[f"{case}.loss"])) <= 1e-6 * max(1.0, abs(float(z[f"{case}.loss"])))
    np.testing.assert_allclose(x.grad.numpy(), z[f"{case}.grad"], rtol=1e-5, atol=1e-9)
    # closed-form gradient (what the HIP backward implements) == autograd of the reference
    g = odl.dynamic_loss_grad(logits, target, **kw)
    np.testing.assert_allclose(g.numpy(), z[f"{case}.grad"], rtol=1e-4, atol=1e-9)


def test_dynamic_loss_batch_mismatch_raises():
    with pytest.raises(ValueError):
        odl.dynamic_loss(torch.zeros(2, 1, 4, 4), torch.zeros(3, 4, 4))


def test_state_dict_contract(golden_dir):
    """Our param_spec == the reference MSUNetSys.state_dict() (Swin-B @1024) key/shape list,
    and == the encoder part dumped in network/pretrained_weights/structure_of_MSUNet.txt."""
    with open(os.path.join(golden_dir, "state_dict_swin_b_1024.json")) as f:
        ref = json.load(f)
    cfg = make_cfg(img_size=1024, **SWIN_B)
    ours = [[k, list(s)] for k, s in param_spec(cfg)]
    assert [r[:2] for r in ref] == ours
    with open(os.path.join(golden_dir, "structure_of_MSUNet.json")) as f:
        dump = json.load(f)
    ours_prefixed = {"ms_unet." + k: s for k, s in ours}
    for key, shape in dump:
        assert ours_prefixed[key] == shape, key


@pytest.mark.parametrize("case", list(cases.model_cases().keys()))
def test_msunet_forward_backward_matches_reference(golden_dir, case):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    z = _load(golden_dir, f"msunet_{case}.npz")
    spec = cases.model_cases()[case]
    cfg = make_cfg(**spec["cfg"])
    params = cases.model_params(cfg, spec["seed"])
    for k, v in params.items():
        if v.is_floating_point():
            v.requires_grad_(True)
    x, target = cases.model_inputs(cfg, spec["batch"], spec["seed"])
    logits = msunet_forward(params, cfg, x)
    np.testing.assert_allclose(logits.detach().numpy(), z["logits"], rtol=1e-4, atol=1e-5)
    loss = odl.dynamic_loss(logits, target, 0.2, 0.8, 0.45)
    assert abs(loss.item() - float(z["loss"])) < 1e-5
    loss.backward()
    names = list(z["grad_names"])
    for k, n, s in zip(names, z["grad_norm"], z["grad_sum"]):
        g = params[k].grad
        assert g is not None, k
        assert abs(float(g.norm()) - n) <= 1e-3 * abs(n) + 1e-7, k
    dead = tuple(dead_prefixes(cfg))
    for k in z["no_grad_names"]:
        assert k.startswith(dead), k
        assert params[k].grad is None, k
    for k in cases.FULL_GRAD_KEYS:
        np.testing.assert_allclose(params[k].grad.numpy(), z["grad." + k], rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("case", list(cases.op_cases().keys()))
def test_oracle_ops_match_reference(golden_dir, case):
    from oracle import msunet as om
    z = _load(golden_dir, "ops_reference.npz")
    kind, args, x = cases.op_cases()[case]
    sd = cases.op_params(kind, args)
    p = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    xi = x.clone().requires_grad_(True)
    if kind == "merge":
        y = om.patch_merging(p, "", xi, args["res"])
    elif kind == "expand":
        y = om.patch_expand(p, "", xi, args["res"])
    else:
        y = om.final_expand_x4(p, "", xi, args["res"], args["dim"])
    np.testing.assert_allclose(y.detach().numpy(), z[f"{case}.y"], rtol=1e-5, atol=1e-5)
    y.backward(cases.op_upstream(y))
    np.testing.assert_allclose(xi.grad.numpy(), z[f"{case}.dx"], rtol=1e-4, atol=1e-5)
    for k, v in p.items():
        np.testing.assert_allclose(v.grad.numpy(), z[f"{case}.d.{k}"], rtol=1e-4, atol=1e-4)
