"""GPU: parameter gradients written straight into trainer-style ``.grad`` (direct parameters) equal
the plain autograd gradients bitwise -- the same partials summed in the same order:

* the LayerNorm parameter gradients accumulated into ``.grad`` by the backward's reduction (or, deferred,
  by the batched reduction at the end of backward: to f32 rounding), for
  the four LayerNorm forms of the path (torchvision block norms, the fused residual + norm,
  PatchMerging's gather + norm, PatchExpand's rearrange + norm; model_parts.py:87-94, :403-405);
* the refine convs' weight / bias gradients added into ``.grad`` on the side stream
  (ops._conv_wgrad_param; model_parts.py:447-448, :468-471)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ops():
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    return ops


def _params(C, seed, direct):
    g = torch.Generator().manual_seed(seed)
    w = torch.nn.Parameter((1 + 0.1 * torch.randn(C, generator=g)).to(DEV))
    b = torch.nn.Parameter((0.1 * torch.randn(C, generator=g)).to(DEV))
    if direct:
        flat = torch.zeros(2 * C, device=DEV)  # contiguous [dgamma | dbeta], like the trainer's
        w.grad = flat[:C]
        b.grad = flat[C:]
        w._msu_direct = b._msu_direct = True
    return w, b


@pytest.mark.parametrize("defer", [False, True], ids=["tail", "deferred"])
@pytest.mark.parametrize("form", ["plain", "add", "merge", "d2s"])
def test_ln_param_grads_direct_equal_autograd(form, defer, monkeypatch):
    """In-kernel tail reduction: bitwise the autograd gradients.  Deferred (MSU_LN_DEFER: the
    partials summed by a batched reduction at the end of backward, another fixed order): to f32
    rounding; dx bitwise either way."""
    ops = _ops()
    monkeypatch.setattr(ops, "_LN_DEFER", defer)
    batches = ops.ln_batches
    g = torch.Generator().manual_seed(3)
    B, H, W, C = 2, 32, 32, 96
    x = torch.randn(B, H, W, C, generator=g).to(DEV, torch.bfloat16)
    br = torch.randn(B, H, W, C, generator=g).to(DEV, torch.bfloat16)
    res = {}
    for direct in (False, True):
        Cn = 4 * C if form == "merge" else (C // 4 if form == "d2s" else C)
        w, b = _params(Cn, 9, direct)
        xg = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if form == "plain":
                y = ops.layer_norm(xg, w, b)
            elif form == "add":
                s, y = ops.add_layer_norm(xg, br, None, w, b)
                y = y + s
            elif form == "merge":
                y = ops.merge_layer_norm(xg, w, b)
            else:
                y = ops.d2s_layer_norm(xg, w, b)
        dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(5)).to(DEV, y.dtype)
        y.backward(dy)
        ops.join_side_streams()
        torch.cuda.synchronize()
        res[direct] = (xg.grad.clone(), w.grad.clone(), b.grad.clone())
    assert ops.ln_batches - batches == (1 if defer else 0)
    assert not ops._ln_pending
    for name, a, r in zip(("dx", "dgamma", "dbeta"), res[True], res[False]):
        if defer and name != "dx":
            assert ((a - r).norm() / r.norm()).item() <= 1e-6, name
        else:
            assert torch.equal(a, r), name


@pytest.mark.parametrize("d2s", [False, True])
def test_refine_conv_param_grads_on_side_stream_equal_autograd(d2s):
    """The refine convs' weight / bias gradients added into trainer-style .grad on the side
    stream (ops._conv_wgrad_param) equal the autograd gradients bitwise (same kernel, added
    into zeros); the input gradient is unchanged."""
    ops = _ops()
    assert ops._CONV_SIDE
    g = torch.Generator().manual_seed(11)
    B, H, W, C = 1, 64, 64, 96
    xin = torch.randn(B, H // 4, W // 4, 16 * C, generator=g) if d2s else torch.randn(B, H, W, C, generator=g)
    xin = xin.to(DEV, torch.bfloat16)
    a = torch.nn.functional.gelu(xin.float()).to(torch.bfloat16)
    w0 = (0.05 * torch.randn(C, C, 3, 3, generator=g)).to(DEV)
    b0 = (0.1 * torch.randn(C, generator=g)).to(DEV)
    dz = torch.randn(B, H, W, C, generator=g).to(DEV, torch.bfloat16)
    res = {}
    for direct in (False, True):
        w = torch.nn.Parameter(w0.clone())
        b = torch.nn.Parameter(b0.clone())
        if direct:
            flat = torch.zeros(w.numel() + C, device=DEV)
            w.grad = flat[:w.numel()].view_as(w)
            b.grad = flat[w.numel():]
            w._msu_direct = b._msu_direct = True
        xg = xin.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            z = ops.refine_conv_act(xg, a, w, b, d2s, (H, W))
        z.backward(dz)
        ops.join_side_streams()
        torch.cuda.synchronize()
        res[direct] = (xg.grad.clone(), w.grad.clone(), b.grad.clone())
    for name, u, r in zip(("dx", "dw", "db"), res[True], res[False]):
        assert torch.equal(u, r), name
