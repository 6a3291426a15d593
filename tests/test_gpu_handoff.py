"""GPU: the residual-gradient handoff (ops.residual_handoff_key).  A stage's first Swin block
reads its input x twice (norm1's LayerNorm, norm2's residual add); with the handoff the two
gradients of x are summed inside norm1's LayerNorm backward kernel instead of by an autograd
add.  Same BasicLayer forward / backward with the handoff on and off: fp32 gradients equal to
f32 rounding (one f32 add moved into the kernel), 16-bit ones within two 16-bit roundings of
each other (the kernel sums in f32 and rounds once; the autograd add rounds the LayerNorm
gradient first).  Reference: model_parts.py:160-173 (torchvision block) via BasicLayer."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _layer(seed):
    from semantic_segmentation_of_stylegan2_artifacts_amd.network.model_parts import BasicLayer
    torch.manual_seed(seed)
    layer = BasicLayer(dim=96, input_resolution=(28, 28), depth=2, num_heads=3, window_size=7,
                       drop_path=0.0).to(DEV).train()
    for p in layer.parameters():  # non-trivial LayerNorm affine parameters
        if p.dim() == 1:
            p.data.normal_(1.0 if p.shape[0] == 96 else 0.0, 0.1)
    return layer


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16], ids=["f32", "bf16", "f16"])
def test_handoff_equals_autograd_sum(dt, monkeypatch):
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    x0 = torch.randn(2, 28 * 28, 96, generator=torch.Generator().manual_seed(1)).to(DEV)
    dy = torch.randn(2, 28 * 28, 96, generator=torch.Generator().manual_seed(2)).to(DEV)
    out = {}
    for on in (False, True):
        monkeypatch.setattr(ops, "_RES_HANDOFF", on)
        layer = _layer(0)
        x = x0.clone().requires_grad_(True)
        n0 = ops.res_handoff_calls
        with torch.autocast("cuda", dtype=dt, enabled=dt != torch.float32):
            y = layer(x)
        y.float().backward(dy.reshape(y.shape))
        torch.cuda.synchronize()
        assert ops.res_handoff_calls - n0 == (1 if on else 0)
        assert not ops._res_handoff, "a parked gradient outlived its backward"
        out[on] = [x.grad] + [p.grad for p in layer.parameters()]
    tol = 1e-5 if dt == torch.float32 else 1.6e-2
    for a, b in zip(out[False], out[True]):
        rel = ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()
        assert rel <= tol, rel


def test_handoff_keys_only_under_grad():
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    with torch.no_grad():
        assert ops.residual_handoff_key() == 0
    if ops._RES_HANDOFF:
        k1, k2 = ops.residual_handoff_key(), ops.residual_handoff_key()
        assert k1 and k2 and k1 != k2


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_skip_handoff_model_equals_autograd_sum(dt, monkeypatch):
    """The whole MSUNetSys (swinT224 golden case): with the handoff on, every stage input's
    readers -- its first block's norm2, the skip fusions' skip halves, the central decoders'
    PatchExpand Linears -- hand their gradients to the first block's norm1 backward kernel
    (up to three per key); off, autograd adds them.  Every parameter gradient agrees
    (f32: to rounding; bf16: within the 16-bit roundings the adds move), nothing parked is left
    untaken, and the skip halves did park (model_parts.py:775-829)."""
    import cases
    from oracle.msunet import make_cfg
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    from semantic_segmentation_of_stylegan2_artifacts_amd.network.model_parts import MSUNetSys
    spec = cases.model_cases()["swinT224"]
    cfg = make_cfg(**spec["cfg"])
    x0, _ = cases.model_inputs(cfg, 2, spec["seed"])
    out = {}
    for on in (False, True):
        monkeypatch.setattr(ops, "_RES_HANDOFF", on)
        torch.manual_seed(0)
        model = MSUNetSys(img_size=cfg["img_size"], patch_size=cfg["patch_size"], in_chans=cfg["in_chans"],
                          num_classes=cfg["num_classes"], embed_dim=cfg["embed_dim"], depths=cfg["depths"],
                          num_heads=cfg["num_heads"], window_size=cfg["window_size"], mlp_ratio=cfg["mlp_ratio"],
                          drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.0)
        model.load_state_dict(cases.model_params(cfg, spec["seed"]), strict=True)
        model = model.to(DEV).train()
        x = x0.to(DEV)
        parked, calls, dropped = ops.res_parked, ops.res_handoff_calls, ops.res_dropped
        with torch.autocast("cuda", dtype=dt, enabled=dt != torch.float32):
            y = model(x)
        dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(3)).to(DEV)
        y.float().backward(dy)
        torch.cuda.synchronize()
        assert ops.res_dropped == dropped
        assert not ops._res_handoff
        if on:
            # the first blocks of 4 encoder stages, the live central up-layer (layers_cent1[1])
            # and 3 decoder up-layers take their norm2's gradient; the stage inputs also take the
            # central PatchExpand Linears' input gradients (stages 1-2) and, in 16-bit, the skip
            # halves of the fused skip concatenations (stages 0-2 and the central stage-1 output;
            # fp32 concatenates with torch.cat)
            assert ops.res_handoff_calls - calls == 8
            extra = 6 if dt != torch.float32 else 2
            assert ops.res_parked - parked == (ops.res_handoff_calls - calls) + extra
        else:
            assert ops.res_parked == parked
        out[on] = [p.grad for p in model.parameters() if p.grad is not None]  # (patchify: no image grad)
    tol = 1e-5 if dt == torch.float32 else 2e-2
    assert len(out[False]) == len(out[True])
    for a, b in zip(out[False], out[True]):
        rel = ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()
        assert rel <= tol, rel
