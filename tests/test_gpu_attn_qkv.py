"""GPU: the fused stage-0 unit qkv Linear -> window attention -> proj Linear (ops.window_attention_qkv,
csrc/window_attention_mfma.hip attn_qkv_fwd_mfma, one window per workgroup step with proj inside)
against fp32 PyTorch and against the unfused path it replaces (ops.linear -> ops.window_attention -> ops.linear; reference
network/model_parts.py:166-170 -> torchvision qkv Linear + shifted_window_attention + proj).

* forward vs fp32: attention(x W^T + b) on the same 16-bit operands (tests/_parity_refs.py), at
  small padded / shifted maps and at stage 0 of 1 x 1024^2 (1369 windows, each persistent
  workgroup loops over ~5 windows), bf16 and f16, dropout off and on (the stored keep bits are
  the reference's mask);
* the training outputs: the qkv tensor it keeps for the backward equals the qkv Linear's output,
  and the keep bits equal the unfused forward's (same dropout streams);
* backward (dx, dW, db, d table) equals the unfused path's to 16-bit rounding, and the trainer's
  direct-.grad parameters take the same values;
* inference (no grad) writes no qkv;
* parameters in 16 bits (a model cast with .to(bfloat16)) are converted, not read as f32, and
  frozen ones get no gradient.
"""
import math

import pytest
import torch

from _parity_refs import attn_ref_from_qkv, decode_keep_bits

pytestmark = pytest.mark.gpu

DEV = "cuda"
TOL = {torch.bfloat16: 3e-2, torch.float16: 7.5e-3}
C, NH = 96, 3


def _ops():
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    return ops


def _check(y, ref, t, what):
    y, ref = y.detach().float(), ref.detach().float()
    scale = ref.abs().max().item()
    err = (y - ref).abs().max().item()
    rel2 = ((y - ref).norm() / ref.norm()).item()
    assert err <= t * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"
    assert rel2 <= t / 4, f"{what}: relative L2 {rel2:.3e}"


def _inputs(B, H, W, seed, low):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, H, W, C, generator=g).to(DEV, low)
    w = (torch.randn(3 * C, C, generator=g) / math.sqrt(C)).to(DEV)
    b = (0.3 * torch.randn(3 * C, generator=g)).to(DEV)
    table = torch.randn(169, NH, generator=g).to(DEV)
    dy = torch.randn(B, H, W, C, generator=g).to(DEV, low)
    return x, w, b, table, dy


def _proj(seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(C, C, generator=g) / math.sqrt(C)).to(DEV), (0.1 * torch.randn(C, generator=g)).to(DEV)


@pytest.fixture(params=[torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def low(request):
    return request.param


CASES = [(2, 8, 8, 3), (1, 14, 14, 0), (2, 28, 28, 3), (1, 10, 12, 3), (1, 256, 256, 3), (1, 256, 256, 0)]


@pytest.mark.parametrize("proj", [False, True], ids=["attn", "attn_proj"])
@pytest.mark.parametrize("p_drop", [0.0, 0.05])
@pytest.mark.parametrize("B,H,W,shift", CASES)
def test_fused_forward_matches_fp32(B, H, W, shift, p_drop, proj, low):
    ops = _ops()
    x, w, b, table, _ = _inputs(B, H, W, B * H + W + shift, low)
    wp, bp = _proj(B + H) if proj else (None, None)
    with torch.no_grad(), torch.autocast("cuda", dtype=low):
        assert ops.window_attention_qkv_fusable(x, NH, b)
        y, o, qkv, keep, _ = torch.ops.msunet.window_attention_qkv(x, w, b, table, wp, bp, NH, shift, p_drop, 99, None,
                                                                True)
    torch.cuda.synchronize()
    nwin = B * ((H + 6) // 7) * ((W + 6) // 7)
    mask = decode_keep_bits(keep, nwin * NH) if p_drop > 0 else None
    qkv_ref = torch.nn.functional.linear(x.float(), w.to(low).float(), b)
    _check(qkv, qkv_ref, TOL[low] / 4, "qkv kept for the backward")
    ref = attn_ref_from_qkv(qkv.float(), b, table, NH, shift, keep=mask, p_drop=p_drop)
    if proj:
        _check(o, ref, TOL[low], "o kept for the proj backward")
        ref = torch.nn.functional.linear(o.float(), wp.to(low).float(), bp)
    _check(y, ref, TOL[low], "out")


@pytest.mark.parametrize("B,H,W,shift", [(2, 28, 28, 3), (1, 256, 256, 3)])
def test_fused_equals_unfused_including_backward(B, H, W, shift, low):
    """Same keep bits and qkv as the unfused forward; the outputs and all gradients agree to
    16-bit rounding (the backward kernels are the unfused path's own)."""
    ops = _ops()
    x, w, b, table, dy = _inputs(B, H, W, 7 + H, low)
    res = {}
    wp0, bp0 = _proj(11)
    for fused in (True, False):
        xg = x.clone().requires_grad_(True)
        wg, bg, tg, wpg, bpg = [t.clone().requires_grad_(True) for t in (w, b, table, wp0, bp0)]
        with torch.autocast("cuda", dtype=low):
            if fused:
                y, _, qkv, keep, _ = torch.ops.msunet.window_attention_qkv(xg, wg, bg, tg, wpg, bpg, NH, shift, 0.1, 1234,
                                                                        None, True)
            else:
                qkv = ops.linear(xg, wg, bg)
                o, keep, _ = torch.ops.msunet.window_attention(qkv, bg, tg, NH, shift, 0.1, 1234, None)
                y = ops.linear(o, wpg, bpg)
        y.backward(dy)
        torch.cuda.synchronize()
        res[fused] = (y, qkv.detach(), keep, xg.grad, wg.grad, bg.grad, tg.grad, wpg.grad, bpg.grad)
    assert torch.equal(res[True][2], res[False][2]), "keep bits differ"
    t = TOL[low] / 2
    for name, a, r in zip(("out", "qkv", "keep", "dx", "dW", "db", "dtable", "dWproj", "dbproj"), res[True], res[False]):
        if name != "keep":
            _check(a, r, t, name)


def test_fused_direct_params_match_autograd_params():
    """Trainer-style parameters (flat .grad, bf16 shadow, direct accumulation: the one-pass Linear
    backward and the side-stream attention tail) give the plain autograd gradients."""
    ops = _ops()
    B, H, W, shift = 2, 64, 64, 3
    x, w, b, table, dy = _inputs(B, H, W, 5, torch.bfloat16)
    res = {}
    wp0, bp0 = _proj(3)
    for direct in (False, True):
        xg = x.clone().requires_grad_(True)
        pw, pb, pt, ppw, ppb = (torch.nn.Parameter(t.clone()) for t in (w, b, table, wp0, bp0))
        if direct:
            for p_ in (pw, pb, pt, ppw, ppb):
                p_.grad = torch.zeros_like(p_)
                p_._msu_direct = True
            for p_ in (pw, ppw):
                p_._msu_shadow = p_.detach().to(torch.bfloat16)
                p_._msu_shadow_t = p_.detach().t().contiguous().to(torch.bfloat16)
                p_._msu_shadow_ver = p_._version
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = ops.window_attention_qkv(xg, pw, pb, pt, NH, shift, 0.05, 77, None, ppw, ppb)
        y.backward(dy)
        ops.join_side_streams()
        torch.cuda.synchronize()
        res[direct] = (xg.grad.float(), pw.grad.clone(), pb.grad.clone(), pt.grad.clone(), ppw.grad.clone(),
                       ppb.grad.clone())
    for name, a, r in zip(("dx", "dW", "db", "dtable", "dWproj", "dbproj"), res[True], res[False]):
        _check(a, r, 1e-2, name)


def test_fused_inference_keeps_no_qkv():
    ops = _ops()
    x, w, b, table, _ = _inputs(1, 28, 28, 3, torch.bfloat16)
    wp, bp = _proj(5)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        y1 = ops.window_attention_qkv(x, w, b, table, NH, 3, proj_weight=wp, proj_bias=bp)
        _, o, qkv, _, _ = torch.ops.msunet.window_attention_qkv(x, w, b, table, wp, bp, NH, 3, 0.0, 0, None, False)
        y2 = ops.linear(ops.window_attention(ops.linear(x, w, b), b, table, NH, 3), wp, bp)
    assert qkv.numel() == 0 and o.numel() == 0
    _check(y1, y2, 1.5e-2, "no-grad fused vs unfused")


def test_fused_16bit_params_are_converted():
    """a model cast to bf16 hands the fused unit bf16 biases and table; they must be
    read as their values (converted to f32), exactly as the f32 parameters' rounded values."""
    ops = _ops()
    B, H, W, shift = 1, 28, 28, 3
    x, w, b, table, _ = _inputs(B, H, W, 21, torch.bfloat16)
    wp, bp = _proj(9)
    p16 = [torch.nn.Parameter(t.to(torch.bfloat16)) for t in (w, b, table, wp, bp)]
    p32 = [t.detach().float() for t in p16]  # the same values in f32
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        y16 = ops.window_attention_qkv(x, p16[0], p16[1], p16[2], NH, shift, proj_weight=p16[3], proj_bias=p16[4])
        y32 = ops.window_attention_qkv(x, p32[0], p32[1], p32[2], NH, shift, proj_weight=p32[3], proj_bias=p32[4])
    torch.cuda.synchronize()
    assert torch.equal(y16, y32)


def test_fused_frozen_params_get_no_grad():
    """Frozen qkv / proj weights and biases: no gradient for them (no weight-gradient
    work for parameters that need none), the input gradient equals the unfrozen run's."""
    ops = _ops()
    B, H, W, shift = 1, 28, 28, 3
    x, w, b, table, dy = _inputs(B, H, W, 23, torch.bfloat16)
    wp0, bp0 = _proj(13)
    res = {}
    for frozen in (False, True):
        xg = x.clone().requires_grad_(True)
        ps = [torch.nn.Parameter(t.clone(), requires_grad=not frozen) for t in (w, b, wp0, bp0)]
        pt = torch.nn.Parameter(table.clone())
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = ops.window_attention_qkv(xg, ps[0], ps[1], pt, NH, shift, 0.0, 0, None, ps[2], ps[3])
        y.backward(dy)
        ops.join_side_streams()
        torch.cuda.synchronize()
        res[frozen] = (xg.grad.clone(), pt.grad.clone(), [p.grad for p in ps])
    assert all(g is None for g in res[True][2])
    assert all(g is not None for g in res[False][2])
    assert torch.equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])
