"""GPU parity of the persistent kernels AT THE SIZES THE BENCH RUNS THEM.

The per-op tests in test_gpu_ops.py use small maps on which every persistent workgroup gets
at most one window / tile, so the loop-carried code (the next-window prefetch and the
double-buffered token table of the attention kernels, the relative-bias gradient kept in
registers across a backward block's windows, the conv kernels' next-tile halo prefetch) is
never reached there.  Here:

* window attention (16-bit MFMA kernels, csrc/window_attention_mfma.hip; reference
  network/model_parts.py:166-170 -> torchvision shifted_window_attention): stage 0 of a
  1024^2 image (256 x 256 tokens, 3 heads, 37^2 = 1369 windows: each forward wave walks 2-3
  windows, each backward workgroup 4-5) and stage 1 at batch 2 (128^2, 6 heads, 722 windows),
  shift 0 and 3, dropout off and at the training rate 0.05 (the reference applies it to the
  probabilities; the reference here uses the forward's stored keep bits, decoded);
  out, dqkv, d relative-position table, d qkv bias against fp32 PyTorch on the same
  16-bit-rounded operands;
* the C = 96 refine conv as the model runs it (refine_conv_act, reference
  model_parts.py:447-448,459-475): the 16-row persistent v3 forward, the v3 dgrad with the
  GELU' epilogue and the LDS-DMA weight gradient at 1 x 1024 x 1024 (2048 tiles on a 256-CU
  grid: 8 per workgroup), d2s (refine1) and plain (refine2) input;
* the one-pass stage-0 Linear backward (msu_linear_bwd) at M = 524288 lives in
  test_gpu_linbwd.py (its M list).

Tolerances: |y - ref| <= t * max|ref| with t = 3e-2 (bf16) / 7.5e-3 (f16) as the per-op tests
(16-bit operands, P and dS rounded to 16 bits before their MFMAs), and the relative L2 error
<= t / 4, which a systematic error in a looped code path (a stale prefetch buffer, a window
computed twice or skipped) would exceed by orders of magnitude.
"""
import math

import pytest
import torch

from _parity_refs import attn_ref_from_qkv, conv3x3_ref, d2s4, decode_keep_bits, gelu_grad

pytestmark = pytest.mark.gpu

DEV = "cuda"
TOL = {torch.bfloat16: 3e-2, torch.float16: 7.5e-3}


def _check(y, ref, t, what):
    y = y.detach().float()
    ref = ref.detach().float()
    scale = ref.abs().max().item()
    err = (y - ref).abs().max().item()
    rel2 = ((y - ref).norm() / ref.norm()).item()
    assert err <= t * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"
    assert rel2 <= t / 4, f"{what}: relative L2 {rel2:.3e}"


@pytest.fixture(params=[torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def low(request):
    return request.param


# B, H, W, heads: stage 0 of 1 x 1024^2, stage 1 of 2 x 1024^2
ATTN_PROD = [(1, 256, 256, 3), (2, 128, 128, 6)]


@pytest.mark.parametrize("p_drop", [0.0, 0.05])
@pytest.mark.parametrize("shift", [0, 3])
@pytest.mark.parametrize("B,H,W,nh", ATTN_PROD)
def test_window_attention_production_size(B, H, W, nh, shift, p_drop, low):
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops  # noqa: F401 (registers torch.ops.msunet)
    C = 32 * nh
    g = torch.Generator().manual_seed(B * H + nh + shift + int(p_drop * 100))
    qkv = torch.randn(B, H, W, 3 * C, generator=g).to(DEV, low)
    qb = (0.3 * torch.randn(3 * C, generator=g)).to(DEV)
    table = torch.randn(169, nh, generator=g).to(DEV)
    dy = torch.randn(B, H, W, C, generator=g).to(DEV, low)
    nwin = B * ((H + 6) // 7) * ((W + 6) // 7)
    # the kernels' own grids must loop at these sizes (the point of the test)
    assert nwin > 4 * 168, nwin

    seed = 1234 + shift
    qg = qkv.clone().requires_grad_(True)
    qbg, tg = qb.clone().requires_grad_(True), table.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=low):
        y, keep, _ = torch.ops.msunet.window_attention(qg, qbg, tg, nh, shift, p_drop, seed, None)
    assert y.dtype == low
    y.backward(dy)
    torch.cuda.synchronize()

    mask = None
    if p_drop > 0:
        assert keep.numel() == nwin * nh * 128
        mask = decode_keep_bits(keep, nwin * nh)
        kept = mask.float().mean().item()
        assert abs(kept - (1 - p_drop)) < 5e-3, kept
    qr = qkv.float().clone().requires_grad_(True)
    qbr, tr = qb.clone().requires_grad_(True), table.clone().requires_grad_(True)
    yr = attn_ref_from_qkv(qr, qbr, tr, nh, shift, keep=mask, p_drop=p_drop)
    yr.backward(dy.float())
    t = TOL[low]
    _check(y, yr, t, "out")
    _check(qg.grad, qr.grad, t, "dqkv")
    _check(tg.grad, tr.grad, t, "d relative_position_bias_table")
    _check(qbg.grad, qbr.grad, t, "d qkv bias (padded tokens)")


def test_window_attention_production_size_side_tail():
    """The trainer's parameters (direct .grad) at stage 0 of 1 x 1024^2: the parameter-gradient
    tail runs on the side stream; same gradients as the autograd path at this size."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    B, H, W, nh, shift = 1, 256, 256, 3, 3
    C = 32 * nh
    g = torch.Generator().manual_seed(77)
    qkv = torch.randn(B, H, W, 3 * C, generator=g).to(DEV, torch.bfloat16)
    qb = (0.3 * torch.randn(3 * C, generator=g)).to(DEV)
    table = torch.randn(169, nh, generator=g).to(DEV)
    dy = torch.randn(B, H, W, C, generator=g).to(DEV, torch.bfloat16)
    res = {}
    for direct in (False, True):
        q = qkv.clone().requires_grad_(True)
        pb, pt = torch.nn.Parameter(qb.clone()), torch.nn.Parameter(table.clone())
        if direct:
            for p in (pb, pt):
                p.grad = torch.zeros_like(p)
                p._msu_direct = True
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = ops.window_attention(q, pb, pt, nh, shift, 0.05, 99)
        y.backward(dy)
        ops.join_side_streams()
        torch.cuda.synchronize()
        res[direct] = (q.grad.float(), pb.grad.clone(), pt.grad.clone())
    for a, b, what in zip(res[True], res[False], ("dqkv", "dbias", "dtable")):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6, msg=what)


@pytest.mark.parametrize("d2s", [True, False], ids=["refine1_d2s", "refine2_plain"])
def test_refine_conv_production_size(d2s, low):
    """refine_conv_act at 1 x 1024 x 1024, C = 96: z, GELU(z) (dual epilogue), dx (dgrad with
    GELU'(x) in its epilogue, d2s scatter), dW, db against nine shifted fp32 matmuls of the
    same 16-bit activation and 16-bit-rounded weights."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    B, H, W, C = 1, 1024, 1024, 96
    g = torch.Generator().manual_seed(1024 + int(d2s))
    xs = (B, H // 4, W // 4, 16 * C) if d2s else (B, H, W, C)
    x = torch.randn(xs, generator=g).to(DEV, low)           # pre-activation (producer's E / z1)
    with torch.autocast("cuda", dtype=low):
        a = ops.gelu(x)                                      # its activation, as the producer stores it
    assert a.dtype == low
    w = (torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)).to(DEV)
    b = (0.1 * torch.randn(C, generator=g)).to(DEV)
    dz = torch.randn(B, H, W, C, generator=g).to(DEV, low)
    xg = x.clone().requires_grad_(True)
    wg, bg = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=low):
        z, z2 = ops.refine_conv_act(xg, a, wg, bg, d2s, (H, W), dual=True)
    z.backward(dz)
    torch.cuda.synchronize()

    af = a.float()
    if d2s:
        af = d2s4(af, C)
    ar = af.clone().requires_grad_(True)
    wr = w.to(low).float().clone().requires_grad_(True)      # the kernels run 16-bit weights
    br = b.clone().requires_grad_(True)
    zr = conv3x3_ref(ar, wr, br)
    zr.backward(dz.float())
    t = TOL[low]
    _check(z, zr, t, "z")
    _check(z2, torch.nn.functional.gelu(z.float()), t, "GELU(z)")
    dxr = ar.grad
    if d2s:  # back through the depth-to-space: [B, 4h, 4w, C] -> [B, h, w, 16 C]
        dxr = dxr.view(B, H // 4, 4, W // 4, 4, C).permute(0, 1, 3, 2, 4, 5).reshape(xs)
    dxr = dxr * gelu_grad(x.float())
    _check(xg.grad, dxr, t, "dx (GELU' epilogue)")
    _check(wg.grad, wr.grad, t, "dW")
    _check(bg.grad, br.grad, t, "db")
