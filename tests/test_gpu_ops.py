"""GPU parity of every HIP op against the CPU oracle / a plain fp32 PyTorch reference.

fp32 mode: tolerance 1e-4 relative (kernels compute in f32; only summation order differs).
bf16 mode: tolerance stated per test (bf16 storage has 8 significant bits).
f16 mode (the reference's autocast float16): a quarter of the bf16 tolerance (f16 storage has
11 significant bits, every statistic and accumulation is f32 in both).
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from oracle import swin_block as osb  # noqa: E402
from oracle import msunet as om  # noqa: E402
from oracle import dynamic_loss as odl  # noqa: E402

DEV = "cuda"


def _ops():
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    return ops


def _close(a, b, rtol, atol, what=""):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item()
    assert err <= atol + rtol * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


def _g(seed):
    return torch.Generator().manual_seed(seed)


def _tol(dtype, f32, bf16):
    return f32 if dtype == torch.float32 else (bf16 if dtype == torch.bfloat16 else bf16 / 4)


LOW = [torch.bfloat16, torch.float16]
ALL = [torch.float32] + LOW


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 3e-2), (torch.float16, 7.5e-3)])
@pytest.mark.parametrize("C,rows", [(96, 1000), (32, 64), (384, 333), (1536, 77)])
def test_layer_norm(dtype, tol, C, rows):
    ops = _ops()
    g = _g(C)
    x = (torch.randn(rows, C, generator=g) * 2 + 0.5)
    w = 1 + 0.1 * torch.randn(C, generator=g)
    b = 0.1 * torch.randn(C, generator=g)
    dy = torch.randn(rows, C, generator=g)
    xr = x.clone().requires_grad_(True); wr = w.clone().requires_grad_(True); br = b.clone().requires_grad_(True)
    yr = F.layer_norm(xr, (C,), wr, br, 1e-5)
    yr.backward(dy)
    xg = x.to(DEV, dtype).requires_grad_(True)
    wg = w.to(DEV).requires_grad_(True)
    bg = b.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=dtype, enabled=dtype != torch.float32):
        y = ops.layer_norm(xg, wg, bg)
    y.backward(dy.to(DEV, dtype))
    _close(y, yr, tol, tol, "y")
    _close(xg.grad, xr.grad, tol, tol, "dx")
    _close(wg.grad, wr.grad, tol, tol * rows ** 0.5, "dw")
    _close(bg.grad, br.grad, tol, tol * rows ** 0.5, "db")


@pytest.mark.parametrize("use_scale", [False, True])
def test_add_layer_norm(use_scale):
    ops = _ops()
    g = _g(7)
    B, H, W, C = 3, 5, 6, 192
    a = torch.randn(B, H, W, C, generator=g)
    br = torch.randn(B, H, W, C, generator=g)
    sc = torch.tensor([0.0, 1.25, 1.25]) if use_scale else None
    w = 1 + 0.1 * torch.randn(C, generator=g)
    bb = 0.1 * torch.randn(C, generator=g)
    ds_up = torch.randn(B, H, W, C, generator=g)
    dy_up = torch.randn(B, H, W, C, generator=g)
    ar, brr, wr, bbr = [t.clone().requires_grad_(True) for t in (a, br, w, bb)]
    s_ref = ar + brr * (sc.view(B, 1, 1, 1) if sc is not None else 1.0)
    y_ref = F.layer_norm(s_ref, (C,), wr, bbr, 1e-5)
    (s_ref * ds_up + y_ref * dy_up).sum().backward()
    ag, bgg, wg, bbg = [t.to(DEV).requires_grad_(True) for t in (a, br, w, bb)]
    s, y = ops.add_layer_norm(ag, bgg, sc.to(DEV) if sc is not None else None, wg, bbg)
    (s * ds_up.to(DEV) + y * dy_up.to(DEV)).sum().backward()
    _close(s, s_ref, 1e-5, 1e-5, "s")
    _close(y, y_ref, 1e-4, 1e-4, "y")
    _close(ag.grad, ar.grad, 1e-4, 1e-4, "da")
    _close(bgg.grad, brr.grad, 1e-4, 1e-4, "dbranch")
    _close(wg.grad, wr.grad, 1e-4, 1e-3, "dw")
    _close(bbg.grad, bbr.grad, 1e-4, 1e-3, "db")


@pytest.mark.parametrize("B,H,W,C", [(2, 8, 8, 16), (1, 14, 10, 96), (2, 64, 64, 96)])
def test_merge_layer_norm(B, H, W, C):
    ops = _ops()
    g = _g(H * W)
    x = torch.randn(B, H, W, C, generator=g)
    w = 1 + 0.1 * torch.randn(4 * C, generator=g)
    b = 0.1 * torch.randn(4 * C, generator=g)
    xr = x.clone().requires_grad_(True)
    x0, x1, x2, x3 = xr[:, 0::2, 0::2], xr[:, 1::2, 0::2], xr[:, 0::2, 1::2], xr[:, 1::2, 1::2]
    yr = F.layer_norm(torch.cat([x0, x1, x2, x3], -1).view(B, -1, 4 * C), (4 * C,), w, b, 1e-5)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    xg = x.to(DEV).requires_grad_(True)
    y = ops.merge_layer_norm(xg, w.to(DEV), b.to(DEV))
    y.backward(dy.to(DEV))
    _close(y, yr, 1e-4, 1e-4, "y")
    _close(xg.grad, xr.grad, 1e-4, 1e-4, "dx")


@pytest.mark.parametrize("B,H,W,c", [(2, 4, 4, 16), (1, 7, 5, 48), (2, 32, 32, 96)])
def test_d2s_layer_norm(B, H, W, c):
    from einops import rearrange
    ops = _ops()
    g = _g(c)
    x = torch.randn(B, H, W, 4 * c, generator=g)
    w = 1 + 0.1 * torch.randn(c, generator=g)
    b = 0.1 * torch.randn(c, generator=g)
    xr = x.clone().requires_grad_(True)
    yr = F.layer_norm(rearrange(xr, "b h w (p1 p2 c)-> b (h p1) (w p2) c", p1=2, p2=2, c=c).reshape(B, -1, c),
                      (c,), w, b, 1e-5)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    xg = x.to(DEV).requires_grad_(True)
    y = ops.d2s_layer_norm(xg, w.to(DEV), b.to(DEV))
    y.backward(dy.to(DEV))
    _close(y, yr, 1e-4, 1e-4, "y")
    _close(xg.grad, xr.grad, 1e-4, 1e-4, "dx")


ATTN_CASES = [
    # B, H, W, heads, shift
    (2, 8, 8, 1, 3),     # pad 8 -> 14, shifted
    (1, 14, 14, 2, 0),   # no pad, no shift
    (1, 14, 14, 2, 3),   # no pad, shifted
    (2, 7, 7, 3, 3),     # window covers the map -> torchvision zeroes the shift
    (1, 10, 12, 2, 3),   # non-square, padded both axes
    (2, 28, 28, 3, 3),
    (1, 16, 16, 4, 0),   # pad 16 -> 21, padded tokens attend unmasked
]


@pytest.mark.parametrize("B,H,W,nh,shift", ATTN_CASES)
def test_window_attention_fp32(B, H, W, nh, shift):
    """ops.window_attention (qkv Linear outside) == torchvision v1 restatement, fwd + bwd."""
    ops = _ops()
    C = 32 * nh
    g = _g(B * H * W + nh)
    x = torch.randn(B, H, W, C, generator=g)
    qw = torch.randn(3 * C, C, generator=g) / math.sqrt(C)
    qb = 0.3 * torch.randn(3 * C, generator=g)
    table = torch.randn(169, nh, generator=g)
    index = osb.relative_position_index(7)
    eye, zero = torch.eye(C), torch.zeros(C)
    xr, qwr, qbr, tr = [t.clone().requires_grad_(True) for t in (x, qw, qb, table)]
    yr = osb.shifted_window_attention(xr, qwr, qbr, eye, zero, tr, index, 7, nh, shift)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    xg, qwg, qbg, tg = [t.to(DEV).requires_grad_(True) for t in (x, qw, qb, table)]
    qkv = F.linear(xg, qwg, qbg)
    y = ops.window_attention(qkv, qbg, tg, nh, shift)
    y.backward(dy.to(DEV))
    _close(y, yr, 1e-4, 1e-5, "out")
    _close(xg.grad, xr.grad, 1e-4, 1e-5, "dx")
    _close(qwg.grad, qwr.grad, 1e-4, 1e-5, "dWqkv")
    _close(qbg.grad, qbr.grad, 1e-4, 1e-5, "dbqkv (incl. padded tokens)")
    _close(tg.grad, tr.grad, 1e-4, 1e-5, "d relative_position_bias_table")


@pytest.mark.parametrize("low", LOW)
@pytest.mark.parametrize("B,H,W,nh,shift", [(2, 8, 8, 1, 3), (1, 28, 28, 3, 3), (2, 64, 64, 3, 0)])
def test_window_attention_bf16(B, H, W, nh, shift, low):
    ops = _ops()
    C = 32 * nh
    g = _g(3 + H)
    qkv = torch.randn(B, H, W, 3 * C, generator=g)
    qb = 0.3 * torch.randn(3 * C, generator=g)
    table = torch.randn(169, nh, generator=g)
    y32 = ops.window_attention(qkv.to(DEV), qb.to(DEV), table.to(DEV), nh, shift)
    with torch.autocast("cuda", dtype=low):
        y16 = ops.window_attention(qkv.to(DEV), qb.to(DEV), table.to(DEV), nh, shift)
    assert y16.dtype == low
    t = _tol(low, 0, 3e-2)
    _close(y16, y32, t, t, f"{low} vs f32")


def test_window_attention_dropout_statistics():
    """p=0 is exact; with p>0 the kept fraction is ~1-p and output is unbiased; fwd/bwd use
    the same mask (checked via linearity: <dy, y> == <dqkv_v, v> for the v-part)."""
    ops = _ops()
    B, H, W, nh, C = 2, 28, 28, 2, 64
    g = _g(99)
    qkv = torch.randn(B, H, W, 3 * C, generator=g).to(DEV)
    qb = torch.zeros(3 * C, device=DEV)
    table = torch.zeros(169, nh, device=DEV)
    y0 = ops.window_attention(qkv, qb, table, nh, 0, 0.0, 1)
    ys = torch.stack([ops.window_attention(qkv, qb, table, nh, 0, 0.25, s) for s in range(64)])
    rel = ((ys.mean(0) - y0).norm() / y0.norm()).item()
    assert rel < 0.1, rel
    assert not torch.equal(ys[0], ys[1])
    q = qkv.clone().requires_grad_(True)
    y = ops.window_attention(q, qb, table, nh, 0, 0.5, 1234)
    dy = torch.randn_like(y)
    y.backward(dy)
    v = q[..., 2 * C:]
    lhs = (dy * y).sum()
    rhs = (q.grad[..., 2 * C:] * v).sum()
    assert abs(lhs.item() - rhs.item()) <= 1e-3 * abs(lhs.item()) + 1e-3


@pytest.mark.parametrize("shift", [0, 3])
def test_window_attention_dropout_masks_agree_f32_bf16(shift):
    """The f32 parity kernels draw the same dropout masks as the 16-bit MFMA kernels (one
    element at a time from the same per-row streams): with p = 0.3 the outputs agree to bf16
    rounding, which a single differing mask element per row would break."""
    ops = _ops()
    B, H, W, nh = 2, 21, 26, 2
    C = 32 * nh
    g = _g(31 + shift)
    qkv = torch.randn(B, H, W, 3 * C, generator=g).to(DEV)
    qb = (torch.randn(3 * C, generator=g) * 0.1).to(DEV)
    table = (torch.randn(169, nh, generator=g) * 0.1).to(DEV)
    q16 = qkv.bfloat16()
    y32 = ops.window_attention(q16.float(), qb, table, nh, shift, 0.3, 77)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y16 = ops.window_attention(q16, qb, table, nh, shift, 0.3, 77)
    err = (y16.float() - y32).abs().max().item()
    assert err <= 3e-2 * y32.abs().max().item(), err


@pytest.mark.parametrize("low", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shift", [0, 3])
def test_window_attention_keep_bits_equal_rehash(low, shift):
    """16-bit dropout: the backward reading the forward's stored keep bits (the op's path) gives
    bit-identical dqkv / dtable / dbias to the backward that re-hashes the mask from the seed
    (keep = null), and the stored bits have the kept fraction ~1 - p."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import _lib
    ops = _ops()
    B, H, W, nh = 2, 30, 33, 3
    C = 32 * nh
    g = _g(7 + shift)
    qkv = torch.randn(B, H, W, 3 * C, generator=g).to(DEV, low)
    qb = (torch.randn(3 * C, generator=g) * 0.1).to(DEV)
    table = (torch.randn(169, nh, generator=g) * 0.1).to(DEV)
    dout = torch.randn(B, H, W, C, generator=g).to(DEV, low)
    p, seed = 0.3, 4321
    y, keep, _ = torch.ops.msunet.window_attention(qkv, qb, table, nh, shift, p, seed, None)
    nwin = B * ((H + 6) // 7) * ((W + 6) // 7)
    assert keep.numel() == nwin * nh * 128
    # bit b of word [item][it][lane]: query i = 32 it + (lane & 31), key j = 32 (b >> 4) + crow(b & 15)
    it, lane, b = torch.meshgrid(torch.arange(2), torch.arange(64), torch.arange(32), indexing="ij")
    r = b & 15
    i = 32 * it + (lane & 31)
    j = 32 * (b >> 4) + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
    real = ((i < 49) & (j < 49)).to(DEV)
    bits = (keep.view(nwin * nh, 2, 64, 1) >> torch.arange(32, device=DEV)) & 1
    kept = (bits.bool() & real).sum().item() / (real.sum().item() * nwin * nh)
    assert abs(kept - (1 - p)) < 0.01, kept
    L = _lib.lib()
    dt = ops._dt(qkv)
    outs = []
    for kp in (keep.data_ptr(), None):
        ws = torch.empty(L.msu_win_attn_bwd_workspace(dt, B, H, W, C, nh), device=DEV)
        dqkv = torch.empty_like(qkv)
        dtab = torch.empty_like(table)
        dbias = torch.empty(3 * C, device=DEV)
        _lib.call("msu_win_attn_bwd", dt, qkv.data_ptr(), qb.data_ptr(), table.data_ptr(), dout.data_ptr(),
                  dqkv.data_ptr(), dtab.data_ptr(), dbias.data_ptr(), ws.data_ptr(), B, H, W, C, nh, shift, p,
                  seed, None, kp, torch.cuda.current_stream().cuda_stream)
        outs.append((dqkv, dtab, dbias))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # and the op's own backward is that result
    q = qkv.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=low):
        y2 = ops.window_attention(q, qb, table, nh, shift, p, seed)
    assert torch.equal(y2, y)
    y2.backward(dout)
    assert torch.equal(q.grad, outs[0][0])


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2), (torch.float16, 5e-3)])
def test_gelu(dtype, tol):
    ops = _ops()
    x = torch.randn(4096, generator=_g(1)) * 3
    xr = x.clone().requires_grad_(True)
    yr = F.gelu(xr)
    yr.backward(torch.ones_like(x))
    xg = x.to(DEV, dtype).requires_grad_(True)
    with torch.autocast("cuda", dtype=dtype, enabled=dtype != torch.float32):
        y = ops.gelu(xg)
    y.backward(torch.ones_like(y))
    _close(y, yr, tol, tol, "gelu")
    _close(xg.grad, xr.grad, tol, tol, "gelu'")


CONV_CASES = [
    # B, H, W (output), C, d2s
    (2, 24, 24, 16, True),
    (1, 32, 20, 32, True),
    (1, 20, 36, 32, False),
    (2, 64, 64, 96, True),
    (1, 48, 32, 96, False),
    (1, 32, 32, 128, True),
    (1, 40, 56, 96, True),     # partial 8x32 tiles of the persistent bf16 kernel
    (2, 20, 36, 96, False),
]


def _conv_ref(x, w, b, d2s, H, W):
    from einops import rearrange
    C = w.shape[1]
    if d2s:
        x = rearrange(x, "b h w (p1 p2 c) -> b (h p1) (w p2) c", p1=4, p2=4, c=C)
    x = F.gelu(x).permute(0, 3, 1, 2)
    return F.conv2d(x, w, b, padding=1).permute(0, 2, 3, 1)


@pytest.mark.parametrize("Cout,Cin", [(96, 96), (5, 40), (33, 7), (192, 224)])
@pytest.mark.parametrize("dtype", ALL)
def test_conv_weight_layouts(Cout, Cin, dtype):
    """msu_conv3x3_weight against the ATen expression it replaces (flip / permute / zero pad to
    32 / cast), bit-exact, both layouts, ragged widths included."""
    ops = _ops()
    w = torch.randn(Cout, Cin, 3, 3, generator=_g(Cout * Cin)).to(DEV)

    def pad32(t):
        p = (-t.shape[2]) % 32
        return torch.cat([t, t.new_zeros(t.shape[0], t.shape[1], p)], 2)

    wt = pad32(w.permute(2, 3, 0, 1).reshape(9, Cout, Cin)).to(dtype)
    wf = pad32(w.flip(2, 3).permute(2, 3, 1, 0).reshape(9, Cin, Cout)).to(dtype)
    assert torch.equal(ops._conv_weight(w, dtype, 0), wt)
    assert torch.equal(ops._conv_weight(w, dtype, 1), wf)


@pytest.mark.parametrize("mode", [0, 2], ids=["plain", "d2s"])
@pytest.mark.parametrize("C", [96, 64])
def test_conv_wgrad_accumulate_equals_add(C, mode):
    """msu_conv3x3_wgrad2 with accumulate: dW / db added into existing f32 gradients bitwise equal
    to the overwrite form followed by an f32 add (the side stream's .grad accumulation)."""
    ops = _ops()
    g = _g(C + mode)
    B, H, W = 2, 32, 32
    xs = (B, H // 4, W // 4, 16 * C) if mode == 2 else (B, H, W, C)
    a = torch.randn(xs, generator=g).to(DEV, torch.bfloat16)
    dz = torch.randn(B, H, W, C, generator=g).to(DEV, torch.bfloat16)
    w0 = torch.randn(C, C, 3, 3, generator=g).to(DEV)
    b0 = torch.randn(C, generator=g).to(DEV)
    dw, db = ops._conv_wgrad(a, dz, mode, B, H, W, C, C)
    w, b = torch.nn.Parameter(w0.clone()), torch.nn.Parameter(b0.clone())
    w.grad, b.grad = w0.clone(), b0.clone()
    ops._conv_wgrad(a, dz, mode, B, H, W, C, C, into=(w, b))
    torch.cuda.synchronize()
    assert torch.equal(w.grad, w0 + dw)
    assert torch.equal(b.grad, b0 + db)


@pytest.mark.parametrize("B,H,W,C,d2s", CONV_CASES)
@pytest.mark.parametrize("dtype", ALL)
def test_refine_conv(B, H, W, C, d2s, dtype):
    ops = _ops()
    g = _g(H * W + C)
    xs = (B, H // 4, W // 4, 16 * C) if d2s else (B, H, W, C)
    x = torch.randn(xs, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)
    b = 0.1 * torch.randn(C, generator=g)
    dz = torch.randn(B, H, W, C, generator=g)
    xr, wr, br = [t.clone().requires_grad_(True) for t in (x, w, b)]
    zr = _conv_ref(xr, wr, br, d2s, H, W)
    zr.backward(dz)
    xg = x.to(DEV, dtype).requires_grad_(True)
    wg, bg = w.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=dtype, enabled=dtype != torch.float32):
        z = ops.refine_conv(xg, wg, bg, d2s, (H, W))
    z.backward(dz.to(DEV, dtype))
    tol = _tol(dtype, 1e-4, 3e-2)
    _close(z, zr, tol, tol, "z")
    _close(xg.grad, xr.grad, tol, tol, "dx")
    _close(wg.grad, wr.grad, tol, tol, "dW")
    _close(bg.grad, br.grad, tol, tol, "db")


@pytest.mark.parametrize("B,H,W,C,d2s", CONV_CASES)
@pytest.mark.parametrize("dtype", ALL)
def test_refine_conv_act(B, H, W, C, d2s, dtype):
    """refine_conv_act (activation supplied by the producer, conv loads it as is; dual
    epilogue) against refine_conv (GELU on load) on the same pre-activation: same z, dz->dx,
    dW, db; the dual output equals GELU(z) as the GELU op computes it."""
    ops = _ops()
    g = _g(H * W + C + 7)
    xs = (B, H // 4, W // 4, 16 * C) if d2s else (B, H, W, C)
    x = torch.randn(xs, generator=g).to(DEV, dtype)
    w = (torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)).to(DEV)
    b = (0.1 * torch.randn(C, generator=g)).to(DEV)
    dz = torch.randn(B, H, W, C, generator=g).to(DEV, dtype)
    with torch.autocast("cuda", dtype=dtype, enabled=dtype != torch.float32):
        x1, w1, b1 = [t.clone().requires_grad_(True) for t in (x, w, b)]
        z1 = ops.refine_conv(x1, w1, b1, d2s, (H, W))
        z1.backward(dz)
        x2, w2, b2 = [t.clone().requires_grad_(True) for t in (x, w, b)]
        a = ops.gelu(x2.detach())
        z2, g2 = ops.refine_conv_act(x2, a, w2, b2, d2s, (H, W), dual=True)
        z2.backward(dz)
        gz = ops.gelu(z2.detach())
    # bf16: the conv's on-load GELU (fast erf) and the GELU op (erf) may round a few inputs
    # one bf16 ulp apart
    tol = _tol(dtype, 1e-5, 2e-2)
    _close(z2, z1, tol, tol, "z")
    _close(g2, gz, tol, tol, "GELU(z)")
    _close(x2.grad, x1.grad, tol, tol, "dx")
    _close(w2.grad, w1.grad, tol, tol, "dW")
    _close(b2.grad, b1.grad, tol, tol, "db")


@pytest.mark.parametrize("B,H,W,d2s", [(2, 64, 64, True), (1, 48, 32, False), (1, 40, 56, True),
                                        (2, 20, 36, False), (1, 16, 32, False), (1, 128, 96, True)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_refine_conv_act_fwd_matches_fp32(B, H, W, d2s, dtype):
    """The 16-bit C = 96 forward as the model runs it (activation precomputed by the producer:
    the 16-row x 32-pixel persistent kernel, conv3x3_v4_kernel) against fp32 conv2d of the same
    16-bit activation -- z and the dual output GELU(z); tiles cut by the image edge included."""
    ops = _ops()
    C = 96
    g = _g(H * W + 11)
    xs = (B, H // 4, W // 4, 16 * C) if d2s else (B, H, W, C)
    a = torch.randn(xs, generator=g).to(dtype)
    w = torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)
    b = 0.1 * torch.randn(C, generator=g)
    from einops import rearrange
    af = a.float()
    if d2s:
        af = rearrange(af, "b h w (p1 p2 c) -> b (h p1) (w p2) c", p1=4, p2=4, c=C)
    zr = F.conv2d(af.permute(0, 3, 1, 2), w, b, padding=1).permute(0, 2, 3, 1)
    with torch.autocast("cuda", dtype=dtype):
        ad = a.to(DEV)
        z, z2 = ops.refine_conv_act(ad, ad, w.to(DEV), b.to(DEV), d2s, (H, W), dual=True)
    tol = _tol(dtype, 1e-4, 2e-2)
    _close(z, zr, tol, tol, "z")
    _close(z2, F.gelu(z.float()), tol, tol, "GELU(z)")


@pytest.mark.parametrize("M,N,K", [(4096, 1536, 96), (1000, 256, 16)])
@pytest.mark.parametrize("dtype", ALL)
def test_linear_gelu(M, N, K, dtype):
    """linear_gelu: (x W^T, GELU(x W^T)) with gradients of the first output = ops.linear's."""
    ops = _ops()
    g = _g(M + N + K)
    x = torch.randn(M, K, generator=g).to(DEV, dtype)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV)
    dy = torch.randn(M, N, generator=g).to(DEV, dtype)
    with torch.autocast("cuda", dtype=dtype, enabled=dtype != torch.float32):
        x1, w1 = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
        y1 = ops.linear(x1, w1)
        y1.backward(dy)
        g1 = ops.gelu(y1.detach())
        x2, w2 = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
        y2, g2 = ops.linear_gelu(x2, w2)
        y2.backward(dy)
    tol = _tol(dtype, 1e-4, 2e-2)
    _close(y2, y1, tol, tol, "y")
    _close(g2, g1, tol, tol, "GELU(y)")
    _close(x2.grad, x1.grad, tol, tol, "dx")
    _close(w2.grad, w1.grad, tol, tol, "dW")


@pytest.mark.parametrize("dtype,C,W", [(torch.float32, 96, 12), (torch.bfloat16, 96, 13), (torch.bfloat16, 128, 7),
                                       (torch.float16, 96, 13), (torch.float16, 128, 7), (torch.float16, 64, 5)])
def test_head_norm_output(dtype, C, W):
    ops = _ops()
    g = _g(5)
    B, H = 2, 16
    z = torch.randn(B, H, W, C, generator=g)
    gm = 1 + 0.1 * torch.randn(C, generator=g)
    bt = 0.1 * torch.randn(C, generator=g)
    wo = torch.randn(1, C, 1, 1, generator=g) / math.sqrt(C)
    zr, gr, btr, wr = [t.clone().requires_grad_(True) for t in (z, gm, bt, wo)]
    yr = F.conv2d(F.layer_norm(zr, (C,), gr, btr, 1e-5).permute(0, 3, 1, 2), wr)
    dl = torch.randn(yr.shape, generator=g)
    yr.backward(dl)
    zg = z.to(DEV, dtype).requires_grad_(True)
    gg, bg, wg = [t.to(DEV).requires_grad_(True) for t in (gm, bt, wo)]
    with torch.autocast("cuda", dtype=dtype, enabled=dtype != torch.float32):
        y = ops.head_norm_output(zg, gg, bg, wg)
    y.backward(dl.to(DEV))
    tol = _tol(dtype, 1e-4, 3e-2)
    _close(y, yr, tol, 1e-5 if dtype == torch.float32 else tol, "logits")
    _close(zg.grad, zr.grad, tol, 1e-5 if dtype == torch.float32 else tol, "dz")
    _close(gg.grad, gr.grad, tol, tol, "dgamma")
    _close(bg.grad, btr.grad, tol, tol, "dbeta")
    _close(wg.grad, wr.grad, tol, tol, "dw_out")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_head_direct_params_accumulate_into_grad(dtype):
    """Trainer-direct gamma / beta / output weight: the head backward adds its sums into the
    existing .grad (msu_head_bwd2, accumulate) -- bitwise the autograd gradients added to it; dz
    bitwise."""
    ops = _ops()
    g = _g(8)
    B, H, W, C = 2, 16, 13, 96
    z = torch.randn(B, H, W, C, generator=g).to(DEV, dtype)
    p0 = [(1 + 0.1 * torch.randn(C, generator=g)).to(DEV), (0.1 * torch.randn(C, generator=g)).to(DEV),
          (torch.randn(1, C, 1, 1, generator=g) / math.sqrt(C)).to(DEV)]
    g0 = [torch.randn(t.shape, generator=g).to(DEV) for t in p0]
    dl = torch.randn(B, 1, H, W, generator=g).to(DEV)
    res = {}
    for direct in (False, True):
        ps = [torch.nn.Parameter(t.clone()) for t in p0]
        if direct:
            for p, g1 in zip(ps, g0):
                p.grad = g1.clone()
                p._msu_direct = True
        zg = z.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=dtype):
            y = ops.head_norm_output(zg, *ps)
        y.backward(dl)
        torch.cuda.synchronize()
        res[direct] = (zg.grad, [p.grad if direct else g1 + p.grad for p, g1 in zip(ps, g0)])
    assert torch.equal(res[True][0], res[False][0])
    for a, b in zip(res[True][1], res[False][1]):
        assert torch.equal(a, b)


def test_patchify_matches_conv():
    ops = _ops()
    g = _g(6)
    img = torch.rand(2, 3, 32, 48, generator=g)
    w = torch.randn(96, 3, 4, 4, generator=g)
    b = torch.randn(96, generator=g)
    ref = F.conv2d(img, w, b, stride=4).flatten(2).transpose(1, 2).reshape(-1, 96)
    cols = ops.patchify(img.to(DEV), 4, torch.float32)
    out = F.linear(cols, w.to(DEV).reshape(96, -1), b.to(DEV))
    _close(out, ref, 1e-5, 1e-5, "patch embed")


def test_dynamic_loss_golden(golden_dir):
    import os
    import cases
    from semantic_segmentation_of_stylegan2_artifacts_amd.loss import DynamicLoss
    z = np.load(os.path.join(golden_dir, "dynamic_loss.npz"))
    for name, (logits, target, kw) in cases.loss_cases().items():
        lossf = DynamicLoss(alpha=kw["alpha"], beta=kw["beta"], tversky_bce_mix=kw["mix"])
        x = logits.to(DEV).requires_grad_(True)
        loss = lossf(x, target.to(DEV))
        loss.backward()
        ref = float(z[f"{name}.loss"])
        assert abs(loss.item() - ref) <= 1e-5 * max(1, abs(ref)), name
        _close(x.grad, torch.from_numpy(z[f"{name}.grad"]), 1e-4, 1e-9, name)


def test_dynamic_loss_resets_the_registered_step_flag():
    """ops.set_step_flag: the DynamicLoss forward's final launch zeroes the registered flag (the
    trainer's non-finite flag) and reports it; the loss value is unchanged; unregistered: the flag
    is left alone."""
    import cases
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    from semantic_segmentation_of_stylegan2_artifacts_amd.loss import DynamicLoss
    logits, target, kw = cases.loss_cases()["mixed3d"]
    lossf = DynamicLoss(alpha=kw["alpha"], beta=kw["beta"], tversky_bce_mix=kw["mix"])
    x, t = logits.to(DEV), target.to(DEV)
    ref = lossf(x, t).item()
    flag = torch.ones(1, device=DEV)
    ops.set_step_flag(flag)
    try:
        assert not ops.step_flag_reset()
        out = lossf(x, t).item()
        assert ops.step_flag_reset()
    finally:
        ops.set_step_flag(None)
    assert out == ref
    assert flag.item() == 0.0
    flag.fill_(1.0)
    lossf(x, t)
    assert flag.item() == 1.0


@pytest.mark.parametrize("low", LOW)
def test_dynamic_loss_bf16_logits(low):
    from semantic_segmentation_of_stylegan2_artifacts_amd.loss import DynamicLoss
    import cases
    logits, target, kw = cases.loss_cases()["mixed3d"]
    lb = logits.to(low)
    ref = odl.dynamic_loss(lb.float(), target, **kw)
    out = DynamicLoss(alpha=kw["alpha"], beta=kw["beta"], tversky_bce_mix=kw["mix"])(lb.to(DEV), target.to(DEV))
    assert abs(out.item() - ref.item()) < 1e-5


def test_adamw_matches_torch():
    ops = _ops()
    g = _g(8)
    n = 10007
    p0 = torch.randn(n, generator=g)
    grads = [torch.randn(n, generator=g) for _ in range(5)]
    pr = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([pr], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01)
    pg = p0.to(DEV)
    m = torch.zeros_like(pg)
    v = torch.zeros_like(pg)
    for step, gr in enumerate(grads, 1):
        pr.grad = gr.clone()
        opt.step()
        ops.adamw_(pg, gr.to(DEV), m, v, 1e-3, 0.9, 0.999, 1e-8, 0.01, step)
    _close(pg, pr, 1e-6, 1e-6, "adamw")


@pytest.mark.parametrize("M,N,K", [(100, 96, 288), (4096, 288, 96), (777, 32, 48), (65536, 384, 96),
                                   (3000, 1536, 96), (512, 192, 768), (8192, 1152, 384), (2000, 384, 384),
                                   # wave splits of the weight-gradient plan (N x K tiles of 96): 1x4, 1x2, 2x1
                                   (65536, 96, 384), (1024, 96, 192), (1024, 192, 96), (8192, 576, 192)])
@pytest.mark.parametrize("dtype", ALL)
def test_linear(M, N, K, dtype):
    """ops.linear: hipBLASLt fwd/dgrad + HIP split-M weight/bias gradient vs fp32 torch."""
    ops = _ops()
    g = _g(M + N + K)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / math.sqrt(K)
    b = torch.randn(N, generator=g)
    dy = torch.randn(M, N, generator=g)
    xr, wr, br = [t.clone().requires_grad_(True) for t in (x, w, b)]
    yr = F.linear(xr, wr, br)
    yr.backward(dy)
    xg = x.to(DEV, dtype).requires_grad_(True)
    wg, bg = w.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=dtype, enabled=dtype != torch.float32):
        y = ops.linear(xg, wg, bg)
    y.backward(dy.to(DEV, dtype))
    tol = _tol(dtype, 1e-4, 3e-2)
    _close(y, yr, tol, tol, "y")
    _close(xg.grad, xr.grad, tol, tol, "dx")
    _close(wg.grad, wr.grad, tol, tol, "dW")
    _close(bg.grad, br.grad, tol, tol, "db")


@pytest.mark.parametrize("low", LOW)
@pytest.mark.parametrize("B,H,W,nh,shift", ATTN_CASES)
def test_window_attention_bf16_grad(B, H, W, nh, shift, low):
    """bf16 MFMA attention (32x32x16, transposed scores) fwd + bwd vs the fp32 torchvision
    restatement; tolerance 3e-2 of the max magnitude (bf16 operands)."""
    ops = _ops()
    C = 32 * nh
    g = _g(5 * B * H * W + nh)
    qkv = torch.randn(B, H, W, 3 * C, generator=g)
    qb = 0.3 * torch.randn(3 * C, generator=g)
    table = torch.randn(169, nh, generator=g)
    dy = torch.randn(B, H, W, C, generator=g)
    q16 = qkv.to(low).float()  # reference sees the same rounded inputs
    qr, qbr, tr = [t.clone().requires_grad_(True) for t in (q16, qb, table)]
    # restatement driven directly with qkv: identity qkv projection
    index = osb.relative_position_index(7)
    x_eye = qr  # [B,H,W,3C] -> apply shifted_window_attention to q,k,v via a block-diagonal trick
    yr = _attn_ref_from_qkv(qr, qbr, tr, index, nh, shift)
    yr.backward(dy)
    qg = qkv.to(DEV, low).requires_grad_(True)
    qbg, tg = qb.to(DEV).requires_grad_(True), table.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=low):
        y = ops.window_attention(qg, qbg, tg, nh, shift)
    y.backward(dy.to(DEV, low))
    t = _tol(low, 0, 3e-2)
    _close(y, yr, t, t, "out")
    _close(qg.grad, qr.grad, t, t, "dqkv")
    _close(qbg.grad, qbr.grad, t, t, "dbias (padded tokens)")
    _close(tg.grad, tr.grad, t, t, "dtable")


def _attn_ref_from_qkv(qkv, qkv_bias, table, index, nh, shift):
    """torchvision semantics given the post-Linear qkv of real tokens (tests/_parity_refs.py)."""
    from _parity_refs import attn_ref_from_qkv
    return attn_ref_from_qkv(qkv, qkv_bias, table, nh, shift)


def test_window_attention_bf16_dropout_consistency():
    ops = _ops()
    B, H, W, nh, C = 2, 28, 28, 2, 64
    g = _g(77)
    qkv = torch.randn(B, H, W, 3 * C, generator=g).to(DEV, torch.bfloat16)
    qb = torch.zeros(3 * C, device=DEV)
    table = torch.zeros(169, nh, device=DEV)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y0 = ops.window_attention(qkv, qb, table, nh, 3, 0.0, 1).float()
        ys = torch.stack([ops.window_attention(qkv, qb, table, nh, 3, 0.25, s).float() for s in range(64)])
    rel = ((ys.mean(0) - y0).norm() / y0.norm()).item()
    assert rel < 0.1, rel
    q = qkv.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = ops.window_attention(q, qb, table, nh, 3, 0.5, 1234)
    dy = torch.randn(y.shape, generator=_g(78)).to(DEV, torch.bfloat16)
    y.backward(dy)
    # sum_i dy_i . y_i == sum_j dv_j . v_j holds exactly only when the backward regenerates
    # the forward's dropout mask; bf16 rounding of y and dv leaves noise that scales with
    # sum |dy . y| (~2^-8 per term, random signs), not with the (possibly small) total
    terms = dy.float() * y.float()
    lhs = terms.sum().item()
    rhs = (q.grad[..., 2 * C:].float() * q[..., 2 * C:].float()).sum().item()
    assert abs(lhs - rhs) <= 4e-3 * terms.abs().sum().item(), (lhs, rhs)
    # the masks are live: another seed gives another output, by O(1)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y2 = ops.window_attention(qkv, qb, table, nh, 3, 0.5, 4321)
    assert ((y2.float() - y.float()).norm() / y.float().norm()).item() > 0.3


@pytest.mark.parametrize("dtype", ALL)
def test_residual_add(dtype):
    """ops.residual_add = x + br * scale[sample] (StochasticDepth row scale) and its grads."""
    ops = _ops()
    g = _g(77)
    x = torch.randn(3, 9, 7, 16, generator=g)
    br = torch.randn(3, 9, 7, 16, generator=g)
    sc = torch.tensor([0.0, 1.25, 1.25])
    dy = torch.randn(3, 9, 7, 16, generator=g)
    xr, brr = x.clone().requires_grad_(True), br.clone().requires_grad_(True)
    yr = xr + brr * sc.view(-1, 1, 1, 1)
    yr.backward(dy)
    xg = x.to(DEV, dtype).requires_grad_(True)
    bg = br.to(DEV, dtype).requires_grad_(True)
    with torch.autocast("cuda", dtype=dtype, enabled=dtype != torch.float32):
        y = ops.residual_add(xg, bg, sc.to(DEV))
    y.backward(dy.to(DEV, dtype))
    tol = _tol(dtype, 1e-6, 1e-2)
    _close(y, yr, tol, tol, "y")
    _close(xg.grad, xr.grad, tol, tol, "dx")
    _close(bg.grad, brr.grad, tol, tol, "dbr")


def test_window_attention_param_tail_on_side_stream():
    """With direct .grad parameters the relative-table / qkv-bias gradient tail runs on the
    side stream (msu_win_attn_bwd2) and is added there: same gradients as the autograd path."""
    ops = _ops()
    B, H, W, nh, shift = 2, 20, 27, 2, 3
    C = 32 * nh
    g = _g(4242)
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
            y = ops.window_attention(q, pb, pt, nh, shift)
        y.backward(dy)
        torch.cuda.synchronize()
        res[direct] = (q.grad.float(), pb.grad.clone(), pt.grad.clone())
    for a, b, what in zip(res[True], res[False], ("dqkv", "dbias", "dtable")):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7, msg=what)


@pytest.mark.parametrize("d2s", [False, True])
def test_conv_tile_queue_equals_static_schedule(d2s):
    """The refine-conv kernel's device tile queue (msu_conv_mode 1, the default) against the
    static schedule (mode 0): bit-identical forward (dual) and dgrad at 1024 tiles > one
    workgroup per CU, over repeated launches (the queue slot resets itself at each launch's
    end) and on a second stream (its own slot)."""
    ops = _ops()
    from semantic_segmentation_of_stylegan2_artifacts_amd import _lib
    B, H, W, C = 8, 256, 256, 96
    g = _g(17 + d2s)
    x = torch.randn((B, H // 4, W // 4, 16 * C) if d2s else (B, H, W, C), generator=g).to(DEV, torch.bfloat16)
    a = torch.nn.functional.gelu(x.float()).to(torch.bfloat16)
    w = (torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)).to(DEV)
    b = (0.1 * torch.randn(C, generator=g)).to(DEV)
    dz = torch.randn(B, H, W, C, generator=g).to(DEV, torch.bfloat16)

    def run():
        xg = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            z, z2 = ops.refine_conv_act(xg, a, w, b, d2s, (H, W), dual=True)
        (dx,) = torch.autograd.grad(z, (xg,), dz)
        return z, z2, dx

    L = _lib.lib()
    prev = L.msu_conv_mode(0)
    try:
        ref = run()
        L.msu_conv_mode(1)
        outs = [run() for _ in range(3)]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            outs.append(run())
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
    finally:
        L.msu_conv_mode(prev)
    for o in outs:
        for u, r, name in zip(o, ref, ("z", "gelu(z)", "dx")):
            assert torch.equal(u, r), name
