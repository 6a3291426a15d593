"""Oracle: torchvision-v1 Swin block semantics, restated functionally (TEST INFRASTRUCTURE).

The reference instantiates ``torchvision.models.swin_transformer.SwinTransformerBlock``
at ``network/model_parts.py:143-151`` (encoder) and ``:511-519`` (decoder) and calls it at
``:170`` / ``:538``.  torchvision is a third-party dependency that is NOT present in
``/root/reference`` (nor installed in this image); the reference does not pin its version.
This module restates the published torchvision (>=0.13, "v1" block, no logit scale)
algorithm:

* ``shifted_window_attention``: pad (after norm1) to a multiple of the window,
  zero the shift on any axis where window >= padded size, roll(-shift), partition
  into windows, qkv = x W^T + b, q *= head_dim^-0.5, attn = q k^T + B_rel[idx],
  shift mask (-100 where region ids differ, regions defined on the padded grid),
  softmax, dropout, @v, proj, un-partition, roll(+shift), crop.
* ``StochasticDepth(p, "row")``: per-sample Bernoulli(1-p)/(1-p) in training.
* ``MLP``: Linear(C,4C) -> GELU(erf) -> Dropout -> Linear(4C,C) -> Dropout
  (state-dict keys ``mlp.0`` / ``mlp.3``, ``structure_of_MSUNet.txt:14-17``).

Parity status: UNPINNED by any reference test/fixture (none exist);
only the parameter layout is pinned (``relative_position_index`` int64 [2401],
``relative_position_bias_table`` [169, heads]).
"""
import torch
import torch.nn.functional as F


def relative_position_index(ws: int = 7) -> torch.Tensor:
    """torchvision ``define_relative_position_index``: (dh + ws-1)*(2ws-1) + (dw + ws-1)."""
    coords = torch.stack(torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij"))
    flat = coords.flatten(1)
    rel = (flat[:, :, None] - flat[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += ws - 1
    rel[:, :, 1] += ws - 1
    rel[:, :, 0] *= 2 * ws - 1
    return rel.sum(-1).flatten()


def relative_position_bias(table: torch.Tensor, index: torch.Tensor, ws: int) -> torch.Tensor:
    n = ws * ws
    return table[index].view(n, n, -1).permute(2, 0, 1).contiguous().unsqueeze(0)


def shift_mask(pad_h: int, pad_w: int, ws: int, shift, dtype=torch.float32) -> torch.Tensor:
    """[num_windows, ws*ws, ws*ws] additive mask (0 / -100) on the padded, rolled grid."""
    m = torch.zeros((pad_h, pad_w), dtype=dtype)
    hs = ((0, -ws), (-ws, -shift[0]), (-shift[0], None))
    wsl = ((0, -ws), (-ws, -shift[1]), (-shift[1], None))
    cnt = 0
    for h in hs:
        for w in wsl:
            m[h[0]:h[1], w[0]:w[1]] = cnt
            cnt += 1
    nw = (pad_h // ws) * (pad_w // ws)
    m = m.view(pad_h // ws, ws, pad_w // ws, ws).permute(0, 2, 1, 3).reshape(nw, ws * ws)
    m = m.unsqueeze(1) - m.unsqueeze(2)
    return m.masked_fill(m != 0, -100.0).masked_fill(m == 0, 0.0)


def effective_shift(h: int, w: int, ws: int, shift: int):
    pad_h = h + (ws - h % ws) % ws
    pad_w = w + (ws - w % ws) % ws
    sh = 0 if ws >= pad_h else shift
    sw = 0 if ws >= pad_w else shift
    return pad_h, pad_w, [sh, sw]


def shifted_window_attention(x, qkv_w, qkv_b, proj_w, proj_b, table, index, ws, num_heads,
                             shift, attn_drop=0.0, training=False, generator=None):
    """x: [B, H, W, C] (already normed by norm1).  Returns [B, H, W, C]."""
    B, H, W, C = x.shape
    pad_r = (ws - W % ws) % ws
    pad_b = (ws - H % ws) % ws
    x = F.pad(x, (0, 0, 0, pad_r, 0, pad_b))
    _, pH, pW, _ = x.shape
    _, _, sh = effective_shift(H, W, ws, shift)
    if sum(sh) > 0:
        x = torch.roll(x, shifts=(-sh[0], -sh[1]), dims=(1, 2))
    nW = (pH // ws) * (pW // ws)
    x = x.view(B, pH // ws, ws, pW // ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B * nW, ws * ws, C)
    qkv = F.linear(x, qkv_w, qkv_b)
    qkv = qkv.reshape(x.size(0), x.size(1), 3, num_heads, C // num_heads).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    q = q * (C // num_heads) ** -0.5
    attn = q.matmul(k.transpose(-2, -1))
    attn = attn + relative_position_bias(table, index, ws)
    if sum(sh) > 0:
        mask = shift_mask(pH, pW, ws, sh, dtype=attn.dtype)
        attn = attn.view(x.size(0) // nW, nW, num_heads, x.size(1), x.size(1))
        attn = attn + mask.unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, num_heads, x.size(1), x.size(1))
    attn = F.softmax(attn, dim=-1)
    if training and attn_drop > 0:
        keep = (torch.rand(attn.shape, generator=generator) >= attn_drop).to(attn.dtype)
        attn = attn * keep / (1.0 - attn_drop)
    x = attn.matmul(v).transpose(1, 2).reshape(x.size(0), x.size(1), C)
    x = F.linear(x, proj_w, proj_b)
    x = x.view(B, pH // ws, pW // ws, ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B, pH, pW, C)
    if sum(sh) > 0:
        x = torch.roll(x, shifts=(sh[0], sh[1]), dims=(1, 2))
    return x[:, :H, :W, :].contiguous()


def stochastic_depth(x, p, training, generator=None):
    if not training or p == 0.0:
        return x
    survival = 1.0 - p
    noise = torch.empty([x.shape[0]] + [1] * (x.ndim - 1), dtype=x.dtype)
    noise.bernoulli_(survival, generator=generator)
    if survival > 0.0:
        noise.div_(survival)
    return x * noise


def swin_block(p: dict, prefix: str, x, num_heads: int, ws: int, shift: int,
               drop_path=0.0, attn_drop=0.0, training=False, generator=None):
    """torchvision ``SwinTransformerBlock.forward`` on x [B, H, W, C] with params ``p[prefix+...]``."""
    C = x.shape[-1]
    g = lambda n: p[prefix + n]
    xn = F.layer_norm(x, (C,), g("norm1.weight"), g("norm1.bias"), 1e-5)
    a = shifted_window_attention(xn, g("attn.qkv.weight"), g("attn.qkv.bias"),
                                 g("attn.proj.weight"), g("attn.proj.bias"),
                                 g("attn.relative_position_bias_table"),
                                 g("attn.relative_position_index"), ws, num_heads, shift,
                                 attn_drop, training, generator)
    x = x + stochastic_depth(a, drop_path, training, generator)
    xn = F.layer_norm(x, (C,), g("norm2.weight"), g("norm2.bias"), 1e-5)
    h = F.gelu(F.linear(xn, g("mlp.0.weight"), g("mlp.0.bias")))
    m = F.linear(h, g("mlp.3.weight"), g("mlp.3.bias"))
    return x + stochastic_depth(m, drop_path, training, generator)
