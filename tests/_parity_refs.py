"""Plain fp32 PyTorch references shared by the GPU parity tests (test infrastructure only).

* ``attn_ref_from_qkv``: torchvision v1 ``shifted_window_attention`` (restated in
  oracle/swin_block.py, which cites it) driven by the post-Linear qkv of the real tokens, with
  an optional dropout keep mask on the softmax probabilities (``F.dropout`` after the softmax,
  kept values scaled by 1 / (1 - p)).
* ``decode_keep_bits``: the 16-bit attention forward's stored keep bits
  (csrc/window_attention_mfma.hip, ``[window x head][query tile][lane]`` words; bit jt*16 + r of
  lane l in tile it <-> query 32 it + (l & 31), key 32 jt + crow(r, l >> 5)) -> [items, 49, 49].
* ``conv3x3_ref``: ``conv2d(a, W, b, padding=1)`` on NHWC tensors as nine shifted fp32
  matmuls (autograd gives dA, dW, db), so the 1024^2 references need neither the CPU nor a
  library convolution.
"""
import math

import torch
import torch.nn.functional as F

from oracle import swin_block as osb


def gelu_grad(h):
    return 0.5 * (1.0 + torch.erf(h / math.sqrt(2.0))) + h * torch.exp(-0.5 * h * h) / math.sqrt(2.0 * math.pi)


def decode_keep_bits(keep, n_items):
    """[n_items * 128] int32 keep words -> bool [n_items, 49, 49] (query, key)."""
    dev = keep.device
    it, lane, b = torch.meshgrid(torch.arange(2), torch.arange(64), torch.arange(32), indexing="ij")
    r = b & 15
    i = (32 * it + (lane & 31)).reshape(-1).to(dev)
    j = (32 * (b >> 4) + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)).reshape(-1).to(dev)
    bits = ((keep.view(n_items, 2, 64, 1) >> torch.arange(32, device=dev, dtype=torch.int32)) & 1).bool()
    full = torch.zeros(n_items, 64, 64, dtype=torch.bool, device=dev)
    full[:, i, j] = bits.reshape(n_items, -1)
    return full[:, :49, :49]


def attn_ref_from_qkv(qkv, qkv_bias, table, nh, shift, keep=None, p_drop=0.0):
    """torchvision semantics given the post-Linear qkv of real tokens; padded tokens take
    qkv_bias (= Linear of the zero pad).  keep: bool [windows * nh, 49, 49] dropout mask in the
    kernels' (window, head) item order, or None."""
    B, H, W, C3 = qkv.shape
    C = C3 // 3
    ws = 7
    pad_r, pad_b = (ws - W % ws) % ws, (ws - H % ws) % ws
    x = F.pad(qkv - qkv_bias, (0, 0, 0, pad_r, 0, pad_b)) + qkv_bias
    _, pH, pW, _ = x.shape
    _, _, sh = osb.effective_shift(H, W, ws, shift)
    if sum(sh) > 0:
        x = torch.roll(x, shifts=(-sh[0], -sh[1]), dims=(1, 2))
    nW = (pH // ws) * (pW // ws)
    x = x.view(B, pH // ws, ws, pW // ws, ws, C3).permute(0, 1, 3, 2, 4, 5).reshape(B * nW, ws * ws, C3)
    qkv_ = x.reshape(x.size(0), x.size(1), 3, nh, C // nh).permute(2, 0, 3, 1, 4)
    q, k, v = qkv_[0] * (C // nh) ** -0.5, qkv_[1], qkv_[2]
    attn = q.matmul(k.transpose(-2, -1)) + osb.relative_position_bias(table, index_for(table.device), ws)
    if sum(sh) > 0:
        mask = osb.shift_mask(pH, pW, ws, sh).to(attn.device)
        attn = attn.view(B, nW, nh, ws * ws, ws * ws) + mask.unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, nh, ws * ws, ws * ws)
    attn = torch.softmax(attn, -1)
    if keep is not None:
        attn = attn * keep.view(attn.shape).to(attn.dtype) * (1.0 / (1.0 - p_drop))
    o = attn.matmul(v).transpose(1, 2).reshape(B * nW, ws * ws, C)
    o = o.view(B, pH // ws, pW // ws, ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B, pH, pW, C)
    if sum(sh) > 0:
        o = torch.roll(o, shifts=(sh[0], sh[1]), dims=(1, 2))
    return o[:, :H, :W, :]


_INDEX = {}


def index_for(device):
    key = str(device)
    if key not in _INDEX:
        _INDEX[key] = osb.relative_position_index(7).to(device)
    return _INDEX[key]


def conv3x3_ref(a, w, b):
    """a: [B, H, W, Cin] f32, w: [Cout, Cin, 3, 3], b: [Cout] -> [B, H, W, Cout] (padding 1)."""
    B, H, W, _ = a.shape
    ap = F.pad(a, (0, 0, 1, 1, 1, 1))
    z = b.view(1, 1, 1, -1).expand(B, H, W, -1)
    for dy in range(3):
        for dx in range(3):
            z = z + ap[:, dy:dy + H, dx:dx + W, :].matmul(w[:, :, dy, dx].t())
    return z


def d2s4(x, C):
    """FinalPatchExpand_X4_V2's rearrange 'b h w (p1 p2 c) -> b (h p1) (w p2) c' (p = 4)."""
    B, h, w, _ = x.shape
    return x.view(B, h, w, 4, 4, C).permute(0, 1, 3, 2, 4, 5).reshape(B, 4 * h, 4 * w, C)
