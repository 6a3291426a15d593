"""Oracle: functional restatement of MS-UNet (TEST INFRASTRUCTURE ONLY).

Follows ``/root/reference/network/model_parts.py::MSUNetSys`` (543-894) and
``network/MSUNet.py::MSUNet`` (16-58).  Parameters live in a flat ``dict`` keyed exactly
like the reference ``MSUNetSys.state_dict()`` (``structure_of_MSUNet.txt``); the forward is
plain PyTorch fp32 so it is differentiable on the CPU for gradient parity.

Topology (pinned by ``tests/golden`` vectors produced by importing the reference
``model_parts.py`` with this package's Swin block standing in for torchvision):

* PatchEmbed ``:217-225``: conv k=s=patch, flatten, LN.
* encoder ``forward_features`` ``:775-815``: before stage 1 run ``layers_cent2``
  (``:785-795``), before stage 2 run ``layers_cent1`` (``:797-807``); these rewrite
  ``x_downsample`` entries through the *shared* ``concat_back_dim[i+2]`` / ``[i+1]``.
  The last entry of each central decoder is dead compute (output discarded).
* decoder ``forward_up_features`` ``:818-829``; head ``up_x4`` ``:832-848`` with
  ``FinalPatchExpand_X4_V2`` ``:451-476`` and the 1x1 ``output`` conv ``:751``.
"""
import math
from collections import OrderedDict

import torch
import torch.nn.functional as F
from einops import rearrange

from .swin_block import relative_position_index, swin_block

SWIN_T = dict(embed_dim=96, depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24])
SWIN_S = dict(embed_dim=96, depths=[2, 2, 18, 2], num_heads=[3, 6, 12, 24])
SWIN_B = dict(embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32])


def make_cfg(img_size=224, embed_dim=96, depths=(2, 2, 6, 2), num_heads=(3, 6, 12, 24),
             patch_size=4, in_chans=3, num_classes=1, window_size=7, mlp_ratio=4.0,
             drop_path_rate=0.1, attn_drop_rate=0.0, drop_rate=0.0):
    return dict(img_size=img_size, embed_dim=embed_dim, depths=list(depths),
                num_heads=list(num_heads), patch_size=patch_size, in_chans=in_chans,
                num_classes=num_classes, window_size=window_size, mlp_ratio=mlp_ratio,
                drop_path_rate=drop_path_rate, attn_drop_rate=attn_drop_rate,
                drop_rate=drop_rate)


# ----------------------------------------------------------------------------- params
def _block_spec(prefix, dim, heads, hidden, ws):
    n = (2 * ws - 1) ** 2
    return [
        (prefix + "norm1.weight", (dim,)), (prefix + "norm1.bias", (dim,)),
        (prefix + "attn.relative_position_bias_table", (n, heads)),
        (prefix + "attn.relative_position_index", (ws ** 4,)),
        (prefix + "attn.qkv.weight", (3 * dim, dim)), (prefix + "attn.qkv.bias", (3 * dim,)),
        (prefix + "attn.proj.weight", (dim, dim)), (prefix + "attn.proj.bias", (dim,)),
        (prefix + "norm2.weight", (dim,)), (prefix + "norm2.bias", (dim,)),
        (prefix + "mlp.0.weight", (hidden, dim)), (prefix + "mlp.0.bias", (hidden,)),
        (prefix + "mlp.3.weight", (dim, hidden)), (prefix + "mlp.3.bias", (dim,)),
    ]


def _expand_spec(prefix, dim):
    return [(prefix + "expand.weight", (2 * dim, dim)),
            (prefix + "norm.weight", (dim // 2,)), (prefix + "norm.bias", (dim // 2,))]


def _layer_up_spec(prefix, dim, depth, heads, cfg, upsample):
    hidden = int(dim * cfg["mlp_ratio"])
    out = []
    for j in range(depth):
        out += _block_spec(f"{prefix}blocks.{j}.", dim, heads, hidden, cfg["window_size"])
    if upsample:
        out += _expand_spec(prefix + "upsample.", dim)
    return out


def param_spec(cfg):
    """(name, shape) in ``MSUNetSys.state_dict()`` order (own params, buffers, children)."""
    C, L = cfg["embed_dim"], len(cfg["depths"])
    ps, ws = cfg["patch_size"], cfg["window_size"]
    spec = [("patch_embed.proj.weight", (C, cfg["in_chans"], ps, ps)),
            ("patch_embed.proj.bias", (C,)),
            ("patch_embed.norm.weight", (C,)), ("patch_embed.norm.bias", (C,))]
    for i in range(L):
        dim = C * 2 ** i
        hidden = int(dim * cfg["mlp_ratio"])
        for j in range(cfg["depths"][i]):
            spec += _block_spec(f"layers.{i}.blocks.{j}.", dim, cfg["num_heads"][i], hidden, ws)
        if i < L - 1:
            spec += [(f"layers.{i}.downsample.reduction.weight", (2 * dim, 4 * dim)),
                     (f"layers.{i}.downsample.norm.weight", (4 * dim,)),
                     (f"layers.{i}.downsample.norm.bias", (4 * dim,))]
    for k in range(L):  # layers_up
        s = L - 1 - k
        dim = C * 2 ** s
        if k == 0:
            spec += _expand_spec("layers_up.0.", dim)
        else:
            spec += _layer_up_spec(f"layers_up.{k}.", dim, cfg["depths"][s], cfg["num_heads"][s],
                                   cfg, upsample=k < L - 1)
    for k in range(1, L):  # concat_back_dim (index 0 is Identity)
        dim = C * 2 ** (L - 1 - k)
        spec += [(f"concat_back_dim.{k}.weight", (dim, 2 * dim)), (f"concat_back_dim.{k}.bias", (dim,))]
    for k in range(L - 1):  # layers_cent1
        s = L - 2 - k
        dim = C * 2 ** s
        if k == 0:
            spec += _expand_spec("layers_cent1.0.", dim)
        else:
            spec += _layer_up_spec(f"layers_cent1.{k}.", dim, cfg["depths"][s], cfg["num_heads"][s],
                                   cfg, upsample=k < L - 2)
    for k in range(L - 2):  # layers_cent2
        s = L - 3 - k
        dim = C * 2 ** s
        if k == 0:
            spec += _expand_spec("layers_cent2.0.", dim)
        else:
            spec += _layer_up_spec(f"layers_cent2.{k}.", dim, cfg["depths"][s], cfg["num_heads"][s],
                                   cfg, upsample=k < L - 3)
    nf = C * 2 ** (L - 1)
    spec += [("norm.weight", (nf,)), ("norm.bias", (nf,)),
             ("norm_up.weight", (C,)), ("norm_up.bias", (C,)),
             ("up.expand.weight", (16 * C, C)),
             ("up.refine1.weight", (C, C, 3, 3)), ("up.refine1.bias", (C,)),
             ("up.refine2.weight", (C, C, 3, 3)), ("up.refine2.bias", (C,)),
             ("up.norm.weight", (C,)), ("up.norm.bias", (C,)),
             ("output.weight", (cfg["num_classes"], C, 1, 1))]
    return spec


def dead_prefixes(cfg):
    """Modules whose outputs the reference discards (``model_parts.py:795,807``)."""
    L = len(cfg["depths"])
    return [f"layers_cent1.{L - 2}.", f"layers_cent2.{L - 3}."]


def init_params(cfg, seed=0, scale=1.0):
    """Deterministic test parameters (CPU generator).  Not the reference init: LayerNorm
    affine and every bias are randomised too, so that tests exercise them."""
    g = torch.Generator().manual_seed(seed)
    p = OrderedDict()
    for name, shape in param_spec(cfg):
        if name.endswith("relative_position_index"):
            p[name] = relative_position_index(cfg["window_size"])
        elif name.endswith("relative_position_bias_table"):
            p[name] = torch.randn(shape, generator=g) * 0.5 * scale
        elif ".norm" in name and name.endswith(".weight") or name.startswith("norm"):
            if name.endswith(".weight"):
                p[name] = 1.0 + 0.1 * torch.randn(shape, generator=g)
            else:
                p[name] = 0.1 * torch.randn(shape, generator=g)
        elif name.endswith(".bias"):
            p[name] = 0.05 * torch.randn(shape, generator=g)
        else:
            fan_in = math.prod(shape[1:])
            p[name] = torch.randn(shape, generator=g) * (scale / math.sqrt(fan_in))
    return p


# ----------------------------------------------------------------------------- forward
def _ln(x, p, prefix):
    return F.layer_norm(x, (x.shape[-1],), p[prefix + "weight"], p[prefix + "bias"], 1e-5)


def patch_expand(p, prefix, x, res):
    """``PatchExpand.forward`` ``model_parts.py:382-407`` (x: [B, L, C] or [B, H, W, C])."""
    B = x.shape[0]
    H, W = res
    x = x.reshape(B, H * W, x.shape[-1])
    x = F.linear(x, p[prefix + "expand.weight"])
    C = x.shape[-1]
    x = x.view(B, H, W, C)
    x = rearrange(x, "b h w (p1 p2 c)-> b (h p1) (w p2) c", p1=2, p2=2, c=C // 4)
    x = x.reshape(B, -1, C // 4)
    return _ln(x, p, prefix + "norm.")


def patch_merging(p, prefix, x, res):
    """``PatchMerging.forward`` ``model_parts.py:75-97`` (x: [B, H, W, C])."""
    B, H, W, C = x.shape
    assert (H, W) == tuple(res)
    x0 = x[:, 0::2, 0::2, :]
    x1 = x[:, 1::2, 0::2, :]
    x2 = x[:, 0::2, 1::2, :]
    x3 = x[:, 1::2, 1::2, :]
    x = torch.cat([x0, x1, x2, x3], -1).view(B, -1, 4 * C)
    x = _ln(x, p, prefix + "norm.")
    return F.linear(x, p[prefix + "reduction.weight"])


def _drop_path_list(cfg):
    d = cfg["depths"]
    return [v.item() for v in torch.linspace(0, cfg["drop_path_rate"], sum(d))]


def basic_layer(p, prefix, x, cfg, stage, train_opts, resample):
    """``BasicLayer.forward`` ``:160-173`` / ``BasicLayer_up.forward`` ``:528-541``.
    x: [B, L, C] -> 4-D [B, H, W, C] if no resampler, else the resampler's 3-D output."""
    res0 = cfg["img_size"] // cfg["patch_size"]
    H = W = res0 // 2 ** stage
    B, _, C = x.reshape(x.shape[0], -1, x.shape[-1]).shape
    x = x.reshape(B, H, W, C)
    dpr = _drop_path_list(cfg)
    d0 = sum(cfg["depths"][:stage])
    training, gen = train_opts.get("training", False), train_opts.get("generator")
    for j in range(cfg["depths"][stage]):
        shift = 0 if j % 2 == 0 else cfg["window_size"] // 2
        x = swin_block(p, f"{prefix}blocks.{j}.", x, cfg["num_heads"][stage], cfg["window_size"],
                       shift, drop_path=dpr[d0 + j] if training else 0.0,
                       attn_drop=cfg["attn_drop_rate"] if training else 0.0,
                       training=training, generator=gen)
    if resample == "down":
        x = patch_merging(p, prefix + "downsample.", x, (H, W))
    elif resample == "up":
        x = patch_expand(p, prefix + "upsample.", x, (H, W))
    return x


def forward_features(p, cfg, x, train_opts):
    """``MSUNetSys.forward_features`` ``:775-815``."""
    C, L = cfg["embed_dim"], len(cfg["depths"])
    ps = cfg["patch_size"]
    res0 = cfg["img_size"] // ps
    x = F.conv2d(x, p["patch_embed.proj.weight"], p["patch_embed.proj.bias"], stride=ps)
    x = x.flatten(2).transpose(1, 2)
    x = _ln(x, p, "patch_embed.norm.")
    xd = []
    for i in range(L):
        if i == 1:
            x2 = x
            for k in range(L - 2):
                s = L - 3 - k
                if k == 0:
                    x2 = patch_expand(p, "layers_cent2.0.", x2, (res0 // 2 ** s,) * 2)
                else:
                    x2 = torch.cat([x2.reshape(x2.shape[0], -1, x2.shape[-1]), xd[i - k]], -1)
                    x2 = F.linear(x2, p[f"concat_back_dim.{k + 2}.weight"], p[f"concat_back_dim.{k + 2}.bias"])
                    xd[i - k] = x2
                    x2 = basic_layer(p, f"layers_cent2.{k}.", x2, cfg, s, train_opts,
                                     "up" if k < L - 3 else None)
        if i == 2:
            x1 = x
            for k in range(L - 1):
                s = L - 2 - k
                if k == 0:
                    x1 = patch_expand(p, "layers_cent1.0.", x1, (res0 // 2 ** s,) * 2)
                else:
                    x1 = torch.cat([x1.reshape(x1.shape[0], -1, x1.shape[-1]), xd[i - k]], -1)
                    x1 = F.linear(x1, p[f"concat_back_dim.{k + 1}.weight"], p[f"concat_back_dim.{k + 1}.bias"])
                    xd[i - k] = x1
                    x1 = basic_layer(p, f"layers_cent1.{k}.", x1, cfg, s, train_opts,
                                     "up" if k < L - 2 else None)
        xd.append(x)
        x = basic_layer(p, f"layers.{i}.", x, cfg, i, train_opts, "down" if i < L - 1 else None)
    x = _ln(x, p, "norm.")
    return x, xd


def forward_up_features(p, cfg, x, xd, train_opts):
    """``MSUNetSys.forward_up_features`` ``:818-829``."""
    L = len(cfg["depths"])
    res0 = cfg["img_size"] // cfg["patch_size"]
    for k in range(L):
        s = L - 1 - k
        if k == 0:
            x = patch_expand(p, "layers_up.0.", x, (res0 // 2 ** s,) * 2)
        else:
            x = torch.cat([x.reshape(x.shape[0], -1, x.shape[-1]), xd[3 - k]], -1)
            x = F.linear(x, p[f"concat_back_dim.{k}.weight"], p[f"concat_back_dim.{k}.bias"])
            x = basic_layer(p, f"layers_up.{k}.", x, cfg, s, train_opts, "up" if k < L - 1 else None)
    return _ln(x, p, "norm_up.")


def final_expand_x4(p, prefix, x, res, C):
    """``FinalPatchExpand_X4_V2.forward`` ``:451-476``; x [B, H*W, C] -> [B, 16*H*W, C]."""
    H, W = res
    B = x.shape[0]
    x = x.reshape(B, H * W, C)
    x = F.gelu(F.linear(x, p[prefix + "expand.weight"]))
    x = x.reshape(B, H, W, 16 * C)
    x = rearrange(x, "b h w (p1 p2 c) -> b (h p1) (w p2) c", p1=4, p2=4, c=C)
    x = x.permute(0, 3, 1, 2).contiguous()
    x = F.gelu(F.conv2d(x, p[prefix + "refine1.weight"], p[prefix + "refine1.bias"], padding=1))
    x = F.conv2d(x, p[prefix + "refine2.weight"], p[prefix + "refine2.bias"], padding=1)
    x = x.permute(0, 2, 3, 1).contiguous().reshape(B, -1, C)
    return _ln(x, p, prefix + "norm.")


def up_x4(p, cfg, x):
    """``MSUNetSys.up_x4`` ``:832-848``."""
    C = cfg["embed_dim"]
    H = W = cfg["img_size"] // cfg["patch_size"]
    B = x.shape[0]
    x = final_expand_x4(p, "up.", x, (H, W), C)
    x = x.view(B, 4 * H, 4 * W, -1).permute(0, 3, 1, 2)
    return F.conv2d(x, p["output.weight"])


def msunet_forward(p, cfg, x, training=False, generator=None):
    """``MSUNet.forward`` ``network/MSUNet.py:47-52`` -> ``MSUNetSys.forward`` ``:850-855``."""
    if x.size(1) != 3:
        raise ValueError(f"Expected 3 channels, but got {x.size(1)}")
    opts = dict(training=training, generator=generator)
    x, xd = forward_features(p, cfg, x, opts)
    x = forward_up_features(p, cfg, x, xd, opts)
    return up_x4(p, cfg, x)
