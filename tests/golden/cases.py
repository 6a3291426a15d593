"""Seeded inputs for the golden fixtures (shared by gen_golden.py and the tests).

Everything here is regenerated from CPU ``torch.Generator`` seeds, so the committed
fixtures only hold reference OUTPUTS.  No dependency on /root/reference.
"""
import math

import torch

from oracle.msunet import init_params

FULL_GRAD_KEYS = [
    "output.weight", "up.norm.weight", "up.refine2.bias", "patch_embed.proj.weight",
    "layers.0.blocks.1.attn.relative_position_bias_table", "concat_back_dim.3.bias",
    "layers_cent1.0.norm.weight", "layers.3.blocks.0.attn.qkv.bias",
]


def _g(seed):
    return torch.Generator().manual_seed(seed)


def blob_masks(B, H, W, seed, fake=None):
    """Binary masks [B, H, W] f32: 'fake' samples get 1-4 filled ellipses, 'real' are empty."""
    g = _g(seed)
    yy, xx = torch.meshgrid(torch.arange(H, dtype=torch.float32),
                            torch.arange(W, dtype=torch.float32), indexing="ij")
    out = torch.zeros(B, H, W)
    for b in range(B):
        is_fake = fake[b] if fake is not None else True
        if not is_fake:
            continue
        n = int(torch.randint(1, 5, (1,), generator=g))
        for _ in range(n):
            cy, cx = float(torch.rand(1, generator=g)) * H, float(torch.rand(1, generator=g)) * W
            ry = 2 + float(torch.rand(1, generator=g)) * H / 8
            rx = 2 + float(torch.rand(1, generator=g)) * W / 8
            out[b][((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1.0] = 1.0
    return out


def loss_cases():
    g = _g(0)
    B, H, W = 4, 64, 64
    logits = torch.randn(B, 1, H, W, generator=g) * 3.0
    masks = blob_masks(B, H, W, 1, fake=[True, False, True, False])
    kw = dict(alpha=0.2, beta=0.8, mix=0.45)
    return {
        "mixed3d": (logits, masks.clone(), kw),
        "mixed4d": (logits, masks.unsqueeze(1).clone(), kw),
        "u8_0_255": (logits, masks * 255.0, kw),
        "all_empty": (logits, torch.zeros(B, H, W), kw),
        "all_fake_defaults": (logits * 0.5, blob_masks(B, H, W, 2), dict(alpha=0.4, beta=0.6, mix=0.5)),
        "single": (logits[:1] - 2.0, masks[:1], kw),
    }


def op_cases():
    g = _g(3)
    return {
        "merge_8x8_c16": ("merge", dict(res=(8, 8), dim=16), torch.randn(2, 8, 8, 16, generator=g)),
        "merge_14x14_c32": ("merge", dict(res=(14, 14), dim=32), torch.randn(1, 14, 14, 32, generator=g)),
        "expand_4x4_c32_3d": ("expand", dict(res=(4, 4), dim=32), torch.randn(2, 16, 32, generator=g)),
        "expand_7x7_c64_4d": ("expand", dict(res=(7, 7), dim=64), torch.randn(1, 7, 7, 64, generator=g)),
        "final_6x6_c16": ("final", dict(res=(6, 6), dim=16), torch.randn(2, 36, 16, generator=g)),
        "final_8x5_c32": ("final", dict(res=(8, 5), dim=32), torch.randn(1, 40, 32, generator=g)),
    }


def op_params(kind, args):
    g = _g(4)
    d = args["dim"]
    rn = lambda *s: torch.randn(*s, generator=g)
    if kind == "merge":
        return {"reduction.weight": rn(2 * d, 4 * d) / math.sqrt(4 * d),
                "norm.weight": 1 + 0.1 * rn(4 * d), "norm.bias": 0.1 * rn(4 * d)}
    if kind == "expand":
        return {"expand.weight": rn(2 * d, d) / math.sqrt(d),
                "norm.weight": 1 + 0.1 * rn(d // 2), "norm.bias": 0.1 * rn(d // 2)}
    return {"expand.weight": rn(16 * d, d) / math.sqrt(d),
            "refine1.weight": rn(d, d, 3, 3) / math.sqrt(9 * d), "refine1.bias": 0.05 * rn(d),
            "refine2.weight": rn(d, d, 3, 3) / math.sqrt(9 * d), "refine2.bias": 0.05 * rn(d),
            "norm.weight": 1 + 0.1 * rn(d), "norm.bias": 0.1 * rn(d)}


def op_upstream(y):
    g = _g(5)
    return torch.randn(y.shape, generator=g)


def model_cases():
    return {
        "tiny224": dict(cfg=dict(img_size=224, embed_dim=32, depths=[2, 2, 2, 2],
                                 num_heads=[1, 2, 4, 8], drop_path_rate=0.0), batch=2, seed=11),
        "tiny256": dict(cfg=dict(img_size=256, embed_dim=32, depths=[2, 2, 2, 2],
                                 num_heads=[1, 2, 4, 8], drop_path_rate=0.0), batch=1, seed=12),
        "swinT224": dict(cfg=dict(img_size=224, embed_dim=96, depths=[2, 2, 2, 2],
                                  num_heads=[3, 6, 12, 24], drop_path_rate=0.0), batch=1, seed=13),
        # the Swin-S / Swin-B stacks (depth-18 stage 2, C=128 for B) at 224^2
        "swinS224": dict(cfg=dict(img_size=224, embed_dim=96, depths=[2, 2, 18, 2],
                                  num_heads=[3, 6, 12, 24], drop_path_rate=0.0), batch=1, seed=14),
        "swinB224": dict(cfg=dict(img_size=224, embed_dim=128, depths=[2, 2, 18, 2],
                                  num_heads=[4, 8, 16, 32], drop_path_rate=0.0), batch=2, seed=15),
    }


def model_params(cfg, seed):
    return init_params(cfg, seed)


def model_inputs(cfg, batch, seed):
    g = _g(seed + 1000)
    n = cfg["img_size"]
    x = torch.floor(torch.rand(batch, 3, n, n, generator=g) * 256.0).clamp(max=255) / 255.0
    fake = [b % 2 == 0 for b in range(batch)]
    target = blob_masks(batch, n, n, seed + 2000, fake=fake)
    return x, target
