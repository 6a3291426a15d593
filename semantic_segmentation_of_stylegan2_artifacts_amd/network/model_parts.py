"""MS-UNet building blocks on the gfx950 HIP kernels (drop-in for the reference's
``network/model_parts.py`` and the torchvision ``SwinTransformerBlock`` it imports).

Class names, constructor signatures, submodule names and the state-dict layout follow the
reference (``structure_of_MSUNet.txt``), so reference checkpoints load with
``strict=True``.  The forward passes are re-planned for MI355X rather than translated:

* activations stay channels-last ``[B, H, W, C]`` / ``[B, L, C]`` end to end;
* the window attention core never materialises pad / roll / partition (``ops.window_attention``);
* residual adds + StochasticDepth are fused into the next LayerNorm and chained across
  blocks (``SwinTransformerBlock.forward_fused``);
* PatchMerging's 2x2 gather and PatchExpand's depth-to-space are fused into their norms;
* FinalPatchExpand_X4_V2 runs expand -> [d2s + GELU fused into conv1's loads] -> conv1+bias
  -> [GELU fused into conv2's loads] -> conv2+bias -> LayerNorm fused with the 1x1 head.

Dense GEMMs (qkv / proj / MLP / merge reduction / expand / skip fusion / patch embed) are the
``torch.ops.msunet`` linear family (ops.py): the HIP token GEMM (gemm_tok.h) for the
HBM-bound stage-0/1 shapes and every fused epilogue (bias, GELU, GELU', skip concat), the HIP
weight-gradient kernel for every weight gradient, and the library GEMM (hipBLASLt) for the
remaining MFMA-bound stage-2/3 forward / input-gradient products.
"""
import math
import random

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


def _trunc_normal_(t, std=0.02):
    """timm ``trunc_normal_`` (cut at absolute +-2, as the reference's import)."""
    return nn.init.trunc_normal_(t, std=std)


def _to_2tuple(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


def _relative_position_index(ws):
    coords = torch.stack(torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij"))
    flat = coords.flatten(1)
    rel = (flat[:, :, None] - flat[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += ws - 1
    rel[:, :, 1] += ws - 1
    rel[:, :, 0] *= 2 * ws - 1
    return rel.sum(-1).flatten()


_seed_rng = random.Random(0x5EED)


def _next_seed():
    return _seed_rng.getrandbits(62)


def reseed(seed):
    """Restart the attention-dropout seed stream (per rank under data parallelism) and drop
    the pooled stochastic-depth draws made under the previous seed."""
    _seed_rng.seed(int(seed) ^ 0x5EED)
    _SCALE_POOL.clear()


# Device-resident dropout counter (int64 [1]) mixed into every attention-dropout seed when set:
# a trainer that replays its step from a HIP graph advances it inside the graph, so each replay
# draws new attention-dropout masks although the host-side seeds were fixed at capture.
_dev_seed = None


def set_device_seed(t):
    global _dev_seed
    _dev_seed = t


def refresh_drop_pools():
    """Redraw every stochastic-depth pool in place and restart its row cursor.  Called at the
    start of a captured training step: the draws become part of the graph (torch's generator is
    graph-safe), so every replay reads fresh scales from the same rows."""
    for (p, _, _, _), pool in _SCALE_POOL.items():
        survival = 1.0 - p
        pool[0].bernoulli_(survival)
        if survival > 0.0:
            pool[0].div_(survival)
        pool[1] = 0


_SCALE_POOL = {}
_POOL_ROWS = 64


def _drop_path_scale(p, training, B, device):
    """torchvision StochasticDepth(p, 'row'): per-sample Bernoulli(1-p)/(1-p) or None.
    Draws come from a per-(p, B, device) pool refilled 64 rows at a time (one Bernoulli
    kernel and one divide per 64 calls instead of three tiny kernels per call); each call
    takes a fresh row, so draws stay independent and identically distributed."""
    if not training or p == 0.0:
        return None
    survival = 1.0 - p
    device = torch.device(device)
    # one pool per stream: a row is read on the stream whose kernel produced it
    sid = torch.cuda.current_stream(device).stream_id if device.type == "cuda" else 0
    key = (float(p), int(B), str(device), sid)
    pool = _SCALE_POOL.get(key)
    if pool is None or pool[1] >= _POOL_ROWS:
        noise = torch.empty(_POOL_ROWS, B, device=device, dtype=torch.float32).bernoulli_(survival)
        if survival > 0.0:
            noise.div_(survival)
        pool = _SCALE_POOL[key] = [noise, 0]
    row = pool[0][pool[1]]
    pool[1] += 1
    return row


# ============================================================================ Swin block
class ShiftedWindowAttention(nn.Module):
    """Parameter layout of torchvision ``ShiftedWindowAttention`` (relative_position_bias_table,
    relative_position_index, qkv, proj); forward = qkv Linear -> fused window core -> proj."""

    def __init__(self, dim, window_size, shift_size, num_heads, qkv_bias=True, proj_bias=True,
                 attention_dropout=0.0, dropout=0.0):
        super().__init__()
        if len(window_size) != 2 or len(shift_size) != 2:
            raise ValueError("window_size and shift_size must be of length 2")
        if window_size[0] != 7 or window_size[1] != 7:
            raise ValueError("the gfx950 window-attention kernel is built for 7x7 windows")
        if shift_size[0] != shift_size[1]:
            raise ValueError("square shifts only")
        if dim % num_heads or dim // num_heads != 32:
            raise ValueError(f"head dim must be 32 (dim={dim}, heads={num_heads})")
        self.window_size = list(window_size)
        self.shift_size = list(shift_size)
        self.num_heads = num_heads
        self.attention_dropout = attention_dropout
        self.dropout = dropout
        ws = window_size[0]
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * ws - 1) ** 2, num_heads))
        _trunc_normal_(self.relative_position_bias_table, std=0.02)
        self.register_buffer("relative_position_index", _relative_position_index(ws))
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim, bias=proj_bias)

    def forward(self, x):
        """x: [B, H, W, C] (already norm1-ed)."""
        p = self.attention_dropout if self.training else 0.0
        if ops.window_attention_qkv_fusable(x, self.num_heads, self.qkv.bias) and self.proj.bias is not None:
            # stage 0: qkv Linear -> window attention -> proj Linear in one kernel (no qkv / o
            # round trip through HBM; ops.window_attention_qkv)
            o = ops.window_attention_qkv(x, self.qkv.weight, self.qkv.bias, self.relative_position_bias_table,
                                         self.num_heads, self.shift_size[0], p, _next_seed() if p > 0 else 0,
                                         _dev_seed if p > 0 else None, self.proj.weight, self.proj.bias)
            if self.dropout > 0 and self.training:
                o = F.dropout(o, self.dropout, True)
            return o
        else:
            qkv = ops.linear(x, self.qkv.weight, self.qkv.bias)
            qb = self.qkv.bias if self.qkv.bias is not None else torch.zeros(
                3 * x.shape[-1], device=x.device, dtype=torch.float32)
            o = ops.window_attention(qkv, qb, self.relative_position_bias_table, self.num_heads,
                                     self.shift_size[0], p, _next_seed() if p > 0 else 0,
                                     _dev_seed if p > 0 else None)
        o = ops.linear(o, self.proj.weight, self.proj.bias)
        if self.dropout > 0 and self.training:
            o = F.dropout(o, self.dropout, True)
        return o


class SwinTransformerBlock(nn.Module):
    """torchvision ``SwinTransformerBlock`` (v1) drop-in: keys norm1 / attn / norm2 / mlp.0 / mlp.3."""

    def __init__(self, dim, num_heads, window_size, shift_size, mlp_ratio=4.0, dropout=0.0,
                 attention_dropout=0.0, stochastic_depth_prob=0.0, norm_layer=nn.LayerNorm):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.attn = ShiftedWindowAttention(dim, window_size, shift_size, num_heads,
                                           attention_dropout=attention_dropout, dropout=dropout)
        self.stochastic_depth_prob = stochastic_depth_prob
        self.norm2 = norm_layer(dim)
        hidden = int(dim * mlp_ratio)
        self.mlp = nn.Sequential(nn.Linear(dim, hidden), nn.GELU(), nn.Dropout(dropout),
                                 nn.Linear(hidden, dim), nn.Dropout(dropout))
        self.dropout = dropout
        for m in self.mlp.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    nn.init.normal_(m.bias, std=1e-6)

    def forward_fused(self, state, hk=0):
        """state: a residual-stream tensor [B, H, W, C] or a pending ``(x, branch, scale)``
        whose add is fused into this block's norm1.  Returns this block's pending state.  hk:
        the handoff key of a plain-tensor state shared with its other readers outside the block
        (MSUNetSys.forward_features), else 0 (a fresh key pairs norm1 and norm2 only)."""
        if isinstance(state, tuple):
            x, br, sc = state
            x, xn = ops.add_layer_norm(x, br, sc, self.norm1.weight, self.norm1.bias, self.norm1.eps)
        else:
            # x's two readers (norm1, norm2's residual add) sum their gradients inside norm1's
            # LayerNorm backward (ops.residual_handoff_key), not in an autograd add
            x = state
            hk = hk or ops.residual_handoff_key()
            xn = ops.layer_norm(x, self.norm1.weight, self.norm1.bias, self.norm1.eps, handoff=hk)
        B = x.shape[0]
        a = self.attn(xn)
        sc1 = _drop_path_scale(self.stochastic_depth_prob, self.training, B, x.device)
        fc1, fc2 = self.mlp[0], self.mlp[3]
        drop = self.dropout > 0 and self.training
        if not drop and not torch.is_grad_enabled():
            # no-grad blocks (the reference's discarded branches): norm2's residual-add LayerNorm
            # and the MLP in one kernel when covered
            r = ops.add_layer_norm_mlp(x, a, sc1, self.norm2.weight, self.norm2.bias, self.norm2.eps,
                                       fc1.weight, fc1.bias, fc2.weight, fc2.bias)
            if r is not None:
                sc2 = _drop_path_scale(self.stochastic_depth_prob, self.training, B, x.device)
                return (r[0], r[1], sc2)
        x1, xn2 = ops.add_layer_norm(x, a, sc1, self.norm2.weight, self.norm2.bias, self.norm2.eps, handoff=hk)
        if not drop and fc1.bias is not None and fc2.bias is not None and \
                ops.mlp_fusable(xn2, fc1.weight, fc2.weight):
            m = ops.mlp(xn2, fc1.weight, fc1.bias, fc2.weight, fc2.bias)
        else:
            h = ops.gelu(ops.linear(xn2, fc1.weight, fc1.bias))
            if drop:
                h = F.dropout(h, self.dropout, True)
            m = ops.linear(h, fc2.weight, fc2.bias)
            if drop:
                m = F.dropout(m, self.dropout, True)
        sc2 = _drop_path_scale(self.stochastic_depth_prob, self.training, B, x.device)
        return (x1, m, sc2)

    def forward(self, x):
        return materialize(self.forward_fused(x))


def materialize(state):
    """Resolve a pending ``(x, branch, scale)`` residual into a tensor."""
    if not isinstance(state, tuple):
        return state
    x, br, sc = state
    if sc is None:
        return x + br.to(x.dtype)
    if x.is_cuda and x.dtype == br.dtype and x[0].numel() % 4 == 0:
        return ops.residual_add(x, br, sc)
    br = br.to(x.dtype)
    return x + br * sc.view(-1, *([1] * (br.dim() - 1))).to(br.dtype)


# ============================================================================ reference parts
class PatchMerging(nn.Module):
    """``model_parts.py:59-106``: x [B,H,W,C] -> gather 2x2 -> LN(4C) -> Linear(4C, 2C)."""

    def __init__(self, input_resolution, dim, norm_layer=nn.LayerNorm):
        super().__init__()
        self.input_resolution = input_resolution
        self.dim = dim
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = norm_layer(4 * dim)

    def forward(self, x):
        Hi, Wi = self.input_resolution
        B, H, W, C = x.shape
        assert Hi == H, "input feature has wrong size"
        assert Wi == W, "input feature has wrong size"
        assert H % 2 == 0 and W % 2 == 0, f"x size ({H}*{W}) are not even."
        x = ops.merge_layer_norm(x, self.norm.weight, self.norm.bias, self.norm.eps)
        return ops.linear(x, self.reduction.weight)

    def extra_repr(self):
        return f"input_resolution={self.input_resolution}, dim={self.dim}"


class BasicLayer(nn.Module):
    """``model_parts.py:109-184``: Swin stage (shift 0 / ws//2 alternating) + PatchMerging."""

    def __init__(self, dim, input_resolution, depth, num_heads, window_size, mlp_ratio=4.0,
                 qkv_bias=True, qk_scale=None, drop=0.0, attn_drop=0.0, drop_path=0.1,
                 norm_layer=nn.LayerNorm, downsample=None, use_checkpoint=False,
                 fused_window_process=False):
        super().__init__()
        self.dim = dim
        self.input_resolution = input_resolution
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        w = [window_size, window_size]
        self.blocks = nn.ModuleList([
            SwinTransformerBlock(dim=dim, num_heads=num_heads, window_size=w,
                                 shift_size=[0 if i % 2 == 0 else s // 2 for s in w],
                                 mlp_ratio=mlp_ratio, dropout=drop, attention_dropout=attn_drop,
                                 stochastic_depth_prob=drop_path[i] if isinstance(drop_path, list) else drop_path,
                                 norm_layer=norm_layer)
            for i in range(depth)])
        self.downsample = downsample(input_resolution, dim=dim, norm_layer=norm_layer) if downsample is not None else None

    def forward(self, x, hk=0):
        """hk: x's handoff key (its other readers' gradients are added in the first block's
        norm1 backward; only without checkpointing, see MSUNetSys._key_for)."""
        B, N, C = x.shape
        H, W = self.input_resolution
        assert H * W == N, f"{N=} passt nicht zu {H}x{W}"
        state = x.view(B, H, W, C)
        for i, blk in enumerate(self.blocks):
            if self.use_checkpoint and torch.is_grad_enabled():
                state = torch.utils.checkpoint.checkpoint(blk, materialize(state), use_reentrant=False)
            else:
                state = blk.forward_fused(state, hk if i == 0 else 0)
        x = materialize(state)
        if self.downsample is not None:
            x = self.downsample(x)
        return x

    def extra_repr(self):
        return f"dim={self.dim}, input_resolution={self.input_resolution}, depth={self.depth}"


class PatchEmbed(nn.Module):
    """``model_parts.py:187-232``: Conv2d(k=s=patch) as im2col (HIP) + GEMM, then LN."""

    def __init__(self, img_size=224, patch_size=4, in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        img_size = _to_2tuple(img_size)
        patch_size = _to_2tuple(patch_size)
        self.img_size = img_size
        self.patch_size = patch_size
        self.patches_resolution = [img_size[0] // patch_size[0], img_size[1] // patch_size[1]]
        self.num_patches = self.patches_resolution[0] * self.patches_resolution[1]
        self.in_chans = in_chans
        self.embed_dim = embed_dim
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None

    def forward(self, x):
        B, C, H, W = x.shape
        assert H == self.img_size[0] and W == self.img_size[1], \
            f"Input image size ({H}*{W}) doesn't match model ({self.img_size[0]}*{self.img_size[1]})."
        if self.patch_size[0] != self.patch_size[1]:
            raise ValueError("square patches only")
        cols = ops.patchify(x, self.patch_size[0], ops.act_dtype())
        t = ops.linear(cols, ops.param_view(self.proj.weight, (self.embed_dim, -1)), self.proj.bias)
        t = t.view(B, self.num_patches, self.embed_dim)
        if self.norm is not None:
            t = ops.layer_norm(t, self.norm.weight, self.norm.bias, self.norm.eps)
        return t


class PatchExpand(nn.Module):
    """``model_parts.py:374-407``: Linear(C, 2C) -> depth-to-space 2x2 -> LN(C/2) (fused)."""

    def __init__(self, input_resolution, dim, dim_scale=2, norm_layer=nn.LayerNorm):
        super().__init__()
        self.input_resolution = input_resolution
        self.dim = dim
        self.expand = nn.Linear(dim, 2 * dim, bias=False) if dim_scale == 2 else nn.Identity()
        self.norm = norm_layer(dim // dim_scale)

    def forward(self, x, hk=0):
        """hk: x's handoff key (the Linear's input gradient goes to the keyed LayerNorm)."""
        if x.dim() == 4:
            B, H, W, C_in = x.shape
        elif x.dim() == 3:
            B, L, C_in = x.shape
            H, W = self.input_resolution
            if L != H * W:
                assert L == H * W, "input feature has wrong size"
        else:
            raise ValueError(f"Unexpected dimensionality: x.dim()={x.dim()}")
        x = x.reshape(B, H, W, C_in)
        x = self.expand(x) if isinstance(self.expand, nn.Identity) else ops.linear(x, self.expand.weight, handoff=hk)
        C = x.shape[-1]
        if C % 4 != 0:
            raise ValueError(f"channels C={C} are not divisible by 4 (required for ×2 upsampling).")
        return ops.d2s_layer_norm(x, self.norm.weight, self.norm.bias, self.norm.eps)


class FinalPatchExpand_X4_V2(nn.Module):
    """``model_parts.py:437-476``: Linear(C, 16C) -> GELU -> d2s 4x4 -> conv3x3+b -> GELU ->
    conv3x3+b -> LN(C).  d2s is folded into refine1's loads (no NCHW permutes); each GELU
    output is stored by its producer's epilogue next to the pre-activation."""

    def __init__(self, input_resolution, dim, dim_scale=4, norm_layer=nn.LayerNorm):
        super().__init__()
        self.input_resolution = input_resolution
        self.dim = dim
        self.dim_scale = dim_scale
        if dim_scale != 4:
            raise ValueError("FinalPatchExpand_X4_V2 is a x4 expand")
        self.expand = nn.Linear(dim, 16 * dim, bias=False)
        self.act = nn.GELU()
        self.output_dim = dim
        self.refine1 = nn.Conv2d(dim, dim, kernel_size=3, padding=1, bias=True)
        self.refine2 = nn.Conv2d(dim, dim, kernel_size=3, padding=1, bias=True)
        self.norm = norm_layer(self.output_dim)

    def pre_norm(self, x):
        """-> refine2 output z2 [B, 4H, 4W, C] (before the final LayerNorm)."""
        H, W = self.input_resolution
        B, L, C = x.shape
        assert L == H * W, "input feature has wrong size"
        # expand's epilogue also stores act(e) and refine1's also stores act(z1): each conv
        # loads its activation, while the dgrad epilogues apply act' to e / z1
        e, a0 = ops.linear_gelu(x, self.expand.weight)
        e, a0 = e.view(B, H, W, 16 * C), a0.view(B, H, W, 16 * C)
        z1, a1 = ops.refine_conv_act(e, a0, self.refine1.weight, self.refine1.bias, True, (4 * H, 4 * W), dual=True)
        return ops.refine_conv_act(z1, a1, self.refine2.weight, self.refine2.bias, False, (4 * H, 4 * W))

    def forward(self, x):
        z2 = self.pre_norm(x)
        B = z2.shape[0]
        y = ops.layer_norm(z2, self.norm.weight, self.norm.bias, self.norm.eps)
        return y.reshape(B, -1, self.output_dim)


class BasicLayer_up(nn.Module):
    """``model_parts.py:478-541``: Swin decoder stage + optional PatchExpand."""

    def __init__(self, dim, input_resolution, depth, num_heads, window_size, mlp_ratio=4.0,
                 qkv_bias=True, qk_scale=None, drop=0.0, attn_drop=0.0, drop_path=0.0,
                 norm_layer=nn.LayerNorm, upsample=None, use_checkpoint=False):
        super().__init__()
        self.dim = dim
        self.input_resolution = input_resolution
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        w = [window_size, window_size]
        self.blocks = nn.ModuleList([
            SwinTransformerBlock(dim=dim, num_heads=num_heads, window_size=w,
                                 shift_size=[0 if i % 2 == 0 else s // 2 for s in w],
                                 mlp_ratio=mlp_ratio, dropout=drop, attention_dropout=attn_drop,
                                 stochastic_depth_prob=drop_path[i] if isinstance(drop_path, list) else drop_path,
                                 norm_layer=norm_layer)
            for i in range(depth)])
        self.upsample = PatchExpand(input_resolution, dim=dim, dim_scale=2, norm_layer=norm_layer) if upsample is not None else None

    def forward(self, x, hk=0):
        """hk: as BasicLayer.forward."""
        B, N, C = x.shape
        H, W = self.input_resolution
        assert H * W == N, f"{N=} passt nicht zu {H}x{W}"
        state = x.view(B, H, W, C)
        for i, blk in enumerate(self.blocks):
            if self.use_checkpoint and torch.is_grad_enabled():
                state = torch.utils.checkpoint.checkpoint(blk, materialize(state), use_reentrant=False)
            else:
                state = blk.forward_fused(state, hk if i == 0 else 0)
        x = materialize(state)
        if self.upsample is not None:
            x = self.upsample(x)
        return x


def _skip_fuse(lin, x, skip, hk=0):
    """``torch.cat([x, skip], -1)`` -> ``concat_back_dim[k]`` (model_parts.py:792-793 etc.);
    hk: the skip's handoff key."""
    B = x.shape[0]
    return ops.linear_cat(x.reshape(B, -1, x.shape[-1]), skip.reshape(B, -1, skip.shape[-1]), lin.weight, lin.bias,
                          handoff=hk)


# ============================================================================ MSUNetSys
class MSUNetSys(nn.Module):
    """``model_parts.py:543-894`` (same constructor, submodules and state-dict keys)."""

    def __init__(self, img_size=1024, patch_size=4, in_chans=3, num_classes=1, embed_dim=128,
                 depths=[2, 2, 18, 2], depths_decoder=[2, 2, 6, 2], num_heads=[4, 8, 16, 32],
                 window_size=7, mlp_ratio=4.0, qkv_bias=True, qk_scale=None, drop_rate=0.0,
                 attn_drop_rate=0.0, drop_path_rate=0.1, norm_layer=nn.LayerNorm, ape=False,
                 patch_norm=True, use_checkpoint=False, final_upsample="expand_first", **kwargs):
        super().__init__()
        self.num_classes = num_classes
        self.num_layers = len(depths)
        self.embed_dim = embed_dim
        self.ape = ape
        self.patch_norm = patch_norm
        self.num_features = int(embed_dim * 2 ** (self.num_layers - 1))
        self.num_features_up = int(embed_dim * 2)
        self.mlp_ratio = mlp_ratio
        self.final_upsample = final_upsample
        # the reference runs layers_cent1[-1] / layers_cent2[-1] and discards the result
        # (model_parts.py:795, :807); they are still executed (no autograd record) unless
        # skip_dead_branches is set -- both are exact
        self.skip_dead_branches = False

        self.patch_embed = PatchEmbed(img_size=img_size, patch_size=patch_size, in_chans=in_chans,
                                      embed_dim=embed_dim, norm_layer=norm_layer if self.patch_norm else None)
        num_patches = self.patch_embed.num_patches
        pr = self.patch_embed.patches_resolution
        self.patches_resolution = pr
        if self.ape:
            self.absolute_pos_embed = nn.Parameter(torch.zeros(1, num_patches, embed_dim))
            _trunc_normal_(self.absolute_pos_embed, std=0.02)
        self.pos_drop = nn.Dropout(p=drop_rate)
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, sum(depths))]
        L = self.num_layers

        def up_layer(s, upsample):
            return BasicLayer_up(dim=int(embed_dim * 2 ** s), input_resolution=(pr[0] // 2 ** s, pr[1] // 2 ** s),
                                 depth=depths[s], num_heads=num_heads[s], window_size=window_size,
                                 mlp_ratio=self.mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale,
                                 drop=drop_rate, attn_drop=attn_drop_rate,
                                 drop_path=dpr[sum(depths[:s]):sum(depths[:s + 1])],
                                 norm_layer=norm_layer, upsample=PatchExpand if upsample else None,
                                 use_checkpoint=use_checkpoint)

        def expand(s):
            return PatchExpand(input_resolution=(pr[0] // 2 ** s, pr[1] // 2 ** s),
                               dim=int(embed_dim * 2 ** s), dim_scale=2, norm_layer=norm_layer)

        self.layers = nn.ModuleList()
        for i in range(L):
            self.layers.append(BasicLayer(dim=int(embed_dim * 2 ** i),
                                          input_resolution=(pr[0] // 2 ** i, pr[1] // 2 ** i),
                                          depth=depths[i], num_heads=num_heads[i], window_size=window_size,
                                          mlp_ratio=self.mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale,
                                          drop=drop_rate, attn_drop=attn_drop_rate,
                                          drop_path=dpr[sum(depths[:i]):sum(depths[:i + 1])],
                                          norm_layer=norm_layer,
                                          downsample=PatchMerging if (i < L - 1) else None,
                                          use_checkpoint=use_checkpoint))
        self.layers_up = nn.ModuleList()
        self.concat_back_dim = nn.ModuleList()
        for k in range(L):
            s = L - 1 - k
            d = int(embed_dim * 2 ** s)
            self.concat_back_dim.append(nn.Linear(2 * d, d) if k > 0 else nn.Identity())
            self.layers_up.append(expand(s) if k == 0 else up_layer(s, k < L - 1))
        self.layers_cent1 = nn.ModuleList()
        for k in range(L - 1):
            s = L - 2 - k
            self.layers_cent1.append(expand(s) if k == 0 else up_layer(s, k < L - 2))
        self.layers_cent2 = nn.ModuleList()
        for k in range(L - 2):
            s = L - 3 - k
            self.layers_cent2.append(expand(s) if k == 0 else up_layer(s, k < L - 3))
        self.norm = norm_layer(self.num_features)
        self.norm_up = norm_layer(self.embed_dim)
        if self.final_upsample == "expand_first":
            self.up = FinalPatchExpand_X4_V2(input_resolution=(img_size // patch_size, img_size // patch_size),
                                             dim_scale=4, dim=embed_dim)
            self.output = nn.Conv2d(in_channels=embed_dim, out_channels=self.num_classes, kernel_size=1, bias=False)
        self.apply(self._init_weights)

    def _init_weights(self, m):
        if isinstance(m, nn.Linear):
            _trunc_normal_(m.weight, std=0.02)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    @torch.jit.ignore
    def no_weight_decay(self):
        return {"absolute_pos_embed"}

    @torch.jit.ignore
    def no_weight_decay_keywords(self):
        return {"relative_position_bias_table"}

    def dead_modules(self):
        return [self.layers_cent1[self.num_layers - 2], self.layers_cent2[self.num_layers - 3]]

    def _run_dead(self, mod, x):
        """Run a branch whose result the reference discards.  On a GPU it goes to the side
        stream (ops.side stream, joined with the weight-gradient work at the end of backward):
        nothing reads its output, so it overlaps the rest of the forward pass."""
        if self.skip_dead_branches:
            return
        if not x.is_cuda or not ops._side_enabled:
            with torch.no_grad():
                mod(x)
            return
        side = ops._side_stream_for(x.device)
        side.wait_stream(torch.cuda.current_stream(x.device))
        with torch.no_grad(), torch.cuda.stream(side):
            mod(x)
        x.record_stream(side)

    @staticmethod
    def _key_for(layer):
        """A handoff key for a tensor whose first-block reader is `layer` (a Swin stage): its
        other readers -- skip fusions, the central decoders' PatchExpand Linears -- hand their
        input gradients to that block's norm1 backward kernel (ops.residual_handoff_key; 0
        under checkpointing, where the blocks make their own keys)."""
        return 0 if layer.use_checkpoint else ops.residual_handoff_key()

    def forward_features(self, x):
        """``model_parts.py:775-815``."""
        x, xd, self._skip_keys = self._forward_features(x)
        return x, xd

    def _forward_features(self, x):
        x = self.patch_embed(x)
        if self.ape:
            x = x + self.absolute_pos_embed
        x = self.pos_drop(x)
        xd, xk = [], []  # the skip tensors and their handoff keys
        dead = []  # issued after the stage's own blocks: the main stream is not starved while
        # the host launches a branch nobody reads
        for i, layer in enumerate(self.layers):
            kx = self._key_for(layer)  # x's readers: this stage, a central branch, a skip fusion
            xd.append(x)
            xk.append(kx)
            xs, x = x, layer(x, kx)
            # the central decoders: layers_cent2 on stage 1's input, layers_cent1 on stage 2's,
            # each ending in a branch the reference discards (model_parts.py:795, :807).  Run
            # after the stage (independent of it; the reference runs them before): their nodes
            # are then newer than the stage's, so autograd runs their backwards first and their
            # input gradients reach the stage's first norm1 through the handoff, not an add
            for cent, cat0, start in ((self.layers_cent2, 2, 1), (self.layers_cent1, 1, 2)):
                if i != start:
                    continue
                xc = xs
                for k, mod in enumerate(cent):
                    if k == 0:
                        xc = mod(xc, kx)
                    else:
                        xc = _skip_fuse(self.concat_back_dim[k + cat0], xc, xd[i - k], xk[i - k])
                        xd[i - k] = xc
                        if k == len(cent) - 1:
                            xk[i - k] = 0  # read by the discarded branch (no gradient) and a skip
                            dead.append((mod, xc))
                        else:
                            xk[i - k] = self._key_for(mod)
                            xc = mod(xc, xk[i - k])
            for mod, xin in dead:
                self._run_dead(mod, xin)
            dead.clear()
        x = ops.layer_norm(x, self.norm.weight, self.norm.bias, self.norm.eps)
        return x, xd, xk

    def forward_up_features(self, x, xd, keys=None):
        """``model_parts.py:818-829``; keys: the skips' handoff keys (forward_features')."""
        for k, layer_up in enumerate(self.layers_up):
            if k == 0:
                x = layer_up(x)
            else:
                x = _skip_fuse(self.concat_back_dim[k], x, xd[3 - k], keys[3 - k] if keys else 0)
                x = layer_up(x)
        return ops.layer_norm(x, self.norm_up.weight, self.norm_up.bias, self.norm_up.eps)

    def up_x4(self, x):
        """``model_parts.py:832-848``: FinalPatchExpand_X4_V2 + 1x1 ``output`` conv; the final
        LayerNorm and the 1x1 conv are one fused kernel (f32 logits [B, 1, 4H, 4W])."""
        H, W = self.patches_resolution
        if x.dim() == 4:
            B, H, W, C = x.shape
            x = x.reshape(B, H * W, C)
        else:
            B, L, C = x.shape
            assert L == H * W, "input features has wrong size"
        if self.final_upsample != "expand_first":
            return x
        z2 = self.up.pre_norm(x)
        if self.num_classes == 1:
            return ops.head_norm_output(z2, self.up.norm.weight, self.up.norm.bias, self.output.weight,
                                        self.up.norm.eps)
        y = ops.layer_norm(z2, self.up.norm.weight, self.up.norm.bias, self.up.norm.eps)
        return ops.linear(y, self.output.weight.reshape(self.num_classes, -1)).permute(0, 3, 1, 2)

    def forward(self, x):
        x, xd, xk = self._forward_features(x)
        x = self.forward_up_features(x, xd, xk)
        return self.up_x4(x)

    def freeze_encoder(self, freeze=True):
        for p in self.patch_embed.parameters():
            p.requires_grad = not freeze
        for layer in self.layers:
            for p in layer.parameters():
                p.requires_grad = not freeze

    def unfreeze_encoder(self, num_stage: int):
        n_stages = len(self.layers)
        if not (0 <= num_stage < n_stages):
            raise ValueError(f"num_stage={num_stage} out of range [0, {n_stages - 1}]")
        for p in self.layers[num_stage].parameters():
            if not p.requires_grad:
                p.requires_grad_(True)
        if num_stage == 0:
            for p in self.patch_embed.parameters():
                if not p.requires_grad:
                    p.requires_grad_(True)
