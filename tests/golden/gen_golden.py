"""Generate the golden fixtures under ``tests/golden/`` by running the REFERENCE code.

Run in the survey/dev container only (needs ``/root/reference``; never runs on the GPU box):

    python tests/golden/gen_golden.py

What is imported from the reference:

* ``loss/DynamicLoss.py`` -- imported directly (pure torch).
* ``network/model_parts.py`` -- imported with two test-only ``sys.modules`` shims because
  the image lacks its third-party deps: ``timm.layers`` (``to_2tuple``,
  ``trunc_normal_``, ``DropPath``; trivial) and ``torchvision.models.swin_transformer``
  (``SwinTransformerBlock``), for which this script supplies the oracle's restatement of
  the torchvision v1 block.  The MS-UNet topology (central decoders, shared
  ``concat_back_dim``, PatchMerging / PatchExpand / FinalPatchExpand_X4_V2 / head) is the
  reference's own code; the block arithmetic is the restatement (parity of the block
  itself is therefore unpinned, see oracle/swin_block.py).

Outputs (data only -- inputs are regenerated from seeds by ``tests/golden/cases.py``):
``dynamic_loss.npz``, ``ops_reference.npz``, ``msunet_<case>.npz``,
``state_dict_swin_b_1024.json``, ``structure_of_MSUNet.json``.
"""
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from oracle import swin_block as osb  # noqa: E402
from oracle.msunet import make_cfg  # noqa: E402
import cases  # noqa: E402


# ----------------------------------------------------------------------------- shims
class _Attn(nn.Module):
    def __init__(self, dim, ws, heads):
        super().__init__()
        n = (2 * ws - 1) ** 2
        self.relative_position_bias_table = nn.Parameter(torch.zeros(n, heads))
        self.register_buffer("relative_position_index", osb.relative_position_index(ws))
        self.qkv = nn.Linear(dim, 3 * dim)
        self.proj = nn.Linear(dim, dim)


class SwinTransformerBlock(nn.Module):
    """Shim with torchvision's parameter names; forward = oracle restatement."""

    def __init__(self, dim, num_heads, window_size, shift_size, mlp_ratio=4.0, dropout=0.0,
                 attention_dropout=0.0, stochastic_depth_prob=0.0, norm_layer=nn.LayerNorm):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.attn = _Attn(dim, window_size[0], num_heads)
        self.norm2 = norm_layer(dim)
        hid = int(dim * mlp_ratio)
        self.mlp = nn.Sequential(nn.Linear(dim, hid), nn.GELU(), nn.Dropout(dropout),
                                 nn.Linear(hid, dim), nn.Dropout(dropout))
        self.heads, self.ws, self.shift = num_heads, window_size[0], shift_size[0]
        self.sdp, self.adrop = stochastic_depth_prob, attention_dropout

    def forward(self, x):
        p = dict(self.named_parameters())
        p.update(dict(self.named_buffers()))
        return osb.swin_block(p, "", x, self.heads, self.ws, self.shift,
                              self.sdp, self.adrop, self.training)


def install_shims():
    timm = types.ModuleType("timm")
    layers = types.ModuleType("timm.layers")
    layers.to_2tuple = lambda v: tuple(v) if isinstance(v, (tuple, list)) else (v, v)
    layers.trunc_normal_ = nn.init.trunc_normal_
    layers.DropPath = lambda p=0.0: nn.Identity()
    timm.layers = layers
    tv = types.ModuleType("torchvision")
    tvm = types.ModuleType("torchvision.models")
    tvs = types.ModuleType("torchvision.models.swin_transformer")
    tvs.SwinTransformerBlock = SwinTransformerBlock
    tv.models, tvm.swin_transformer = tvm, tvs
    sys.modules.update({"timm": timm, "timm.layers": layers, "torchvision": tv,
                        "torchvision.models": tvm, "torchvision.models.swin_transformer": tvs})


def ref_msunetsys(cfg):
    import importlib
    mp = importlib.import_module("network.model_parts")
    return mp.MSUNetSys(img_size=cfg["img_size"], patch_size=cfg["patch_size"],
                        in_chans=cfg["in_chans"], num_classes=cfg["num_classes"],
                        embed_dim=cfg["embed_dim"], depths=cfg["depths"],
                        num_heads=cfg["num_heads"], window_size=cfg["window_size"],
                        mlp_ratio=cfg["mlp_ratio"], qkv_bias=True, qk_scale=None,
                        drop_rate=0.0, drop_path_rate=cfg["drop_path_rate"],
                        attn_drop_rate=0.0, ape=False, patch_norm=True, use_checkpoint=False)


# ----------------------------------------------------------------------------- fixtures
def gen_dynamic_loss():
    from loss.DynamicLoss import DynamicLoss
    out = {}
    for name, (logits, target, kw) in cases.loss_cases().items():
        ref = DynamicLoss(alpha=kw["alpha"], beta=kw["beta"], tversky_bce_mix=kw["mix"])
        x = logits.clone().requires_grad_(True)
        loss = ref(x, target.clone())
        loss.backward()
        out[f"{name}.loss"] = np.array(loss.item(), dtype=np.float64)
        out[f"{name}.grad"] = x.grad.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "dynamic_loss.npz"), **out)
    print("dynamic_loss.npz:", len(out) // 2, "cases")


def gen_ops():
    import importlib
    mp = importlib.import_module("network.model_parts")
    out = {}
    for name, (kind, args, x) in cases.op_cases().items():
        torch.manual_seed(0)
        if kind == "merge":
            m = mp.PatchMerging(args["res"], dim=args["dim"])
        elif kind == "expand":
            m = mp.PatchExpand(args["res"], dim=args["dim"], dim_scale=2)
        elif kind == "final":
            m = mp.FinalPatchExpand_X4_V2(args["res"], dim=args["dim"], dim_scale=4)
        sd = cases.op_params(kind, args)
        m.load_state_dict(sd, strict=True)
        xi = x.clone().requires_grad_(True)
        y = m(xi)
        y.backward(cases.op_upstream(y))
        out[f"{name}.y"] = y.detach().numpy()
        out[f"{name}.dx"] = xi.grad.numpy()
        for k, v in m.named_parameters():
            out[f"{name}.d.{k}"] = v.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "ops_reference.npz"), **out)
    print("ops_reference.npz:", len(out), "arrays")


def gen_msunet(only=None):
    for name, spec in cases.model_cases().items():
        if only and name not in only:
            continue
        cfg = make_cfg(**spec["cfg"])
        model = ref_msunetsys(cfg)
        params = cases.model_params(cfg, spec["seed"])
        missing = model.load_state_dict(params, strict=True)
        assert not missing.missing_keys and not missing.unexpected_keys
        model.train()  # drop rates are zero in the fixture configs
        x, target = cases.model_inputs(cfg, spec["batch"], spec["seed"])
        logits = model(x)
        from loss.DynamicLoss import DynamicLoss
        loss = DynamicLoss(alpha=0.2, beta=0.8, tversky_bce_mix=0.45)(logits, target)
        loss.backward()
        out = {"logits": logits.detach().numpy(), "loss": np.array(loss.item())}
        names, norms, sums = [], [], []
        for k, v in model.named_parameters():
            if v.grad is None:
                continue
            names.append(k)
            norms.append(float(v.grad.norm()))
            sums.append(float(v.grad.sum()))
        out["grad_names"] = np.array(names)
        out["grad_norm"] = np.array(norms)
        out["grad_sum"] = np.array(sums)
        no_grad = [k for k, v in model.named_parameters() if v.grad is None]
        out["no_grad_names"] = np.array(no_grad)
        for k in cases.FULL_GRAD_KEYS:
            out["grad." + k] = dict(model.named_parameters())[k].grad.numpy()
        np.savez_compressed(os.path.join(HERE, f"msunet_{name}.npz"), **out)
        print(f"msunet_{name}.npz: loss={loss.item():.6f} grads={len(names)} no_grad={len(no_grad)}")


def gen_state_dict_contract():
    cfg = make_cfg(img_size=1024, embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32])
    model = ref_msunetsys(cfg)
    sd = [[k, list(v.shape), str(v.dtype)] for k, v in model.state_dict().items()]
    with open(os.path.join(HERE, "state_dict_swin_b_1024.json"), "w") as f:
        json.dump(sd, f)
    dump = []
    with open(os.path.join(REF, "network/pretrained_weights/structure_of_MSUNet.txt")) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            _, rest = line.split(" : ", 1)
            key, shape = rest.split(" torch.Size(")
            dump.append([key.strip(), json.loads(shape.rstrip(")"))])
    with open(os.path.join(HERE, "structure_of_MSUNet.json"), "w") as f:
        json.dump(dump, f)
    print("state dict contract:", len(sd), "entries; structure dump:", len(dump))


def gen_pretrained_layouts():
    """Key / shape lists of the two pretrained checkpoints the reference remaps
    (network/pretrained_weights/structure_of_SegFace.txt, IMAGENET1K_structure.txt): data
    files of the reference, kept as JSON fixtures for the key-remap tests."""
    out = {}
    for name, fname in (("segface", "structure_of_SegFace.txt"), ("imagenet1k", "IMAGENET1K_structure.txt")):
        rows = []
        with open(os.path.join(REF, "network/pretrained_weights", fname)) as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                _, rest = line.split(":", 1)
                key, shape = rest.split("torch.Size(")
                rows.append([key.strip(), json.loads(shape.split(")")[0])])
        out[name] = rows
    with open(os.path.join(HERE, "pretrained_layouts.json"), "w") as f:
        json.dump(out, f)
    print("pretrained layouts:", {k: len(v) for k, v in out.items()})


if __name__ == "__main__":
    sys.path.insert(0, REF)
    install_shims()
    torch.set_num_threads(8)
    only = sys.argv[1:]  # model case names: regenerate just those fixtures
    if only == ["layouts"]:
        gen_pretrained_layouts()
        sys.exit(0)
    if only:
        gen_msunet(only)
        sys.exit(0)
    gen_dynamic_loss()
    gen_ops()
    gen_msunet()
    gen_state_dict_contract()
