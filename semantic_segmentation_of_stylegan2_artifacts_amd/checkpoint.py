"""Checkpoint I/O and pretrained-weight key remapping.

* ``save_best`` -- the reference's best-model payload ``{"model", "epoch", "best_score"}``
  written to a temporary file with the legacy (non-zip) serialization and moved into place
  with ``os.replace`` (/root/reference/trainer.py:361-385);
* ``save_last`` -- the last-epoch payload ``{"epoch", "model", "optimizer", "iter_num",
  "dice"}`` (trainer.py:403-409) with the optimizer state in ``torch.optim.AdamW`` format;
* ``load_checkpoint`` -- test.py:96-110: ``{"model": sd}``, ``{"state_dict": sd}`` or a bare
  state dict, loaded with ``strict=True``;
* ``remap_segface`` / ``remap_imagenet1k`` -- the key maps of ``MSUNet.load_segface_weight``
  and ``MSUNet.load_IMAGENET1K_weight`` (network/MSUNet.py:61-229): SegFace
  ``state_dict_backbone`` ``backbone.0.*`` and torchvision swin_b ``features.*`` keys onto the
  MS-UNet encoder (``patch_embed`` + ``layers.0-3``), same error rules (unknown key ->
  ValueError, shape mismatch -> ValueError), loaded with ``strict=False``.

Every file this module reads goes through ``torch.load(weights_only=True)``: checkpoints are
data, never code.  Model state is written from per-key CPU copies, so a model whose
parameters live in the trainer's flat buffers saves the same keys / shapes as the reference.
"""
import os

import torch


def _cpu_state(module):
    return {k: v.detach().to("cpu", copy=True) for k, v in module.state_dict().items()}


def core(model):
    """The MSUNetSys inside an MSUNet wrapper (the reference's checkpoints hold the wrapper's
    keys, ``ms_unet.*``: trainer.py:372 saves core(model).state_dict() of the wrapper)."""
    return model.module if isinstance(model, torch.nn.DataParallel) else model


def save_best(model, epoch, best_score, log_save_path, name="best_model.pth"):
    """trainer.py:365-379: tmp file + os.replace, legacy serialization."""
    payload = {"model": _cpu_state(core(model)), "epoch": epoch, "best_score": best_score}
    best_path = os.path.join(log_save_path, name)
    tmp = best_path + ".tmp"
    torch.save(payload, tmp, _use_new_zipfile_serialization=False)
    os.replace(tmp, best_path)
    return best_path


def save_last(model, optimizer_state, epoch, iter_num, dice, log_save_path):
    """trainer.py:403-409 (``epoch_<n>.pth``)."""
    path = os.path.join(log_save_path, "epoch_" + str(epoch) + ".pth")
    torch.save({"epoch": epoch, "model": _cpu_state(core(model)), "optimizer": optimizer_state,
                "iter_num": iter_num, "dice": dice}, path)
    return path


def load_checkpoint(model, path, map_location="cpu", strict=True):
    """test.py:96-110: the state dict under 'model' / 'state_dict' or the bare dict; strict."""
    if not os.path.exists(path):
        raise FileNotFoundError(f"Checkpoint not found: {path}")
    ckpt = torch.load(path, map_location=map_location, weights_only=True)
    if isinstance(ckpt, dict) and "model" in ckpt:
        state = ckpt["model"]
    elif isinstance(ckpt, dict) and "state_dict" in ckpt:
        state = ckpt["state_dict"]
    else:
        state = ckpt
    return core(model).load_state_dict(state, strict=strict)


# ----------------------------------------------------------------------------- key remaps
def _encoder_prefix_map(src, n_stage2=18):
    """(source prefix, MS-UNet prefix) pairs of the encoder, for src 'backbone.0' (SegFace)
    or 'features' (torchvision)."""
    m = [(f"{src}.0.0.", "patch_embed.proj."), (f"{src}.0.2.", "patch_embed.norm."),
         (f"{src}.1.0.", "layers.0.blocks.0."), (f"{src}.1.1.", "layers.0.blocks.1."),
         (f"{src}.2.", "layers.0.downsample."),
         (f"{src}.3.0.", "layers.1.blocks.0."), (f"{src}.3.1.", "layers.1.blocks.1."),
         (f"{src}.4.", "layers.1.downsample.")]
    m += [(f"{src}.5.{i}.", f"layers.2.blocks.{i}.") for i in range(n_stage2)]
    m += [(f"{src}.6.", "layers.2.downsample."),
          (f"{src}.7.0.", "layers.3.blocks.0."), (f"{src}.7.1.", "layers.3.blocks.1.")]
    return m


def _remap(state, src, owner, skip=()):
    """Rename every key under ``src.`` by the encoder map; keys outside ``owner`` are
    ignored, keys under a ``skip`` prefix dropped, any other unmatched key is an error."""
    table = _encoder_prefix_map(src)
    out, seen = {}, False
    for k, v in state.items():
        if not k.startswith(owner):
            continue
        seen = True
        if any(k.startswith(s) for s in skip):
            continue
        # stage-2 block prefixes: longest match first ('.5.1' must not take '.5.10.*')
        hits = [(a, b) for a, b in table if k.startswith(a)]
        if not hits:
            raise ValueError(f"Key {k} not found in dictionary!!")
        a, b = max(hits, key=lambda ab: len(ab[0]))
        out[b + k[len(a):]] = v
    if not seen:
        raise ValueError("No new keys from backbone!!")
    return out


def remap_segface(segface_ckpt):
    """network/MSUNet.py:71-135: SegFace ``state_dict_backbone`` -> MS-UNet encoder keys
    (``backbone.1.*``, SegFace's final norm, is dropped)."""
    if "state_dict_backbone" not in segface_ckpt:
        raise KeyError("'state_dict_backbone' not found in checkpoint")
    return _remap(segface_ckpt["state_dict_backbone"], "backbone.0", "backbone", skip=("backbone.1.",))


def remap_imagenet1k(state):
    """network/MSUNet.py:160-216: torchvision swin_b ``features.*`` -> MS-UNet encoder keys
    (``norm.*`` / ``head.*`` are not under ``features`` and are ignored)."""
    return _remap(state, "features", "features")


def load_encoder(ms_unet, new_state):
    """Shape check against the model (ValueError on mismatch, MSUNet.py:137-144) and a
    non-strict load (:146)."""
    model_dict = ms_unet.state_dict()
    for k, v in new_state.items():
        if k in model_dict and tuple(v.shape) != tuple(model_dict[k].shape):
            raise ValueError(f"Key {k} does not match the dictionary of MSUNet!")
    return ms_unet.load_state_dict(new_state, strict=False)


def load_pretrained_file(ms_unet, path, kind, logging=None):
    """MSUNet.load_segface_weight / load_IMAGENET1K_weight: a missing file logs an error and
    returns None (as the reference); kind 'segface' | 'imagenet1k'."""
    if not path or not os.path.exists(path):
        if logging is not None:
            logging.error(f"No {kind} pretrain found at: {path}")
        return None
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    new_state = remap_segface(ckpt) if kind == "segface" else remap_imagenet1k(ckpt)
    return load_encoder(ms_unet, new_state)
