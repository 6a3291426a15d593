"""Configuration: the reference's yacs keys (``config.py:13-138`` + ``config.yaml``) as a
plain attribute-dict, merged from YAML with ``yaml.safe_load`` (yacs is not needed).

Only the keys the training hot path reads are interpreted; unknown keys are kept.
"""
import copy
import os

import yaml


class CfgNode(dict):
    """dict with attribute access (``cfg.MODEL.SWIN.EMBED_DIM``), like yacs.CfgNode."""

    def __init__(self, d=None):
        super().__init__()
        for k, v in (d or {}).items():
            self[k] = CfgNode(v) if isinstance(v, dict) else v

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = CfgNode(v) if isinstance(v, dict) and not isinstance(v, CfgNode) else v

    def merge(self, other):
        for k, v in other.items():
            if isinstance(v, dict) and isinstance(self.get(k), dict):
                self[k].merge(v)
            else:
                self[k] = CfgNode(v) if isinstance(v, dict) else v
        return self

    def clone(self):
        return copy.deepcopy(self)


# values of the reference config.yaml (the Swin-B MS-UNet it trains by default)
_DEFAULTS = {
    "DATA": {"BATCH_SIZE": 2, "IMG_SIZE": 1024, "DATA_PATH": "./dataset", "NUM_WORKERS": 2,
             "PIN_MEMORY": True},
    "HARDWARE": {"N_GPU": 1},
    "MODEL": {
        "TYPE": "swin", "NAME": "swin_b", "NUM_CLASSES": 1, "DROP_RATE": 0.0,
        "DROP_PATH_RATE": 0.1, "ATTN_DROP_RATE": 0.05, "FREEZE_ENCODER": False,
        "PRETRAIN_WEIGHTS": "segface",
        "PRETRAIN_SEGFACE": "./network/pretrained_weights/SegFace_swin_celaba_512.pt",
        "PRETRAIN_IMAGENET1K": "./network/pretrained_weights/swin_b-68c6b09e.pth",
        "SWIN": {"PATCH_SIZE": 4, "IN_CHANS": 3, "EMBED_DIM": 128, "DEPTHS": [2, 2, 18, 2],
                 "DECODER_DEPTHS": [2, 2, 6, 2], "NUM_HEADS": [4, 8, 16, 32], "WINDOW_SIZE": 7,
                 "MLP_RATIO": 4.0, "QKV_BIAS": True, "QK_SCALE": None, "APE": False,
                 "PATCH_NORM": True, "FINAL_UPSAMPLE": "expand_first"},
    },
    "TRAIN": {
        "MAX_EPOCHS": 60, "START_EPOCH": 0, "WARMUP_EPOCHS": 20, "WEIGHT_DECAY": 0.001,
        "BASE_LR": 1e-5, "WARMUP_LR": 1e-6, "MIN_LR": 1e-6, "ACCUMULATION_STEPS": 1,
        "USE_CHECKPOINT": False, "TVERSKY_LOSS_ALPHA": 0.2, "TVERSKY_LOSS_BETA": 0.8,
        "LOSS_TVERSKY_BCE_MIX": 0.45, "SIG_THRESHOLD": 0.5,
        "LR_SCHEDULER": {"NAME": "cosine", "WARMUP_PREFIX": True},
        "OPTIMIZER": {"NAME": "adamw", "EPS": 1e-8, "BETAS": [0.9, 0.999]},
    },
    "TEST": {"SIG_THRESHOLD": 0.5},
    "SEED": 120,
    "DETERMINISTIC": True,
    "OUTPUT_DIR": "./model_out",
    "SAVE_BEST_RUN": False,
    "SAVE_LAST_RUN": False,
}

BACKBONES = {
    "swin_t": {"EMBED_DIM": 96, "DEPTHS": [2, 2, 6, 2], "NUM_HEADS": [3, 6, 12, 24]},
    "swin_s": {"EMBED_DIM": 96, "DEPTHS": [2, 2, 18, 2], "NUM_HEADS": [3, 6, 12, 24]},
    "swin_b": {"EMBED_DIM": 128, "DEPTHS": [2, 2, 18, 2], "NUM_HEADS": [4, 8, 16, 32]},
}


def default_config():
    return CfgNode(copy.deepcopy(_DEFAULTS))


def load_config(path=None, backbone=None, **overrides):
    """Defaults <- YAML file (``BASE`` includes honoured) <- backbone preset <- overrides
    given as dotted keys, e.g. ``load_config(None, 'swin_t', **{'DATA.IMG_SIZE': 512})``."""
    cfg = default_config()
    if path is not None:
        _merge_file(cfg, path)
    if backbone is not None:
        cfg.MODEL.NAME = backbone
        cfg.MODEL.SWIN.merge(BACKBONES[backbone])
    for key, val in overrides.items():
        node = cfg
        parts = key.split(".")
        for p in parts[:-1]:
            node = node[p]
        node[parts[-1]] = val
    return cfg


def _merge_file(cfg, path):
    with open(path) as f:
        y = yaml.safe_load(f) or {}
    for base in y.get("BASE", []) or []:
        if base:
            _merge_file(cfg, os.path.join(os.path.dirname(path), base))
    y.pop("BASE", None)
    cfg.merge(y)
