"""``network/MSUNet.py`` drop-in: config -> MSUNetSys adapter (``MSUNet.py:16-58``)."""
import logging

import torch.nn as nn

from .model_parts import MSUNetSys

logger = logging.getLogger(__name__)


class MSUNet(nn.Module):
    def __init__(self, config, img_size=1024, num_classes=1, zero_head=False, vis=False):
        super().__init__()
        self.num_classes = num_classes
        self.zero_head = zero_head
        self.config = config
        sw = config.MODEL.SWIN
        self.ms_unet = MSUNetSys(img_size=img_size, patch_size=sw.PATCH_SIZE, in_chans=sw.IN_CHANS,
                                 num_classes=self.num_classes, embed_dim=sw.EMBED_DIM, depths=sw.DEPTHS,
                                 num_heads=sw.NUM_HEADS, window_size=sw.WINDOW_SIZE, mlp_ratio=sw.MLP_RATIO,
                                 qkv_bias=sw.QKV_BIAS, qk_scale=None, drop_rate=config.MODEL.DROP_RATE,
                                 drop_path_rate=config.MODEL.DROP_PATH_RATE, ape=sw.APE,
                                 patch_norm=sw.PATCH_NORM, use_checkpoint=config.TRAIN.USE_CHECKPOINT,
                                 attn_drop_rate=config.MODEL.ATTN_DROP_RATE)

    def forward(self, x):
        if x.size()[1] != 3:
            msg = f"Expected 3 channels, but got {x.size(1)}"
            logger.error(msg)
            raise ValueError(msg)
        return self.ms_unet(x)

    def freeze_encoder(self, freeze):
        self.ms_unet.freeze_encoder(freeze)

    def unfreeze_encoder(self, layer_num):
        self.ms_unet.unfreeze_encoder(layer_num)

    def load_segface_weight(self, config, logging):
        """``MSUNet.py:61-148``: SegFace backbone -> encoder (checkpoint.remap_segface)."""
        from .. import checkpoint
        msg = checkpoint.load_pretrained_file(self.ms_unet, config.MODEL.PRETRAIN_SEGFACE, "segface", logging)
        if msg is not None:
            logging.info("End of the Segface pretrained copying process")
        return msg

    def load_IMAGENET1K_weight(self, config, logging):
        """``MSUNet.py:150-229``: torchvision swin_b IMAGENET1K -> encoder
        (checkpoint.remap_imagenet1k)."""
        from .. import checkpoint
        msg = checkpoint.load_pretrained_file(self.ms_unet, config.MODEL.PRETRAIN_IMAGENET1K, "imagenet1k", logging)
        if msg is not None:
            logging.info("End of MAGENET1K the pretrained copying process")
        return msg
