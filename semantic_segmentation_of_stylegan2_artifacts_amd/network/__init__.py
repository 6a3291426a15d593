from .MSUNet import MSUNet  # noqa: F401
from .model_parts import (MSUNetSys, PatchEmbed, PatchMerging, PatchExpand,  # noqa: F401
                          FinalPatchExpand_X4_V2, BasicLayer, BasicLayer_up, SwinTransformerBlock)
