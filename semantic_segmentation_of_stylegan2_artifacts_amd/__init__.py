"""MI355X-native (gfx950) MS-UNet / Swin training hot path.

Drop-in for Sara-H-dev/Semantic_Segmentation_Of_StyleGAN2_Artifacts' ``network/MSUNet.py``,
``network/model_parts.py`` and ``loss/DynamicLoss.py``: same class names, signatures and
state-dict keys; compute in hand-written HIP kernels (``libmsunet_hip.so``).
"""
from .config import load_config, default_config  # noqa: F401
