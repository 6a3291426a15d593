from .dataset import (SegArtifact_dataset, SegArtifact_no_label_dataset, RandomGenerator,  # noqa: F401
                      DataPrepartion, random_flip, augment_batch)
from .loader import GpuBatchLoader, epoch_plan, real_ratio_for_epoch  # noqa: F401
