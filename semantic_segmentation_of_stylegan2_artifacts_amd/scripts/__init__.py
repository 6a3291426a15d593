from .batch_data_loader_V2 import BatchPatternSampler  # noqa: F401
