from .DynamicLoss import DynamicLoss  # noqa: F401
