from .adamw import AdamW, AdamW8bit, FlatParams, LRScheduler, build_optimizer

__all__ = ["AdamW", "AdamW8bit", "FlatParams", "LRScheduler", "build_optimizer"]
