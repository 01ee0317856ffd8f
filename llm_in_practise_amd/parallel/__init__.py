from .ddp import DDP, DistributedDataParallel
from .dist import barrier, destroy, init_distributed, is_dist, is_main, rank, world_size
from .ds_config import DSConfig, load_ds_config
from .zero import ZeroEngine, initialize

__all__ = ["DDP", "DistributedDataParallel", "barrier", "destroy", "init_distributed", "is_dist", "is_main",
           "rank", "world_size", "DSConfig", "load_ds_config", "ZeroEngine", "initialize"]
