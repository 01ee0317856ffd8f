from .device import get_device, is_gfx950, hbm_stats, synchronize  # noqa: F401
from .env import DistEnv, dist_env  # noqa: F401
