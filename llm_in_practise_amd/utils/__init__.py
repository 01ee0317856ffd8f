from .logging import get_logger, rank0_print
from .metrics import MetricsWriter
from .timer import StepTimer
from .faults import FaultInjector, InjectedFault

__all__ = ["get_logger", "rank0_print", "MetricsWriter", "StepTimer", "FaultInjector", "InjectedFault"]
