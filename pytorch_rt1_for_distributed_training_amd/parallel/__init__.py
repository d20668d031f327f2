"""Data parallelism over RCCL (xGMI): process bootstrap, flat buffers, bucketed all-reduce."""
from .dist import DistContext, barrier, context, init_distributed, shutdown  # noqa: F401
from .ddp import DataParallel, gradient_ready_order  # noqa: F401
from .flat import FlatParameters, flatten_buffers  # noqa: F401
