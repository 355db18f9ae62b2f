"""Parallelism: flat parameter buffers, RCCL all-reduce DP, process-group bootstrap."""
from .flat import FlatParams, FlatGroup  # noqa: F401
from .ddp import DataParallel  # noqa: F401
from . import comm  # noqa: F401
from .async_ps import AsyncPSServer, AsyncPSWorker  # noqa: F401
from .strategy import MirroredStrategy  # noqa: F401
from .graphs import GraphedStep, capture_supported  # noqa: F401
from . import overlap  # noqa: F401
