"""Multi-rank execution: strip decomposition, RCCL (GPU) and gloo (CPU) halos."""
from .strips import balanced_columns, uniform_columns  # noqa: F401
from .dist import DistributedSimulation, init_from_env  # noqa: F401
