"""I/O readers for the reference-compatible files and small profiling helpers."""
from .io import RECORD_DTYPE, read_hf2d, read_meta, read_plt, read_rms
from .profiling import StepTimer, rocprof_kernel_table

__all__ = ["RECORD_DTYPE", "read_hf2d", "read_meta", "read_plt", "read_rms", "StepTimer", "rocprof_kernel_table"]
