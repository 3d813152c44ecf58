"""openhyperflow2d_amd — an MI355X-native re-build of OpenHyperFLOW2D.

A 2D flat/axisymmetric, transient, compressible, multicomponent, reacting
Euler/Navier-Stokes solver (explicit DEEPS blended LxF/central scheme) with
the reference's ``.dat`` deck format, Tecplot/RMS outputs and ``.hf2d``
checkpoint layout.  The time march runs as hand-written HIP kernels for
gfx950 over device-resident SoA state; strip-decomposed multi-GPU runs use
RCCL over xGMI (one process per GPU, bootstrapped with torch.distributed).

Layout
  models/    deck generators for the BASELINE configs, high-level Simulation
  ops/       Python entry points to the native kernels (tests / tooling)
  parallel/  strip decomposition, RCCL / gloo halo exchange, launchers
  utils/     output readers, profiling helpers
  csrc/      C++ core (deck parser, pre-processor, CPU steppers) + HIP kernels
"""
from __future__ import annotations

import importlib
import os

__version__ = "0.1.0"

_native = None


def native():
    """Load the in-tree native extension (building it if it is missing).

    torch (when importable) is imported first so that its bundled HIP runtime
    and RCCL are the ones our extension binds to (same SONAMEs)."""
    global _native
    if _native is not None:
        return _native
    try:  # keep a single HIP runtime in the process
        import torch  # noqa: F401
    except Exception:
        pass
    from . import _build

    if not _build.is_built() or os.environ.get("HF2D_REBUILD") == "1":
        _build.build()
    _native = importlib.import_module(__name__ + "._hf2d")
    return _native


def gpu_available() -> bool:
    return bool(native().gpu_available())


from .models.simulation import Simulation  # noqa: E402,F401
