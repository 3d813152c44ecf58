"""High-level simulation object: deck -> pre-processed case -> stepper.

Backends
  ``gpu``  DeviceSolver: HIP kernels on an MI355X (default when a GPU exists)
  ``cpu``  CpuSolver: the same per-cell kernels on the host (Jacobi order)
  ``ref``  RefSolver: the reference's in-place sweep order (golden oracle)
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np


class Simulation:
    def __init__(self, deck_text: str, backend: Optional[str] = None, *, workdir: str = ".",
                 use_checkpoint: bool = False, device: int = 0, semantics: str = "mpi",
                 gi0: int = 0, gi1: int = -1, fused: bool = True, lean: Optional[bool] = None):
        from .. import native

        hf = native()
        self.hf = hf
        self.case = hf.Case.from_deck(deck_text, workdir, use_checkpoint)
        self.case.set_semantics(semantics)
        if backend is None:
            backend = "gpu" if hf.gpu_available() else "cpu"
        self.backend = backend
        if backend == "gpu":
            self.solver = hf.DeviceSolver(self.case, device, gi0, gi1)
            self.solver.fused = fused
            self.solver.lean = True if lean is None else bool(lean)
        elif backend == "cpu":
            self.solver = hf.CpuSolver(self.case, gi0, gi1)
            self.solver.lean = False if lean is None else bool(lean)
        elif backend == "ref":
            self.solver = hf.RefSolver(self.case)
        else:
            raise ValueError("unknown backend %r" % backend)

    @classmethod
    def from_file(cls, path: str, backend: Optional[str] = None, **kw) -> "Simulation":
        with open(path, "r", errors="replace") as f:
            text = f.read()
        kw.setdefault("workdir", os.path.dirname(os.path.abspath(path)))
        return cls(text, backend, **kw)

    # -- time march ------------------------------------------------------
    def step(self, n: int = 1, residual: bool = False) -> None:
        self.solver.run_steps(int(n), bool(residual))

    def run(self, max_cycles: int = 1, outdir: str = ".", outputs: bool = True, checkpoint: bool = True,
            verbose: bool = True, metrics: str = ""):
        """Reference driver: outer cycles with outputs; returns (cycles, log text)."""
        return self.solver.run(max_cycles, outdir, outputs, checkpoint, verbose, metrics)

    def summary(self) -> dict:
        return dict(self.solver.summary())

    # -- data access -------------------------------------------------------
    def field(self, name: str) -> np.ndarray:
        self.solver.download()
        return np.asarray(self.case.field(name))

    def records(self) -> bytes:
        self.solver.download()
        return self.case.records()

    @property
    def shape(self):
        return (self.case.nx, self.case.ny)
