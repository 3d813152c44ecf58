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


def maybe_autotune(case, solver) -> str:
    """Deck key ThreadBlockSize = 0 (the reference's "auto-calibrate") tunes
    the lean kernel geometry on the device before the first step
    (DeviceSolver.autotune; results are unaffected).  HF2D_AUTOTUNE=0 skips."""
    if case.thread_block_size != 0 or os.environ.get("HF2D_AUTOTUNE", "1") == "0":
        return ""
    return solver.autotune()


def parse_fault(spec: str):
    """``step:N[,rank:R][,kind:nan|kill]`` -> (N, R, kind); "" -> (-1, 0, "nan").

    Fault injection for the failure paths: ``nan`` poisons one
    active cell's energy at global iteration N on rank R (Tg < 0 -> error
    snapshot ``<Project>-err.plt``, the last good checkpoint is kept),
    ``kill`` SIGKILLs that rank (restart from the checkpoint)."""
    if not spec:
        return -1, 0, "nan"
    kv = {}
    for part in spec.split(","):
        k, _, v = part.partition(":")
        kv[k.strip()] = v.strip()
    if "step" not in kv:
        raise ValueError("fault spec needs step:N, got %r" % spec)
    kind = kv.get("kind", "nan")
    if kind not in ("nan", "kill"):
        raise ValueError("fault kind must be nan or kill, got %r" % kind)
    return int(kv["step"]), int(kv.get("rank", 0)), kind


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
            self.autotune_log = maybe_autotune(self.case, self.solver)
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
            verbose: bool = True, metrics: str = "", profile: str = "", fault: str = ""):
        """Reference driver: outer cycles with outputs; returns (cycles, log text)."""
        step, rank, kind = parse_fault(fault)
        return self.solver.run(max_cycles, outdir, outputs, checkpoint, verbose, metrics, profile, step, rank, kind)

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
