"""Finite-rate kinetics operators on the GPU.

The reference's chemistry is the Zeldovich "infinite speed" global reaction
(deeps2d_core.cpp:4697-4780, reproduced in the fill kernels); its
``CRM_ARRENIUS`` slot (hyper_flow_bound.hpp:37-42) is declared and never
implemented.  Mechanism mode fills it (``ops/mechanism.py`` for the data and
the NumPy oracle, ``csrc/core/mechanism.hpp`` for the solver coupling).  This
module runs the two device implementations of the kinetics operator as
standalone operators -- the same kernels the time step launches:

* ``kernel="fast"`` -- ``hf2d_chem_fast`` (chem_fast.hip): compiled mechanisms
  (the built-in Li et al. 2004 H2/air set), one cell per lane, the system of a
  cell in registers, sparse Jacobian accumulation;
* ``kernel="mfma"`` -- ``hf2d_chem_mech`` (chem_mech.hip): any mechanism loaded
  at run time (<= 16 species, <= 64 reactions); Gibbs / collider / rate /
  Jacobian algebra as ``v_mfma_f64_16x16x4_f64`` tiles, 16 cells per wavefront.

Both advance ``rhoY [ns, n]`` at constant density and internal energy over
``dt`` with ``nsub`` linearised backward-Euler substeps and return the new
partial densities and temperatures; :func:`mechanism.point_implicit_step` is
their FP64 oracle.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from .mechanism import (Mechanism, Reaction, Species, h2_air_li2004, mixture_e,  # noqa: F401
                        point_implicit_step, premixed_Y)

MAX_SPECIES = 16


def _native():
    import openhyperflow2d_amd as hf

    m = hf.native()
    if not m.gpu_available():
        raise RuntimeError("the kinetics kernels need a HIP device")
    return m


def mech_step_gpu(mech: Mechanism, rhoY: np.ndarray, rho: np.ndarray, e: np.ndarray, T: np.ndarray, dt: float,
                  nsub: int = 1, kernel: str = "mfma", repeats: int = 1) -> Tuple[np.ndarray, np.ndarray, float]:
    """One kinetics call on the GPU.  Returns (rhoY_new, T_new, mean kernel ms)."""
    m = _native()
    rhoY = np.ascontiguousarray(rhoY, dtype=np.float64)
    args = (rhoY, np.ascontiguousarray(rho, dtype=np.float64), np.ascontiguousarray(e, dtype=np.float64),
            np.ascontiguousarray(T, dtype=np.float64), float(dt), int(nsub), int(repeats))
    if kernel == "fast":
        return m.chem_fast_run(mech.name, *args)
    if kernel not in ("mfma", "valu"):
        raise ValueError("kernel must be 'fast', 'mfma' or 'valu'")
    # 'valu': the runtime-data VALU form of the MFMA kernel's operator (equal terms)
    return m.chem_mech_run(mech.to_text(), *args, valu=kernel == "valu")


def demo_state(mech: Mechanism, ncell: int, seed: int = 0, T_range=(1000.0, 2600.0)):
    """Partially burnt premixed H2/air-like states: (rhoY [ns, n], rho, e, T)."""
    rng = np.random.default_rng(seed)
    Y = np.zeros((mech.ns, ncell))
    base = premixed_Y(mech, 1.0) if all(s in mech.names for s in ("H2", "O2", "N2")) else None
    if base is not None:
        Y[:] = base[:, None]
        # a little product and radicals
        for s, f in (("H2O", 0.05), ("OH", 2e-3), ("H", 2e-4), ("O", 5e-4), ("HO2", 1e-5)):
            if s in mech.names:
                Y[mech.index(s)] = f * rng.random(ncell)
        Y[-1] = 0.0
        Y[-1] = 1.0 - Y.sum(0)
    else:
        Y = rng.random((mech.ns, ncell))
        Y /= Y.sum(0)
    T = T_range[0] + (T_range[1] - T_range[0]) * rng.random(ncell)
    rho = 0.05 + 0.5 * rng.random(ncell)
    return rho * Y, rho, mixture_e(mech, Y.T, T), T


def increment_error(got: np.ndarray, ref: np.ndarray, y0: np.ndarray) -> float:
    """max over species of max|got - ref| / max|ref - y0|: each species against its
    own increment, so radicals are not hidden behind the bath gas.  The increment
    is floored at 1e-6 of the species' level (an inert bath gas changes by
    rounding only)."""
    inc = np.abs(ref - y0).max(1)
    lvl = np.abs(y0).max(1)
    err = np.abs(got - ref).max(1)
    return float((err / np.maximum(np.maximum(inc, 1e-6 * lvl), 1e-300)).max())


def benchmark(mech: Mechanism, ncell: int, dt: float = 1e-7, nsub: int = 1, repeats: int = 10,
              kernel: str = "fast", check_cells: int = 4096, seed: int = 11) -> dict:
    """Time one kernel on ``ncell`` synthetic states; check a subset against the
    NumPy FP64 oracle (per-species increment error)."""
    Y, rho, e, T = demo_state(mech, ncell, seed=seed)
    got, Tg, ms = mech_step_gpu(mech, Y, rho, e, T, dt, nsub, kernel=kernel, repeats=repeats)
    sel = np.random.default_rng(0).choice(ncell, size=min(ncell, check_cells), replace=False)
    ref, Tref = point_implicit_step(mech, Y[:, sel], rho[sel], e[sel], T[sel], dt, nsub)
    err = increment_error(got[:, sel], ref, Y[:, sel])
    return {"metric": "K12 kinetics operator (%s kernel)" % kernel, "mechanism": mech.name, "cells": ncell,
            "species": mech.ns, "reactions": mech.nr, "nsub": nsub, "dt": dt, "ms_per_call": ms,
            "Mcells_per_s": ncell / ms / 1e3, "incr_err_vs_numpy_fp64": err,
            "T_err_K": float(np.abs(Tg[sel] - Tref).max())}


__all__ = ["Mechanism", "Reaction", "Species", "h2_air_li2004", "mech_step_gpu", "demo_state", "benchmark",
           "increment_error", "point_implicit_step"]
