"""Finite-rate multi-reaction chemistry.

The reference's chemistry is the Zeldovich "infinite speed" global reaction
(deeps2d_core.cpp:4697-4780, reproduced in the fill kernels); its
``CRM_ARRENIUS`` model slot (hyper_flow_bound.hpp:37-42) is declared and never
implemented.  This module supplies that slot as a standalone operator:

* :class:`Mechanism` - a mass-action mechanism: up to 16 species, irreversible
  Arrhenius steps ``kf = A T^b exp(-Ta/T)`` (SI units, concentrations in mol/m^3)
  with up to 3 distinct reactants of integer order 0..3 (a reversible step is two
  entries);
* :func:`reference_step` - the plain PyTorch FP64 reference of one call:
  ``nsub`` linearised backward-Euler substeps ``(I - h N D) dc = h N q``,
  ``c <- max(c + dc, 0)`` at frozen temperature;
* :func:`mech_step_gpu` - the same update on the MFMA matrix cores
  (``csrc/hip/chem_mech.hip``: rates and per-cell Jacobians as
  ``v_mfma_f64_16x16x4_f64`` products; the ns x ns point-implicit systems are
  solved by Gauss-Jordan in registers, 16 lanes per cell).

Species are carried as ``rhoY`` in a species-major ``[ns, ncell]`` array (the
solver's SoA layout).  Heat release enters the caller's energy balance through
the formation enthalpies, as in the reference (the fill recomputes T from rhoE).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple

import numpy as np

MAX_SPECIES = 16


@dataclass
class Reaction:
    reactants: Dict[str, int]
    products: Dict[str, int]
    A: float            # SI: (m^3/mol)^(order-1) / s
    b: float = 0.0
    Ta: float = 0.0     # activation temperature Ea/Ru [K]


@dataclass
class Mechanism:
    species: List[str]
    W: np.ndarray                     # [ns] kg/mol
    reactions: List[Reaction] = field(default_factory=list)

    def __post_init__(self):
        self.W = np.asarray(self.W, dtype=np.float64)
        ns = len(self.species)
        if not 1 <= ns <= MAX_SPECIES or self.W.shape != (ns,):
            raise ValueError("mechanism needs 1..16 species with one molar mass each")
        if len(self.reactions) > 64:
            raise ValueError("at most 64 reactions (the kernel's reactant table)")
        for r in self.reactions:
            if len(r.reactants) > 3 or any(not 0 <= o <= 3 for o in r.reactants.values()):
                raise ValueError("at most 3 distinct reactants of order 0..3 per reaction")
            for s in list(r.reactants) + list(r.products):
                if s not in self.species:
                    raise ValueError("unknown species %r" % s)

    def to_dict(self) -> dict:
        return {"species": list(self.species), "W": [float(w) for w in self.W],
                "reactions": [{"reactants": r.reactants, "products": r.products, "A": r.A, "b": r.b, "Ta": r.Ta}
                              for r in self.reactions]}

    @classmethod
    def from_dict(cls, d: dict) -> "Mechanism":
        return cls(list(d["species"]), np.asarray(d["W"], dtype=np.float64),
                   [Reaction(dict(r["reactants"]), dict(r["products"]), float(r["A"]), float(r.get("b", 0.0)),
                             float(r.get("Ta", 0.0))) for r in d["reactions"]])

    def save(self, path: str) -> None:
        """JSON mechanism file (SI units: A in (m^3/mol)^(order-1)/s, Ta = Ea/Ru in K)."""
        import json

        with open(path, "w") as f:
            json.dump(self.to_dict(), f, indent=1)

    @classmethod
    def load(cls, path: str) -> "Mechanism":
        import json

        with open(path) as f:
            return cls.from_dict(json.load(f))

    @property
    def ns(self) -> int:
        return len(self.species)

    def packed(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
        """Device layout: nmat [16][R], arr [3R] (A|b|Ta), rsp/rord [R][3]; R padded to a multiple of 4."""
        n = len(self.reactions)
        R = max(4, (n + 3) // 4 * 4)
        idx = {s: i for i, s in enumerate(self.species)}
        nmat = np.zeros((MAX_SPECIES, R))
        arr = np.zeros((3, R))
        rsp = np.zeros((R, 3), dtype=np.int32)
        rord = np.zeros((R, 3), dtype=np.int32)
        for j, r in enumerate(self.reactions):
            for s, o in r.reactants.items():
                nmat[idx[s], j] -= o
            for s, o in r.products.items():
                nmat[idx[s], j] += o
            arr[:, j] = (r.A, r.b, r.Ta)
            for t, (s, o) in enumerate(r.reactants.items()):
                rsp[j, t], rord[j, t] = idx[s], o
        return nmat, arr.reshape(-1), rsp, rord


def h2_air_demo() -> Mechanism:
    """8-species / 12-step H2-O2 mechanism in N2 for tests and benchmarks.

    The step list follows the usual reduced H2/air chain (branching, shuffle,
    HO2 and termolecular recombination with N2 as the collider); the rate
    constants are literature-style magnitudes converted from cm^3/mol/s and are
    NOT a validated mechanism - load a real one into :class:`Mechanism` for
    production runs.
    """
    sp = ["H2", "O2", "H2O", "H", "O", "OH", "HO2", "N2"]
    W = [2.016e-3, 31.998e-3, 18.015e-3, 1.008e-3, 15.999e-3, 17.007e-3, 33.006e-3, 28.014e-3]
    c2, c3 = 1e-6, 1e-12      # cm^3/mol -> m^3/mol, cm^6/mol^2 -> m^6/mol^2
    R = Reaction
    rx = [
        R({"H": 1, "O2": 1}, {"OH": 1, "O": 1}, 3.52e16 * c2, -0.7, 8590.0),
        R({"OH": 1, "O": 1}, {"H": 1, "O2": 1}, 2.0e13 * c2, 0.0, 0.0),
        R({"O": 1, "H2": 1}, {"OH": 1, "H": 1}, 5.06e4 * c2, 2.67, 3166.0),
        R({"OH": 1, "H": 1}, {"O": 1, "H2": 1}, 2.2e4 * c2, 2.67, 2190.0),
        R({"OH": 1, "H2": 1}, {"H2O": 1, "H": 1}, 1.17e9 * c2, 1.3, 1829.0),
        R({"H2O": 1, "H": 1}, {"OH": 1, "H2": 1}, 6.4e9 * c2, 1.3, 9270.0),
        R({"OH": 2}, {"O": 1, "H2O": 1}, 3.57e4 * c2, 2.4, -1062.0),
        R({"H": 1, "O2": 1, "N2": 1}, {"HO2": 1, "N2": 1}, 5.75e19 * c3, -1.4, 0.0),
        R({"HO2": 1, "H": 1}, {"OH": 2}, 7.08e13 * c2, 0.0, 148.0),
        R({"HO2": 1, "H": 1}, {"H2": 1, "O2": 1}, 1.66e13 * c2, 0.0, 414.0),
        R({"HO2": 1, "OH": 1}, {"H2O": 1, "O2": 1}, 2.89e13 * c2, 0.0, -250.0),
        R({"H": 1, "OH": 1, "N2": 1}, {"H2O": 1, "N2": 1}, 2.2e22 * c3, -2.0, 0.0),
    ]
    return Mechanism(sp, np.array(W), rx)


def demo_state(mech: Mechanism, ncell: int, seed: int = 0, T_range=(1100.0, 2400.0)):
    """Synthetic premixed H2/air-like states: rhoY [ns, ncell], T [ncell]."""
    rng = np.random.default_rng(seed)
    ns = mech.ns
    Y = np.full((ns, ncell), 1e-6)
    name = {s: i for i, s in enumerate(mech.species)}
    if "H2" in name:
        Y[name["H2"]] = 0.028 * (0.5 + rng.random(ncell))
    if "O2" in name:
        Y[name["O2"]] = 0.226
    Y[:] *= 1.0 + 0.5 * rng.random((ns, ncell))
    if "N2" in name:
        Y[name["N2"]] = 0.0
        Y[name["N2"]] = 1.0 - Y.sum(axis=0)
    rho = 0.1 + 0.3 * rng.random(ncell)
    T = T_range[0] + (T_range[1] - T_range[0]) * rng.random(ncell)
    return rho * Y, T


def reference_step(mech: Mechanism, rhoY: np.ndarray, T: np.ndarray, dt: float, nsub: int = 1) -> np.ndarray:
    """Plain PyTorch FP64 reference of the K12 kernel (same algorithm, batched linalg.solve)."""
    import torch

    nmat, arr, rsp, rord = mech.packed()
    ns, R = mech.ns, nmat.shape[1]
    N = torch.tensor(nmat[:ns], dtype=torch.float64)                 # [ns, R]
    A, b, Ta = (torch.tensor(a, dtype=torch.float64) for a in arr.reshape(3, R))
    W = torch.tensor(mech.W, dtype=torch.float64)
    Tt = torch.tensor(np.asarray(T, dtype=np.float64))
    c = torch.tensor(np.asarray(rhoY, dtype=np.float64)).T / W      # [ncell, ns]
    kf = A * torch.exp(b * torch.log(Tt)[:, None] - Ta * (1.0 / Tt)[:, None])   # [ncell, R]
    h = dt / nsub
    eye = torch.eye(ns, dtype=torch.float64)
    for _ in range(nsub):
        pw = [c[:, rsp[:, t]] ** torch.tensor(rord[:, t], dtype=torch.float64) for t in range(3)]   # [ncell, R] each
        q = kf * pw[0] * pw[1] * pw[2]
        omega = q @ N.T                                                # [ncell, ns]
        D = torch.zeros(c.shape[0], R, ns, dtype=torch.float64)
        for t in range(3):
            o = torch.tensor(rord[:, t], dtype=torch.float64)
            dpw = o * c[:, rsp[:, t]] ** torch.clamp(o - 1, min=0)
            others = kf * pw[(t + 1) % 3] * pw[(t + 2) % 3] * dpw
            live = torch.tensor(rord[:, t] > 0)
            D[:, torch.arange(R)[live], torch.tensor(rsp[:, t])[live]] = others[:, live]
        J = N @ D                                                      # [ncell, ns, ns]
        dc = torch.linalg.solve(eye - h * J, h * omega)
        c = torch.clamp(c + dc, min=0.0)
    return (c * W).T.contiguous().numpy()


def mech_step_gpu(mech: Mechanism, rhoY: np.ndarray, T: np.ndarray, dt: float, nsub: int = 1,
                  repeats: int = 1) -> Tuple[np.ndarray, float]:
    """K12 on the GPU (``hf2d_chem_mech`` HIP kernel).  Returns (rhoY_new, mean kernel ms)."""
    import openhyperflow2d_amd as hf

    m = hf.native()
    if not m.gpu_available():
        raise RuntimeError("mech_step_gpu needs a HIP device")
    nmat, arr, rsp, rord = mech.packed()
    out = np.ascontiguousarray(rhoY, dtype=np.float64).copy()
    ms = m.chem_mech_run(nmat, arr, rsp, rord, mech.W, out, np.ascontiguousarray(T, dtype=np.float64), float(dt),
                         int(nsub), int(repeats))
    return out, ms


def benchmark(mech: Mechanism, ncell: int, dt: float = 1e-7, nsub: int = 4, repeats: int = 10,
              check_cells: int = 4096, seed: int = 11) -> dict:
    """Time the K12 kernel on ``ncell`` synthetic states and check a cell subset against
    :func:`reference_step`.  Returns a JSON-able dict (``rel_err_vs_torch_fp64`` included)."""
    Y, T = demo_state(mech, ncell, seed=seed)
    got, ms = mech_step_gpu(mech, Y, T, dt, nsub, repeats=repeats)
    sel = np.random.default_rng(0).choice(ncell, size=min(ncell, check_cells), replace=False)
    ref = reference_step(mech, Y[:, sel], T[sel], dt, nsub)
    err = float(np.abs(got[:, sel] - ref).max() / np.abs(ref).max())
    R = mech.packed()[0].shape[1]
    # MFMA work issued: per 16-cell tile and substep, (1 + 16) chains of R/4 16x16x4 f64 MFMAs
    mfma_flop = (ncell / 16) * nsub * 17 * (R / 4) * (2 * 16 * 16 * 4)
    return {"metric": "K12 mechanism chemistry", "cells": ncell, "species": mech.ns, "reactions": len(mech.reactions),
            "nsub": nsub, "dt": dt, "ms_per_call": ms, "Mcells_per_s": ncell / ms / 1e3,
            "mfma_f64_tflops": mfma_flop / ms / 1e9, "rel_err_vs_torch_fp64": err}


def element_mass(mech: Mechanism, rhoY: np.ndarray) -> np.ndarray:
    """Total mass per cell (sum of rhoY); conserved by a balanced mechanism before clipping."""
    return np.asarray(rhoY).sum(axis=0)


__all__ = ["Mechanism", "Reaction", "h2_air_demo", "demo_state", "reference_step", "mech_step_gpu", "benchmark", "element_mass"]
