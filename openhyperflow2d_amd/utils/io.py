"""Readers for the files the solver writes (and the reference writes):

* ``<Project>.hf2d``  -- raw x-major array of 1248-byte FlowNode2D<double,3>
  records, read with a numpy structured dtype
  (memory-mapped, no pickling) -- the reference's FlowField2D utility.
* ``<Project>.hf2d.meta`` -- JSON sidecar (iteration, dt, time).
* ``<Project>.plt`` / ``tp-<Project>.plt`` -- Tecplot/GNUPlot ASCII fields.
* ``RMS-<Project>.plt`` -- residual history.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Tuple

import numpy as np

NEQ = 9
NSPEC = 4

# Mirrors csrc/core/common.hpp CellRecord (static_asserts there pin the offsets).
RECORD_DTYPE = np.dtype([
    ("S", "<f8", NEQ), ("dSdx", "<f8", NEQ), ("dSdy", "<f8", NEQ),
    ("TurbType", "<u8"), ("l_min", "<f8"), ("y_plus", "<f8"), ("Re_local", "<f8"), ("mu_t", "<f8"),
    ("lam_t", "<f8"), ("dkdx", "<f8"), ("dkdy", "<f8"), ("depsdx", "<f8"), ("depsdy", "<f8"),
    ("x", "<f8"), ("y", "<f8"), ("ix", "<i4"), ("iy", "<i4"), ("nb_ptr", "<u8", 4), ("p", "<f8"),
    ("idXl", "<i4"), ("idYu", "<i4"), ("idXr", "<i4"), ("idYd", "<i4"), ("NGX", "<i4"), ("NGY", "<i4"),
    ("CT", "<u8"), ("i_wall", "<i4"), ("j_wall", "<i4"), ("beta", "<f8", NEQ), ("Q_conv", "<f8"),
    ("time", "<f8"), ("k", "<f8"), ("R", "<f8"), ("lam", "<f8"), ("mu", "<f8"), ("CP", "<f8"),
    ("Diff", "<f8"), ("Tf", "<f8"), ("A", "<f8", NEQ), ("B", "<f8", NEQ), ("F", "<f8", NEQ),
    ("RX", "<f8", NEQ), ("RY", "<f8", NEQ), ("Src", "<f8", NEQ), ("SrcAdd", "<f8", NEQ),
    ("Tg", "<f8"), ("U", "<f8"), ("V", "<f8"), ("Y", "<f8", NSPEC), ("Uw", "<f8"), ("Vw", "<f8"),
    ("droYdx", "<f8", NSPEC), ("droYdy", "<f8", NSPEC), ("dUdx", "<f8"), ("dUdy", "<f8"), ("dVdx", "<f8"),
    ("dVdy", "<f8"), ("dTdx", "<f8"), ("dTdy", "<f8"), ("BGX", "<f8"), ("BGY", "<f8"),
])
assert RECORD_DTYPE.itemsize == 1248, RECORD_DTYPE.itemsize


def read_hf2d(path: str, nx: int, ny: int, mmap: bool = True) -> np.ndarray:
    """(nx, ny) structured array of cell records (x-major, like the file)."""
    n = os.path.getsize(path) // RECORD_DTYPE.itemsize
    if n != nx * ny:
        raise ValueError("%s holds %d records, expected %d x %d" % (path, n, nx, ny))
    if mmap:
        a = np.memmap(path, dtype=RECORD_DTYPE, mode="r", shape=(nx * ny,))
    else:
        a = np.fromfile(path, dtype=RECORD_DTYPE)
    return a.reshape(nx, ny)


def read_meta(path: str) -> Dict:
    p = path if path.endswith(".meta") else path + ".meta"
    with open(p) as f:
        return json.load(f)


def read_plt(path: str) -> Tuple[List[str], List[np.ndarray]]:
    """Variable names and one (npoints, nvars) array per ZONE."""
    names: List[str] = []
    zones: List[np.ndarray] = []
    rows: List[List[float]] = []
    with open(path, errors="replace") as f:
        for line in f:
            s = line.strip()
            if not s:
                continue
            u = s.upper()
            if u.startswith("VARIABLES"):
                names = [t.strip().strip('"') for t in s.split("=", 1)[1].replace(",", " ").split() if t.strip('" ')]
                continue
            if u.startswith("TITLE"):
                continue
            if u.startswith("ZONE"):
                if rows:
                    zones.append(np.array(rows))
                    rows = []
                continue
            try:
                rows.append([float(t) for t in s.split()])
            except ValueError:
                continue
    if rows:
        zones.append(np.array(rows))
    return names, zones


def read_rms(path: str) -> np.ndarray:
    """Residual history: one row per output step (N, RMS[...])."""
    rows = []
    with open(path, errors="replace") as f:
        for line in f:
            try:
                rows.append([float(t) for t in line.split()])
            except ValueError:
                continue
    return np.array([r for r in rows if r])
