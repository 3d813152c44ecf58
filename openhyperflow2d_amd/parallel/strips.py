"""1-D strip domain decomposition along X (one strip per rank / GPU).

The reference splits the columns so every rank holds about the same number
of active (non-solid) cells (ScanArea, libDEEPS2D/deeps2d_core.cpp:2143-2226)
and exchanges one ghost column with each neighbour.  Here every rank owns the
contiguous columns [gi0, gi1); the native steppers add the ghost columns.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


def balanced_columns(solid: np.ndarray, nparts: int) -> List[Tuple[int, int]]:
    """Cut [0, nx) into nparts contiguous ranges with ~equal active cells.

    ``solid`` is the (nx, ny) 0/1 solid mask.  Every part gets >= 1 column."""
    nx = solid.shape[0]
    if nparts <= 1:
        return [(0, nx)]
    if nparts > nx:
        raise ValueError("more strips than columns")
    active = (solid < 0.5).sum(axis=1).astype(np.float64)
    cum = np.concatenate([[0.0], np.cumsum(active)])
    total = cum[-1]
    cuts = [0]
    for k in range(1, nparts):
        target = total * k / nparts
        c = int(np.searchsorted(cum, target, side="left"))
        c = max(c, cuts[-1] + 1)
        c = min(c, nx - (nparts - k))
        cuts.append(c)
    cuts.append(nx)
    return [(cuts[k], cuts[k + 1]) for k in range(nparts)]


def uniform_columns(nx: int, nparts: int) -> List[Tuple[int, int]]:
    base, rem = divmod(nx, nparts)
    out, s = [], 0
    for k in range(nparts):
        w = base + (1 if k < rem else 0)
        out.append((s, s + w))
        s += w
    return out
