"""Deck generators for the BASELINE.json configurations.

The reference ships only four decks (TestCases/*.dat) and none at the
BASELINE grid sizes, so the benchmark/test decks are derived
here from the shipped Wedge deck (same property tables and key catalogue) by
rewriting grid, physics and geometry keys.  Every generated deck is a plain
OpenHyperFLOW2D ``.dat`` file and runs unchanged in the reference binary.

* ``wedge15``       — 15° compression ramp, M=2.5 air (BASELINE config 1 and the
                      headline Wedge15 2000×200 metric); Euler by default.
* ``step``          — Mach-3 forward-facing step (Woodward–Colella), laminar N-S.
* ``resonator``     — Hartmann–Sprenger-style axisymmetric jet/cavity, k-ε.
* ``triple_point``  — three-state shock interaction with a 3-component mix.
* ``scramjet``      — axisymmetric Mach-8 H2/air inlet-combustor channel, SST +
                      finite-rate chemistry (new physics keys, see docs).
"""
from __future__ import annotations

import math
import os
import re
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

_HERE = os.path.dirname(os.path.abspath(__file__))
_TEMPLATE_DIRS = [
    os.path.join(_HERE, "..", "..", "tests", "fixtures", "decks"),
    os.path.join(_HERE, "..", "..", "decks"),
]


def template_text(name: str = "Wedge.dat") -> str:
    for d in _TEMPLATE_DIRS:
        p = os.path.join(d, name)
        if os.path.exists(p):
            with open(p, "r", errors="replace") as f:
                return f.read()
    raise FileNotFoundError(name)


def set_key(text: str, key: str, value) -> str:
    """Replace the first ``<data/key=...>`` directive (append if absent)."""
    pat = re.compile(r"<data/" + re.escape(key) + r"=[^>]*>")
    val = value if isinstance(value, str) else repr(value) if isinstance(value, float) else str(value)
    if isinstance(value, float):
        val = "%.17g" % value
    if pat.search(text):
        return pat.sub("<data/%s=%s>" % (key, val), text, count=1)
    end = re.search(r"<end/[^>]*>", text)
    ins = "<data/%s=%s>\n" % (key, val)
    return text[: end.start()] + ins + text[end.start():]


def set_table(text: str, name: str, rows: Sequence[Tuple[float, float]]) -> str:
    body = "<table=%s/%d>\n" % (name, len(rows)) + "".join("%.17g %.17g\n" % (x, y) for x, y in rows) + "<endtable>"
    pat = re.compile(r"<table=" + re.escape(name) + r"/\d+>.*?<endtable>", re.S)
    if pat.search(text):
        return pat.sub(lambda m: body, text, count=1)
    end = re.search(r"<end/[^>]*>", text)
    return text[: end.start()] + body + "\n" + text[end.start():]


def remove_commented_directives(text: str) -> str:
    """Lines starting with ';' still define keys in the reference parser;
    drop those that would shadow generated keys."""
    out = []
    for line in text.splitlines():
        s = line.lstrip()
        if s.startswith(";") and ("<data/" in s or "<table=" in s):
            continue
        out.append(line)
    return "\n".join(out) + "\n"


def _rename(text: str, project: str) -> str:
    text = re.sub(r"<start/[^>]*>", "<start/%s>" % project, text, count=1)
    text = re.sub(r"<end/[^>]*>", "<end/%s>" % project, text, count=1)
    return set_key(text, "ProjectName", project)


def wedge15(nx: int = 200, ny: int = 40, *, navier_stokes: bool = False, turbulence: int = 0,
            nmax: int = 200, nout: int = 100, mach: float = 2.5, angle_deg: float = 15.0,
            project: Optional[str] = None, ramp_start: Optional[float] = None,
            exit_time: float = 1.0e-30) -> str:
    """15° wedge/ramp in a supersonic stream (cf. TestCases/Wedge.dat:447-519).

    The physical height is ``ny*dy`` with dx = dy = 1 mm; the ramp starts at
    ``ramp_start*L`` and rises at ``angle_deg`` to the outlet.  The ramp start
    is chosen so at least 1/3 of the outlet height stays gas."""
    t = remove_commented_directives(template_text("Wedge.dat"))
    project = project or "Wedge15_%dx%d" % (nx, ny)
    t = _rename(t, project)
    dx = dy = 1.0e-3
    L, H = nx * dx, ny * dy
    tan_a = math.tan(math.radians(angle_deg))
    if ramp_start is None:
        # ramp height at outlet <= 2/3 H
        run = min(0.7 * L, (2.0 / 3.0) * H / tan_a)
        ramp_start = 1.0 - run / L
    x0 = ramp_start * L
    h_out = (L - x0) * tan_a
    t = set_key(t, "MaxX", nx)
    t = set_key(t, "MaxY", ny)
    t = set_key(t, "dx", dx)
    t = set_key(t, "dy", dy)
    t = set_key(t, "ProblemType", 1 if navier_stokes else 0)
    t = set_key(t, "TurbulenceModel", turbulence)
    t = set_key(t, "TurbExtModel", 4)
    t = set_key(t, "isTurbulenceReset", 1 if turbulence else 0)
    t = set_key(t, "Nmax", nmax)
    t = set_key(t, "NOutStep", nout)
    t = set_key(t, "MonitorIndex", 5)
    t = set_key(t, "ExitMonitorValue", exit_time)
    t = set_key(t, "isAdiabaticWall", 1 if not navier_stokes else 0)
    t = set_key(t, "Flow2D-1.Mach", mach)
    eps = 1e-5
    rows = [(0.0, H), (L - eps, H), (L - eps, h_out), (x0, 0.0), (0.0, 0.0)]
    t = set_table(t, "Contour1", rows)
    tm = turbulence
    for b in range(1, 6):
        t = set_key(t, "Contour1.Bound%d.TurbulenceModel" % b, tm)
    t = set_table(t, "Area1", [(3, ny // 2)])
    t = set_table(t, "Area2", [(nx - 3, 1)])
    return t


def flat_plate(nx: int = 250, ny: int = 100, *, dx: float = 1.0e-3, dy: float = 1.0e-4, x_le: float = 0.2,
               mach: float = 2.5, p: float = 1.0e3, T: float = 288.9, turbulence: int = 0,
               nmax: int = 200, nout: int = 100, project: Optional[str] = None, cfl: Optional[float] = None) -> str:
    """Zero-pressure-gradient flat plate (validation): the Wedge template with a
    0-degree ramp, so the no-slip bound runs along y = 0 from ``x_le*L`` to
    the outlet, a symmetry line ahead of it, far-field inflow and top, a
    non-reflecting outlet.  ``turbulence``: the deck's TurbulenceModel code
    (0 laminar, 4 k-eps, 6 k-omega SST)."""
    t = remove_commented_directives(template_text("Wedge.dat"))
    project = project or "FlatPlate_%dx%d" % (nx, ny)
    t = _rename(t, project)
    L, H = nx * dx, ny * dy
    x0 = x_le * L
    t = set_key(t, "MaxX", nx)
    t = set_key(t, "MaxY", ny)
    t = set_key(t, "dx", dx)
    t = set_key(t, "dy", dy)
    t = set_key(t, "ProblemType", 1)
    t = set_key(t, "TurbulenceModel", turbulence)
    t = set_key(t, "TurbExtModel", 4)
    t = set_key(t, "isTurbulenceReset", 1 if turbulence else 0)
    t = set_key(t, "Nmax", nmax)
    t = set_key(t, "NOutStep", nout)
    t = set_key(t, "MonitorIndex", 5)
    t = set_key(t, "ExitMonitorValue", 1.0e-30)
    t = set_key(t, "isAdiabaticWall", 0)
    t = set_key(t, "Ts0", T)
    for f in (1, 2):
        t = set_key(t, "Flow2D-%d.p" % f, p)
        t = set_key(t, "Flow2D-%d.T" % f, T)
    t = set_key(t, "Flow2D-1.Mach", mach)
    if cfl is not None:
        t = set_key(t, "CFL", cfl)
        t = set_table(t, "CFL_Scenario", [(0.0, cfl), (1.0e9, cfl)])
    eps = 1e-9
    t = set_table(t, "Contour1", [(0.0, H), (L - eps, H), (L - eps, 0.0), (x0, 0.0), (0.0, 0.0)])
    for b in range(1, 6):
        t = set_key(t, "Contour1.Bound%d.TurbulenceModel" % b, turbulence)
    t = set_table(t, "Area1", [(3, ny // 2)])
    t = set_key(t, "Area1.TurbulenceModel", turbulence)
    t = set_key(t, "NumArea", 1)   # no solid under the plate: it is the domain edge
    return t


def mixing_layer(nx: int = 600, ny: int = 300, *, dx: float = 5.0e-4, dy: float = 1.0e-4, mach1: float = 2.0,
                 mach2: float = 1.2, p: float = 5.0e4, T: float = 300.0, turbulence: int = 6, nmax: int = 200,
                 nout: int = 100, project: Optional[str] = None, cfl: Optional[float] = None) -> str:
    """Compressible plane mixing layer (validation of the turbulence models):
    the Wedge template's five-bound contour re-shaped so the inflow edge is
    split at mid height -- the fast stream (Flow2D-1, ``mach1``) above, the
    slow one (Flow2D-2, ``mach2``) below, both at ``p``, ``T`` -- with
    far-field top (stream 1) and bottom (stream 2) edges and a
    non-reflecting outlet.  ``turbulence``: TurbulenceModel code (6 SST)."""
    t = remove_commented_directives(template_text("Wedge.dat"))
    project = project or "MixingLayer_%dx%d" % (nx, ny)
    t = _rename(t, project)
    L, H = nx * dx, ny * dy
    eps = 1e-9
    t = set_key(t, "MaxX", nx)
    t = set_key(t, "MaxY", ny)
    t = set_key(t, "dx", dx)
    t = set_key(t, "dy", dy)
    t = set_key(t, "ProblemType", 1)
    t = set_key(t, "TurbulenceModel", turbulence)
    t = set_key(t, "TurbExtModel", 4)
    t = set_key(t, "isTurbulenceReset", 1 if turbulence else 0)
    t = set_key(t, "Nmax", nmax)
    t = set_key(t, "NOutStep", nout)
    t = set_key(t, "MonitorIndex", 5)
    t = set_key(t, "ExitMonitorValue", 1.0e-30)
    t = set_key(t, "isAdiabaticWall", 1)
    t = set_key(t, "Ts0", T)
    t = set_key(t, "Flow2D-1.Mode", 2)
    t = set_key(t, "Flow2D-2.Mode", 2)
    t = set_key(t, "Flow2D-1.Mach", mach1)
    t = set_key(t, "Flow2D-2.Mach", mach2)
    t = set_key(t, "Flow2D-2.Angle", 0.0)
    for f in (1, 2):
        t = set_key(t, "Flow2D-%d.p" % f, p)
        t = set_key(t, "Flow2D-%d.T" % f, T)
    if cfl is not None:
        t = set_key(t, "CFL", cfl)
        t = set_table(t, "CFL_Scenario", [(0.0, cfl), (1.0e9, cfl)])
    # top (stream 1), outlet, bottom (stream 2), lower inflow (2), upper inflow (1)
    t = set_table(t, "Contour1", [(0.0, H), (L - eps, H), (L - eps, 0.0), (0.0, 0.0), (0.0, 0.5 * H)])
    far = "NT_FARFIELD_2D, TCT_k_CONST_2D, TCT_eps_CONST_2D"
    conds = [far, "NT_D0X_2D, TCT_dkdx_NULL_2D, TCT_depsdx_NULL_2D,  CT_NONREFLECTED_2D", far, far, far]
    flows = [1, 1, 2, 2, 1]
    for b in range(1, 6):
        t = set_key(t, "Contour1.Bound%d.Cond" % b, conds[b - 1])
        t = set_key(t, "Contour1.Bound%d.Flow2D" % b, flows[b - 1])
        t = set_key(t, "Contour1.Bound%d.TurbulenceModel" % b, turbulence)
    t = set_table(t, "Area1", [(3, 3)])
    t = set_key(t, "Area1.Flow2D", 2)
    t = set_key(t, "Area1.TurbulenceModel", turbulence)
    t = set_key(t, "NumArea", 1)
    return t


def step(nx: int = 1200, ny: int = 400, *, navier_stokes: bool = True, nmax: int = 200, nout: int = 100,
         project: Optional[str] = None, exit_time: float = 1.0e-30) -> str:
    """Mach-3 forward-facing step (TestCases/Step.dat rescaled)."""
    t = remove_commented_directives(template_text("Step.dat"))
    project = project or "Step_%dx%d" % (nx, ny)
    t = _rename(t, project)
    ref = _keys(t)
    ox, oy = int(ref["MaxX"]), int(ref["MaxY"])
    sx, sy = ox / nx, oy / ny
    dx = float(ref["dx"]) * sx
    dy = float(ref["dy"]) * sy
    t = set_key(t, "MaxX", nx)
    t = set_key(t, "MaxY", ny)
    t = set_key(t, "dx", dx)
    t = set_key(t, "dy", dy)
    t = set_key(t, "ProblemType", 1 if navier_stokes else 0)
    t = set_key(t, "Nmax", nmax)
    t = set_key(t, "NOutStep", nout)
    t = set_key(t, "MonitorIndex", 5)
    t = set_key(t, "ExitMonitorValue", exit_time)
    # area seeds are in nodes: rescale
    for name in _tables(t):
        if re.fullmatch(r"Area\d+", name):
            rows = _table_rows(t, name)
            t = set_table(t, name, [(min(max(int(x / sx), 2), nx - 3), min(max(int(y / sy), 2), ny - 3))
                                    for x, y in rows])
    return t


def _keys(text: str) -> Dict[str, str]:
    d: Dict[str, str] = {}
    for m in re.finditer(r"<data/([^=>]+)=([^>]*)>", text):
        d.setdefault(m.group(1), m.group(2))
    return d


def _tables(text: str) -> List[str]:
    return [m.group(1) for m in re.finditer(r"<table=([^/]+)/\d+>", text)]


def _table_rows(text: str, name: str) -> List[Tuple[float, float]]:
    m = re.search(r"<table=" + re.escape(name) + r"/\d+>\n(.*?)<endtable>", text, re.S)
    rows = []
    for line in m.group(1).splitlines():
        parts = line.split()
        if len(parts) >= 2:
            rows.append((float(parts[0]), float(parts[1])))
    return rows


def write(text: str, path: str) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)
    return path


# boundary conditions with the turbulence-equation conditions of Wedge.dat
_AXIS = "NT_AX_2D, TCT_dkdy_NULL_2D, TCT_depsdy_NULL_2D"
_OUTFLOW = "NT_D0X_2D, TCT_dkdx_NULL_2D, TCT_depsdx_NULL_2D, CT_NONREFLECTED_2D"
_FARFIELD = "NT_FARFIELD_2D, TCT_k_CONST_2D, TCT_eps_CONST_2D"
_WALL = "NT_WNS_2D, TCT_eps_Cmk2kXn_WALL_2D"
_INFLOW = "NT_FC_2D, TCT_k_CONST_2D, TCT_eps_CONST_2D"


def _defaults_from_wedge(t: str, keys: Iterable[str]) -> str:
    """Add keys the stale reference decks lack (e.g. TriplePoint.dat, SURVEY
    Q13) with the values of the maintained Wedge.dat deck."""
    w = _keys(template_text("Wedge.dat"))
    have = _keys(t)
    for k in keys:
        if k not in have:
            t = set_key(t, k, w[k])
    return t


def _const_table(v: float) -> List[Tuple[float, float]]:
    return [(0.0, v), (1.0e5, v)]


def triple_point(nx: int = 4000, ny: int = 1000, *, nmax: int = 200, nout: int = 100,
                 project: Optional[str] = None, exit_time: float = 1.0e-30,
                 gammas: Sequence[float] = (1.5, 1.4, 1.5)) -> str:
    """Three-state shock interaction (TestCases/TriplePoint.dat, axisymmetric
    Euler) at a BASELINE grid, with the three states carried by three
    different gases (fuel/oxidiser/product slots given non-dimensional
    properties R = 1, Cp = gamma/(gamma-1), no reaction): a 3-component mix.

    The shipped deck is stale (no isAlternateRMS / MonitorIndex / ... keys,
    SURVEY Q13); the missing keys are filled from Wedge.dat.  Geometry stays in
    metres (0.07 x 0.03); the grid spacing follows nx, ny."""
    t = remove_commented_directives(template_text("TriplePoint.dat"))
    t = _defaults_from_wedge(t, ["isIgnoreUnsetNodes", "ThreadBlockSize", "isAlternateRMS", "MonitorIndex",
                                 "beta_NonReflectedBC"])
    project = project or "TriplePoint_%dx%d" % (nx, ny)
    t = _rename(t, project)
    ref = _keys(t)
    ox, oy = int(ref["MaxX"]), int(ref["MaxY"])
    Lx, Ly = ox * float(ref["dx"]), oy * float(ref["dy"])
    t = set_key(t, "MaxX", nx)
    t = set_key(t, "MaxY", ny)
    t = set_key(t, "dx", Lx / nx)
    t = set_key(t, "dy", Ly / ny)
    t = set_key(t, "Nmax", nmax)
    t = set_key(t, "NOutStep", nout)
    t = set_key(t, "MonitorIndex", 5)
    t = set_key(t, "ExitMonitorValue", exit_time)
    t = set_key(t, "isAlternateRMS", 1)
    for name in _tables(t):
        if re.fullmatch(r"Area\d+", name):
            rows = _table_rows(t, name)
            t = set_table(t, name, [(max(1, int(x * nx / ox)), max(1, int(y * ny / oy))) for x, y in rows])
    # three gases, one per state; no reaction
    for comp, (flow, sp, g) in enumerate(zip((1, 2, 3), ("Fuel", "OX", "cp"), gammas)):
        t = set_key(t, "Flow2D-%d.CompIndex" % flow, comp)
        t = set_key(t, "R_%s" % sp, 1.0)
        t = set_key(t, "H_%s" % sp, 0.0)
        t = set_table(t, "Cp_%s" % sp, _const_table(g / (g - 1.0)))
    t = set_key(t, "Tf", 1.0e30)
    return t


def resonator(nx: int = 2000, ny: int = 200, *, nmax: int = 200, nout: int = 100, turbulence: int = 4,
              project: Optional[str] = None, exit_time: float = 1.0e-30, jet_mach: float = 1.05,
              jet_p: float = 2.6e5, jet_T: float = 250.0) -> str:
    """Hartmann-Sprenger resonator: an under-expanded axisymmetric air jet
    (nozzle radius 2 mm) impinging on a closed-end tube on the axis, k-eps
    URANS, no-slip walls.  Domain 0.1 m x 0.01 m (dx = dy = 0.05 mm at
    2000x200).  No reference deck exists (Makefile:50 names an absent
    CIAM-Resonator.dat); the geometry is authored here from the Wedge.dat key
    catalogue (contour + two solid rectangles)."""
    t = remove_commented_directives(template_text("Wedge.dat"))
    project = project or "Resonator_%dx%d" % (nx, ny)
    t = _rename(t, project)
    L, H = 0.1, 0.01
    dx, dy = L / nx, H / ny
    t = set_key(t, "MaxX", nx)
    t = set_key(t, "MaxY", ny)
    t = set_key(t, "dx", dx)
    t = set_key(t, "dy", dy)
    t = set_key(t, "FlowType", 1)
    t = set_key(t, "ProblemType", 1)
    t = set_key(t, "TurbulenceModel", turbulence)
    t = set_key(t, "isTurbulenceReset", 1)
    t = set_key(t, "isAdiabaticWall", 1)
    t = set_key(t, "Nmax", nmax)
    t = set_key(t, "NOutStep", nout)
    t = set_key(t, "MonitorIndex", 5)
    t = set_key(t, "ExitMonitorValue", exit_time)
    # flows: 1 jet (Mach/angle/static p,T), 2 ambient, 3 ambient for the rects
    # (SolidBoundRect2D zeroes the velocity of the flow it references)
    t = set_key(t, "NumFlow2D", 3)
    t = set_key(t, "Flow2D-1.Mode", 2)
    t = set_key(t, "Flow2D-1.Mach", jet_mach)
    t = set_key(t, "Flow2D-1.Angle", 0.0)
    t = set_key(t, "Flow2D-1.p", jet_p)
    t = set_key(t, "Flow2D-1.T", jet_T)
    t = set_key(t, "Flow2D-1.U", 0.0)
    t = set_key(t, "Flow2D-1.V", 0.0)
    for f in (2, 3):
        t = set_key(t, "Flow2D-%d.CompIndex" % f, 3)
        t = set_key(t, "Flow2D-%d.Mode" % f, 0)
        t = set_key(t, "Flow2D-%d.p" % f, 1.0e5)
        t = set_key(t, "Flow2D-%d.T" % f, 288.0)
        t = set_key(t, "Flow2D-%d.U" % f, 0.0)
        t = set_key(t, "Flow2D-%d.V" % f, 0.0)
    r_n = 0.002
    # contour on the outermost grid nodes: the reference maps contour points to
    # nodes as (int)(x / dx), (int)(y / dy - 1)
    xe, ye = (nx - 0.75) * dx, (ny + 0.25) * dy
    # resonator tube (inner radius r_t, wall w, open end at x_t facing the
    # nozzle, closed at x_c) carried by a solid sting to the outlet: the
    # closed end and the sting are part of the domain contour, the annular
    # tube wall is a solid rectangle.
    x_t, x_c, r_t, w = 0.012, 0.024, 0.0022, 0.001
    r_s = r_t + w
    rows = [(0.0, 0.0), (x_c, 0.0), (x_c, r_s + dy), (xe, r_s + dy), (xe, ye), (0.0, ye), (0.0, r_n + dy)]
    t = set_table(t, "Contour1", rows)
    conds = [_AXIS, _WALL, _WALL, _OUTFLOW, _FARFIELD, _WALL, _INFLOW]
    flows = [2, 2, 2, 2, 2, 2, 1]
    for b in range(1, len(conds) + 1):
        t = set_key(t, "Contour1.Bound%d.Cond" % b, conds[b - 1])
        t = set_key(t, "Contour1.Bound%d.Flow2D" % b, flows[b - 1])
        t = set_key(t, "Contour1.Bound%d.TurbulenceModel" % b, turbulence)
        t = set_key(t, "Contour1.Bound%d.isReset" % b, 0)
    for b in range(len(conds) + 1, 12):
        t = re.sub(r"<data/Contour1\.Bound%d\.[^>]*>\n?" % b, "", t)
    t = set_key(t, "NumRects", 1)
    for k, (xs, ys, dxr, dyr) in enumerate([(x_t, r_t, x_c - x_t, w)], 1):
        t = set_key(t, "Rect%d.Xstart" % k, xs)
        t = set_key(t, "Rect%d.Ystart" % k, ys)
        t = set_key(t, "Rect%d.DX" % k, dxr)
        t = set_key(t, "Rect%d.DY" % k, dyr)
        t = set_key(t, "Rect%d.Flow2D" % k, 3)
        t = set_key(t, "Rect%d.TurbulenceModel" % k, turbulence)
    t = set_key(t, "NumArea", 2)
    t = set_table(t, "Area1", [(3, ny // 2)])
    t = set_key(t, "Area1.Type", 1)
    t = set_key(t, "Area1.Flow2D", 2)
    t = set_key(t, "Area1.TurbulenceModel", turbulence)
    t = set_key(t, "Area1.MaterialID", 0)
    # the sting (outside the contour) is solid
    t = set_table(t, "Area2", [(nx - 3, 1)])
    t = set_key(t, "Area2.Type", 0)
    t = set_key(t, "Area2.Flow2D", 3)
    t = set_key(t, "Area2.TurbulenceModel", 0)
    t = set_key(t, "Area2.MaterialID", 0)
    return t


def scramjet(nx: int = 6000, ny: int = 400, *, nmax: int = 200, nout: int = 100, project: Optional[str] = None,
             exit_time: float = 1.0e-30, chemistry: int = 2, turbulence: int = 6,
             mechanism: Optional[str] = "h2_air_li2004", substeps: int = 1) -> str:
    """Axisymmetric Mach-8 H2/air scramjet channel: converging inlet, constant
    area combustor with a wall H2 injection slot, straight to the outlet.
    Finite-rate chemistry (ChemicalReactionsModel=2 with the built-in
    9-species / 21-step Li et al. H2/air mechanism, mechanism mode) and k-omega SST
    (TurbulenceModel=6, the default here) are new physics keys (not in the
    reference).  SST runs with point-implicit k/omega destruction and a
    free-stream eddy-viscosity ratio <= 10; tools/stability_probe.py shows the
    6000x400 start stable for 3000+ steps (profiles/sst_scramjet_probe.log).
    Domain 0.6 m x 0.04 m (dx = dy = 0.1 mm at 6000x400)."""
    t = remove_commented_directives(template_text("Wedge.dat"))
    project = project or "Scramjet_%dx%d" % (nx, ny)
    t = _rename(t, project)
    L, H = 0.6, 0.04
    t = set_key(t, "MaxX", nx)
    t = set_key(t, "MaxY", ny)
    t = set_key(t, "dx", L / nx)
    t = set_key(t, "dy", H / ny)
    t = set_key(t, "FlowType", 1)
    t = set_key(t, "ProblemType", 1)
    t = set_key(t, "TurbulenceModel", turbulence)
    t = set_key(t, "isTurbulenceReset", 1)
    t = set_key(t, "isAdiabaticWall", 1)
    t = set_key(t, "ChemicalReactionsModel", chemistry)
    t = set_key(t, "Nmax", nmax)
    t = set_key(t, "NOutStep", nout)
    t = set_key(t, "MonitorIndex", 5)
    t = set_key(t, "ExitMonitorValue", exit_time)
    # 1: Mach-8 air (inflow and initial fill), 2: sonic H2 jet (fuel),
    # 3: wall state at rest (300 K) for the no-slip walls
    t = _h2_air_species(t)
    t = set_key(t, "NumFlow2D", 3)
    t = set_key(t, "Flow2D-1.CompIndex", 4)      # air = O2 + N2 mixture
    t = set_key(t, "Flow2D-1.Y_fuel", 0.0)
    t = set_key(t, "Flow2D-1.Y_ox", AIR_Y_O2)
    t = set_key(t, "Flow2D-1.Y_cp", 0.0)
    t = set_key(t, "Flow2D-1.Mode", 2)
    t = set_key(t, "Flow2D-1.Mach", 8.0)
    t = set_key(t, "Flow2D-1.Angle", 0.0)
    t = set_key(t, "Flow2D-1.p", 1.2e3)
    t = set_key(t, "Flow2D-1.T", 226.5)
    t = set_key(t, "Flow2D-2.CompIndex", 0)
    t = set_key(t, "Flow2D-2.Mode", 2)
    t = set_key(t, "Flow2D-2.Mach", 1.0)
    t = set_key(t, "Flow2D-2.Angle", -90.0)
    t = set_key(t, "Flow2D-2.p", 2.0e4)
    t = set_key(t, "Flow2D-2.T", 250.0)
    t = set_key(t, "Flow2D-3.CompIndex", 4)
    t = set_key(t, "Flow2D-3.Y_fuel", 0.0)
    t = set_key(t, "Flow2D-3.Y_ox", AIR_Y_O2)
    t = set_key(t, "Flow2D-3.Y_cp", 0.0)
    t = set_key(t, "Flow2D-3.Mode", 0)
    t = set_key(t, "Flow2D-3.p", 1.2e3)
    t = set_key(t, "Flow2D-3.T", 300.0)
    for f in (1, 2, 3):
        t = set_key(t, "Flow2D-%d.U" % f, 0.0)
        t = set_key(t, "Flow2D-%d.V" % f, 0.0)
    # outermost grid nodes: contour points map to (int)(x / dx), (int)(y / dy - 1)
    L, H = (nx - 0.75) * (L / nx), (ny + 0.25) * (H / ny)
    Hc = 0.6 * H             # combustor radius
    x_r0, x_r1 = 0.05, 0.2   # inlet compression ramp (~6 deg)
    x_in, w_in = 0.22, 0.002  # injector slot on the outer wall
    x_c1 = 0.42               # combustor end / nozzle start
    ddx = 2.0 * L / nx
    # corners where a wall meets the in/outflow belong to the open boundary
    # (a no-slip node holding the free-stream energy would start at T0); the
    # combustor runs straight to the outlet (a free expansion would need a
    # far-field boundary along an inclined line)
    rows = [(0.0, 0.0), (L, 0.0), (L, Hc), (L - ddx, Hc), (x_in + w_in, Hc), (x_in, Hc),
            (x_r1, Hc), (x_r0, H), (ddx, H), (0.0, H)]
    t = set_table(t, "Contour1", rows)
    conds = [_AXIS, _OUTFLOW, _OUTFLOW, _WALL, _INFLOW, _WALL, _WALL, _WALL, _INFLOW, _INFLOW]
    # the junction node of the last wall and the inflow is both no-slip and
    # Dirichlet: give that short inflow piece the wall state (at rest, 300 K)
    flows = [1, 1, 3, 3, 2, 3, 3, 3, 3, 1]
    for b in range(1, len(conds) + 1):
        t = set_key(t, "Contour1.Bound%d.Cond" % b, conds[b - 1])
        t = set_key(t, "Contour1.Bound%d.Flow2D" % b, flows[b - 1])
        t = set_key(t, "Contour1.Bound%d.TurbulenceModel" % b, turbulence)
        t = set_key(t, "Contour1.Bound%d.isReset" % b, 0)
    t = set_key(t, "NumArea", 2)
    t = set_table(t, "Area1", [(3, 3)])
    t = set_key(t, "Area1.Type", 1)
    t = set_key(t, "Area1.Flow2D", 1)
    t = set_key(t, "Area1.TurbulenceModel", turbulence)
    t = set_key(t, "Area1.MaterialID", 0)
    t = set_table(t, "Area2", [(nx // 2, ny - 3)])
    t = set_key(t, "Area2.Type", 0)
    t = set_key(t, "Area2.Flow2D", 3)
    t = set_key(t, "Area2.TurbulenceModel", 0)
    t = set_key(t, "Area2.MaterialID", 0)
    if chemistry == 2 and mechanism:
        # detailed kinetics (9 species / 21 reversible steps by default); the
        # free stream (226 K) and the cold fuel jet do not react
        t = with_mechanism(t, mechanism, substeps=substeps, tmin=600.0)
    return t


# H2 / O2 / H2O / N2 in the fuel / oxidiser / product / inert slots, for the
# finite-rate chemistry decks (Wedge.dat's species data describe an H2/air
# Zeldovich model with air as the oxidiser and no usable heat of formation).
# Cp(T) from JANAF-level tables (J/kg/K), formation enthalpies per unit mass.
_H2_AIR = {
    "Fuel": (4124.2, 0.0, [(200, 13300), (300, 14310), (600, 14550), (1000, 14990), (1500, 16000),
                           (2000, 16980), (3000, 18080), (4000, 18800)]),
    "OX": (259.8, 0.0, [(200, 914), (300, 918), (600, 1003), (1000, 1090), (1500, 1145), (2000, 1181),
                        (3000, 1240), (4000, 1280)]),
    "cp": (461.5, -1.3435e7, [(200, 1850), (300, 1864), (600, 2003), (1000, 2288), (1500, 2575),
                              (2000, 2837), (3000, 3070), (4000, 3180)]),
    "air": (296.8, 0.0, [(200, 1039), (300, 1040), (600, 1075), (1000, 1167), (1500, 1244), (2000, 1284),
                         (3000, 1323), (4000, 1340)]),
}
AIR_Y_O2 = 0.2329   # air = O2 + N2 by mass


def _h2_air_species(t: str) -> str:
    for sp, (R, H, cp) in _H2_AIR.items():
        t = set_key(t, "R_%s" % sp, R)
        t = set_key(t, "H_%s" % sp, H)
        t = set_table(t, "Cp_%s" % sp, [(float(a), float(b)) for a, b in cp])
    return t


def reactor0d(nx: int = 8, ny: int = 8, *, T: float = 1500.0, p: float = 1.0e5, phi: float = 1.0,
              nmax: int = 200, nout: int = 100, project: Optional[str] = None) -> str:
    """Closed slip-wall box at rest with a premixed H2/air charge: every cell is
    a constant-volume reactor (finite-rate chemistry validation)."""
    t = remove_commented_directives(template_text("Wedge.dat"))
    project = project or "Reactor0D"
    t = _rename(t, project)
    t = _h2_air_species(t)
    dx = dy = 1.0e-3
    t = set_key(t, "MaxX", nx)
    t = set_key(t, "MaxY", ny)
    t = set_key(t, "dx", dx)
    t = set_key(t, "dy", dy)
    t = set_key(t, "ProblemType", 0)
    t = set_key(t, "FlowType", 0)
    t = set_key(t, "TurbulenceModel", 0)
    t = set_key(t, "ChemicalReactionsModel", 2)
    t = set_key(t, "Nmax", nmax)
    t = set_key(t, "NOutStep", nout)
    t = set_key(t, "MonitorIndex", 5)
    t = set_key(t, "ExitMonitorValue", 1.0e-30)
    # stoichiometric H2/air: Y_H2 / Y_O2 = 2 M_H2 / M_O2
    r = 2 * 2.016 / 31.999 * phi
    y_ox = AIR_Y_O2 / (1.0 + r * AIR_Y_O2)
    y_fu = r * y_ox
    t = set_key(t, "NumFlow2D", 2)
    for f in (1, 2):
        t = set_key(t, "Flow2D-%d.CompIndex" % f, 4)
        t = set_key(t, "Flow2D-%d.Mode" % f, 0)
        t = set_key(t, "Flow2D-%d.p" % f, p)
        t = set_key(t, "Flow2D-%d.T" % f, T)
        t = set_key(t, "Flow2D-%d.U" % f, 0.0)
        t = set_key(t, "Flow2D-%d.V" % f, 0.0)
        t = set_key(t, "Flow2D-%d.Y_fuel" % f, y_fu)
        t = set_key(t, "Flow2D-%d.Y_ox" % f, y_ox)
        t = set_key(t, "Flow2D-%d.Y_cp" % f, 0.0)
    xe, ye = (nx - 0.75) * dx, (ny + 0.25) * dy
    t = set_table(t, "Contour1", [(0.0, 0.0), (xe, 0.0), (xe, ye), (0.0, ye)])
    conds = ["NT_AX_2D", "NT_AY_2D", "NT_AX_2D", "NT_AY_2D"]
    for b in range(1, 5):
        t = set_key(t, "Contour1.Bound%d.Cond" % b, conds[b - 1])
        t = set_key(t, "Contour1.Bound%d.Flow2D" % b, 1)
        t = set_key(t, "Contour1.Bound%d.TurbulenceModel" % b, 0)
        t = set_key(t, "Contour1.Bound%d.isReset" % b, 0)
    for b in range(5, 12):
        t = re.sub(r"<data/Contour1\.Bound%d\.[^>]*>\n?" % b, "", t)
    t = set_key(t, "NumArea", 1)
    t = set_table(t, "Area1", [(nx // 2, ny // 2)])
    t = set_key(t, "Area1.Type", 1)
    t = set_key(t, "Area1.Flow2D", 1)
    t = set_key(t, "Area1.TurbulenceModel", 0)
    t = set_key(t, "Area1.MaterialID", 0)
    return t


def with_mechanism(text: str, mechanism: str = "h2_air_li2004", substeps: int = 1, tmin: float = 300.0) -> str:
    """Switch a deck to mechanism mode: detailed finite-rate kinetics
    (ChemicalReactionsModel = 2 + Mechanism, new keys; the reference's
    four species slots map to the mechanism species through its slot table)."""
    t = set_key(text, "ChemicalReactionsModel", 2)
    t = set_key(t, "Mechanism", mechanism)
    t = set_key(t, "ChemSubsteps", substeps)
    return set_key(t, "ChemTmin", tmin)


GENERATORS = {"wedge15": wedge15, "step": step, "triple_point": triple_point, "resonator": resonator,
              "scramjet": scramjet, "reactor0d": reactor0d, "flat_plate": flat_plate}
