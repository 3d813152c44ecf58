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
            t = set_table(t, name, [(int(x / sx), int(y / sy)) for x, y in rows])
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


GENERATORS = {"wedge15": wedge15, "step": step}
