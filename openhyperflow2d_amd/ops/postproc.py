"""libOutCFD equivalents on the host records of a Simulation (refreshed from
the device before every call).  Coordinates in metres like the deck keys
(x0_body, y0_body, dx_body, dy_body, XCut...)."""
from __future__ import annotations

import numpy as np


def _case(sim):
    sim.solver.download()
    return sim.case


def mass_flow_x(sim, x0: float, y0: float, dy: float) -> float:
    """Mass flow rate through the cut x = x0, y in [y0, y0+dy] (kg/s per m or
    per radian for axisymmetric flows) -- CalcMassFlowRateX2D."""
    return _case(sim).mass_flow_x(x0, y0, dy)


def force(sim, x0: float, y0: float, dx: float, dy: float):
    """Pressure + friction force on the body in the box (x0, y0, dx, dy)."""
    c = _case(sim)
    return c.x_force(x0, y0, dx, dy), c.y_force(x0, y0, dx, dy)


def x_force_ysym(sim, x0: float, l: float, d: float) -> float:
    """x force on the wall cells of x in [x0, x0+l] below y = d (CalcXForceYSym2D)."""
    return _case(sim).x_force_ysym(x0, l, d)


def mid_section_area(sim, x0, y0, dx, dy) -> float:
    """Frontal area of the body rows inside the box (GetFmid)."""
    return _case(sim).mid_section_area(x0, y0, dx, dy)


def smooth(a: np.ndarray, axis: int) -> np.ndarray:
    """SmoothX (axis=0) / SmoothY (axis=1) of an x-major (nx, ny) field: a cell
    whose two neighbours along the axis are > 0 becomes their mean, in place in
    the reference's sweep order.  Returns a smoothed copy."""
    from .. import native
    out = np.ascontiguousarray(a, dtype=np.float64).copy()
    native().smooth(out, int(axis))
    return out


def cx(sim, x0, y0, dx, dy, flow: int = 1) -> float:
    """Drag coefficient against Flow2D-<flow> (Calc_Cx_2D)."""
    return _case(sim).cx(x0, y0, dx, dy, flow)


def cy(sim, x0, y0, dx, dy, flow: int = 1) -> float:
    return _case(sim).cy(x0, y0, dx, dy, flow)


def cd(sim, x0, y0, dy, flow: int = 1) -> float:
    """Discharge coefficient of a cut (Calc_Cd)."""
    return _case(sim).cd(x0, y0, dy, flow)


def cv(sim, x0, y0, dy, p_amb: float, flow: int = 1) -> float:
    """Velocity coefficient of a cut (Calc_Cv)."""
    return _case(sim).cv(x0, y0, dy, p_amb, flow)


def average_pressure(sim, x0: float, l: float, d: float) -> float:
    return _case(sim).average_pressure(x0, l, d)


def average_temperature(sim, x0: float, l: float, d: float, mid_enthalpy: bool = False) -> float:
    return _case(sim).average_temperature(x0, l, d, int(mid_enthalpy))


def derived_field(sim, name: str) -> np.ndarray:
    """'p_total' (p*), 'T_total' (T*) or 'schlieren' as the reference outputs them."""
    return np.asarray(_case(sim).derived_field(name))


def mach(sim) -> np.ndarray:
    return sim.field("mach")


def vorticity(sim) -> np.ndarray:
    """dV/dx - dU/dy by central differences on the x-major (nx, ny) grid."""
    U, V = sim.field("U"), sim.field("V")
    dx, dy = sim.case.dx, sim.case.dy
    return np.gradient(V, dx, axis=0) - np.gradient(U, dy, axis=1)
