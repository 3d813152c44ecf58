"""Field-level operators on a simulation's host records.

The solver kernels themselves live in csrc/hip (device) and csrc/core
(host); this package exposes the reference's post-processing library
(libOutCFD/out_cfd_param.cpp: integral forces and coefficients, mass flow,
total-state and schlieren fields) and derived fields for Python users.
"""
from . import chemistry
from .postproc import (average_pressure, average_temperature, cd, cv, cx, cy, derived_field, force,
                       mach, mass_flow_x, mid_section_area, smooth, vorticity, x_force_ysym)

__all__ = ["chemistry", "average_pressure", "average_temperature", "cd", "cv", "cx", "cy", "derived_field", "force", "mach",
           "mass_flow_x", "mid_section_area", "smooth", "vorticity", "x_force_ysym"]
