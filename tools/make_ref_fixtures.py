"""Record golden hashes of the reference solver's outputs for small decks.

Run where a serial build of the reference exists (built from its sources in a
scratch directory with -O2 -ffp-contract=off):

  python tools/make_ref_fixtures.py --ref /tmp/refexact/bin/OpenHyperFLOW2D-1.03

For every case the deck actually run is stored as tests/fixtures/ref/<case>/deck.dat
and the sha256 of every output file (.plt, .hf2d) in sha256.json.  The tests
(tests/test_reference_golden.py) run our reference-order backend on the same
deck and require byte-identical outputs.
"""
import argparse
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from openhyperflow2d_amd.models import decks  # noqa: E402

FIX = os.path.join(ROOT, "tests", "fixtures")


def _fixture_deck(name):
    with open(os.path.join(FIX, "decks", name), errors="replace") as f:
        return f.read()


def _finite(text, nmax, nout=None):
    """Run exactly one outer cycle of nmax steps (exit monitor forced)."""
    t = decks.set_key(text, "Nmax", nmax)
    t = decks.set_key(t, "NOutStep", nout or max(1, nmax // 4))
    t = decks.set_key(t, "MonitorIndex", 5)
    t = decks.set_key(t, "ExitMonitorValue", 1e-30)
    return t


def _wedge(turb=0, tem=None, ns=None, ft=0, nx=120, ny=40, steps=30, **kw):
    """Small Wedge15 variant: turbulence model / extension, flow type, extra keys."""
    ns = bool(turb) if ns is None else ns
    t = decks.wedge15(nx, ny, navier_stokes=ns, turbulence=turb, nmax=steps, nout=10)
    t = decks.set_key(t, "FlowType", ft)
    if tem is not None:
        t = decks.set_key(t, "TurbExtModel", tem)
    for k, v in kw.items():
        t = decks.set_key(t, k.replace("__", ".").replace("Point_", "Point-"), v)
    return _finite(t, steps, 10)


def _with_objects(text, **kw):
    for k, v in kw.items():
        text = decks.set_key(text, k.replace("__", "."), v)
    return text


def cases():
    return {
        "wedge15_200x40_euler": _finite(decks.wedge15(200, 40, nmax=101, nout=25), 101, 25),
        "oblique_shock": _finite(_fixture_deck("ObliqueShock.dat"), 40),
        "step_euler": _finite(_fixture_deck("Step.dat"), 20),
        "wedge_keps_wallheat": _finite(_fixture_deck("Wedge.dat"), 30),
        "wedge15_200x60_ns_keps": _finite(decks.wedge15(200, 60, navier_stokes=True, turbulence=4,
                                                        nmax=30, nout=10), 30, 10),
        # round 2: the rest of the reference's feature surface
        "axisym_euler": _wedge(ft=1),
        "axisym_keps": _wedge(turb=4, ft=1),
        # the reference's SA diverges on this deck at iteration 3: the full SA path
        # runs until then and the error snapshot must match as well
        "spalart_allmaras_blowup": _wedge(turb=3, tem=10),
        "spalart_allmaras_start": _wedge(turb=3, tem=10, TurbStartIter=100),
        "prandtl": _wedge(turb=2, tem=0),
        "van_driest": _wedge(turb=2, tem=1),
        "escudier": _wedge(turb=2, tem=2, delta_bl=0.004),
        "klebanoff": _wedge(turb=2, tem=3, delta_bl=0.004),
        "smagorinsky": _wedge(turb=5),
        "keps_chien": _wedge(turb=4, tem=5),
        "keps_jones_launder": _wedge(turb=4, tem=6),
        "keps_launder_sharma": _wedge(turb=4, tem=7),
        "keps_rng": _wedge(turb=4, tem=8),
        "bff_linear": _wedge(BFF=0),
        "bff_square_relax": _wedge(BFF=3),
        "bff_sqrt_relax": _wedge(BFF=5),
        "zeldovich_reacting": _finite(decks.set_key(decks.reactor0d(12, 12, T=1500.0, nmax=20, nout=5),
                                                    "ChemicalReactionsModel", 1), 20, 5),
        "gas_source": _wedge(NumSrc=1, Src1__GasSrcSX=20, Src1__GasSrcSY=10, Src1__GasSrcEX=20,
                             Src1__GasSrcEY=20, Src1__GasSrcIndex=3, Src1__Msrc=0.5, Src1__Tsrc=600.0,
                             Src1__Tf_src=1000.0, Src1__StartIter=0),
        "solid_rect": _wedge(NumRects=1, Rect1__Xstart=0.03, Rect1__Ystart=0.015, Rect1__DX=0.012, Rect1__DY=0.008,
                             Rect1__Flow2D=1, Rect1__TurbulenceModel=0),
        "circle": _wedge(NumCircles=1, Circle1__Xstart=0.04, Circle1__Ystart=0.02, Circle1__X0=0.047,
                         Circle1__Y0=0.02, Circle1__MaterialID=1, Circle1__TurbulenceModel=0, Circle1__Flow2D=1),
        "naca_airfoil": _wedge(NumAirfoils=1, Airfoil1__Xstart=0.025, Airfoil1__Ystart=0.022, Airfoil1__Type=0,
                               Airfoil1__pp=0.4, Airfoil1__mm=0.02, Airfoil1__thick=0.12, Airfoil1__scale=0.04,
                               Airfoil1__attack_angle=5.0, Airfoil1__Flow2D=1, Airfoil1__TurbulenceModel=0,
                               # the reference reads Cx_Flow_Index for the airfoil Re only when is_Cx_calc = 1
                               is_Cx_calc=1, x_body=0.02, y_body=0.01, dx_body=0.05, dy_body=0.025, Cx_Flow_Index=1),
        "monitors_heatflux_cx": _wedge(turb=4, NumMonitorPoints=2, Point_1__X=0.05, Point_1__Y=0.02,
                                       Point_2__X=0.1, Point_2__Y=0.01, isOutHeatFluxX=1, Cp_Flow_Index=1,
                                       y_max=20, y_min=0, isOutHeatFluxY=1, is_Cx_calc=1, x_body=0.07,
                                       y_body=0.0, dx_body=0.05, dy_body=0.012, Cx_Flow_Index=1),
        "restart_from_hf2d": (_wedge(steps=20), 2),
        # round 3: the last unpinned paths
        # TsAGI table airfoil (hyper_flow_airfoil.cpp:99-150): the contour
        # comes from the UpperSurface / LowerSurface tables of a second file
        "tsagi_airfoil": (_wedge(NumAirfoils=1, Airfoil1__Xstart=0.03, Airfoil1__Ystart=0.022, Airfoil1__Type=1,
                                 Airfoil1__InputData="airfoil_tsagi.dat", Airfoil1__scale=0.035,
                                 Airfoil1__attack_angle=4.0, Airfoil1__Flow2D=1, Airfoil1__TurbulenceModel=0,
                                 # (the reference prints the airfoil Re from Cx_Flow_Index, so the Cx block is on)
                                 is_Cx_calc=1, x_body=0.025, y_body=0.01, dx_body=0.05, dy_body=0.025,
                                 Cx_Flow_Index=1), 1,
                          {"airfoil_tsagi.dat": _tsagi_table()}),
        # wall-law nodes (NT_WALL_LAW_2D, hyper_flow_node.hpp:447 ff): the ramp
        # and the plate ahead of it as wall-law boundaries of the turbulent
        # wedge.  The reference's wall-law projection diverges on this deck at
        # iteration 3 (next to the inflow corner): three full steps of the
        # path and the error snapshot are pinned
        "wall_law": decks.set_key(decks.set_key(_wedge(turb=4), "Contour1.Bound3.Cond",
                                                "NT_WALL_LAW_2D, TCT_eps_Cmk2kXn_WALL_2D"),
                                  "Contour1.Bound4.Cond", "NT_WALL_LAW_2D, TCT_eps_Cmk2kXn_WALL_2D"),
        # the Integral turbulence model (TurbulenceModel = 1: Re_local only,
        # hyper_flow_node.hpp:921-924)
        "integral_model": _wedge(turb=1),
        # round 4: forces on an airfoil.  The reference's airfoil only exists
        # at attack_angle = 0 (RotateBoundContour2D compares node coordinates
        # against an unset Bound2D::dx and fails), and Calc_Cx_2D /
        # CalcXForce2D (out_cfd_param.cpp:256-496) count only no-slip /
        # wall-law nodes, which an N-S deck gives the airfoil contour: a
        # cambered NACA section in the turbulent wedge with non-zero Cx, Cy,
        # Fx, Fy after 30 steps
        "naca_airfoil_ns": _wedge(turb=4, NumAirfoils=1, Airfoil1__Xstart=0.02, Airfoil1__Ystart=0.026,
                                  Airfoil1__Type=0, Airfoil1__pp=0.4, Airfoil1__mm=0.2, Airfoil1__thick=0.12,
                                  Airfoil1__scale=0.04, Airfoil1__attack_angle=0.0, Airfoil1__Flow2D=1,
                                  Airfoil1__TurbulenceModel=0, is_Cx_calc=1, x_body=0.015, y_body=0.015,
                                  dx_body=0.05, dy_body=0.02, Cx_Flow_Index=1),
        # wall-law nodes that stay bounded: the no-slip plate of the flat-plate
        # deck (k-eps, M = 0.8) as NT_WALL_LAW_2D, 60 steps
        # (hyper_flow_node.hpp:447 ff; the velocity projection onto BGX/BGY)
        "wall_law_plate": _finite(decks.set_key(decks.flat_plate(120, 40, mach=0.8, p=1.0e5, turbulence=4),
                                                "Contour1.Bound3.Cond", "NT_WALL_LAW_2D, TCT_eps_Cmk2kXn_WALL_2D"),
                                  60, 20),
    }


def _tsagi_table():
    """A 12 % thick cambered section as UpperSurface / LowerSurface tables
    (x, y in chord units), the external-deck format of the TsAGI airfoil."""
    import math

    xs = [0.0, 0.0125, 0.025, 0.05, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9, 1.0]

    def half(x):   # NACA-00xx thickness with a closed trailing edge
        return 0.6 * (0.2969 * math.sqrt(x) - 0.126 * x - 0.3516 * x * x + 0.2843 * x ** 3 - 0.1036 * x ** 4)

    def camber(x):
        return 0.02 * x * (1.0 - x) * 4.0

    up = ["%.6f %.6f" % (x, camber(x) + half(x)) for x in xs]
    lo = ["%.6f %.6f" % (x, camber(x) - half(x)) for x in xs]
    return ("<start/Airfoil>\n<table=UpperSurface/%d>\n%s\n<endtable>\n<table=LowerSurface/%d>\n%s\n<endtable>\n"
            "<end/Airfoil>\n" % (len(up), "\n".join(up), len(lo), "\n".join(lo)))


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/tmp/refexact/bin/OpenHyperFLOW2D-1.03")
    ap.add_argument("--only", nargs="*")
    a = ap.parse_args()
    for name, spec in cases().items():
        if a.only and name not in a.only:
            continue
        text, runs, extra = (spec + ({},))[:3] if isinstance(spec, tuple) else (spec, 1, {})
        d = os.path.join(FIX, "ref", name)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "deck.dat"), "w") as f:
            f.write(text)
        for fn, body in extra.items():   # files the deck names (e.g. an airfoil table deck)
            with open(os.path.join(d, fn), "w") as f:
                f.write(body)
        with tempfile.TemporaryDirectory() as tmp:
            for fn in ["deck.dat"] + list(extra):
                shutil.copy(os.path.join(d, fn), tmp)
            # runs > 1: the later runs resume from the .hf2d the previous one wrote
            for _ in range(runs):
                r = subprocess.run([a.ref, "deck.dat"], cwd=tmp, capture_output=True, text=True, errors="replace",
                                   timeout=1800)
            outs = sorted(f for f in os.listdir(tmp) if f.endswith((".plt", ".hf2d")) and f not in extra)
            rec = {f: sha256(os.path.join(tmp, f)) for f in outs}
            rec["_returncode"] = r.returncode
            rec["_runs"] = runs
            # integral-quantity lines of the log (XCut mass flow, Cx/Cy/Fx/Fy)
            rec["_log_lines"] = [ln.strip() for ln in r.stdout.splitlines() if ln.strip().startswith(("Cx", "Cut("))]
            for f in outs:
                if f.endswith(".hf2d"):
                    import numpy as np

                    arr = np.fromfile(os.path.join(tmp, f), dtype=np.float64).copy()
                    if np.isnan(arr).any():   # NaN-sign-insensitive hash (see test_reference_golden.py)
                        arr[np.isnan(arr)] = np.nan
                        rec["_hf2d_nan_canonical"] = hashlib.sha256(arr.tobytes()).hexdigest()
        with open(os.path.join(d, "sha256.json"), "w") as f:
            json.dump(rec, f, indent=1, sort_keys=True)
        print(name, r.returncode, outs)


if __name__ == "__main__":
    main()
