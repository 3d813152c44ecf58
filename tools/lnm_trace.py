"""Phase timeline of one lean mechanism step (hip/lean_mech.hpp) from the
in-kernel trace (HF2D_LNM_TRACE=1: s_memrealtime at 100 MHz, per workgroup).

  python tools/lnm_trace.py [--nx 6000 --ny 400 --ti 16 --steps 20]

Prints, per phase, the median / p90 duration over workgroups in microseconds
(wave 0: ring fill, own fill, barrier wait, flow predictor, species
predictor, state E + dt; the last wavefront: own fill), the dispatch ramp and
the kernel span, and workgroups per CU.
"""
import argparse
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=6000)
    ap.add_argument("--ny", type=int, default=400)
    ap.add_argument("--ti", type=int, default=16)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    os.environ["HF2D_LNM_TRACE"] = "1"
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    sim = hf.Simulation(decks.scramjet(a.nx, a.ny, nmax=10 ** 9, nout=10 ** 8), "gpu")
    sim.solver.use_graph = False
    sim.solver.lnm_ti = a.ti
    sim.step(a.steps)
    assert sim.solver.lnm_steps > 0, sim.solver.lnm_why
    t = np.array(sim.solver.lnm_trace_fetch(), dtype=np.uint64).reshape(-1, 12).astype(np.int64)
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    us = lambda x: x / 100.0   # 100 MHz ticks -> microseconds
    ph = {
        "ring fill (wave 0)": t[:, 1] - t[:, 0],
        "own fill (wave 0)": t[:, 2] - t[:, 1],
        "own fill (last wave)": t[:, 9] - t[:, 0],
        "barrier wait (wave 0)": t[:, 3] - t[:, 2],
        "flow predictor": t[:, 4] - t[:, 3],
        "species predictor": t[:, 5] - t[:, 4],
        "state E + list": t[:, 6] - t[:, 5],
        "reduction + dt": t[:, 7] - t[:, 6],
        "workgroup total": t[:, 7] - t[:, 0],
    }
    print("lean mechanism step %dx%d, tile %dx16: %d workgroups" % (a.nx, a.ny, a.ti, len(t)))
    print("%-24s %9s %9s %9s" % ("phase", "median us", "p90 us", "mean us"))
    for k, v in ph.items():
        print("%-24s %9.2f %9.2f %9.2f" % (k, us(np.median(v)), us(np.percentile(v, 90)), us(v.mean())))
    print("dispatch ramp (last start) %.1f us, kernel span %.1f us" % (us(t[:, 0].max() - t0), us(t[:, 7].max() - t0)))
    cu = collections.Counter((int(x) >> 8) & 0xFFF for x in t[:, 8])
    print("workgroups per (CU, SE) id: mean %.1f max %d over %d ids" % (np.mean(list(cu.values())), max(cu.values()),
                                                                       len(cu)))


if __name__ == "__main__":
    main()
