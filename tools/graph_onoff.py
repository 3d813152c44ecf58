#!/usr/bin/env python3
"""Step graphs on vs off for a BASELINE config (no autotune for it, e.g. the
scramjet's mechanism step), interleaved, two reps:

  python tools/graph_onoff.py --config scramjet --warm 60 --steps 120"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="scramjet")
    ap.add_argument("--warm", type=int, default=60)
    ap.add_argument("--steps", type=int, default=120)
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    text = decks.GENERATORS[a.config](nmax=10 ** 9, nout=10 ** 8)
    for rep in range(2):
        for g in (True, False):
            s = hf.Simulation(text, "gpu")
            s.solver.use_graph = g
            s.step(a.warm)
            s.solver.synchronize()
            t0 = time.perf_counter()
            s.step(a.steps)
            s.solver.synchronize()
            print("%s rep %d graphs=%d: %.1f us/step" % (a.config, rep, g, (time.perf_counter() - t0) / a.steps * 1e6),
                  flush=True)
            del s


if __name__ == "__main__":
    main()
