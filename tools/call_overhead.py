#!/usr/bin/env python3
"""Fixed cost of one Simulation.step(n) call on the headline grid (the
driver times 20 steps in one call, so a per-call cost weighs 1/20 per step).

  python tools/call_overhead.py [--config wedge15] [--reps 40]

Prints the median wall time of step(n) for several n and the least-squares
a + b n fit (a = per-call cost, b = steady per-step time), plus step(0)
(the closing scalar read-back alone) and an idle synchronize()."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--nx", type=int, default=2000)
    ap.add_argument("--ny", type=int, default=200)
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    sim = hf.Simulation(decks.wedge15(a.nx, a.ny, nmax=10 ** 9, nout=10 ** 8), "gpu")
    sim.step(300)
    sim.solver.synchronize()

    def timed(fn):
        t = []
        for _ in range(a.reps):
            sim.solver.synchronize()
            t0 = time.perf_counter()
            fn()
            sim.solver.synchronize()
            t.append(time.perf_counter() - t0)
        return statistics.median(t) * 1e6

    out = {"sync_idle_us": timed(lambda: None), "step0_us": timed(lambda: sim.step(0))}
    ns = [1, 2, 5, 10, 20, 50, 100]
    ts = [timed(lambda n=n: sim.step(n)) for n in ns]
    out["step_n_us"] = dict(zip(ns, [round(x, 2) for x in ts]))
    mx, my = sum(ns) / len(ns), sum(ts) / len(ts)
    b = sum((x - mx) * (y - my) for x, y in zip(ns, ts)) / sum((x - mx) ** 2 for x in ns)
    out["fit_call_us"] = round(my - b * mx, 2)
    out["fit_step_us"] = round(b, 3)
    out["per_step_at_20_us"] = round(ts[ns.index(20)] / 20, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
