"""Interleaved A/B timing of solver variants inside one process (same GPU,
same clocks), e.g.  python tools/ab_bench.py --variants plain,noplain"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=2000)
    ap.add_argument("--ny", type=int, default=200)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--variants", default="tile,nosg,plain,flat")
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    text = decks.wedge15(a.nx, a.ny, nmax=10 ** 9, nout=10 ** 8)
    sims = {}
    for v in a.variants.split(","):
        s = hf.Simulation(text, "gpu")
        for part in v.split("+")[1:]:
            if part.startswith("tj"):
                s.solver.lean_tj = int(part[2:])
        v0 = v.split("+")[0]
        if v0 == "plain":
            s.solver.lean_plain = True
        elif v0 == "nograph":
            s.solver.use_graph = False
        elif v0 == "nosg":
            s.solver.lean_sg = False
        elif v0.startswith("cpt"):
            s.solver.lean_cpt = int(v0[3:])
        elif v0.startswith("occ"):
            s.solver.lean_occ = int(v0[3:])
        elif v0.startswith("tj"):
            s.solver.lean_tj = int(v0[2:])
        elif v0 == "flat":
            s.solver.lean_tile = False
        elif v0 == "split":
            s.solver.lean = False
            s.solver.fused = False
        elif v0 == "fused":
            s.solver.lean = False
        s.step(20)
        sims[v] = s
    res = {v: [] for v in sims}
    for r in range(a.rounds):
        for v, s in sims.items():
            s.solver.synchronize()
            t0 = time.perf_counter()
            s.step(a.steps)
            s.solver.synchronize()
            res[v].append((time.perf_counter() - t0) / a.steps * 1e6)
    cells = a.nx * a.ny
    for v, ts in res.items():
        best = min(ts)
        print("%-10s us/step best %.2f  all %s  -> %.0f Mcells*it/s" % (v, best, " ".join("%.2f" % t for t in ts),
                                                                      cells / best))


if __name__ == "__main__":
    main()
