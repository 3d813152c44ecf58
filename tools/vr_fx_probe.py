"""Fused lean N-S strips as in-process virtual ranks, chunk by chunk with
progress lines (diagnostic for a stalled multi-rank case): prints each
chunk's wall time, the solvers' fused / prologue step counters and, at the
end, whether the fields equal one GPU.

  GPU_MAX_HW_QUEUES=16 python tools/vr_fx_probe.py --deck resonator --ranks 8
"""
import argparse
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--deck", default="resonator")
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--chunks", default="4r,17,5r,14")
    ap.add_argument("--graphs", type=int, default=1)
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks
    from openhyperflow2d_amd.parallel.strips import balanced_columns

    nat = hf.native()
    if a.deck == "resonator":
        text = decks.resonator(300, 40, nmax=10 ** 6, nout=10 ** 5)
    elif a.deck == "step":
        text = decks.step(240, 80, nmax=10 ** 6, nout=10 ** 5)
    else:
        text = decks.scramjet(300, 48, nmax=10 ** 6, nout=10 ** 5)
    n = a.ranks
    cases = [nat.Case.from_deck(text, ".", False) for _ in range(n)]
    parts = balanced_columns(np.asarray(cases[0].field("solid")), n)
    group = nat.LocalGroup(n)
    solvers = []
    for r, (lo, hi) in enumerate(parts):
        s = nat.DeviceSolver(cases[r], 0, lo, hi)
        s.init_local(group, r)
        s.use_graph = bool(a.graphs)
        solvers.append(s)
    descs = [s.p2p_export(r, n) for r, s in enumerate(solvers)]
    for s in solvers:
        s.p2p_import(descs)
        s.p2p_fuse = True
    blobs = [None] * n
    th = [threading.Thread(target=lambda r=r: blobs.__setitem__(r, solvers[r].p2p_probe()), daemon=True)
          for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    print("probe", nat.DeviceSolver.p2p_probe_ok(blobs, 0), flush=True)
    sched = [(int(c.rstrip("r")), c.endswith("r")) for c in a.chunks.split(",")]
    errors = []
    for k, (steps, res) in enumerate(sched):
        t0 = time.time()

        def run(s):
            try:
                s.run_steps(steps, res)
            except Exception as e:   # reported below
                errors.append(repr(e))

        th = [threading.Thread(target=run, args=(s,), daemon=True) for s in solvers]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=60)
        alive = sum(t.is_alive() for t in th)
        print("chunk %d (%d steps, res=%d): %.3f s, alive %d, errors %s, fx %s, prologue %s" % (
            k, steps, res, time.time() - t0, alive, errors[:2], [s.lns_fx_steps for s in solvers],
            [s.lns_prologue_steps for s in solvers]), flush=True)
        if alive or errors:
            return 1
    ref = hf.Simulation(text, "gpu")
    for steps, res in sched:
        ref.step(steps, residual=res)
    ok = solvers[0].summary()["dt"] == ref.summary()["dt"]
    for f in ["rho", "U", "V", "p", "T"]:
        full = None
        for r, (lo, hi) in enumerate(parts):
            solvers[r].download()
            fr = np.asarray(cases[r].field(f))
            full = np.zeros_like(fr) if full is None else full
            full[lo:hi] = fr[lo:hi]
        ok = ok and np.array_equal(full, ref.field(f))
    print("EQUAL" if ok else "DIFFER", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
