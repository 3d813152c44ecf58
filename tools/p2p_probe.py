"""Time the xGMI mailbox transport with N in-process strip ranks on one GPU.

  python tools/p2p_probe.py --ranks 2 --steps 600
Each rank runs its strip on its own stream/host thread; every step is the
lean tile kernel + one hf2d_p2p_xchg kernel (captured in step graphs).  On a
single device the ranks share the CUs, so us/step is NOT the multi-GPU step
time -- use rocprofv3 --kernel-trace --stats on this to read the exchange
kernel's own duration.
"""
import argparse
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--nx", type=int, default=2000)
    ap.add_argument("--ny", type=int, default=200)
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--warmup", type=int, default=60)
    ap.add_argument("--nofuse", action="store_true", help="separate exchange kernel instead of the fused tile kernel")
    ap.add_argument("--tail", type=int, default=0,
                    help="2 ranks, the last one owning only this many columns: its kernel barely competes for "
                         "the shared GPU, so us/step ~ rank 0's kernel + its exchange overhead")
    ap.add_argument("--autotune", action="store_true", help="DeviceSolver.autotune() on every strip first")
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks
    from openhyperflow2d_amd.parallel.strips import balanced_columns

    nat = hf.native()
    text = decks.wedge15(a.nx, a.ny, nmax=10 ** 9, nout=10 ** 8)
    cases = [nat.Case.from_deck(text, ".", False) for _ in range(a.ranks)]
    parts = balanced_columns(np.asarray(cases[0].field("solid")), a.ranks)
    if a.tail:
        parts = [(0, a.nx - a.tail), (a.nx - a.tail, a.nx)]
    group = nat.LocalGroup(a.ranks)
    solvers = []
    for r, (lo, hi) in enumerate(parts):
        s = nat.DeviceSolver(cases[r], 0, lo, hi)
        if a.autotune:
            # before the rank joins the group, as in a multi-GPU run
            # (DistributedSimulation tunes each strip before wiring the transport)
            print("rank %d autotune: %s" % (r, s.autotune().strip().replace("; ", "\n    ")), flush=True)
        s.init_local(group, r)
        solvers.append(s)
    descs = [s.p2p_export(r, a.ranks) for r, s in enumerate(solvers)]
    for s in solvers:
        s.p2p_import(descs)
        s.p2p_fuse = not a.nofuse

    def run_all(n):
        th = [threading.Thread(target=s.run_steps, args=(n, False)) for s in solvers]
        for t in th:
            t.start()
        for t in th:
            t.join()

    run_all(a.warmup)
    t0 = time.perf_counter()
    run_all(a.steps)
    for s in solvers:
        s.synchronize()
    dt = time.perf_counter() - t0
    print("ranks %d  %.2f us/step  graphs %s  dt %s" % (a.ranks, dt / a.steps * 1e6,
                                                        [s.graph_launches for s in solvers],
                                                        solvers[0].summary()["dt"]), flush=True)


if __name__ == "__main__":
    main()
