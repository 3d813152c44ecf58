"""In-process virtual ranks vs HIP hardware queues (diagnostic for the round-5
4-rank mailbox probe timeout).

N DeviceSolvers in ONE process each create their own HIP stream; HIP maps a
process's streams onto at most GPU_MAX_HW_QUEUES hardware queues (default 4)
and, past that, makes two streams share one queue.  A queue runs its packets in
order, so when rank a's exchange kernel (whose last workgroup spins until every
peer has published) sits in front of rank b's kernel on a shared queue, b never
starts and a times out.  This tool runs the start-up probe (one fused mailbox
exchange of the full state) with N in-process ranks and reports the verdict
and wall time; run it under different GPU_MAX_HW_QUEUES values:

  GPU_MAX_HW_QUEUES=4  python tools/hwq_probe.py --ranks 4
  GPU_MAX_HW_QUEUES=16 python tools/hwq_probe.py --ranks 8
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=4)
    ap.add_argument("--nx", type=int, default=300)
    ap.add_argument("--ny", type=int, default=60)
    ap.add_argument("--unchecked", action="store_true", help="skip the native queue-count guard")
    a = ap.parse_args()
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks
    from openhyperflow2d_amd.parallel.strips import balanced_columns

    nat = hf.native()
    text = decks.wedge15(a.nx, a.ny, nmax=10 ** 6, nout=10 ** 5)
    n = a.ranks
    cases = [nat.Case.from_deck(text, ".", False) for _ in range(n)]
    parts = balanced_columns(np.asarray(cases[0].field("solid")), n)
    group = nat.LocalGroup(n)
    solvers = []
    for r, (lo, hi) in enumerate(parts):
        s = nat.DeviceSolver(cases[r], 0, lo, hi)
        s.init_local(group, r)
        solvers.append(s)
    rec = {"ranks": n, "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", "(unset)")}
    try:
        descs = [s.p2p_export(r, n) for r, s in enumerate(solvers)]
        for s in solvers:
            if a.unchecked and hasattr(s, "p2p_queue_check"):
                s.p2p_queue_check = False
            s.p2p_import(descs)
            s.p2p_fuse = True
    except Exception as e:
        rec["refused"] = str(e)
        print(json.dumps(rec), flush=True)
        return 0
    blobs = [None] * n

    def probe(r):
        blobs[r] = solvers[r].p2p_probe()

    t0 = time.time()
    th = [threading.Thread(target=probe, args=(r,), daemon=True) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    rec["probe_s"] = round(time.time() - t0, 3)
    if not all(b is not None for b in blobs):
        rec["verdict"] = "hung"
        print(json.dumps(rec), flush=True)
        return 1
    ok, why = nat.DeviceSolver.p2p_probe_ok(blobs, 0)
    rec["ok"], rec["why"] = bool(ok), why
    print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
