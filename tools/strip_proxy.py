#!/usr/bin/env python3
"""One-GPU proxy of an N-GPU strip run: N DeviceSolvers (virtual ranks, one
host thread each) on ONE MI355X, halos and dt through the xGMI mailbox
transport (the same device kernels an N-GPU run launches), step graphs on.

  python tools/strip_proxy.py --config resonator --ranks 4 --steps 60
  rocprofv3 --kernel-trace --stats -d DIR -- python3 tools/strip_proxy.py ...

Prints one JSON line: wall time per step of the whole group and the config.
Run under rocprofv3 the kernel table splits each step into the strips'
compute kernels and the exchange kernels (hf2d_p2p_xchg / pack / unpack):
on N GPUs every rank runs one strip's kernels, so the exchange share of a
rank's step is (exchange kernel time) / (all kernel time) of the proxy.
"""
import argparse
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

SHAPES = {"resonator": (2000, 200), "scramjet": (6000, 400), "step": (1200, 400), "wedge15": (2000, 200)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="resonator", choices=sorted(SHAPES))
    ap.add_argument("--ranks", type=int, default=4)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=24)
    ap.add_argument("--nx", type=int, default=0)
    ap.add_argument("--ny", type=int, default=0)
    ap.add_argument("--nofuse", action="store_true", help="separate exchange kernel (hf2d_p2p_xchg) after each step")
    args = ap.parse_args()

    import numpy as np
    import torch  # noqa: F401

    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks
    from openhyperflow2d_amd.parallel.strips import balanced_columns

    nx, ny = SHAPES[args.config]
    nx, ny = args.nx or nx, args.ny or ny
    gen = decks.GENERATORS.get(args.config) if args.config != "wedge15" else decks.wedge15
    text = gen(nx, ny, nmax=10 ** 9, nout=10 ** 8)
    nat = hf.native()
    n = args.ranks
    cases = [nat.Case.from_deck(text, ".", False) for _ in range(n)]
    parts = balanced_columns(np.asarray(cases[0].field("solid")), n)
    group = nat.LocalGroup(n)
    solvers = []
    for r, (a, b) in enumerate(parts):
        s = nat.DeviceSolver(cases[r], 0, a, b)
        s.init_local(group, r)
        solvers.append(s)
    if n > 1:
        descs = [s.p2p_export(r, n) for r, s in enumerate(solvers)]
        for s in solvers:
            s.p2p_import(descs)
            # the exchange fused into the tile kernels, as DistributedSimulation
            # sets it (HF2D_P2P_FUSE=0: separate exchange kernel)
            s.p2p_fuse = not args.nofuse
        blobs = [None] * n

        def probe(r):
            blobs[r] = solvers[r].p2p_probe()

        th = [threading.Thread(target=probe, args=(r,), daemon=True) for r in range(n)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        ok, why = nat.DeviceSolver.p2p_probe_ok(blobs, 0)
        if not ok:
            raise SystemExit("p2p probe failed: %s" % why)
    errors = []

    def run(s, k):
        try:
            s.run_steps(k, False)
        except Exception as e:  # pragma: no cover
            errors.append(e)

    def steps(k):
        th = [threading.Thread(target=run, args=(s, k), daemon=True) for s in solvers]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=600)
        if errors or any(t.is_alive() for t in th):
            raise SystemExit("virtual-rank step failed: %s" % errors)

    steps(args.warmup)
    for s in solvers:
        s.synchronize()
    t0 = time.perf_counter()
    steps(args.steps)
    for s in solvers:
        s.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({
        "config": args.config, "grid": "%dx%d" % (nx, ny), "ranks": n, "steps": args.steps,
        "ms_per_step_group": round(dt / args.steps * 1e3, 4),
        "strips": [[int(a), int(b)] for a, b in parts],
        "lean_ns_steps": [int(s.lns_steps) for s in solvers], "lean_mech_steps": [int(s.lnm_steps) for s in solvers],
        "graph_launches": [int(s.graph_launches) for s in solvers],
        "fused_exchange": not args.nofuse, "lean_ns_fx_steps": [int(s.lns_fx_steps) for s in solvers],
        "summary_dt": solvers[0].summary()["dt"],
    }), flush=True)


if __name__ == "__main__":
    main()
