#!/usr/bin/env python3
"""The virtual-rank strip driver (N DeviceSolvers on one GPU, LocalGroup
transport, generic path) against one GPU: which output files differ and where
(tests/test_gpu_strips.py::test_virtual_rank_driver_outputs_match_single_gpu
without pytest's diff of megabyte files).

  python tools/strip_outputs_check.py --ranks 4 [--repeat 2] [--jitter 200]

--jitter J sets HF2D_LOCAL_JITTER_US: every virtual rank sleeps a random
0..J us before each LocalGroup barrier (host collectives and halo copies), so
the ranks' threads interleave differently on every collective.  Equal files
under jitter mean no host-side ordering hole on this path."""
import argparse
import os
import sys
import tempfile
import threading

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=4)
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--jitter", type=int, default=0)
    a = ap.parse_args()
    if a.jitter:
        os.environ["HF2D_LOCAL_JITTER_US"] = str(a.jitter)
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.parallel.strips import balanced_columns

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    from test_gpu_strips import _outputs_deck

    nat = hf.native()
    text = _outputs_deck()
    stem = "Wedge15_160x40"
    names = [stem + ".plt", "tp-" + stem + ".plt", stem + ".hf2d", "HeatFlux-X-" + stem + ".plt",
             "HeatFlux-Y-" + stem + ".plt"]
    bad = 0
    for rep in range(a.repeat):
        with tempfile.TemporaryDirectory() as td:
            one, many = os.path.join(td, "one"), os.path.join(td, "many")
            os.mkdir(one)
            os.mkdir(many)
            ref = hf.Simulation(text, "gpu", lean=False)
            ref.run(max_cycles=2, outdir=one, verbose=False)
            cases = [nat.Case.from_deck(text, ".", False) for _ in range(a.ranks)]
            parts = balanced_columns(np.asarray(cases[0].field("solid")), a.ranks)
            group = nat.LocalGroup(a.ranks)
            solvers = []
            for r, (c0, c1) in enumerate(parts):
                s = nat.DeviceSolver(cases[r], 0, c0, c1)
                s.lean = False
                s.init_local(group, r)
                cases[r].trim_to_columns(c0 - 1, c1 + 1)
                solvers.append(s)
            errors = []

            def run(r):
                try:
                    solvers[r].run(2, many)
                except Exception as e:   # reported below
                    errors.append(repr(e))

            th = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(a.ranks)]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=180)
            if errors or any(t.is_alive() for t in th):
                print("rep %d: errors %s alive %s" % (rep, errors, [t.is_alive() for t in th]), flush=True)
                return 1
            for n in names:
                x = open(os.path.join(one, n), "rb").read()
                y = open(os.path.join(many, n), "rb").read()
                if x == y:
                    print("rep %d %s: equal (%d bytes)" % (rep, n, len(x)), flush=True)
                    continue
                bad += 1
                k = next((i for i in range(min(len(x), len(y))) if x[i] != y[i]), min(len(x), len(y)))
                print("rep %d %s: DIFFER sizes %d / %d, first byte %d" % (rep, n, len(x), len(y), k), flush=True)
                if n.endswith(".plt"):
                    lx, ly = x.decode(errors="replace").splitlines(), y.decode(errors="replace").splitlines()
                    nd = [i for i in range(min(len(lx), len(ly))) if lx[i] != ly[i]]
                    print("   %d lines differ; first: %r / %r" % (len(nd), lx[nd[0]][:160] if nd else "",
                                                                  ly[nd[0]][:160] if nd else ""), flush=True)
                else:
                    rec = 1248
                    print("   record %d (i=%d j=%d), byte %d within" % (k // rec, (k // rec) // 40, (k // rec) % 40,
                                                                    k % rec), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
