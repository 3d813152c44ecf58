#!/usr/bin/env python3
"""Cost of the multi-GPU halo exchange on one GPU, without a second strip
competing for the device.

One strip of an N-rank decomposition is timed twice on the same GPU:

  alone     the strip's DeviceSolver with no transport (its ghost columns
            are never refreshed): the step kernels only;
  loopback  the same strip as rank r of N on the xGMI mailbox transport with
            every peer already published and the neighbours' mailboxes
            looped back into its own (DeviceSolver.p2p_loopback): every edge
            push, publication, flag poll, dt fold and ghost staging of a real
            exchange, no waiting.

loopback - alone is the exchange's device-side cost per step (the xGMI link
latency itself is not in it).  Both use the tile geometry the autotune picks
for the strip alone.

  python tools/exchange_loopback.py --config wedge15 --ranks 8 [--rank 4] [--lagged-dt]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="wedge15", choices=["wedge15", "step", "resonator", "triple_point", "scramjet"])
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--rank", type=int, default=-1, help="strip (default: the middle one)")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--lagged-dt", action="store_true")
    ap.add_argument("--nofuse", action="store_true", help="separate exchange kernel instead of the fused tail")
    ap.add_argument("--trace", action="store_true", help="phase clocks of the fused tail (last workgroup), median us")
    a = ap.parse_args()
    if a.trace:   # (read once, at the first fused step)
        os.environ["HF2D_FX_SKIP"] = str(int(os.environ.get("HF2D_FX_SKIP", "0")) | 16)
    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks
    from openhyperflow2d_amd.models.simulation import maybe_autotune
    from openhyperflow2d_amd.parallel.strips import balanced_columns

    import bench

    nat = hf.native()
    if a.config == "wedge15":
        text = decks.wedge15(2000, 200, nmax=10 ** 9, nout=10 ** 8)
    else:
        nx, ny, _ = bench.CONFIGS[a.config]
        text = decks.GENERATORS[a.config](nx, ny, nmax=10 ** 9, nout=10 ** 8)
    if a.lagged_dt:
        text = decks.set_key(text, "LaggedDt", 1)
    r = a.rank if a.rank >= 0 else a.ranks // 2
    case0 = nat.Case.from_deck(text, ".", False)
    parts = balanced_columns(np.asarray(case0.field("solid")), a.ranks)
    gi0, gi1 = parts[r]

    def timed(s, n):
        s.synchronize()
        t0 = time.perf_counter()
        s.run_steps(n, False)
        s.synchronize()
        return (time.perf_counter() - t0) / n * 1e6

    alone = nat.DeviceSolver(nat.Case.from_deck(text, ".", False), 0, gi0, gi1)
    tune = maybe_autotune(case0, alone)
    geom = dict(lean_nt=alone.lean_nt, lean_cpt=alone.lean_cpt, lean_tj=alone.lean_tj, lean_wgcu=alone.lean_wgcu,
                use_graph=alone.use_graph)
    loop = nat.DeviceSolver(nat.Case.from_deck(text, ".", False), 0, gi0, gi1)
    for k, v in geom.items():
        setattr(loop, k, v)
    loop.p2p_loopback(r, a.ranks)
    loop.p2p_fuse = not a.nofuse
    res = {"alone": [], "loopback": []}
    for s in (alone, loop):
        s.run_steps(a.warmup, False)
    for _ in range(a.repeat):   # interleaved, so drifts of the box hit both
        res["alone"].append(timed(alone, a.steps))
        res["loopback"].append(timed(loop, a.steps))
    rec = {"config": a.config, "ranks": a.ranks, "rank": r, "strip": [gi0, gi1], "cells": (gi1 - gi0) * case0.ny,
           "lagged_dt": a.lagged_dt, "fused": not a.nofuse, "geometry": geom, "autotune": tune or None,
           "alone_us": [round(x, 3) for x in res["alone"]], "loopback_us": [round(x, 3) for x in res["loopback"]],
           "exchange_us": round(min(res["loopback"]) - min(res["alone"]), 3),
           "exchange_rel": round(min(res["loopback"]) / min(res["alone"]) - 1.0, 4),
           "stats": {"overlap_steps": loop.overlap_steps, "lns_fx_steps": loop.lns_fx_steps,
                     "p2p_mwg_exchanges": loop.p2p_mwg_exchanges, "lnm_steps": loop.lnm_steps}}
    if a.trace:
        tr = np.asarray(loop.fx_trace(), dtype=np.float64).reshape(-1, 8)
        tr = tr[tr[:, 7] > 0]
        names = ["drain", "count", "dt_min", "dt_publish", "flags", "wait_fold", "store", "total"]
        d = np.diff(tr, axis=1) / 100.0   # 100 MHz clock -> us
        med = np.median(d, axis=0).tolist() + [float(np.median((tr[:, 7] - tr[:, 0]) / 100.0))]
        rec["tail_us"] = {k: round(v, 3) for k, v in zip(names, med)}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
