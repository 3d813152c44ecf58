#!/usr/bin/env python3
"""Peak host RSS of every rank of a strip run's set-up (pre-processing +
solver construction), gloo CPU ranks:

  python tools/rank_rss.py --config triple_point --ranks 8 [--single]

Each rank builds DistributedSimulation(deck, "cpu") -- strip-local
pre-processing (Case.from_deck_window) and its CpuSolver -- and reports
ru_maxrss; --single also measures one rank holding the whole grid.  Prints
one JSON line."""
import argparse
import json
import os
import resource
import socket
import sys
import tempfile

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _deck(cfg):
    from openhyperflow2d_amd.models import decks

    return decks.GENERATORS[cfg](nmax=10 ** 6, nout=10 ** 5)


def _rank(rank, world, port, cfg, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from openhyperflow2d_amd.parallel.dist import DistributedSimulation

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sim = DistributedSimulation(_deck(cfg), "cpu", rank=rank, world=world)
        rec = {"rank": rank, "peak_mb": resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024,
               "cols": list(sim.case.resident_columns)}
        with open(os.path.join(outdir, "r%d.json" % rank), "w") as f:
            json.dump(rec, f)
    finally:
        dist.barrier()
        dist.destroy_process_group()


def _single(cfg, outdir):
    import openhyperflow2d_amd as hf

    hf.Simulation(_deck(cfg), "cpu")
    with open(os.path.join(outdir, "single.json"), "w") as f:
        json.dump({"peak_mb": resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024}, f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="triple_point")
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--single", action="store_true")
    a = ap.parse_args()
    import torch.multiprocessing as mp

    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rank, args=(a.ranks, _port(), a.config, d), nprocs=a.ranks, join=True,
                           start_method="spawn")
        ranks = [json.load(open(os.path.join(d, "r%d.json" % r))) for r in range(a.ranks)]
        out = {"config": a.config, "ranks": a.ranks, "peak_mb": [round(r["peak_mb"]) for r in ranks],
               "cols": [r["cols"] for r in ranks]}
        workers = out["peak_mb"][1:]
        out["rank0_over_worker_mean"] = round(out["peak_mb"][0] / (sum(workers) / len(workers)), 3)
        if a.single:
            p = mp.get_context("spawn").Process(target=_single, args=(a.config, d))
            p.start()
            p.join()
            out["single_rank_peak_mb"] = round(json.load(open(os.path.join(d, "single.json")))["peak_mb"])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
