"""Command-line front end.

  python -m openhyperflow2d_amd run  deck.dat [--backend gpu|cpu|ref] [--cycles N]
                                     [--outdir DIR] [--semantics mpi|serial]
                                     [--no-checkpoint] [--no-lean] [--metrics FILE]
                                     [--profile FILE] [--fault-inject step:N,rank:R,kind:nan|kill]
                                     [--transport p2p|rccl]
  python -m openhyperflow2d_amd deck wedge15 --nx 2000 --ny 200 -o w.dat
  python -m openhyperflow2d_amd info deck.dat
  python -m openhyperflow2d_amd build

`run` is the reference driver (hf2d_start.cpp:32-368: pre-processing, outer
cycles of Nmax DEEPS steps, RMS/monitor/field/transient outputs, .hf2d
checkpoint and restart, exit monitor).  Launched under torchrun
(WORLD_SIZE > 1) it runs one x-strip per rank -- one GPU per process with the
device halo exchange over RCCL, or CPU ranks over gloo -- and rank 0 writes
the gathered outputs.  SIGINT/SIGTERM finish the cycle, write the outputs
and the checkpoint, then exit 0.  The native CLI `openhyperflow2d_amd/bin/hf2d`
offers the same single-process driver without Python.
"""
from __future__ import annotations

import argparse
import os
import sys


def _cmd_run(a) -> int:
    import openhyperflow2d_amd as hf

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    with open(a.deck, errors="replace") as f:
        text = f.read()
    workdir = os.path.dirname(os.path.abspath(a.deck))
    outdir = a.outdir or workdir
    os.makedirs(outdir, exist_ok=True)
    nat = hf.native()
    backend = a.backend or ("gpu" if hf.gpu_available() else "cpu")
    if world > 1:
        import torch
        import torch.distributed as dist

        from .parallel.dist import DistributedSimulation

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "gpu":
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        sim = DistributedSimulation(text, backend, rank=rank, world=world, device=local_rank,
                                    semantics=a.semantics, lean=not a.no_lean, workdir=workdir,
                                    use_checkpoint=not a.no_checkpoint, transport=a.transport)
    else:
        sim = hf.Simulation(text, backend, workdir=workdir, use_checkpoint=not a.no_checkpoint,
                            semantics=a.semantics, device=a.device,
                            lean=(not a.no_lean) if backend != "ref" else None)
    nat.install_signal_handlers()
    if rank == 0:
        print("hf2d: %s  %dx%d  backend=%s  ranks=%d" % (os.path.basename(a.deck), sim.case.nx, sim.case.ny,
                                                          backend, world), flush=True)
    try:
        cycles, log = sim.run(max_cycles=a.cycles, outdir=outdir, outputs=True, checkpoint=not a.no_checkpoint,
                              verbose=True, metrics=a.metrics or "", profile=a.profile or "",
                              fault=a.fault_inject or "")
    except RuntimeError as e:
        print(str(e), file=sys.stderr, flush=True)
        return 3
    if rank == 0:
        sys.stdout.write(log)
        print("\nReady. Computation finished (%d cycles)." % cycles, flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()
    return 0


def _cmd_deck(a) -> int:
    from .models import decks

    gen = decks.GENERATORS[a.name]
    kw = {}
    if a.nx:
        kw["nx"] = a.nx
    if a.ny:
        kw["ny"] = a.ny
    text = gen(**kw)
    if a.output:
        with open(a.output, "w") as f:
            f.write(text)
    else:
        sys.stdout.write(text)
    return 0


def _cmd_info(a) -> int:
    import openhyperflow2d_amd as hf

    nat = hf.native()
    with open(a.deck, errors="replace") as f:
        text = f.read()
    case = nat.Case.from_deck(text, os.path.dirname(os.path.abspath(a.deck)), False)
    import numpy as np

    solid = np.asarray(case.field("solid"))
    print("project      %s" % case.project)
    print("grid         %d x %d  (dx=%g, dy=%g)" % (case.nx, case.ny, case.dx, case.dy))
    print("problem      %s, %s" % ("Navier-Stokes" if case.problem_type == 1 else "Euler",
                                   "axisymmetric" if case.flow_type else "flat"))
    print("solid cells  %d (%.1f%%)" % (solid.sum(), 100 * solid.mean()))
    print("dt0          %g s" % case.dt0)
    print("Nmax         %d" % case.nmax)
    return 0


def _cmd_build(a) -> int:
    from . import _build

    print(_build.build(verbose=True))
    return 0


def _cmd_chem(a) -> int:
    """K12 kinetics operator on the GPU: time one call on a synthetic field, check vs the FP64 oracle."""
    import json

    from .ops import chemistry as ch
    from .ops import mechanism as mech

    m = mech.Mechanism.load(a.mech) if a.mech else mech.h2_air_li2004()
    if a.save_builtin:
        mech.h2_air_li2004().save(a.save_builtin)
        return 0
    res = ch.benchmark(m, a.nx * a.ny, a.dt, a.nsub, a.repeats, kernel=a.kernel)
    print(json.dumps(res))
    return 0 if res["incr_err_vs_numpy_fp64"] < 1e-7 else 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m openhyperflow2d_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run", help="run a .dat deck (reference driver)")
    r.add_argument("deck")
    r.add_argument("--backend", choices=["gpu", "cpu", "ref"])
    r.add_argument("--cycles", type=int, default=-1, help="stop after N outer cycles (-1: exit monitor)")
    r.add_argument("--outdir")
    r.add_argument("--semantics", default="mpi", choices=["mpi", "serial"])
    r.add_argument("--no-checkpoint", action="store_true")
    r.add_argument("--no-lean", action="store_true")
    r.add_argument("--device", type=int, default=0)
    r.add_argument("--metrics", help="append per-output-step JSON lines to this file")
    r.add_argument("--profile", help="write per-phase wall-clock JSON (steps/sync/gather/outputs) to this file")
    r.add_argument("--fault-inject", dest="fault_inject", metavar="SPEC",
                   help="step:N[,rank:R][,kind:nan|kill] -- test hook for the failure/restart paths")
    r.add_argument("--transport", choices=["p2p", "rccl"], help="multi-GPU exchange (default p2p)")
    d = sub.add_parser("deck", help="write a generated deck")
    d.add_argument("name")
    d.add_argument("--nx", type=int)
    d.add_argument("--ny", type=int)
    d.add_argument("-o", "--output")
    i = sub.add_parser("info", help="pre-process a deck and print a summary")
    i.add_argument("deck")
    sub.add_parser("build", help="build the native extension and CLIs")
    c = sub.add_parser("chem", help="run/benchmark the K12 kinetics kernels on a mechanism")
    c.add_argument("--mech", help="mechanism file (.mech); default: the built-in Li et al. 2004 H2/air set")
    c.add_argument("--kernel", default="mfma", choices=["mfma", "fast"],
                   help="mfma: runtime-mechanism MFMA kernel; fast: compiled-mechanism kernel")
    c.add_argument("--save-builtin", dest="save_builtin", metavar="PATH", help="write the built-in mechanism and exit")
    c.add_argument("--nx", type=int, default=6000)
    c.add_argument("--ny", type=int, default=400)
    c.add_argument("--nsub", type=int, default=1)
    c.add_argument("--dt", type=float, default=1e-7)
    c.add_argument("--repeats", type=int, default=10)
    a = ap.parse_args(argv)
    return {"run": _cmd_run, "deck": _cmd_deck, "info": _cmd_info, "build": _cmd_build, "chem": _cmd_chem}[a.cmd](a)


if __name__ == "__main__":
    sys.exit(main())
