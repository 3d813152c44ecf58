#!/usr/bin/env python3
"""Rehearsal of the Python multi-rank driver (DistributedSimulation.run: outer
cycles, strip outputs, checkpoints) as N processes sharing the GPUs of one box
(gloo host collectives, IPC-mapped mailbox halos), compared file by file with
one process -- the strip decomposition is bitwise by design:

  python tools/rehearse_run.py OUTDIR                                    one rank
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
      tools/rehearse_run.py OUTDIR                                       N ranks
  python tools/rehearse_run.py --compare DIR_ONE DIR_N                   byte check

The compare step checks every file both runs wrote (checkpoint slabs are
per rank, so files only one run has are listed, not compared) and exits
non-zero on the first difference.  Deck: Wedge15 400 x 80 Euler, up to 2 cycles of
40 steps, outputs every 20, autotune on (ThreadBlockSize 0): each rank's
tuning choices come from its own timings, as on a multi-GPU node."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _digest(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def compare(a, b):
    fa = {f for f in os.listdir(a) if os.path.isfile(os.path.join(a, f))}
    fb = {f for f in os.listdir(b) if os.path.isfile(os.path.join(b, f))}
    common = sorted(fa & fb)
    bad = [f for f in common if _digest(os.path.join(a, f)) != _digest(os.path.join(b, f))]
    print("compared %d files; only in %s: %s; only in %s: %s" % (len(common), a, sorted(fa - fb), b, sorted(fb - fa)))
    for f in bad:
        print("DIFFERS:", f)
    return 1 if bad or not common else 0


def main():
    if sys.argv[1] == "--compare":
        return compare(sys.argv[2], sys.argv[3])
    outdir = os.path.abspath(sys.argv[1])
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    ndev = max(1, torch.cuda.device_count())
    torch.cuda.set_device(local % ndev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from openhyperflow2d_amd.models import decks
    from openhyperflow2d_amd.parallel.dist import DistributedSimulation

    os.makedirs(outdir, exist_ok=True)
    text = decks.wedge15(400, 80, nmax=40, nout=20)
    sim = DistributedSimulation(text, "gpu", rank=rank, world=world, device=local % ndev, workdir=outdir)
    cycles, _ = sim.run(max_cycles=2, outdir=outdir, verbose=False)
    if rank == 0:
        print("rank 0: %d cycles, transport %s, %d files" % (cycles, sim.transport, len(os.listdir(outdir))),
              flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
