"""Run an N-strip decomposition with RCCL halos on ONE GPU (all ranks share
device 0; torch.distributed/gloo only bootstraps the RCCL unique id) and
compare with the single-rank GPU run.  Exercises the device halo pack/unpack,
ncclSend/Recv grouping and the dt MIN all-reduce without a multi-GPU node.

  python tools/multirank_gpu_check.py --ranks 2
"""
import argparse
import os
import socket
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FIELDS = ["rho", "U", "V", "p", "T"]


def _worker(rank, world, port, text, steps, lean, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch  # noqa: F401
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    from openhyperflow2d_amd.parallel.dist import DistributedSimulation

    sim = DistributedSimulation(text, "gpu", rank=rank, world=world, device=0, lean=lean)
    for s in range(3):
        sim.step(steps, residual=(s != 1))
    res = {f: sim.gather_field(f) for f in FIELDS}
    summ = sim.summary()
    if rank == 0:
        np.savez(out, dt=summ["dt"], rms=np.array(summ["rms"]), **res)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--nx", type=int, default=240)
    ap.add_argument("--ny", type=int, default=60)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--physics", default="euler")
    ap.add_argument("--no-lean", action="store_true")
    a = ap.parse_args()
    import torch.multiprocessing as mp

    import openhyperflow2d_amd as hf
    from openhyperflow2d_amd.models import decks

    ns = a.physics != "euler"
    text = decks.wedge15(a.nx, a.ny, navier_stokes=ns, turbulence=4 if a.physics == "kes" else 0,
                         nmax=10 ** 6, nout=10 ** 5)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = "/tmp/hf2d_multirank_%d.npz" % os.getpid()
    mp.start_processes(_worker, args=(a.ranks, port, text, a.steps, not a.no_lean, out), nprocs=a.ranks,
                       join=True, start_method="spawn")
    got = np.load(out)
    ref = hf.Simulation(text, "gpu", lean=not a.no_lean)
    for s_ in range(3):
        ref.step(a.steps, residual=(s_ != 1))
    ok = float(got["dt"]) == ref.summary()["dt"]
    print("dt equal:", ok, float(got["dt"]), ref.summary()["dt"])
    for f in FIELDS:
        d = np.abs(got[f] - ref.field(f)).max()
        print(f, "max abs diff", d)
        ok = ok and d == 0
    print("MULTIRANK_OK" if ok else "MULTIRANK_MISMATCH")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
