"""Strip decomposition over torch.distributed (gloo, 2 ranks on 127.0.0.1):
results must be bit-identical to the single-rank run (Jacobi semantics,
deterministic lexicographic residual reduction).  The GPU path uses the same
halo groups over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from openhyperflow2d_amd.models import decks

FIELDS = ["rho", "U", "V", "p", "T"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fields(text):
    return FIELDS + (["Y:H2", "Y:O2", "Y:H2O", "Y:OH", "Y:N2"] if "<data/Mechanism=" in text else [])


def _worker(rank, world, port, text, steps, lean, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from openhyperflow2d_amd.parallel.dist import DistributedSimulation

        sim = DistributedSimulation(text, "cpu", rank=rank, world=world, lean=lean)
        for s in range(3):
            sim.step(steps, residual=(s != 1))
        out = {f.replace(":", "_"): sim.gather_field(f) for f in _fields(text)}
        summ = sim.summary()
        if rank == 0:
            np.savez(os.path.join(outdir, "res.npz"), dt=summ["dt"], time=summ["time"],
                     rms=np.array(summ["rms"]), **out)
    finally:
        dist.barrier()
        dist.destroy_process_group()


CASES = {
    "wedge15_euler": (lambda: decks.wedge15(90, 30, nmax=10 ** 6, nout=10 ** 5), 5),
    "wedge15_ns_keps": (lambda: decks.wedge15(90, 30, navier_stokes=True, turbulence=4, nmax=10 ** 6,
                                              nout=10 ** 5), 4),
    # mechanism mode (species block + operator-split kinetics + SST)
    "scramjet_mech": (lambda: decks.with_mechanism(decks.scramjet(120, 40, nmax=10 ** 6, nout=10 ** 5), substeps=2,
                                                   tmin=250.0), 4),
}


@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("lean", [False, True])
def test_two_strips_match_single_rank(hf, case, lean, tmp_path):
    mk, steps = CASES[case]
    text = mk()
    ref = hf.Simulation(text, "cpu", lean=lean)
    for s in range(3):
        ref.step(steps, residual=(s != 1))
    mp.start_processes(_worker, args=(2, _free_port(), text, steps, lean, str(tmp_path)), nprocs=2,
                       join=True, start_method="spawn")
    got = np.load(tmp_path / "res.npz")
    summ = ref.summary()
    assert float(got["dt"]) == summ["dt"]
    np.testing.assert_allclose(got["rms"], summ["rms"], rtol=1e-12, atol=0)
    for f in _fields(text):
        np.testing.assert_array_equal(got[f.replace(":", "_")], ref.field(f), err_msg=f)


def _run_worker(rank, world, port, text, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from openhyperflow2d_amd.parallel.dist import DistributedSimulation

        # generic stepper: it maintains the full record incl. the dS scratch
        sim = DistributedSimulation(text, "cpu", rank=rank, world=world, lean=False)
        os.makedirs(outdir, exist_ok=True)
        sim.run(max_cycles=2, outdir=outdir)
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_two_strip_driver_outputs_match_single_rank(hf, tmp_path):
    """Full driver (2 outer cycles): rank 0 gathers the strips and writes the
    field dump and checkpoint; they must equal the single-rank run's bytes."""
    text = decks.wedge15(90, 30, nmax=12, nout=4)
    one = tmp_path / "one"
    two = tmp_path / "two"
    one.mkdir()
    sim = hf.Simulation(text, "cpu")
    sim.run(max_cycles=2, outdir=str(one))
    mp.start_processes(_run_worker, args=(2, _free_port(), text, str(two)), nprocs=2, join=True,
                       start_method="spawn")
    for name in ["Wedge15_90x30.plt", "Wedge15_90x30.hf2d", "tp-Wedge15_90x30.plt"]:
        assert (one / name).read_bytes() == (two / name).read_bytes(), name
    r1 = (one / "RMS-Wedge15_90x30.plt").read_text().split()
    r2 = (two / "RMS-Wedge15_90x30.plt").read_text().split()
    assert len(r1) == len(r2)


def _fault_worker(rank, world, port, text, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from openhyperflow2d_amd.parallel.dist import DistributedSimulation

        sim = DistributedSimulation(text, "cpu", rank=rank, world=world, workdir=outdir)
        try:
            sim.run(max_cycles=3, outdir=outdir, checkpoint=True, verbose=True, fault="step:27,rank:1")
            msg = "no error"
        except RuntimeError as e:
            msg = str(e)
        with open(os.path.join(outdir, "msg%d.txt" % rank), "w") as f:
            f.write(msg)
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_fault_on_one_rank_stops_every_rank(hf, tmp_path):
    """A NaN fault injected on rank 1 makes every rank stop with the Tg < 0
    error (the flag is MAX-reduced), each rank writes its own
    rank-<r>-<P>-err.plt, and the checkpoint of the last completed cycle stays."""
    text = decks.wedge15(90, 30, nmax=20, nout=5)
    text = decks.set_key(text, "MonitorIndex", 1)
    text = decks.set_key(text, "ExitMonitorValue", 1e-30)
    mp.start_processes(_fault_worker, args=(2, _free_port(), text, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    for r in (0, 1):
        msg = (tmp_path / ("msg%d.txt" % r)).read_text()
        assert "unstability" in msg, msg
        assert (tmp_path / ("rank-%d-Wedge15_90x30-err.plt" % r)).exists()
    assert "in cell (" in (tmp_path / "msg1.txt").read_text()   # the poisoned rank names the cell
    import json

    assert json.loads((tmp_path / "Wedge15_90x30.hf2d.meta").read_text())["iteration"] == 20
