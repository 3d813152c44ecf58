"""Strip-local pre-processing: no rank holds the whole field, rank 0
included.  Every rank pre-processes its own columns on the whole
grid's 16 B/cell flag plane (Case.from_deck_window, tests in
test_window_preprocess.py) instead of the reference's rank-0 pre-processing
and scatter (hf2d_start.cpp:143-205): its peak host memory for the case +
solver follows its share of the grid, and the merged eligibility facts make
every rank run the same kernel path (the strip runs themselves are compared
byte for byte with one rank in test_distributed.py).  Case.pack_strip /
unpack_strip remain as an API (a strip Case as bytes)."""
import json
import os
import resource
import socket

import numpy as np
import torch.multiprocessing as mp

from openhyperflow2d_amd.models import decks


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _peak_kb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss


def _cur_kb():
    with open("/proc/self/statm") as f:
        return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE") // 1024


def _deck():
    return decks.wedge15(3200, 400, nmax=10 ** 6, nout=10 ** 5)


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from openhyperflow2d_amd.parallel.dist import DistributedSimulation

    text = _deck()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dist.barrier()
        before = _cur_kb()
        sim = DistributedSimulation(text, "cpu", rank=rank, world=world)
        peak = _peak_kb() - before
        a, b = sim.case.resident_columns
        with open(os.path.join(outdir, "r%d.json" % rank), "w") as f:
            json.dump({"peak_kb": peak, "cols": [a, b], "parts": sim.parts}, f)
    finally:
        dist.barrier()
        dist.destroy_process_group()


def _single(outdir):
    import openhyperflow2d_amd as hf

    text = _deck()
    before = _cur_kb()
    sim = hf.Simulation(text, "cpu")
    with open(os.path.join(outdir, "single.json"), "w") as f:
        json.dump({"peak_kb": _peak_kb() - before, "nx": sim.case.nx}, f)


def test_strip_ranks_never_hold_the_whole_field(hf, tmp_path):
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_single, args=(str(tmp_path),))
    p.start()
    p.join()
    assert p.exitcode == 0
    world = 8
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    one = json.load(open(tmp_path / "single.json"))
    ranks = [json.load(open(tmp_path / ("r%d.json" % r))) for r in range(world)]
    for r, d in enumerate(ranks):
        gi0, gi1 = d["parts"][r]
        assert d["cols"] == [max(gi0 - 1, 0), min(gi1 + 1, one["nx"])]
    # every rank's case + solver memory follows its share of the grid (the
    # strips are balanced by active cells, so their widths differ) -- rank 0
    # too: its peak is within 2x of the other ranks' mean
    peaks = [d["peak_kb"] for d in ranks]
    share = [(d["parts"][r][1] - d["parts"][r][0]) / one["nx"] for r, d in enumerate(ranks)]
    assert peaks[0] <= 2.0 * sum(peaks[1:]) / len(peaks[1:]), peaks
    assert sum(peaks) / len(peaks) <= 0.25 * one["peak_kb"], (peaks, one["peak_kb"])
    for p, f in zip(peaks, share):
        assert p <= (1.5 * f + 0.05) * one["peak_kb"], (peaks, share, one["peak_kb"])


def test_pack_unpack_roundtrip_keeps_the_strip_and_facts(hf):
    text = decks.wedge15(120, 40, navier_stokes=True, turbulence=4, nmax=10 ** 6, nout=10 ** 5)
    nat = hf.native()
    full = nat.Case.from_deck(text, ".", False)
    blob = full.pack_strip(30, 71)
    part = nat.Case.unpack_strip(blob)
    assert part.resident_columns == (30, 71) and part.facts_valid
    for name in ("rho", "U", "T", "mu_t", "CT", "l_min"):
        a, b = np.asarray(full.field(name)), np.asarray(part.field(name))
        np.testing.assert_array_equal(a[30:71], b[30:71], err_msg=name)
        assert not b[:30].any() and not b[71:].any()
    # header + chunked payload == one blob
    hdr = full.pack_strip_header(30, 71)
    n = full.strip_payload_bytes(30, 71)
    chunks = nat.Case.unpack_strip_header(np.frombuffer(hdr, dtype=np.uint8))
    buf = np.empty(1000, dtype=np.uint8)
    for off in range(0, n, 1000):
        k = min(1000, n - off)
        full.read_strip_payload(30, 71, off, buf[:k])
        chunks.write_strip_payload(off, buf[:k])
    assert chunks.resident_columns == (30, 71)
    np.testing.assert_array_equal(np.asarray(chunks.field("rho")), np.asarray(part.field("rho")))
