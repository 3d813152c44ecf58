"""Strip-decomposed DEEPS driver on the GPU without a gather: N DeviceSolvers
(in-process virtual ranks, one host thread each, LocalGroup transport) run the
full driver into ONE output directory -- each writes its share of the field
dumps and checkpoint, the Cut / Cx / heat-flux integrals are folded from
per-strip term lists and y+ from the merged wall friction velocities.  The
files must equal the single-GPU run's bytes."""
import threading

import numpy as np
import pytest

from openhyperflow2d_amd.models import decks

pytestmark = pytest.mark.gpu


def _outputs_deck():
    t = decks.wedge15(160, 40, navier_stokes=True, turbulence=4, nmax=12, nout=4)
    kv = {"NSaveStep": 1, "isOutHeatFluxX": 1, "isOutHeatFluxY": 1, "Cp_Flow_Index": 1, "y_max": 30, "y_min": 0,
          "is_Cx_calc": 1, "x_body": 0.05, "y_body": 0.0, "dx_body": 0.06, "dy_body": 0.015, "Cx_Flow_Index": 1,
          "NumXCut": 2, "CutX-1.x0": 0.0305, "CutX-1.y0": 0.0, "CutX-1.dy": 0.03, "CutX-2.x0": 0.12,
          "CutX-2.y0": 0.005, "CutX-2.dy": 0.03}
    for k, v in kv.items():
        t = decks.set_key(t, k, v)
    return t


def _assert_same_bytes(a, b):
    """Byte equality with a short report (pytest's own diff of megabyte files
    outruns the test time limit)."""
    x, y = a.read_bytes(), b.read_bytes()
    if x == y:
        return
    k = next((i for i in range(min(len(x), len(y))) if x[i] != y[i]), min(len(x), len(y)))
    pytest.fail("%s: %d / %d bytes, first difference at byte %d: %r / %r" % (
        a.name, len(x), len(y), k, x[max(0, k - 60):k + 60], y[max(0, k - 60):k + 60]))


def _cut_lines(log):
    return [ln for ln in log.splitlines() if ln.startswith(("Cut(", "Cx ="))]


@pytest.mark.parametrize("nranks,jitter", [(4, 0), (8, 0), (4, 300)])
def test_virtual_rank_driver_outputs_match_single_gpu(gpu, tmp_path, monkeypatch, nranks, jitter):
    """N DeviceSolvers on threads (LocalGroup transport, generic k-eps path,
    outputs without a gather) write the same bytes as one GPU.  jitter > 0:
    every rank sleeps a random 0..jitter us before each LocalGroup barrier
    (HF2D_LOCAL_JITTER_US), so the threads reach every host collective and
    halo copy in a different order -- an ordering hole on this path would
    show as a byte difference (README, round 6: the one unexplained round-5
    mismatch)."""
    from openhyperflow2d_amd.parallel.strips import balanced_columns

    if jitter:
        monkeypatch.setenv("HF2D_LOCAL_JITTER_US", str(jitter))
    nat = gpu.native()
    text = _outputs_deck()
    one, many = tmp_path / "one", tmp_path / "many"
    one.mkdir()
    many.mkdir()
    ref = gpu.Simulation(text, "gpu", lean=False)
    _, log1 = ref.run(max_cycles=2, outdir=str(one))

    cases = [nat.Case.from_deck(text, ".", False) for _ in range(nranks)]
    parts = balanced_columns(np.asarray(cases[0].field("solid")), nranks)
    group = nat.LocalGroup(nranks)
    solvers = []
    for r, (a, b) in enumerate(parts):
        s = nat.DeviceSolver(cases[r], 0, a, b)
        s.lean = False
        s.init_local(group, r)
        cases[r].trim_to_columns(a - 1, b + 1)
        solvers.append(s)
    logs, errors = {}, []

    def run(r):
        try:
            logs[r] = solvers[r].run(2, str(many))[1]
        except Exception as e:   # pragma: no cover - reported below
            errors.append(e)

    th = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=180)
    assert not errors, errors
    assert not any(t.is_alive() for t in th), "virtual-rank driver hung"
    stem = "Wedge15_160x40"
    for name in [stem + ".plt", "tp-" + stem + ".plt", stem + ".hf2d", "HeatFlux-X-" + stem + ".plt",
                 "HeatFlux-Y-" + stem + ".plt"]:
        _assert_same_bytes(one / name, many / name)
    assert _cut_lines(logs[0]) == _cut_lines(log1) and len(_cut_lines(log1)) >= 3
    # each host keeps only its strip and one ghost column each side
    for r, (a, b) in enumerate(parts):
        assert tuple(cases[r].resident_columns) == (max(a - 1, 0), min(b + 1, cases[r].nx))


def test_native_cli_two_gpu_ranks_match_one(gpu, tmp_path):
    """bin/OpenHyperFLOW2D.sh <Project> 2 with the GPU backend: two native
    processes (TCP rendezvous, IPC-mapped xGMI mailboxes validated at start-up
    -- here both ranks share the box's one GPU) write the same bytes as one."""
    import os
    import subprocess

    from tests.conftest import ROOT

    text = _outputs_deck()
    sh = os.path.join(ROOT, "openhyperflow2d_amd", "bin", "OpenHyperFLOW2D.sh")
    logs = {}
    for k in (1, 2):
        d = tmp_path / ("r%d" % k)
        d.mkdir()
        (d / "W.dat").write_text(text)
        r = subprocess.run(["timeout", "-k", "10", "240", sh, "W", str(k), "--backend", "gpu", "--cycles", "2",
                            "--no-checkpoint"], cwd=d, capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, HF2D_MASTER_PORT=str(29800 + k), HF2D_AUTOTUNE="0"))
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        logs[k] = r.stdout
    assert "halo transport p2p" in logs[2], logs[2][-2000:]
    stem = "Wedge15_160x40"
    for name in [stem + ".plt", "tp-" + stem + ".plt", stem + ".hf2d", "HeatFlux-X-" + stem + ".plt"]:
        _assert_same_bytes(tmp_path / "r1" / name, tmp_path / "r2" / name)
    assert _cut_lines(logs[1]) == _cut_lines(logs[2])


def _mailbox_deck(deck, lagged):
    if deck == "wedge":       # the headline deck family (inviscid, fused mailbox exchange in the tile kernel)
        t = decks.wedge15(320, 60, nmax=24, nout=12)
    elif deck == "resonator":  # axisymmetric k-eps, lean N-S tiles, fused push in the tile kernel
        t = decks.resonator(320, 40, nmax=24, nout=12)
    else:                      # SST + 9-species kinetics, lean mechanism step + push / unpack
        t = decks.scramjet(320, 48, nmax=24, nout=12)
    return decks.set_key(t, "LaggedDt", int(lagged))


@pytest.mark.parametrize("deck", ["wedge", "resonator", "scramjet"])
def test_native_cli_mailbox_ranks_match_one(gpu, tmp_path, deck):
    """The default multi-GPU transport (xGMI mailboxes, IPC-mapped, validated
    at start-up) at the BASELINE rank counts: 4 and 8 native processes (one
    GPU here, so the ranks share it) write the same bytes as one process, with
    lagged dt off and on.  Separate OS processes, because in-process virtual
    ranks cannot co-schedule more spinning exchange kernels than the process
    has HIP hardware queues (DeviceSolver::p2p_import refuses that case)."""
    import os
    import subprocess

    from tests.conftest import ROOT

    sh = os.path.join(ROOT, "openhyperflow2d_amd", "bin", "OpenHyperFLOW2D.sh")
    port = 29820 + 10 * ["wedge", "resonator", "scramjet"].index(deck)
    for lagged in (0, 1):
        text = _mailbox_deck(deck, lagged)
        dirs = {}
        for k in (1, 4, 8):
            d = tmp_path / ("l%d_r%d" % (lagged, k))
            d.mkdir()
            (d / "D.dat").write_text(text)
            r = subprocess.run(["timeout", "-k", "10", "240", sh, "D", str(k), "--backend", "gpu", "--cycles", "2"],
                               cwd=d, capture_output=True, text=True, timeout=300,
                               env=dict(os.environ, HF2D_MASTER_PORT=str(port + k), HF2D_AUTOTUNE="0"))
            assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
            if k > 1:
                assert "halo transport p2p" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
                assert "using RCCL" not in r.stderr, r.stderr[-2000:]
            dirs[k] = d
        names = sorted(p.name for p in dirs[1].iterdir() if p.suffix in (".plt", ".hf2d", ".species", ".meta"))
        assert any(n.endswith(".hf2d") for n in names), names
        for k in (4, 8):
            for name in names:
                _assert_same_bytes(dirs[1] / name, dirs[k] / name)
