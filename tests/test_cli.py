"""Python CLI (python -m openhyperflow2d_amd) and graceful SIGINT handling."""
import json
import os
import signal
import subprocess
import sys
import time

import pytest

from tests.conftest import ROOT


def _py(*args, **kw):
    env = dict(os.environ, PYTHONPATH=ROOT)
    return subprocess.run([sys.executable, "-m", "openhyperflow2d_amd", *args], capture_output=True, text=True,
                          env=env, **kw)


def test_deck_info_run(hf, tmp_path):
    deck = tmp_path / "w.dat"
    r = _py("deck", "wedge15", "--nx", "80", "--ny", "30", "-o", str(deck))
    assert r.returncode == 0, r.stderr
    r = _py("info", str(deck))
    assert r.returncode == 0 and "80 x 30" in r.stdout, r.stdout + r.stderr
    r = _py("run", str(deck), "--backend", "cpu", "--cycles", "1", "--metrics", str(tmp_path / "m.jsonl"),
            timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "Computation finished" in r.stdout
    for f in ["Wedge15_80x30.plt", "RMS-Wedge15_80x30.plt", "Wedge15_80x30.hf2d", "Wedge15_80x30.hf2d.meta"]:
        assert (tmp_path / f).exists(), f
    lines = [json.loads(x) for x in (tmp_path / "m.jsonl").read_text().splitlines()]
    assert lines and all(len(x["rms"]) == 9 for x in lines)


def test_sigint_finishes_cycle_and_checkpoints(hf, tmp_path):
    from openhyperflow2d_amd.models import decks

    text = decks.wedge15(200, 60, nmax=10 ** 7, nout=20)
    (tmp_path / "w.dat").write_text(text)
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.Popen([sys.executable, "-m", "openhyperflow2d_amd", "run", "w.dat", "--backend", "cpu"],
                         cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    time.sleep(8)
    p.send_signal(signal.SIGINT)
    out, _ = p.communicate(timeout=300)
    assert p.returncode == 0, out[-3000:]
    assert "Interrupted by user" in out
    assert (tmp_path / "Wedge15_200x60.hf2d").exists()
    meta = json.loads((tmp_path / "Wedge15_200x60.hf2d.meta").read_text())
    assert meta["iteration"] > 0


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_native_ranks_match_one_rank(hf, tmp_path, n):
    """bin/OpenHyperFLOW2D.sh <Project> [n]: the reference's launcher contract
    (Project -> Project.dat in the working directory) running n processes of
    the native binary (TCP rendezvous from RANK/WORLD_SIZE/MASTER_*, no
    Python): the outputs of n strip ranks equal one rank's byte for byte."""
    from openhyperflow2d_amd.models import decks

    text = decks.wedge15(90, 30, navier_stokes=True, turbulence=4, nmax=8, nout=4)
    for k, v in {"NSaveStep": 1, "is_Cx_calc": 1, "x_body": 0.03, "y_body": 0.0, "dx_body": 0.03,
                 "dy_body": 0.01, "Cx_Flow_Index": 1, "NumXCut": 1, "CutX-1.x0": 0.0405, "CutX-1.y0": 0.0,
                 "CutX-1.dy": 0.02}.items():
        text = decks.set_key(text, k, v)
    sh = os.path.join(ROOT, "openhyperflow2d_amd", "bin", "OpenHyperFLOW2D.sh")
    logs = {}
    for k in (1, n):
        d = tmp_path / ("r%d" % k)
        d.mkdir()
        (d / "W.dat").write_text(text)
        r = subprocess.run([sh, "W", str(k), "--backend", "cpu", "--cycles", "2", "--no-checkpoint"], cwd=d,
                           capture_output=True, text=True, timeout=600,
                           env=dict(os.environ, HF2D_MASTER_PORT=str(29700 + 10 * n + k),
                                    HF2D_BIN=os.path.join(ROOT, "openhyperflow2d_amd", "bin", "hf2d_cpu")))
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        assert r.stdout.count("Computation finished") == 1
        logs[k] = r.stdout
    assert "halo transport tcp" in logs[n]
    for name in ["Wedge15_90x30.plt", "tp-Wedge15_90x30.plt", "Wedge15_90x30.hf2d"]:
        assert (tmp_path / "r1" / name).read_bytes() == (tmp_path / ("r%d" % n) / name).read_bytes(), name
    cut = [ln for ln in logs[1].splitlines() if ln.startswith(("Cut(", "Cx ="))]
    assert cut and cut == [ln for ln in logs[n].splitlines() if ln.startswith(("Cut(", "Cx ="))]


def test_sigint_two_native_ranks_checkpoint(hf, tmp_path):
    """Ctrl-C on a 2-rank native run (both ranks get SIGINT, as from a
    terminal): a signal landing inside the TCP halo exchange must not abort
    the exchange (poll EINTR is retried); the ranks agree to stop at the next
    output step and write the cycle outputs and the checkpoint."""
    from openhyperflow2d_amd.models import decks

    text = decks.wedge15(300, 80, nmax=10 ** 7, nout=20)
    (tmp_path / "w.dat").write_text(text)
    exe = os.path.join(ROOT, "openhyperflow2d_amd", "bin", "hf2d_cpu")
    port = 29800 + os.getpid() % 100
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([exe, "--backend", "cpu", "w.dat"], cwd=tmp_path, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    time.sleep(6)
    for _ in range(5):   # several signals, most land inside an exchange
        for p in procs:
            p.send_signal(signal.SIGINT)
        time.sleep(0.05)
    outs = [p.communicate(timeout=300)[0] for p in procs]
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]
    assert "Interrupted by user" in outs[0]
    assert (tmp_path / "Wedge15_300x80.hf2d").stat().st_size == 300 * 80 * 1248
    meta = json.loads((tmp_path / "Wedge15_300x80.hf2d.meta").read_text())
    assert meta["iteration"] > 0
