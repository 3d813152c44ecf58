"""Python CLI (python -m openhyperflow2d_amd) and graceful SIGINT handling."""
import json
import os
import signal
import subprocess
import sys
import time

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


def test_launcher_script_one_and_two_ranks(hf, tmp_path):
    """bin/OpenHyperFLOW2D.sh <Project> [n]: the reference's launcher contract
    (Project -> Project.dat, outputs next to the deck), n ranks via torchrun."""
    from openhyperflow2d_amd.models import decks

    (tmp_path / "W.dat").write_text(decks.wedge15(60, 20, nmax=10, nout=5))
    sh = os.path.join(ROOT, "openhyperflow2d_amd", "bin", "OpenHyperFLOW2D.sh")
    for n in ("1", "2"):
        r = subprocess.run([sh, "W", n, "--backend", "cpu", "--cycles", "1", "--no-checkpoint"], cwd=tmp_path,
                           capture_output=True, text=True, timeout=600,
                           env=dict(os.environ, HF2D_MASTER_PORT=str(29700 + int(n))))
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        assert "Computation finished" in r.stdout
    assert (tmp_path / "Wedge15_60x20.plt").exists()
