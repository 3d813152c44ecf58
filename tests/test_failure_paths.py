"""Failure detection, fault injection and restart.

The reference reports Tg < 0 with an error Tecplot snapshot <P>-err.plt and
aborts (deeps2d_core.cpp:1246-1316); recovery is a restart from the last
.hf2d image.  Here: --fault-inject poisons a cell (kind nan) or SIGKILLs a
rank (kind kill); the error snapshot is written, the previous cycle's
checkpoint survives, and a rerun resumes from it.
"""
import json
import os
import signal
import subprocess
import sys

import pytest

from openhyperflow2d_amd.models import decks
from openhyperflow2d_amd.models.simulation import parse_fault
from tests.conftest import ROOT

STEM = "Wedge15_80x30"


def _deck(tmp_path, nmax=20, nout=5):
    text = decks.wedge15(80, 30, nmax=nmax, nout=nout)
    text = decks.set_key(text, "MonitorIndex", 1)           # residual exit monitor ...
    text = decks.set_key(text, "ExitMonitorValue", 1e-30)   # ... never met: run every requested cycle
    p = tmp_path / "w.dat"
    p.write_text(text)
    return p, text


def _cli(tmp_path, *args):
    env = dict(os.environ, PYTHONPATH=ROOT)
    return subprocess.run([sys.executable, "-m", "openhyperflow2d_amd", "run", "w.dat", "--backend", "cpu", *args],
                          cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)


def test_parse_fault():
    assert parse_fault("") == (-1, 0, "nan")
    assert parse_fault("step:12,rank:1,kind:kill") == (12, 1, "kill")
    with pytest.raises(ValueError):
        parse_fault("rank:1")
    with pytest.raises(ValueError):
        parse_fault("step:3,kind:segv")


@pytest.mark.parametrize("backend", ["cpu", "ref"])
def test_nan_fault_writes_error_snapshot_and_keeps_checkpoint(hf, tmp_path, backend):
    _, text = _deck(tmp_path)
    sim = hf.Simulation(text, backend, workdir=str(tmp_path))
    with pytest.raises(RuntimeError) as ei:
        sim.run(max_cycles=3, outdir=str(tmp_path), verbose=True, fault="step:27",
                profile=str(tmp_path / "prof.json"))
    msg = str(ei.value)
    assert "unstability" in msg and "Error snapshot" in msg and "last good checkpoint (iteration 20)" in msg
    assert "CT_NODE_IS_SET_2D" in msg and "in cell (" in msg     # PrintCond of the failing cell
    err = tmp_path / (STEM + "-err.plt")
    assert err.exists() and err.stat().st_size > 0
    meta = json.loads((tmp_path / (STEM + ".hf2d.meta")).read_text())
    assert meta["iteration"] == 20     # the cycle before the fault
    prof = json.loads((tmp_path / "prof.json").read_text())
    assert prof["phases"]["steps"]["calls"] >= 27


def test_profile_json_phases(hf, tmp_path):
    _, text = _deck(tmp_path)
    sim = hf.Simulation(text, "cpu", workdir=str(tmp_path))
    n, _ = sim.run(max_cycles=2, outdir=str(tmp_path), verbose=False, profile=str(tmp_path / "p.json"))
    assert n == 2
    prof = json.loads((tmp_path / "p.json").read_text())
    ph = prof["phases"]
    assert ph["steps"]["calls"] == 40 and ph["sync"]["calls"] == 2 and ph["download"]["calls"] == 2
    assert ph["outputs.checkpoint"]["calls"] == 2
    assert prof["iterations"] == 40 and prof["grid"] == [80, 30] and prof["mcells_it_per_s"] > 0
    assert set(sim.solver.phase_times) >= {"steps", "sync", "download", "outputs"}


def test_kill_fault_then_restart_resumes(hf, tmp_path):
    _deck(tmp_path)
    r = _cli(tmp_path, "--cycles", "3", "--fault-inject", "step:45,kind:kill")
    assert r.returncode == -signal.SIGKILL, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    meta = json.loads((tmp_path / (STEM + ".hf2d.meta")).read_text())
    assert meta["iteration"] == 40     # two completed cycles before the kill
    r = _cli(tmp_path, "--cycles", "1")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    meta = json.loads((tmp_path / (STEM + ".hf2d.meta")).read_text())
    assert meta["iteration"] == 60     # resumed from the checkpoint, one more cycle


def test_cli_nan_fault_exit_code(hf, tmp_path):
    _deck(tmp_path)
    r = _cli(tmp_path, "--cycles", "2", "--fault-inject", "step:7")
    assert r.returncode == 3, r.stdout[-2000:] + r.stderr[-2000:]
    assert "unstability" in r.stderr
    assert (tmp_path / (STEM + "-err.plt")).exists()


def test_cond_names(native):
    assert native.cond_names(0) == "CT_NO_COND_2D"
    assert native.cond_names(0x02 | 0x080000000) == "CT_U_CONST_2D | CT_NODE_IS_SET_2D"
    assert "TCT_k_eps_Model_2D" in native.turb_cond_names(0x0400)
