"""FP32 build of the GPU solver (the reference's -DFP=float for
the whole program): bin/hf2d_fp32 is the native CLI with every device kernel
compiled for real = float (_build.gpu_fp32_path; the finite-rate kinetics
kernels stay FP64-only and the mechanism mode is refused with a message).
Checked against the FP64 GPU CLI on the same decks: the Tecplot fields agree
to float rounding away from discontinuities and within a few percent at the
shocks, and the 680-byte float record is written."""
import glob
import os
import subprocess

import numpy as np
import pytest

from openhyperflow2d_amd.models import decks

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "openhyperflow2d_amd", "bin")

DECKS = {
    "wedge_euler": (lambda: decks.wedge15(240, 80, nmax=400, nout=200), (240, 80)),
    "wedge_keps": (lambda: decks.wedge15(240, 80, navier_stokes=True, turbulence=4, nmax=300, nout=150), (240, 80)),
    "wedge_laminar_ns": (lambda: decks.wedge15(240, 80, navier_stokes=True, turbulence=0, nmax=300, nout=150),
                         (240, 80)),
    "triple_point_3gas": (lambda: decks.triple_point(168, 72, nmax=200, nout=100), (168, 72)),
}


def _plt(d):
    rows = []
    for line in open(glob.glob(os.path.join(d, "tp-*.plt"))[0]):
        try:
            rows.append([float(x) for x in line.split()])
        except ValueError:
            pass
    n = max(len(r) for r in rows)
    return np.array([r for r in rows if len(r) == n])


def _run(exe, d, text):
    (d / "d.dat").write_text(text)
    return subprocess.run([exe, "--backend", "gpu", "--cycles", "1", "d.dat"], cwd=d, capture_output=True, text=True,
                          timeout=300)


@pytest.mark.parametrize("name", sorted(DECKS))
def test_fp32_gpu_cli_tracks_the_fp64_gpu_cli(gpu, tmp_path, name):
    make, (nx, ny) = DECKS[name]
    text = make()
    out = {}
    for tag, exe in (("fp64", "hf2d"), ("fp32", "hf2d_fp32")):
        d = tmp_path / tag
        d.mkdir()
        r = _run(os.path.join(BIN, exe), d, text)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        assert "Computation finished" in r.stdout
        out[tag] = _plt(str(d))
    a, b = out["fp64"], out["fp32"]
    assert a.shape == b.shape and np.isfinite(b).all()
    rel = np.abs(a - b) / np.maximum(np.abs(a).max(axis=0), 1e-30)
    assert np.median(rel, axis=0).max() <= 1e-4, np.median(rel, axis=0)
    assert rel.max() < 0.05, rel.max(axis=0)
    assert rel.max() > 0.0   # it is a float build
    rec32 = glob.glob(str(tmp_path / "fp32" / "*.hf2d"))[0]
    assert os.path.getsize(rec32) == nx * ny * 680


def test_fp32_gpu_cli_refuses_the_mechanism_mode(gpu, tmp_path):
    """The kinetics kernels work on FP64 state only: a runtime-mechanism deck
    stops with a message instead of running a mixed-precision step."""
    r = _run(os.path.join(BIN, "hf2d_fp32"), tmp_path, decks.scramjet(150, 20, nmax=60, nout=30))
    assert r.returncode != 0
    assert "FP32 build" in r.stdout + r.stderr
