"""FP32 build option (the reference's FP_OPTS = -DFP=double,
gcc.compiler:22, switchable to float): the host CLI compiled with
real = float (bin/hf2d_cpu_fp32, _build.build_fp32).  The deck, its tables and
the geometry stay in double (cell indices of contour points are formed from
the deck's values, as in the FP64 build); the flow state, fluxes and steppers
run in float.  Checked against the FP64 CLI on the same deck: the Tecplot
fields agree to float rounding away from discontinuities (median relative
difference <= 1e-4, y+ the loosest) and within a few percent at the shocks, and the float
record is written (.hf2d of (MaxX * MaxY) 680-byte records)."""
import glob
import os
import subprocess

import numpy as np
import pytest

from openhyperflow2d_amd.models import decks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FP64 = os.path.join(ROOT, "openhyperflow2d_amd", "bin", "hf2d_cpu")

DECKS = {
    "wedge_euler": (lambda: decks.wedge15(120, 40, nmax=200, nout=100), (120, 40)),
    "wedge_keps": (lambda: decks.wedge15(120, 40, navier_stokes=True, turbulence=4, nmax=200, nout=100), (120, 40)),
    "scramjet_sst_mech": (lambda: decks.scramjet(150, 20, nmax=60, nout=30), (150, 20)),
    "triple_point_3gas": (lambda: decks.triple_point(84, 36, nmax=100, nout=50), (84, 36)),
}


@pytest.fixture(scope="module")
def fp32_cli(hf):
    from openhyperflow2d_amd import _build

    return _build.build_fp32()


def _plt(d):
    rows = []
    for line in open(glob.glob(os.path.join(d, "tp-*.plt"))[0]):
        try:
            rows.append([float(x) for x in line.split()])
        except ValueError:
            pass
    n = max(len(r) for r in rows)
    return np.array([r for r in rows if len(r) == n])


@pytest.mark.parametrize("name", sorted(DECKS))
def test_fp32_cli_tracks_the_fp64_cli(fp32_cli, tmp_path, name):
    make, (nx, ny) = DECKS[name]
    text = make()
    out = {}
    for tag, exe in (("fp64", FP64), ("fp32", fp32_cli)):
        d = tmp_path / tag
        d.mkdir()
        (d / "d.dat").write_text(text)
        r = subprocess.run([exe, "--backend", "cpu", "--cycles", "1", "d.dat"], cwd=d, capture_output=True, text=True,
                           timeout=600)
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


def test_fp32_gpu_cli_is_built():
    """The default build also links the FP32 GPU CLI (bin/hf2d_fp32, every
    device kernel with real = float; tests/test_gpu_fp32.py runs it)."""
    from openhyperflow2d_amd import _build

    exe = _build.gpu_fp32_path()
    assert os.path.isfile(exe) and os.access(exe, os.X_OK)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)   # (no deck: the banner)
    assert "(FP32)" in r.stdout, r.stdout[-500:] + r.stderr[-500:]
