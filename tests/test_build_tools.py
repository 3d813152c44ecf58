"""Build-system and plot-helper coverage (Makefile/.compiler fragments,
viewplt.sh, view_RMS.sh).  The CMake test only configures (the full build is exercised by
_build.py through the other tests)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("cmake") is None or not os.path.isdir("/opt/rocm"), reason="cmake/ROCm missing")
def test_cmake_configures(tmp_path):
    r = subprocess.run(["cmake", "-S", ROOT, "-B", str(tmp_path / "b"), "-G", "Ninja"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    ninja = (tmp_path / "b" / "build.ninja").read_text()
    for tgt in ("_hf2d", "hf2d_cpu", "hf2d"):
        assert f"build {tgt}" in ninja
    assert "--offload-arch=gfx950" in ninja


def test_plot_helpers_write_gnuplot_scripts(native, tmp_path):
    deck = os.path.join(ROOT, "tests", "fixtures", "ref", "wedge15_200x40_euler", "deck.dat")
    shutil.copy(deck, tmp_path / "deck.dat")
    cli = os.path.join(ROOT, "openhyperflow2d_amd", "bin", "hf2d_cpu")
    r = subprocess.run([cli, "deck.dat"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    plt = tmp_path / "Wedge15_200x40.plt"
    env = dict(os.environ, PATH="/usr/bin:/bin")   # no gnuplot: scripts only
    r = subprocess.run([os.path.join(ROOT, "tools", "viewplt.sh"), str(plt), "Mach"], capture_output=True,
                       text=True, env=env)
    assert r.returncode == 0, r.stderr
    gp = (tmp_path / "Wedge15_200x40.plt.Mach.gp").read_text()
    assert "using 1:2:13" in gp   # Mach is the 13th variable
    rows = (tmp_path / "Wedge15_200x40.plt.Mach.dat").read_text().split("\n\n")
    assert len(rows) == 40 and all(len(b.strip().splitlines()) == 200 for b in rows)
    r = subprocess.run([os.path.join(ROOT, "tools", "view_RMS.sh"), str(tmp_path / "RMS-Wedge15_200x40.plt")],
                       capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "RMS-Wedge15_200x40.plt.gp").read_text().count("with lines") == 9
