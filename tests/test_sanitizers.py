"""Host sanitizers: the CPU CLI built with AddressSanitizer +
UndefinedBehaviorSanitizer (bin/hf2d_cpu_asan, _build.build_asan) runs the
pre-processor, the Jacobi and reference-order steppers, outputs and the
checkpoint of viscous/turbulent, reacting and inviscid decks without a report."""
import os
import subprocess

import pytest

from openhyperflow2d_amd.models import decks

DECKS = {
    "wedge_keps": lambda: decks.wedge15(80, 30, navier_stokes=True, turbulence=4, nmax=12, nout=6),
    "scramjet_sst_h2": lambda: decks.scramjet(150, 20, nmax=12, nout=6, mechanism=None),
    # mechanism mode (species block, kinetics, species checkpoint); no reference-order backend
    "scramjet_sst_mech": lambda: decks.scramjet(150, 20, nmax=12, nout=6),
    "triple_point_euler": lambda: decks.triple_point(84, 36, nmax=12, nout=6),
}


@pytest.fixture(scope="module")
def asan_cli(hf):
    from openhyperflow2d_amd import _build

    return _build.build_asan()


@pytest.mark.parametrize("backend", ["cpu", "ref"])
@pytest.mark.parametrize("name", sorted(DECKS))
def test_asan_ubsan_clean(asan_cli, tmp_path, name, backend):
    if backend == "ref" and name.endswith("mech"):
        pytest.skip("the reference order has no mechanism mode")
    text = DECKS[name]()
    text = decks.set_key(text, "MonitorIndex", 1)
    text = decks.set_key(text, "ExitMonitorValue", 1e-30)
    (tmp_path / "d.dat").write_text(text)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([asan_cli, "--backend", backend, "--cycles", "2", "d.dat"], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert "Computation finished" in r.stdout


def test_asan_ubsan_clean_strip_ranks(asan_cli, tmp_path):
    """Four native CPU strip ranks (TCP rendezvous) of the outputs deck of the
    virtual-rank driver test -- trimmed host fields (strip + ghost columns),
    per-strip Tecplot rows and checkpoint slabs, folded cut / Cx / heat-flux
    integrals -- without an AddressSanitizer or UBSan report: no output path
    reads a non-resident column (Field::at is unchecked)."""
    import sys

    from tests.conftest import ROOT

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_strips import _outputs_deck

    (tmp_path / "W.dat").write_text(_outputs_deck())
    sh = os.path.join(ROOT, "openhyperflow2d_amd", "bin", "OpenHyperFLOW2D.sh")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", HF2D_BIN=asan_cli, HF2D_MASTER_PORT="29761")
    r = subprocess.run(["timeout", "-k", "10", "500", sh, "W", "4", "--backend", "cpu", "--cycles", "2"], cwd=tmp_path,
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert "Computation finished" in r.stdout
