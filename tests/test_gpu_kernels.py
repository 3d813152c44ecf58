"""GPU numerics: the HIP kernels against the CPU Jacobi stepper (which runs the
same per-cell code on the host) and against the reference-order oracle."""
import numpy as np
import pytest

from openhyperflow2d_amd.models import decks

pytestmark = pytest.mark.gpu

FIELDS = ["rho", "U", "V", "p", "T"]


def _run_pair(hf, text, steps, fused=True):
    g = hf.Simulation(text, "gpu", fused=fused)
    c = hf.Simulation(text, "cpu")
    g.step(steps, residual=True)
    c.step(steps, residual=True)
    return g, c


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


@pytest.mark.parametrize("fused", [True, False])
def test_wedge_euler_gpu_matches_cpu(gpu, fused):
    text = decks.wedge15(200, 40, nmax=1000, nout=10)
    g, c = _run_pair(gpu, text, 50, fused)
    for f in FIELDS:
        assert _rel(g.field(f), c.field(f)) < 1e-11, f
    sg, sc = g.summary(), c.summary()
    assert abs(sg["dt"] - sc["dt"]) <= 1e-12 * sc["dt"]
    assert abs(sg["time"] - sc["time"]) <= 1e-10 * sc["time"]
    np.testing.assert_allclose(sg["rms"], sc["rms"], rtol=1e-8, atol=1e-300)


def test_wedge_ns_keps_gpu_matches_cpu(gpu):
    text = decks.wedge15(200, 60, navier_stokes=True, turbulence=4, nmax=1000, nout=10)
    g, c = _run_pair(gpu, text, 30)
    for f in FIELDS + ["mu_t"]:
        assert _rel(g.field(f), c.field(f)) < 1e-9, f


def test_reference_deck_wedge_keps_wall_heat(gpu):
    from tests.conftest import read_deck

    text = decks.set_key(read_deck("Wedge.dat"), "Nmax", 100)
    g, c = _run_pair(gpu, text, 10)
    for f in FIELDS:
        assert _rel(g.field(f), c.field(f)) < 1e-9, f


def test_step_euler_gpu(gpu):
    from tests.conftest import read_deck

    g, c = _run_pair(gpu, read_deck("Step.dat"), 20)
    for f in FIELDS:
        assert _rel(g.field(f), c.field(f)) < 1e-11, f


def test_euler_gpu_equals_reference_order(gpu):
    """For Euler decks without Neumann/Cauchy chains the Jacobi GPU step equals
    the reference in-place sweep bit-for-bit at the field level."""
    from tests.conftest import read_deck

    text = decks.set_key(read_deck("ObliqueShock.dat"), "Nmax", 100)
    g = gpu.Simulation(text, "gpu")
    r = gpu.Simulation(text, "ref")
    g.step(40)
    r.step(40)
    for f in FIELDS:
        assert _rel(g.field(f), r.field(f)) < 1e-12, f
