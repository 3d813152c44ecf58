"""Mechanism mode on the MI355X: the compiled-mechanism kinetics kernel
(chem_fast.hip), the runtime-data kernels and the coupled SK_MECH time step
against the host implementation (core/mechanism.hpp, itself pinned to the
independent NumPy/SciPy oracle in tests/test_mechanism.py).  The transport
part of the step is bitwise equal between host and device; the kinetics use
the device exp/log, so tolerances are at the rounding level of those."""
import numpy as np
import pytest

from openhyperflow2d_amd.models import decks
from openhyperflow2d_amd.ops import mechanism as M

pytestmark = pytest.mark.gpu


def _states(m, n, seed=3):
    rng = np.random.default_rng(seed)
    Y = rng.random((m.ns, n)) * np.array([0.03, 0.2, 0.1, 1e-3, 1e-3, 3e-3, 1e-4, 1e-5, 0.0])[:, None]
    Y[-1] = 1 - Y[:-1].sum(0)
    T = 900 + 1800 * rng.random(n)
    rho = 0.05 + 0.5 * rng.random(n)
    return rho * Y, rho, M.mixture_e(m, Y.T, T), T


def _incr_err(got, ref, y0):
    inc = np.abs(ref - y0).max(1)[:-1]
    return float((np.abs(got - ref).max(1)[:-1] / inc).max())


@pytest.mark.parametrize("dt,nsub", [(1e-8, 1), (1e-7, 2), (2e-6, 4)])
def test_chem_fast_kernel_matches_host(gpu, dt, nsub):
    nat = gpu.native()
    m = M.h2_air_li2004()
    rhoY, rho, e, T = _states(m, 5000)
    ref, Tref = nat.mech_chem_host("h2_air_li2004", rhoY, rho, e, T, dt, nsub)
    got, Tg, ms = nat.chem_fast_run("h2_air_li2004", rhoY, rho, e, T, dt, nsub, 1)
    assert _incr_err(got, ref, rhoY) < 1e-9
    assert np.abs(Tg - Tref).max() < 1e-8
    assert np.abs(got.sum(0) - rho).max() < 1e-12 * rho.max()


def _reactor(T0=1200.0):
    return decks.with_mechanism(decks.reactor0d(8, 8, T=T0, p=101325.0), substeps=2)


@pytest.mark.parametrize("fast", [True, False])
def test_gpu_reactor_matches_cpu(gpu, fast):
    text = _reactor()
    g = gpu.Simulation(text, "gpu")
    g.solver.chem_fast = fast
    assert g.solver.chem_fast_ok
    c = gpu.Simulation(text, "cpu")
    for _ in range(4):
        g.step(200)
        c.step(200)
    Tg, Tc = g.field("T"), c.field("T")
    assert Tc.max() > 2500.0   # ignited
    assert np.abs(Tg - Tc).max() < 1e-6 * Tc.max()
    for s in ("H2", "O2", "H2O", "OH", "H"):
        a, b = g.field("Y:" + s), c.field("Y:" + s)
        assert np.abs(a - b).max() < 1e-9, s


def test_gpu_scramjet_mech_matches_cpu(gpu):
    text = decks.scramjet(150, 50, nmax=10 ** 6, nout=10 ** 5)
    g = gpu.Simulation(text, "gpu")
    c = gpu.Simulation(text, "cpu")
    assert g.case.mech_mode and g.solver.chem_fast_ok
    g.step(40, residual=True)
    c.step(40, residual=True)
    for f in ("rho", "U", "V", "p", "T", "Y:H2", "Y:O2", "Y:OH"):
        a, b = g.field(f), c.field(f)
        assert np.abs(a - b).max() <= 1e-9 * max(np.abs(b).max(), 1e-30), f
    assert abs(g.summary()["dt"] - c.summary()["dt"]) <= 1e-12 * c.summary()["dt"]


def test_gpu_mech_transport_bitwise_without_kinetics(gpu):
    """With ChemTmin above every temperature the kinetics copy through and the
    SK_MECH transport (species block, Newton T, mixture transport) must equal
    the host stepper bit for bit."""
    text = decks.with_mechanism(decks.scramjet(150, 50, nmax=10 ** 6, nout=10 ** 5), tmin=1e9)
    g = gpu.Simulation(text, "gpu")
    c = gpu.Simulation(text, "cpu")
    g.step(30, residual=True)
    c.step(30, residual=True)
    for f in ("rho", "U", "V", "p", "T", "mu", "Y:H2", "Y:N2"):
        assert np.array_equal(g.field(f), c.field(f)), f


@pytest.mark.parametrize("deck", ["reactor", "scramjet"])
def test_compacted_kinetics_match_per_cell_kernel(gpu, deck):
    """hf2d_chem_fast over a compacted list of the reacting cells (mark pass +
    dense pass) == the one-cell-per-lane kernel over the grid, bit for bit."""
    from openhyperflow2d_amd.models import decks

    if deck == "reactor":
        text = decks.with_mechanism(decks.reactor0d(16, 16, T=1300.0, p=101325.0), substeps=2)
        n = 200
    else:
        text = decks.scramjet(600, 60, nmax=10 ** 9, nout=10 ** 8)
        n = 300
    a = gpu.Simulation(text, "gpu")
    b = gpu.Simulation(text, "gpu")
    b.solver.chem_compact = False
    a.step(n)
    b.step(n)
    assert a.solver.chem_kernel_used == b.solver.chem_kernel_used == "hf2d_chem_fast"
    np.testing.assert_array_equal(a.field("T"), b.field("T"))
    for s in ("H2", "O2", "H2O", "OH", "N2"):
        np.testing.assert_array_equal(a.field("Y:" + s), b.field("Y:" + s), err_msg=s)


def test_rtc_kernel_equals_compiled_kernel(gpu):
    """The hiprtc-specialised kernel (generated mechanism struct + the shared
    chem_fast_dev.hpp bodies) == the kernel compiled into the library for the
    same mechanism, bit for bit."""
    from tests.test_chem_rtc import MECH

    nat = gpu.native()
    m = M.h2_air_li2004()
    rhoY, rho, e, T = _states(m, 5000)
    a, Ta, _ = nat.chem_fast_run("h2_air_li2004", rhoY, rho, e, T, 2e-7, 2, 1)
    b, Tb, _, _ = nat.chem_rtc_run(open(MECH).read(), rhoY, rho, e, T, 2e-7, 2, 1)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(Ta, Tb)


def test_file_mechanism_runs_the_rtc_kernel_and_matches_cpu(gpu, tmp_path):
    """A mechanism without built-in kernels (the Li et al. file with a scaled
    chain-branching rate) runs hf2d_rtc_chem in the coupled step and matches
    the host integrator like the built-in does."""
    from tests.test_chem_rtc import modified_mechanism

    path = tmp_path / "h2_air_mod.mech"
    path.write_text(modified_mechanism())
    text = decks.with_mechanism(decks.scramjet(150, 50, nmax=10 ** 6, nout=10 ** 5), mechanism=str(path), substeps=2,
                                tmin=250.0)
    g = gpu.Simulation(text, "gpu")
    c = gpu.Simulation(text, "cpu")
    assert not g.solver.chem_fast_ok and g.solver.chem_rtc_ok, g.solver.chem_rtc_why
    g.step(40, residual=True)
    c.step(40, residual=True)
    assert g.solver.chem_kernel_used == "hf2d_rtc_chem"
    for f in ("rho", "U", "V", "p", "T", "Y:H2", "Y:O2", "Y:OH"):
        a, b = g.field(f), c.field(f)
        assert np.abs(a - b).max() <= 1e-9 * max(np.abs(b).max(), 1e-30), f


@pytest.mark.parametrize("deck", ["sst", "sst_graphs", "laminar", "hot", "sst_ti12"])
def test_lean_mech_equals_split(gpu, deck):
    """Lean mechanism step (hip/lean_mech.hpp: flow, turbulence and species
    fluxes recomputed in the LDS tile, the Newton T once per cell and step,
    kinetics and the state of the reacting cells over a list) == the split
    predict + kinetics + fill kernels on every field, dt and time, across
    entry / materialize / re-entry transitions (residual steps, downloads
    between windows, graph windows).  'hot': ChemTmin 200 K, so every active
    cell goes through the kinetics list and hf2d_lnm_hot."""
    if deck == "laminar":
        text = decks.scramjet(300, 48, nmax=10 ** 6, nout=10 ** 5, turbulence=0)
    elif deck == "hot":
        text = decks.with_mechanism(decks.scramjet(300, 48, nmax=10 ** 6, nout=10 ** 5), tmin=200.0)
    else:
        text = decks.scramjet(300, 48, nmax=10 ** 6, nout=10 ** 5)
    a = gpu.Simulation(text, "gpu")
    b = gpu.Simulation(text, "gpu")
    b.solver.lean_mech = False
    if deck.endswith("_ti12"):   # 12 x 16 tiles: ring cells on their own threads
        a.solver.lnm_ti = 12
    graphs = deck.endswith("_graphs")
    if not graphs:
        a.solver.use_graph = b.solver.use_graph = False
    assert a.solver.lnm_ok, a.solver.lnm_why
    assert a.solver.lnm_turb == (0 if deck == "laminar" else 3)
    sched = [(4, True), (30, False), (6, True), (19, False)] if not graphs else [(40, False), (13, True), (61, False)]
    for n, res in sched:
        a.step(n, residual=res)
        b.step(n, residual=res)
        assert a.summary()["dt"] == b.summary()["dt"]
    assert a.solver.lnm_steps > 0
    assert b.solver.lnm_steps == 0
    assert a.solver.chem_kernel_used == b.solver.chem_kernel_used
    assert a.summary()["time"] == b.summary()["time"]
    np.testing.assert_allclose(a.summary()["rms"], b.summary()["rms"], rtol=1e-12, atol=0)
    for f in ("rho", "U", "V", "p", "T", "k", "R", "CP", "mu", "lam", "mu_t", "S7", "S8", "Y:H2", "Y:O2", "Y:OH",
              "Y:H2O", "Y:N2"):
        np.testing.assert_array_equal(a.field(f), b.field(f), err_msg=f)
    ra = np.frombuffer(a.records(), dtype=np.float64).reshape(-1, 156).copy()
    rb = np.frombuffer(b.records(), dtype=np.float64).reshape(-1, 156).copy()
    assert (np.isnan(ra) == np.isnan(rb)).all()
    ra[np.isnan(ra)] = 0
    rb[np.isnan(rb)] = 0
    np.testing.assert_array_equal(ra.view(np.uint64), rb.view(np.uint64))


def test_lnm_phase_timing_is_measurement_only(gpu):
    """DeviceSolver.lnm_timing (hipEvents around the tile kernel, the
    kinetics and the reacting-cell state kernel; tools/scramjet_phases.py)
    times every lean mechanism step and leaves the results bit for bit."""
    text = decks.with_mechanism(decks.scramjet(300, 48, nmax=10 ** 6, nout=10 ** 5), tmin=200.0)
    a = gpu.Simulation(text, "gpu")
    b = gpu.Simulation(text, "gpu")
    a.solver.use_graph = b.solver.use_graph = False
    a.solver.lnm_timing = True
    a.step(20)
    b.step(20)
    tile, chem, state, n = a.solver.lnm_phase_ms
    assert n == a.solver.lnm_steps > 0
    assert tile > 0 and chem > 0 and state > 0
    assert a.summary()["dt"] == b.summary()["dt"]
    for f in ("rho", "U", "T", "Y:H2", "Y:OH"):
        np.testing.assert_array_equal(a.field(f), b.field(f), err_msg=f)
