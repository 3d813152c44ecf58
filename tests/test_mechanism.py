"""Detailed finite-rate chemistry (mechanism mode, CRM_ARRENIUS slot): data,
thermodynamics, the kinetics operator and its coupling into the time step.

No kinetics package exists in this image: the oracles are the repo's own
independent NumPy/SciPy code (openhyperflow2d_amd/ops/mechanism.py), so every
result here is "parity unpinned" against Cantera/CHEMKIN.  The thermo data are
pinned to literature values (formation enthalpies, standard entropies)."""
import os

import numpy as np
import pytest

from openhyperflow2d_amd.models import decks
from openhyperflow2d_amd.ops import mechanism as M
from tests.conftest import ROOT

MECH_FILE = os.path.join(ROOT, "openhyperflow2d_amd", "data", "h2_air_li2004.mech")
INC_FILE = os.path.join(ROOT, "openhyperflow2d_amd", "csrc", "core", "mech_builtin.inc")


def test_builtin_file_and_embedded_copy_match_python_data():
    txt = M.h2_air_li2004().to_text()
    assert open(MECH_FILE).read() == txt
    inc = open(INC_FILE).read()
    assert 'R"MECH(' + txt + ')MECH"' in inc


def test_nasa7_thermo_literature_values_and_continuity():
    m = M.h2_air_li2004()
    # standard formation enthalpy (kJ/mol) and entropy (J/mol/K) at 298.15 K
    ref = {"H2": (0.0, 130.68), "O2": (0.0, 205.15), "H2O": (-241.83, 188.83), "H": (218.0, 114.72),
           "O": (249.17, 161.06), "OH": (39.35, 183.74), "N2": (0.0, 191.61)}
    T = np.array(298.15)
    h = M.h_RT(m, T) * M.RU * 298.15 / 1e3
    s = M.s_R(m, T) * M.RU
    for sp, (hf, s0) in ref.items():
        k = m.index(sp)
        assert abs(h[k] - hf) < 0.05, sp
        assert abs(s[k] - s0) < 0.15, sp
    for sp in m.species:
        lo, hi = np.array(sp.low), np.array(sp.high)
        T = sp.Tmid
        cp = lambda a: a[0] + T * (a[1] + T * (a[2] + T * (a[3] + T * a[4])))
        assert abs(cp(lo) - cp(hi)) < 2e-6 * cp(hi), sp.name


def test_mechanism_rejects_bad_input():
    m = M.h2_air_li2004()
    with pytest.raises(ValueError):
        M.Mechanism("x", m.species, [M.Reaction({"H2": 0.5, "O2": 1}, {"H2O": 1}, 1.0)])
    bad = [M.Species("A", -1.0, 200, 1000, 3000, [1] * 7, [1] * 7)]
    with pytest.raises(ValueError):
        M.Mechanism("x", bad, [])
    txt = m.to_text().replace("H2 + OH <=> H2O + H", "H2 + OH <=> H2O + Xx")
    with pytest.raises(ValueError):
        M.Mechanism.from_text(txt)


def test_native_thermo_matches_numpy(native):
    m = M.h2_air_li2004()
    Y = np.array([0.028, 0.22, 0.01, 1e-4, 2e-4, 3e-3, 1e-5, 1e-6, 0.0])
    Y[-1] = 1 - Y.sum()
    for T in (300.0, 999.0, 1000.0, 1800.0, 3200.0):
        d = native.mech_thermo_host("h2_air_li2004", list(Y), T)
        assert d["e"] == pytest.approx(M.mixture_e(m, Y, T), rel=1e-13)
        assert d["cv"] == pytest.approx(M.mixture_cv(m, Y, T), rel=1e-13)
        assert d["T_from_e"] == pytest.approx(T, rel=1e-10)
        mu = (Y * M.viscosity(m, T)).sum()
        assert d["mu"] == pytest.approx(mu, rel=2e-3)   # 50 K uniform table vs exact


def test_thermo_below_the_fit_range_extrapolates_at_constant_cp(native):
    """Below T_LO = 200 K (the NASA-7 fits' lower limit) every species runs at
    constant cp: e is linear in T with the cv of 200 K, continuous at 200 K,
    the Newton recovers T down to the 20 K floor (the under-expanded fuel jet
    of the scramjet deck cools to ~105 K), and the NumPy oracle agrees."""
    m = M.h2_air_li2004()
    Y = np.array([0.5, 0.1, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0])
    Y[-1] = 1 - Y.sum()
    ref = native.mech_thermo_host("h2_air_li2004", list(Y), 200.0)
    for T in (199.999, 150.0, 105.0, 60.0, 25.0):
        d = native.mech_thermo_host("h2_air_li2004", list(Y), T)
        assert d["cv"] == ref["cv"]
        assert d["e"] == pytest.approx(ref["e"] + ref["cv"] * (T - 200.0), rel=1e-13)
        assert d["e"] == pytest.approx(M.mixture_e(m, Y, T), rel=1e-12)
        assert d["cv"] == pytest.approx(M.mixture_cv(m, Y, T), rel=1e-13)
        assert d["T_from_e"] == pytest.approx(T, rel=1e-10)
    # continuity of the oracle's h and s at T_LO (the Gibbs energies of the kinetics)
    for f in (M.h_RT, M.s_R, M.cp_R):
        a, b = f(m, np.array(200.0)), f(m, np.array(200.0 - 1e-7))
        np.testing.assert_allclose(a, b, rtol=1e-8)


def _states(m, n, seed=1):
    rng = np.random.default_rng(seed)
    Y = rng.random((m.ns, n)) * np.array([0.03, 0.2, 0.1, 1e-3, 1e-3, 3e-3, 1e-4, 1e-5, 0.0])[:, None]
    Y[-1] = 1 - Y[:-1].sum(0)
    T = 1000 + 1500 * rng.random(n)
    rho = 0.1 + 0.5 * rng.random(n)
    return rho * Y, rho, M.mixture_e(m, Y.T, T), T


def test_host_kinetics_operator_matches_numpy_reference(native):
    m = M.h2_air_li2004()
    rhoY, rho, e, T = _states(m, 96)
    for dt, nsub in ((1e-8, 1), (2e-7, 2), (5e-6, 4)):
        a, Ta = M.point_implicit_step(m, rhoY, rho, e, T, dt, nsub)
        b, Tb = native.mech_chem_host("h2_air_li2004", rhoY, rho, e, T, dt, nsub)
        # per-species error relative to that species' own increment
        # (the inert bath gas, last, changes by rounding only: checked absolutely)
        inc = np.abs(a - rhoY).max(1)[:-1]
        assert (np.abs(a - b).max(1)[:-1] / inc).max() < 1e-9, (dt, nsub)
        assert np.abs(a[-1] - b[-1]).max() < 1e-14 * np.abs(rhoY[-1]).max()
        assert np.abs(Ta - Tb).max() < 1e-8
        # mass conserved
        assert np.abs(b.sum(0) - rho).max() < 1e-12 * rho.max()


def test_fine_substep_operator_converges_to_scipy_bdf():
    """Constant-volume ignition: the point-implicit operator with small
    substeps reproduces the stiff BDF solution (ignition delay within 1 %)."""
    m = M.h2_air_li2004()
    Y0 = M.premixed_Y(m, 1.0)
    T0, p0 = 1200.0, M.P_ATM
    rho0 = p0 / (M.RU * T0 * (Y0 / m.W).sum())
    e0 = M.mixture_e(m, Y0, T0)
    from scipy.integrate import solve_ivp

    dt, nst = 1e-7, 1000
    rhoY, T = (rho0 * Y0)[:, None], np.array([T0])
    ts, Ts = [0.0], [T0]
    for k in range(nst):
        rhoY, T = M.point_implicit_step(m, rhoY, np.array([rho0]), np.array([e0]), T, dt, 2)
        ts.append((k + 1) * dt)
        Ts.append(T[0])
    ts, Ts = np.array(ts), np.array(Ts)
    sol = solve_ivp(M.reactor_rhs(m, "cv", rho0, p0), (0, ts[-1]), np.concatenate([Y0, [T0]]), method="BDF",
                    rtol=1e-10, atol=1e-14, t_eval=ts)
    Tref = sol.y[-1]
    tau = ts[np.argmax(np.gradient(Ts, ts))]
    tau_ref = ts[np.argmax(np.gradient(Tref, ts))]
    assert abs(tau - tau_ref) / tau_ref < 0.01
    assert abs(Ts[-1] - Tref[-1]) < 2.0


def _reactor_deck(T0=1200.0, nsub=2):
    t = decks.reactor0d(8, 8, T=T0, p=101325.0)
    t = decks.set_key(t, "Mechanism", "h2_air_li2004")
    return decks.set_key(t, "ChemSubsteps", nsub)


def test_coupled_0d_reactor_matches_scipy_constant_volume(hf):
    """The full time step (transport predictor, kinetics, Newton T recovery)
    on a closed box at rest is a constant-volume reactor."""
    from scipy.integrate import solve_ivp

    T0 = 1200.0
    sim = hf.Simulation(_reactor_deck(T0), "cpu")
    assert sim.case.mech_mode and sim.case.mech_species[-1] == "N2"
    ts, Ts = [0.0], [T0]
    for _ in range(60):
        sim.step(20)
        ts.append(sim.summary()["time"])
        Ts.append(sim.field("T")[3, 3])
    ts, Ts = np.array(ts), np.array(Ts)
    m = M.h2_air_li2004()
    Y = np.array([sim.field("Y:%s" % s)[3, 3] for s in m.names])
    Y0 = np.zeros(m.ns)
    r = 2 * 2.016 / 31.999
    yox = decks.AIR_Y_O2 / (1 + r * decks.AIR_Y_O2)
    Y0[m.index("H2")], Y0[m.index("O2")] = r * yox, yox
    Y0[-1] = 1 - Y0.sum()
    rho0 = 101325.0 / (M.RU * T0 * (Y0 / m.W).sum())
    sol = solve_ivp(M.reactor_rhs(m, "cv", rho0, 101325.0), (0, ts[-1]), np.concatenate([Y0, [T0]]), method="BDF",
                    rtol=1e-10, atol=1e-14, t_eval=ts)
    Tref = sol.y[-1]
    tau = ts[np.argmax(np.gradient(Ts, ts))]
    tau_ref = ts[np.argmax(np.gradient(Tref, ts))]
    assert abs(tau - tau_ref) <= 1.01 * (ts[1] - ts[0])
    assert abs(Ts[-1] - Tref[-1]) < 1.0
    assert abs(Y.sum() - 1) < 1e-12
    assert np.allclose(Y, sol.y[:-1, -1], atol=2e-4)


def test_species_checkpoint_sidecar_restart(hf, tmp_path):
    t = decks.set_key(_reactor_deck(1500.0), "Nmax", 40)
    sim = hf.Simulation(t, "cpu", workdir=str(tmp_path))
    sim.run(max_cycles=1, outdir=str(tmp_path), verbose=False)
    sp = tmp_path / "Reactor0D.hf2d.species"
    assert sp.exists()
    raw = sp.read_bytes()
    assert raw[:8] == b"HF2DSPC2"
    assert os.path.getsize(tmp_path / "Reactor0D.hf2d") == 8 * 8 * 1248
    a = sim.field("Y:OH")
    sim2 = hf.Simulation(t, "cpu", workdir=str(tmp_path), use_checkpoint=True)
    assert sim2.case.mech_mode
    assert np.array_equal(sim2.field("Y:OH"), a)
    assert np.array_equal(sim2.field("T"), sim.field("T"))
    os.remove(sp)
    with pytest.raises(Exception):
        hf.Simulation(t, "cpu", workdir=str(tmp_path), use_checkpoint=True)
