"""K12 kinetics kernels as standalone operators: the runtime-mechanism MFMA
kernel (chem_mech.hip) and the compiled-mechanism kernel (chem_fast.hip)
against the independent NumPy FP64 oracle (ops/mechanism.point_implicit_step).
The reference's CRM_ARRENIUS slot is empty (hyper_flow_bound.hpp:37-42): parity
unpinned, no external kinetics package in the image."""
import numpy as np
import pytest

from openhyperflow2d_amd.ops import chemistry as ch
from openhyperflow2d_amd.ops import mechanism as M


def _random_mech(ns, nr, seed, reversible=True):
    """Random mechanism over species of equal molar mass (so a step conserves
    mass when its coefficient sums agree), reversible / irreversible / third-body
    steps of orders 1..3."""
    rng = np.random.default_rng(seed)
    n2 = M.h2_air_li2004().species[-1]
    sp = []
    for i in range(ns):
        # N2-like thermo with the formation enthalpy / entropy constants shifted by
        # up to +-2000 K / +-2: moderate equilibrium constants and heat release
        lo, hi = list(n2.low), list(n2.high)
        dh, ds = rng.uniform(-2000, 2000), rng.uniform(-2, 2)
        lo[5] += dh
        hi[5] += dh
        lo[6] += ds
        hi[6] += ds
        sp.append(M.Species("S%d" % i, 0.02, n2.Tlo, n2.Tmid, n2.Thi, lo, hi, n2.sigma, n2.eps_k))
    names = [s.name for s in sp]
    rx = []
    for r in range(nr):
        k = int(rng.integers(1, 4))
        reac = {names[i]: int(rng.integers(1, 3)) for i in rng.choice(ns, size=k, replace=False)}
        order = sum(reac.values())
        # equal molar masses: mass balance <=> equal total coefficients
        pk = int(rng.integers(1, min(3, order) + 1))
        prods = list(rng.choice(ns, size=pk, replace=False))
        prod = {names[i]: 0 for i in prods}
        for t in range(order):
            prod[names[prods[t % pk]]] += 1
        if any(v > 3 for v in prod.values()):
            prod = {names[prods[0]]: min(order, 3)}
            if order > 3:
                continue
            prod[names[prods[0]]] = order
        tb = bool(rng.random() < 0.2)
        rx.append(M.Reaction(reac, prod, float(10 ** rng.uniform(-1, 2)), float(rng.uniform(-1, 1)),
                             float(rng.uniform(0, 3000)), reversible=reversible and bool(rng.random() < 0.7),
                             third_body=tb, eff={names[0]: 2.0} if tb else {}))
    return M.Mechanism("rand%d" % seed, sp, rx)


def test_random_mechanism_text_roundtrip():
    m = _random_mech(10, 17, 3)
    m2 = M.Mechanism.from_text(m.to_text())
    assert m2.to_text() == m.to_text()


def _random_case(ns, nr):
    m = _random_mech(ns, nr, ns)
    rng = np.random.default_rng(ns + nr)
    n = 16 * 9 + 7
    Y = rng.random((ns, n)) * 0.05 + 1e-4
    T = 900.0 + 1500.0 * rng.random(n)
    rho = Y.sum(0)
    return m, Y, rho, M.mixture_e(m, (Y / rho).T, T), T


@pytest.mark.parametrize("ns,nr", [(3, 5), (10, 17), (13, 21), (16, 40)])
def test_host_operator_random_mechanisms(native, ns, nr):
    """The host integrator (the device kernels' oracle in the solver) on
    runtime mechanisms of every size against the NumPy FP64 oracle."""
    m, Y, rho, e, T = _random_case(ns, nr)
    ref, Tref = M.point_implicit_step(m, Y, rho, e, T, 1e-4, 2)
    got, Tg = native.mech_chem_host(m.to_text(), Y, rho, e, T, 1e-4, 2)
    assert np.isfinite(ref).all()
    # random steps reach order 5 with species on both sides: the systems are
    # far worse conditioned than a real mechanism's (1e-9 on the built-in set)
    assert ch.increment_error(got, ref, Y) < 1e-7
    assert np.abs(Tg - Tref).max() < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("dt,nsub", [(1e-8, 1), (1e-7, 2), (2e-6, 4)])
def test_mfma_kernel_builtin_mechanism_matches_oracle(gpu, dt, nsub):
    m = M.h2_air_li2004()
    Y, rho, e, T = ch.demo_state(m, 16 * 37 + 5, seed=7)      # partial last tile
    ref, Tref = M.point_implicit_step(m, Y, rho, e, T, dt, nsub)
    got, Tg, ms = ch.mech_step_gpu(m, Y, rho, e, T, dt, nsub, kernel="mfma")
    assert np.isfinite(got).all() and ms > 0
    assert ch.increment_error(got, ref, Y) < 1e-9, (dt, nsub)
    assert np.abs(Tg - Tref).max() < 1e-8


@pytest.mark.gpu
def test_fast_and_mfma_kernels_agree(gpu):
    m = M.h2_air_li2004()
    Y, rho, e, T = ch.demo_state(m, 4096, seed=2)
    a, Ta, _ = ch.mech_step_gpu(m, Y, rho, e, T, 1e-7, 2, kernel="fast")
    b, Tb, _ = ch.mech_step_gpu(m, Y, rho, e, T, 1e-7, 2, kernel="mfma")
    assert ch.increment_error(a, b, Y) < 1e-9
    assert np.abs(Ta - Tb).max() < 1e-8


@pytest.mark.gpu
@pytest.mark.parametrize("ns,nr", [(3, 5), (10, 17), (13, 21), (16, 40)])
def test_mfma_kernel_random_mechanisms(gpu, ns, nr):
    """Every padded system size (4, 12, 16) and reaction padding (16..48)."""
    m, Y, rho, e, T = _random_case(ns, nr)
    ref, Tref = M.point_implicit_step(m, Y, rho, e, T, 1e-4, 2)
    got, Tg, _ = ch.mech_step_gpu(m, Y, rho, e, T, 1e-4, 2, kernel="mfma")
    assert ch.increment_error(got, ref, Y) < 1e-7
    assert np.abs(Tg - Tref).max() < 1e-6


@pytest.mark.gpu
def test_mfma_kernel_rejects_bad_temperature(gpu):
    m = M.h2_air_li2004()
    Y, rho, e, T = ch.demo_state(m, 32, seed=1)
    T[3] = -5.0
    with pytest.raises(RuntimeError):
        ch.mech_step_gpu(m, Y, rho, e, T, 1e-7, 1, kernel="mfma")


def test_cli_chem_save_builtin(tmp_path):
    from openhyperflow2d_amd import cli

    p = str(tmp_path / "h2.mech")
    assert cli.main(["chem", "--save-builtin", p]) == 0
    assert M.Mechanism.load(p).to_text() == M.h2_air_li2004().to_text()


@pytest.mark.gpu
def test_cli_chem_runs_file_mechanism(gpu, tmp_path, capsys):
    import json

    from openhyperflow2d_amd import cli

    p = str(tmp_path / "m.mech")
    _random_mech(6, 9, 2).save(p)
    assert cli.main(["chem", "--mech", p, "--nx", "40", "--ny", "10", "--repeats", "2", "--dt", "1e-4"]) == 0
    res = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert res["cells"] == 400 and res["species"] == 6 and res["incr_err_vs_numpy_fp64"] < 1e-7


@pytest.mark.gpu
def test_solver_uses_mfma_kernel_for_file_mechanism(gpu, tmp_path):
    """A mechanism read from a file at run time (here the built-in set with one
    rate constant changed, so no compiled kernel matches) runs the MFMA kernel
    inside the time step (with the hiprtc-specialised kernels switched off;
    they are the default, tests/test_gpu_mechanism.py) and agrees with the
    host stepper."""
    from openhyperflow2d_amd.models import decks

    m = M.h2_air_li2004()
    m.reactions[0].A *= 1.1
    m.name = "h2_air_modified"
    path = tmp_path / "h2mod.mech"
    m.save(str(path))
    text = decks.with_mechanism(decks.reactor0d(8, 8, T=1200.0, p=101325.0), mechanism=str(path), substeps=2)
    g = gpu.Simulation(text, "gpu")
    assert not g.solver.chem_fast_ok
    g.solver.chem_rtc = False
    c = gpu.Simulation(text, "cpu")
    g.step(300)
    c.step(300)
    assert g.solver.chem_kernel_used == "hf2d_chem_mech"
    Tg, Tc = g.field("T"), c.field("T")
    assert np.abs(Tg - Tc).max() < 1e-6 * Tc.max()
    for s in ("H2", "OH", "H2O"):
        assert np.abs(g.field("Y:" + s) - c.field("Y:" + s)).max() < 1e-9, s
