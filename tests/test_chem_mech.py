"""K12 finite-rate mechanism chemistry: PyTorch FP64 reference properties (CPU) and the
MFMA HIP kernel against that reference (GPU).  No reference fixture covers this path
(the reference's CRM_ARRENIUS slot is empty, hyper_flow_bound.hpp:37-42): parity unpinned."""
import numpy as np
import pytest

from openhyperflow2d_amd.ops import chemistry as ch


def _rates(m, Y, T):
    nmat, arr, rsp, rord = m.packed()
    c = Y.T / m.W
    A, b, Ta = arr.reshape(3, -1)
    kf = A * T[:, None] ** b * np.exp(-Ta / T[:, None])
    q = kf * np.prod([c[:, rsp[:, t]] ** rord[:, t] for t in range(3)], axis=0)
    return q @ nmat[: m.ns].T


def test_packing_and_validation():
    m = ch.h2_air_demo()
    nmat, arr, rsp, rord = m.packed()
    assert nmat.shape == (16, 12) and arr.shape == (36,) and rsp.shape == (12, 3)
    assert np.all(nmat[m.ns:] == 0)
    # every step is mass balanced: sum_i W_i N_ir = 0
    assert np.abs(m.W @ nmat[: m.ns]).max() < 1e-15
    with pytest.raises(ValueError):
        ch.Mechanism(["A"], [1.0], [ch.Reaction({"B": 1}, {"A": 1}, 1.0)])
    with pytest.raises(ValueError):
        ch.Mechanism(["A"], [1.0], [ch.Reaction({"A": 4}, {"A": 1}, 1.0)])


def test_reference_conserves_mass_and_matches_explicit_limit():
    m = ch.h2_air_demo()
    Y, T = ch.demo_state(m, 48, seed=3)
    Y1 = ch.reference_step(m, Y, T, 1e-7, nsub=4)
    assert (Y1 > 0).all()
    assert np.abs(Y1.sum(0) - Y.sum(0)).max() < 1e-13 * Y.sum(0).max()
    dt = 1e-12   # h*|J| ~ 1e-4: the implicit step is the explicit rate to that order
    Y2 = ch.reference_step(m, Y, T, dt, nsub=1)
    om = _rates(m, Y, T)
    assert np.abs((Y2.T / m.W - Y.T / m.W) / dt - om).max() < 1e-3 * np.abs(om).max()


def test_reference_single_reaction_closed_form():
    # A -> B first order: point-implicit substep gives c_A / (1 + k h) per substep
    m = ch.Mechanism(["A", "B"], [1.0, 1.0], [ch.Reaction({"A": 1}, {"B": 1}, 50.0)])
    Y = np.array([[2.0, 1.0], [0.0, 0.5]])
    T = np.array([300.0, 900.0])
    Y1 = ch.reference_step(m, Y, T, 0.01, nsub=5)
    np.testing.assert_allclose(Y1[0], Y[0] / (1 + 50.0 * 0.002) ** 5, rtol=1e-14)
    np.testing.assert_allclose(Y1.sum(0), Y.sum(0), rtol=1e-14)


@pytest.mark.gpu
def test_chem_mech_gpu_matches_reference():
    import openhyperflow2d_amd as hf

    assert hf.native().gpu_available(), "HIP device required"
    m = ch.h2_air_demo()
    Y, T = ch.demo_state(m, 16 * 37 + 5, seed=7)      # partial last tile
    for dt, nsub in ((1e-7, 1), (1e-7, 4), (2e-6, 3)):
        ref = ch.reference_step(m, Y, T, dt, nsub)
        got, ms = ch.mech_step_gpu(m, Y, T, dt, nsub)
        assert np.isfinite(got).all() and ms > 0
        err = np.abs(got - ref).max() / np.abs(ref).max()
        assert err < 1e-10, (dt, nsub, err)


@pytest.mark.gpu
def test_chem_mech_gpu_closed_form_and_padding():
    m = ch.Mechanism(["A", "B"], [1.0, 1.0], [ch.Reaction({"A": 1}, {"B": 1}, 50.0)])
    Y = np.array([[2.0, 1.0, 3.0], [0.0, 0.5, 0.1]])
    T = np.array([300.0, 900.0, 1200.0])
    got, _ = ch.mech_step_gpu(m, Y, T, 0.01, nsub=5)
    np.testing.assert_allclose(got[0], Y[0] / (1 + 50.0 * 0.002) ** 5, rtol=1e-13)
    np.testing.assert_allclose(got.sum(0), Y.sum(0), rtol=1e-13)


def _random_mech(ns, nr, seed):
    rng = np.random.default_rng(seed)
    sp = ["S%d" % i for i in range(ns)]
    rx = []
    for _ in range(nr):
        k = int(rng.integers(1, 4))
        reac = {sp[i]: int(rng.integers(1, 3)) for i in rng.choice(ns, size=k, replace=False)}
        prod = {sp[i]: 1 for i in rng.choice(ns, size=int(rng.integers(1, 3)), replace=False)}
        rx.append(ch.Reaction(reac, prod, float(10 ** rng.uniform(0, 3)), float(rng.uniform(-1, 1)),
                              float(rng.uniform(0, 3000))))
    return ch.Mechanism(sp, 0.001 + 0.05 * rng.random(ns), rx)


def test_random_mechanism_reference_runs():
    m = _random_mech(13, 21, 5)
    assert m.packed()[0].shape == (16, 24)
    Y = np.random.default_rng(1).random((13, 40)) * 0.05
    out = ch.reference_step(m, Y, np.full(40, 1500.0), 1e-4, nsub=2)
    assert np.isfinite(out).all() and (out >= 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("ns,nr", [(3, 5), (10, 17), (13, 21), (16, 40)])
def test_chem_mech_gpu_random_mechanisms(ns, nr):
    """Every padded system size (4, 12, 16) and reaction padding against the FP64 reference."""
    m = _random_mech(ns, nr, ns)
    rng = np.random.default_rng(ns + nr)
    n = 16 * 9 + 7
    Y = rng.random((ns, n)) * 0.05
    T = 900.0 + 1500.0 * rng.random(n)
    ref = ch.reference_step(m, Y, T, 1e-4, nsub=2)
    got, _ = ch.mech_step_gpu(m, Y, T, 1e-4, nsub=2)
    assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-10


def test_mechanism_json_roundtrip(tmp_path):
    m = ch.h2_air_demo()
    p = str(tmp_path / "mech.json")
    m.save(p)
    m2 = ch.Mechanism.load(p)
    for a, b in zip(m.packed(), m2.packed()):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(m.W, m2.W)


def test_cli_chem_save_demo(tmp_path):
    from openhyperflow2d_amd import cli

    p = str(tmp_path / "demo.json")
    assert cli.main(["chem", "--save-demo", p]) == 0
    assert ch.Mechanism.load(p).species == ch.h2_air_demo().species


@pytest.mark.gpu
def test_cli_chem_runs_json_mechanism(tmp_path, capsys):
    import json

    from openhyperflow2d_amd import cli

    p = str(tmp_path / "m.json")
    _random_mech(6, 9, 2).save(p)
    assert cli.main(["chem", "--mech", p, "--nx", "40", "--ny", "10", "--repeats", "2", "--dt", "1e-4"]) == 0
    res = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert res["cells"] == 400 and res["species"] == 6 and res["rel_err_vs_torch_fp64"] < 1e-10
