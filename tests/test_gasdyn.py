"""Isentropic gas-dynamics helpers (reference libFlow/flow.cpp, flow2d.cpp)
against closed-form textbook relations (plain float64 Python)."""
import math

import pytest

CP, R, T0, P0 = 1005.0, 287.0, 300.0, 101325.0


@pytest.fixture
def flow(native):
    return native.GasFlow(CP, T0, P0, R)


def test_k(flow):
    assert flow.kg() == pytest.approx(CP / (CP - R))


@pytest.mark.parametrize("mach", [0.2, 0.8, 1.0, 2.5, 4.0])
def test_mach_roundtrip_and_isentropic_ratios(flow, mach):
    k = CP / (CP - R)
    flow.set_mach(mach)
    assert flow.mach() == pytest.approx(mach, rel=1e-10)
    lam2 = (k + 1) / 2 * mach ** 2 / (1 + (k - 1) / 2 * mach ** 2)
    assert flow.LAM() == pytest.approx(math.sqrt(lam2), rel=1e-10)
    tau = 1 - (k - 1) / (k + 1) * lam2
    assert flow.TAU() == pytest.approx(tau, rel=1e-12)
    assert flow.PF() == pytest.approx(tau ** (k / (k - 1)), rel=1e-12)
    assert flow.EPS() == pytest.approx(tau ** (1 / (k - 1)), rel=1e-12)
    assert flow.Tg() == pytest.approx(T0 * tau, rel=1e-12)
    assert flow.Pg() == pytest.approx(P0 * tau ** (k / (k - 1)), rel=1e-12)
    a_kr = math.sqrt(2 * k / (k + 1) * R * T0)
    assert flow.Akr() == pytest.approx(a_kr, rel=1e-12)
    assert flow.wg() == pytest.approx(math.sqrt(lam2) * a_kr, rel=1e-10)
    assert flow.Asound() == pytest.approx(math.sqrt(k * R * flow.Tg()), rel=1e-10)


def test_correct_flow_static_state(flow, native):
    # CorrectFlow(T, p, M, fixed_mach): choose T0/P0 so that the static
    # state is (T, p) at Mach M
    flow.correct_flow(250.0, 5.0e4, 2.0, True)
    assert flow.Tg() == pytest.approx(250.0, rel=1e-9)
    assert flow.Pg() == pytest.approx(5.0e4, rel=1e-9)
    assert flow.mach() == pytest.approx(2.0, rel=1e-9)


def test_flow2d_velocity_components(native):
    f = native.GasFlow.make2d(1.8e-5, 0.025, CP, 288.0, 1.0e5, R, 600.0, -100.0)
    assert f.U() == pytest.approx(600.0)
    assert f.V() == pytest.approx(-100.0)
    assert f.Wg2d() == pytest.approx(math.sqrt(600.0 ** 2 + 100.0 ** 2 + 1e-5))
    # Flow2D(mu, lam, Cp, T, P, R, u, v) takes T, P as stagnation values
    assert f.T0() == 288.0 and f.P0() == 1.0e5
    w2 = 600.0 ** 2 + 100.0 ** 2
    assert f.Tg() == pytest.approx(288.0 - w2 / (2 * CP), rel=1e-9)
    m = f.mach()
    f.mach2d(2 * m)   # keeps the flow angle
    assert f.V() / f.U() == pytest.approx(-100.0 / 600.0, rel=1e-9)
