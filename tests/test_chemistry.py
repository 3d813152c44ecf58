"""Finite-rate global H2/air chemistry (ChemicalReactionsModel=2, new
physics): a closed slip-wall box at rest is a constant-volume reactor in
every cell.  The rate law is checked against a float64 Python evaluation of
the same expression; conservation and heat release are checked on the run
(no reference implementation exists: parity unpinned)."""
import math

import numpy as np
import pytest

from openhyperflow2d_amd.models import decks

RU = 8.314462618


def _cell(sim, nx=8, ny=8, i=4, j=4):
    r = np.frombuffer(sim.records(), dtype=np.uint8).reshape(nx, ny, 1248)[i, j]
    S = r[0:72].copy().view(np.float64)
    Tg = float(r[1048:1056].copy().view(np.float64)[0])
    Src = r[544 + 5 * 72:544 + 6 * 72].copy().view(np.float64)
    return S, Tg, Src


def test_rate_law_matches_python(hf):
    s = hf.Simulation(decks.reactor0d(T=1200.0), "cpu")
    s.step(1)
    S, T, Src = _cell(s)
    Mfu, Mox = RU / 4124.2, RU / 259.8
    cfu, cox = S[4] / Mfu, S[5] / Mox
    W = 1.8e10 * math.exp(-17614.0 / T) * cfu ** 1.0 * cox ** 0.5
    W = min(W, min(0.5 * cfu, cox) / s.summary()["dt"])
    assert Src[4] == pytest.approx(-2 * Mfu * W, rel=1e-12)
    assert Src[5] == pytest.approx(-Mox * W, rel=1e-12)
    assert Src[6] == pytest.approx((2 * Mfu + Mox) * W, rel=1e-12)
    assert Src[4] + Src[5] + Src[6] == pytest.approx(0.0, abs=1e-9 * abs(Src[6]))


def test_reactor_burns_to_completion_and_conserves_mass(hf):
    s = hf.Simulation(decks.reactor0d(T=1500.0), "cpu")
    S0, T0, _ = _cell(s)
    m0 = S0[4:7].sum()
    prev_fu, prev_T = S0[4], T0
    for _ in range(8):
        s.step(3)
        S, T, _ = _cell(s)
        # (T relaxes by ~1e-5 after burnout: Cp(T) is lagged one step)
        assert S[4] <= prev_fu + 1e-15 and T >= prev_T * (1 - 1e-4)
        prev_fu, prev_T = S[4], T
        assert S[4:7].sum() == pytest.approx(m0, rel=1e-8)
    s.step(200)
    S, T, _ = _cell(s)
    assert S[4] < 1e-3 * S0[4]             # stoichiometric (to the molar masses): fuel consumed
    assert 2500.0 < T < 4000.0             # constant-volume H2/air flame, no dissociation
    assert S[0] == pytest.approx(S0[0], rel=1e-12)   # closed box: density unchanged
    T_all = s.field("T")
    assert np.ptp(T_all) < 1e-6 * T_all.mean()      # every cell the same reactor


def test_no_reaction_without_fuel(hf):
    text = decks.set_key(decks.reactor0d(T=1500.0), "Flow2D-1.Y_fuel", 0.0)
    text = decks.set_key(text, "Flow2D-2.Y_fuel", 0.0)
    s = hf.Simulation(text, "cpu")
    S0, T0, _ = _cell(s)
    s.step(20)
    S, T, Src = _cell(s)
    assert np.all(Src[4:7] == 0.0)
    assert T == pytest.approx(T0, rel=1e-9)
