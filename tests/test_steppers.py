"""Host steppers: the Jacobi stepper (same per-cell code as the HIP kernels),
its lean inviscid variant and the LDS-tile emulation must agree bit for bit;
the reference-order stepper is the golden oracle (test_reference_golden)."""
import numpy as np
import pytest

from openhyperflow2d_amd.models import decks
from tests.conftest import read_deck

FIELDS = ["rho", "U", "V", "p", "T", "k", "R", "CP"]


def _decks():
    return {
        "wedge15": decks.wedge15(120, 40, nmax=10 ** 6, nout=10 ** 5),
        "wedge15_odd": decks.wedge15(97, 53, nmax=10 ** 6, nout=10 ** 5),
        "oblique": decks.set_key(read_deck("ObliqueShock.dat"), "Nmax", 1000),
    }


def _records_wo_scratch(sim):
    """Cell records with the dS/dx, dS/dy scratch (bytes 72..215) masked: the
    lean path only maintains them where a Cauchy neighbour reads them."""
    r = np.frombuffer(sim.records(), dtype=np.uint8).reshape(-1, 1248).copy()
    r[:, 72:216] = 0
    return r


@pytest.mark.parametrize("name", list(_decks()))
@pytest.mark.parametrize("tile,sg,cpt,tj,nt", [(False, False, 1, 0, 256), (True, False, 1, 0, 256),
                                              (True, True, 1, 0, 256), (True, True, 2, 0, 256),
                                              (True, False, 2, 11, 256), (True, True, 1, 16, 64),
                                              (True, True, 2, 0, 128), (True, True, 2, 32, 64)])
def test_lean_equals_generic(hf, name, tile, sg, cpt, tj, nt):
    """nt: threads per emulated tile workgroup (the small-strip geometries)."""
    text = _decks()[name]
    a = hf.Simulation(text, "cpu", lean=False)
    b = hf.Simulation(text, "cpu", lean=True)
    b.solver.lean_tile = tile
    b.solver.lean_sg = sg
    b.solver.lean_cpt = cpt
    b.solver.lean_tj = tj
    b.solver.lean_nt = nt
    assert b.solver.lean_ok, b.solver.lean_why
    assert b.solver.lean_sg_ok
    for s in range(3):
        res = s != 1
        a.step(4, residual=res)
        b.step(4, residual=res)
        sa, sb = a.summary(), b.summary()
        assert sa["dt"] == sb["dt"]
        np.testing.assert_allclose(sa["rms"], sb["rms"], rtol=1e-12, atol=0)
        for f in FIELDS:
            np.testing.assert_array_equal(a.field(f), b.field(f), err_msg=f)
    # the whole record (species, Y, fluxes, k, Tg, ...) except dS scratch
    np.testing.assert_array_equal(_records_wo_scratch(a), _records_wo_scratch(b))


def test_lean_generic_switching(hf):
    text = _decks()["wedge15"]
    a = hf.Simulation(text, "cpu", lean=False)
    b = hf.Simulation(text, "cpu", lean=True)
    for s in range(6):
        b.solver.lean = s % 2 == 0
        a.step(3)
        b.step(3)
    for f in FIELDS:
        np.testing.assert_array_equal(a.field(f), b.field(f), err_msg=f)


def test_lean_not_eligible_for_viscous(hf):
    text = decks.wedge15(60, 30, navier_stokes=True, turbulence=4, nmax=100, nout=10)
    b = hf.Simulation(text, "cpu", lean=True)
    assert not b.solver.lean_ok
    assert "viscous" in b.solver.lean_why


def test_jacobi_equals_reference_order_on_oblique_shock(hf):
    """Without Neumann chains along the sweep the in-place reference sweep
    and the Jacobi update coincide."""
    text = decks.set_key(read_deck("ObliqueShock.dat"), "Nmax", 1000)
    a = hf.Simulation(text, "cpu")
    r = hf.Simulation(text, "ref")
    a.step(25)
    r.step(25)
    for f in ["rho", "U", "V", "p", "T"]:
        np.testing.assert_array_equal(a.field(f), r.field(f), err_msg=f)


def test_jacobi_close_to_reference_order_on_wedge(hf):
    text = decks.wedge15(200, 40, nmax=1000, nout=100)
    a = hf.Simulation(text, "cpu")
    r = hf.Simulation(text, "ref")
    a.step(100)
    r.step(100)
    rho_a, rho_r = a.field("rho"), r.field("rho")
    assert np.isfinite(rho_a).all()
    # Jacobi vs Gauss-Seidel-like order: same solution, small transient differences
    assert np.abs(rho_a - rho_r).max() / rho_r.max() < 0.05


def test_checkpoint_roundtrip(hf, tmp_path):
    text = decks.wedge15(80, 30, nmax=1000, nout=100)
    a = hf.Simulation(text, "cpu")
    a.step(10)
    a.solver.download()
    p = str(tmp_path / "x.hf2d")
    a.case.write_checkpoint(p)
    import os

    assert os.path.getsize(p) == 80 * 30 * hf.native().CELL_RECORD_BYTES
    b = hf.Simulation(text, "cpu")
    b.case.read_checkpoint(p)
    assert b.case.records() == a.case.records()


def test_negative_temperature_is_reported(hf):
    text = decks.wedge15(60, 20, nmax=1000, nout=100)
    s = hf.Simulation(text, "cpu")
    # corrupt the energy of one interior cell: Tg < 0 after the next fill
    import struct

    rec = bytearray(s.case.records())
    idx = 30 * 20 + 10
    off = idx * 1248 + 3 * 8   # S[RHOE]
    struct.pack_into("<d", rec, off, -1.0e6)
    s.case.set_records(bytes(rec))
    s.solver.upload()
    with pytest.raises(RuntimeError, match="unstability"):
        s.step(2)
