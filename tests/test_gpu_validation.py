"""Flat-plate skin friction against boundary-layer correlations (SST /
viscous validation, models/validation.py; numbers in
profiles/flat_plate_validation.md).  Mach 2.5 air over a no-slip plate,
Eckert reference-temperature correlations."""
import numpy as np
import pytest

from openhyperflow2d_amd.models import decks, validation

pytestmark = pytest.mark.gpu


def _run(gpu, model, nx, ny, dx, dy, p, flow_throughs, cfl=None):
    text = decks.flat_plate(nx, ny, dx=dx, dy=dy, x_le=0.2, mach=2.5, p=p, turbulence=model,
                            nmax=10 ** 9, nout=10 ** 8, cfl=cfl)
    # the plate is the domain edge (no solid cells): adiabatic, lean N-S kernels
    sim = gpu.Simulation(decks.set_key(text, "isAdiabaticWall", 1), "gpu")
    t_end = flow_throughs * nx * dx / (2.5 * 341.0)
    while sim.summary()["time"] < t_end:
        sim.step(2000)
    return validation.plate_cf(sim, 0.2)


def test_laminar_plate_follows_blasius(gpu):
    """Cf ~ Re_x^-1/2 (Blasius): 0.90-0.92 of the correlation at CFL 0.4 on
    this 30-cells-per-thickness grid (0.85 at the deck's CFL 0.1: the DEEPS
    blend's diffusion scales with dy^2 / dt, profiles/flat_plate_validation.md)."""
    r = _run(gpu, 0, 250, 100, 1e-3, 1e-4, 1e3, 3.0, cfl=0.4)
    sel = (r["Re_x"] > 1.5e4) & (r["Re_x"] < 1.0e5)
    ratio = r["Cf"][sel] / r["Cf_lam"][sel]
    assert 0.87 < ratio.mean() < 1.05, ratio.mean()
    assert ratio.std() < 0.05, ratio.std()
    slope = np.polyfit(np.log(r["Re_x"][sel]), np.log(r["Cf"][sel]), 1)[0]
    assert -0.56 < slope < -0.44, slope


@pytest.fixture(scope="module")
def turbulent_runs(request):
    import openhyperflow2d_amd as hf

    if not hf.gpu_available():
        pytest.fail("GPU test requires a HIP device")
    # k-omega SST on three wall-normal grids (dy 40 / 20 / 10 um; the finest
    # at CFL 0.3, the others at 0.4: it is unstable at 0.4) and the k-eps
    # reference model
    return {6: _run(hf, 6, 312, 750, 1e-3, 4e-5, 1e4, 5.0, cfl=0.4), 4: _run(hf, 4, 312, 750, 2e-3, 4e-5, 1e4, 2.0),
            "6_dy20": _run(hf, 6, 312, 1500, 1e-3, 2e-5, 1e4, 5.0, cfl=0.4),
            "6_dy10": _run(hf, 6, 312, 3000, 1e-3, 1e-5, 1e4, 5.0, cfl=0.3)}


def test_sst_plate_molecular_wall_friction_converges_to_van_driest(turbulent_runs):
    """k-omega SST (Menter's wall omega at the first cell) on a developed
    turbulent layer, Re_x 0.7-1.3e6, asserting on the MOLECULAR wall friction
    mu_w dU/dy against van Driest II.  The DEEPS predictor's blend adds a
    diffusion D = (1 - beta) dyy/2 dy^2/dt across the first cell, which
    carries part of the sublayer stress (profiles/flat_plate_validation.md);
    D / nu_w falls from ~0.5 (dy 40 um) to ~0.25 (20 um) and ~0.17 (10 um at
    CFL 0.3), and the molecular Cf rises monotonically with it: 0.47-0.49,
    0.61-0.64, 0.70-0.73 of van Driest II.  The zero-D limit of the three
    grids (quadratic in D / nu_w) is within +-15 % of van Driest II; so is the
    linear limit of the two finest grids.  Cf > 1.6x the laminar law: the
    layer is turbulent.  The modelled stress over 30 <= y+ <= 100 (Cf_eff) is
    a diagnostic only."""
    runs = [turbulent_runs[6], turbulent_runs["6_dy20"], turbulent_runs["6_dy10"]]
    sel = [(r["Re_x"] > 7e5) & (r["Re_x"] < 1.3e6) for r in runs]
    assert (runs[0]["Cf"][sel[0]] / runs[0]["Cf_lam"][sel[0]]).min() > 1.6
    mol = [float((r["Cf"][s] / r["Cf_turb_vd2"][s]).mean()) for r, s in zip(runs, sel)]
    dnu = [float(r["blend_nu"][s].mean()) for r, s in zip(runs, sel)]
    lim3 = validation.extrapolate_to_zero(dnu, mol)
    lim2 = validation.extrapolate_to_zero(dnu[1:], mol[1:])
    msg = "molecular Cf / van Driest II %s at D/nu_w %s; zero-D limit %.3f (3 grids), %.3f (2 finest)" % (
        ["%.3f" % m for m in mol], ["%.3f" % d for d in dnu], lim3, lim2)
    assert dnu[0] > dnu[1] > dnu[2] > 0, msg
    assert mol[0] < mol[1] < mol[2], msg   # monotone convergence as the blend diffusion vanishes
    assert 0.45 < mol[0] < 0.62, msg       # (the coarse grid's deficit, round 4's pin)
    assert 0.85 < lim3 < 1.15, msg
    assert 0.85 < lim2 < 1.15, msg


def test_keps_plate_keeps_the_reference_eddy_viscosity_cap(turbulent_runs):
    """The reference's k-eps update takes mu_t = min(mu_t_new, mu_t_old)
    (libOpenHyperFLOW2D/hyper_flow_node.hpp:783, reproduced bit for bit): mu_t can only
    fall from its free-stream initial value, so no turbulent layer forms and
    Cf stays near / below the laminar law (0.6-0.7 of it)."""
    r = turbulent_runs[4]
    hi = r["Re_x"] > 1.4e6
    assert (r["Cf"][hi] / r["Cf_lam"][hi]).max() < 1.0


def test_sst_mixing_layer_grows_linearly_at_the_incompressible_rate(gpu):
    """Compressible plane mixing layer (decks.mixing_layer: Mach 2.0 over
    Mach 1.2 air, Mc = 0.40, lambda = 0.25) with k-omega SST: the vorticity
    thickness grows linearly (measured R^2 = 1.000 over 30-90 % of the
    domain) at 0.98 x the incompressible Brown-Roshko rate 0.18 lambda and
    1.47 x the Langley-corrected compressible rate: SST without a
    compressibility correction reproduces the incompressible spreading, the
    known behaviour of the model (profiles/mixing_layer_validation.md)."""
    text = decks.mixing_layer(600, 300, turbulence=6, nmax=10 ** 9, nout=10 ** 8)
    sim = gpu.Simulation(text, "gpu")
    t_end = 2.5 * 600 * 5e-4 / (1.2 * 347.0)
    while sim.summary()["time"] < t_end:
        sim.step(2000)
    g = validation.mixing_layer_growth(sim)
    assert abs(g["Mc"] - 0.40) < 0.02, g["Mc"]
    assert g["r2"] > 0.98, g["r2"]
    assert 0.7 < g["rate"] / g["rate_incompressible"] < 1.3, g["rate"] / g["rate_incompressible"]
    assert g["rate"] > g["rate_compressible"]
