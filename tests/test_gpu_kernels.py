"""GPU numerics: the HIP kernels against the CPU Jacobi stepper (which runs the
same per-cell code on the host) and against the reference-order oracle."""
import numpy as np
import pytest

from openhyperflow2d_amd.models import decks

pytestmark = pytest.mark.gpu

FIELDS = ["rho", "U", "V", "p", "T"]


MODES = {
    "lean_tile": dict(lean=True, lean_tile=True),
    "lean_tile_nosg": dict(lean=True, lean_tile=True, lean_sg=False),
    "lean_flat": dict(lean=True, lean_tile=False),
    "fused": dict(lean=False, fused=True),
    "split": dict(lean=False, fused=False),
}


def _gpu_sim(hf, text, mode):
    kw = dict(MODES[mode])
    tile = kw.pop("lean_tile", True)
    sg = kw.pop("lean_sg", True)
    g = hf.Simulation(text, "gpu", **kw)
    g.solver.lean_tile = tile
    g.solver.lean_sg = sg
    return g


def _run_pair(hf, text, steps, mode="lean_tile"):
    g = _gpu_sim(hf, text, mode)
    c = hf.Simulation(text, "cpu")
    g.step(steps, residual=True)
    c.step(steps, residual=True)
    return g, c


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


@pytest.mark.parametrize("mode", list(MODES))
def test_wedge_euler_gpu_matches_cpu(gpu, mode):
    text = decks.wedge15(200, 40, nmax=1000, nout=10)
    g, c = _run_pair(gpu, text, 50, mode)
    if mode.startswith("lean"):
        assert g.solver.lean_ok, g.solver.lean_why
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


@pytest.mark.parametrize("mode", list(MODES))
def test_step_euler_gpu(gpu, mode):
    """Step has ny=250 so i+-1 neighbours live in other workgroups: catches
    any read-after-write race between the predictor and the fill."""
    from tests.conftest import read_deck

    g, c = _run_pair(gpu, read_deck("Step.dat"), 20, mode)
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


@pytest.mark.parametrize("nt,cpt,tj", [(128, 1, 0), (128, 2, 16), (64, 1, 16), (64, 2, 8), (64, 1, 64)])
def test_small_workgroup_tiles_bitwise(gpu, nt, cpt, tj):
    """The small-strip tile geometries (64 / 128-thread workgroups, one or two
    cells per thread) == the 256-thread tile kernel bit for bit: fields, dt,
    time (residual sums: reduced over other partials)."""
    text = decks.wedge15(250, 200, nmax=10 ** 6, nout=10 ** 5)
    ref = gpu.Simulation(text, "gpu")
    s = gpu.Simulation(text, "gpu")
    ref.solver.lean_nt, ref.solver.lean_cpt, ref.solver.lean_tj = 256, 2, 0
    s.solver.lean_nt, s.solver.lean_cpt, s.solver.lean_tj = nt, cpt, tj
    for n, res in [(5, True), (30, False), (7, True)]:
        s.step(n, residual=res)
        ref.step(n, residual=res)
        assert s.summary()["dt"] == ref.summary()["dt"]
    assert s.summary()["time"] == ref.summary()["time"]
    np.testing.assert_allclose(s.summary()["rms"], ref.summary()["rms"], rtol=1e-12, atol=0)
    for f in FIELDS + ["k", "R", "CP"]:
        np.testing.assert_array_equal(s.field(f), ref.field(f), err_msg=f)


@pytest.mark.parametrize("nt", [256, 128])
def test_host_tail_scalars_equal_the_read_back_kernel(gpu, nt):
    """Single GPU: the last lean tile step of a host call writes dt, time and
    the error flag into the pinned host mirror from its own tail
    (DeviceSolver.host_tail) -- the same values, call for call, as the
    separate read-back kernel; a Tg < 0 in that last step is still reported."""
    text = decks.wedge15(300, 64, nmax=10 ** 6, nout=10 ** 5)
    a = gpu.Simulation(text, "gpu")
    b = gpu.Simulation(text, "gpu")
    for s in (a, b):
        s.solver.lean_nt, s.solver.lean_cpt, s.solver.lean_tj = nt, 1, 0
    b.solver.host_tail = False
    assert a.solver.host_tail
    for n, res in [(1, False), (2, False), (7, False), (1, True), (20, False), (3, True), (5, False)]:
        a.step(n, residual=res)
        b.step(n, residual=res)
        sa, sb = a.summary(), b.summary()
        assert sa["dt"] == sb["dt"] and sa["time"] == sb["time"], (n, res)
    for f in FIELDS:
        np.testing.assert_array_equal(a.field(f), b.field(f), err_msg=f)
    a.solver.poison_cell(150, 30)
    with pytest.raises(RuntimeError, match="Tg < 0"):
        a.step(1)


def test_lean_bitwise_with_switches(gpu):
    """Lean GPU steps interleaved with downloads and generic steps stay
    bit-identical to the generic CPU stepper (dt, residuals, fields)."""
    text = decks.wedge15(301, 77, nmax=10 ** 6, nout=10 ** 5)
    g = gpu.Simulation(text, "gpu", lean=True)
    c = gpu.Simulation(text, "cpu")
    assert g.solver.lean_ok, g.solver.lean_why
    for it in range(6):
        g.solver.lean = it != 3          # one generic GPU segment in the middle
        g.step(7, residual=(it % 2 == 0))
        c.step(7, residual=(it % 2 == 0))
        sg, sc = g.summary(), c.summary()
        assert sg["dt"] == sc["dt"]
        # residual sums are reduced in a different order on the device
        np.testing.assert_allclose(sg["rms"], sc["rms"], rtol=1e-12, atol=0)
        for f in FIELDS + ["k", "R", "CP"]:
            np.testing.assert_array_equal(g.field(f), c.field(f), err_msg=f)
    rg = np.frombuffer(g.records(), dtype=np.uint8).reshape(-1, 1248).copy()
    rc = np.frombuffer(c.records(), dtype=np.uint8).reshape(-1, 1248).copy()
    rg[:, 72:216] = 0   # dS/dx, dS/dy scratch: only kept where a Cauchy node reads it
    rc[:, 72:216] = 0
    np.testing.assert_array_equal(rg, rc)


def _virtual_ranks(hf, text, nranks, schedule, lean=True, p2p=False, fuse=True, toggle=False, corrupt=False,
                   stats=None, setup=None, chunk_hook=None, fields=FIELDS, parts=None):
    """Run the strip decomposition as `nranks` DeviceSolvers on ONE GPU, one
    host thread each, halos through the in-process LocalGroup transport (or,
    p2p=True, the device-side mailbox transport: one exchange kernel per step,
    step graphs on)."""
    import threading

    from openhyperflow2d_amd.parallel.strips import balanced_columns

    nat = hf.native()
    cases = [nat.Case.from_deck(text, ".", False) for _ in range(nranks)]
    parts = parts or balanced_columns(np.asarray(cases[0].field("solid")), nranks)
    group = nat.LocalGroup(nranks)
    solvers = []
    for r, (a, b) in enumerate(parts):
        s = nat.DeviceSolver(cases[r], 0, a, b)
        s.lean = lean
        if setup is not None:
            setup(s)
        s.init_local(group, r)
        solvers.append(s)
    if p2p:
        descs = [s.p2p_export(r, nranks) for r, s in enumerate(solvers)]
        for s in solvers:
            s.p2p_import(descs)
            s.p2p_fuse = fuse
            assert s.p2p_active
        # start-up self-validation (collective: one thread per rank)
        blobs = [None] * nranks

        def probe(r):
            blobs[r] = solvers[r].p2p_probe()

        th = [threading.Thread(target=probe, args=(r,), daemon=True) for r in range(nranks)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=60)
        assert all(b is not None for b in blobs), "p2p probe hung"
        ok, why = nat.DeviceSolver.p2p_probe_ok(blobs, 0)
        if corrupt:
            # a wrong halo on one rank must be caught; every rank falls back
            bad = bytearray(blobs[1])
            bad[16] ^= 1   # sent_l checksum of rank 1 -> rank 0's right halo mismatches
            ok, why = nat.DeviceSolver.p2p_probe_ok([bytes(b) if k != 1 else bytes(bad) for k, b in enumerate(blobs)], 0)
            assert not ok and "right halo of rank 0" in why, why
            th = [threading.Thread(target=s.p2p_fallback, daemon=True) for s in solvers]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=60)
            assert not any(t.is_alive() for t in th), "p2p fallback hung"
            assert not any(s.p2p_active for s in solvers)
            p2p = False
        else:
            assert ok, why
    errors = []

    def run(s, n, res):
        try:
            s.run_steps(n, res)
        except Exception as e:   # pragma: no cover - reported below
            errors.append(e)

    for k, (n, res) in enumerate(schedule):
        if toggle:   # alternate fused / separate-kernel exchange between chunks
            for s in solvers:
                s.p2p_fuse = (k % 2 == 0)
        if chunk_hook is not None:
            chunk_hook(k, solvers)
        th = [threading.Thread(target=run, args=(s, n, res), daemon=True) for s in solvers]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not errors, errors
        assert not any(t.is_alive() for t in th), "virtual-rank step hung"
    if p2p:
        assert all(s.graph_launches > 0 for s in solvers) or max(n for n, _ in schedule) < 12
    if stats is not None:
        stats["overlap_steps"] = [s.overlap_steps for s in solvers]
        stats["lns_steps"] = [s.lns_steps for s in solvers]
        stats["lnm_steps"] = [s.lnm_steps for s in solvers]
        stats["lns_fx_steps"] = [s.lns_fx_steps for s in solvers]
        stats["lns_prologue_steps"] = [s.lns_prologue_steps for s in solvers]
        stats["p2p_mwg_exchanges"] = [s.p2p_mwg_exchanges for s in solvers]
    out = {}
    for f in fields:
        full = None
        for r, (a, b) in enumerate(parts):
            solvers[r].download()
            fr = np.asarray(cases[r].field(f))
            if full is None:
                full = np.zeros_like(fr)
            full[a:b] = fr[a:b]
        out[f] = full
    return out, dict(solvers[0].summary())


@pytest.mark.parametrize("nranks,physics,lean", [(2, "euler", True), (3, "euler", True), (2, "euler", False),
                                                 (3, "kes", False), (8, "euler", True), (8, "kes", False)])
def test_virtual_ranks_match_single_gpu(gpu, nranks, physics, lean):
    ns = physics != "euler"
    text = decks.wedge15(240, 60, navier_stokes=ns, turbulence=4 if ns else 0, nmax=10 ** 6, nout=10 ** 5)
    schedule = [(5, True), (6, False), (5, True)]
    got, summ = _virtual_ranks(gpu, text, nranks, schedule, lean=lean)
    ref = gpu.Simulation(text, "gpu", lean=lean)
    for n, res in schedule:
        ref.step(n, residual=res)
    assert summ["dt"] == ref.summary()["dt"]
    for f in FIELDS:
        np.testing.assert_array_equal(got[f], ref.field(f), err_msg=f)


def _gas_source_ns():
    import os

    d = os.path.join(os.path.dirname(__file__), "fixtures", "ref", "gas_source")
    with open(os.path.join(d, "deck.dat")) as fh:
        return decks.set_key(fh.read(), "ProblemType", 1)


@pytest.mark.parametrize("deck,p2p", [("mech", False), ("mech", True), ("generic", False), ("generic", True),
                                      ("sgt_toggle", False), ("sgt_toggle", True)])
def test_compact_state_halo_matches_single_gpu(gpu, deck, p2p):
    """Split-path halos carry only what the next kernels read of a ghost
    column (S and the x flux A of the live equations, dS/dx only with Cauchy-x
    nodes, no y flux B; mid-step only rho, the species, k/eps -- plus rhoU,
    rhoV, rhoE where mechanism strips react their ghosts).  The strips still
    equal one GPU bit for bit: mechanism (SK_MECH), generic species N-S
    (gas sources) and single-gas k-eps (SK_SGT) switching to the generic
    stepper mid-run, which refreshes the ghost columns in full first."""
    nat = gpu.native()
    fields = list(FIELDS) + ["k", "mu_t"]
    if deck == "mech":
        text = decks.scramjet(150, 50, nmax=10 ** 6, nout=10 ** 5)
        fields += ["Y:H2", "Y:O2", "Y:OH", "Y:H2O"]
        nranks = 3
    elif deck == "generic":
        text = _gas_source_ns()
        fields += ["S4", "S5", "S6"]
        nranks = 3
    else:
        text = decks.wedge15(240, 60, navier_stokes=True, turbulence=4, nmax=10 ** 6, nout=10 ** 5)
        nranks = 3
    schedule = [(5, True), (14, False), (5, True), (12, False)]
    counts = {}

    def setup(s):
        counts["compact"] = s.halo_field_count(1, False)
        counts["full"] = s.halo_field_count(1, True)

    def hook(k, solvers):   # single-gas specialisation off for the second half
        if deck == "sgt_toggle" and k == 2:
            for s in solvers:
                s.sgl = False

    got, summ = _virtual_ranks(gpu, text, nranks, schedule, lean=False, p2p=p2p, fuse=False, setup=setup,
                               chunk_hook=hook, fields=fields)
    assert counts["compact"] < counts["full"], counts
    ref = gpu.Simulation(text, "gpu", lean=False)
    for k, (n, res) in enumerate(schedule):
        if deck == "sgt_toggle" and k == 2:
            ref.solver.sgl = False
        ref.step(n, residual=res)
    assert summ["dt"] == ref.summary()["dt"]
    for f in fields:
        np.testing.assert_array_equal(got[f], ref.field(f), err_msg=f)


@pytest.mark.parametrize("deck", ["scramjet", "resonator", "step"])
def test_download_after_every_step_leaves_the_trajectory_unchanged(gpu, deck):
    """One-step calls with a download (materialise of the lean N-S /
    mechanism representation) after each: every step is then a re-entry
    split step followed by a materialise, which must give the same trajectory
    as the lean steps of the same calls without downloads (bitwise) and the
    CPU stepper's dt."""
    gen = {"scramjet": lambda: decks.scramjet(214, 48, nmax=10 ** 6, nout=10 ** 5),
           "resonator": lambda: decks.resonator(214, 40, nmax=10 ** 6, nout=10 ** 5),
           "step": lambda: decks.step(214, 80, nmax=10 ** 6, nout=10 ** 5)}[deck]
    cont = gpu.Simulation(gen(), "gpu")
    down = gpu.Simulation(gen(), "gpu")
    cpu = gpu.Simulation(gen(), "cpu")
    for s in range(8):
        cont.step(1)
        down.step(1)
        cpu.step(1)
        down.field("rho")
        assert cont.summary()["dt"] == down.summary()["dt"], s
        assert abs(down.summary()["dt"] / cpu.summary()["dt"] - 1) < 1e-12, s
    lean = (lambda sv: sv.lnm_steps) if deck == "scramjet" else (lambda sv: sv.lns_steps)
    assert lean(cont.solver) > 0 and lean(down.solver) == 0
    for f in FIELDS:
        np.testing.assert_array_equal(cont.field(f), down.field(f), err_msg=f)


@pytest.mark.parametrize("deck", ["scramjet", "resonator", "wedge"])
def test_graph_windows_after_a_download_replay_the_right_buffers(gpu, deck):
    """Step graphs on, a download between calls: the materialise + re-entry
    step shifts the ping-pong parities, so a 6-step window captured before
    the download must not replay after it with the old buffer pointers (it
    did: the lean mechanism run then read the previous level's buffers).
    Equal bitwise to the same calls without downloads and to eager launches."""
    gen = {"scramjet": lambda: decks.scramjet(300, 48, nmax=10 ** 6, nout=10 ** 5),
           "resonator": lambda: decks.resonator(300, 40, nmax=10 ** 6, nout=10 ** 5),
           "wedge": lambda: decks.wedge15(300, 60, nmax=10 ** 6, nout=10 ** 5)}[deck]
    runs = [gpu.Simulation(gen(), "gpu") for _ in range(3)]
    for r in runs:
        r.solver.use_graph = True
    runs[2].solver.use_graph = False
    for n in (24, 11, 24, 13, 24):
        for k, r in enumerate(runs):
            r.step(n)
            if k == 0:
                r.solver.download()   # materialise; the next call re-enters
    assert runs[0].solver.graph_launches > 0 and runs[1].solver.graph_launches > 0
    dt = [r.summary()["dt"] for r in runs]
    assert dt[0] == dt[1] == dt[2], dt
    fields = FIELDS + (["Y:H2", "Y:OH", "mu_t"] if deck == "scramjet" else ["mu_t"] if deck == "resonator" else [])
    for f in fields:
        np.testing.assert_array_equal(runs[0].field(f), runs[1].field(f), err_msg=f)
        np.testing.assert_array_equal(runs[0].field(f), runs[2].field(f), err_msg=f)


@pytest.mark.parametrize("deck,nranks,p2p", [("step", 3, False), ("resonator", 4, False), ("sst_plate", 3, False),
                                            ("scramjet", 8, False), ("resonator", 3, True), ("scramjet", 3, True),
                                            ("resonator", 3, "fx"), ("step", 2, "fx"), ("sst_plate", 3, "fx"),
                                            ("scramjet", 3, "fx"), ("resonator", 4, "fx"), ("resonator", 8, "fx"),
                                            ("scramjet", 4, "fx"), ("scramjet", 8, "fx"), ("scramjet", 4, "fx16")])
def test_lean_ns_strips_match_single_gpu(gpu, deck, nranks, p2p):
    """Lean N-S / mechanism tiles on strips (two ghost columns: the tile
    evaluates the fill of the first one, which reads the second; HALO_LNS
    carries the next lean step's inputs of both, the second column only what
    a neighbour's fill reads) == one GPU bit for bit, across residual steps,
    downloads (materialize) and re-entry, over the in-process and the xGMI
    mailbox transports; p2p="fx": the mailbox exchange fused into the lean
    N-S tile kernel (edge cells push, the last workgroup publishes and folds
    the dt, hf2d_p2p_unpack fills the ghosts), and for the mechanism step
    (whose halo includes the kinetics' state update) the multi-workgroup
    push / unpack pair after it -- asserted to have run."""
    fields = list(FIELDS) + ["k", "mu", "mu_t"]
    if deck == "step":
        text = decks.step(240, 80, nmax=10 ** 6, nout=10 ** 5)
    elif deck == "resonator":
        text = decks.resonator(300, 40, nmax=10 ** 6, nout=10 ** 5)
        fields += ["S7", "S8"]
    elif deck == "sst_plate":
        text = decks.set_key(decks.flat_plate(200, 60, turbulence=6, nmax=10 ** 6, nout=10 ** 5), "isAdiabaticWall", 1)
        fields += ["S7", "S8"]
    else:
        text = decks.scramjet(300, 48, nmax=10 ** 6, nout=10 ** 5)
        fields += ["S7", "S8", "Y:H2", "Y:O2", "Y:OH", "Y:H2O"]
    schedule = [(4, True), (17, False), (5, True), (14, False)]
    stats = {}
    # (mechanism: the edge-first split step is opt-in, lnm_overlap; the fused
    # mailbox case runs the default: all tiles, then push / unpack)
    # ("fx16": the mailbox push kernel with 16 halo values per thread instead of one)
    fx = p2p in ("fx", "fx16")
    setup = (lambda s: setattr(s, "lnm_overlap", True)) if deck == "scramjet" and not fx else None
    if p2p == "fx16":
        setup = lambda s: setattr(s, "push_per", 16)  # noqa: E731
    got, summ = _virtual_ranks(gpu, text, nranks, schedule, lean=True, p2p=bool(p2p), fuse=fx,
                               stats=stats, fields=fields, setup=setup)
    lean_steps = stats["lnm_steps"] if deck == "scramjet" else stats["lns_steps"]
    assert min(lean_steps) > 0, stats
    if fx:
        assert min(stats["p2p_mwg_exchanges" if deck == "scramjet" else "lns_fx_steps"]) > 0, stats
        if deck != "scramjet":   # the next fused step unpacked the halo in its edge tiles
            assert min(stats["lns_prologue_steps"]) > 0, stats
    if not p2p:   # in-process transport: edge tiles first, halo overlapped (mechanism: + their kinetics)
        assert min(stats["overlap_steps"]) > 0, stats
    ref = gpu.Simulation(text, "gpu")
    for n, res in schedule:
        ref.step(n, residual=res)
    assert (ref.solver.lnm_steps if deck == "scramjet" else ref.solver.lns_steps) > 0
    assert summ["dt"] == ref.summary()["dt"]
    assert summ["time"] == ref.summary()["time"]
    for f in fields:
        np.testing.assert_array_equal(got[f], ref.field(f), err_msg=f)


@pytest.mark.parametrize("deck,p2p", [("resonator", False), ("scramjet", False), ("scramjet", "fx"),
                                      ("scramjet_hot", False), ("scramjet_hot", "fx")])
def test_overlap_with_a_one_column_last_tile(gpu, deck, p2p):
    """Strips 97 columns wide: the edge-first launches' last tile column holds
    a single column (97 = 6 x 16 + 1 = 8 x 12 + 1), so the edge part takes the
    last two tile columns (the halo's second column, LeanTile::ne) -- and a
    20-column strip, too narrow to split, runs all its tiles at once while its
    neighbours split (the exchange sequence is the same on every rank).
    'scramjet_hot': ChemTmin 200 K (every active cell on the kinetics lists)
    with 90-column strips, whose last tile column holds 10 columns: the
    interior list starts after the edge part's real cell count, not after
    (1 + ne) full tile columns (which overran the list by 6 columns)."""
    fields = list(FIELDS) + ["k", "mu_t"]
    parts = [(0, 97), (97, 194), (194, 214)]
    if deck == "resonator":
        text = decks.resonator(214, 40, nmax=10 ** 6, nout=10 ** 5)
    elif deck == "scramjet_hot":
        text = decks.with_mechanism(decks.scramjet(214, 48, nmax=10 ** 6, nout=10 ** 5), tmin=200.0)
        fields += ["Y:H2", "Y:OH"]
        parts = [(0, 90), (90, 180), (180, 214)]
    else:
        text = decks.scramjet(214, 48, nmax=10 ** 6, nout=10 ** 5)
        fields += ["Y:H2", "Y:OH"]
    schedule = [(4, True), (13, False), (3, True)]
    stats = {}
    setup = (lambda s: setattr(s, "lnm_overlap", True)) if deck.startswith("scramjet") else None
    got, summ = _virtual_ranks(gpu, text, 3, schedule, lean=True, p2p=bool(p2p), fuse=p2p == "fx", stats=stats,
                               fields=fields, parts=parts, setup=setup)
    assert min(stats["overlap_steps"][:2]) > 0, stats
    ref = gpu.Simulation(text, "gpu")
    for n, res in schedule:
        ref.step(n, residual=res)
    assert summ["dt"] == ref.summary()["dt"]
    for f in fields:
        np.testing.assert_array_equal(got[f], ref.field(f), err_msg=f)


def test_comm_overlap_split_step_matches_single_gpu(gpu):
    """Host-transport strips (the RCCL fallback's structure): edge tiles first,
    their halo on a comm stream while the interior tiles compute, then the dt
    MIN -- bitwise equal to one GPU, and the split path really ran."""
    text = decks.wedge15(480, 60, nmax=10 ** 6, nout=10 ** 5)
    schedule = [(5, True), (16, False), (5, True)]
    stats = {}
    got, summ = _virtual_ranks(gpu, text, 3, schedule, lean=True, stats=stats)
    assert min(stats["overlap_steps"]) > 0, stats
    ref = gpu.Simulation(text, "gpu", lean=True)
    for n, res in schedule:
        ref.step(n, residual=res)
    assert summ["dt"] == ref.summary()["dt"]
    for f in FIELDS:
        np.testing.assert_array_equal(got[f], ref.field(f), err_msg=f)


# In-process ranks need a hardware queue each plus one (conftest sets
# GPU_MAX_HW_QUEUES=16; test_p2p_import_refuses_too_few_queues covers the
# guard); separate processes (the real deployment) have queues of their own.
@pytest.mark.parametrize("nranks,physics,lean,fuse,nt", [(2, "euler", True, False, 256), (3, "euler", True, False, 256),
                                                         (3, "kes", False, True, 256), (2, "euler", True, True, 256),
                                                         (3, "euler", True, True, 256), (3, "euler", True, "toggle", 256),
                                                         (3, "euler", True, True, 64), (2, "euler", True, True, 128),
                                                         (4, "euler", True, True, 256), (8, "euler", True, True, 256),
                                                         (4, "kes", False, True, 256), (8, "euler", True, False, 256)])
def test_p2p_virtual_ranks_match_single_gpu(gpu, nranks, physics, lean, fuse, nt):
    """xGMI mailbox transport (hf2d_p2p_xchg: direct peer stores, system-scope
    flags, device-side dt MIN; fuse: the same exchange folded into the lean
    tile kernel, hf2d_lean_tile_fx + hf2d_p2p_complete) inside captured step
    graphs == one GPU, bit for bit (in-process ranks share the device; the
    protocol is the multi-GPU one)."""
    ns = physics != "euler"
    text = decks.wedge15(240, 60, navier_stokes=ns, turbulence=4 if ns else 0, nmax=10 ** 6, nout=10 ** 5)
    schedule = [(5, True), (30, False), (7, True), (25, False)]
    def setup(s):
        s.lean_nt = nt

    got, summ = _virtual_ranks(gpu, text, nranks, schedule, lean=lean, p2p=True, fuse=fuse is True,
                               toggle=fuse == "toggle", setup=setup)
    ref = gpu.Simulation(text, "gpu", lean=lean)
    for n, res in schedule:
        ref.step(n, residual=res)
    assert summ["dt"] == ref.summary()["dt"]
    assert summ["time"] == ref.summary()["time"]
    for f in FIELDS:
        np.testing.assert_array_equal(got[f], ref.field(f), err_msg=f)


def test_p2p_self_validation_failure_falls_back(gpu):
    """A checksum mismatch in the start-up probe makes every rank drop the
    xGMI mailboxes for the host-side group transport; the poisoned ghost
    columns are refilled and the run still equals one GPU bit for bit."""
    text = decks.wedge15(240, 60, nmax=10 ** 6, nout=10 ** 5)
    schedule = [(5, True), (20, False), (7, True)]
    got, summ = _virtual_ranks(gpu, text, 3, schedule, lean=True, p2p=True, fuse=True, corrupt=True)
    ref = gpu.Simulation(text, "gpu", lean=True)
    for n, res in schedule:
        ref.step(n, residual=res)
    assert summ["dt"] == ref.summary()["dt"]
    for f in FIELDS:
        np.testing.assert_array_equal(got[f], ref.field(f), err_msg=f)


def test_p2p_import_refuses_too_few_queues(gpu):
    """More in-process mailbox ranks than the process's HIP hardware queues
    can co-schedule (n ranks need GPU_MAX_HW_QUEUES >= n + 1): p2p_import
    refuses with a message naming the setting, instead of a start-up probe
    that times out (the round-5 4-rank failure, tools/hwq_probe.py)."""
    import json
    import os
    import subprocess
    import sys

    from tests.conftest import ROOT

    tool = os.path.join(ROOT, "tools", "hwq_probe.py")
    env = dict(os.environ, GPU_MAX_HW_QUEUES="4")
    out = {}
    for n in (3, 4):
        r = subprocess.run([sys.executable, tool, "--ranks", str(n), "--nx", "120", "--ny", "24"], env=env,
                           capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        out[n] = json.loads(r.stdout.strip().splitlines()[-1])
    assert out[3].get("ok") is True, out[3]
    assert "GPU_MAX_HW_QUEUES >= 5" in out[4].get("refused", ""), out[4]


def _p2p_proc_worker(rank, world, port, text, schedule, out):
    import os

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    from openhyperflow2d_amd.parallel.dist import DistributedSimulation

    sim = DistributedSimulation(text, "gpu", rank=rank, world=world, device=0, transport="p2p")
    assert sim.transport == "p2p", sim.transport
    sim.solver.p2p_fuse = True   # fused exchange across processes (IPC-mapped mailboxes)
    sim.solver.use_graph = True  # (the autotune may have turned step graphs off for this grid)
    for n, res in schedule:
        sim.step(n, residual=res)
    fields = {f: sim.gather_field(f) for f in FIELDS}
    if rank == 0:
        np.savez(out, dt=sim.summary()["dt"], graphs=sim.solver.graph_launches, **fields)
    dist.barrier()
    dist.destroy_process_group()


def test_p2p_two_processes_ipc(gpu, tmp_path):
    """Two OS processes (one GPU, gloo bootstrap): mailboxes mapped through
    hipIpcOpenMemHandle, the exact multi-GPU code path; == one GPU bitwise."""
    import socket

    import torch.multiprocessing as mp

    text = decks.wedge15(240, 60, nmax=10 ** 6, nout=10 ** 5)
    schedule = [(5, True), (30, False), (7, True)]
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    out = str(tmp_path / "p2p.npz")
    mp.start_processes(_p2p_proc_worker, args=(2, port, text, schedule, out), nprocs=2, join=True,
                       start_method="spawn")
    got = np.load(out)
    assert int(got["graphs"]) > 0
    ref = gpu.Simulation(text, "gpu")
    for n, res in schedule:
        ref.step(n, residual=res)
    assert float(got["dt"]) == ref.summary()["dt"]
    for f in FIELDS:
        np.testing.assert_array_equal(got[f], ref.field(f), err_msg=f)


def _rccl_proc_worker(rank, world, port, text, schedule, fields, out):
    import os

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    from openhyperflow2d_amd.parallel.dist import DistributedSimulation

    sim = DistributedSimulation(text, "gpu", rank=rank, world=world, device=rank, transport="rccl")
    sim.solver.lnm_overlap = True   # (the mechanism step's edge-first split is opt-in)
    assert sim.transport == "rccl", sim.transport
    for n, res in schedule:
        sim.step(n, residual=res)
    got = {f: sim.gather_field(f) for f in fields}
    ov = [None] * world
    dist.all_gather_object(ov, int(sim.solver.overlap_steps))
    if rank == 0:
        np.savez(out, dt=sim.summary()["dt"], overlap=np.array(ov), **got)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("deck", ["resonator", "scramjet"])
def test_rccl_two_processes_overlap_match_single_gpu(gpu, deck, tmp_path):
    """Two OS processes on two GPUs over RCCL (the truly asynchronous comm
    stream: the edge tiles' halo goes out with ncclSend/ncclRecv on the comm
    stream, ordered after the edge tiles by an event, while the interior tiles
    run; the dt MIN waits for it) == one GPU bitwise, and the split ran on
    both ranks.  RCCL refuses two ranks on one device, so this needs >= 2 GPUs
    (skipped on a one-GPU box; the in-process group covers the same launch
    order with host-ordered copies in test_lean_ns_strips_match_single_gpu)."""
    import socket

    import torch
    import torch.multiprocessing as mp

    if torch.cuda.device_count() < 2:
        pytest.skip("RCCL needs one device per rank")
    fields = list(FIELDS) + ["k", "mu_t"]
    if deck == "resonator":
        text = decks.resonator(300, 40, nmax=10 ** 6, nout=10 ** 5)
    else:
        text = decks.scramjet(300, 48, nmax=10 ** 6, nout=10 ** 5)
        fields += ["Y:H2", "Y:OH"]
    schedule = [(4, True), (17, False), (5, True)]
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    out = str(tmp_path / "rccl.npz")
    mp.start_processes(_rccl_proc_worker, args=(2, port, text, schedule, fields, out), nprocs=2, join=True,
                       start_method="spawn")
    got = np.load(out)
    assert got["overlap"].min() > 0, got["overlap"]
    ref = gpu.Simulation(text, "gpu")
    for n, res in schedule:
        ref.step(n, residual=res)
    assert float(got["dt"]) == ref.summary()["dt"]
    for f in fields:
        np.testing.assert_array_equal(got[f], ref.field(f), err_msg=f)


@pytest.mark.parametrize("name", ["triple_point", "resonator", "scramjet", "step"])
def test_baseline_config_decks_gpu_match_cpu(gpu, name):
    """Small versions of the BASELINE.json config decks (axisymmetric k-eps
    with no-slip tube walls, SST + wall injection, 3-gas triple point,
    laminar N-S step): GPU == CPU Jacobi stepper."""
    size = {"triple_point": (210, 90), "resonator": (300, 40), "scramjet": (450, 40), "step": (240, 80)}[name]
    text = decks.GENERATORS[name](*size, nmax=10 ** 6, nout=10 ** 5)
    g = gpu.Simulation(text, "gpu")
    c = gpu.Simulation(text, "cpu")
    for n, res in [(7, True), (8, False), (5, True)]:
        g.step(n, residual=res)
        c.step(n, residual=res)
    tol = 1e-9 if name != "triple_point" else 1e-12
    for f in FIELDS:
        assert _rel(g.field(f), c.field(f)) < tol, f


@pytest.mark.parametrize("physics", ["euler", "kes"])
def test_step_graphs_bitwise(gpu, physics):
    """Plain steps replayed as captured 6-step hipGraphs (device-side dt,
    time and CFL/beta scenario) == eager launches, bit for bit."""
    ns = physics != "euler"
    text = decks.wedge15(300, 60, navier_stokes=ns, turbulence=4 if ns else 0, nmax=10 ** 6, nout=10 ** 5)
    a = gpu.Simulation(text, "gpu")
    b = gpu.Simulation(text, "gpu")
    a.solver.use_graph = True   # (the autotune picks graphs on / off by speed)
    b.solver.use_graph = False
    for n, res in [(40, False), (13, True), (61, False)]:
        a.step(n, residual=res)
        b.step(n, residual=res)
    assert a.solver.graph_launches > 0
    assert b.solver.graph_launches == 0
    assert a.summary()["dt"] == b.summary()["dt"]
    assert a.summary()["time"] == b.summary()["time"]
    for f in FIELDS + ["k", "R", "CP"]:
        np.testing.assert_array_equal(a.field(f), b.field(f), err_msg=f)


def test_rccl_single_rank_comm(gpu, tmp_path):
    """The RCCL communicator path (ncclCommInitRank, host reductions, strip
    gather for outputs) on a one-rank communicator == no communicator."""
    text = decks.wedge15(200, 40, nmax=30, nout=10)
    a = gpu.Simulation(text, "gpu", workdir=str(tmp_path))
    b = gpu.Simulation(text, "gpu")
    a.solver.init_comm(gpu.native().DeviceSolver.nccl_unique_id(), 0, 1)
    assert a.solver.comm_size() == 1
    for n, res in [(13, False), (7, True), (12, False)]:
        a.step(n, residual=res)
        b.step(n, residual=res)
    for f in FIELDS:
        np.testing.assert_array_equal(a.field(f), b.field(f), err_msg=f)
    a.run(1, str(tmp_path), outputs=True, checkpoint=False, verbose=False)
    assert any(p.suffix == ".plt" for p in tmp_path.iterdir())


@pytest.mark.parametrize("deck", ["step", "step_ref_ns", "step_graphs", "resonator", "resonator_graphs", "sst_plate",
                                  "sst_plate_graphs", "sa_wedge"])
def test_lean_ns_equals_split(gpu, deck):
    """Lean laminar N-S kernel (hip/lean_ns.hpp: fluxes recomputed in the LDS
    tile, one kernel per step) == the split predict + fill kernels on every
    field, dt and time, across entry / materialize / re-entry transitions
    (residual steps, downloads between windows, graph windows)."""
    from tests.conftest import read_deck

    if deck in ("step", "step_graphs"):
        text = decks.step(240, 80, nmax=10 ** 6, nout=10 ** 5)
    elif deck == "step_ref_ns":
        text = decks.set_key(read_deck("Step.dat"), "ProblemType", 1)   # reference deck, laminar N-S
    elif deck.startswith("resonator"):   # axisymmetric k-eps, no-slip tube walls (turbulent lean kernel)
        text = decks.resonator(300, 40, nmax=10 ** 6, nout=10 ** 5)
    elif deck.startswith("sst_plate"):   # k-omega SST kernel
        # (no solid cells: the wall heat kernels have nothing to do)
        text = decks.set_key(decks.flat_plate(200, 60, turbulence=6, nmax=10 ** 6, nout=10 ** 5), "isAdiabaticWall", 1)
    elif deck == "sa_wedge":   # Spalart-Allmaras kernel (the reference's SA blows up after ~55 steps here)
        text = decks.set_key(decks.wedge15(200, 60, navier_stokes=True, turbulence=3, nmax=10 ** 6, nout=10 ** 5),
                             "isAdiabaticWall", 1)
    else:
        text = decks.wedge15(200, 60, navier_stokes=True, turbulence=4, nmax=10 ** 6, nout=10 ** 5)
    a = gpu.Simulation(text, "gpu")
    b = gpu.Simulation(text, "gpu")
    b.solver.lean_ns = False
    graphs = deck.endswith("_graphs")
    if not graphs:
        a.solver.use_graph = b.solver.use_graph = False
    assert a.solver.lns_ok, a.solver.lns_why
    if deck.startswith("sst") or deck.startswith("sa_"):
        assert a.solver.lns_turb == (3 if deck.startswith("sst") else 4)
    sched = [(4, True), (30, False), (6, True), (19, False)] if not graphs else [(40, False), (13, True), (61, False)]
    if deck == "sa_wedge":
        sched = [(4, True), (20, False), (6, True), (10, False)]
    for n, res in sched:
        a.step(n, residual=res)
        b.step(n, residual=res)
        assert a.summary()["dt"] == b.summary()["dt"]
    assert a.solver.lns_steps > 0
    assert b.solver.lns_steps == 0
    assert a.summary()["time"] == b.summary()["time"]
    # residual sums are accumulated per tile instead of per 256-cell block
    np.testing.assert_allclose(a.summary()["rms"], b.summary()["rms"], rtol=1e-12, atol=0)
    for f in FIELDS + ["k", "R", "CP", "mu", "lam", "mu_t", "dUdx", "dTdy", "Diff", "S7", "S8"]:
        np.testing.assert_array_equal(a.field(f), b.field(f), err_msg=f)
    # whole records (fluxes, sources, gradients, ...) after materialization;
    # NaN payloads may differ (the resonator deck carries NaN k/eps in some
    # never-transported cells on both paths)
    ra = np.frombuffer(a.records(), dtype=np.float64).reshape(-1, 156).copy()
    rb = np.frombuffer(b.records(), dtype=np.float64).reshape(-1, 156).copy()
    assert (np.isnan(ra) == np.isnan(rb)).all()
    ra[np.isnan(ra)] = 0
    rb[np.isnan(rb)] = 0
    np.testing.assert_array_equal(ra.view(np.uint64), rb.view(np.uint64))


@pytest.mark.parametrize("deck,mode", [("step", 1), ("step_ref_ns", 1), ("resonator", 2), ("wedge_keps", 2)])
def test_single_gas_ns_specialisation_equals_generic(gpu, deck, mode):
    """Single-gas N-S split kernels (fill_cell/predict_cell_t <SK_SGL> laminar:
    equations 0..3 only; <SK_SGT> turbulent: 0..3 + k, eps) == the generic
    split kernels on every field (+-0 of never-read species fluxes aside),
    dt, time and residuals."""
    from tests.conftest import read_deck

    if deck == "step":
        text = decks.step(240, 80, nmax=10 ** 6, nout=10 ** 5)
    elif deck == "step_ref_ns":
        text = decks.set_key(read_deck("Step.dat"), "ProblemType", 1)   # reference deck, laminar N-S
    elif deck == "resonator":
        text = decks.resonator(300, 40, nmax=10 ** 6, nout=10 ** 5)
    else:
        text = decks.wedge15(200, 60, navier_stokes=True, turbulence=4, nmax=10 ** 6, nout=10 ** 5)
    a = gpu.Simulation(text, "gpu")
    b = gpu.Simulation(text, "gpu")
    b.solver.sgl = False
    a.solver.lean_ns = False   # the split SGL/SGT kernels themselves (lean N-S: test_lean_ns_equals_split)
    assert a.solver.sk_mode == mode, a.solver.sgl_why
    for n, res in [(4, True), (30, False), (6, True), (19, False)]:
        a.step(n, residual=res)
        b.step(n, residual=res)
    assert a.summary()["dt"] == b.summary()["dt"]
    assert a.summary()["time"] == b.summary()["time"]
    np.testing.assert_array_equal(a.summary()["rms"], b.summary()["rms"])
    for f in FIELDS + ["k", "R", "CP", "mu", "lam", "mu_t", "dUdx", "dTdy", "Diff", "S7", "S8"]:
        np.testing.assert_array_equal(a.field(f), b.field(f), err_msg=f)


@pytest.mark.parametrize("physics", ["euler", "ns"])
def test_monitor_probes_device_gather(gpu, tmp_path, physics):
    """K8: monitor probes gathered on the device (hf2d_probe_gather, 16 B per
    probe instead of a full download) == the CPU driver's Monitors-<P>.plt."""
    ns = physics == "ns"
    text = decks.wedge15(200, 40, navier_stokes=ns, nmax=20, nout=5)
    text = decks.set_key(text, "NumMonitorPoints", 3)
    for q, (x, y) in enumerate([(0.05, 0.02), (0.15, 0.035), (0.199, 0.001)]):
        text = decks.set_key(text, "Point-%d.X" % (q + 1), x)
        text = decks.set_key(text, "Point-%d.Y" % (q + 1), y)
    text = decks.set_key(text, "MonitorIndex", 1)
    text = decks.set_key(text, "ExitMonitorValue", 1e-30)
    out = {}
    for be in ("gpu", "cpu"):
        d = tmp_path / be
        d.mkdir()
        s = gpu.Simulation(text, be, workdir=str(d))
        s.run(max_cycles=2, outdir=str(d), checkpoint=False, verbose=False)
        mon = [f for f in d.iterdir() if f.name.startswith("Monitors-")]
        assert mon, list(d.iterdir())
        out[be] = np.loadtxt(mon[0], comments="#")
    assert out["gpu"].shape == out["cpu"].shape and out["gpu"].shape[0] >= 4
    np.testing.assert_allclose(out["gpu"], out["cpu"], rtol=1e-10, atol=0)


def test_autotune_thread_block_size_zero(gpu, monkeypatch):
    """ThreadBlockSize = 0 (reference: auto-calibrate) times the lean tile
    geometries on the device before the first step; the run is unchanged."""
    text = decks.wedge15(300, 60, nmax=10 ** 6, nout=10 ** 5)
    a = gpu.Simulation(text, "gpu")
    assert "best nt=" in a.autotune_log and "nt=64 cpt=1" in a.autotune_log, a.autotune_log
    monkeypatch.setenv("HF2D_AUTOTUNE", "0")
    b = gpu.Simulation(text, "gpu")
    assert b.autotune_log == ""
    for n, res in [(5, True), (40, False), (7, True)]:
        a.step(n, residual=res)
        b.step(n, residual=res)
    assert a.summary()["dt"] == b.summary()["dt"] and a.summary()["iteration"] == b.summary()["iteration"]
    assert a.summary()["time"] == b.summary()["time"]
    for f in FIELDS:
        np.testing.assert_array_equal(a.field(f), b.field(f), err_msg=f)


@pytest.mark.parametrize("deck", ["step", "resonator"])
def test_autotune_lean_ns_tile_height(gpu, monkeypatch, deck):
    """The lean N-S tile height is tuned too (one cell per thread); the tuning
    steps leave no trace: same fields, dt and time as an untuned run, and the
    tuned run's lean steps are the run's own."""
    text = decks.step(240, 80, nmax=10 ** 6, nout=10 ** 5) if deck == "step" else \
        decks.resonator(300, 40, nmax=10 ** 6, nout=10 ** 5)
    a = gpu.Simulation(text, "gpu")
    assert "best nt=256 cpt=1 tj=" in a.autotune_log, a.autotune_log
    assert a.solver.lns_steps == 0
    monkeypatch.setenv("HF2D_AUTOTUNE", "0")
    b = gpu.Simulation(text, "gpu")
    assert b.autotune_log == ""
    for n, res in [(4, True), (30, False), (6, True)]:
        a.step(n, residual=res)
        b.step(n, residual=res)
    assert a.solver.lns_steps > 0
    assert a.summary()["dt"] == b.summary()["dt"] and a.summary()["time"] == b.summary()["time"]
    for f in FIELDS:
        np.testing.assert_array_equal(a.field(f), b.field(f), err_msg=f)


@pytest.mark.parametrize("stagger", [0, 150, -300])
def test_tile_stagger_is_timing_only(gpu, monkeypatch, stagger):
    """The staggered start of the tile kernel's dispatch rounds (HF2D_STAGGER,
    whole rounds or a ramp) delays workgroups only: bitwise the same run."""
    text = decks.wedge15(600, 80, nmax=10 ** 6, nout=10 ** 5)
    monkeypatch.setenv("HF2D_AUTOTUNE", "0")
    ref = gpu.Simulation(text, "gpu")
    ref.solver.tile_stagger = 0
    monkeypatch.setenv("HF2D_STAGGER", str(stagger))
    s = gpu.Simulation(text, "gpu")
    assert s.solver.tile_stagger == stagger
    s.solver.lean_cpt = ref.solver.lean_cpt = 2
    for n, res in [(5, True), (25, False), (3, True)]:
        s.step(n, residual=res)
        ref.step(n, residual=res)
    assert s.summary()["dt"] == ref.summary()["dt"]
    for f in FIELDS:
        np.testing.assert_array_equal(s.field(f), ref.field(f), err_msg=f)


@pytest.mark.parametrize("mode,nt,graphs", [(0, 256, True), (2, 256, True), (2, 64, False), (2, 128, True)])
def test_tile_dt_read_modes_match_cpu(gpu, monkeypatch, mode, nt, graphs):
    """How the tile kernel reads the step's dt (StepParams::dt_read): one
    vector load per lane of the word + 16 shards (1), or the one word that the
    previous step's last workgroup folded the shards into (2, dt_fold) -- the
    same MIN, so the dt sequence and the fields equal the CPU stepper bit for
    bit across residual steps, one-step calls (host mirror tail), downloads
    and graph windows."""
    text = decks.wedge15(600, 80, nmax=10 ** 6, nout=10 ** 5)
    monkeypatch.setenv("HF2D_AUTOTUNE", "0")
    g = gpu.Simulation(text, "gpu")
    g.solver.dt_read_mode = mode
    g.solver.lean_nt = nt
    g.solver.use_graph = graphs
    c = gpu.Simulation(text, "cpu")
    for n, res in [(1, False), (5, True), (25, False), (1, False), (13, False), (3, True), (12, False)]:
        g.step(n, residual=res)
        c.step(n, residual=res)
        assert g.summary()["dt"] == c.summary()["dt"], n
    assert g.summary()["time"] == c.summary()["time"]
    for f in FIELDS:
        np.testing.assert_array_equal(g.field(f), c.field(f), err_msg=f)


@pytest.mark.parametrize("multigas", [False, True])
def test_tile_skip_same_stores_match_cpu(gpu, monkeypatch, multigas):
    """StepParams::skip_same: the tile kernel skips the stores of beta and CP
    whose new bits equal the old ones (the in-place arrays then hold the same
    bits either way): GPU == CPU bit for bit, fields, dt, beta and CP included,
    single gas and the multi-gas (3-species) tile kernel."""
    text = decks.wedge15(600, 80, nmax=10 ** 6, nout=10 ** 5)
    if multigas:
        text = decks.triple_point(300, 80, nmax=10 ** 6, nout=10 ** 5)
    monkeypatch.setenv("HF2D_AUTOTUNE", "0")
    g = gpu.Simulation(text, "gpu")
    g.solver.tile_skip_same = True
    c = gpu.Simulation(text, "cpu")
    for n, res in [(1, False), (5, True), (40, False), (3, True), (30, False)]:
        g.step(n, residual=res)
        c.step(n, residual=res)
        assert g.summary()["dt"] == c.summary()["dt"], n
    for f in FIELDS + ["CP", "R"]:
        np.testing.assert_array_equal(g.field(f), c.field(f), err_msg=f)
    rg = np.frombuffer(g.records(), dtype=np.uint8).reshape(-1, 1248).copy()
    rc = np.frombuffer(c.records(), dtype=np.uint8).reshape(-1, 1248).copy()
    rg[:, 72:216] = 0   # dS/dx, dS/dy scratch
    rc[:, 72:216] = 0
    np.testing.assert_array_equal(rg, rc)


def _lagged(text):
    return decks.set_key(text, "LaggedDt", 1)


@pytest.mark.parametrize("deck", ["wedge", "resonator", "scramjet_transport"])
def test_lagged_dt_gpu_equals_cpu(gpu, deck):
    """LaggedDt = 1 (step n + 1 runs with the MIN of step n - 1): the device
    slots (DevScalars::dt_lag, lag_head in every step's first kernel) give the
    CPU stepper's dt sequence and fields bit for bit, across residual steps,
    downloads and graph windows -- lean tile, lean N-S and lean mechanism
    kernels (kinetics off: ChemTmin above every temperature)."""
    if deck == "wedge":
        text = decks.wedge15(200, 40, nmax=10 ** 6, nout=10 ** 5)
    elif deck == "resonator":
        text = decks.resonator(214, 40, nmax=10 ** 6, nout=10 ** 5)
    else:
        text = decks.with_mechanism(decks.scramjet(150, 48, nmax=10 ** 6, nout=10 ** 5), tmin=1e9)
    text = _lagged(text)
    g = gpu.Simulation(text, "gpu")
    c = gpu.Simulation(text, "cpu")
    for n, res in [(1, False), (1, True), (9, False), (4, True), (20, False)]:
        g.step(n, residual=res)
        c.step(n, residual=res)
        assert g.summary()["dt"] == c.summary()["dt"], n
    assert g.summary()["time"] == c.summary()["time"]
    for f in FIELDS:
        np.testing.assert_array_equal(g.field(f), c.field(f), err_msg=f)
    std = gpu.Simulation(decks.set_key(text, "LaggedDt", 0), "gpu")
    std.step(35)
    assert std.summary()["dt"] != g.summary()["dt"]


@pytest.mark.parametrize("deck,nranks,p2p", [("wedge", 4, "fx"), ("wedge", 8, "fx"), ("wedge", 3, "fx"),
                                            ("wedge", 3, False), ("resonator", 3, "fx"), ("resonator", 4, "fx"),
                                            ("resonator", 8, "fx")])
def test_lagged_dt_strips_match_single_gpu(gpu, deck, nranks, p2p):
    """Lagged dt on strips: with the fused mailbox exchange the tail of a
    step waits for its two neighbours only and the next step's first
    workgroup folds the other ranks' dt (hf2d_p2p_complete before any other
    consumer); N strips == one GPU bit for bit."""
    if deck == "wedge":
        text = _lagged(decks.wedge15(300, 60, nmax=10 ** 6, nout=10 ** 5))
    else:
        text = _lagged(decks.resonator(300, 40, nmax=10 ** 6, nout=10 ** 5))
    schedule = [(4, True), (17, False), (5, True), (14, False)]
    stats = {}
    got, summ = _virtual_ranks(gpu, text, nranks, schedule, lean=True, p2p=bool(p2p), fuse=p2p == "fx",
                               stats=stats)
    ref = gpu.Simulation(text, "gpu")
    for n, res in schedule:
        ref.step(n, residual=res)
    assert summ["dt"] == ref.summary()["dt"]
    assert summ["time"] == ref.summary()["time"]
    for f in FIELDS:
        np.testing.assert_array_equal(got[f], ref.field(f), err_msg=f)


def test_wall_blend_gpu_equals_cpu(gpu):
    """WallBlendCells (near-wall blend of the tangential momentum, GF_WBX /
    GF_WBY from the global wall list) runs on the split predict / fill path
    (the lean tile kernels compile the blend out): == the CPU stepper bit for
    bit, and it differs from the reference scheme."""
    text = decks.set_key(decks.flat_plate(120, 80, dx=1e-3, dy=4e-5, p=1e4, turbulence=6, nmax=10 ** 6, nout=10 ** 5),
                         "isAdiabaticWall", 1)
    on = decks.set_key(text, "WallBlendCells", 12)
    g = gpu.Simulation(on, "gpu")
    c = gpu.Simulation(on, "cpu")
    r = gpu.Simulation(text, "gpu")
    for n, res in [(3, True), (40, False), (5, True)]:
        g.step(n, residual=res)
        c.step(n, residual=res)
        r.step(n, residual=res)
    assert g.solver.lns_steps == 0 and "WallBlendCells" in g.solver.lns_why
    assert g.summary()["dt"] == c.summary()["dt"]
    for f in FIELDS + ["mu_t"]:
        np.testing.assert_array_equal(g.field(f), c.field(f), err_msg=f)
    assert not np.array_equal(g.field("U"), r.field("U"))
