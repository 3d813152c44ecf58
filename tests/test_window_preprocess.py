"""Strip-local pre-processing (no whole-field copy anywhere).

Case.from_deck_window runs the pre-processor with 1248-byte records for a
column window only and the whole grid's CT / TurbType words in a 16 B/cell
plane (case.hpp Field::ct/tt); Case.partition_deck cuts the strips from a
flags-only pass.  The reference instead pre-processes the whole field on rank
0 and sends every rank its subdomain (hf2d_start.cpp:115-116,143-205), which
the strip runs here no longer do.  These tests pin that the windowed records
are byte-identical to the same columns of the whole-field pre-processing, for
every reference fixture deck (contours, rects, circles, airfoils, areas,
sources, NRBC, boundary layers, wall distance, y+, k-eps / SA / SST / ...,
Zeldovich chemistry) and the generated BASELINE configs (mechanism mode
included), that the merged per-strip facts equal the whole field's, and that
a restart reads each rank's slab of the .hf2d (and of the species sidecar)."""
import os
import shutil

import numpy as np
import pytest

from openhyperflow2d_amd.models import decks
from openhyperflow2d_amd.parallel.strips import balanced_columns
from tests.conftest import FIXTURES

REC = 1248
REF = sorted(os.listdir(os.path.join(FIXTURES, "ref")))


def _stage(case, tmp_path):
    d = os.path.join(FIXTURES, "ref", case)
    for fn in os.listdir(d):
        if fn != "sha256.json":
            shutil.copy(os.path.join(d, fn), tmp_path / fn)
    return (tmp_path / "deck.dat").read_text()


def _check_windows(nat, text, workdir, nparts, use_checkpoint=False):
    full = nat.Case.from_deck(text, workdir, use_checkpoint)
    full.compute_facts()
    ny, nx = full.ny, full.nx
    whole = full.resident_records()
    parts = nat.Case.partition_deck(text, workdir, use_checkpoint, nparts)
    assert [tuple(p) for p in parts] == balanced_columns(np.asarray(full.field("solid")), nparts)
    strips, blobs = [], []
    for a, b in parts:
        lo, hi = max(a - 1, 0), min(b + 1, nx)
        c = nat.Case.from_deck_window(text, workdir, use_checkpoint, lo, hi)
        assert c.resident_columns == (lo, hi)
        got = c.resident_records()
        want = whole[lo * ny * REC:hi * ny * REC]
        if got != want:   # name the first differing cell
            k = next(q for q in range(0, len(got), REC) if got[q:q + REC] != want[q:q + REC]) // REC
            pytest.fail("window [%d, %d): record (%d, %d) differs" % (lo, hi, lo + k // ny, k % ny))
        assert c.wall_nodes == full.wall_nodes
        assert c.global_time == full.global_time and c.dt0 == full.dt0
        if full.mech_mode:
            sp = np.asarray(full.resident_species()).reshape(-1, nx * ny)
            np.testing.assert_array_equal(np.asarray(c.resident_species()).reshape(-1, (hi - lo) * ny),
                                          sp[:, lo * ny:hi * ny])
        strips.append(c)
        blobs.append(c.facts_part())
    for c in strips:
        c.merge_facts(blobs)
        assert c.facts == full.facts
    return full, strips


@pytest.mark.parametrize("case", REF)
def test_windowed_preprocessing_matches_the_whole_field(hf, case, tmp_path):
    text = _stage(case, tmp_path)
    _check_windows(hf.native(), text, str(tmp_path), 3)


@pytest.mark.parametrize("name", ["step", "resonator", "triple_point", "scramjet"])
def test_windowed_preprocessing_of_the_baseline_configs(hf, name, tmp_path):
    text = decks.GENERATORS[name](160, 48, nmax=10 ** 6, nout=10 ** 5)
    _check_windows(hf.native(), text, str(tmp_path), 4)


def test_merged_facts_name_the_first_failing_cell(hf, tmp_path):
    """lean inviscid eligibility fails on a gas source: the merged reason is
    the whole field's (deck-level reasons win over cell-level ones), and a
    k-eps deck's split-kernel mode is SK_SGT on every strip."""
    nat = hf.native()
    for text in (decks.wedge15(120, 40, navier_stokes=True, turbulence=4, nmax=10, nout=5),
                 open(os.path.join(FIXTURES, "ref", "gas_source", "deck.dat")).read()):
        _check_windows(nat, text, str(tmp_path), 5)


@pytest.mark.parametrize("mech,reset", [(False, False), (True, False), (False, True)])
def test_windowed_restart_reads_the_rank_slab(hf, mech, reset, tmp_path):
    """A restart of a strip rank reads its own slab of the .hf2d (and of the
    species sidecar), plus the flag words of the other columns: the records
    equal the whole-field restart's columns.  reset: the restart runs with
    isTurbulenceReset = 1, so the wall records another strip owns (read for
    y+) must get scan_area's turbulence reset too."""
    if mech:
        text = decks.scramjet(96, 32, nmax=6, nout=3)
    else:
        text = decks.wedge15(96, 30, navier_stokes=True, turbulence=4, nmax=6, nout=3)
    sim = hf.Simulation(text, "cpu", workdir=str(tmp_path))
    sim.run(max_cycles=1, outdir=str(tmp_path), verbose=False)
    assert any(p.suffix == ".hf2d" for p in tmp_path.iterdir())
    if reset:
        text = decks.set_key(decks.set_key(text, "isTurbulenceReset", 1), "TurbulenceModel", 6)
    full, strips = _check_windows(hf.native(), text, str(tmp_path), 3, use_checkpoint=True)
    assert full.field("rho").any() and all(c.global_time == full.global_time for c in strips)
