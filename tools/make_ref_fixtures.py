"""Record golden hashes of the reference solver's outputs for small decks.

Run where a serial build of the reference exists (built from its sources in a
scratch directory with -O2 -ffp-contract=off):

  python tools/make_ref_fixtures.py --ref /tmp/refexact/bin/OpenHyperFLOW2D-1.03

For every case the deck actually run is stored as tests/fixtures/ref/<case>/deck.dat
and the sha256 of every output file (.plt, .hf2d) in sha256.json.  The tests
(tests/test_reference_golden.py) run our reference-order backend on the same
deck and require byte-identical outputs.
"""
import argparse
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from openhyperflow2d_amd.models import decks  # noqa: E402

FIX = os.path.join(ROOT, "tests", "fixtures")


def _fixture_deck(name):
    with open(os.path.join(FIX, "decks", name), errors="replace") as f:
        return f.read()


def _finite(text, nmax, nout=None):
    """Run exactly one outer cycle of nmax steps (exit monitor forced)."""
    t = decks.set_key(text, "Nmax", nmax)
    t = decks.set_key(t, "NOutStep", nout or max(1, nmax // 4))
    t = decks.set_key(t, "MonitorIndex", 5)
    t = decks.set_key(t, "ExitMonitorValue", 1e-30)
    return t


def cases():
    return {
        "wedge15_200x40_euler": _finite(decks.wedge15(200, 40, nmax=101, nout=25), 101, 25),
        "oblique_shock": _finite(_fixture_deck("ObliqueShock.dat"), 40),
        "step_euler": _finite(_fixture_deck("Step.dat"), 20),
        "wedge_keps_wallheat": _finite(_fixture_deck("Wedge.dat"), 30),
        "wedge15_200x60_ns_keps": _finite(decks.wedge15(200, 60, navier_stokes=True, turbulence=4,
                                                        nmax=30, nout=10), 30, 10),
    }


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/tmp/refexact/bin/OpenHyperFLOW2D-1.03")
    ap.add_argument("--only", nargs="*")
    a = ap.parse_args()
    for name, text in cases().items():
        if a.only and name not in a.only:
            continue
        d = os.path.join(FIX, "ref", name)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "deck.dat"), "w") as f:
            f.write(text)
        with tempfile.TemporaryDirectory() as tmp:
            shutil.copy(os.path.join(d, "deck.dat"), tmp)
            r = subprocess.run([a.ref, "deck.dat"], cwd=tmp, capture_output=True, text=True, errors="replace",
                               timeout=1800)
            outs = sorted(f for f in os.listdir(tmp) if f.endswith((".plt", ".hf2d")))
            rec = {f: sha256(os.path.join(tmp, f)) for f in outs}
            rec["_returncode"] = r.returncode
        with open(os.path.join(d, "sha256.json"), "w") as f:
            json.dump(rec, f, indent=1, sort_keys=True)
        print(name, r.returncode, outs)


if __name__ == "__main__":
    main()
