"""Byte-for-byte parity with the reference solver.

tests/fixtures/ref/<case>/sha256.json holds the hashes of the outputs the
reference (serial build of /root/reference compiled from source in scratch,
-O2 -ffp-contract=off; tools/make_ref_fixtures.py) wrote for deck.dat.  Our
reference-order backend (RefSolver, CLI `hf2d --backend ref --semantics
serial`) must write identical bytes: field dump, RMS history, transient
append file and the 1248-byte-per-cell .hf2d checkpoint.
"""
import hashlib
import json
import os
import shutil
import subprocess

import pytest

from tests.conftest import FIXTURES, ROOT

CASES = sorted(os.listdir(os.path.join(FIXTURES, "ref")))


def _sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


@pytest.fixture(scope="module")
def cli(hf):
    exe = os.path.join(ROOT, "openhyperflow2d_amd", "bin", "hf2d_cpu")
    assert os.path.exists(exe), "build the native CLI first (python -m openhyperflow2d_amd._build)"
    return exe


@pytest.mark.parametrize("case", CASES)
def test_reference_outputs_bitwise(case, cli, tmp_path):
    d = os.path.join(FIXTURES, "ref", case)
    want = json.load(open(os.path.join(d, "sha256.json")))
    shutil.copy(os.path.join(d, "deck.dat"), tmp_path / "deck.dat")
    r = subprocess.run([cli, "--backend", "ref", "--semantics", "serial", "deck.dat"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == want["_returncode"], r.stdout[-2000:] + r.stderr[-2000:]
    for name, h in want.items():
        if name.startswith("_"):
            continue
        p = tmp_path / name
        assert p.exists(), name
        assert _sha(p) == h, "%s differs from the reference" % name
