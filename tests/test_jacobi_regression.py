"""The CPU Jacobi stepper (whose per-cell code the HIP kernels share) must
keep producing bit-identical states on the viscous / turbulent / reacting /
multi-gas decks (hashes recorded with tools/make_jacobi_fixtures.py)."""
import json
import os

import pytest

from tests.conftest import FIXTURES

HASHES = json.load(open(os.path.join(FIXTURES, "jacobi_hashes.json")))


@pytest.mark.parametrize("name", sorted(HASHES))
def test_jacobi_state_hash(hf, name):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(FIXTURES), "..", "tools"))
    from make_jacobi_fixtures import run_case

    assert run_case(hf, name) == HASHES[name]
