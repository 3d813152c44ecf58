"""Record hashes of the CPU Jacobi stepper's state after a few steps on the
viscous/turbulent/reacting decks, so optimisations of the shared per-cell
code can be checked to be bit-exact (tests/test_jacobi_regression.py).

Masked before hashing: dS/dx, dS/dy scratch (only maintained where a Cauchy
node reads it) and, for flat cases, the axisymmetric source F (never read)."""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from openhyperflow2d_amd.models import decks  # noqa: E402

CASES = {
    "wedge15_ns_keps": (lambda: decks.wedge15(120, 50, navier_stokes=True, turbulence=4, nmax=10 ** 6, nout=10 ** 5), 12),
    "wedge15_ns_lam": (lambda: decks.wedge15(120, 50, navier_stokes=True, turbulence=0, nmax=10 ** 6, nout=10 ** 5), 12),
    "resonator": (lambda: decks.resonator(300, 40, nmax=10 ** 6, nout=10 ** 5), 12),
    "scramjet_sst": (lambda: decks.scramjet(450, 40, nmax=10 ** 6, nout=10 ** 5, turbulence=6, mechanism=None), 12),
    "scramjet_mech": (lambda: decks.scramjet(450, 40, nmax=10 ** 6, nout=10 ** 5, turbulence=6), 12),
    "step_ns": (lambda: decks.step(240, 80, nmax=10 ** 6, nout=10 ** 5), 12),
    "triple_point": (lambda: decks.triple_point(210, 90, nmax=10 ** 6, nout=10 ** 5), 12),
    "reactor0d": (lambda: decks.reactor0d(T=1200.0), 12),
}


def masked_hash(sim) -> str:
    r = np.frombuffer(sim.records(), dtype=np.uint8).reshape(-1, 1248).copy()
    r[:, 72:216] = 0
    if sim.case.flow_type == 0:
        r[:, 544 + 2 * 72:544 + 3 * 72] = 0   # F
    return hashlib.sha256(r.tobytes()).hexdigest()


def run_case(hf, name):
    mk, steps = CASES[name]
    s = hf.Simulation(mk(), "cpu", lean=False)
    s.step(steps // 2, residual=True)
    s.step(steps - steps // 2, residual=True)
    return masked_hash(s)


def main():
    import openhyperflow2d_amd as hf

    out = {name: run_case(hf, name) for name in CASES}
    path = os.path.join(ROOT, "tests", "fixtures", "jacobi_hashes.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
