"""K12 kinetics benchmark: one kinetics call on a scramjet-sized field (6000x400 =
2.4 M cells, the built-in 9-species / 21-step Li et al. H2/air mechanism) with the
compiled VALU kernel, the runtime-mechanism MFMA kernel and the same runtime-data
operator on the vector ALUs (the MFMA kernel's equal-terms baseline), each checked on a cell
subset against the NumPy FP64 oracle.  Prints one JSON line per kernel."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from openhyperflow2d_amd.ops import chemistry as ch  # noqa: E402
from openhyperflow2d_amd.ops import mechanism as mech  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=6000)
    ap.add_argument("--ny", type=int, default=400)
    ap.add_argument("--nsub", type=int, default=1)
    ap.add_argument("--dt", type=float, default=1e-7)
    ap.add_argument("--repeats", type=int, default=10)
    ap.add_argument("--mech", help="mechanism file; default: built-in H2/air")
    a = ap.parse_args()
    m = mech.Mechanism.load(a.mech) if a.mech else mech.h2_air_li2004()
    bad = False
    for k in (["fast", "mfma", "valu"] if not a.mech else ["mfma", "valu"]):
        res = ch.benchmark(m, a.nx * a.ny, a.dt, a.nsub, a.repeats, kernel=k)
        print(json.dumps(res), flush=True)
        bad = bad or not res["incr_err_vs_numpy_fp64"] < 1e-8
    if bad:
        raise SystemExit("mismatch vs the FP64 oracle")


if __name__ == "__main__":
    main()
