"""K12 MFMA mechanism chemistry benchmark: one chemistry call on a scramjet-sized
field (6000x400 = 2.4 M cells, demo 8-species / 12-step H2-air mechanism), checked on
a cell subset against the PyTorch FP64 reference.  Prints one JSON line."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from openhyperflow2d_amd.ops import chemistry as ch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=6000)
    ap.add_argument("--ny", type=int, default=400)
    ap.add_argument("--nsub", type=int, default=4)
    ap.add_argument("--dt", type=float, default=1e-7)
    ap.add_argument("--repeats", type=int, default=10)
    ap.add_argument("--mech", help="mechanism JSON (Mechanism.save format); default: demo H2-air set")
    a = ap.parse_args()
    m = ch.Mechanism.load(a.mech) if a.mech else ch.h2_air_demo()
    res = ch.benchmark(m, a.nx * a.ny, a.dt, a.nsub, a.repeats)
    print(json.dumps(res))
    err = res["rel_err_vs_torch_fp64"]
    if not err < 1e-10:
        raise SystemExit("mismatch vs reference: %g" % err)


if __name__ == "__main__":
    main()
