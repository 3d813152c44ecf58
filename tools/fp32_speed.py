#!/usr/bin/env python3
"""Step rate of the FP32 GPU build (bin/hf2d_fp32) against the FP64 one
(bin/hf2d) on the headline deck (Wedge15 2000x200, inviscid), through the
native CLI: one cycle of N steps each for two N, the per-step time from the
difference of the CLI's cycle times (the cycle time also holds the end-of-cycle
field download, which the difference cancels).  A separate measurement -- the
headline metric is FP64, as the reference's default build.

  python tools/fp32_speed.py [--steps 2000,12000] [--nx 2000 --ny 200]"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", default="2000,12000")
    ap.add_argument("--nx", type=int, default=2000)
    ap.add_argument("--ny", type=int, default=200)
    a = ap.parse_args()
    from openhyperflow2d_amd.models import decks

    n1, n2 = (int(x) for x in a.steps.split(","))
    res = {"grid": [a.nx, a.ny], "steps": [n1, n2]}

    def cycle_seconds(exe, n):
        text = decks.wedge15(a.nx, a.ny, nmax=n, nout=n)
        with tempfile.TemporaryDirectory() as d:
            open(os.path.join(d, "d.dat"), "w").write(text)
            r = subprocess.run([os.path.join(ROOT, "openhyperflow2d_amd", "bin", exe), "--backend", "gpu", "--cycles",
                                "1", "d.dat"], cwd=d, capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                raise RuntimeError(r.stdout[-2000:] + r.stderr[-2000:])
            return float(re.findall(r"cycle time=([0-9.eE+-]+) sec", r.stdout)[-1])

    for tag, exe in (("fp64", "hf2d"), ("fp32", "hf2d_fp32")):
        t1, t2 = cycle_seconds(exe, n1), cycle_seconds(exe, n2)
        us = (t2 - t1) / (n2 - n1) * 1e6
        res[tag] = {"cycle_s": [t1, t2], "us_per_step": us, "mcells_it_per_s": a.nx * a.ny / us}
    res["speedup_fp32"] = res["fp64"]["us_per_step"] / res["fp32"]["us_per_step"]
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
