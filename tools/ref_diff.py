"""Run a fixture deck through the reference oracle binary and our reference-order
backend side by side and report the first differing line of every output file.

  python tools/ref_diff.py tests/fixtures/ref/<case> [--ref /tmp/refexact/bin/OpenHyperFLOW2D-1.03]
"""
import argparse
import json
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case")
    ap.add_argument("--ref", default="/tmp/refexact/bin/OpenHyperFLOW2D-1.03")
    a = ap.parse_args()
    want = json.load(open(os.path.join(a.case, "sha256.json")))
    runs = want.get("_runs", 1)
    cli = os.path.join(ROOT, "openhyperflow2d_amd", "bin", "hf2d_cpu")
    with tempfile.TemporaryDirectory() as t:
        A, B = os.path.join(t, "ref"), os.path.join(t, "ours")
        for d, cmd in ((A, [a.ref, "deck.dat"]), (B, [cli, "--backend", "ref", "--semantics", "serial", "deck.dat"])):
            os.makedirs(d)
            shutil.copy(os.path.join(a.case, "deck.dat"), d)
            for _ in range(runs):
                r = subprocess.run(cmd, cwd=d, capture_output=True, text=True, errors="replace")
            open(os.path.join(d, "stdout.txt"), "w").write(r.stdout)
        for f in sorted(os.listdir(A)):
            if not f.endswith(".plt"):
                continue
            pa, pb = os.path.join(A, f), os.path.join(B, f)
            if not os.path.exists(pb):
                print(f, "MISSING in ours")
                continue
            la, lb = open(pa, errors="replace").read().splitlines(), open(pb, errors="replace").read().splitlines()
            for i, (x, y) in enumerate(zip(la, lb)):
                if x != y:
                    print("%s line %d:\n  ref : %s\n  ours: %s" % (f, i + 1, x[:200], y[:200]))
                    break
            else:
                print(f, "same" if len(la) == len(lb) else "length %d vs %d" % (len(la), len(lb)))


if __name__ == "__main__":
    main()
