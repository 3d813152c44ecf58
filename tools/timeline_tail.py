"""Tail of a rocprofv3 kernel + memory-copy trace as a timeline (us relative
to the first listed event): where the fixed cost of a short timed region goes.

  python tools/timeline_tail.py gpurun_out/tl/run [--n 40]
reads <prefix>_kernel_trace.csv and <prefix>_memory_copy_trace.csv.
"""
import argparse
import csv
import os


def load(path, kind):
    if not os.path.exists(path):
        return []
    out = []
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Direction") or kind
        out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, name.split("(")[0][:70]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("--n", type=int, default=40)
    a = ap.parse_args()
    ev = load(a.prefix + "_kernel_trace.csv", "K") + load(a.prefix + "_memory_copy_trace.csv", "M")
    ev.sort()
    ev = ev[-a.n:]
    t0 = ev[0][0]
    prev_end = None
    print("| start us | dur us | gap us | kind | name |\n|---:|---:|---:|---|---|")
    for s, e, k, n in ev:
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        print("| %.2f | %.2f | %.2f | %s | %s |" % ((s - t0) / 1e3, (e - s) / 1e3, gap, k, n))
        prev_end = e if prev_end is None else max(prev_end, e)


if __name__ == "__main__":
    main()
