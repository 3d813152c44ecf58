#!/usr/bin/env python3
"""Markdown table of a rocprofv3 --kernel-trace CSV: per kernel (name + grid
+ workgroup, so autotune candidates stay apart) the call count, median and
minimum duration, VGPRs, LDS and scratch, and the share of the total.

  python tools/ktrace_summary.py gpurun_out/prof_bench/run_kernel_trace.csv [--top 15] [--last N]
--last N keeps only the last N dispatches of each kernel (the timed steps of a
bench run rather than its autotune / warm-up)."""
import argparse
import collections
import csv
import statistics as st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--last", type=int, default=0)
    a = ap.parse_args()
    rows = collections.defaultdict(list)
    info = {}
    for r in csv.DictReader(open(a.csv)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hf2d::", "")
        key = (name, int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
        rows[key].append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
        info[key] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"])
    tot = {}
    for k, v in rows.items():
        v.sort()
        d = [x[1] for x in (v[-a.last:] if a.last else v)]
        tot[k] = (len(d), sum(d), st.median(d), min(d))
    allt = sum(t[1] for t in tot.values()) or 1.0
    print("| kernel | grid | wg | calls | median us | min us | VGPR | AGPR | SGPR | LDS B | scratch B | share |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k, (n, s, med, mn) in sorted(tot.items(), key=lambda kv: -kv[1][1])[: a.top]:
        vg, ag, sg, lds, scr = info[k]
        print("| `%s` | %d | %d | %d | %.2f | %.2f | %s | %s | %s | %s | %s | %.1f %% |"
              % (k[0], k[1] // max(k[2], 1), k[2], n, med, mn, vg, ag, sg, lds, scr, 100 * s / allt))


if __name__ == "__main__":
    main()
