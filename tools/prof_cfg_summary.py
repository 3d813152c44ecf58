"""Summarise tools/gpu_prof_cfg.sh output for one config as markdown:
kernel median time (kernel trace) + HBM bytes and VALU instructions per cell
(PMC; FETCH_SIZE counts half the read bytes on MI355X, calibrated with
tools/bw_calibrate.py).   python tools/prof_cfg_summary.py <config> <cells>"""
import collections
import csv
import sqlite3
import statistics as st
import sys


def main():
    cfg, cells = sys.argv[1], float(sys.argv[2])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in "fws":
        for r in csv.DictReader(open("gpurun_out/pmc_%s/%s_counter_collection.csv" % (cfg, f))):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = collections.defaultdict(list)
    c = sqlite3.connect("gpurun_out/prof_%s/k_results.db" % cfg)
    for name, s, e in c.execute("select name, start, end from kernels order by start"):
        dur[name.split("(")[0].replace("void ", "")].append((e - s) / 1e3)
    print("| kernel | median us | read B/cell | write B/cell | TB/s | VALU instr/cell |")
    print("|---|---:|---:|---:|---:|---:|")
    for k, d in agg.items():
        if "hf2d" not in k or k not in dur:
            continue
        m = {n: st.median(v) for n, v in d.items()}
        rd = m.get("FETCH_SIZE", 0) * 2048 / cells
        wr = m.get("WRITE_SIZE", 0) * 1024 / cells
        us = st.median(dur[k])
        print("| `%s` | %.1f | %.0f | %.0f | %.2f | %.0f |" % (k, us, rd, wr, (rd + wr) * cells / (us * 1e-6) / 1e12,
                                                            m.get("SQ_INSTS_VALU", 0) * 64 / cells))


if __name__ == "__main__":
    main()
