"""Per-kernel duration and dispatch gap statistics from a rocprofv3 database.

  python tools/kernel_gaps.py gpurun_out/prof/x_results.db [--skip 100]
For each queue, consecutive dispatches are paired: gap = start(next) - end(prev).
Median duration per kernel name and median gap show whether a short step is
bound by the kernel itself or by dispatch latency between kernels.
"""
import argparse
import sqlite3
import statistics as st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--skip", type=int, default=50, help="ignore the first N dispatches (warmup)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, queue_id, start, end, vgpr_count, lds_size, grid_x, workgroup_x "
                          "from kernels order by start"))[a.skip:]
    dur, meta = {}, {}
    gaps = []
    last_end = {}
    for name, q, s, e, vg, lds, gx, wx in rows:
        short = name.split("(")[0].replace("void ", "")
        dur.setdefault(short, []).append((e - s) / 1e3)
        meta[short] = (vg, lds, gx // max(wx, 1))
        if q in last_end:
            gaps.append((s - last_end[q]) / 1e3)
        last_end[q] = e
    print("| kernel | n | median us | p10 us | VGPR | LDS B | WGs |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        print("| `%s` | %d | %.2f | %.2f | %s | %s | %s |" % (k, len(v), st.median(v), v[len(v) // 10], *meta[k]))
    if gaps:
        gaps.sort()
        print("\ndispatch gap (same queue): median %.2f us, p10 %.2f, p90 %.2f (n=%d)" %
              (st.median(gaps), gaps[len(gaps) // 10], gaps[9 * len(gaps) // 10], len(gaps)))


if __name__ == "__main__":
    main()
