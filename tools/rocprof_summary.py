"""Summarise a rocprofv3 results database (kernel trace) as a markdown table.

  python tools/rocprof_summary.py gpurun_out/prof/run_results.db [--steps K]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=0, help="timed steps, to print per-step cost")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    print("| kernel | calls | total (us) | avg (us) | % |")
    print("|---|---:|---:|---:|---:|")
    for name, calls, tot, avg, pct in rows:
        short = name.split("(")[0].replace("void ", "")
        print("| `%s` | %d | %.1f | %.2f | %.1f |" % (short, calls, tot, avg, pct))


if __name__ == "__main__":
    main()
