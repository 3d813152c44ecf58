#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table from a hipcc
``-Rpass-analysis=kernel-resource-usage`` remark log.

  hipcc ... -c device_solver.hip -Rpass-analysis=kernel-resource-usage 2> res.txt
  python tools/kernel_resources.py res.txt [substring ...]
"""
import re
import subprocess
import sys


def parse(path):
    rows, cur = {}, None
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"(VGPRs|AGPRs|SGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)",
                      line)
        if m and cur:
            rows[cur][m.group(1).split()[0]] = int(m.group(2))
    return rows


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout
        return out.splitlines()
    except OSError:
        return names


def main():
    rows = parse(sys.argv[1])
    keys = sys.argv[2:]
    names = list(rows)
    for n, d in zip(names, demangle(names)):
        if keys and not any(k in d for k in keys):
            continue
        r = rows[n]
        print("%-100s vgpr %3s agpr %3s scratch %4s occ %s" % (d[:100], r.get("VGPRs"), r.get("AGPRs"),
                                                              r.get("ScratchSize"), r.get("Occupancy")))


if __name__ == "__main__":
    main()
