#!/usr/bin/env python3
"""Register / scratch / LDS use of the gfx950 kernels in a built extension,
read from the code objects' metadata notes (no GPU needed).

  python tools/kernel_resources.py [--so PATH] [--other PATH] [--match SUBSTR ...]

With --other, only kernels whose resources differ between the two builds are
listed (a quick check of what a source change did to register allocation)."""
import argparse
import os
import re
import subprocess
import sys
import tempfile

import yaml

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_SO = os.path.join(ROOT, "openhyperflow2d_amd", "_hf2d.cpython-310-x86_64-linux-gnu.so")
KEYS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
        ".private_segment_fixed_size", ".group_segment_fixed_size")


def code_objects(so, tmp):
    fb = os.path.join(tmp, "fatbin.bin")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "-O", "binary", "--only-section=.hip_fatbin", so, fb],
                   check=True)
    data = open(fb, "rb").read()
    offs = [m.start() for m in re.finditer(b"__CLANG_OFFLOAD_BUNDLE__", data)]
    out = []
    for i, o in enumerate(offs):
        e = offs[i + 1] if i + 1 < len(offs) else len(data)
        b = os.path.join(tmp, "b%d.bin" % i)
        co = os.path.join(tmp, "co%d.o" % i)
        open(b, "wb").write(data[o:e])
        r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + b,
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], capture_output=True)
        if r.returncode == 0:
            out.append(co)
    return out


def resources(so):
    res = {}
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(so, tmp):
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], capture_output=True,
                                   text=True).stdout
            i = notes.find("amdhsa.kernels")
            if i < 0:
                continue
            txt = notes[notes.rfind("---", 0, i):]
            txt = txt[:txt.find("\n...")]
            for k in yaml.safe_load(txt)["amdhsa.kernels"]:
                res[k[".name"]] = tuple(k.get(x, 0) for x in KEYS)
    return res


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", default=DEFAULT_SO)
    ap.add_argument("--other", default=None)
    ap.add_argument("--match", nargs="*", default=[])
    a = ap.parse_args()
    h = resources(a.so)
    o = resources(a.other) if a.other else None
    names = sorted(h)
    pretty = dict(zip(names, demangle(names)))
    print("%-70s %5s %4s %4s %5s %5s %6s %6s" % ("kernel", "vgpr", "agpr", "sgpr", "vspil", "sspil", "scratch", "lds"))
    for n in names:
        p = pretty[n]
        if a.match and not any(m in p for m in a.match):
            continue
        if o is not None and o.get(n) == h[n]:
            continue
        print("%-70s %5d %4d %4d %5d %5d %6d %6d" % ((p[:70],) + h[n]))
        if o is not None:
            print("%-70s %s" % ("   (other)", o.get(n)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
