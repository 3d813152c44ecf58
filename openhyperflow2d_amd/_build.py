"""In-tree native build of the hf2d runtime (no JIT cache, no pip install).

Produces, next to this file:
  _hf2d.<ext-suffix>.so   pybind11 module: host core + gfx950 HIP kernels + RCCL
  bin/hf2d                C++ CLI (argv-compatible with OpenHyperFLOW2D-<ver> <deck>)
  bin/hf2d_cpu            host-only CLI (g++; CPU / reference-order steppers)

Uses ninja for incremental builds; every HIP source is compiled with
``hipcc --offload-arch=gfx950``.  Device code is built with
``-ffp-contract=off`` so the GPU matches the CPU Jacobi stepper to rounding.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "..", "build", "native")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("HF2D_OFFLOAD_ARCH", "gfx950")

CORE_SRCS = ["deck.cpp", "gasdyn.cpp", "config.cpp", "preprocess.cpp", "checkpoint.cpp", "postproc.cpp", "stripio.cpp", "case_io.cpp", "tcpcomm.cpp", "solver.cpp", "lean.cpp", "mechanism.cpp"]
HIP_SRCS = ["device_solver.hip", "chem_mech.hip", "chem_fast.hip", "chem_rtc.hip", "numerics.hip"]
# headers handed to hiprtc by chem_rtc.hip (embedded as string literals)
RTC_EMBED = [("kChemTypesSrc", "chem_fast_types.hpp"), ("kChemDevSrc", "chem_fast_dev.hpp")]


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(HERE, "_hf2d" + suffix)


def _pybind_include() -> str:
    import pybind11

    return pybind11.get_include()


def _ninja_file() -> str:
    py_inc = sysconfig.get_paths()["include"]
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    common = "-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable"
    lines = [
        "ninja_required_version = 1.5",
        f"hipcc = {hipcc}",
        f"cxxflags = {common} -x c++ -I{CSRC}",
        f"hipflags = {common} -x hip --offload-arch={ARCH} -ffp-contract=off -munsafe-fp-atomics -I{CSRC} -I{os.path.abspath(BUILD)}"
        + ((" " + os.environ["HF2D_HIPFLAGS_EXTRA"]) if os.environ.get("HF2D_HIPFLAGS_EXTRA") else ""),
        f"pyflags = -I{_pybind_include()} -I{py_inc}",
        f"ldflags = -L{ROCM}/lib -Wl,-rpath,{ROCM}/lib -lamdhip64 -lhiprtc -lrccl -lrocprofiler-sdk-roctx",
        f"python = {sys.executable}",
        "rule cxx",
        "  command = $hipcc $cxxflags $extra -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "rule hip",
        "  command = $hipcc $hipflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "rule gxx",
        "  command = g++ -O2 -std=c++17 -fPIC -I" + CSRC + " -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "rule link_so",
        "  command = $hipcc -shared --offload-arch=" + ARCH + " $in -o $out $ldflags",
        "rule link_exe",
        "  command = $hipcc --offload-arch=" + ARCH + " $in -o $out $ldflags",
        "rule link_gxx",
        "  command = g++ $in -o $out",
        # host AddressSanitizer / UBSan build of the CPU CLI (host code only)
        "rule gxx_asan",
        "  command = g++ -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -std=c++17 -fPIC -I" + CSRC
        + " -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "rule link_gxx_asan",
        "  command = g++ -fsanitize=address,undefined $in -o $out",
        # FP32 build option of the CPU CLI (the reference's FP_OPTS = -DFP=float)
        "rule gxx_fp32",
        "  command = g++ -O2 -std=c++17 -fPIC -DHF2D_FP32 -I" + CSRC + " -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
    ]
    lines.append("rule embed")
    lines.append(f"  command = $python {os.path.abspath(__file__)} --embed $out $in")
    emb = os.path.join(os.path.abspath(BUILD), "chem_rtc_embed.inc")
    lines.append(f"build {emb}: embed " + " ".join(os.path.join(CSRC, "hip", f) for _, f in RTC_EMBED))
    objs = []
    for s in CORE_SRCS:
        o = f"core_{s[:-4]}.o"
        lines.append(f"build {o}: cxx {os.path.join(CSRC, 'core', s)}")
        objs.append(o)
    hobjs = []
    for s in HIP_SRCS:
        o = f"hip_{s[:-4]}.o"
        lines.append(f"build {o}: hip {os.path.join(CSRC, 'hip', s)}" + (f" || {emb}" if s == "chem_rtc.hip" else ""))
        hobjs.append(o)
    lines.append(f"build bind_module.o: cxx {os.path.join(CSRC, 'bind', 'module.cpp')}")
    lines.append("  extra = $pyflags")
    lines.append(f"build main.o: cxx {os.path.join(CSRC, 'core', 'hf2d_main.cpp')}")
    gobjs = []
    for s in CORE_SRCS + ["hf2d_main.cpp"]:
        o = f"gxx_{s[:-4]}.o"
        lines.append(f"build {o}: gxx {os.path.join(CSRC, 'core', s)}")
        gobjs.append(o)
    lines.append(f"build {ext_path()}: link_so {' '.join(objs + hobjs)} bind_module.o")
    lines.append(f"build {os.path.join(HERE, 'bin', 'hf2d')}: link_exe {' '.join(objs + hobjs)} main.o")
    lines.append(f"build {os.path.join(HERE, 'bin', 'hf2d_cpu')}: link_gxx {' '.join(gobjs)}")
    aobjs = []
    for s in CORE_SRCS + ["hf2d_main.cpp"]:
        o = f"asan_{s[:-4]}.o"
        lines.append(f"build {o}: gxx_asan {os.path.join(CSRC, 'core', s)}")
        aobjs.append(o)
    lines.append(f"build {asan_path()}: link_gxx_asan {' '.join(aobjs)}")
    fobjs = []
    for s in CORE_SRCS + ["hf2d_main.cpp"]:
        o = f"fp32_{s[:-4]}.o"
        lines.append(f"build {o}: gxx_fp32 {os.path.join(CSRC, 'core', s)}")
        fobjs.append(o)
    lines.append(f"build {fp32_path()}: link_gxx {' '.join(fobjs)}")
    # FP32 build of the GPU CLI (every kernel with real = float; the
    # finite-rate kinetics stay FP64-only and are refused at run time)
    f2objs = []
    for s in CORE_SRCS + ["hf2d_main.cpp"]:
        o = f"f32_{s[:-4]}.o"
        lines.append(f"build {o}: cxx {os.path.join(CSRC, 'core', s)}")
        lines.append("  extra = -DHF2D_FP32")
        f2objs.append(o)
    for s in HIP_SRCS:
        o = f"f32hip_{s[:-4]}.o"
        lines.append(f"build {o}: hip {os.path.join(CSRC, 'hip', s)}" + (f" || {emb}" if s == "chem_rtc.hip" else ""))
        lines.append("  hipflags = $hipflags -DHF2D_FP32")
        f2objs.append(o)
    lines.append(f"build {gpu_fp32_path()}: link_exe {' '.join(f2objs)}")
    lines.append(f"default {ext_path()} {os.path.join(HERE, 'bin', 'hf2d')} {os.path.join(HERE, 'bin', 'hf2d_cpu')} "
                 f"{gpu_fp32_path()}")
    return "\n".join(lines) + "\n"


def fp32_path() -> str:
    return os.path.join(HERE, "bin", "hf2d_cpu_fp32")


def gpu_fp32_path() -> str:
    """FP32 build of the GPU CLI (the reference's -DFP=float for the device solver)."""
    return os.path.join(HERE, "bin", "hf2d_fp32")


def build_fp32(verbose: bool = False) -> str:
    """FP32 build of the CPU CLI (real = float; not part of the default build)."""
    build(verbose=verbose, targets=[fp32_path()])
    return fp32_path()


def asan_path() -> str:
    return os.path.join(HERE, "bin", "hf2d_cpu_asan")


def build_asan(verbose: bool = False) -> str:
    """Host ASan/UBSan build of the CPU CLI (not part of the default build)."""
    build(verbose=verbose, targets=[asan_path()])
    return asan_path()


def build(verbose: bool = False, jobs: int | None = None, targets=None) -> str:
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(os.path.join(HERE, "bin"), exist_ok=True)
    nf = os.path.join(BUILD, "build.ninja")
    txt = _ninja_file()
    old = open(nf).read() if os.path.exists(nf) else ""
    if old != txt:
        with open(nf, "w") as f:
            f.write(txt)
    ninja = shutil.which("ninja")
    if ninja is None:
        try:
            import ninja as _n  # type: ignore

            ninja = os.path.join(_n.BIN_DIR, "ninja")
        except Exception as e:  # pragma: no cover
            raise RuntimeError("ninja not found") from e
    jobs = jobs or min(8, os.cpu_count() or 4)
    cmd = [ninja, "-C", BUILD, f"-j{jobs}"] + list(targets or [])
    if verbose:
        cmd.append("-v")
    import fcntl

    with open(os.path.join(BUILD, ".lock"), "w") as lk:   # concurrent callers (pytest -n) share one build dir
        fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(cmd, capture_output=not verbose, text=True)
    if r.returncode != 0:
        sys.stderr.write((r.stdout or "") + (r.stderr or ""))
        raise RuntimeError("native build failed")
    return ext_path()


def is_built() -> bool:
    bindir = os.path.join(os.path.dirname(ext_path()), "bin")
    return all(os.path.exists(p) for p in (ext_path(), os.path.join(bindir, "hf2d"), os.path.join(bindir, "hf2d_cpu")))


def embed(out: str, inputs) -> None:
    """chem_rtc_embed.inc: the RTC_EMBED headers as raw string literals."""
    names = dict((f, v) for v, f in RTC_EMBED)
    parts = ["// generated by _build.py from %s -- do not edit" % ", ".join(os.path.basename(i) for i in inputs)]
    for path in inputs:
        text = open(path).read()
        if ")HF2DRTC\"" in text:
            raise RuntimeError("embed delimiter found in " + path)
        parts.append('static const char %s[] = R"HF2DRTC(%s)HF2DRTC";' % (names[os.path.basename(path)], text))
    data = "\n".join(parts) + "\n"
    if not os.path.exists(out) or open(out).read() != data:
        with open(out, "w") as f:
            f.write(data)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--embed":
        embed(sys.argv[2], sys.argv[3:])
    else:
        print(build(verbose="-v" in sys.argv))
