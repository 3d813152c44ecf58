"""Run-time specialised kinetics for mechanisms loaded from a file
(csrc/hip/chem_rtc.hip): the constexpr mechanism struct generated in C++ from
the runtime MechData, and the hiprtc compile of the shared chem_fast_dev.hpp
kernels for it.  Host only (hiprtc needs no device); the device runs are in
tests/test_gpu_mechanism.py."""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MECH = os.path.join(ROOT, "openhyperflow2d_amd", "data", "h2_air_li2004.mech")


def _numbers(text):
    text = re.sub(r"//[^\n]*", "", text)
    text = text[text.index("NS ="):]
    return re.findall(r"-?\d+(?:\.\d+)?(?:e[-+]?\d+)?", text)


def modified_mechanism(factor=1.5):
    """The Li et al. H2/air file with the chain-branching rate scaled: a
    mechanism no built-in kernel covers."""
    lines = open(MECH).read().splitlines()
    for k, ln in enumerate(lines):
        if ln.startswith("reaction H + O2 <=> O + OH"):
            a = float(re.search(r"A=(\S+)", ln).group(1))
            lines[k] = re.sub(r"A=\S+", "A=%r" % (a * factor), ln)
            break
    lines[1] = "mechanism h2_air_li2004_mod"
    return "\n".join(lines) + "\n"


def test_generated_struct_matches_the_header_generator(hf):
    """C++ mech_struct_source == tools/gen_mech_header.py, number for number
    (833 values: masses, NASA-7 tables, reactions, efficiencies)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from gen_mech_header import header

    from openhyperflow2d_amd.ops.mechanism import Mechanism

    want = _numbers(header(Mechanism.load(MECH)))
    got = _numbers(hf.native().mech_struct_source("h2_air_li2004"))
    assert len(want) > 800 and got == want


def test_hiprtc_compiles_file_mechanisms_and_caches(hf, tmp_path, monkeypatch):
    monkeypatch.setenv("HF2D_RTC_CACHE", str(tmp_path / "cache"))
    nat = hf.native()
    mod = modified_mechanism()
    for text in ("h2_air_li2004", mod):
        n, cached, log = nat.chem_rtc_compile(text)
        assert n > 10000 and not cached, log
        n2, cached2, _ = nat.chem_rtc_compile(text)
        assert n2 == n and cached2
    assert len(os.listdir(tmp_path / "cache")) == 2
    # the struct carries the modified rate
    assert "5320500000" in nat.mech_struct_source(mod)
