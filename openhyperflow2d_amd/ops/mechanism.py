"""Detailed gas-phase mechanisms for the finite-rate chemistry (CRM_ARRENIUS slot).

The reference declares ``CRM_ARRENIUS`` / ``CRM_EDM`` and never implements them
(libOpenHyperFLOW2D/hyper_flow_bound.hpp:37-42); its species set is hard-wired
to fuel / oxidiser / products / air (``NUM_COMPONENTS 3``,
hyper_flow_node.hpp:33-39).  This module is the data side of the replacement:

* a line-based mechanism file format (``*.mech``, SI units) read by this module
  and by the C++ runtime (``csrc/core/mechanism.cpp``);
* the built-in H2/O2 mechanism of Li, Zhao, Kazakov & Dryer (Int. J. Chem. Kinet.
  36, 2004: 9 species incl. N2, 21 reversible steps with third-body
  efficiencies and Troe fall-off) with NASA-7 thermodynamics (GRI-Mech 3.0
  polynomials) and Chapman-Enskog viscosities;
* thermodynamics (cp, h, s, Gibbs), equilibrium constants and the net rates of
  progress, as plain NumPy/PyTorch FP64 code that is independent of the HIP and
  C++ implementations (the oracle of their tests);
* 0-D reactors (constant volume / constant pressure) integrated with SciPy's BDF
  for ignition-delay checks.  No external kinetics package exists in this
  image, so these results are "parity unpinned" against Cantera/CHEMKIN.

File format (``#`` starts a comment; one record per line)::

    mechanism <name>
    species <s1> <s2> ...                      # <= 16 species
    thermo <s> <W kg/mol> <Tlo> <Tmid> <Thi> <a1..a7 low> <a1..a7 high>
    transport <s> <sigma A> <eps/k K>          # Lennard-Jones (viscosity tables)
    reaction <lhs> <=>|=> <rhs> A=<SI> b=<> Ta=<K> [M] [falloff A0=.. b0=.. Ta0=..]
             [troe=a,T3,T1[,T2]] [eff=s:v,s:v]
    slot fuel|ox|cp|air s:y[,s:y]              # reference 4-slot -> species map

``<lhs>``/``<rhs>`` are ``+``-separated species with optional integer
coefficients (``2 OH``); ``M`` marks a third-body reaction (the collider
concentration multiplies the rate; ``falloff`` gives the Lindemann/Troe blend
instead).  A is in SI: (m^3/mol)^(n-1)/s with n the reaction order counting M
for third-body reactions (k_inf of a fall-off step counts it not).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

RU = 8.314462618          # J/mol/K
P_ATM = 101325.0          # Pa (standard state of the NASA polynomials)
CAL = 4.184               # J/cal
MAX_SPECIES = 16
MAX_REACTIONS = 64
DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "data")


@dataclass
class Species:
    name: str
    W: float                       # kg/mol
    Tlo: float
    Tmid: float
    Thi: float
    low: Sequence[float]           # a1..a7 for Tlo <= T < Tmid
    high: Sequence[float]          # a1..a7 for Tmid <= T <= Thi
    sigma: float = 3.5             # Lennard-Jones diameter [Angstrom]
    eps_k: float = 100.0           # Lennard-Jones well depth / k_B [K]


@dataclass
class Reaction:
    reactants: Dict[str, int]
    products: Dict[str, int]
    A: float                       # SI
    b: float = 0.0
    Ta: float = 0.0                # Ea / Ru [K]
    reversible: bool = True
    third_body: bool = False       # "+ M"
    falloff: bool = False          # "(+M)": k = k_inf * Pr/(1+Pr) * F
    A0: float = 0.0
    b0: float = 0.0
    Ta0: float = 0.0
    troe: Optional[Tuple[float, ...]] = None   # (a, T3, T1[, T2])
    eff: Dict[str, float] = field(default_factory=dict)

    def equation(self) -> str:
        def side(d):
            return " + ".join(("%d %s" % (n, s)) if n != 1 else s for s, n in d.items())
        m = " (+M)" if self.falloff else (" + M" if self.third_body else "")
        return side(self.reactants) + m + (" <=> " if self.reversible else " => ") + side(self.products) + m


@dataclass
class Mechanism:
    name: str
    species: List[Species]
    reactions: List[Reaction]
    slots: Dict[str, Dict[str, float]] = field(default_factory=dict)

    def __post_init__(self):
        ns = len(self.species)
        if not 1 <= ns <= MAX_SPECIES:
            raise ValueError("mechanism needs 1..%d species, got %d" % (MAX_SPECIES, ns))
        if len(self.reactions) > MAX_REACTIONS:
            raise ValueError("at most %d reactions" % MAX_REACTIONS)
        names = self.names
        if len(set(names)) != ns:
            raise ValueError("duplicate species name")
        for s in self.species:
            if not s.W > 0:
                raise ValueError("species %s: molar mass must be > 0" % s.name)
            if not (0 < s.Tlo < s.Tmid < s.Thi):
                raise ValueError("species %s: need 0 < Tlo < Tmid < Thi" % s.name)
        for r in self.reactions:
            for side in (r.reactants, r.products):
                if not 1 <= len(side) <= 3:
                    raise ValueError("%s: 1..3 distinct species per side" % r.equation())
                for s, n in side.items():
                    if s not in names:
                        raise ValueError("%s: unknown species %r" % (r.equation(), s))
                    if not (isinstance(n, (int, np.integer)) or float(n).is_integer()) or not 1 <= int(n) <= 3:
                        raise ValueError("%s: stoichiometric coefficients must be integers 1..3" % r.equation())
            for s in r.eff:
                if s not in names:
                    raise ValueError("%s: efficiency for unknown species %r" % (r.equation(), s))
            if r.falloff and not r.A0 > 0:
                raise ValueError("%s: fall-off step needs A0 > 0" % r.equation())
            if not r.A > 0:
                raise ValueError("%s: A must be > 0" % r.equation())
        for slot, comp in self.slots.items():
            if slot not in ("fuel", "ox", "cp", "air"):
                raise ValueError("unknown slot %r" % slot)
            for s in comp:
                if s not in names:
                    raise ValueError("slot %s: unknown species %r" % (slot, s))

    # -- basic properties ----------------------------------------------------
    @property
    def names(self) -> List[str]:
        return [s.name for s in self.species]

    @property
    def ns(self) -> int:
        return len(self.species)

    @property
    def nr(self) -> int:
        return len(self.reactions)

    @property
    def W(self) -> np.ndarray:
        return np.array([s.W for s in self.species])

    def index(self, name: str) -> int:
        return self.names.index(name)

    def stoich(self) -> Tuple[np.ndarray, np.ndarray]:
        """nu' (reactants) and nu'' (products), shape [nr, ns]."""
        f = np.zeros((self.nr, self.ns))
        r = np.zeros((self.nr, self.ns))
        for j, rx in enumerate(self.reactions):
            for s, n in rx.reactants.items():
                f[j, self.index(s)] += n
            for s, n in rx.products.items():
                r[j, self.index(s)] += n
        return f, r

    def efficiencies(self) -> np.ndarray:
        """[nr, ns] third-body efficiencies (1 by default; 0 rows for plain steps)."""
        e = np.zeros((self.nr, self.ns))
        for j, rx in enumerate(self.reactions):
            if rx.third_body or rx.falloff:
                e[j, :] = 1.0
                for s, v in rx.eff.items():
                    e[j, self.index(s)] = v
        return e

    def slot_matrix(self) -> np.ndarray:
        """[4, ns] map from the reference's (fuel, ox, cp, air) mass fractions."""
        m = np.zeros((4, self.ns))
        for k, slot in enumerate(("fuel", "ox", "cp", "air")):
            comp = self.slots.get(slot, {})
            tot = sum(comp.values())
            for s, v in comp.items():
                m[k, self.index(s)] = v / tot
        return m

    # -- file IO -----------------------------------------------------------------
    def to_text(self) -> str:
        out = ["# hf2d mechanism file (SI units; see openhyperflow2d_amd/ops/mechanism.py)",
               "mechanism %s" % self.name, "species " + " ".join(self.names)]
        for s in self.species:
            out.append("thermo %s %.17g %.17g %.17g %.17g %s %s" % (
                s.name, s.W, s.Tlo, s.Tmid, s.Thi, " ".join("%.17g" % a for a in s.low),
                " ".join("%.17g" % a for a in s.high)))
        for s in self.species:
            out.append("transport %s %.6g %.6g" % (s.name, s.sigma, s.eps_k))
        for r in self.reactions:
            def side(d):
                return " + ".join(("%d %s" % (n, s)) if n != 1 else s for s, n in d.items())
            line = "reaction %s %s %s A=%.17g b=%.17g Ta=%.17g" % (side(r.reactants), "<=>" if r.reversible else "=>",
                                                                  side(r.products), r.A, r.b, r.Ta)
            if r.third_body:
                line += " M"
            if r.falloff:
                line += " falloff A0=%.17g b0=%.17g Ta0=%.17g" % (r.A0, r.b0, r.Ta0)
            if r.troe:
                line += " troe=" + ",".join("%.17g" % v for v in r.troe)
            if r.eff:
                line += " eff=" + ",".join("%s:%.17g" % kv for kv in r.eff.items())
            out.append(line)
        for slot in ("fuel", "ox", "cp", "air"):
            if slot in self.slots:
                out.append("slot %s %s" % (slot, ",".join("%s:%.17g" % kv for kv in self.slots[slot].items())))
        return "\n".join(out) + "\n"

    def save(self, path: str) -> None:
        with open(path, "w") as f:
            f.write(self.to_text())

    @classmethod
    def from_text(cls, text: str) -> "Mechanism":
        name, order, thermo, trans, rx, slots = "mech", [], {}, {}, [], {}
        for lineno, raw in enumerate(text.splitlines(), 1):
            line = raw.split("#", 1)[0].strip()
            if not line:
                continue
            tok = line.split()
            kw = tok[0]
            try:
                if kw == "mechanism":
                    name = tok[1]
                elif kw == "species":
                    order = tok[1:]
                elif kw == "thermo":
                    v = [float(x) for x in tok[2:]]
                    if len(v) != 18:
                        raise ValueError("thermo needs W Tlo Tmid Thi + 14 coefficients")
                    thermo[tok[1]] = v
                elif kw == "transport":
                    trans[tok[1]] = (float(tok[2]), float(tok[3]))
                elif kw == "reaction":
                    rx.append(_parse_reaction(tok[1:]))
                elif kw == "slot":
                    slots[tok[1]] = {k: float(v) for k, v in (p.split(":") for p in tok[2].split(","))}
                else:
                    raise ValueError("unknown record %r" % kw)
            except (ValueError, IndexError) as e:
                raise ValueError("mechanism line %d: %s" % (lineno, e)) from None
        sp = []
        for s in order:
            if s not in thermo:
                raise ValueError("species %s has no thermo record" % s)
            v = thermo[s]
            sig, ek = trans.get(s, (3.5, 100.0))
            sp.append(Species(s, v[0], v[1], v[2], v[3], v[4:11], v[11:18], sig, ek))
        return cls(name, sp, rx, slots)

    @classmethod
    def load(cls, path: str) -> "Mechanism":
        with open(path) as f:
            return cls.from_text(f.read())


def _parse_side(tokens: List[str]) -> Tuple[Dict[str, int], bool, bool]:
    d: Dict[str, int] = {}
    tb = fo = False
    for term in " ".join(tokens).split("+"):
        t = term.split()
        if not t:
            continue
        if t == ["M"]:
            tb = True
            continue
        if t == ["(", "M)"] or t == ["(M)"]:
            fo = True
            continue
        n = 1
        if len(t) == 2:
            n = int(t[0])
            s = t[1]
        elif len(t) == 1:
            s = t[0]
        else:
            raise ValueError("bad species term %r" % term)
        d[s] = d.get(s, 0) + n
    return d, tb, fo


def _parse_reaction(tok: List[str]) -> Reaction:
    arrow = next(i for i, t in enumerate(tok) if t in ("<=>", "=>"))
    rev = tok[arrow] == "<=>"
    rest = tok[arrow + 1:]
    k = next(i for i, t in enumerate(rest) if "=" in t)
    lhs, _, _ = _parse_side(tok[:arrow])
    rhs, _, _ = _parse_side(rest[:k])
    kv: Dict[str, str] = {}
    flags = set()
    for t in rest[k:]:
        if "=" in t:
            a, b = t.split("=", 1)
            kv[a] = b
        else:
            flags.add(t)
    r = Reaction(lhs, rhs, float(kv["A"]), float(kv.get("b", 0)), float(kv.get("Ta", 0)), rev,
                 third_body="M" in flags, falloff="falloff" in flags)
    if r.falloff:
        r.A0, r.b0, r.Ta0 = float(kv["A0"]), float(kv.get("b0", 0)), float(kv.get("Ta0", 0))
    if "troe" in kv:
        r.troe = tuple(float(x) for x in kv["troe"].split(","))
    if "eff" in kv:
        r.eff = {a: float(b) for a, b in (p.split(":") for p in kv["eff"].split(","))}
    return r


# ---------------------------------------------------------------------------
# Built-in mechanism: H2/O2 of Li, Zhao, Kazakov & Dryer (2004) + N2 (inert).
# Rate data in the published CGS / cal units, converted to SI here.
# ---------------------------------------------------------------------------
# NASA-7 polynomials (GRI-Mech 3.0 thermo data), Tmid = 1000 K.
_NASA = {
    "H2": (2.01588e-3, 200.0, 1000.0, 3500.0,
           (2.34433112e+00, 7.98052075e-03, -1.94781510e-05, 2.01572094e-08, -7.37611761e-12, -9.17935173e+02,
            6.83010238e-01),
           (3.33727920e+00, -4.94024731e-05, 4.99456778e-07, -1.79566394e-10, 2.00255376e-14, -9.50158922e+02,
            -3.20502331e+00)),
    "O2": (31.9988e-3, 200.0, 1000.0, 3500.0,
           (3.78245636e+00, -2.99673416e-03, 9.84730201e-06, -9.68129509e-09, 3.24372837e-12, -1.06394356e+03,
            3.65767573e+00),
           (3.28253784e+00, 1.48308754e-03, -7.57966669e-07, 2.09470555e-10, -2.16717794e-14, -1.08845772e+03,
            5.45323129e+00)),
    "H2O": (18.01528e-3, 200.0, 1000.0, 3500.0,
            (4.19864056e+00, -2.03643410e-03, 6.52040211e-06, -5.48797062e-09, 1.77197817e-12, -3.02937267e+04,
             -8.49032208e-01),
            (3.03399249e+00, 2.17691804e-03, -1.64072518e-07, -9.70419870e-11, 1.68200992e-14, -3.00042971e+04,
             4.96677010e+00)),
    "H": (1.00794e-3, 200.0, 1000.0, 3500.0,
          (2.50000000e+00, 7.05332819e-13, -1.99591964e-15, 2.30081632e-18, -9.27732332e-22, 2.54736599e+04,
           -4.46682853e-01),
          (2.50000001e+00, -2.30842973e-11, 1.61561948e-14, -4.73515235e-18, 4.98197357e-22, 2.54736599e+04,
           -4.46682914e-01)),
    "O": (15.9994e-3, 200.0, 1000.0, 3500.0,
          (3.16826710e+00, -3.27931884e-03, 6.64306396e-06, -6.12806624e-09, 2.11265971e-12, 2.91222592e+04,
           2.05193346e+00),
          (2.56942078e+00, -8.59741137e-05, 4.19484589e-08, -1.00177799e-11, 1.22833691e-15, 2.92175791e+04,
           4.78433864e+00)),
    "OH": (17.00734e-3, 200.0, 1000.0, 3500.0,
           (3.99201543e+00, -2.40131752e-03, 4.61793841e-06, -3.88113333e-09, 1.36411470e-12, 3.61508056e+03,
            -1.03925458e-01),
           (3.09288767e+00, 5.48429716e-04, 1.26505228e-07, -8.79461556e-11, 1.17412376e-14, 3.85865700e+03,
            4.47669610e+00)),
    "HO2": (33.00674e-3, 200.0, 1000.0, 3500.0,
            (4.30179801e+00, -4.74912051e-03, 2.11582891e-05, -2.42763894e-08, 9.29225124e-12, 2.94808040e+02,
             3.71666245e+00),
            (4.01721090e+00, 2.23982013e-03, -6.33658150e-07, 1.14246370e-10, -1.07908535e-14, 1.11856713e+02,
             3.78510215e+00)),
    "H2O2": (34.01468e-3, 200.0, 1000.0, 3500.0,
             (4.27611269e+00, -5.42822417e-04, 1.67335701e-05, -2.15770813e-08, 8.62454363e-12, -1.77025821e+04,
              3.43505074e+00),
             (4.16500285e+00, 4.90831694e-03, -1.90139225e-06, 3.71185986e-10, -2.87908305e-14, -1.78617877e+04,
              2.91615662e+00)),
    "N2": (28.0134e-3, 300.0, 1000.0, 5000.0,
           (3.29867700e+00, 1.40824040e-03, -3.96322200e-06, 5.64151500e-09, -2.44485400e-12, -1.02089990e+03,
            3.95037200e+00),
           (2.92664000e+00, 1.48797680e-03, -5.68476000e-07, 1.00970380e-10, -6.75335100e-15, -9.22797700e+02,
            5.98052800e+00)),
}
# Lennard-Jones parameters (GRI-Mech 3.0 transport data): sigma [A], eps/k [K]
_LJ = {"H2": (2.92, 38.0), "O2": (3.458, 107.4), "H2O": (2.605, 572.4), "H": (2.05, 145.0), "O": (2.75, 80.0),
       "OH": (2.75, 80.0), "HO2": (3.458, 107.4), "H2O2": (3.458, 107.4), "N2": (3.621, 97.53)}

# (equation, A [cm, mol, s], b, Ea [cal/mol], options)
_LI2004 = [
    ("H + O2 <=> O + OH", 3.547e15, -0.406, 16599.0, {}),
    ("O + H2 <=> H + OH", 0.508e05, 2.67, 6290.0, {}),
    ("H2 + OH <=> H2O + H", 0.216e09, 1.51, 3430.0, {}),
    ("O + H2O <=> OH + OH", 2.97e06, 2.02, 13400.0, {}),
    ("H2 + M <=> H + H + M", 4.577e19, -1.40, 104380.0, {"eff": {"H2": 2.5, "H2O": 12.0}}),
    ("O + O + M <=> O2 + M", 6.165e15, -0.50, 0.0, {"eff": {"H2": 2.5, "H2O": 12.0}}),
    ("O + H + M <=> OH + M", 4.714e18, -1.00, 0.0, {"eff": {"H2": 2.5, "H2O": 12.0}}),
    ("H + OH + M <=> H2O + M", 3.800e22, -2.00, 0.0, {"eff": {"H2": 2.5, "H2O": 12.0}}),
    ("H + O2 (+M) <=> HO2 (+M)", 1.475e12, 0.60, 0.0,
     {"low": (6.366e20, -1.72, 524.8), "troe": (0.8, 1e-30, 1e30), "eff": {"H2": 2.0, "H2O": 11.0, "O2": 0.78}}),
    ("HO2 + H <=> H2 + O2", 1.66e13, 0.00, 823.0, {}),
    ("HO2 + H <=> OH + OH", 7.079e13, 0.00, 295.0, {}),
    ("HO2 + O <=> O2 + OH", 0.325e14, 0.00, 0.0, {}),
    ("HO2 + OH <=> H2O + O2", 2.890e13, 0.00, -497.0, {}),
    ("HO2 + HO2 <=> H2O2 + O2", 4.200e14, 0.00, 11982.0, {}),
    ("HO2 + HO2 <=> H2O2 + O2", 1.300e11, 0.00, -1629.3, {}),
    ("H2O2 (+M) <=> OH + OH (+M)", 2.951e14, 0.00, 48430.0,
     {"low": (1.202e17, 0.00, 45500.0), "troe": (0.5, 1e-30, 1e30), "eff": {"H2": 2.5, "H2O": 12.0}}),
    ("H2O2 + H <=> H2O + OH", 0.241e14, 0.00, 3970.0, {}),
    ("H2O2 + H <=> HO2 + H2", 0.482e14, 0.00, 7950.0, {}),
    ("H2O2 + O <=> OH + HO2", 9.550e06, 2.00, 3970.0, {}),
    ("H2O2 + OH <=> HO2 + H2O", 1.000e12, 0.00, 0.0, {}),
    ("H2O2 + OH <=> HO2 + H2O", 5.800e14, 0.00, 9557.0, {}),
]


def _cgs_reaction(eq: str, A: float, b: float, Ea: float, opt: dict) -> Reaction:
    lhs_s, rhs_s = [p.strip() for p in eq.split("<=>")]
    lhs, tb, fo = _parse_side(lhs_s.replace("(+M)", "+ (M)").split())
    rhs, _, _ = _parse_side(rhs_s.replace("(+M)", "+ (M)").split())
    order = sum(lhs.values())
    # k (or k_inf for fall-off) has order sum(nu') (+1 for a "+ M" step)
    n = order + (1 if tb else 0)
    r = Reaction(lhs, rhs, A * 1e-6 ** (n - 1), b, Ea * CAL / RU, True, third_body=tb, falloff=fo,
                 eff=dict(opt.get("eff", {})))
    if fo:
        A0, b0, E0 = opt["low"]
        r.A0, r.b0, r.Ta0 = A0 * 1e-6 ** order, b0, E0 * CAL / RU   # k0 has one more order (M)
        r.troe = tuple(opt["troe"]) if "troe" in opt else None
    return r


def h2_air_li2004() -> Mechanism:
    """Li et al. (2004) H2/O2 kinetics with N2 as the bath gas (9 species / 21 steps)."""
    order = ["H2", "O2", "H2O", "H", "O", "OH", "HO2", "H2O2", "N2"]
    sp = []
    for s in order:
        W, lo, mid, hi, a_lo, a_hi = _NASA[s]
        sig, ek = _LJ[s]
        sp.append(Species(s, W, lo, mid, hi, a_lo, a_hi, sig, ek))
    rx = [_cgs_reaction(*r) for r in _LI2004]
    slots = {"fuel": {"H2": 1.0}, "ox": {"O2": 1.0}, "cp": {"H2O": 1.0}, "air": {"N2": 1.0}}
    return Mechanism("h2_air_li2004", sp, rx, slots)


def builtin(name: str = "h2_air_li2004") -> Mechanism:
    if name in ("h2_air_li2004", "H2Air-Li2004", "h2air"):
        return h2_air_li2004()
    p = os.path.join(DATA_DIR, name if name.endswith(".mech") else name + ".mech")
    if os.path.exists(p):
        return Mechanism.load(p)
    raise KeyError("unknown mechanism %r" % name)


# ---------------------------------------------------------------------------
# Thermodynamics and kinetics (NumPy FP64; independent oracle)
# ---------------------------------------------------------------------------
def nasa_coeffs(mech: Mechanism, T: np.ndarray) -> np.ndarray:
    """[..., ns, 7] coefficient set per species for temperatures T (shape [...])."""
    T = np.asarray(T, dtype=np.float64)
    lo = np.array([s.low for s in mech.species])
    hi = np.array([s.high for s in mech.species])
    mid = np.array([s.Tmid for s in mech.species])
    sel = (T[..., None] < mid)[..., None]
    return np.where(sel, lo, hi)


# Below T_LO (the lower limit of the NASA-7 fits) every species is
# extrapolated at constant cp (the solver's MECH_TLO rule, core/mechanism.hpp).
T_LO = 200.0


def _cp_R_poly(mech, T):
    a = nasa_coeffs(mech, T)
    T = np.asarray(T, dtype=np.float64)[..., None]
    return a[..., 0] + T * (a[..., 1] + T * (a[..., 2] + T * (a[..., 3] + T * a[..., 4])))


def _h_RT_poly(mech, T):
    a = nasa_coeffs(mech, T)
    T = np.asarray(T, dtype=np.float64)[..., None]
    return a[..., 0] + T * (a[..., 1] / 2 + T * (a[..., 2] / 3 + T * (a[..., 3] / 4 + T * a[..., 4] / 5))) + a[..., 5] / T


def _s_R_poly(mech, T):
    a = nasa_coeffs(mech, T)
    T = np.asarray(T, dtype=np.float64)[..., None]
    return (a[..., 0] * np.log(T) + T * (a[..., 1] + T * (a[..., 2] / 2 + T * (a[..., 3] / 3 + T * a[..., 4] / 4)))
            + a[..., 6])


def cp_R(mech, T):
    return _cp_R_poly(mech, np.maximum(np.asarray(T, dtype=np.float64), T_LO))


def h_RT(mech, T):
    T = np.asarray(T, dtype=np.float64)
    Te = np.maximum(T, T_LO)
    h = _h_RT_poly(mech, Te) * Te[..., None] + _cp_R_poly(mech, Te) * (T - Te)[..., None]
    return h / T[..., None]


def s_R(mech, T):
    T = np.asarray(T, dtype=np.float64)
    Te = np.maximum(T, T_LO)
    return _s_R_poly(mech, Te) + _cp_R_poly(mech, Te) * np.log(T / Te)[..., None]


def mixture_e(mech, Y, T):
    """Specific internal energy (J/kg, incl. formation) of mass fractions Y [..., ns] at T."""
    W = mech.W
    h = h_RT(mech, T) * RU * np.asarray(T)[..., None] / W
    return (Y * (h - RU / W * np.asarray(T)[..., None])).sum(-1)


def mixture_h(mech, Y, T):
    W = mech.W
    return (Y * h_RT(mech, T) * RU * np.asarray(T)[..., None] / W).sum(-1)


def mixture_cv(mech, Y, T):
    W = mech.W
    return (Y * (cp_R(mech, T) - 1.0) * RU / W).sum(-1)


def T_from_e(mech, Y, e, T0=1000.0, tol=1e-10, maxit=50):
    T = np.array(np.broadcast_to(T0, np.shape(e)), dtype=np.float64)
    for _ in range(maxit):
        f = mixture_e(mech, Y, T) - e
        dT = -f / mixture_cv(mech, Y, T)
        T = T + dT
        if np.all(np.abs(dT) < tol * T):
            break
    return T


def viscosity(mech, T):
    """Chapman-Enskog species viscosities [..., ns] (Pa s), Neufeld collision integral."""
    T = np.asarray(T, dtype=np.float64)[..., None]
    sig = np.array([s.sigma for s in mech.species])
    ek = np.array([s.eps_k for s in mech.species])
    Ts = T / ek
    om = 1.16145 * Ts ** -0.14874 + 0.52487 * np.exp(-0.77320 * Ts) + 2.16178 * np.exp(-2.43787 * Ts)
    return 2.6693e-6 * np.sqrt(mech.W * 1e3 * T) / (sig * sig * om)


def rates_of_progress(mech: Mechanism, c: np.ndarray, T: np.ndarray) -> np.ndarray:
    """Net rate of progress q [..., nr] (mol/m^3/s) for concentrations c [..., ns] (mol/m^3)."""
    kf, kr, mult, _ = rate_parts(mech, c, T)
    nf, nr_ = mech.stoich()
    cpos = np.maximum(c, 0.0)
    pf = np.prod(cpos[..., None, :] ** nf, axis=-1)
    pr = np.prod(cpos[..., None, :] ** nr_, axis=-1)
    return mult * (kf * pf - kr * pr)


def rate_parts(mech: Mechanism, c: np.ndarray, T: np.ndarray):
    """(kf incl. fall-off, kr, rate multiplier (collider conc. of '+M' steps, else 1),
    dM flag (1 for '+M' steps: d mult / dc_j = eff_j)), each [..., nr]."""
    nf, nr_ = mech.stoich()
    T = np.asarray(T, dtype=np.float64)
    eff = mech.efficiencies()
    g = h_RT(mech, T) - s_R(mech, T)                             # [..., ns]
    dnu = (nr_ - nf).sum(1)                                      # [nr]
    lnKc = -(g @ (nr_ - nf).T) + dnu * np.log(P_ATM / (RU * T))[..., None]
    A = np.array([r.A for r in mech.reactions])
    b = np.array([r.b for r in mech.reactions])
    Ta = np.array([r.Ta for r in mech.reactions])
    lnT = np.log(T)[..., None]
    kf = A * np.exp(b * lnT - Ta / T[..., None])
    M = c @ eff.T                                                # [..., nr]
    for j, r in enumerate(mech.reactions):
        if r.falloff:
            k0 = r.A0 * np.exp(r.b0 * lnT[..., 0] - r.Ta0 / T)
            Pr = k0 * M[..., j] / kf[..., j]
            F = np.ones_like(Pr)
            if r.troe:
                a, T3, T1 = r.troe[:3]
                Fc = (1 - a) * np.exp(-T / T3) + a * np.exp(-T / T1)
                if len(r.troe) > 3:
                    Fc = Fc + np.exp(-r.troe[3] / T)
                lFc = np.log10(np.maximum(Fc, 1e-300))
                lPr = np.log10(np.maximum(Pr, 1e-300))
                cc = -0.4 - 0.67 * lFc
                nn = 0.75 - 1.27 * lFc
                f1 = (lPr + cc) / (nn - 0.14 * (lPr + cc))
                F = 10.0 ** (lFc / (1 + f1 * f1))
            kf[..., j] = kf[..., j] * Pr / (1 + Pr) * F
            M[..., j] = 1.0
        elif not r.third_body:
            M[..., j] = 1.0
    kr = kf * np.exp(-lnKc)
    for j, r in enumerate(mech.reactions):
        if not r.reversible:
            kr[..., j] = 0.0
    dM = np.array([1.0 if (r.third_body and not r.falloff) else 0.0 for r in mech.reactions])
    return kf, kr, M, dM


def point_implicit_step(mech: Mechanism, rhoY: np.ndarray, rho: np.ndarray, e: np.ndarray, T: np.ndarray,
                        dt: float, nsub: int = 1):
    """Batched NumPy FP64 reference of the solver's kinetics operator.

    rhoY [ns, n] partial densities at constant density rho [n] and specific
    internal energy e [n] (J/kg, formation included); nsub linearised
    backward-Euler substeps (I - h J) dc = h w(c, T) with the analytic
    Jacobian (fall-off blending factors frozen), c <- max(c + dc, 0), mass
    re-normalised to rho, T re-solved from e after every substep.  Independent
    of the C++/HIP implementations.  Returns (rhoY, T)."""
    W = mech.W
    nf, nr_ = mech.stoich()
    nu = nr_ - nf
    eff = mech.efficiencies()
    rho = np.asarray(rho, dtype=np.float64)
    c = np.maximum(np.asarray(rhoY, dtype=np.float64).T, 0.0) / W          # [n, ns]
    Tc = T_from_e(mech, c * W / rho[:, None], e, T0=np.asarray(T, dtype=np.float64))
    h = dt / nsub
    eye = np.eye(mech.ns)
    for _ in range(nsub):
        kf, kr, mult, dM = rate_parts(mech, c, Tc)
        pf = np.prod(c[:, None, :] ** nf, axis=-1)
        pr = np.prod(c[:, None, :] ** nr_, axis=-1)
        net = kf * pf - kr * pr
        om = (mult * net) @ nu                                              # [n, ns]
        D = np.zeros((c.shape[0], mech.nr, mech.ns))
        for j in range(mech.ns):
            ef = nf.copy()
            ef[:, j] = np.maximum(ef[:, j] - 1, 0)
            er = nr_.copy()
            er[:, j] = np.maximum(er[:, j] - 1, 0)
            dpf = nf[:, j] * np.prod(c[:, None, :] ** ef, axis=-1)
            dpr = nr_[:, j] * np.prod(c[:, None, :] ** er, axis=-1)
            D[:, :, j] = mult * (kf * dpf - kr * dpr) + dM * eff[:, j] * net
        J = np.einsum("ri,nrj->nij", nu, D)
        dc = np.linalg.solve(eye - h * J, h * om[..., None])[..., 0]
        c = np.maximum(c + dc, 0.0)
        c *= (rho / (c * W).sum(1))[:, None]
        Tc = T_from_e(mech, c * W / rho[:, None], e, T0=Tc)
    return (c * W).T, Tc


def wdot(mech, c, T):
    nf, nr_ = mech.stoich()
    return rates_of_progress(mech, c, T) @ (nr_ - nf)           # [..., ns] mol/m^3/s


def reactor_rhs(mech: Mechanism, mode: str, rho0: float, p0: float):
    """d/dt of [Y_0..Y_ns-1, T] for a closed adiabatic reactor ('cv' or 'cp')."""
    W = mech.W

    def f(t, y):
        Y = np.maximum(y[:-1], 0.0)
        T = y[-1]
        if mode == "cv":
            rho = rho0
        else:
            rho = p0 / (RU * T * (Y / W).sum())
        c = rho * Y / W
        om = wdot(mech, c, T)                                    # mol/m^3/s
        dY = om * W / rho
        if mode == "cv":
            ek = (h_RT(mech, T) - 1.0) * RU * T / W              # J/kg per species
            dT = -(ek * dY).sum() / mixture_cv(mech, Y, T)
        else:
            hk = h_RT(mech, T) * RU * T / W
            cp = (Y * cp_R(mech, T) * RU / W).sum()
            dT = -(hk * dY).sum() / cp
        return np.concatenate([dY, [dT]])

    return f


def ignition_delay(mech: Mechanism, T0: float, p0: float, Y0: np.ndarray, mode: str = "cp", t_end: float = 5e-3,
                   rtol: float = 1e-9, atol: float = 1e-14):
    """Ignition delay (time of max dT/dt) of a 0-D reactor with SciPy BDF (FP64).

    Returns (tau, t, T(t), Y(t))."""
    from scipy.integrate import solve_ivp

    Y0 = np.asarray(Y0, dtype=np.float64)
    rho0 = p0 / (RU * T0 * (Y0 / mech.W).sum())
    f = reactor_rhs(mech, mode, rho0, p0)
    sol = solve_ivp(f, (0.0, t_end), np.concatenate([Y0, [T0]]), method="BDF", rtol=rtol, atol=atol,
                    dense_output=False, max_step=t_end / 200)
    t, T = sol.t, sol.y[-1]
    dTdt = np.gradient(T, t)
    return float(t[int(np.argmax(dTdt))]), t, T, sol.y[:-1]


def premixed_Y(mech: Mechanism, phi: float = 1.0) -> np.ndarray:
    """H2/air (O2 : N2 = 1 : 3.76 by mole) at equivalence ratio phi."""
    X = np.zeros(mech.ns)
    X[mech.index("H2")] = 2.0 * phi
    X[mech.index("O2")] = 1.0
    X[mech.index("N2")] = 3.76
    Y = X * mech.W
    return Y / Y.sum()


__all__ = ["Species", "Reaction", "Mechanism", "h2_air_li2004", "builtin", "cp_R", "h_RT", "s_R", "mixture_e",
           "mixture_h", "mixture_cv", "T_from_e", "viscosity", "rates_of_progress", "wdot", "ignition_delay",
           "premixed_Y", "RU", "P_ATM", "rate_parts", "point_implicit_step"]
