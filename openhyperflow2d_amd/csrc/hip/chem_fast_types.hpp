// Reaction record of a compiled (constexpr) mechanism (tools/gen_mech_header.py).
#pragma once

namespace hf2d {

struct CRx {
  int nrs, nps;
  int rs[3], rn[3];   // reactant species / stoichiometric coefficients
  int ps[3], pn[3];   // product species / coefficients
  int rev, tb, fo;    // reversible, "+ M" third body, "(+M)" fall-off
  int eff;            // efficiency row (-1: all 1)
  int ntroe, dnu;
  double A, b, Ta, A0, b0, Ta0;
  double troe[4];
};

}  // namespace hf2d
