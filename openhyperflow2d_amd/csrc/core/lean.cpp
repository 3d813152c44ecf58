// Host side of the lean inviscid path (lean_euler.hpp): eligibility and the
// per-cell neighbour/publish byte.
#include <cstring>
#include <string>
#include <vector>

#include "lean_euler.hpp"
#include "solver.hpp"

namespace hf2d {

bool lean_eligible(const Case& cs, std::string* why) {
  if (!cs.J.whole() && cs.facts.valid) {   // strip rank: the whole field's answer
    if (why) *why = cs.facts.lean_why;
    return cs.facts.lean_ok;
  }
  auto no = [&](const char* w) {
    if (why) *why = w;
    return false;
  };
  const Config& C = cs.cfg;
  if (C.ProblemType == SM_NS) return no("viscous problem");
  if (!C.sources.empty()) return no("gas sources");
  if (!C.isAdiabaticWall) return no("wall heat transfer");
  if (C.chem_model == CRM_ARRENIUS) return no("finite-rate chemistry sources");
  for (const CellRecord& c : cs.J.c) {
    if (c.is(CT_SOLID)) continue;
    if (!c.is(CT_NODE_IS_SET)) return no("unset non-solid node");
    // equations >= 4 + NCOMP are frozen for inviscid nodes: their Src/SrcAdd
    // (e.g. left by a k-eps initialisation) are never read
    for (int k = 0; k < 4 + NCOMP; k++)
      if (c.Src[k] != 0.) return no("non-zero Src");
    if (!c.is(CT_WALL_NO_SLIP))
      for (int k = 0; k < 4 + NCOMP; k++)
        if (c.SrcAdd[k] != 0.) return no("non-zero SrcAdd off no-slip walls");
  }
  if (why) why->clear();
  return true;
}

// Single-gas laminar N-S specialisation of the generic stepper (fill_cell /
// predict_cell_t <SGL>): only equations 0..3 and the fields the next step
// reads move through memory.  Requires species +0 everywhere, no species
// sources, no turbulence model, mu_t = lam_t = 0, Y = (0,0,0,1) and (with
// chemistry on) R = R_air everywhere -- then the generic stepper leaves every
// skipped field unchanged.
int sk_eligible(const Case& cs, std::string* why) {
  if (!cs.J.whole() && cs.facts.valid) {
    if (why) *why = cs.facts.sk_why;
    return cs.facts.sk_mode;
  }
  auto no = [&](const char* w) {
    if (why) *why = w;
    return (int)SK_GENERIC;
  };
  const Config& C = cs.cfg;
  if (C.mech_mode()) {   // species block on SK_MECH for Euler and N-S decks
    if (why) *why = "mechanism: SK_MECH";
    return SK_MECH;
  }
  if (C.ProblemType != SM_NS) return no("inviscid problem");
  if (!C.sources.empty()) return no("gas sources");
  if (C.chem_model == CRM_ARRENIUS) return no("finite-rate chemistry sources");
  if (!lean_single_gas(cs)) return no("species present");
  const real Rair = C.species.R[H_AIR];
  // boundary-condition bits alone leave turb_model() a no-op; the model bits
  // (or an initial-reset pass on any TurbType, which sets mu_t = 5 mu) do not
  const u64 model = TCT_k_eps_Model | TCT_Prandtl_Model | TCT_Integral_Model | TCT_Spalart_Allmaras_Model |
                    TCT_k_omega_Model | TCT_k_omega_SST_Model | TCT_Baldwin_Lomax_Model | TCT_nut_92_Model |
                    TCT_Smagorinsky_Model;
  bool laminar = true;
  for (const CellRecord& c : cs.J.c) {
    if ((c.TurbType & model) != 0 || (c.TurbType != 0 && C.isTurbulenceReset)) laminar = false;
    if (c.is(CT_SOLID)) continue;
    if (c.mu_t != 0. || c.lam_t != 0.) laminar = false;
    for (int k = 4; k < 4 + NCOMP; k++)
      if (c.Src[k] != 0.) return no("species sources");
    if (!(c.Y[0] == 0. && c.Y[1] == 0. && c.Y[2] == 0. && c.Y[3] == 1.)) return no("mixture fractions");
    if (C.chem_model != NO_REACTIONS && std::memcmp(&c.R, &Rair, sizeof(real)) != 0) return no("R != R_air");
  }
  if (why) *why = laminar ? "" : "turbulent: SK_SGT";
  return laminar ? SK_SGL : SK_SGT;
}

bool mech_species_cauchy(const Case& cs) {
  if (!cs.J.whole() && cs.facts.valid) return cs.facts.species_cauchy;
  for (const CellRecord& c : cs.J.c) {
    if (!is_active(c.CT)) continue;
    const EqFlags f = eq_flags(I_YFU, c.CT, c.TurbType, cs.cfg.ProblemType);
    if (f.dx2 || f.dy2) return true;
  }
  return false;
}

bool lean_single_gas(const Case& cs) {
  if (!cs.J.whole() && cs.facts.valid) return cs.facts.single_gas;
  static const real zero = 0.0;
  for (const CellRecord& c : cs.J.c)
    for (int k = 4; k < 4 + NCOMP; k++)
      if (std::memcmp(&c.S[k], &zero, sizeof(real)) != 0) return false;   // +0 only
  return true;
}

bool lean_any_cauchy_x(const Case& cs) {
  if (!cs.J.whole() && cs.facts.valid) return cs.facts.any_cauchy_x;
  for (const CellRecord& c : cs.J.c) {
    if (!is_active(c.CT)) continue;
    for (int k = 0; k < NEQ; k++)
      if (eq_flags(k, c.CT, c.TurbType, cs.cfg.ProblemType).dx2) return true;
  }
  return false;
}

std::vector<uint8_t> lean_flags(const HostArrays& h, int sm) {
  const long N = h.N;
  const int ny = h.ny;
  std::vector<uint8_t> lb(N);
  for (long idx = 0; idx < N; idx++) lb[idx] = h.nb[idx] & (NB_XL | NB_XR | NB_YU | NB_YD);
  // flag-free interior nodes (predict_core PLAIN fast path)
  for (long idx = 0; idx < N; idx++) {
    const u64 CT = h.CT[idx];
    if (!is_active(CT) || (h.nb[idx] & 15) != 15 || has_all(CT, CT_NONREFLECTED)) continue;
    bool plain = true;
    for (int k = 0; k < 4 + NCOMP && plain; k++) {
      const EqFlags f = eq_flags(k, CT, h.TT[idx], sm);
      plain = f.upd && f.dx && f.dy && !f.dx2 && !f.dy2 && !pass2_frozen(k, CT, h.TT[idx], sm);
    }
    if (plain) lb[idx] |= LB_PLAIN;
  }
  // a node whose predictor applies d2S/dx2 = 0 reads dS/dx of its x
  // neighbours (likewise y): those neighbours must keep publishing dS/dx.
  for (int i = 0; i < h.nx; i++)
    for (int j = 0; j < ny; j++) {
      const long idx = (long)i * ny + j;
      const u64 CT = h.CT[idx];
      if (!is_active(CT)) continue;
      bool dx2 = false, dy2 = false;
      for (int k = 0; k < NEQ; k++) {
        const EqFlags f = eq_flags(k, CT, h.TT[idx], sm);
        dx2 = dx2 || f.dx2;
        dy2 = dy2 || f.dy2;
      }
      const uint8_t nbm = h.nb[idx];
      const int n1 = (nbm & NB_XL) ? 1 : 0, n2 = (nbm & NB_XR) ? 1 : 0;
      const int n3 = (nbm & NB_YU) ? 1 : 0, n4 = (nbm & NB_YD) ? 1 : 0;
      if (dx2) {
        if (i - n1 >= 0) lb[(long)(i - n1) * ny + j] |= LB_DX_OUT;
        if (i + n2 < h.nx) lb[(long)(i + n2) * ny + j] |= LB_DX_OUT;
      }
      if (dy2) {
        lb[idx + n3] |= LB_DY_OUT;
        lb[idx - n4] |= LB_DY_OUT;
      }
    }
  return lb;
}

}  // namespace hf2d

namespace hf2d {

void compute_generic_flags(const Case& cs, HostArrays& h) {
  const long N = h.N;
  const std::vector<uint8_t> lb = lean_flags(h, cs.cfg.ProblemType);
  // (mechanism mode: the kinetics are operator-split, no species Src)
  const bool src_all = (cs.cfg.chem_model == CRM_ARRENIUS && !cs.cfg.mech_mode()) || !cs.cfg.sources.empty();
  static const real zero = 0.0;
  auto nonzero = [&](const std::vector<real>& a, long idx, int k0, int k1) {
    for (int k = k0; k < k1; k++)
      if (std::memcmp(&a[(size_t)k * N + idx], &zero, sizeof(real)) != 0) return true;   // +0 only
    return false;
  };
  h.gf.assign(N, 0);
  for (long idx = 0; idx < N; idx++) {
    uint8_t g = 0;
    if (lb[idx] & LB_DX_OUT) g |= GF_DX_OUT;
    if (lb[idx] & LB_DY_OUT) g |= GF_DY_OUT;
    if (src_all || nonzero(h.Src, idx, 0, 4 + NCOMP)) g |= GF_SRC;
    const u64 CT = h.CT[idx];
    const bool wall_gas = !has_all(CT, CT_SOLID) && (has_all(CT, CT_WALL_NO_SLIP) || has_all(CT, CT_WALL_LAW));
    if (wall_gas || nonzero(h.SrcAdd, idx, 0, NEQ)) g |= GF_SRCADD;
    h.gf[idx] = g;
  }
}

}  // namespace hf2d
