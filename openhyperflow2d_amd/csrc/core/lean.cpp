// Host side of the lean inviscid path (lean_euler.hpp): eligibility and the
// per-cell neighbour/publish byte.
#include <cstring>
#include <string>
#include <vector>

#include "lean_euler.hpp"
#include "solver.hpp"

namespace hf2d {

// The cell-level conditions of the eligibility tests below over the resident
// records of this Case (the whole field, or one strip of a windowed
// pre-processing), in x-major order; facts_merge() adds the deck-level
// conditions.  A strip rank's facts are the merge of every strip's part.
FactsPart Case::facts_part() const {
  FactsPart f;
  const Config& C = cfg;
  static const real zero = 0.0;
  const real Rair = C.species.R[H_AIR];
  const u64 model = TCT_k_eps_Model | TCT_Prandtl_Model | TCT_Integral_Model | TCT_Spalart_Allmaras_Model |
                    TCT_k_omega_Model | TCT_k_omega_SST_Model | TCT_Baldwin_Lomax_Model | TCT_nut_92_Model |
                    TCT_Smagorinsky_Model;
  for (const CellRecord& c : J.c) {
    for (int k = 4; k < 4 + NCOMP; k++)
      if (std::memcmp(&c.S[k], &zero, sizeof(real)) != 0) f.single_gas = false;   // +0 only
    if (is_active(c.CT)) {
      const EqFlags y = eq_flags(I_YFU, c.CT, c.TurbType, C.ProblemType);
      if (y.dx2 || y.dy2) f.species_cauchy = true;
      for (int k = 0; k < NEQ && !f.any_cauchy_x; k++)
        if (eq_flags(k, c.CT, c.TurbType, C.ProblemType).dx2) f.any_cauchy_x = true;
    }
    // lean inviscid: set nodes, no Src, no SrcAdd off no-slip walls
    // (equations >= 4 + NCOMP are frozen for inviscid nodes: their Src/SrcAdd
    // -- e.g. left by a k-eps initialisation -- are never read)
    if (f.lean_cells_ok && !c.is(CT_SOLID)) {
      const char* w = nullptr;
      if (!c.is(CT_NODE_IS_SET)) w = "unset non-solid node";
      for (int k = 0; k < 4 + NCOMP && !w; k++)
        if (c.Src[k] != 0.) w = "non-zero Src";
      if (!c.is(CT_WALL_NO_SLIP))
        for (int k = 0; k < 4 + NCOMP && !w; k++)
          if (c.SrcAdd[k] != 0.) w = "non-zero SrcAdd off no-slip walls";
      if (w) {
        f.lean_cells_ok = false;
        f.lean_why = w;
      }
    }
    // single-gas split kernels: the laminar test covers every cell up to the
    // first failing one (the whole-field scan stops there)
    if (f.sk_cells_ok) {
      if ((c.TurbType & model) != 0 || (c.TurbType != 0 && C.isTurbulenceReset)) f.laminar = false;
      if (!c.is(CT_SOLID)) {
        if (c.mu_t != 0. || c.lam_t != 0.) f.laminar = false;
        const char* w = nullptr;
        for (int k = 4; k < 4 + NCOMP && !w; k++)
          if (c.Src[k] != 0.) w = "species sources";
        if (!w && !(c.Y[0] == 0. && c.Y[1] == 0. && c.Y[2] == 0. && c.Y[3] == 1.)) w = "mixture fractions";
        if (!w && C.chem_model != NO_REACTIONS && std::memcmp(&c.R, &Rair, sizeof(real)) != 0) w = "R != R_air";
        if (w) {
          f.sk_cells_ok = false;
          f.sk_why = w;
        }
      }
    }
  }
  return f;
}

void Case::merge_facts(const std::vector<FactsPart>& parts) { facts = fold_facts(parts); }

CaseFacts Case::fold_facts(const std::vector<FactsPart>& parts) const {
  CaseFacts f;
  const Config& C = cfg;
  f.single_gas = true;
  for (const FactsPart& p : parts) {
    f.single_gas = f.single_gas && p.single_gas;
    f.any_cauchy_x = f.any_cauchy_x || p.any_cauchy_x;
    f.species_cauchy = f.species_cauchy || p.species_cauchy;
  }
  // lean inviscid
  f.lean_ok = false;
  if (C.ProblemType == SM_NS) f.lean_why = "viscous problem";
  else if (!C.sources.empty()) f.lean_why = "gas sources";
  else if (!C.isAdiabaticWall) f.lean_why = "wall heat transfer";
  else if (C.chem_model == CRM_ARRENIUS) f.lean_why = "finite-rate chemistry sources";
  else {
    f.lean_ok = true;
    for (const FactsPart& p : parts)   // the first failing cell in x-major (= rank) order
      if (!p.lean_cells_ok) {
        f.lean_ok = false;
        f.lean_why = p.lean_why;
        break;
      }
  }
  // single-gas split kernels
  f.sk_mode = SK_GENERIC;
  if (C.mech_mode()) {   // species block on SK_MECH for Euler and N-S decks
    f.sk_mode = SK_MECH;
    f.sk_why = "mechanism: SK_MECH";
  } else if (C.ProblemType != SM_NS) f.sk_why = "inviscid problem";
  else if (!C.sources.empty()) f.sk_why = "gas sources";
  else if (C.chem_model == CRM_ARRENIUS) f.sk_why = "finite-rate chemistry sources";
  else if (!f.single_gas) f.sk_why = "species present";
  else {
    bool laminar = true, ok = true;
    for (const FactsPart& p : parts) {
      laminar = laminar && p.laminar;
      if (!p.sk_cells_ok) {
        ok = false;
        f.sk_why = p.sk_why;
        break;
      }
    }
    if (ok) {
      f.sk_mode = laminar ? SK_SGL : SK_SGT;
      f.sk_why = laminar ? "" : "turbulent: SK_SGT";
    }
  }
  f.valid = true;
  return f;
}

std::string FactsPart::pack() const {
  std::string b;
  b += (char)single_gas;
  b += (char)any_cauchy_x;
  b += (char)species_cauchy;
  b += (char)lean_cells_ok;
  b += (char)sk_cells_ok;
  b += (char)laminar;
  b += lean_why;
  b += '\0';
  b += sk_why;
  return b;
}

FactsPart FactsPart::unpack(const std::string& b) {
  if (b.size() < 7) throw std::runtime_error("FactsPart::unpack: short blob");
  FactsPart f;
  f.single_gas = b[0];
  f.any_cauchy_x = b[1];
  f.species_cauchy = b[2];
  f.lean_cells_ok = b[3];
  f.sk_cells_ok = b[4];
  f.laminar = b[5];
  const size_t z = b.find('\0', 6);
  if (z == std::string::npos) throw std::runtime_error("FactsPart::unpack: bad blob");
  f.lean_why = b.substr(6, z - 6);
  f.sk_why = b.substr(z + 1);
  return f;
}

// The whole field's facts: a strip rank's merged ones (they must be there:
// a strip alone cannot tell), else one pass over the whole resident field.
static const CaseFacts& whole_facts(const Case& cs, CaseFacts& tmp) {
  if (!cs.J.whole()) {
    if (!cs.facts.valid) throw std::runtime_error("eligibility of a strip Case without the merged whole-field facts");
    return cs.facts;
  }
  // (folded into a local: the Case is not touched, so threads may share it)
  tmp = cs.fold_facts({cs.facts_part()});
  return tmp;
}

bool lean_eligible(const Case& cs, std::string* why) {
  CaseFacts t;
  const CaseFacts& f = whole_facts(cs, t);
  if (why) *why = f.lean_ok ? "" : f.lean_why;
  return f.lean_ok;
}

// Single-gas laminar N-S specialisation of the generic stepper (fill_cell /
// predict_cell_t <SGL>): only equations 0..3 and the fields the next step
// reads move through memory.  Requires species +0 everywhere, no species
// sources, no turbulence model, mu_t = lam_t = 0, Y = (0,0,0,1) and (with
// chemistry on) R = R_air everywhere -- then the generic stepper leaves every
// skipped field unchanged.  Boundary-condition bits alone leave turb_model()
// a no-op; the model bits (or an initial-reset pass on any TurbType, which
// sets mu_t = 5 mu) do not.
int sk_eligible(const Case& cs, std::string* why) {
  CaseFacts t;
  const CaseFacts& f = whole_facts(cs, t);
  if (why) *why = f.sk_why;
  return f.sk_mode;
}

bool mech_species_cauchy(const Case& cs) {
  CaseFacts t;
  return whole_facts(cs, t).species_cauchy;
}

bool lean_single_gas(const Case& cs) {
  CaseFacts t;
  return whole_facts(cs, t).single_gas;
}

bool lean_any_cauchy_x(const Case& cs) {
  CaseFacts t;
  return whole_facts(cs, t).any_cauchy_x;
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

void compute_generic_flags(const Case& cs, HostArrays& h, int gx0) {
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
  // WallBlendCells: the first N cells off every no-slip wall node along its
  // directions into the flow.  The ray lengths come from the whole grid
  // (Case::wall_rays: the first solid cell or the grid edge ends a ray,
  // whichever strip holds it), so every decomposition flags the same cells.
  const int nwb = cs.cfg.WallBlendCells;
  if (nwb > 0 && cs.cfg.ProblemType == SM_NS && cs.wall_rays.size() == 4 * cs.wall_nodes.size()) {
    static const int di[4] = {1, -1, 0, 0}, dj[4] = {0, 0, 1, -1};
    for (size_t w = 0; w < cs.wall_nodes.size(); w++) {
      for (int d = 0; d < 4; d++) {
        const int len = cs.wall_rays[4 * w + d];
        for (int n = 1; n <= len; n++) {
          const int gi = cs.wall_nodes[w].first + n * di[d], j = cs.wall_nodes[w].second + n * dj[d];
          const int li = gi - gx0;
          if (li < 0 || li >= h.nx) continue;   // (another strip's column)
          h.gf[(long)li * h.ny + j] |= d < 2 ? GF_WBX : GF_WBY;
        }
      }
    }
  }
}

}  // namespace hf2d
