// Geometry pre-processor: builds the initial cell field from the deck.
//
// Behavioural reference (re-implemented; the reference's ordering and
// integer-rounding rules are kept because they decide which cells become
// boundary / solid cells and therefore change the flow):
//   flow lists             deeps2d_core.cpp:2919-3164
//   SingleBounds/Contours  deeps2d_core.cpp:3267-3803, hyper_flow_bound.cpp:258-351,
//                          hyper_flow_bound_contour.cpp:52-220
//   init + first-init      deeps2d_core.cpp:3845-3965, :4510-4616
//   Rect/Circle/Airfoil    hyper_flow_solid_bound_rect.cpp, hyper_flow_bound_circle.cpp,
//                          hyper_flow_airfoil.cpp
//   Area flood fill        hyper_flow_area.cpp:66-186
//   wall / NRBC / BL / y+  deeps2d_core.cpp:2025-2388, :4783-4889
//   sources                hyper_flow_source.cpp:13-285
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <sstream>

#include "case.hpp"
#include <thread>
#include <atomic>
#include <limits>
#include "checkpoint.hpp"

namespace hf2d {

namespace {

constexpr real PI = 3.14159265358979323846;

u64 turb_model_bits(int m) {
  switch (m) {
    case 1: return TCT_Integral_Model;
    case 2: return TCT_Prandtl_Model;
    case 3: return TCT_Spalart_Allmaras_Model;
    case 4: return TCT_k_eps_Model;
    case 5: return TCT_Smagorinsky_Model;
    case 6: return TCT_k_omega_SST_Model;   // new: SST (not in the reference)
    default: return TCT_No_Turbulence;
  }
}

bool has(const std::string& s, const char* tok) { return s.find(tok) != std::string::npos; }

// strstr-based "Cond" token parsing (deeps2d_core.cpp:3311-3439 / :3569-3694).
void parse_cond(const std::string& s, bool single_bound, u64& ct, u64& tct) {
  struct T {
    const char* n;
    u64 v;
  };
  static const T atomic[] = {
      {"CT_Rho_CONST_2D", CT_Rho_CONST},         {"CT_U_CONST_2D", CT_U_CONST},
      {"CT_V_CONST_2D", CT_V_CONST},             {"CT_T_CONST_2D", CT_T_CONST},
      {"CT_Y_CONST_2D", CT_Y_CONST},             {"CT_WALL_LAW_2D", CT_WALL_LAW},
      {"CT_WALL_NO_SLIP_2D", CT_WALL_NO_SLIP},   {"CT_dRhodx_NULL_2D", CT_dRhodx_NULL},
      {"CT_dUdx_NULL_2D", CT_dUdx_NULL},         {"CT_dVdx_NULL_2D", CT_dVdx_NULL},
      {"CT_dTdx_NULL_2D", CT_dTdx_NULL},         {"CT_dYdx_NULL_2D", CT_dYdx_NULL},
      {"CT_dRhody_NULL_2D", CT_dRhody_NULL},     {"CT_dUdy_NULL_2D", CT_dUdy_NULL},
      {"CT_dVdy_NULL_2D", CT_dVdy_NULL},         {"CT_dTdy_NULL_2D", CT_dTdy_NULL},
      {"CT_dYdy_NULL_2D", CT_dYdy_NULL},         {"CT_d2Rhodx2_NULL_2D", CT_d2Rhodx2_NULL},
      {"CT_d2Udx2_NULL_2D", CT_d2Udx2_NULL},     {"CT_d2Vdx2_NULL_2D", CT_d2Vdx2_NULL},
      {"CT_d2Tdx2_NULL_2D", CT_d2Tdx2_NULL},     {"CT_d2Ydx2_NULL_2D", CT_d2Ydx2_NULL},
      {"CT_d2Rhody2_NULL_2D", CT_d2Rhody2_NULL}, {"CT_d2Udy2_NULL_2D", CT_d2Udy2_NULL},
      {"CT_d2Vdy2_NULL_2D", CT_d2Vdy2_NULL},     {"CT_d2Tdy2_NULL_2D", CT_d2Tdy2_NULL},
      {"CT_d2Ydy2_NULL_2D", CT_d2Ydy2_NULL},     {"CT_SOLID_2D", CT_SOLID},
      {"CT_BL_REFINEMENT_2D", CT_BL_REFINEMENT}, {"CT_NONREFLECTED_2D", CT_NONREFLECTED},
  };
  for (auto& t : atomic) {
    const char* name = t.n;
    // SingleBound parser looks for a misspelled token (deeps2d_core.cpp:3343)
    if (single_bound && t.v == CT_dYdy_NULL) name = "CT_dYdy_NULL_2D_2D";
    if (has(s, name)) ct |= t.v;
  }
  if (has(s, "TCT_k_eps_Model_2D"))
    tct |= TCT_k_eps_Model;
  else if (has(s, "TCT_Smagorinsky_Model_2D"))
    tct |= TCT_Smagorinsky_Model;
  else if (has(s, "TCT_Spalart_Allmaras_Model_2D"))
    tct |= TCT_Spalart_Allmaras_Model;
  else if (has(s, "TCT_Prandtl_Model_2D"))
    tct |= TCT_Prandtl_Model;
  else if (has(s, "TCT_Integral_Model_2D"))
    tct |= TCT_Integral_Model;
  else if (has(s, "TCT_k_omega_SST_Model_2D"))
    tct |= TCT_k_omega_SST_Model;
  if (has_all(tct, TCT_k_eps_Model) || has_all(tct, TCT_Spalart_Allmaras_Model) ||
      has_all(tct, TCT_k_omega_SST_Model)) {
    static const T turb[] = {
        {"TCT_k_CONST_2D", TCT_k_CONST},
        {"TCT_eps_CONST_2D", TCT_eps_CONST},
        {"TCT_dkdx_NULL_2D", TCT_dkdx_NULL},
        {"TCT_depsdx_NULL_2D", TCT_depsdx_NULL},
        {"TCT_dkdy_NULL_2D", TCT_dkdy_NULL},
        {"TCT_depsdy_NULL_2D", TCT_depsdy_NULL},
        {"TCT_d2kdx2_NULL_2D", TCT_d2kdx2_NULL},
        {"TCT_d2epsdx2_NULL_2D", TCT_d2epsdx2_NULL},
        {"TCT_d2kdy2_NULL_2D", TCT_d2kdy2_NULL},
        {"TCT_d2epsdy2_NULL_2D", TCT_d2epsdy2_NULL},
        {"TCT_eps_mud2kdx2_WALL_2D", TCT_eps_mud2kdx2_WALL},
        {"TCT_eps_mud2kdy2_WALL_2D", TCT_eps_mud2kdy2_WALL},
        {"TCT_eps_Cmk2kXn_WALL_2D", TCT_eps_Cmk2kXn_WALL},
    };
    for (auto& t : turb)
      if (has(s, t.n)) tct |= t.v;
  }
  if (has(s, "NT_AX_2D"))
    ct |= NT_AX;
  else if (has(s, "NT_AY_2D"))
    ct |= NT_AY;
  if (has(s, "NT_D0X_2D")) ct |= NT_D0X;
  if (has(s, "NT_D0Y_2D")) ct |= NT_D0Y;
  if (has(s, "NT_D2X_2D")) ct |= NT_D2X;
  if (has(s, "NT_D2Y_2D")) ct |= NT_D2Y;
  if (has(s, "NT_WALL_LAW_2D"))
    ct |= NT_WALL_LAW;
  else if (has(s, "NT_WNS_2D"))
    ct |= NT_WNS;
  if (has(s, "NT_FC_2D")) ct |= NT_FC;
  if (has(s, "NT_FARFIELD_2D")) ct |= NT_FARFIELD;
  if (has(s, "NT_S_2D")) ct |= NT_S;
  if (has(s, "NT_FALSE_2D")) ct |= CT_NODE_IS_SET;
}

const real* comp_Y(int comp, const real* mix) {
  static const real Yfu[4] = {1., 0., 0., 0.};
  static const real Yox[4] = {0., 1., 0., 0.};
  static const real Ycp[4] = {0., 0., 1., 0.};
  static const real Yair[4] = {0., 0., 0., 1.};
  switch (comp) {
    case 0: return Yfu;
    case 1: return Yox;
    case 2: return Ycp;
    case 3: return Yair;
    case 4: return mix;
    default: return nullptr;
  }
}

// One boundary segment (Bound2D).  Coordinates are node indices; the "f"
// versions keep the pre-truncation values used for the slope.
struct Segment {
  unsigned sx, sy, ex, ey;
  real fsx, fsy, fex, fey;
  int32_t bnt;   // int in the reference: OR-ing it sign-extends bit 31
  u64 btc;
  GasFlow* flow = nullptr;     // 1-D flow
  GasFlow* flow2d = nullptr;   // 2-D flow
  bool hasY = false;
  real Y[NSPEC] = {0, 0, 0, 0};
  bool active = false;
};

}  // namespace

// ---------------------------------------------------------------------------
// Pre-processing context: holds mutable state shared by the geometry steps.
// ---------------------------------------------------------------------------
struct PreCtx {
  Case& cs;
  real Ymix[4] = {0, 0, 0, 0};
  explicit PreCtx(Case& c) : cs(c) {}

  void assign_flow2d(CellRecord& n, const GasFlow& f) {
    const FillParams P = cs.cfg.fill_params();
    n.S[I_RHO] = f.ROG();
    n.S[I_RHOU] = f.ROG() * f.U();
    n.S[I_RHOV] = f.ROG() * f.V();
    n.S[I_K] = n.S[I_EPS] = 0.;
    n.U = f.U();
    n.V = f.V();
    n.p = f.Pg();
    n.R = f.Rg();
    n.lam = f.lam;
    n.mu = f.mu;
    n.Tg = f.Tg();
    n.CP = f.C;
    n.k = n.CP / (n.CP - n.R);
    n.Diff = (n.lam + n.lam_t) / n.CP;
    n.S[I_RHO] = f.Pg() / n.R / f.Tg();
    for (int i = 0; i < NCOMP; i++) n.S[i + 4] = n.Y[i] * n.S[I_RHO];
    real Tmp1 = n.S[I_RHO], Tmp3 = 0.;
    for (int i = 0; i < NCOMP; i++) {
      Tmp3 += P.Hu[i] * n.S[i + 4];
      Tmp1 -= n.S[i + 4];
    }
    Tmp3 += P.Hu[NCOMP] * Tmp1;
    n.S[I_RHOE] = n.p / (n.k - 1) + n.S[I_RHO] * (f.U() * f.U() + f.V() * f.V()) * 0.5 + Tmp3;
    for (int i = 0; i < NEQ; i++) n.Src[i] = 0;
    cs.fill_node(n, 0, 1);
  }

  // FlowNode2D::operator=(Flow&) — reproduces the reference's use of the
  // node's previous rho and Tg (hyper_flow_node.hpp:978-1012).
  void assign_flow(CellRecord& n, const GasFlow& f) {
    const FillParams P = cs.cfg.fill_params();
    n.S[I_RHOU] = f.ROG();
    n.S[I_RHOV] = f.ROG() * f.flow_Wg();
    n.S[I_RHOE] = n.S[NCOMP + 4] = n.S[NCOMP + 5] = 0.;
    n.p = f.P0();
    n.R = f.Rg();
    n.lam = f.lam;
    n.mu = f.mu;
    n.CP = f.C;
    n.k = n.CP / (n.CP - n.R);
    for (int i = 0; i < NCOMP; i++) n.S[i + 4] = n.S[I_RHO] * n.Y[i];
    real Tmp1 = n.S[I_RHO], Tmp3 = 0.;
    for (int i = 0; i < NCOMP; i++) {
      Tmp3 += P.Hu[i] * n.S[i + 4];
      Tmp1 -= n.S[i + 4];
    }
    Tmp3 += P.Hu[NCOMP] * Tmp1;
    n.S[I_RHO] = n.p / n.R / n.Tg;
    n.S[I_RHOE] = n.p / (n.k - 1.) + n.S[I_RHO] * (f.flow_Wg() * f.flow_Wg()) * 0.5 + Tmp3;
    for (int i = 0; i < NEQ; i++) n.Src[i] = 0;
    cs.fill_node(n, 0, 1);
  }

  // (flags of every cell; the rest of the record only where it is resident)
  void mark_cell(int i, int j, const Segment& s, real alpha) {
    Field& J = cs.J;
    J.ct(i, j) = J.ct(i, j) | (u64)(int64_t)s.bnt | CT_NODE_IS_SET;
    J.tt(i, j) = s.btc;
    if (!J.resident(i)) return;
    CellRecord& n = J.at(i, j);
    n.NGX = (3 - n.idXr - n.idXl);
    n.NGY = (3 - n.idYu - n.idYd);
    n.BGX = std::cos(alpha);
    n.BGY = std::sin(alpha);
    if (s.hasY)
      for (int ii = 0; ii < NSPEC; ii++) n.Y[ii] = s.Y[ii];
    if (s.flow)
      assign_flow(n, *s.flow);
    else if (s.flow2d)
      assign_flow2d(n, *s.flow2d);
    else
      cs.fill_node(n, 0, 0);
  }

  // Bound2D::SetBound (hyper_flow_bound.cpp:258-351)
  bool set_segment(Segment s) {
    Field& J = cs.J;
    const unsigned MX = (unsigned)J.nx, MY = (unsigned)J.ny;
    if (s.sx > MX || s.sy > MY || s.ex > MX || s.ey > MY) return false;
    if (s.sx == MX) s.sx = MX - 1;
    if (s.sy == MY) s.sy = MY - 1;
    if (s.ex == MX) s.ex = MX - 1;
    if (s.ey == MY) s.ey = MY - 1;
    const real DX = s.fsx - s.fex, DY = s.fsy - s.fey;
    real Alpha;
    if (DX != 0) {
      Alpha = std::atan(DY / DX);
    } else {
      Alpha = PI / 2.;
    }
    auto mark = [&](unsigned i, unsigned j) {
      if (i >= MX || j >= MY) throw DeckError("bound segment leaves the computation area");
      mark_cell((int)i, (int)j, s, Alpha);
    };
    if (std::fabs(DX) > std::fabs(DY)) {
      const unsigned j1 = std::min(s.sx, s.ex);
      const unsigned k1 = (j1 == s.sx) ? s.sy : s.ey;
      const unsigned j2 = std::max(s.sx, s.ex);
      for (unsigned i = j1; i <= j2; i++) {
        const unsigned j = k1 + (int)((real)(i - j1) * std::tan(Alpha));
        mark(i, j);
      }
    } else {
      const unsigned j1 = std::min(s.sy, s.ey);
      const unsigned k1 = (j1 == s.sy) ? s.sx : s.ex;
      const unsigned j2 = std::max(s.sy, s.ey);
      for (unsigned i = j1; i <= j2; i++) {
        unsigned j;
        if (std::tan(Alpha) != 0.)
          j = k1 + (int)((real)(i - j1) / std::tan(Alpha));
        else
          j = k1;
        mark(j, i);
      }
    }
    return true;
  }

  Segment make_segment(unsigned x1, unsigned y1, unsigned x2, unsigned y2, u64 bt, GasFlow* f1,
                       GasFlow* f2, const real* Y, u64 btc) {
    Segment s;
    s.sx = x1;
    s.sy = y1;
    s.ex = x2;
    s.ey = y2;
    s.fsx = (real)x1;
    s.fsy = (real)y1;
    s.fex = (real)x2;
    s.fey = (real)y2;
    s.bnt = (int32_t)(uint32_t)(bt & 0xffffffffULL);
    s.btc = (u64)(int64_t)(int32_t)(uint32_t)(btc & 0xffffffffULL);
    s.flow = f1;
    s.flow2d = f2;
    if (Y) {
      s.hasY = true;
      for (int i = 0; i < NSPEC; i++) s.Y[i] = Y[i];
    }
    return s;
  }

  // BoundContour2D: closed polyline of segments.
  struct Contour {
    unsigned first_x, first_y, cur_x, cur_y;
    std::vector<Segment> segs;
    bool closed = false;
  };

  void contour_add(Contour& c, unsigned x, unsigned y, u64 bt, GasFlow* f1, GasFlow* f2, const real* Y,
                   u64 btc) {
    if (c.closed) return;
    c.segs.push_back(make_segment(c.cur_x, c.cur_y, x, y, bt, f1, f2, Y, btc));
    c.cur_x = x;
    c.cur_y = y;
  }
  bool contour_close(Contour& c, u64 bt, GasFlow* f1, GasFlow* f2, const real* Y, u64 btc) {
    if (c.closed || c.segs.size() < 2) return false;
    c.segs.push_back(make_segment(c.cur_x, c.cur_y, c.first_x, c.first_y, bt, f1, f2, Y, btc));
    c.cur_x = c.first_x;
    c.cur_y = c.first_y;
    c.closed = true;
    return true;
  }
  void contour_set(Contour& c, const std::string& name) {
    if (!c.closed) throw DeckError("Contour \"" + name + "\" is not looped.");
    for (size_t i = 0; i < c.segs.size(); i++)
      if (!set_segment(c.segs[i]))
        throw DeckError("Set Bound error (bound No. " + std::to_string(i + 1) + ") in \"" + name + "\"");
  }
  // Rotation of an inactive contour about (x0, y0) in node units.  The
  // reference reads an uninitialised dx here (Bound2D::RotateBound2D), so
  // this path has no pinned reference behaviour.
  bool contour_rotate(Contour& c, real x0, real y0, real angle) {
    auto rot = [&](real x, real y, real& xn, real& yn) {
      real dxs = x - x0, dys = y - y0;
      real fi = std::atan2(dxs, dys), r = std::sqrt(dxs * dxs + dys * dys + 1.e-30);
      xn = x0 + r * std::sin(fi + angle);
      yn = y0 + r * std::cos(fi + angle);
      return xn >= 0 && yn >= 0 && xn < cs.J.nx && yn < cs.J.ny;
    };
    for (auto& s : c.segs) {
      real a, b;
      if (!rot(s.fsx, s.fsy, a, b) || !rot(s.fex, s.fey, a, b)) return false;
    }
    for (auto& s : c.segs) {
      real a, b;
      rot(s.fsx, s.fsy, a, b);
      s.fsx = a;
      s.fsy = b;
      s.sx = (unsigned)a;
      s.sy = (unsigned)b;
      rot(s.fex, s.fey, a, b);
      s.fex = a;
      s.fey = b;
      s.ex = (unsigned)a;
      s.ey = (unsigned)b;
    }
    return true;
  }

  // Area2D::FillArea2D — level-synchronous flood fill from a seed node
  // (over the whole grid's flags; flows and fills of resident records only).
  void fill_area(unsigned X, unsigned Y, u64 bnt, const GasFlow* f2d, const real* pY, u64 att) {
    Field& J = cs.J;
    const unsigned XMax = (unsigned)J.nx, YMax = (unsigned)J.ny;
    if (!(XMax > X && YMax > Y))
      throw DeckError("Init Area point [" + std::to_string(X) + "," + std::to_string(Y) + "] out of range.");
    if (J.is(X, Y, CT_NODE_IS_SET))
      throw DeckError("Init Area point [" + std::to_string(X) + "," + std::to_string(Y) +
                      "] already in initialized node.");
    const u64 ANT = bnt | CT_NODE_IS_SET;
    const u64 ATT = att;
    std::vector<std::pair<unsigned, unsigned>> BNA, FNA;
    J.ct(X, Y) = ANT;
    J.tt(X, Y) = ATT;
    BNA.push_back({X, Y});
    while (!BNA.empty()) {
      for (size_t q = 0; q < BNA.size(); q++) {
        const unsigned tX = BNA[q].first, tY = BNA[q].second;
        CellRecord* n = J.resident(tX) ? &J.at(tX, tY) : nullptr;
        if (n) {
          if (pY)
            for (int ii = 0; ii < NSPEC; ii++) n->Y[ii] = pY[ii];
          if (f2d) assign_flow2d(*n, *f2d);
          n->BGX = 1.;
          n->BGY = 1.;
          n->NGX = 1;
          n->NGY = 1;
          n->idXl = n->idYu = n->idXr = n->idYd = 1;
        }
        const bool n_solid = J.is(tX, tY, CT_SOLID);
        auto visit = [&](unsigned x, unsigned y, int side) {
          if (!J.is(x, y, CT_NODE_IS_SET)) {
            J.ct(x, y) = ANT;
            J.tt(x, y) = ATT;
            FNA.push_back({x, y});
          } else if (!J.is(x, y, CT_SOLID) && n_solid && J.resident(x)) {
            CellRecord& m = J.at(x, y);
            switch (side) {
              case 0: m.NGX = 0; m.idXr = 0; break;   // left neighbour
              case 1: m.NGX = 0; m.idXl = 0; break;   // right neighbour
              case 2: m.NGY = 0; m.idYu = 0; break;   // down neighbour
              case 3: m.NGY = 0; m.idYd = 0; break;   // up neighbour
            }
          }
        };
        if (tX > 0) visit(tX - 1, tY, 0);
        if (tX < XMax - 1) visit(tX + 1, tY, 1);
        if (tY > 0) visit(tX, tY - 1, 2);
        if (tY < YMax - 1) visit(tX, tY + 1, 3);
        if (n) cs.fill_node(*n, 1, 0);
      }
      BNA.swap(FNA);
      FNA.clear();
    }
  }
};

// ---------------------------------------------------------------------------

void Field::resize(int X, int Y) {
  nx = X;
  ny = Y;
  i0 = 0;
  nxl = X;
  c.assign((size_t)X * Y, CellRecord{});
  std::memset((void*)c.data(), 0, c.size() * sizeof(CellRecord));
}

void Field::resize_window(int X, int Y, int a, int b) {
  a = std::max(a, 0);
  b = std::min(b, X);
  nx = X;
  ny = Y;
  i0 = a;
  nxl = std::max(b - a, 0);
  c.assign((size_t)nxl * Y, CellRecord{});
  if (!c.empty()) std::memset((void*)c.data(), 0, c.size() * sizeof(CellRecord));
  g.assign((size_t)X * Y, CellFlags{});
}

void Field::trim(int a, int b) {
  a = std::max(a, i0);
  b = std::min(b, i0 + nxl);
  if (a >= b) throw std::runtime_error("Field::trim: empty column range");
  std::vector<CellRecord> k((size_t)(b - a) * ny);
  std::memcpy((void*)k.data(), (const void*)&at(a, 0), k.size() * sizeof(CellRecord));
  c.swap(k);
  i0 = a;
  nxl = b - a;
}

void Case::trim_to_columns(int a, int b) {
  if (J.whole() && !facts.valid) compute_facts();   // a strip alone cannot tell
  a = std::max(a, J.i0);
  b = std::min(b, J.i0 + J.nxl);
  if (!mech_rhoY.empty()) {
    const int ns = (int)(mech_rhoY.size() / (size_t)mech_n());
    std::vector<real> k((size_t)ns * (b - a) * J.ny);
    const size_t per = (size_t)(b - a) * J.ny;
    for (int s = 0; s < ns; s++)
      std::memcpy(&k[(size_t)s * per], &mech_rhoY[mech_idx(s, a, 0)], per * sizeof(real));
    mech_rhoY.swap(k);
  }
  J.trim(a, b);
}

void Case::fill_node(CellRecord& n, int is_mu_t, int is_init) const {
  FillParams P = cfg.fill_params();
  P.is_mu_t = is_mu_t;
  P.is_init = is_init;
  P.sm = SM_NS;   // FillNode2D default argument
  hf2d::fill_node(n, P);
}

// (a record of another strip's column, read from the checkpoint: it gets
// every per-record change the whole-field pre-processing made to it by the
// time of the call -- scan_area's turbulence reset)
const CellRecord* Case::far_record(int i, int j) {
  if (J.resident(i)) return &J.at(i, j);
  if (!preloaded) return nullptr;
  const long key = (long)i * J.ny + j;
  FarRec* e = nullptr;
  for (auto& f : far_cache)
    if (f.key == key) e = &f;
  if (!e) {
    CellRecord r;
    if (!read_hf2d_record(swap_path, J.nx, J.ny, i, j, r)) throw std::runtime_error("cannot read record of " + swap_path);
    far_cache.push_back({key, r, false});
    e = &far_cache.back();
  }
  if (far_turb_reset && !e->reset) {
    turb_reset_record(e->r, J.tt(i, j));
    e->reset = true;
  }
  return &e->r;
}

Case Case::from_deck_window(InputDeck deck, const std::string& workdir, bool use_checkpoint, int a, int b,
                            std::ostream* log) {
  Case cs;
  cs.win_a = std::max(a, 0);
  cs.win_b = b;
  cs.log = log;
  cs.load_and_preprocess(deck, workdir, use_checkpoint);
  cs.J.drop_flags();
  std::vector<FarRec>().swap(cs.far_cache);
  cs.win_a = cs.win_b = -1;
  return cs;
}

std::vector<std::pair<int, int>> Case::partition_deck(InputDeck deck, const std::string& workdir, bool use_checkpoint,
                                                      int nparts) {
  Case cs;   // flags only: an empty window
  cs.win_a = cs.win_b = 0;
  cs.load_and_preprocess(deck, workdir, use_checkpoint, true);
  return balanced_columns(cs.J, nparts);
}

Case Case::from_deck(InputDeck deck, const std::string& workdir, bool use_checkpoint, std::ostream* log) {
  Case cs;
  cs.log = log;
  cs.load_and_preprocess(deck, workdir, use_checkpoint);
  return cs;
}

void Case::load_and_preprocess(InputDeck& deck, const std::string& workdir, bool use_checkpoint, bool flags_only) {
  Case& cs = *this;
  cs.cfg.load_globals(deck);
  if (cs.cfg.chem_model == CRM_ARRENIUS && !cs.cfg.mechanism.empty()) {
    cs.cfg.mech = load_mechanism(cs.cfg.mechanism, workdir);
    cs.cfg.mech->data.nsub = cs.cfg.chem_nsub;
    cs.cfg.mech->data.Tchem = cs.cfg.chem_tmin;
    if (cs.cfg.mech->data.slot_sp[3] < 0 && cs.cfg.mech->data.slot_sp[0] < 0)
      throw DeckError("mechanism " + cs.cfg.mech->name + " has no slot map (slot fuel|ox|cp|air records)");
  }
  cs.preprocess(deck, workdir, use_checkpoint);
  if (cs.cfg.mech_mode() && !flags_only) {
    if (!cs.cfg.sources.empty())
      throw DeckError("SourceList2D species sources are not supported in mechanism mode (NumSrc must be 0)");
    if (!(cs.preloaded && read_species_sidecar(cs.species_path(), *cs.cfg.mech, cs.J.nx, cs.J.ny, cs.mech_rhoY,
                                                cs.J.i0, cs.J.i0 + cs.J.nxl))) {
      if (cs.preloaded)
        throw DeckError("checkpoint " + cs.swap_path + " has no matching species sidecar (" + cs.species_path() +
                        ") for mechanism " + cs.cfg.mech->name);
      cs.init_mechanism(cs.mech_rhoY);
      cs.apply_mechanism_state(cs.mech_rhoY);
    } else {
      cs.refresh_mechanism_primitives();
    }
  }
}

void Case::preprocess(InputDeck& d, const std::string& workdir, bool use_checkpoint) {
  Config& C = cfg;
  PreCtx px(*this);
  auto say = [&](const std::string& s) {
    if (log) *log << s << std::flush;
  };
  const int NumFlow = d.get_int("NumFlow");
  const int NumFlow2D = d.get_int("NumFlow2D");
  const int NumArea = d.get_int("NumArea");
  const int NumContour = d.get_int("NumContour");
  C.project = d.get_string("ProjectName");
  C.swap_file = C.project + d.get_string("GasSwapFile");
  C.out_file = C.project + d.get_string("OutputFile");
  C.tecplot_file = "tp-" + C.out_file;
  C.err_file = C.project + d.get_string("ErrorFile");
  C.Ts0 = d.get_float("Ts0");
  C.isOutHeatFluxX = d.get_int("isOutHeatFluxX");
  if (C.isOutHeatFluxX) {
    C.Cp_Flow_index = d.get_int("Cp_Flow_Index");
    C.y_max = d.get_int("y_max");
    C.y_min = d.get_int("y_min");
  }
  C.isOutHeatFluxY = d.get_int("isOutHeatFluxY");
  C.is_p_asterisk_out = d.get_int("is_p_asterisk_out");
  const SpeciesProps& sp = C.species;

  auto props_for = [&](int comp, real Tg, const std::string& prefix, real& Cp, real& lam, real& mu,
                       real& Rg) {
    if (comp >= 0 && comp <= 3) {
      const int h = comp == 0 ? H_FU : comp == 1 ? H_OX : comp == 2 ? H_CP : H_AIR;
      Cp = table_eval(sp.Cp[h], Tg);
      lam = table_eval(sp.lam[h], Tg);
      mu = table_eval(sp.mu[h], Tg);
      Rg = sp.R[h];
    } else if (comp == 4) {
      px.Ymix[0] = d.get_float(prefix + ".Y_fuel");
      px.Ymix[1] = d.get_float(prefix + ".Y_ox");
      px.Ymix[2] = d.get_float(prefix + ".Y_cp");
      // Reference sign error kept (Q10): Y_air = 1 - Yf + Yo + Yc.  Decks
      // using the new finite-rate chemistry get the corrected closure.
      if (C.chem_model == CRM_ARRENIUS)
        px.Ymix[3] = 1 - (px.Ymix[0] + px.Ymix[1] + px.Ymix[2]);
      else
        px.Ymix[3] = 1 - px.Ymix[0] + px.Ymix[1] + px.Ymix[2];
      Cp = px.Ymix[0] * table_eval(sp.Cp[H_FU], Tg) + px.Ymix[1] * table_eval(sp.Cp[H_OX], Tg) +
           px.Ymix[2] * table_eval(sp.Cp[H_CP], Tg) + px.Ymix[3] * table_eval(sp.Cp[H_AIR], Tg);
      lam = px.Ymix[0] * table_eval(sp.lam[H_FU], Tg) + px.Ymix[1] * table_eval(sp.lam[H_OX], Tg) +
            px.Ymix[2] * table_eval(sp.lam[H_CP], Tg) + px.Ymix[3] * table_eval(sp.lam[H_AIR], Tg);
      mu = px.Ymix[0] * table_eval(sp.mu[H_FU], Tg) + px.Ymix[1] * table_eval(sp.mu[H_OX], Tg) +
           px.Ymix[2] * table_eval(sp.mu[H_CP], Tg) + px.Ymix[3] * table_eval(sp.mu[H_AIR], Tg);
      Rg = px.Ymix[0] * sp.R[H_FU] + px.Ymix[1] * sp.R[H_OX] + px.Ymix[2] * sp.R[H_CP] +
           px.Ymix[3] * sp.R[H_AIR];
    } else {
      throw DeckError("Bad component index \"" + std::to_string(comp) + "\" use in " + prefix);
    }
  };

  // ---- Flow list ----
  flows.clear();
  for (int i = 0; i < NumFlow; i++) {
    const std::string pre = "Flow" + std::to_string(i + 1);
    real Pg = d.get_float(pre + ".p");
    real Tg = d.get_float(pre + ".T");
    int comp = d.get_int(pre + ".CompIndex");
    real Cp, lam, mu, Rg;
    props_for(comp, Tg, pre, Cp, lam, mu, Rg);
    GasFlow f(Cp, Tg, Pg, Rg, lam, mu);
    int type = d.get_int(pre + ".Type");
    if (type == 0)
      f.flow_LAM(d.get_float(pre + ".Lam"));
    else
      f.flow_Wg(d.get_float(pre + ".W"));
    flows.push_back(f);
  }
  // ---- Flow2D list ----
  flows2d.clear();
  for (int i = 0; i < NumFlow2D; i++) {
    const std::string pre = "Flow2D-" + std::to_string(i + 1);
    int comp = d.get_int(pre + ".CompIndex");
    real Pg = d.get_float(pre + ".p");
    real Tg = d.get_float(pre + ".T");
    real Cp, lam, mu, Rg;
    props_for(comp, Tg, pre, Cp, lam, mu, Rg);
    real Ug = d.get_float(pre + ".U");
    real Vg = d.get_float(pre + ".V");
    int mode = d.get_int(pre + ".Mode");
    if (mode == 2) Ug = Vg = 0;
    GasFlow f = GasFlow::make2d(mu, lam, Cp, Tg, Pg, Rg, Ug, Vg);
    if (mode == 0) f.CorrectFlow(Tg, Pg, std::sqrt(Ug * Ug + Vg * Vg + 1.e-30), false);
    if (mode == 2 || mode == 3) {
      real Mach = d.get_float(pre + ".Mach");
      real Angle = d.get_float(pre + ".Angle");
      if (mode == 2) f.CorrectFlow(Tg, Pg, Mach, true);
      f.MACH2d(Mach);
      real Wg = f.Wg2d();
      Ug = std::cos(Angle * M_PI / 180) * Wg;
      Vg = std::sin(Angle * M_PI / 180) * Wg;
      f.set_UV(Ug, Vg);
    }
    flows2d.push_back(f);
    if (log) {
      char b[512];
      std::snprintf(b, sizeof b, "Add object \"Flow2D-%d Mach=%g U=%g m/sec V=%g m/sec Wg=%g m/sec T=%g K p=%g Pa\"...OK\n",
                    i + 1, f.flow_MACH(), f.U(), f.V(), f.Wg2d(), f.Tg(), f.Pg());
      say(b);
    }
  }
  // ---- XCuts ----
  C.xcuts.clear();
  int NumXCut = d.get_int("NumXCut");
  for (int i = 0; i < NumXCut; i++) {
    const std::string pre = "CutX-" + std::to_string(i + 1);
    XCut x;
    x.x0 = d.get_float(pre + ".x0");
    x.y0 = d.get_float(pre + ".y0");
    x.dy = d.get_float(pre + ".dy");
    C.xcuts.push_back(x);
  }

  // ---- Swap file (checkpoint) ----
  if (win_a >= 0)
    J.resize_window(C.MaxX, C.MaxY, win_a, win_b);
  else
    J.resize(C.MaxX, C.MaxY);
  preloaded = false;
  swap_path = workdir.empty() ? C.swap_file : (workdir + "/" + C.swap_file);
  if (use_checkpoint) {
    // an all-zero image is the placeholder a failed first cycle leaves behind
    // (create_zero_hf2d): not a checkpoint
    bool any_set = false;
    if (J.windowed() ? read_hf2d_window(swap_path, J) : read_hf2d(swap_path, J)) {
      for (const CellRecord& c : J.c)
        if (c.CT != 0) {
          any_set = true;
          break;
        }
      for (size_t q = 0; q < J.g.size() && !any_set; q++) any_set = J.g[q].CT != 0;
    }
    if (!any_set) {
      std::fill(J.c.begin(), J.c.end(), CellRecord{});
      std::fill(J.g.begin(), J.g.end(), CellFlags{});
    }
    if (any_set) {
      preloaded = true;
      say("Mapping computation area...OK (preloaded " + swap_path + ")\n");
      // the reference restarts its iteration counter at 0 (it is not in the
      // .hf2d image); the sidecar makes a resumed run continue the count
      double mdt = 0, mtime = 0;
      long mit = 0;
      if (read_meta(swap_path, mit, mdt, mtime) && mit > 0) restart_iter = mit;
    }
  }
  const bool PreloadFlag = preloaded;
  const bool p_g = preloaded;

  auto flow_index = [&](const std::string& key2d, const std::string& key1d, GasFlow*& f1, GasFlow*& f2,
                        int& comp) {
    int FlowIndex = d.get_int_or(key2d, 0);
    f1 = f2 = nullptr;
    if (FlowIndex < 1) {
      FlowIndex = d.get_int(key1d);
      if (FlowIndex < 1 || FlowIndex > (int)flows.size())
        throw DeckError("Bad Flow index [" + std::to_string(FlowIndex) + "]");
      f1 = &flows[FlowIndex - 1];
      comp = d.get_int("Flow" + std::to_string(FlowIndex) + ".CompIndex");
    } else if (FlowIndex <= (int)flows2d.size()) {
      f2 = &flows2d[FlowIndex - 1];
      comp = d.get_int("Flow2D-" + std::to_string(FlowIndex) + ".CompIndex");
    } else {
      throw DeckError("Bad Flow index [" + std::to_string(FlowIndex) + "]");
    }
  };

  // ---- Single bounds ----
  const int numSingleBounds = d.get_int("NumSingleBounds");
  for (int i = 1; i <= numSingleBounds; i++) {
    const std::string nm = "SingleBound" + std::to_string(i);
    const Table& T = d.get_table(nm + ".Points");
    unsigned s_x = (unsigned)(T.X(0) / C.dx), s_y = (unsigned)(T.Y(0) / C.dy);
    unsigned e_x = (unsigned)(T.X(1) / C.dx), e_y = (unsigned)(T.Y(1) / C.dy);
    std::string cond = d.get_string(nm + ".Cond");
    int tm = d.get_int(nm + ".TurbulenceModel");
    u64 ct = CT_NO_COND, tct = turb_model_bits(tm);
    parse_cond(cond, true, ct, tct);
    if (ct == CT_NO_COND) throw DeckError("Unknown condition type " + cond + " in " + nm);
    GasFlow *f1, *f2;
    int comp = 3;
    flow_index(nm + ".Flow2D", nm + ".Flow", f1, f2, comp);
    const real* Y = comp_Y(comp, px.Ymix);
    int is_reset = d.get_int(nm + ".isReset");
    if (!p_g) is_reset = 1;
    d.get_int_or(nm + ".MaterialID", 0);
    if (!is_reset) f1 = f2 = nullptr;
    Segment s = px.make_segment(s_x, s_y, e_x, e_y, ct, f1, f2, Y, tct);
    s.fsx = (real)s_x;
    s.fsy = (real)s_y;
    s.fex = (real)e_x;
    s.fey = (real)e_y;
    px.set_segment(s);
  }

  // ---- Contours ----
  for (int jc = 0; jc < NumContour; jc++) {
    const std::string nm = "Contour" + std::to_string(jc + 1);
    const Table& T = d.get_table(nm);
    PreCtx::Contour c;
    c.first_x = c.cur_x = (unsigned)std::max((int)(T.X(0) / C.dx), 0);
    c.first_y = c.cur_y = (unsigned)std::max((int)(T.Y(0) / C.dy - 1), 0);
    d.get_int_or(nm + ".MaterialID", 0);
    u64 ct = 0, tct = 0;
    GasFlow *f1 = nullptr, *f2 = nullptr;
    const real* Y = nullptr;
    int is_reset = 1;
    const int nn = T.size();
    for (int i = 1; i < nn + 1; i++) {
      const std::string bn = nm + ".Bound" + std::to_string(i);
      std::string cond = d.get_string(bn + ".Cond");
      int tm = d.get_int(bn + ".TurbulenceModel");
      ct = CT_NO_COND;
      tct = turb_model_bits(tm);
      parse_cond(cond, false, ct, tct);
      if (ct == CT_NO_COND && tct == 0) throw DeckError("Unknown condition type " + cond + " in " + bn);
      int comp = 3;
      flow_index(bn + ".Flow2D", nm + ".Flow", f1, f2, comp);
      Y = comp_Y(comp, px.Ymix);
      is_reset = d.get_int(bn + ".isReset");
      if (!p_g) is_reset = 1;
      if (i < nn) {
        unsigned ix = (unsigned)std::max((int)(T.X(i) / C.dx), 0);
        unsigned iy = (unsigned)std::max((int)(T.Y(i) / C.dy - 1), 0);
        if (!is_reset) f1 = f2 = nullptr;
        px.contour_add(c, ix, iy, ct, f1, f2, Y, tct);
      }
    }
    if (!is_reset) f1 = f2 = nullptr;
    px.contour_close(c, ct, f1, f2, Y, tct);
    px.contour_set(c, nm);
  }

  // ---- initial dt from the flow lists ----
  dt0 = 1;
  {
    const real CFL_min = std::min<real>(C.CFL, C.CFL_Scenario.eval(0));
    for (auto& f : flows)
      dt0 = std::min<real>(dt0, CFL_min * std::min<real>(C.dx / (f.Asound() + f.flow_Wg()), C.dy / (f.Asound() + f.flow_Wg())));
    for (auto& f : flows2d)
      dt0 = std::min<real>(dt0, CFL_min * std::min<real>(C.dx / (f.Asound() + f.Wg2d()), C.dy / (f.Asound() + f.Wg2d())));
  }

  if (!PreloadFlag) {
    for (int j = 0; j < C.MaxY; j++)
      for (int i = J.i0; i < J.i0 + J.nxl; i++) {
        CellRecord& n = J.at(i, j);
        n.x = (i + 0.5) * C.dx;
        n.y = (j + 0.5) * C.dy;
        n.Tf = sp.Tf;
        n.BGX = 1.;
        n.BGY = 1.;
        n.NGX = 0;
        n.NGY = 0;
        for (int k = 0; k < NEQ; k++) n.Src[k] = n.SrcAdd[k] = 0;
      }
  }

  C.is_Cx_calc = d.get_int("is_Cx_calc");
  if (C.is_Cx_calc) {
    C.x0_body = d.get_float("x_body");
    C.y0_body = d.get_float("y_body");
    C.dx_body = d.get_float("dx_body");
    C.dy_body = d.get_float("dy_body");
    C.Cx_Flow_index = d.get_int("Cx_Flow_Index");
  }
  C.is_Cd_calc = d.get_int("is_Cd_calc");
  if (C.is_Cd_calc) {
    C.x0_nozzle = d.get_float("x_nozzle");
    C.y0_nozzle = d.get_float("y_nozzle");
    C.dy_nozzle = d.get_float("dy_nozzle");
    C.Cd_Flow_index = d.get_int("Cd_Flow_Index");
    C.p_ambient = d.get_float("p_ambient");
  }

  auto flow2d_for = [&](const std::string& key, int& comp) -> GasFlow* {
    int FlowIndex = d.get_int(key);
    if (FlowIndex < 1 || FlowIndex > (int)flows2d.size())
      throw DeckError("Bad Flow index [" + std::to_string(FlowIndex) + "]");
    comp = d.get_int("Flow2D-" + std::to_string(FlowIndex) + ".CompIndex");
    if (comp < 0 || comp > 4) throw DeckError("Bad component index [" + std::to_string(comp) + "]");
    return &flows2d[FlowIndex - 1];
  };

  // ---- Rects ----
  const int numRects = d.get_int("NumRects");
  C.InitTime = d.get_float("InitTime");
  global_time = C.InitTime;
  for (int r = 0; r < numRects; r++) {
    const std::string nm = "Rect" + std::to_string(r + 1);
    real Xs = d.get_float(nm + ".Xstart"), Ys = d.get_float(nm + ".Ystart");
    real DXr = d.get_float(nm + ".DX"), DYr = d.get_float(nm + ".DY");
    int comp;
    GasFlow* f2 = flow2d_for(nm + ".Flow2D", comp);
    int tm = d.get_int(nm + ".TurbulenceModel");
    u64 TM = turb_model_bits(tm);
    const real* Y = comp_Y(comp, px.Ymix);
    if (PreloadFlag) continue;
    // SolidBoundRect2D zeroes the shared Flow2D velocity (kept: Flow2D list is mutated)
    f2->set_U(0.);
    f2->set_V(0.);
    PreCtx::Contour c;
    c.first_x = c.cur_x = (unsigned)(Xs / C.dx + 0.4999);
    c.first_y = c.cur_y = (unsigned)(Ys / C.dy + 0.4999);
    real xx1 = Xs, yy1 = Ys, xx2, yy2;
    const bool ke = has_all(TM, TCT_k_eps_Model);
    auto ttf = [&](u64 extra) { return ke ? (TM | extra) : TM; };
    xx2 = xx1 + DXr;
    yy2 = yy1;
    px.contour_add(c, (unsigned)(xx2 / C.dx + 0.4999), (unsigned)(yy2 / C.dy + 0.4999), NT_WNS, nullptr, f2, Y,
                   ttf(TCT_dkdy_NULL | TCT_k_CONST | TCT_eps_mud2kdy2_WALL));
    xx1 = xx2;
    yy1 = yy2;
    xx2 = xx1;
    yy2 = yy1 + DYr;
    px.contour_add(c, (unsigned)(xx2 / C.dx + 0.4999), (unsigned)(yy2 / C.dy + 0.4999), NT_WNS, nullptr, f2, Y,
                   ttf(TCT_dkdx_NULL | TCT_k_CONST | TCT_eps_mud2kdx2_WALL));
    xx1 = xx2;
    yy1 = yy2;
    xx2 = xx1 - DXr;
    yy2 = yy1;
    px.contour_add(c, (unsigned)(xx2 / C.dx + 0.4999), (unsigned)(yy2 / C.dy + 0.4999), NT_WNS, nullptr, f2, Y,
                   ttf(TCT_dkdy_NULL | TCT_k_CONST | TCT_eps_mud2kdy2_WALL));
    px.contour_close(c, NT_WNS, nullptr, f2, Y, ttf(TCT_dkdx_NULL | TCT_k_CONST | TCT_eps_mud2kdx2_WALL));
    px.contour_set(c, nm);
    unsigned ix = (unsigned)(int)((Xs + DXr / 2) / C.dx + 0.4999);
    unsigned iy = (unsigned)(int)((Ys + DYr / 2) / C.dy + 0.4999);
    px.fill_area(ix, iy, NT_S | CT_NODE_IS_SET, nullptr, nullptr, TCT_No_Turbulence);
  }

  // ---- Circles ----
  const int numCircles = d.get_int_or("NumCircles", 0);
  for (int r = 0; r < numCircles; r++) {
    const std::string nm = "Circle" + std::to_string(r + 1);
    real Xs = d.get_float(nm + ".Xstart"), Ys = d.get_float(nm + ".Ystart");
    real X0 = d.get_float(nm + ".X0"), Y0 = d.get_float(nm + ".Y0");
    int MaterialID = d.get_int(nm + ".MaterialID");
    int tm = d.get_int(nm + ".TurbulenceModel");
    u64 TM = turb_model_bits(tm);
    int comp;
    GasFlow* f2 = flow2d_for(nm + ".Flow2D", comp);
    const real* Y = comp_Y(comp, px.Ymix);
    if (PreloadFlag) continue;
    const u64 ct = MaterialID ? (u64)NT_WNS : (u64)CT_NODE_IS_SET;
    PreCtx::Contour c;
    c.first_x = c.cur_x = (unsigned)(int)(Xs / C.dx + 0.4999);
    c.first_y = c.cur_y = (unsigned)(int)(Ys / C.dy + 0.4999);
    const real rr = std::sqrt((Xs - X0) * (Xs - X0) + (Ys - Y0) * (Ys - Y0) + 1.e-30);
    const real fi0 = std::atan2((Y0 - Ys), (X0 - Xs));
    f2->set_U(0.);
    f2->set_V(0.);
    const int k = std::max(1, (int)(2 * PI * rr / std::sqrt(C.dx * C.dx + C.dy * C.dy)));
    for (int i = 0; i < k; i++) {
      real xx2 = X0 + (rr * std::sin(fi0 + (2. * PI * i) / k - PI / 2.));
      real yy2 = Y0 + (rr * std::cos(fi0 + (2. * PI * i) / k - PI / 2.));
      int ix = (int)(unsigned)(xx2 / C.dx + 0.499999);
      int iy = (int)(unsigned)(yy2 / C.dy + 0.499999);
      if (ix >= 0 && iy >= 0 && ix <= C.MaxX - 1 && iy <= C.MaxY - 1)
        px.contour_add(c, (unsigned)ix, (unsigned)iy, ct, nullptr, f2, Y, TM);
    }
    px.contour_close(c, ct, nullptr, f2, Y, TM);
    px.contour_set(c, nm);
    unsigned sx = (unsigned)(X0 / C.dx), sy = (unsigned)(Y0 / C.dy);
    if (MaterialID)
      px.fill_area(sx, sy, NT_S | CT_NODE_IS_SET, nullptr, nullptr, (u64)MaterialID);
    else
      px.fill_area(sx, sy, NT_F | CT_NODE_IS_SET, f2, Y, TM);
  }

  // ---- Airfoils ----
  const int numAirfoils = d.get_int_or("NumAirfoils", 0);
  for (int r = 0; r < numAirfoils; r++) {
    const std::string nm = "Airfoil" + std::to_string(r + 1);
    real Xs = d.get_float(nm + ".Xstart"), Ys = d.get_float(nm + ".Ystart");
    int type = (int)d.get_float(nm + ".Type");
    real pp = 0, mm = 0, thick = 0;
    InputDeck ext;
    if (type == 0) {
      pp = d.get_float(nm + ".pp");
      mm = d.get_float(nm + ".mm");
      thick = d.get_float(nm + ".thick");
    } else {
      ext = InputDeck::from_file((workdir.empty() ? "" : workdir + "/") + d.get_string(nm + ".InputData"));
    }
    real scale = d.get_float(nm + ".scale");
    real attack = d.get_float(nm + ".attack_angle");
    int comp;
    GasFlow* f2 = flow2d_for(nm + ".Flow2D", comp);
    int tm = d.get_int(nm + ".TurbulenceModel");
    u64 TM = turb_model_bits(tm);
    const real* Y = comp_Y(comp, px.Ymix);
    if (PreloadFlag) continue;
    PreCtx::Contour c;
    c.first_x = c.cur_x = (unsigned)(int)(Xs / C.dx + 0.4999);
    c.first_y = c.cur_y = (unsigned)(int)(Ys / C.dy + 0.4999);
    real xx1, yy1;
    auto add = [&](real xx2, real yy2) {
      int ix = (int)(xx2 / C.dx + 0.4999), iy = (int)(yy2 / C.dy + 0.4999);
      px.contour_add(c, (unsigned)ix, (unsigned)iy, NT_WNS, nullptr, f2, Y, TM);
    };
    // Bezier NACA-like section (Boehm 1987 control polygons)
    auto b4 = [](int i, real t) {
      const real c4[5] = {1, 4, 6, 4, 1};
      return c4[i] * std::pow(1. - t, 4 - i) * std::pow(t, i);
    };
    auto b8 = [](int i, real t) {
      const real c8[9] = {1, 8, 28, 56, 70, 56, 28, 8, 1};
      return c8[i] * std::pow(1. - t, 8 - i) * std::pow(t, i);
    };
    auto mean_y = [&](real t) {
      const real m[5] = {0.0, 0.1, 0.1, 0.1, 0.0};
      real s = 0;
      for (int i = 0; i < 5; i++) s += m[i] * mm * b4(i, t);
      return s;
    };
    auto mean_x = [&](real t) {
      const real p[5] = {0.0, (real)(pp / 2.), pp, (real)((pp + 1.) / 2.), 1.0};
      real s = 0;
      for (int i = 0; i < 5; i++) s += p[i] * b4(i, t);
      return s;
    };
    auto z_x = [&](real t) {
      const real xs[9] = {0.0, 0.0, 0.03571, 0.10714, 0.21429, 0.35714, 0.53571, 0.75000, 1.00000};
      real s = 0;
      for (int i = 0; i < 9; i++) s += xs[i] * b8(i, t);
      return s;
    };
    auto z_y = [&](real t, real tk) {
      const real ys[9] = {0.0, 0.18556, 0.34863, 0.48919, 0.58214, 0.55724, 0.44992, 0.30281, 0.01050};
      real s = 0;
      for (int i = 0; i < 9; i++) s += ys[i] * tk * b8(i, t);
      return s;
    };
    if (type == 0) {
      const int k = (int)(scale / C.dx);
      const real dtp = 2. / k;
      int i;
      for (i = 0; i < k / 2; i++)
        add(Xs + scale * mean_x(z_x((i + 1) * dtp)), Ys + scale * (mean_y(z_x((i + 1) * dtp)) + z_y((i + 1) * dtp, thick)));
      for (; i > 0; i--)
        add(Xs + scale * mean_x(z_x((i - 1) * dtp)), Ys + scale * (mean_y(z_x((i - 1) * dtp)) - z_y((i - 1) * dtp, thick)));
      px.contour_close(c, NT_WNS, nullptr, f2, Y, TM);
      xx1 = Xs + scale * mean_x(z_x(0.5));
      yy1 = Ys + scale * mean_y(z_x(0.5));
    } else {
      const Table& up = ext.get_table("UpperSurface");
      const Table& lo = ext.get_table("LowerSurface");
      for (int i = 0; i < up.size(); i++) add(Xs + scale * up.X(i), Ys + scale * up.Y(i));
      for (int i = lo.size() - 1; i > 0; i--) add(Xs + scale * lo.X(i), Ys + scale * lo.Y(i));
      px.contour_close(c, NT_WNS, nullptr, f2, Y, TM);
      xx1 = Xs + scale * up.X(up.size() / 2);
      yy1 = Ys + scale * (up.Y(up.size() / 2) + lo.Y(lo.size() / 2)) / 2;
    }
    bool ok = true;
    if (attack != 0.) {
      real dcx = Xs - xx1, dcy = Ys - yy1;
      real rr = std::sqrt(dcx * dcx + dcy * dcy + 1.e-30), fi = std::atan2(dcx, dcy);
      xx1 = Xs + rr * std::sin(fi + attack);
      yy1 = Ys + rr * std::cos(fi + attack);
      ok = px.contour_rotate(c, Xs / C.dx, Ys / C.dy, attack);
    }
    if (ok) {
      px.contour_set(c, nm);
      px.fill_area((unsigned)(int)(xx1 / C.dx + 0.4999), (unsigned)(int)(yy1 / C.dy + 0.4999), NT_S | CT_NODE_IS_SET,
                   nullptr, nullptr, TCT_No_Turbulence);
    }
  }

  // ---- Areas ----
  if (!PreloadFlag) {
    for (int a = 0; a < NumArea; a++) {
      const std::string nm = "Area" + std::to_string(a + 1);
      const Table& P = d.get_table(nm);
      int type = d.get_int(nm + ".Type");
      d.get_int_or(nm + ".MaterialID", 0);
      unsigned X = (unsigned)P.X(0), Y = (unsigned)P.Y(0);
      if (type == 0) {
        px.fill_area(X, Y, CT_SOLID | CT_NODE_IS_SET, nullptr, nullptr, TCT_No_Turbulence);
      } else if (type == 1) {
        GasFlow* f1 = nullptr;
        GasFlow* f2 = nullptr;
        int comp;
        int FlowIndex = d.get_int_or(nm + ".Flow2D", -1);
        if (d.has(nm + ".Flow2D")) {
          if (FlowIndex < 1 || FlowIndex > (int)flows2d.size())
            throw DeckError("Bad Flow index [" + std::to_string(FlowIndex) + "]");
          f2 = &flows2d[FlowIndex - 1];
          comp = d.get_int("Flow2D-" + std::to_string(FlowIndex) + ".CompIndex");
        } else {
          FlowIndex = d.get_int(nm + ".Flow");
          if (FlowIndex < 1 || FlowIndex > (int)flows.size())
            throw DeckError("Bad Flow index [" + std::to_string(FlowIndex) + "]");
          f1 = &flows[FlowIndex - 1];
          comp = d.get_int("Flow" + std::to_string(FlowIndex) + ".CompIndex");
        }
        const real* Yc = comp_Y(comp, px.Ymix);
        if (!Yc) throw DeckError("Bad component index [" + std::to_string(comp) + "]");
        u64 TM = turb_model_bits(d.get_int(nm + ".TurbulenceModel"));
        if (f1) {
          GasFlow g = f1->as2d();
          px.fill_area(X, Y, CT_NO_COND | CT_NODE_IS_SET, &g, Yc, TM);
        } else {
          px.fill_area(X, Y, CT_NO_COND, f2, Yc, TM);
        }
      } else {
        throw DeckError("Bad Area type index \"" + std::to_string(type) + "\" use in \"" + nm + "\"");
      }
    }
  }

  // ---- First initialisation ----
  if (!PreloadFlag) {
    auto unset = [&](int i, int j) {
      if (!C.isIgnoreUnsetNodes && !J.is(i, j, CT_NODE_IS_SET))
        throw DeckError("Node (" + std::to_string(i) + "," + std::to_string(j) +
                        ") has not CT_NODE_IS_SET flag. Possible some \"Area\" objects not defined.");
    };
    for (int i = 0; i < C.MaxX; i++) {
      if (!J.resident(i)) {   // windowed: only the unset-node check
        for (int j = 0; j < C.MaxY; j++) unset(i, j);
        continue;
      }
      for (int j = 0; j < C.MaxY; j++) {
        CellRecord& n = J.at(i, j);
        n.idXl = n.idXr = n.idYu = n.idYd = 1;
        n.l_min = std::min(C.dx * C.MaxX, C.dy * C.MaxY);
        for (int k = 0; k < NEQ; k++) n.beta[k] = C.beta0;
        if (j == 0 || J.is(i, j - 1, CT_SOLID)) n.idYd = 0;
        if (j == C.MaxY - 1 || J.is(i, j + 1, CT_SOLID)) n.idYu = 0;
        if (i == 0 || J.is(i - 1, j, CT_SOLID)) n.idXl = 0;
        if (i == C.MaxX - 1 || J.is(i + 1, j, CT_SOLID)) n.idXr = 0;
        if (n.is(CT_WALL_NO_SLIP) || n.is(CT_WALL_LAW)) {
          n.NGX = n.idXl - n.idXr + n.idXl * n.idXr;
          n.NGY = n.idYd - n.idYu + n.idYd * n.idYu;
        }
        unset(i, j);
        if (n.is(CT_SOLID))
          n.Tg = C.Ts0;
        else
          fill_node(n, 0, 1);
        if (n.p == 0.) n.Tg = C.Ts0;
      }
    }
  }

  if (global_time > 0.) {
    if (J.resident(0)) J.at(0, 0).time = global_time;
  } else {
    const CellRecord* c00 = far_record(0, 0);
    global_time = c00 ? c00->time : 0.0;   // (a fresh non-resident record: 0)
  }

  if (C.ProblemType == SM_NS) set_wall_nodes();
  scan_area(1);

  // ---- Sources ----
  const int NumSrc = d.get_int("NumSrc");
  C.sources.clear();
  for (int i = 0; i < NumSrc; i++) {
    const std::string pre = "Src" + std::to_string(i + 1);
    GasSource s;
    s.sx = d.get_int(pre + ".GasSrcSX");
    s.sy = d.get_int(pre + ".GasSrcSY");
    s.ex = d.get_int(pre + ".GasSrcEX");
    s.ey = d.get_int(pre + ".GasSrcEY");
    s.comp = d.get_int(pre + ".GasSrcIndex");
    s.Ms = d.get_float(pre + ".Msrc");
    s.T = d.get_float(pre + ".Tsrc");
    s.Tf = d.get_float(pre + ".Tf_src");
    s.start_iter = (int)d.get_float_or(pre + ".StartIter", 0);
    s.Cp = 0;
    if (s.comp >= 0 && s.comp <= 3) {
      const int h = s.comp == 0 ? H_FU : s.comp == 1 ? H_OX : s.comp == 2 ? H_CP : H_AIR;
      s.Cp = table_eval(sp.Cp[h], s.T);
    } else if (s.comp == 4) {
      real Ym[4];
      Ym[0] = d.get_float(pre + ".Y_fuel");
      Ym[1] = d.get_float(pre + ".Y_ox");
      Ym[2] = d.get_float(pre + ".Y_cp");
      Ym[3] = 1 - Ym[0] + Ym[1] + Ym[2];
      s.Cp = Ym[0] * table_eval(sp.Cp[H_FU], s.T) + Ym[1] * table_eval(sp.Cp[H_OX], s.T) +
             Ym[2] * table_eval(sp.Cp[H_CP], s.T) + Ym[3] * table_eval(sp.Cp[H_AIR], s.T);
    }
    C.sources.push_back(s);
  }
  if (NumSrc) set_sources(0);

  if (!PreloadFlag) set_non_reflected_bc();
  if (C.ProblemType == SM_NS && !PreloadFlag) set_init_boundary_layer(C.delta_bl);

  // Serial-driver tail for N-S (hf2d_start.cpp:295-303)
  if (C.ProblemType == SM_NS) {
    collect_wall_nodes();
    set_min_distance_to_wall(0.0);
    recalc_y_plus();
    if (!PreloadFlag) set_init_boundary_layer(C.delta_bl);
  }
}

// SetWallNodes: gas cells touching a solid become no-slip walls.
void Case::set_wall_nodes() {
  for (int j = 0; j < J.ny; j++)
    for (int i = 0; i < J.nx; i++) {
      if (J.is(i, j, CT_SOLID) || J.is(i, j, NT_FC)) continue;
      bool hit = (j < J.ny - 1 && J.is(i, j + 1, CT_SOLID)) || (j > 0 && J.is(i, j - 1, CT_SOLID)) ||
                 (i > 0 && J.is(i - 1, j, CT_SOLID)) || (i < J.nx - 1 && J.is(i + 1, j, CT_SOLID));
      if (hit) J.ct(i, j) |= NT_WNS;
    }
}

// GetWallNodes: list of wall-flagged gas cells in j-major scan order.
void Case::collect_wall_nodes() {
  wall_nodes.clear();
  wall_dirs.clear();
  wall_rays.clear();
  // (a wall behind the node: a solid cell, or the lower / upper grid edge --
  // a plate on the domain boundary -- but not the inflow / outflow column,
  // which is no wall in x)
  auto solid = [&](int i, int j) { return (J.in(i, j) && J.is(i, j, CT_SOLID)) || (i >= 0 && i < J.nx && (j < 0 || j >= J.ny)); };
  auto gas = [&](int i, int j) { return J.in(i, j) && !J.is(i, j, CT_SOLID); };
  static const int di[4] = {1, -1, 0, 0}, dj[4] = {0, 0, 1, -1};
  static const uint8_t bit[4] = {WD_XP, WD_XM, WD_YP, WD_YM};
  const int nwb = std::min(std::max(cfg.WallBlendCells, 0), 255);
  for (int j = 0; j < J.ny; j++)
    for (int i = 0; i < J.nx; i++)
      if (!J.is(i, j, CT_SOLID) && (J.is(i, j, CT_WALL_LAW) || J.is(i, j, CT_WALL_NO_SLIP))) {
        wall_nodes.push_back({i, j});
        uint8_t d = 0;
        if (gas(i + 1, j) && solid(i - 1, j)) d |= WD_XP;
        if (gas(i - 1, j) && solid(i + 1, j)) d |= WD_XM;
        if (gas(i, j + 1) && solid(i, j - 1)) d |= WD_YP;
        if (gas(i, j - 1) && solid(i, j + 1)) d |= WD_YM;
        wall_dirs.push_back(d);
        for (int q = 0; q < 4; q++) {
          int n = 0;
          if (d & bit[q])
            while (n < nwb && gas(i + (n + 1) * di[q], j + (n + 1) * dj[q])) n++;
          wall_rays.push_back((uint8_t)n);
        }
      }
}

// SetMinDistanceToWall2D (deeps2d_core.cpp:4783-4832) scans every wall node
// per cell: l = sqrt(dx^2 + dy^2); m = min(m, l); if m == l take that wall;
// m = max(min(dx,dy), m), starting from m = L0 = max(X extent, Y extent).
// Order-dependent as written, but its outcome has a closed form: with
// l* = min_k l_k and theta = max(min_l, min(L0, l*)), the final l_min is
// theta and the wall taken is the LAST k (list order) with l_k <= theta
// (none if l* > L0).  [l* >= min_l: only walls at exactly l* can pass after
// the last one; l* < min_l: m sits at min_l once reached and every wall with
// l <= min_l retakes it.]  So the scan becomes a nearest-wall query plus a
// "last index within theta" query over a uniform bucket grid -- exact (same
// expressions, sqrt is monotone), O(cells * nearby walls), threaded over
// columns.  set_min_distance_to_wall_bruteforce() is the literal scan.
void Case::set_min_distance_to_wall_bruteforce(real x0) {
  const real min_l = std::min(cfg.dx, cfg.dy);
  for (int i = J.i0; i < J.i0 + J.nxl; i++)
    for (int j = 0; j < J.ny; j++) {
      CellRecord& n = J.at(i, j);
      if (!n.is(CT_NODE_IS_SET) || n.is(CT_SOLID)) continue;
      if (n.Tg != 0 && n.p == 0.) {
        n.CT |= CT_SOLID;
        continue;
      }
      n.l_min = std::max((x0 + cfg.dx * J.nx), (cfg.dy * J.ny));
      const real x = x0 + i * cfg.dx, y = j * cfg.dy;
      for (auto& w : wall_nodes) {
        const real wx = w.first * cfg.dx, wy = w.second * cfg.dy;
        const real l = std::sqrt((x - wx) * (x - wx) + (y - wy) * (y - wy));
        n.l_min = std::min(n.l_min, l);
        if (n.l_min == l) {
          n.i_wall = w.first;
          n.j_wall = w.second;
        }
        n.l_min = std::max(min_l, n.l_min);
      }
    }
}

void Case::set_min_distance_to_wall(real x0) {
  if (x0 != 0.0) {   // strip-local offsets: cells may lie outside the wall bucket grid
    set_min_distance_to_wall_bruteforce(x0);
    return;
  }
  const real dx = cfg.dx, dy = cfg.dy;
  const real min_l = std::min(dx, dy);
  const real L0 = std::max((x0 + dx * J.nx), (dy * J.ny));
  const int W = (int)wall_nodes.size();
  // buckets of BS x BS grid nodes over the wall index space
  const int BS = 16;
  const int nbx = (J.nx + BS - 1) / BS + 1, nby = (J.ny + BS - 1) / BS + 1;
  std::vector<std::vector<int>> bucket((size_t)nbx * nby);
  for (int k = 0; k < W; k++) {
    const int bx = std::min(std::max(wall_nodes[k].first / BS, 0), nbx - 1);
    const int by = std::min(std::max(wall_nodes[k].second / BS, 0), nby - 1);
    bucket[(size_t)bx * nby + by].push_back(k);   // ascending k within a bucket
  }
  const real bw = BS * dx, bh = BS * dy;   // bucket extent (m)
  auto cell = [&](int i, int j) {
    CellRecord& n = J.at(i, j);
    if (!n.is(CT_NODE_IS_SET) || n.is(CT_SOLID)) return;
    if (n.Tg != 0 && n.p == 0.) {
      n.CT |= CT_SOLID;
      return;
    }
    const real x = x0 + i * dx, y = j * dy;
    auto dist = [&](int k) {
      const real wx = wall_nodes[k].first * dx, wy = wall_nodes[k].second * dy;
      return std::sqrt((x - wx) * (x - wx) + (y - wy) * (y - wy));
    };
    const int cbx = std::min(i / BS, nbx - 1), cby = std::min(j / BS, nby - 1);
    // lower bound of the distance from (x, y) to any node of a bucket in
    // Chebyshev ring r around the cell's bucket (one ring of slack)
    auto ring_lb = [&](int r) { return r <= 2 ? 0.0 : (r - 2) * std::min(bw, bh); };
    // 1. nearest wall (ring by ring until no closer bucket can exist)
    real best = std::numeric_limits<real>::infinity();
    const int rmax = std::max(nbx, nby);
    for (int r = 0; r <= rmax; r++) {
      if (ring_lb(r) > best) break;
      for (int bx = cbx - r; bx <= cbx + r; bx++) {
        if (bx < 0 || bx >= nbx) continue;
        for (int by = cby - r; by <= cby + r; by++) {
          if (by < 0 || by >= nby) continue;
          if (std::max(std::abs(bx - cbx), std::abs(by - cby)) != r) continue;
          for (int k : bucket[(size_t)bx * nby + by]) best = std::min(best, dist(k));
        }
      }
    }
    n.l_min = std::max(min_l, std::min(L0, best));
    if (W == 0 || best > L0) return;   // the scan never takes a wall
    // 2. the last wall (list order) with l <= theta
    const real theta = n.l_min;
    int last = -1;
    const int rr = (int)std::ceil(theta / std::min(bw, bh)) + 2;
    for (int bx = std::max(cbx - rr, 0); bx <= std::min(cbx + rr, nbx - 1); bx++)
      for (int by = std::max(cby - rr, 0); by <= std::min(cby + rr, nby - 1); by++)
        for (int k : bucket[(size_t)bx * nby + by])
          if (k > last && dist(k) <= theta) last = k;
    if (last >= 0) {
      n.i_wall = wall_nodes[last].first;
      n.j_wall = wall_nodes[last].second;
    }
  };
  const int nth = std::max(1, std::min((int)std::thread::hardware_concurrency(), 16));
  std::vector<std::thread> pool;
  std::atomic<int> next{0};
  for (int t = 0; t < nth; t++)
    pool.emplace_back([&] {
      for (int i; (i = J.i0 + next.fetch_add(1)) < J.i0 + J.nxl;)
        for (int j = 0; j < J.ny; j++) cell(i, j);
    });
  for (auto& th : pool) th.join();
}

// Recalc_y_plus (serial variant): u_tau from the nearest wall node.
void Case::recalc_y_plus() {
  static const CellRecord fresh{};   // a wall record no step has touched: no shear (y+ = 0)
  for (int i = J.i0; i < J.i0 + J.nxl; i++)
    for (int j = 0; j < J.ny; j++) {
      CellRecord& n = J.at(i, j);
      if (!n.is(CT_NODE_IS_SET) || n.is(CT_SOLID)) continue;
      const int iw = n.i_wall, jw = n.j_wall;
      if (!J.in(iw, jw)) continue;
      const CellRecord* wp = far_record(iw, jw);
      const CellRecord& w = wp ? *wp : fresh;
      const real tau_w = (std::fabs(w.dUdy) + std::fabs(w.dVdx)) * w.mu;
      if (w.S[I_RHO] > 0.0 && tau_w > 0.0) {
        const real U_w = std::sqrt(tau_w / w.S[I_RHO] + 1e-30);
        n.y_plus = std::fabs(U_w * std::min(cfg.dx, cfg.dy) * n.S[I_RHO] / n.mu);
      } else {
        n.y_plus = 0.0;
      }
    }
}

// SetInitBoundaryLayer (the reference's missing-brace quirk Q6 is kept:
// rhoV is scaled for every fresh cell, rhoU only inside delta).
void Case::set_init_boundary_layer(real delta) {
  for (int i = J.i0; i < J.i0 + J.nxl; i++)
    for (int j = 0; j < J.ny; j++) {
      CellRecord& n = J.at(i, j);
      if (n.is(CT_NODE_IS_SET) && !n.is(CT_SOLID) && n.time == 0. && delta > 0) {
        if (n.l_min <= delta) n.S[I_RHOU] = n.S[I_RHOU] * n.l_min / delta;
        n.S[I_RHOV] = n.S[I_RHOV] * n.l_min / delta;
        fill_node(n, 0, 1);
      }
    }
}

int Case::set_non_reflected_bc() {
  int nr = 0;
  auto ok = [&](int i, int j) {
    return J.is(i, j, CT_NODE_IS_SET) && !J.is(i, j, CT_WALL_NO_SLIP) && !J.is(i, j, CT_SOLID) && !J.is(i, j, NT_FC);
  };
  for (int ii = 0; ii < J.nx; ii++)
    for (int jj = 0; jj < J.ny; jj++) {
      if (!J.is(ii, jj, NT_FARFIELD)) continue;
      nr++;
      if (ii > 0 && ok(ii - 1, jj)) { J.ct(ii - 1, jj) |= CT_NONREFLECTED; nr++; }
      if (ii < J.nx - 1 && ok(ii + 1, jj)) { J.ct(ii + 1, jj) |= CT_NONREFLECTED; nr++; }
      if (jj > 0 && ok(ii, jj - 1)) { J.ct(ii, jj - 1) |= CT_NONREFLECTED; nr++; }
      if (jj < J.ny - 1 && ok(ii, jj + 1)) { J.ct(ii, jj + 1) |= CT_NONREFLECTED; nr++; }
    }
  return nr;
}

// scan_area's turbulence reset of one record (tt: its new TurbType word)
void Case::turb_reset_record(CellRecord& n, u64 tt) const {
  n.TurbType = tt;
  n.dkdx = n.dkdy = n.depsdx = n.depsdy = 0.0;
  n.S[I_K] = n.S[I_EPS] = n.Src[I_K] = n.Src[I_EPS] = 0.0;
  n.mu_t = n.lam_t = 0.0;
  fill_node(n, 0, 1);
}

// ScanArea: mark active cells, optional turbulence-model reset and the
// active-cell-balanced column partition.
void Case::scan_area(int num_parts) {
  for (int j = 0; j < J.ny; j++)
    for (int i = 0; i < J.nx; i++)
      if (!J.is(i, j, CT_SOLID)) J.ct(i, j) |= CT_NODE_IS_SET;
  if (cfg.isTurbulenceReset && cfg.ProblemType == SM_NS) {
    const u64 TM = turb_model_bits(cfg.TurbMod);
    for (int i = 0; i < J.nx; i++)
      for (int j = 0; j < J.ny; j++) {
        u64& tt = J.tt(i, j);
        const u64 models[] = {TCT_Integral_Model, TCT_Prandtl_Model, TCT_Spalart_Allmaras_Model, TCT_k_eps_Model,
                              TCT_Smagorinsky_Model, TCT_k_omega_SST_Model};
        for (u64 m : models)
          if ((tt & m) == m) tt = (tt ^ m) & tt;
        tt |= TM;
        if (!J.resident(i)) continue;
        turb_reset_record(J.at(i, j), tt);
      }
    cfg.isTurbulenceReset = 0;
    far_turb_reset = true;
  }
  subdomains = partition_columns(num_parts);
}

std::vector<std::pair<int, int>> Case::partition_columns(int num_parts) const {
  long active = 0;
  for (int i = 0; i < J.nx; i++)
    for (int j = 0; j < J.ny; j++)
      if (J.is(i, j, CT_NODE_IS_SET) && !J.is(i, j, CT_SOLID)) active++;
  std::vector<std::pair<int, int>> parts;
  const long per = std::max<long>(1, active / std::max(1, num_parts));
  long cnt = 0;
  int start = 0;
  for (int i = 0; i < J.nx; i++) {
    for (int j = 0; j < J.ny; j++) {
      if (J.is(i, j, CT_NODE_IS_SET) && !J.is(i, j, CT_SOLID)) {
        cnt++;
        if (cnt >= per) {
          parts.push_back({start, i + 1});
          start = i;
          cnt = 0;
        }
      }
    }
  }
  return parts;
}

// Source2D::SetSource2D for every source (hyper_flow_source.cpp:36-170).
void Case::set_sources(int iter) {
  const real dx = cfg.dx, dy = cfg.dy;
  for (auto& s : cfg.sources) {
    if (iter < s.start_iter) continue;
    const int DX = s.sx - s.ex, DY = s.sy - s.ey;
    CellRecord scratch;   // a source cell of another strip: its writes go nowhere
    auto at = [&](unsigned x, unsigned y) -> CellRecord& {
      if (!J.in(x, y)) throw DeckError("gas source outside the computation area");
      return J.resident(x) ? J.at((int)x, (int)y) : scratch;
    };
    if (DX == 0 && DY == 0) {
      CellRecord& n = at(s.sx, s.sy);
      if (cfg.FT == FT_AXISYMMETRIC) {
        if (s.sy == 0 || s.ey == 0)
          n.Src[I_RHO] = s.Ms / (M_PI * dx * dy * dy);
        else
          n.Src[I_RHO] = s.Ms / (2 * M_PI * dx * dy * n.y);
      } else {
        n.Src[I_RHO] = s.Ms / (dx * dy);
      }
      n.SrcAdd[I_RHO] = 0.;
      n.Src[I_RHOU] = 0;
      n.Tf = s.Tf;
      if (s.comp < 4) n.Src[s.comp + 4] = n.Src[I_RHO];
      n.Src[I_RHOE] = s.Cp * s.T * n.Src[I_RHO];
      continue;
    }
    auto apply = [&](CellRecord& n, bool axi_line) {
      if (cfg.FT == FT_AXISYMMETRIC) {
        if (s.sy == 0 || s.ey == 0) {
          real DR = DY * dy;
          n.Src[I_RHO] = s.Ms / (M_PI * (dx * DR * DR));
        } else {
          real DR2 = M_PI * std::fabs((real)s.sy * s.sy * dy * dy - (real)s.ey * s.ey * dy * dy);
          n.Src[I_RHO] = s.Ms / (dx * DR2);
        }
      } else if (axi_line) {
        n.Src[I_RHO] = s.Ms / (dx * dy);
      }
      n.SrcAdd[I_RHO] = 0.;
      n.Tf = s.Tf;
      n.Src[I_RHOU] = 0;
      n.Src[I_RHOV] = 0;
      if (s.comp + 4 < NEQ) n.Src[s.comp + 4] = n.Src[I_RHO];
      n.Src[I_RHOE] = s.Cp * s.T * n.Src[I_RHO];
    };
    if (std::abs(DX) > std::abs(DY)) {
      const int SKX = DX > 0 ? 1 : -1, SKY = DY > 0 ? 1 : -1;
      const real dF = std::fabs((real)DY) / std::fabs((real)DX);
      for (int i = 0; i != DX + SKX; i += SKX) apply(at((unsigned)(s.sx + i * SKX), (unsigned)(s.sy + i * dF * SKY)), true);
    } else {
      const int SKY = DY > 0 ? 1 : -1, SKX = DX > 0 ? 1 : -1;
      const real dF = std::fabs((real)DX) / std::fabs((real)DY);
      for (int i = 0; i != DY + SKY; i += SKY) apply(at((unsigned)(s.sx + i * dF * SKX), (unsigned)(s.sy + i * SKY)), false);
    }
  }
}

std::vector<std::pair<int, int>> balanced_columns(const Field& J, int nparts) {
  const int nx = J.nx;
  if (nparts <= 1) return {{0, nx}};
  if (nparts > nx) throw std::runtime_error("more strips than columns");
  std::vector<double> cum(nx + 1, 0.0);
  for (int i = 0; i < nx; i++) {
    double a = 0;
    for (int j = 0; j < J.ny; j++) a += J.is(i, j, CT_SOLID) ? 0.0 : 1.0;
    cum[i + 1] = cum[i] + a;
  }
  const double total = cum[nx];
  std::vector<int> cuts{0};
  for (int k = 1; k < nparts; k++) {
    const double target = total * k / nparts;
    int c = (int)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
    c = std::max(c, cuts.back() + 1);
    c = std::min(c, nx - (nparts - k));
    cuts.push_back(c);
  }
  cuts.push_back(nx);
  std::vector<std::pair<int, int>> out;
  for (int k = 0; k < nparts; k++) out.push_back({cuts[k], cuts[k + 1]});
  return out;
}

int Config::num_active_eq() const { return NEQ; }

}  // namespace hf2d
