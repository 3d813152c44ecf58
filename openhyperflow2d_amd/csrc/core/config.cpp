// Config::load_globals — the deck keys read before pre-processing
// (reference InitSharedData, libDEEPS2D/deeps2d_core.cpp:160-499).
#include <cstdio>

#include "case.hpp"

namespace hf2d {

void Config::load_globals(InputDeck& d) {
  isVerboseOutput = d.get_int("isVerboseOutput");
  bff = d.get_int("BFF");
  MaxX = d.get_int("MaxX");
  MaxY = d.get_int("MaxY");
  dx = d.get_float("dx");
  dy = d.get_float("dy");
  SigW = d.get_float("SigW");
  SigF = d.get_float("SigF");
  delta_bl = d.get_float("delta_bl");
  TurbMod = d.get_int("TurbulenceModel");
  TurbStartIter = d.get_int("TurbStartIter");
  TurbExtModel = d.get_int("TurbExtModel");
  isTurbulenceReset = d.get_int("isTurbulenceReset");
  FT = d.get_int("FlowType");
  ProblemType = d.get_int("ProblemType");
  CFL = d.get_float("CFL");
  CFL_Scenario = d.get_table("CFL_Scenario");
  ViscousCFL = d.get_float_or("ViscousCFL", 0.0);
  SSTWallDistance = d.get_float_or("SSTWallDistance", 1.0);
  LaggedDt = d.get_int_or("LaggedDt", 0) ? 1 : 0;
  WallBlendCells = std::max(0, d.get_int_or("WallBlendCells", 0));
  WallBlendFactor = std::min(1.0, std::max(0.0, (double)d.get_float_or("WallBlendFactor", 0.0)));
  ThreadBlockSize = d.get_int_or("ThreadBlockSize", 0);
  NSaveStep = d.get_int("NSaveStep");
  Nmax = d.get_int("Nmax");
  NOutStep = d.get_int_or("NOutStep", 1);
  if (NOutStep <= 0) NOutStep = 1;
  if (NOutStep >= Nmax) Nmax = NOutStep + 1;
  isAlternateRMS = d.get_int("isAlternateRMS");
  isIgnoreUnsetNodes = d.get_int("isIgnoreUnsetNodes");
  MonitorIndex = d.get_int("MonitorIndex");
  if (MonitorIndex > 5 || MonitorIndex < 0) MonitorIndex = 0;
  ExitMonitorValue = d.get_float("ExitMonitorValue");
  int nmp = d.get_int("NumMonitorPoints");
  monitors.clear();
  for (int i = 0; i < nmp; i++) {
    char k[64];
    MonitorPoint mp;
    std::snprintf(k, sizeof k, "Point-%i.X", i + 1);
    mp.x = d.get_float(k);
    std::snprintf(k, sizeof k, "Point-%i.Y", i + 1);
    mp.y = d.get_float(k);
    if (mp.x < 0.0 || mp.y < 0.0 || mp.x > MaxX * dx || mp.y > MaxY * dy) continue;  // ignored
    monitors.push_back(mp);
  }
  beta0 = d.get_float("beta");
  nrbc_beta0 = d.get_float("beta_NonReflectedBC");
  beta_Scenario = d.get_table("beta_Scenario");
  species.K0 = d.get_float("K0");
  species.gamma = d.get_float("gamma");
  species.Tf = d.get_float("Tf");
  isAdiabaticWall = d.get_int("isAdiabaticWall");
  // new key (not in the reference, which always runs the Zeldovich model):
  // 0 frozen mixture, 1 Zeldovich (default), 2 finite-rate H2/air
  chem_model = d.get_int_or("ChemicalReactionsModel", CRM_ZELDOVICH);
  mechanism = d.get_string_or("Mechanism", "");
  chem_nsub = d.get_int_or("ChemSubsteps", 1);
  if (chem_nsub < 1) chem_nsub = 1;
  chem_tmin = d.get_float_or("ChemTmin", 300.0);
  species.arr_A = d.get_float_or("Arrhenius.A", species.arr_A);
  species.arr_Ta = d.get_float_or("Arrhenius.Ta", species.arr_Ta);
  species.arr_a = d.get_float_or("Arrhenius.FuelOrder", species.arr_a);
  species.arr_b = d.get_float_or("Arrhenius.OxOrder", species.arr_b);
  // combustion products, fuel, oxidizer, air
  species.R[H_CP] = d.get_float("R_cp");
  species.H[H_CP] = d.get_float("H_cp");
  species.lam[H_CP] = d.get_table("lam_cp").pack();
  species.mu[H_CP] = d.get_table("mu_cp").pack();
  species.Cp[H_CP] = d.get_table("Cp_cp").pack();
  species.R[H_FU] = d.get_float("R_Fuel");
  species.H[H_FU] = d.get_float("H_Fuel");
  species.lam[H_FU] = d.get_table("lam_Fuel").pack();
  species.mu[H_FU] = d.get_table("mu_Fuel").pack();
  species.Cp[H_FU] = d.get_table("Cp_Fuel").pack();
  species.R[H_OX] = d.get_float("R_OX");
  species.H[H_OX] = d.get_float("H_OX");
  species.lam[H_OX] = d.get_table("lam_OX").pack();
  species.mu[H_OX] = d.get_table("mu_OX").pack();
  species.Cp[H_OX] = d.get_table("Cp_OX").pack();
  species.R[H_AIR] = d.get_float("R_air");
  species.H[H_AIR] = d.get_float("H_air");
  species.lam[H_AIR] = d.get_table("lam_air").pack();
  species.mu[H_AIR] = d.get_table("mu_air").pack();
  species.Cp[H_AIR] = d.get_table("Cp_air").pack();
  for (int q = 0; q < NSPEC; q++) species.M[q] = species.R[q] > 0 ? 8.314462618 / species.R[q] : 0.0;
  Hu[H_FU] = species.H[H_FU];
  Hu[H_OX] = species.H[H_OX];
  Hu[H_CP] = species.H[H_CP];
  Hu[H_AIR] = species.H[H_AIR];
}

FillParams Config::fill_params() const {
  FillParams P;
  P.FT = FT;
  P.dx = dx;
  P.dy = dy;
  for (int i = 0; i < NSPEC; i++) P.Hu[i] = Hu[i];
  P.sst_d1 = SSTWallDistance;
  return P;
}

}  // namespace hf2d
