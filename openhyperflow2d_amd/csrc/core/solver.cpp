#include "solver.hpp"

#include <algorithm>
#include <limits>
#include <chrono>
#include <csignal>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <ostream>
#include <stdexcept>
#include <unordered_map>

#include "checkpoint.hpp"
#include "postproc.hpp"
#include "stripio.hpp"

namespace hf2d {

static const char* RMS_NAME[11] = {"Rho",     "Rho*U",   "Rho*V", "Rho*E",     "Rho*Yfu", "Rho*Yox",
                                   "Rho*Ycp", "Rho*k",   "Rho*eps", "Rho*omega", "nu_t"};

// ---------------------------------------------------------------------------
// HostArrays
// ---------------------------------------------------------------------------
void HostArrays::allocate(int X, int Yn) {
  nx = X;
  ny = Yn;
  N = (long)X * Yn;
  auto E = [&](std::vector<real>& v, int m) { v.assign((size_t)m * N, 0.0); };
  for (int b = 0; b < 2; b++) {
    E(S[b], NEQ);
    E(dSdx[b], NEQ);
    E(dSdy[b], NEQ);
    E(U[b], 1);
    E(V[b], 1);
    E(Tg[b], 1);
  }
  E(A, NEQ); E(B, NEQ); E(F, NEQ); E(Src, NEQ); E(SrcAdd, NEQ); E(beta, NEQ);
  E(p, 1); E(kk, 1); E(R, 1); E(CP, 1); E(lam, 1); E(mu, 1); E(mu_t, 1); E(lam_t, 1); E(Diff, 1);
  E(Y, NSPEC);
  E(l_min, 1); E(y_plus, 1); E(Re_local, 1); E(BGX, 1); E(BGY, 1); E(Tf, 1); E(Q_conv, 1);
  E(grad, NGRAD); E(qdir, 4); E(time, 1);
  CT.assign(N, 0);
  TT.assign(N, 0);
  nb.assign(N, 0);
  wslot.assign(N, -1);
}

void HostArrays::from_field(const Field& J, int gi0) {
  for (int li = 0; li < nx; li++) {
    // (a second ghost column outside the resident ones -- device N-S strips --
    // starts as a copy of the nearest; the first lean exchange refreshes it)
    const int gi = std::min(std::max(gi0 + li, J.i0), J.i0 + J.nxl - 1);
    for (int j = 0; j < ny; j++) {
      const long idx = (long)li * ny + j;
      const CellRecord& c = J.at(gi, j);
      for (int k = 0; k < NEQ; k++) {
        const long o = k * N + idx;
        S[0][o] = S[1][o] = c.S[k];
        dSdx[0][o] = dSdx[1][o] = c.dSdx[k];
        dSdy[0][o] = dSdy[1][o] = c.dSdy[k];
        A[o] = c.A[k];
        B[o] = c.B[k];
        F[o] = c.F[k];
        Src[o] = c.Src[k];
        SrcAdd[o] = c.SrcAdd[k];
        beta[o] = c.beta[k];
      }
      U[0][idx] = U[1][idx] = c.U;
      V[0][idx] = V[1][idx] = c.V;
      Tg[0][idx] = Tg[1][idx] = c.Tg;
      p[idx] = c.p;
      kk[idx] = c.k;
      R[idx] = c.R;
      CP[idx] = c.CP;
      lam[idx] = c.lam;
      mu[idx] = c.mu;
      mu_t[idx] = c.mu_t;
      lam_t[idx] = c.lam_t;
      Diff[idx] = c.Diff;
      for (int s = 0; s < NSPEC; s++) Y[s * N + idx] = c.Y[s];
      l_min[idx] = c.l_min;
      y_plus[idx] = c.y_plus;
      Re_local[idx] = c.Re_local;
      BGX[idx] = c.BGX;
      BGY[idx] = c.BGY;
      Tf[idx] = c.Tf;
      Q_conv[idx] = c.Q_conv;
      time[idx] = c.time;
      const real g[NGRAD] = {c.dUdx, c.dUdy, c.dVdx, c.dVdy, c.dTdx, c.dTdy, c.dkdx, c.dkdy, c.depsdx, c.depsdy};
      for (int q = 0; q < NGRAD; q++) grad[q * N + idx] = g[q];
      CT[idx] = c.CT;
      TT[idx] = c.TurbType;
      nb[idx] = (c.idXl ? NB_XL : 0) | (c.idXr ? NB_XR : 0) | (c.idYu ? NB_YU : 0) | (c.idYd ? NB_YD : 0);
    }
  }
}

void HostArrays::wall_slots(const Case& cs, int gx0, int gi0, int gi1) {
  std::unordered_map<long, int32_t> slot;
  slot.reserve(cs.wall_nodes.size() * 2 + 1);
  const long NY = cs.J.ny;
  for (size_t k = 0; k < cs.wall_nodes.size(); k++)
    slot[(long)cs.wall_nodes[k].first * NY + cs.wall_nodes[k].second] = (int32_t)k;
  wslot.assign(N, -1);
  for (int li = 0; li < nx; li++) {
    const int gi = gx0 + li;
    if (!cs.J.resident(gi)) continue;
    for (int j = 0; j < ny; j++) {
      const CellRecord& c = cs.J.at(gi, j);
      const auto it = slot.find((long)c.i_wall * NY + c.j_wall);
      if (it != slot.end()) wslot[(long)li * ny + j] = it->second;
    }
  }
  wall_own.clear();
  wall_own_slot.clear();
  for (size_t k = 0; k < cs.wall_nodes.size(); k++) {
    const int gi = cs.wall_nodes[k].first;
    if (gi < gi0 || gi >= gi1) continue;
    wall_own.push_back((long)(gi - gx0) * ny + cs.wall_nodes[k].second);
    wall_own_slot.push_back((int32_t)k);
  }
}

void HostArrays::to_field(Field& J, int gi0, int i_from, int i_to, int pb, int db) const {
  for (int li = i_from; li < i_to; li++) {
    const int gi = gi0 + li;
    for (int j = 0; j < ny; j++) {
      const long idx = (long)li * ny + j;
      CellRecord& c = J.at(gi, j);
      for (int k = 0; k < NEQ; k++) {
        const long o = k * N + idx;
        c.S[k] = S[0][o];
        c.dSdx[k] = dSdx[db][o];
        c.dSdy[k] = dSdy[db][o];
        c.A[k] = A[o];
        c.B[k] = B[o];
        c.F[k] = F[o];
        c.Src[k] = Src[o];
        c.SrcAdd[k] = SrcAdd[o];
        c.beta[k] = beta[o];
      }
      c.U = U[pb][idx];
      c.V = V[pb][idx];
      c.Tg = Tg[pb][idx];
      c.p = p[idx];
      c.k = kk[idx];
      c.R = R[idx];
      c.CP = CP[idx];
      c.lam = lam[idx];
      c.mu = mu[idx];
      c.mu_t = mu_t[idx];
      c.lam_t = lam_t[idx];
      c.Diff = Diff[idx];
      for (int s = 0; s < NSPEC; s++) c.Y[s] = Y[s * N + idx];
      c.l_min = l_min[idx];
      c.y_plus = y_plus[idx];
      c.Re_local = Re_local[idx];
      c.Q_conv = Q_conv[idx];
      c.time = time[idx];
      c.dUdx = grad[G_DUDX * N + idx];
      c.dUdy = grad[G_DUDY * N + idx];
      c.dVdx = grad[G_DVDX * N + idx];
      c.dVdy = grad[G_DVDY * N + idx];
      c.dTdx = grad[G_DTDX * N + idx];
      c.dTdy = grad[G_DTDY * N + idx];
      c.dkdx = grad[G_DKDX * N + idx];
      c.dkdy = grad[G_DKDY * N + idx];
      c.depsdx = grad[G_DEDX * N + idx];
      c.depsdy = grad[G_DEDY * N + idx];
      c.CT = CT[idx];
      c.TurbType = TT[idx];
    }
  }
}

void HostArrays::allocate_mech(const Case& cs) {
  mech = cs.cfg.mech_mode() ? &cs.cfg.mech->data : nullptr;
  nsp = mech ? mech->ns : 0;
  if (!mech) return;
  const size_t n = (size_t)nsp * N;
  for (int b = 0; b < 2; b++) Ys[b].assign(n, 0.0);
  As.assign(n, 0.0);
  Bs.assign(n, 0.0);
  Fs.assign(n, 0.0);
  betas.assign(n, 0.0);
  const bool cauchy = mech_species_cauchy(cs);
  for (int b = 0; b < 2; b++) {
    dSdxs[b].assign(cauchy ? n : 0, 0.0);
    dSdys[b].assign(cauchy ? n : 0, 0.0);
  }
}

void HostArrays::mech_from_case(const Case& cs, int gi0) {
  if (!mech) return;
  const real FT = (real)cs.cfg.FT;
  for (int li = 0; li < nx; li++) {
    const int gi = std::min(std::max(gi0 + li, cs.J.i0), cs.J.i0 + cs.J.nxl - 1);   // (see from_field)
    for (int j = 0; j < ny; j++) {
      const long idx = (long)li * ny + j;
      const CellRecord& c = cs.J.at(gi, j);
      for (int sp = 0; sp < nsp; sp++) {
        const long o = (long)sp * N + idx;
        const real r = cs.mech_rhoY[cs.mech_idx(sp, gi, j)];
        Ys[0][o] = Ys[1][o] = r;
        // inviscid start fluxes (the pre-processor's FillNode2D has no
        // species gradients either); the first fill rewrites them
        As[o] = r * c.U;
        Bs[o] = r * c.V;
        Fs[o] = FT * r * c.V;
        betas[o] = c.beta[I_YFU];
        if (!dSdxs[0].empty()) dSdxs[0][o] = dSdxs[1][o] = dSdys[0][o] = dSdys[1][o] = 0.0;
      }
    }
  }
}

void HostArrays::mech_to_case(Case& cs, int gi0, int i_from, int i_to, int ybuf) const {
  if (!mech) return;
  for (int li = i_from; li < i_to; li++)
    for (int j = 0; j < ny; j++)
      for (int sp = 0; sp < nsp; sp++)
        cs.mech_rhoY[cs.mech_idx(sp, gi0 + li, j)] = Ys[ybuf][(long)sp * N + (long)li * ny + j];
}

void HostArrays::mech_view(SoA& s, int yb, int db) const {
  s.mech = mech;
  s.nsp = nsp;
  if (!mech) return;
  auto P = [](const std::vector<real>& v) { return v.empty() ? nullptr : const_cast<real*>(v.data()); };
  s.Ys = P(Ys[yb]);
  s.As = P(As);
  s.Bs = P(Bs);
  s.Fs = P(Fs);
  s.betas = P(betas);
  s.dSdxs = P(dSdxs[db]);
  s.dSdys = P(dSdys[db]);
}

SoA HostArrays::view(int sb, int db, int pb) {
  SoA s;
  s.nx = nx;
  s.ny = ny;
  s.N = N;
  s.S = S[sb].data();
  s.A = A.data();
  s.B = B.data();
  s.F = F.data();
  s.Src = Src.data();
  s.SrcAdd = SrcAdd.data();
  s.beta = beta.data();
  s.dSdx = dSdx[db].data();
  s.dSdy = dSdy[db].data();
  s.U = U[pb].data();
  s.V = V[pb].data();
  s.Tg = Tg[pb].data();
  s.p = p.data();
  s.kk = kk.data();
  s.R = R.data();
  s.CP = CP.data();
  s.lam = lam.data();
  s.mu = mu.data();
  s.mu_t = mu_t.data();
  s.lam_t = lam_t.data();
  s.Diff = Diff.data();
  s.Y = Y.data();
  s.l_min = l_min.data();
  s.y_plus = y_plus.data();
  s.Re_local = Re_local.data();
  s.BGX = BGX.data();
  s.BGY = BGY.data();
  s.Tf = Tf.data();
  s.Q_conv = Q_conv.data();
  s.grad = grad.data();
  s.CT = CT.data();
  s.TT = TT.data();
  s.nb = nb.data();
  s.gf = gf.empty() ? nullptr : gf.data();
  s.wslot = const_cast<int32_t*>(wslot.data());
  mech_view(s, sb, db);
  return s;
}

// ---------------------------------------------------------------------------
// SolverBase: the time-march driver
// ---------------------------------------------------------------------------
SolverBase::SolverBase(Case& c) : cs(c) {
  comm = &local_comm;
  dt = c.dt0;
  dt_running = c.dt0;
  last_iter = c.restart_iter;
}

StepParams SolverBase::make_params(long it) const {
  const Config& C = cs.cfg;
  StepParams P{};
  P.dx = C.dx;
  P.dy = C.dy;
  P.dt = dt;
  P.dtdx = dt / C.dx;
  P.dtdy = dt / C.dy;
  P.dyy = C.dx / (C.dx + C.dy);
  P.dxx = C.dy / (C.dx + C.dy);
  const real beta_scen = C.beta_Scenario.eval((real)it);
  const real cfl_scen = C.CFL_Scenario.eval((real)it);
  P.beta_min = std::min<real>(C.beta0, beta_scen);
  P.nrbc_beta0 = C.nrbc_beta0;
  P.CFL_min = std::min<real>(C.CFL, cfl_scen);
  P.visc_cfl = C.ViscousCFL;
  P.bff = C.bff;
  P.alternate_rms = C.isAlternateRMS;
  P.sm = C.ProblemType;
  P.lag_dt = (C.LaggedDt && C.semantics == Semantics::MPI) ? 1 : 0;
  P.wall_blend = C.WallBlendCells > 0 ? 1 : 0;
  P.wall_blend_f = C.WallBlendFactor;
  P.chem_model = C.chem_model;
  P.species = &C.species;
  FillParams f = C.fill_params();
  f.sig_w = C.SigW;
  f.sig_f = C.SigF;
  f.tem = C.TurbExtModel;
  f.delta = C.delta_bl;
  f.sm = C.ProblemType;
  f.isSrcAdd = isSrcAdd ? 1 : 0;
  P.ffc = f;
  P.ffc.is_mu_t = 1;
  P.ffc.is_init = 0;
  P.fpa = f;
  if ((int)it < C.TurbStartIter) {
    P.fpa.is_mu_t = 0;
    P.fpa.is_init = C.isTurbulenceReset;
  } else {
    P.fpa.is_mu_t = 1;
    P.fpa.is_init = 0;
  }
  return P;
}

StepResult SolverBase::advance(bool want_res) {
  const long it = last_iter + iter;
  StepParams P = make_params(it);
  StepResult r = do_step(P, want_res);
  if (r.async) {
    if (r.have_residual) {
      comm->allreduce_residual(r.res);
      last_res = residual_finalize(r.res, cs.cfg.isAlternateRMS, cs.cfg.MonitorIndex,
                                   cs.cfg.semantics == Semantics::SERIAL, cs.cfg.ExitMonitorValue);
      last_res_valid = true;
    }
    iter++;
    if (want_res) sync_scalars();
    return r;
  }
  if (comm->allreduce_max_int(r.neg_T)) {
    char b[256];
    std::snprintf(b, sizeof b, "ERROR: Computational unstability (Tg < 0) on iteration %ld, dt=%g", it, P.dt);
    throw std::runtime_error(b);
  }
  const real dtm = comm->allreduce_min(r.dt_min);
  if (cs.cfg.semantics == Semantics::SERIAL) {
    dt_running = std::min(dt_running, dtm);
    dt = dt_running;
  } else if (P.lag_dt) {   // step n + 1 takes the MIN of step n - 1; this one's waits a step
    if (!(dt_lag > 0)) dt_lag = P.dt;
    dt = dt_lag;
    dt_lag = dtm;
  } else {
    dt = dtm;
  }
  if (r.have_residual) {
    comm->allreduce_residual(r.res);
    last_res = residual_finalize(r.res, cs.cfg.isAlternateRMS, cs.cfg.MonitorIndex,
                                 cs.cfg.semantics == Semantics::SERIAL, cs.cfg.ExitMonitorValue);
    last_res_valid = true;
  }
  cur_time_part += P.dt;
  iter++;
  return r;
}

void SolverBase::run_steps(long n, bool want_res_last) {
  for (long s = 0; s < n; s++) {
    if (iter >= cs.cfg.Nmax) {   // roll the inner counter like an outer cycle
      sync_scalars();
      last_iter += iter;
      iter = 0;
      cs.global_time += cur_time_part;
      cur_time_part = 0;
      on_cycle_roll();
      isSrcAdd = true;
      cycle++;
    }
    step_outputs = s == n - 1;   // the host may read the full record afterwards
    advance(want_res_last && s == n - 1);
  }
  step_outputs = true;
  sync_scalars();
}

void SolverBase::merge_wall_uw(const std::vector<int32_t>& slots, const std::vector<real>& vals,
                               std::vector<real>& uw, std::vector<uint8_t>& ok) {
  uw.assign(cs.wall_nodes.size(), 0.);
  ok.assign(cs.wall_nodes.size(), 0);
  auto take = [&](const int32_t* sl, const real* v, size_t n) {
    for (size_t k = 0; k < n; k++) {
      uw[(size_t)sl[k]] = v[k];
      ok[(size_t)sl[k]] = 1;
    }
  };
  if (comm->size() == 1) {
    take(slots.data(), vals.data(), slots.size());
    return;
  }
  std::string m((const char*)slots.data(), slots.size() * sizeof(int32_t));
  m.append((const char*)vals.data(), vals.size() * sizeof(real));
  for (const std::string& b : comm->allgather_bytes(m)) {
    const size_t n = b.size() / (sizeof(int32_t) + sizeof(real));
    std::vector<int32_t> sl(n);
    std::vector<real> v(n);
    if (n == 0) continue;
    std::memcpy(sl.data(), b.data(), n * sizeof(int32_t));
    std::memcpy(v.data(), b.data() + n * sizeof(int32_t), n * sizeof(real));
    take(sl.data(), v.data(), n);
  }
}

void SolverBase::sample_monitors(std::vector<MonitorPoint>& mp) {
  if (mp.empty()) return;
  Field& J = cs.J;
  download(J);
  const auto own = owned_columns();
  for (auto& m : mp) {
    const int i = (int)(m.x / cs.cfg.dx), j = (int)(m.y / cs.cfg.dy);
    real p = 0, T = 0;
    const bool mine = J.in(i, j) && i >= own.first && i < own.second;
    if (mine) {
      p = J.at(i, j).p;
      T = J.at(i, j).Tg;
    }
    if (comm->size() > 1) {   // exactly one rank owns the probe
      p = comm->allreduce_sum(p);
      T = comm->allreduce_sum(T);
    } else if (!J.in(i, j)) {
      continue;
    }
    m.p = p;
    m.T = T;
  }
}

namespace {
volatile std::sig_atomic_t g_stop = 0;
extern "C" void hf2d_on_signal(int) { g_stop = 1; }
}  // namespace

void request_stop() { g_stop = 1; }
bool stop_requested() { return g_stop != 0; }
void clear_stop() { g_stop = 0; }
void install_signal_handlers() {
  struct sigaction sa;
  std::memset(&sa, 0, sizeof sa);
  sa.sa_handler = hf2d_on_signal;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGINT, &sa, nullptr);
  sigaction(SIGTERM, &sa, nullptr);
}

namespace {
using pclk = std::chrono::steady_clock;

// Wall-clock + profiler range around one driver phase.
struct PhaseScope {
  SolverBase& s;
  const char* name;
  pclk::time_point t0;
  PhaseScope(SolverBase& s_, const char* n) : s(s_), name(n), t0(pclk::now()) { s.trace_push(n); }
  ~PhaseScope() {
    s.trace_pop();
    auto& a = s.phase_acc[name];
    a.first += std::chrono::duration<double>(pclk::now() - t0).count();
    a.second++;
  }
};

std::string plt_stem(const std::string& f) {
  const size_t dot = f.rfind('.');
  return dot == std::string::npos ? f : f.substr(0, dot);
}
}  // namespace

void SolverBase::write_profile(const std::string& path, int cycles) const {
  std::FILE* f = std::fopen(path.c_str(), "w");
  if (!f) return;
  double total = 0;   // top-level phases (nested ones are named "<parent>.<child>")
  for (const auto& kv : phase_acc)
    if (kv.first.find('.') == std::string::npos) total += kv.second.first;
  const double iters = (double)(last_iter + iter);
  std::fprintf(f, "{\"rank\": %d, \"ranks\": %d, \"grid\": [%d, %d], \"cycles\": %d, \"iterations\": %.0f, "
               "\"seconds\": %.6f, \"mcells_it_per_s\": %.6g, \"phases\": {",
               comm->rank(), comm->size(), cs.cfg.MaxX, cs.cfg.MaxY, cycles, iters, total,
               total > 0 ? iters * cs.cfg.MaxX * cs.cfg.MaxY / total / 1e6 : 0.0);
  bool first = true;
  for (const auto& kv : phase_acc) {
    std::fprintf(f, "%s\"%s\": {\"seconds\": %.6f, \"calls\": %ld}", first ? "" : ", ", kv.first.c_str(),
                 kv.second.first, kv.second.second);
    first = false;
  }
  std::fprintf(f, "}}\n");
  std::fclose(f);
}

// Numerical failure (Tg < 0) or transport failure: write the error snapshot
// <Project>-err.plt (multi-rank: rank-<r>-<Project>-err.plt with that rank's
// strip, as the reference names them per rank), keep the last good
// checkpoint of the previous cycle for a restart, and report where.
void SolverBase::failure_snapshot(const RunOptions& opt, const std::string& dir, const std::string& why,
                                  std::ostream* log) {
  Config& C = cs.cfg;
  const int nr = comm->size(), r = comm->rank();
  try {
    download(cs.J);   // device state at the failing step
  } catch (...) {
  }
  const std::string name = (nr > 1 ? "rank-" + std::to_string(r) + "-" : std::string()) + plt_stem(C.out_file) +
                           "-err.plt";
  // the reference stamps the snapshot with GlobalTime, which advances only at
  // cycle ends (deeps2d_core.cpp:1264-1279, 1785-1788)
  // (a strip rank writes its own columns: the failure need not be collective)
  if (opt.write_outputs) {
    const auto own = owned_columns();
    save_field_plt_cols(dir + "/" + name, cs, cs.J, cs.global_time, true, nr > 1 ? own.first : 0,
                        nr > 1 ? own.second : cs.J.nx);
  }
  if (log && (r == 0 || nr > 1)) {
    *log << "\n" << why;
    // the first owned active cell with Tg < 0 (deeps2d_core.cpp:1246-1316 report + PrintCond)
    const auto own = owned_columns();
    bool found = false;
    for (int i = own.first; i < own.second && !found; i++)
      for (int j = 0; j < cs.J.ny && !found; j++) {
        const CellRecord& c = cs.J.at(i, j);
        if (has_all(c.CT, CT_NODE_IS_SET) && !has_all(c.CT, CT_SOLID) && !(c.Tg >= 0)) {
          *log << "\nTg=" << c.Tg << " in cell (" << i << ", " << j << ") of rank " << r << "\n  CT: "
               << cond_names(c.CT) << "\n  TurbType: " << turb_cond_names(c.TurbType);
          found = true;
        }
      }
    *log << "\nError snapshot: " << dir << "/" << name;
    if (opt.write_checkpoint && (ckpt_written || cs.preloaded))
      *log << "; last good checkpoint (iteration " << last_iter << "): " << dir << "/" << C.swap_file;
    else if (opt.write_checkpoint)
      *log << "; no checkpoint was written before the failure";
    *log << "\n" << std::flush;
  }
}

void SolverBase::inject_fault(const RunOptions& opt) {
  if (opt.fault_kind == "kill") {
    std::fflush(stdout);
    std::raise(SIGKILL);
    return;
  }
  // an active gas cell nearest the centre of this rank's strip
  const auto own = owned_columns();
  const Field& J = cs.J;
  const int ci = (own.first + own.second) / 2, cj = J.ny / 2;
  for (int d = 0; d < std::max(J.nx, J.ny); d++)
    for (int i = std::max(own.first, ci - d); i <= std::min(own.second - 1, ci + d); i++)
      for (int j = std::max(0, cj - d); j <= std::min(J.ny - 1, cj + d); j++) {
        const u64 CT = J.at(i, j).CT;
        if (has_all(CT, CT_NODE_IS_SET) && !has_all(CT, CT_SOLID) && !has_all(CT, NT_FC)) {
          poison_cell(i, j);
          return;
        }
      }
}

int SolverBase::run(const RunOptions& opt, std::ostream* log) {
  const std::string dir0 = opt.outdir.empty() ? "." : opt.outdir;
  int cycles = 0;
  try {
    cycles = run_cycles(opt, log);
  } catch (const std::runtime_error& e) {
    const std::string msg = e.what();
    if (msg.find("unstability") != std::string::npos || msg.find("P2P") != std::string::npos)
      failure_snapshot(opt, dir0, msg, log);
    if (!opt.profile_path.empty()) write_profile(opt.profile_path, cycle);
    throw;
  }
  if (!opt.profile_path.empty()) write_profile(opt.profile_path, cycles);
  return cycles;
}

int SolverBase::run_cycles(const RunOptions& opt, std::ostream* log) {
  Config& C = cs.cfg;
  const bool root = comm->rank() == 0;
  const std::string dir = opt.outdir.empty() ? "." : opt.outdir;
  const std::string rms_path = dir + "/RMS-" + C.out_file;
  const std::string mon_path = dir + "/Monitors-" + C.out_file;
  if (root && opt.write_outputs) {
    // the pre-processor truncates the field file of a cold start
    // (deeps2d_core.cpp:3858-3860): a run that fails in its first cycle
    // leaves it empty
    if (!cs.preloaded) {
      std::FILE* t = std::fopen((dir + "/" + C.out_file).c_str(), "w");
      if (t) std::fclose(t);
    }
  }
  if (root && opt.write_checkpoint && !cs.preloaded && !checkpoint_image_present(dir + "/" + C.swap_file, C.MaxX, C.MaxY)) {
    // LoadSwapFile2D creates the swap file zero-filled at its full size on a
    // cold start (obj_data.cpp:173-219): a run that fails before its first
    // cycle end leaves that image.  A full-size image that was only ignored
    // (use_checkpoint off) is kept until the first cycle end overwrites it.
    create_zero_hf2d(dir + "/" + C.swap_file, C.MaxX, C.MaxY);
  }
  if (root && opt.write_outputs) {
    save_rms_header(rms_path, C);
    if (!C.monitors.empty()) save_monitors_header(mon_path, C);
  }
  // collective output decisions must agree on every rank
  const bool log_any = comm->allreduce_max_int(log ? 1 : 0) != 0;
  int I = 0;
  int monitor_cond = 1;
  bool interrupted = false;
  int cycles = 0;
  using clk = std::chrono::steady_clock;
  do {
    isSrcAdd = (0 < iter + last_iter);
    iter = 0;
    auto t_cycle = clk::now();
    auto mark = clk::now();
    for (long k = 0; k < C.Nmax; k++) {
      const bool out_step = (iter / C.NOutStep) * C.NOutStep == iter;
      const long this_iter = iter;
      if (opt.fault_step >= 0 && last_iter + iter == opt.fault_step && comm->rank() == opt.fault_rank)
        inject_fault(opt);
      step_outputs = out_step || k == C.Nmax - 1;
      {
        PhaseScope ph(*this, "steps");
        advance(out_step || k == C.Nmax - 1);
      }
      step_outputs = true;
      if (out_step && comm->allreduce_max_int(stop_requested() ? 1 : 0)) {
        interrupted = true;
        if (log && root) *log << "\nInterrupted by user: finishing the cycle outputs and checkpoint.\n";
        break;
      }
      if (out_step) {
        if (!C.monitors.empty()) sample_monitors(C.monitors);
        // nozzle Cd / Cv of the RMS file: evaluated by the owner of the cut
        // column (collective, so every rank takes part)
        real cd_cv[2];
        const bool want_cd = C.isVerboseOutput && opt.write_outputs && C.is_Cd_calc && C.Cd_Flow_index >= 1 &&
                             C.Cd_Flow_index <= (int)cs.flows2d.size();
        if (want_cd) {
          const auto own = owned_columns();
          strip_cd_cv(*comm, cs, cs.J, own.first, own.second, cs.flows2d[C.Cd_Flow_index - 1], cd_cv);
        }
        if (C.isVerboseOutput && root) {
          auto now = clk::now();
          const double d_time = std::chrono::duration<double>(now - mark).count();
          mark = now;
          const double vcomp = d_time > 0 ? C.NOutStep / d_time : 0.;
          if (!opt.metrics_path.empty()) {
            std::FILE* mf = std::fopen(opt.metrics_path.c_str(), "a");
            if (mf) {
              std::fprintf(mf, "{\"step\": %ld, \"time\": %.17g, \"dt\": %.17g, \"max_rms\": %.17g, \"rms\": [",
                           last_iter + this_iter, cs.global_time + cur_time_part, dt, last_res.max_rms);
              for (int q = 0; q < NEQ; q++) std::fprintf(mf, "%s%.17g", q ? ", " : "", last_res.rms[q]);
              std::fprintf(mf, "], \"step_per_s\": %.6g, \"mcells_it_per_s\": %.6g, \"ranks\": %d}\n", vcomp,
                           vcomp * (double)C.MaxX * C.MaxY / 1e6, comm->size());
              std::fclose(mf);
            }
          }
          if (opt.write_outputs) {
            append_rms(rms_path, last_iter + this_iter, last_res.rms, C, want_cd ? cd_cv : nullptr);
            if (!C.monitors.empty()) append_monitors(mon_path, cs.global_time + cur_time_part, C.monitors);
          }
          if (log) {
            char b[512];
            const int kk = last_res.k_max;
            const char* nm = (C.MonitorIndex > 0 && C.MonitorIndex < 5) ? RMS_NAME[C.MonitorIndex - 1]
                             : (kk >= 0 ? RMS_NAME[kk] : "?");
            std::snprintf(b, sizeof b, "Step No %ld maxRMS[%s]=%g %% step_time=%g sec (%g step/sec) dt=%g\n",
                          last_iter + this_iter, nm, last_res.max_rms * 100., d_time, vcomp, dt);
            *log << b << std::flush;
          }
        }
      }
    }
    {
      PhaseScope ph(*this, "sync");
      sync_scalars();
      cycle_update();
    }
    Field& J = cs.J;
    const auto own = owned_columns();
    {
      // each rank refreshes only its strip (+ the neighbours' edge columns
      // that the wall integrals read); nothing is gathered
      PhaseScope ph(*this, "download");
      download(J);
      strip_exchange_ghosts(*comm, J, own.first, own.second);
    }
    PhaseScope ph_out(*this, "outputs");
    step_seconds = std::chrono::duration<double>(clk::now() - t_cycle).count();
    for (size_t x = 0; x < C.xcuts.size() && log_any; x++) {
      const real mf = strip_mass_flow(*comm, cs, J, own.first, own.second, C.xcuts[x].x0, C.xcuts[x].y0, C.xcuts[x].dy);
      if (root && log) {
        char b[256];
        std::snprintf(b, sizeof b, "Cut(%zu) X=%g Y=%g dY=%g MassFlow=%g  (kg/sec*m)\n", x + 1, C.xcuts[x].x0,
                      C.xcuts[x].y0, C.xcuts[x].dy, mf);
        *log << b;
      }
    }
    if (opt.write_outputs) {
      strip_write_plt(*comm, dir + "/" + C.out_file, cs, J, own.first, own.second, cs.global_time, true);
      if ((I / C.NSaveStep) * C.NSaveStep == I)
        strip_write_plt(*comm, dir + "/" + C.tecplot_file, cs, J, own.first, own.second, cs.global_time, false);
    }
    if (root && log) {
      char b[256];
      std::snprintf(b, sizeof b, "HyperFLOW/DEEPS computation cycle time=%g sec ( average  speed %g step/sec).       \n",
                    step_seconds, C.Nmax / step_seconds);
      *log << b << std::flush;
    }
    I++;
    last_iter += iter;
    iter = 0;
    cs.global_time += cur_time_part;
    cur_time_part = 0.;
    on_cycle_roll();
    cycle++;
    cycles++;
    if (opt.write_outputs && C.isOutHeatFluxX)
      strip_heat_flux_x(*comm, dir + "/HeatFlux-X-" + C.out_file, cs, J, own.first, own.second);
    if (opt.write_outputs && C.isOutHeatFluxY)
      strip_heat_flux_y(*comm, dir + "/HeatFlux-Y-" + C.out_file, cs, J, own.first, own.second);
    if (C.is_Cx_calc && log_any && C.Cx_Flow_index >= 1 && C.Cx_Flow_index <= (int)cs.flows2d.size()) {
      real F[4];
      strip_body_forces(*comm, cs, J, own.first, own.second, cs.flows2d[C.Cx_Flow_index - 1], F);
      if (root && log) *log << "\nCx = " << F[0] << " Cy = " << F[1] << " Fx = " << F[2] << " Fy = " << F[3] << "\n";
    }
    if (opt.write_checkpoint) {
      PhaseScope ph(*this, "outputs.checkpoint");   // nested in "outputs"
      strip_write_hf2d(*comm, dir + "/" + C.swap_file, J, own.first, own.second);
      if (root) write_meta(dir + "/" + C.swap_file, last_iter, dt, cs.global_time);
      ckpt_written = true;
    }
    if (opt.write_checkpoint && C.mech_mode()) {
      // versioned species sidecar (mechanism_io.hpp): each rank writes the
      // byte range of its own columns
      PhaseScope ph(*this, "outputs.checkpoint_species");
      write_species_slab(dir + "/" + C.swap_file + ".species", *C.mech, J.nx, J.ny, cs.mech_rhoY.data(), cs.mech_n(),
                         own.first - J.i0, own.first, own.second - own.first);
    }
    if (C.MonitorIndex < 5)
      monitor_cond = last_res.max_rms > C.ExitMonitorValue ? 1 : 0;
    else
      monitor_cond = cs.global_time < C.ExitMonitorValue ? 1 : 0;
  } while (!interrupted && monitor_cond && (opt.max_cycles < 0 || cycles < opt.max_cycles));
  if (opt.write_outputs) {
    const auto own = owned_columns();
    strip_write_plt(*comm, dir + "/" + C.out_file, cs, cs.J, own.first, own.second, cs.global_time, true);
  }
  return cycles;
}

// ---------------------------------------------------------------------------
// CpuSolver
// ---------------------------------------------------------------------------
CpuSolver::CpuSolver(Case& c, int g0, int g1) : SolverBase(c), gi0(g0), gi1(g1 < 0 ? c.J.nx : g1) {
  const int lh = gi0 > 0 ? 1 : 0;
  const int rh = gi1 < c.J.nx ? 1 : 0;
  l_off = lh;
  h.allocate((gi1 - gi0) + lh + rh, c.J.ny);
  h.allocate_mech(c);
  upload();
}

void CpuSolver::poison_cell(int gi, int j) {
  const long idx = (long)(gi - gi0 + l_off) * h.ny + j;
  h.S[sbuf][(long)I_RHOE * h.N + idx] = -1.0e30;
}

void RefSolver::poison_cell(int gi, int j) { cs.J.at(gi, j).S[I_RHOE] = -1.0e30; }

void CpuSolver::upload() {
  h.from_field(cs.J, gi0 - l_off);
  h.wall_slots(cs, gi0 - l_off, gi0, gi1);
  h.mech_from_case(cs, gi0 - l_off);
  compute_generic_flags(cs, h, gi0 - l_off);
  sbuf = 0;
  dsbuf = 0;
  pbuf = 0;
  lean_ok = lean_eligible(cs, &lean_why);
  lean_sg_ok = lean_ok && lean_single_gas(cs);
  lean_state = 0;
  if (lean_ok) {
    lb = lean_flags(h, cs.cfg.ProblemType);
    for (int b = 0; b < 2; b++) {
      Spre[b].assign(NCOMP * h.N, 0.0);
      P2[b].assign(h.N, 0.0);
    }
  }
}

void CpuSolver::download(Field& J) {
  if (lean_state) lean_materialize();
  h.to_field(J, gi0 - l_off, l_off, l_off + (gi1 - gi0), pbuf, dsbuf);
  h.mech_to_case(cs, gi0 - l_off, l_off, l_off + (gi1 - gi0), 0);
}

LeanSoA CpuSolver::lean_view(bool fromg) {
  LeanSoA L;
  L.N = h.N;
  L.Sin = h.S[0].data();
  L.Sout = h.S[1].data();
  L.Pin_s = Spre[pbuf].data();
  L.Pout_s = Spre[1 - pbuf].data();
  L.beta = h.beta.data();
  L.Uin = h.U[pbuf].data();
  L.Vin = h.V[pbuf].data();
  L.Pin = fromg ? h.p.data() : P2[pbuf].data();
  L.Uout = h.U[1 - pbuf].data();
  L.Vout = h.V[1 - pbuf].data();
  L.Pout = P2[1 - pbuf].data();
  L.Tout = h.Tg[1 - pbuf].data();
  L.dSdx_in = h.dSdx[dsbuf].data();
  L.dSdy_in = h.dSdy[dsbuf].data();
  L.dSdx_out = h.dSdx[1 - dsbuf].data();
  L.dSdy_out = h.dSdy[1 - dsbuf].data();
  L.CT = h.CT.data();
  L.lb = lb.data();
  L.CP = h.CP.data();
  L.R = h.R.data();
  L.kk = h.kk.data();
  L.Y = h.Y.data();
  L.Tf = h.Tf.data();
  L.BGX = h.BGX.data();
  L.BGY = h.BGY.data();
  L.SrcAdd = h.SrcAdd.data();
  L.gA = h.A.data();
  L.gB = h.B.data();
  L.gF = h.F.data();
  return L;
}

void CpuSolver::lean_materialize() {
  StepParams P = make_params(last_iter + iter);
  P.nx = h.nx;
  P.ny = h.ny;
  LeanSoA L = lean_view(false);
  SoA g = h.view(0, dsbuf, pbuf);
  for (int i = 0; i < h.nx; i++)
    for (int j = 0; j < h.ny; j++) lean_materialize_cell(P, L, g, i, j);
  lean_state = 0;
}

int CpuSolver::halo_doubles(int g) const {
  const int ns = h.nsp, sdx = h.dSdxs[0].empty() ? 0 : 1;
  if (g == HALO_MID) return NEQ + ns;
  if (g == HALO_QDIR) return 4;
  if (g == HALO_LEAN) return 4 + 2 * NCOMP + 3 + NEQ;
  return 4 * NEQ + 5 + ns * (3 + sdx);
}

void CpuSolver::pack_column(int g, int li, real* o) const {
  const long N = h.N;
  const int ny = h.ny;
  for (int j = 0; j < ny; j++) {
    const long idx = (long)li * ny + j;
    if (g == HALO_MID) {
      for (int k = 0; k < NEQ; k++) *o++ = h.S[1][k * N + idx];
      for (int sp = 0; sp < h.nsp; sp++) *o++ = h.Ys[1][sp * N + idx];
    } else if (g == HALO_QDIR) {
      for (int d = 0; d < 4; d++) *o++ = h.qdir[d * N + idx];
    } else if (g == HALO_LEAN) {
      for (int k = 0; k < 4 + NCOMP; k++) *o++ = h.S[0][k * N + idx];
      for (int k = 0; k < NCOMP; k++) *o++ = Spre[pbuf][k * N + idx];
      *o++ = h.U[pbuf][idx];
      *o++ = h.V[pbuf][idx];
      *o++ = P2[pbuf][idx];
      for (int k = 0; k < NEQ; k++) *o++ = h.dSdx[dsbuf][k * N + idx];
    } else {
      for (int k = 0; k < NEQ; k++) {
        *o++ = h.S[0][k * N + idx];
        *o++ = h.A[k * N + idx];
        *o++ = h.B[k * N + idx];
        *o++ = h.dSdx[dsbuf][k * N + idx];
      }
      *o++ = h.U[pbuf][idx];
      *o++ = h.V[pbuf][idx];
      *o++ = h.Tg[pbuf][idx];
      *o++ = h.lam[idx];
      *o++ = h.lam_t[idx];
      for (int sp = 0; sp < h.nsp; sp++) {
        *o++ = h.Ys[0][sp * N + idx];
        *o++ = h.As[sp * N + idx];
        *o++ = h.Bs[sp * N + idx];
        if (!h.dSdxs[0].empty()) *o++ = h.dSdxs[dsbuf][sp * N + idx];
      }
    }
  }
}

void CpuSolver::unpack_column(int g, int li, const real* o) {
  const long N = h.N;
  const int ny = h.ny;
  for (int j = 0; j < ny; j++) {
    const long idx = (long)li * ny + j;
    if (g == HALO_MID) {
      for (int k = 0; k < NEQ; k++) h.S[1][k * N + idx] = *o++;
      for (int sp = 0; sp < h.nsp; sp++) h.Ys[1][sp * N + idx] = *o++;
    } else if (g == HALO_QDIR) {
      for (int d = 0; d < 4; d++) h.qdir[d * N + idx] = *o++;
    } else if (g == HALO_LEAN) {
      for (int k = 0; k < 4 + NCOMP; k++) h.S[0][k * N + idx] = *o++;
      for (int k = 0; k < NCOMP; k++) Spre[pbuf][k * N + idx] = *o++;
      h.U[pbuf][idx] = *o++;
      h.V[pbuf][idx] = *o++;
      P2[pbuf][idx] = *o++;
      for (int k = 0; k < NEQ; k++) h.dSdx[dsbuf][k * N + idx] = *o++;
    } else {
      for (int k = 0; k < NEQ; k++) {
        h.S[0][k * N + idx] = *o++;
        h.A[k * N + idx] = *o++;
        h.B[k * N + idx] = *o++;
        h.dSdx[dsbuf][k * N + idx] = *o++;
      }
      h.U[pbuf][idx] = *o++;
      h.V[pbuf][idx] = *o++;
      h.Tg[pbuf][idx] = *o++;
      h.lam[idx] = *o++;
      h.lam_t[idx] = *o++;
      for (int sp = 0; sp < h.nsp; sp++) {
        h.Ys[0][sp * N + idx] = *o++;
        h.As[sp * N + idx] = *o++;
        h.Bs[sp * N + idx] = *o++;
        if (!h.dSdxs[0].empty()) h.dSdxs[dsbuf][sp * N + idx] = *o++;
      }
    }
  }
}

StepResult CpuSolver::do_step(const StepParams& P0, bool want_res) {
  StepParams P = P0;
  P.nx = h.nx;
  P.ny = h.ny;
  P.i0 = l_off;
  P.i1 = l_off + (gi1 - gi0);
  P.gx0 = gi0 - l_off;
  P.do_residual = want_res ? 1 : 0;
  StepResult r;
  residual_reset(r.res);
  if (lean && lean_ok) {
    // lean inviscid step: S[0] -> S[1] (swapped back), prims/dS ping-pong
    const bool fromg = lean_state == 0;
    if (fromg) h.S[1] = h.S[0];
    LeanSoA L = lean_view(fromg);
    int negT = 0;
    real dtmin = 1.0;
    ResidualPack* rp = want_res ? &r.res : nullptr;
    if (!fromg && lean_tile && P.ny >= LEAN_TILE_MIN_TJ) {
      // host emulation of the device's LDS-tiled kernel (same staging and
      // indexing); unstaged LDS entries are poisoned with NaN
      const int NT = lean_nt == 128 || lean_nt == 64 ? lean_nt : 256;
      const LeanTile T = lean_tile_geom(P.i1 - P.i0, P.ny, NT, lean_tj, lean_cpt == 2 ? 2 : 1);
      const bool sg = lean_sg && lean_sg_ok;
      std::vector<real> lds((size_t)lean_tile_fields(sg) * T.NC);
      for (int b = 0; b < T.nbi * T.nbj; b++) {
        std::fill(lds.begin(), lds.end(), std::numeric_limits<real>::quiet_NaN());
        int i, j, c, i0, j0;
        lean_tile_cell(P, T, b, 0, &i, &j, &c, &i0, &j0);
        for (int t = 0; t < NT; t++) {
          if (sg)
            lean_tile_stage<true>(P, L, T, i0, j0, lds.data(), t, NT);
          else
            lean_tile_stage<false>(P, L, T, i0, j0, lds.data(), t, NT);
        }
        for (int t = 0; t < NT * T.CPT; t++) {
          if (!lean_tile_cell(P, T, b, t % NT, &i, &j, &c, &i0, &j0, t / NT)) continue;
          if (sg) {
            TileIO<true> io(L, (long)i * P.ny + j, lds.data(), T.NC, T.W, c);
            dtmin = std::min(dtmin, lean_cell_host(P, L, io, i, j, rp, &negT));
          } else {
            TileIO<false> io(L, (long)i * P.ny + j, lds.data(), T.NC, T.W, c);
            dtmin = std::min(dtmin, lean_cell_host(P, L, io, i, j, rp, &negT));
          }
        }
      }
    } else {
      for (int i = P.i0; i < P.i1; i++)
        for (int j = 0; j < P.ny; j++) {
          real d;
          if (fromg) {
            LeanIO<true> io(L, (long)i * P.ny + j);
            d = lean_cell_host(P, L, io, i, j, rp, &negT);
          } else {
            LeanIO<false> io(L, (long)i * P.ny + j);
            d = lean_cell_host(P, L, io, i, j, rp, &negT);
          }
          dtmin = std::min(dtmin, d);
        }
    }
    // halo columns keep their exchanged values
    for (int i = 0; i < h.nx; i++) {
      if (i >= P.i0 && i < P.i1) continue;
      for (int k = 0; k < 4 + NCOMP; k++)
        for (int j = 0; j < P.ny; j++) h.S[1][k * h.N + (long)i * P.ny + j] = h.S[0][k * h.N + (long)i * P.ny + j];
    }
    h.S[0].swap(h.S[1]);
    dsbuf = 1 - dsbuf;
    pbuf = 1 - pbuf;
    lean_state = 1;
    r.have_residual = want_res;
    r.dt_min = dtmin;
    r.neg_T = negT;
    if (halo_exchange) halo_exchange(*this, HALO_LEAN);
    return r;
  }
  if (lean_state) lean_materialize();
  // predict: S[0] -> S[1], dS[dsbuf] -> dS[1-dsbuf]
  const bool mech = h.mech != nullptr;
  SoA in = h.view(0, dsbuf, pbuf);
  SoA mid = h.view(1, 1 - dsbuf, pbuf);
  // halo columns keep their (exchanged) values in the mid buffer as well
  for (int i = P.i0; i < P.i1; i++)
    for (int j = 0; j < P.ny; j++) {
      if (mech) {
        if (want_res)
          predict_cell_t<true, SK_MECH>(P, in, mid, i, j, r.res);
        else {
          ResidualPack d;
          predict_cell_t<false, SK_MECH>(P, in, mid, i, j, d);
        }
      } else {
        predict_cell(P, in, mid, i, j, want_res ? &r.res : nullptr);
      }
    }
  r.have_residual = want_res;
  if (halo_exchange && P.sm == SM_NS) halo_exchange(*this, HALO_MID);
  if (mech) {
    // operator-split kinetics: Ys[1] -> Ys[0] (N-S strips also react the
    // exchanged ghost columns: same inputs, same result as their owner)
    SoA co = h.view(0, 1 - dsbuf, pbuf);
    const int ci0 = (halo_exchange && P.sm == SM_NS) ? 0 : P.i0;
    const int ci1 = (halo_exchange && P.sm == SM_NS) ? P.nx : P.i1;
    for (int i = ci0; i < ci1; i++)
      for (int j = 0; j < P.ny; j++) mech_chem_soa_cell<MECH_MAXSP>(P, mid, co, h.Tg[pbuf].data(), i, j);
  }
  // fill: S[1] (+nbrs) -> S[0]; prims pbuf -> 1-pbuf
  SoA sin = h.view(1, 1 - dsbuf, pbuf);
  if (mech) h.mech_view(sin, 0, 1 - dsbuf);   // post-chemistry species
  SoA pold = sin;
  SoA out = h.view(0, 1 - dsbuf, 1 - pbuf);
  int negT = 0;
  real dtmin = 1.0;
  for (int i = P.i0; i < P.i1; i++)
    for (int j = 0; j < P.ny; j++) {
      const real d = mech ? fill_cell<SK_MECH, MECH_MAXSP>(P, sin, pold, out, i, j, &negT, true)
                          : fill_cell(P, sin, pold, out, i, j, &negT, true);
      dtmin = std::min(dtmin, d);
    }
  dsbuf = 1 - dsbuf;
  pbuf = 1 - pbuf;
  r.dt_min = dtmin;
  r.neg_T = negT;
  if (halo_exchange) halo_exchange(*this, HALO_STATE);
  if (!cs.cfg.isAdiabaticWall) {
    SoA s = h.view(0, dsbuf, pbuf);
    for (int i = P.i0; i < P.i1; i++)
      for (int j = 0; j < P.ny; j++) wall_heat_solid_cell(P, s, h.qdir.data(), i, j);
    if (halo_exchange) halo_exchange(*this, HALO_QDIR);
    for (int i = P.i0; i < P.i1; i++)
      for (int j = 0; j < P.ny; j++) wall_heat_wall_cell(P, s, h.qdir.data(), i, j);
  }
  return r;
}

void CpuSolver::cycle_update() {
  if (cs.cfg.ProblemType != SM_NS || cs.cfg.semantics == Semantics::SERIAL) return;
  SoA s = h.view(0, dsbuf, pbuf);
  std::vector<int32_t> sl;
  std::vector<real> v;
  for (size_t k = 0; k < h.wall_own.size(); k++) {
    if (!is_wall_gas(s.CT[h.wall_own[k]])) continue;
    sl.push_back(h.wall_own_slot[k]);
    v.push_back(wall_friction_velocity(s, h.wall_own[k]));
  }
  std::vector<real> uw;
  std::vector<uint8_t> ok;
  merge_wall_uw(sl, v, uw, ok);
  for (long idx = (long)l_off * h.ny; idx < (long)(l_off + (gi1 - gi0)) * h.ny; idx++)
    y_plus_apply(s, idx, uw.data(), ok.data());
}

// ---------------------------------------------------------------------------
// RefSolver: in-place reference-order sweep (deeps2d_core.cpp:853-1334)
// ---------------------------------------------------------------------------
RefSolver::RefSolver(Case& c) : SolverBase(c) {
  if (c.cfg.mech_mode())
    throw std::runtime_error("the reference-order backend has no mechanism mode (the reference has no detailed kinetics)");
  // the reference does not persist the iteration counter: a resumed run
  // restarts its scenarios and TurbStartIter at 0
  last_iter = 0;
  core.resize(c.J.c.size());
}

StepResult RefSolver::do_step(const StepParams& P, bool /*want_res*/) {
  Field& J = cs.J;
  const Config& C = cs.cfg;
  const int MX = J.nx, MY = J.ny;
  StepResult r;
  residual_reset(r.res);
  r.have_residual = true;
  const bool serial = C.semantics == Semantics::SERIAL;
  // pass 1
  for (int i = 0; i < MX; i++)
    for (int j = 0; j < MY; j++) {
      CellRecord& c = J.at(i, j);
      if (!is_active(c.CT)) continue;
      CellRecord& nx = core[(size_t)i * MY + j];
      c.time = cs.global_time;
      const int n1 = c.idXl, n2 = c.idXr, n3 = c.idYu, n4 = c.idYd;
      CellRecord& Up = J.at(i, j + n3);
      CellRecord& Dn = J.at(i, j - n4);
      CellRecord& Rt = J.at(i + n2, j);
      CellRecord& Lt = J.at(i - n1, j);
      const real n_n_1 = 1. / std::max(n1 + n2, 1), m_m_1 = 1. / std::max(n3 + n4, 1);
      const int Num_Eq = num_eq_for(c.TurbType);
      for (int k = 0; k < Num_Eq; k++) {
        const real beta = c.beta[k], _beta = 1. - beta;
        if (k >= 4 + NCOMP && !(C.ProblemType == SM_NS && has_turb_eq(c.TurbType))) continue;
        const EqFlags f = eq_flags(k, c.CT, c.TurbType, C.ProblemType);
        if (!f.upd) continue;
        real dXX, dYY;
        if (f.dx) {
          dXX = c.dSdx[k] = (Rt.A[k] - Lt.A[k]) * n_n_1;
        } else {
          c.S[k] = (Lt.S[k] * n2 + Rt.S[k] * n1) * n_n_1;
          dXX = c.dSdx[k] = 0.;
        }
        if (f.dy) {
          dYY = c.dSdy[k] = (Up.B[k] - Dn.B[k]) * m_m_1;
        } else {
          c.S[k] = (Up.S[k] * n3 + Dn.S[k] * n4) * m_m_1;
          dYY = c.dSdy[k] = 0;
        }
        if (f.dx2) dXX = (Lt.dSdx[k] + Rt.dSdx[k]) * 0.5;
        if (f.dy2) dYY = (Up.dSdy[k] + Dn.dSdy[k]) * 0.5;
        if (C.FT)
          nx.S[k] = c.S[k] * beta + _beta * (P.dxx * (Lt.S[k] + Rt.S[k]) + P.dyy * (Up.S[k] + Dn.S[k])) * 0.5 -
                    (P.dtdx * dXX + P.dtdy * (dYY + c.F[k] / (j + 1))) + (c.Src[k]) * P.dt + c.SrcAdd[k];
        else
          nx.S[k] = c.S[k] * beta + _beta * (P.dxx * (Lt.S[k] + Rt.S[k]) + P.dyy * (Up.S[k] + Dn.S[k])) * 0.5 -
                    (P.dtdx * dXX + P.dtdy * dYY) + (c.Src[k]) * P.dt + c.SrcAdd[k];
      }
    }
  // pass 2
  real dtmin = 1.0;
  const real dx_1 = 1.0 / C.dx, dy_1 = 1.0 / C.dy;
  for (int i = 0; i < MX; i++)
    for (int j = 0; j < MY; j++) {
      CellRecord& c = J.at(i, j);
      if (is_active(c.CT)) {
        CellRecord& nx = core[(size_t)i * MY + j];
        const int n1 = c.idXl, n2 = c.idXr, n3 = c.idYu, n4 = c.idYd;
        CellRecord& Up = J.at(i, j + n3);
        CellRecord& Dn = J.at(i, j - n4);
        CellRecord& Rt = J.at(i + n2, j);
        CellRecord& Lt = J.at(i - n1, j);
        const real dxn = dx_1 / std::max(n1 + n2, 1), dym = dy_1 / std::max(n3 + n4, 1);
        const int Num_Eq = num_eq_for(c.TurbType);
        for (int k = 0; k < Num_Eq; k++) {
          if (!pass2_frozen(k, c.CT, c.TurbType, C.ProblemType) && c.S[k] != 0.) {
            const real Tmp = c.S[k];
            const real absDD = nx.S[k] - c.S[k];
            real DD, sq = 0;
            if (std::fabs(Tmp) > 1.e-15) {
              DD = std::fabs(absDD / Tmp);
              sq = std::sqrt(DD);
            } else {
              DD = 1.0;
            }
            const real bmin = c.is(CT_NONREFLECTED) ? P.nrbc_beta0 : P.beta_min;
            c.beta[k] = blend_beta(P.bff, bmin, c.beta[k], DD, sq);
            EqResidual& e = r.res.eq[k];
            e.dd_max = std::max(e.dd_max, DD);
            if (e.dd_max == DD) {
              e.i = i;
              e.j = j;
            }
            if (P.alternate_rms) {
              e.rms += serial ? absDD : absDD * absDD;
              e.sum_div += Tmp * Tmp;
              if (serial) e.count += 1;
            } else {
              e.rms += DD * DD;
              e.count += 1;
            }
          }
          if (k < 4 + NCOMP) {
            if (!pass2_frozen(k, c.CT, c.TurbType, C.ProblemType)) c.S[k] = nx.S[k];
          } else if (C.ProblemType == SM_NS && has_turb_eq(c.TurbType)) {
            if (!has_all(c.TurbType, TCT_k_CONST << (k - 4 - NCOMP))) c.S[k] = nx.S[k];
          }
        }
        if (C.ProblemType == SM_NS) {
          real aR = Rt.S[0], aL = Lt.S[0], aU = Up.S[0], aD = Dn.S[0];
          c.droYdx[NCOMP] = c.droYdy[NCOMP] = 0.;
          for (int k = 4; k < NEQ - 2; k++) {
            if (!c.is(CT_dYdx_NULL)) {
              c.droYdx[k - 4] = (Rt.S[k] - Lt.S[k]) * dxn;
              aR -= Rt.S[k];
              aL -= Lt.S[k];
            }
            if (!c.is(CT_dYdy_NULL)) {
              c.droYdy[k - 4] = (Up.S[k] - Dn.S[k]) * dym;
              aU -= Up.S[k];
              aD -= Dn.S[k];
            }
          }
          if (!c.is(CT_dYdx_NULL)) c.droYdx[NCOMP] = (aR - aL) * dxn;
          if (!c.is(CT_dYdy_NULL)) c.droYdy[NCOMP] = (aU - aD) * dym;
          const bool wall = c.is(CT_WALL_NO_SLIP) || c.is(CT_WALL_LAW);
          const real w1 = wall ? n1 : 1, w2 = wall ? n2 : 1, w3 = wall ? n3 : 1, w4 = wall ? n4 : 1;
          c.dUdx = (Rt.U * w1 - Lt.U * w2) * dxn;
          c.dVdx = (Rt.V * w1 - Lt.V * w2) * dxn;
          c.dUdy = (Up.U * w3 - Dn.U * w4) * dym;
          c.dVdy = (Up.V * w3 - Dn.V * w4) * dym;
          if (is_two_eq(c.TurbType)) {
            c.dkdx = (Rt.S[I_K] * w1 - Lt.S[I_K] * w2) * dxn / c.S[I_RHO];
            c.depsdx = (Rt.S[I_EPS] * w1 - Lt.S[I_EPS] * w2) * dxn / c.S[I_RHO];
            c.dkdy = (Up.S[I_K] * w3 - Dn.S[I_K] * w4) * dym / c.S[I_RHO];
            c.depsdy = (Up.S[I_EPS] * w3 - Dn.S[I_EPS] * w4) * dym / c.S[I_RHO];
          } else if (c.is_turb(TCT_Spalart_Allmaras_Model)) {
            c.dkdx = (Rt.S[I_K] * w1 - Lt.S[I_K] * w2) * dxn / c.S[I_RHO];
            c.dkdy = (Up.S[I_K] * w3 - Dn.S[I_K] * w4) * dym / c.S[I_RHO];
          }
          c.dTdx = (Rt.Tg - Lt.Tg) * dxn;
          c.dTdy = (Up.Tg - Dn.Tg) * dym;
        }
        fill_node(c, P.fpa);
        if (c.Tg < 0.) {
          // the reference aborts inside the sweep (deeps2d_core.cpp:1246-1316):
          // cells after this one keep their pass-1 state in its error snapshot
          r.neg_T = 1;
          r.dt_min = dtmin;
          return r;
        } else {
          const real AAA = std::sqrt(c.k * c.R * c.Tg);
          dtmin = std::min<real>(dtmin, P.CFL_min * std::min<real>(C.dx / (AAA + std::fabs(c.U)), C.dy / (AAA + std::fabs(c.V))));
          if (C.chem_model != NO_REACTIONS) chemistry_zeldovich(c, C.species, C.ProblemType, C.chem_model);
          if (C.chem_model == CRM_ARRENIUS) chemistry_arrhenius_src(c, C.species, P.dt);
        }
      } else if (c.is(NT_FC)) {
        fill_node(c, P.ffc);
      }
    }
  r.dt_min = dtmin;
  // wall heat, reference scatter order
  if (!C.isAdiabaticWall) {
    for (int i = 0; i < MX; i++)
      for (int j = 0; j < MY; j++) J.at(i, j).Q_conv = 0.;
    for (int i = 0; i < MX; i++)
      for (int j = 0; j < MY; j++) {
        CellRecord& c = J.at(i, j);
        if (c.is(CT_SOLID) || !(c.is(CT_WALL_LAW) || c.is(CT_WALL_NO_SLIP))) continue;
        auto upd = [&](CellRecord& s, real h) {
          const real lam_eff = c.lam + c.lam_t;
          if (s.Q_conv > 0.)
            s.Q_conv = (s.Q_conv - lam_eff * (s.Tg - c.Tg) / h) * 0.5;
          else
            s.Q_conv = -lam_eff * (s.Tg - c.Tg) / h;
          c.SrcAdd[I_RHOE] = -P.dt * s.Q_conv / h;
        };
        if (j > 0 && J.at(i, j - 1).is(CT_SOLID)) upd(J.at(i, j - 1), C.dy);
        if (j < MY - 1 && J.at(i, j + 1).is(CT_SOLID)) upd(J.at(i, j + 1), C.dy);
        if (i > 0 && J.at(i - 1, j).is(CT_SOLID)) upd(J.at(i - 1, j), C.dx);
        if (i < MX - 1 && J.at(i + 1, j).is(CT_SOLID)) upd(J.at(i + 1, j), C.dx);
      }
  }
  return r;
}

}  // namespace hf2d
