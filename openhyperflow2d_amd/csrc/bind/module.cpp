#include <algorithm>
// Python bindings (pybind11) for the native hf2d runtime.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <iostream>
#include <sstream>

#include "../core/case.hpp"
#include "../core/checkpoint.hpp"
#include "../core/postproc.hpp"
#include "../core/solver.hpp"
#include "../hip/chem_mech.hpp"
#include "../hip/chem_fast.hpp"
#include "../hip/chem_rtc.hpp"
#include "../hip/device_solver.hpp"
#include "../hip/numerics.hpp"

namespace py = pybind11;
using namespace hf2d;

namespace {

// Comm whose reductions are delegated to Python callables (gloo tests).
struct PyComm : Comm {
  int r = 0, n = 1;
  std::function<double(double)> f_min, f_sum;
  std::function<int(int)> f_maxi;
  std::function<py::bytes(py::bytes)> f_res;   // allgather-of-packs, returns concatenated bytes
  // allgather(bytes) -> list of every rank's bytes, in rank order
  std::function<py::object(py::bytes)> f_allgather;
  std::vector<std::string> allgather_bytes(const std::string& mine) override {
    if (!f_allgather || n == 1) return {mine};
    py::gil_scoped_acquire g;
    py::object res = f_allgather(py::bytes(mine));
    std::vector<std::string> out;
    for (auto item : res) out.push_back(item.cast<std::string>());
    if ((int)out.size() != n) throw std::runtime_error("allgather_bytes: wrong rank count");
    return out;
  }
  int rank() const override { return r; }
  int size() const override { return n; }
  real allreduce_min(real v) override { return f_min ? f_min(v) : v; }
  real allreduce_sum(real v) override { return f_sum ? f_sum(v) : v; }
  int allreduce_max_int(int v) override { return f_maxi ? f_maxi(v) : v; }
  void allreduce_residual(ResidualPack& p) override {
    if (!f_res) return;
    py::gil_scoped_acquire g;
    py::bytes all = f_res(py::bytes((const char*)&p, sizeof(ResidualPack)));
    std::string s = all;
    const size_t m = s.size() / sizeof(ResidualPack);
    ResidualPack a;
    std::memcpy(&a, s.data(), sizeof(ResidualPack));
    for (size_t q = 1; q < m; q++) {
      ResidualPack b;
      std::memcpy(&b, s.data() + q * sizeof(ResidualPack), sizeof(ResidualPack));
      residual_merge_lex(a, b);
    }
    p = a;
  }
};

// whole-grid host entry points refuse a trimmed strip rank's Case
void need_whole(const Case& c) {
  if (!c.J.whole())
    throw std::runtime_error("this Case keeps only columns [" + std::to_string(c.J.i0) + ", " +
                             std::to_string(c.J.i0 + c.J.nxl) + ") resident (strip rank)");
}

py::array_t<double> field_scalar(const Field& J, const std::string& name) {
  py::array_t<double> a({J.nx, J.ny});
  auto m = a.mutable_unchecked<2>();
  for (int i = 0; i < J.nx; i++)
    for (int j = 0; j < J.ny; j++) {
      if (!J.resident(i)) {   // trimmed strip rank: other ranks' columns read 0
        m(i, j) = 0.0;
        continue;
      }
      const CellRecord& c = J.at(i, j);
      double v = 0;
      if (name.size() == 2 && name[0] == 'S') v = c.S[name[1] - '0'];
      else if (name.size() == 5 && name.compare(0, 4, "beta") == 0) v = c.beta[name[4] - '0'];   // blending factor
      else if (name == "rho") v = c.S[0];
      else if (name == "U") v = c.U;
      else if (name == "V") v = c.V;
      else if (name == "p") v = c.p;
      else if (name == "T") v = c.Tg;
      else if (name == "mu_t") v = c.mu_t;
      else if (name == "mu") v = c.mu;
      else if (name == "lam") v = c.lam;
      else if (name == "Diff") v = c.Diff;
      else if (name == "dUdx") v = c.dUdx;
      else if (name == "dTdy") v = c.dTdy;
      else if (name == "k") v = c.k;
      else if (name == "R") v = c.R;
      else if (name == "CP") v = c.CP;
      else if (name == "l_min") v = c.l_min;
      else if (name == "i_wall") v = c.i_wall;
      else if (name == "j_wall") v = c.j_wall;
      else if (name == "y_plus") v = c.y_plus;
      else if (name == "mach") {
        const double A = std::sqrt(c.k * c.R * c.Tg + 1e-30);
        v = std::sqrt(c.U * c.U + c.V * c.V + 1e-30) / A;
      } else if (name == "solid") v = c.is(CT_SOLID) ? 1.0 : 0.0;
      else if (name == "CT") v = (double)c.CT;
      else throw std::runtime_error("unknown field " + name);
      m(i, j) = v;
    }
  return a;
}

py::dict summary_dict(const SolverBase& s) {
  py::dict d;
  d["iteration"] = s.last_iter + s.iter;
  d["dt"] = s.dt;
  d["time"] = s.cs.global_time + s.cur_time_part;
  py::list rms;
  for (int k = 0; k < NEQ; k++) rms.append(s.last_res.rms[k]);
  d["rms"] = rms;
  d["max_rms"] = s.last_res.max_rms;
  d["k_max"] = s.last_res.k_max;
  return d;
}

template <class T>
void bind_solver_common(py::class_<T, SolverBase>& c) {}

}  // namespace

PYBIND11_MODULE(_hf2d, m) {
  m.doc() = "hf2d native runtime: OpenHyperFLOW2D-compatible DEEPS solver for AMD MI355X";
  m.attr("CELL_RECORD_BYTES") = (int)sizeof(CellRecord);
  m.attr("NEQ") = NEQ;
  m.def("gpu_available", &gpu_available);
  // hf_div / hf_sqrt evaluated on the GPU (csrc/hip/numerics.hip): (a / b, sqrt(a))
  m.def("div_probe", [](py::array_t<double, py::array::c_style | py::array::forcecast> a,
                        py::array_t<double, py::array::c_style | py::array::forcecast> b) {
    if (a.size() != b.size()) throw std::runtime_error("div_probe: a and b differ in size");
    const long n = (long)a.size();
    py::array_t<double> q(n), s(n);
    div_probe(a.data(), b.data(), q.mutable_data(), s.mutable_data(), n);
    return py::make_tuple(q, s);
  });
  // k-omega SST source / flux terms of single interior, active nodes
  // (physics.hpp turb_sst) for an independent NumPy oracle
  // (tests/test_sst_oracle.py): inputs [17, n] rows rho, rho k, rho omega, mu,
  // U, V, y, l_min, dU/dx, dU/dy, dV/dx, dV/dy, dk/dx, dk/dy, domega/dx,
  // domega/dy, CP; returns [9, n]: mu_t, Src_k, Src_omega, RX_k, RX_omega,
  // RY_k, RY_omega, F_k, F_omega
  m.def(
      "sst_probe",
      [](py::array_t<double, py::array::c_style | py::array::forcecast> in, double dt, double dx, double dy, int FT,
         double turb_I) {
        if (in.ndim() != 2 || in.shape(0) != 17) throw std::runtime_error("sst_probe: inputs [17, n]");
        const long n = (long)in.shape(1);
        py::array_t<double> out({9L, n});
        const double* a = in.data();
        double* o = out.mutable_data();
        FillParams P;
        P.dt = dt;
        P.dx = dx;
        P.dy = dy;
        P.FT = FT;
        P.turb_I = turb_I;
        for (long q = 0; q < n; q++) {
          CellLocal c{};
          auto v = [&](int r) { return a[(long)r * n + q]; };
          c.S[I_RHO] = v(0);
          c.S[I_K] = v(1);
          c.S[I_OMEGA] = v(2);
          c.mu = v(3);
          c.U = v(4);
          c.V = v(5);
          c.y = v(6);
          c.l_min = v(7);
          c.dUdx = v(8);
          c.dUdy = v(9);
          c.dVdx = v(10);
          c.dVdy = v(11);
          c.dkdx = v(12);
          c.dkdy = v(13);
          c.depsdx = v(14);
          c.depsdy = v(15);
          c.CP = v(16);
          c.CT = 0;
          c.TurbType = TCT_k_omega_SST_Model;
          turb_sst(c, P, 1, 0);
          const double r[9] = {c.mu_t, c.Src[I_K], c.Src[I_OMEGA], c.RX[I_K], c.RX[I_OMEGA], c.RY[I_K], c.RY[I_OMEGA],
                               c.F[I_K], c.F[I_OMEGA]};
          for (int k = 0; k < 9; k++) o[(long)k * n + q] = r[k];
        }
        return out;
      },
      py::arg("inputs"), py::arg("dt"), py::arg("dx"), py::arg("dy"), py::arg("FT") = 0, py::arg("turb_I") = 0.005);
  // K12 kinetics for runtime mechanisms on the MFMA cores (csrc/hip/chem_mech.hip): mechanism
  // given as a built-in name or the text of a .mech file; returns (rhoY, T, mean ms)
  m.def(
      "chem_mech_run",
      [](const std::string& mech, py::array_t<double, py::array::c_style | py::array::forcecast> rhoY,
         py::array_t<double, py::array::c_style | py::array::forcecast> rho,
         py::array_t<double, py::array::c_style | py::array::forcecast> e,
         py::array_t<double, py::array::c_style | py::array::forcecast> T, double dt, int nsub, int repeats,
         bool valu) {
        auto mi = mech.find('\n') == std::string::npos ? load_mechanism(mech) : parse_mechanism(mech);
        const long n = (long)rho.size();
        if (rhoY.ndim() != 2 || rhoY.shape(0) != mi->data.ns || rhoY.shape(1) != n || e.size() != n || T.size() != n)
          throw std::runtime_error("chem_mech_run: shapes [ns, n], [n], [n], [n]");
        py::array_t<double> y({(long)mi->data.ns, n});
        std::memcpy(y.mutable_data(), rhoY.data(), sizeof(double) * rhoY.size());
        py::array_t<double> Tout(n);
        std::memcpy(Tout.mutable_data(), T.data(), sizeof(double) * n);
        double ms;
        {
          py::gil_scoped_release nogil;
          ms = chem_mech_run_host(mi->data, y.mutable_data(), rho.data(), e.data(), Tout.mutable_data(), n, dt, nsub,
                                  repeats, valu);
        }
        return py::make_tuple(y, Tout, ms);
      },
      py::arg("mech"), py::arg("rhoY"), py::arg("rho"), py::arg("e"), py::arg("T"), py::arg("dt"), py::arg("nsub") = 1,
      py::arg("repeats") = 1, py::arg("valu") = false);
  m.attr("CHEM_MECH_MAX_REACTIONS") = chem_mech_max_reactions();
  m.def("request_stop", &request_stop, "ask a running driver to finish the cycle, write outputs and return");
  m.def("stop_requested", &stop_requested);
  m.def("clear_stop", &clear_stop);
  m.def("install_signal_handlers", &install_signal_handlers,
        "SIGINT/SIGTERM -> graceful stop of SolverBase.run (C-level, works while the GIL is released)");

  py::register_exception<DeckError>(m, "DeckError");

  py::class_<InputDeck>(m, "InputDeck")
      .def_static("from_file", &InputDeck::from_file)
      .def_static("from_string", &InputDeck::from_string, py::arg("text"), py::arg("origin") = "<string>")
      .def("name", &InputDeck::name)
      .def("has", &InputDeck::has)
      .def("get_int", &InputDeck::get_int)
      .def("get_float", &InputDeck::get_float)
      .def("get_string", &InputDeck::get_string)
      .def("get_table", [](InputDeck& d, const std::string& k) {
        const Table& t = d.get_table(k);
        return py::make_tuple(t.x, t.y);
      })
      .def("table_eval", [](InputDeck& d, const std::string& k, double x) { return d.get_table(k).eval(x); })
      .def("set", &InputDeck::set)
      .def("keys", &InputDeck::keys)
      .def("table_names", &InputDeck::table_names)
      .def("to_text", &InputDeck::to_text);

  py::class_<GasFlow>(m, "GasFlow")
      .def(py::init<real, real, real, real, real, real>(), py::arg("Cp"), py::arg("T0"), py::arg("P0"), py::arg("R"),
           py::arg("lam") = 0.01, py::arg("mu") = 5e-5)
      .def_static("make2d", &GasFlow::make2d)
      .def("kg", &GasFlow::kg)
      .def("Tg", py::overload_cast<>(&GasFlow::Tg, py::const_))
      .def("Pg", &GasFlow::Pg)
      .def("ROG", &GasFlow::ROG)
      .def("T0", &GasFlow::T0)
      .def("P0", &GasFlow::P0)
      .def("LAM", &GasFlow::LAM)
      .def("TAU", &GasFlow::TAU)
      .def("PF", &GasFlow::PF)
      .def("EPS", &GasFlow::EPS)
      .def("QF", &GasFlow::QF)
      .def("Asound", &GasFlow::Asound)
      .def("Akr", &GasFlow::Akr)
      .def("mach", py::overload_cast<>(&GasFlow::flow_MACH, py::const_))
      .def("set_mach", py::overload_cast<real>(&GasFlow::flow_MACH))
      .def("wg", py::overload_cast<>(&GasFlow::flow_Wg, py::const_))
      .def("set_wg", py::overload_cast<real>(&GasFlow::flow_Wg))
      .def("set_lam", &GasFlow::flow_LAM)
      .def("correct_flow", &GasFlow::CorrectFlow)
      .def("U", &GasFlow::U)
      .def("V", &GasFlow::V)
      .def("Wg2d", &GasFlow::Wg2d)
      .def("mach2d", &GasFlow::MACH2d)
      .def("set_uv", &GasFlow::set_UV);

  py::class_<Case, std::shared_ptr<Case>>(m, "Case")
      .def_static(
          "from_deck",
          [](const std::string& text, const std::string& workdir, bool use_checkpoint, bool verbose) {
            InputDeck d = InputDeck::from_string(text);
            std::ostringstream* os = nullptr;
            auto cs = std::make_shared<Case>(Case::from_deck(d, workdir, use_checkpoint, nullptr));
            (void)os;
            (void)verbose;
            return cs;
          },
          py::arg("text"), py::arg("workdir") = ".", py::arg("use_checkpoint") = false, py::arg("verbose") = false)
      .def_property_readonly("nx", [](const Case& c) { return c.J.nx; })
      .def_property_readonly("ny", [](const Case& c) { return c.J.ny; })
      .def_property_readonly("dt0", [](const Case& c) { return c.dt0; })
      .def_property_readonly("dx", [](const Case& c) { return c.cfg.dx; })
      .def_property_readonly("thread_block_size", [](const Case& c) { return c.cfg.ThreadBlockSize; })
      .def_property_readonly("dy", [](const Case& c) { return c.cfg.dy; })
      .def_property_readonly("problem_type", [](const Case& c) { return c.cfg.ProblemType; })
      .def_property_readonly("flow_type", [](const Case& c) { return c.cfg.FT; })
      .def_property_readonly("nmax", [](const Case& c) { return c.cfg.Nmax; })
      .def_property_readonly("project", [](const Case& c) { return c.cfg.project; })
      .def_property_readonly("global_time", [](const Case& c) { return c.global_time; })
      .def_property_readonly("wall_nodes", [](const Case& c) { return c.wall_nodes; })
      .def("set_min_distance_to_wall", &Case::set_min_distance_to_wall, py::arg("x0") = 0.0)
      .def("set_min_distance_to_wall_bruteforce", &Case::set_min_distance_to_wall_bruteforce, py::arg("x0") = 0.0)
      .def("set_semantics", [](Case& c, const std::string& s) {
        c.cfg.semantics = (s == "serial") ? Semantics::SERIAL : Semantics::MPI;
      })
      .def("set_chem_model", [](Case& c, int m) { c.cfg.chem_model = m; })
      .def("partition", &Case::partition_columns)
      .def("field", [](const Case& c, const std::string& n) {
        // mechanism mode: "Y:<species>" mass fraction, "rhoY:<species>" partial density
        if ((n.rfind("Y:", 0) == 0 || n.rfind("rhoY:", 0) == 0) && c.cfg.mech_mode()) {
          const bool frac = n[0] == 'Y';
          const std::string sp = n.substr(n.find(':') + 1);
          const auto& names = c.cfg.mech->species;
          const auto it = std::find(names.begin(), names.end(), sp);
          if (it == names.end()) throw std::runtime_error("unknown species " + sp);
          const int q = (int)(it - names.begin());
          py::array_t<double> a({c.J.nx, c.J.ny});
          auto m = a.mutable_unchecked<2>();
          for (int i = 0; i < c.J.nx; i++)
            for (int j = 0; j < c.J.ny; j++) {
              if (!c.J.resident(i)) {
                m(i, j) = 0.0;
                continue;
              }
              const double r = c.mech_rhoY[c.mech_idx(q, i, j)];
              const double rho = c.J.at(i, j).S[I_RHO];
              m(i, j) = frac ? (rho != 0 ? r / rho : 0.0) : r;
            }
          return a;
        }
        return field_scalar(c.J, n);
      })
      .def_property_readonly("mech_mode", [](const Case& c) { return c.cfg.mech_mode(); })
      .def_property_readonly("chem_tmin", [](const Case& c) { return c.cfg.chem_tmin; })
      .def_property_readonly("mech_species", [](const Case& c) {
        return c.cfg.mech ? c.cfg.mech->species : std::vector<std::string>{};
      })
      .def_property_readonly("mech_name", [](const Case& c) { return c.cfg.mech ? c.cfg.mech->name : std::string(); })
      .def("pack_strip",
           [](const Case& c, int a, int b) {
             std::string blob;
             {
               py::gil_scoped_release nogil;
               blob = c.pack_strip(a, b);
             }
             return py::bytes(blob);
           },
           py::arg("a"), py::arg("b"),
           "rank 0 of a strip run: the per-case data and columns [a, b) as bytes (Case.unpack_strip)")
      .def_static(
          "unpack_strip",
          [](py::buffer b) {
            // any contiguous byte buffer (bytes, numpy uint8): read in place, no copy
            const py::buffer_info bi = b.request();
            return std::make_shared<Case>(
                Case::unpack_strip((const char*)bi.ptr, (size_t)bi.size * (size_t)bi.itemsize, nullptr));
          },
          "the strip Case of a pack_strip blob (columns [a, b) resident; no pre-processing)")
      .def("pack_strip_header", [](const Case& c, int a, int b) { return py::bytes(c.pack_strip_header(a, b)); })
      .def("strip_payload_bytes", &Case::strip_payload_bytes)
      .def("read_strip_payload",
           [](const Case& c, int a, int b, size_t off, py::buffer dst) {
             const py::buffer_info bi = dst.request(true);
             c.read_strip_payload(a, b, off, (char*)bi.ptr, (size_t)bi.size * (size_t)bi.itemsize);
           })
      .def_static("unpack_strip_header",
                  [](py::buffer b) {
                    const py::buffer_info bi = b.request();
                    return std::make_shared<Case>(
                        Case::unpack_strip_header((const char*)bi.ptr, (size_t)bi.size * (size_t)bi.itemsize));
                  })
      .def("write_strip_payload",
           [](Case& c, size_t off, py::buffer src) {
             const py::buffer_info bi = src.request();
             c.write_strip_payload(off, (const char*)bi.ptr, (size_t)bi.size * (size_t)bi.itemsize);
           })
      .def("compute_facts", &Case::compute_facts)
      .def_static(
          "from_deck_window",
          [](const std::string& text, const std::string& workdir, bool use_checkpoint, int a, int b, bool verbose) {
            InputDeck d = InputDeck::from_string(text);
            py::gil_scoped_release nogil;
            return std::make_shared<Case>(
                Case::from_deck_window(d, workdir, use_checkpoint, a, b, verbose ? &std::cout : nullptr));
          },
          py::arg("text"), py::arg("workdir") = ".", py::arg("use_checkpoint") = false, py::arg("a") = 0,
          py::arg("b") = 0, py::arg("verbose") = false,
          "strip-local pre-processing: records of the columns [a, b) only (whole-grid flags in 16 B/cell while it "
          "runs; a restart reads this slab of the .hf2d); facts valid after merge_facts")
      .def_static(
          "partition_deck",
          [](const std::string& text, const std::string& workdir, bool use_checkpoint, int nparts) {
            InputDeck d = InputDeck::from_string(text);
            py::gil_scoped_release nogil;
            return Case::partition_deck(d, workdir, use_checkpoint, nparts);
          },
          py::arg("text"), py::arg("workdir") = ".", py::arg("use_checkpoint") = false, py::arg("nparts") = 1,
          "active-cell-balanced strips of a deck from a flags-only pre-processing pass (16 B/cell)")
      .def("facts_part", [](const Case& c) { return py::bytes(c.facts_part().pack()); },
           "the cell-level eligibility facts of this Case's resident records (Case.merge_facts)")
      .def("merge_facts",
           [](Case& c, const std::vector<std::string>& parts) {
             std::vector<FactsPart> v;
             for (const auto& p : parts) v.push_back(FactsPart::unpack(p));
             c.merge_facts(v);
           },
           py::arg("parts"), "whole-field facts from every strip's facts_part, in rank order")
      .def_property_readonly("facts_valid", [](const Case& c) { return c.facts.valid; })
      .def_property_readonly("facts",
                             [](const Case& c) {
                               if (!c.facts.valid) throw std::runtime_error("facts not computed / merged");
                               py::dict d;
                               d["lean_ok"] = c.facts.lean_ok;
                               d["lean_why"] = c.facts.lean_why;
                               d["sk_mode"] = c.facts.sk_mode;
                               d["sk_why"] = c.facts.sk_why;
                               d["single_gas"] = c.facts.single_gas;
                               d["any_cauchy_x"] = c.facts.any_cauchy_x;
                               d["species_cauchy"] = c.facts.species_cauchy;
                               return d;
                             })
      .def("resident_records",
           [](const Case& c) { return py::bytes((const char*)c.J.c.data(), c.J.c.size() * sizeof(CellRecord)); },
           "the 1248-byte records of the resident columns (x-major)")
      .def("resident_species",
           [](const Case& c) {
             return py::array_t<double>((py::ssize_t)c.mech_rhoY.size(), c.mech_rhoY.data());
           },
           "mechanism mode: the species partial densities of the resident columns, species-major")
      .def_property_readonly("subdomains", [](const Case& c) { return c.subdomains; })
      .def("trim_to_columns", &Case::trim_to_columns, py::arg("a"), py::arg("b"),
           "strip rank: keep only columns [a, b) of the host field resident (after the solver uploaded its strip)")
      .def_property_readonly("resident_columns", [](const Case& c) { return py::make_tuple(c.J.i0, c.J.i0 + c.J.nxl); })
      .def("records", [](const Case& c) {
        need_whole(c);
        return py::bytes((const char*)c.J.c.data(), c.J.c.size() * sizeof(CellRecord));
      })
      .def("set_records", [](Case& c, py::bytes b) {
        need_whole(c);
        std::string s = b;
        if (s.size() != c.J.c.size() * sizeof(CellRecord)) throw std::runtime_error("record size mismatch");
        std::memcpy((void*)c.J.c.data(), s.data(), s.size());
      })
      .def("write_checkpoint", [](const Case& c, const std::string& p) {
        need_whole(c);
        write_hf2d(p, c.J);
      })
      .def("read_checkpoint",
           [](Case& c, const std::string& p) {
             need_whole(c);
             return read_hf2d(p, c.J);
           })
      .def("save_plt", [](const Case& c, const std::string& p, bool rewrite) {
        need_whole(c);
        save_field_plt(p, c, c.J, c.global_time, rewrite);
      })
      .def("mass_flow_x", [](const Case& c, double x0, double y0, double dy) {
        need_whole(c);
        return mass_flow_rate_x(c, c.J, x0, y0, dy);
      })
      // libOutCFD integrals on the host records (out_cfd_param.cpp)
      .def("flow2d_count", [](const Case& c) { return (int)c.flows2d.size(); })
      .def("area_x",
           [](const Case& c, double x0, double y0, double dy) {
             need_whole(c);
             return calc_area(c, c.J, x0, y0, dy);
           })
      .def("x_force", [](const Case& c, double x0, double y0, double dx, double dy) {
        need_whole(c);
        need_whole(c);
        return x_force(c, c.J, x0, y0, dx, dy);
      })
      .def("y_force", [](const Case& c, double x0, double y0, double dx, double dy) {
        need_whole(c);
        return y_force(c, c.J, x0, y0, dx, dy);
      })
      .def("x_force_ysym", [](const Case& c, double x0, double l, double d) {
        need_whole(c);
        return x_force_ysym(c, c.J, x0, l, d);
      })
      .def("mid_section_area", [](const Case& c, double x0, double y0, double dx, double dy) {
        need_whole(c);
        return mid_section_area(c, c.J, x0, y0, dx, dy);
      })
      .def("cx", [](const Case& c, double x0, double y0, double dx, double dy, int flow) {
        need_whole(c);
        return calc_cx(c, c.J, x0, y0, dx, dy, c.flows2d.at(flow - 1));
      })
      .def("cy", [](const Case& c, double x0, double y0, double dx, double dy, int flow) {
        need_whole(c);
        return calc_cy(c, c.J, x0, y0, dx, dy, c.flows2d.at(flow - 1));
      })
      .def("cd", [](const Case& c, double x0, double y0, double dy, int flow) {
        need_whole(c);
        return calc_cd(c, c.J, x0, y0, dy, c.flows2d.at(flow - 1));
      })
      .def("cv", [](const Case& c, double x0, double y0, double dy, double p_amb, int flow) {
        need_whole(c);
        return calc_cv(c, c.J, x0, y0, dy, p_amb, c.flows2d.at(flow - 1));
      })
      .def("average_pressure", [](const Case& c, double x0, double l, double d) {
        need_whole(c);
        return average_pressure(c, c.J, x0, l, d);
      })
      .def("average_temperature", [](const Case& c, double x0, double l, double d, int mid_enthalpy) {
        need_whole(c);
        return average_temperature(c, c.J, x0, l, d, mid_enthalpy);
      })
      .def("derived_field", [](const Case& c, const std::string& name) {
        // p* (total pressure), T* (total temperature), schlieren |grad rho| (libOutCFD)
        py::array_t<double> a({c.J.nx, c.J.ny});
        auto m = a.mutable_unchecked<2>();
        need_whole(c);
        for (int i = 0; i < c.J.nx; i++)
          for (int j = 0; j < c.J.ny; j++) {
            const CellRecord& n = c.J.at(i, j);
            double v;
            if (name == "p_total") v = p_asterisk(n);
            else if (name == "T_total") v = T_asterisk(n);
            else if (name == "schlieren") v = schlieren(n);
            else throw std::runtime_error("unknown derived field " + name);
            m(i, j) = v;
          }
        return a;
      })
      .def("save_heat_flux", [](const Case& c, const std::string& px, const std::string& py_) {
        need_whole(c);
        if (!px.empty()) save_x_heat_flux(px, c, c.J);
        if (!py_.empty()) save_y_heat_flux(py_, c, c.J);
      });

  m.def("sk_eligible", [](const Case& c) { std::string w; const int md = sk_eligible(c, &w); return py::make_tuple(md, w); },
        py::arg("case"), "split-kernel specialisation (0 generic, 1 single-gas laminar, 2 single-gas turbulent; reason)");
  m.def("smooth", [](py::array_t<double, py::array::c_style> a, int axis) {
        if (a.ndim() != 2) throw std::runtime_error("smooth: (nx, ny) array expected");
        auto buf = a.mutable_data();
        if (axis == 0) smooth_x(buf, (int)a.shape(0), (int)a.shape(1));
        else smooth_y(buf, (int)a.shape(0), (int)a.shape(1));
      }, py::arg("a"), py::arg("axis"), "SmoothX (axis 0) / SmoothY (axis 1), in place");
  m.def("cond_names", &cond_names, py::arg("CT"), "PrintCond: names of the set CondType2D bits");
  m.def("turb_cond_names", &turb_cond_names, py::arg("TT"), "PrintTurbCond: names of the set TurbulenceCondType2D bits");

  py::class_<SolverBase>(m, "SolverBase")
      .def("run_steps", &SolverBase::run_steps, py::arg("n"), py::arg("want_residual_last") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("advance", [](SolverBase& s, bool want) { s.advance(want); }, py::arg("want_residual") = false)
      .def_property_readonly("phase_times",
                             [](const SolverBase& s) {
                               py::dict d;
                               for (const auto& kv : s.phase_acc)
                                 d[py::str(kv.first)] = py::make_tuple(kv.second.first, kv.second.second);
                               return d;
                             })
      .def("set_comm",
           [](SolverBase& s, int rank, int size, std::function<double(double)> fmin, std::function<double(double)> fsum,
              std::function<int(int)> fmaxi, std::function<py::bytes(py::bytes)> fres,
              std::function<py::object(py::bytes)> fallgather) {
             auto* c = new PyComm();
             c->r = rank;
             c->n = size;
             c->f_min = fmin;
             c->f_sum = fsum;
             c->f_maxi = fmaxi;
             c->f_res = fres;
             c->f_allgather = fallgather;
             s.comm = c;   // leaked intentionally: lives as long as the solver
           },
           py::arg("rank"), py::arg("size"), py::arg("fmin"), py::arg("fsum"), py::arg("fmaxi"), py::arg("fres"),
           py::arg("fallgather") = nullptr)
      .def("run",
           [](SolverBase& s, int max_cycles, const std::string& outdir, bool outputs, bool checkpoint, bool verbose,
              const std::string& metrics, const std::string& profile, long fault_step, int fault_rank,
              const std::string& fault_kind) {
             RunOptions o;
             o.metrics_path = metrics;
             o.profile_path = profile;
             o.fault_step = fault_step;
             o.fault_rank = fault_rank;
             o.fault_kind = fault_kind;
             o.max_cycles = max_cycles;
             o.outdir = outdir;
             o.write_outputs = outputs;
             o.write_checkpoint = checkpoint;
             std::ostringstream log;
             int n;
             try {
               py::gil_scoped_release rel;   // comm callbacks re-acquire it
               n = s.run(o, verbose ? &log : nullptr);
             } catch (const std::exception& e) {
               // keep the driver log (it names the error snapshot / last checkpoint)
               throw std::runtime_error(std::string(e.what()) + "\n--- driver log ---\n" + log.str());
             }
             return py::make_tuple(n, log.str());
           },
           py::arg("max_cycles") = 1, py::arg("outdir") = ".", py::arg("outputs") = true,
           py::arg("checkpoint") = true, py::arg("verbose") = true, py::arg("metrics") = "",
           py::arg("profile") = "", py::arg("fault_step") = -1, py::arg("fault_rank") = 0,
           py::arg("fault_kind") = "nan")
      .def("download", [](SolverBase& s) { s.download(s.cs.J); })
      .def("upload", &SolverBase::upload)
      .def("sync", &SolverBase::sync_scalars)
      .def("poison_cell", &SolverBase::poison_cell, py::arg("gi"), py::arg("j"),
           "test hook: a negative energy in cell (gi, j) (the next step reports Tg < 0)")
      .def("summary", &summary_dict)
      .def_readwrite("dt", &SolverBase::dt)
      .def_readonly("iter", &SolverBase::iter)
      .def_readonly("last_iter", &SolverBase::last_iter);

  py::class_<CpuSolver, SolverBase>(m, "CpuSolver")
      .def_readwrite("lean", &CpuSolver::lean)
      .def_readwrite("lean_tile", &CpuSolver::lean_tile)
      .def_readwrite("lean_sg", &CpuSolver::lean_sg)
      .def_readwrite("lean_tj", &CpuSolver::lean_tj)
      .def_readwrite("lean_cpt", &CpuSolver::lean_cpt)
      .def_readwrite("lean_nt", &CpuSolver::lean_nt)
      .def_readonly("lean_sg_ok", &CpuSolver::lean_sg_ok)
      .def_readonly("lean_ok", &CpuSolver::lean_ok)
      .def_readonly("lean_why", &CpuSolver::lean_why)
      .def(py::init<Case&, int, int>(), py::arg("case"), py::arg("gi0") = 0, py::arg("gi1") = -1,
           py::keep_alive<1, 2>())
      .def_readonly("gi0", &CpuSolver::gi0)
      .def_readonly("gi1", &CpuSolver::gi1)
      .def_readonly("l_off", &CpuSolver::l_off)
      .def_property_readonly("local_nx", [](const CpuSolver& s) { return s.h.nx; })
      .def("halo_doubles", &CpuSolver::halo_doubles)
      .def("pack_column",
           [](const CpuSolver& s, int g, int li) {
             py::array_t<double> a(s.halo_doubles(g) * s.h.ny);
             s.pack_column(g, li, a.mutable_data());
             return a;
           })
      .def("unpack_column",
           [](CpuSolver& s, int g, int li, py::array_t<double, py::array::c_style | py::array::forcecast> a) {
             if (a.size() != s.halo_doubles(g) * s.h.ny) throw std::runtime_error("halo size mismatch");
             s.unpack_column(g, li, a.data());
           })
      .def("set_exchange", [](CpuSolver& s, std::function<void(CpuSolver&, int)> f) { s.halo_exchange = f; });

  // --- mechanism (mechanism.hpp) host references ---------------------------
  m.def("mech_load", [](const std::string& name) {
    auto mi = load_mechanism(name);
    py::dict d;
    d["name"] = mi->name;
    d["species"] = mi->species;
    d["nr"] = mi->data.nr;
    d["W"] = std::vector<double>(mi->data.W, mi->data.W + mi->data.ns);
    return d;
  });
  m.def("mech_chem_host", [](const std::string& name, py::array_t<double, py::array::c_style | py::array::forcecast> rhoY,
                             py::array_t<double, py::array::c_style | py::array::forcecast> rho,
                             py::array_t<double, py::array::c_style | py::array::forcecast> e,
                             py::array_t<double, py::array::c_style | py::array::forcecast> T, double dt, int nsub) {
    // [ns, ncell] partial densities at constant (rho, e): the scalar point-implicit
    // integrator the device kernels are checked against; returns (rhoY, T)
    auto mi = name.find('\n') == std::string::npos ? load_mechanism(name) : parse_mechanism(name);
    const MechData& md = mi->data;
    const long n = (long)rho.size();
    if (rhoY.ndim() != 2 || rhoY.shape(0) != md.ns || rhoY.shape(1) != n || e.size() != n || T.size() != n)
      throw std::runtime_error("mech_chem_host: shapes [ns, n], [n], [n], [n]");
    py::array_t<double> out({(long)md.ns, n});
    py::array_t<double> Tout(n);
    auto R = rhoY.unchecked<2>();
    auto O = out.mutable_unchecked<2>();
    auto TO = Tout.mutable_unchecked<1>();
    for (long q = 0; q < n; q++) {
      double y[MECH_MAXSP];
      for (int s = 0; s < md.ns; s++) y[s] = R(s, q);
      double Tq = T.data()[q];
      mech_chem_cell<MECH_MAXSP>(md, rho.data()[q], e.data()[q], y, &Tq, dt, nsub);
      for (int s = 0; s < md.ns; s++) O(s, q) = y[s];
      TO(q) = Tq;
    }
    return py::make_tuple(out, Tout);
  });
  m.def("chem_fast_run", [](const std::string& name, py::array_t<double, py::array::c_style | py::array::forcecast> rhoY,
                            py::array_t<double, py::array::c_style | py::array::forcecast> rho,
                            py::array_t<double, py::array::c_style | py::array::forcecast> e,
                            py::array_t<double, py::array::c_style | py::array::forcecast> T, double dt, int nsub,
                            int repeats) {
    // compiled-mechanism kinetics kernel on the GPU: returns (rhoY, T, mean ms)
    const long n = (long)rho.size();
    if (rhoY.ndim() != 2 || rhoY.shape(1) != n || e.size() != n || T.size() != n)
      throw std::runtime_error("chem_fast_run: shapes [ns, n], [n], [n], [n]");
    py::array_t<double> y({(long)rhoY.shape(0), n});
    std::memcpy(y.mutable_data(), rhoY.data(), sizeof(double) * rhoY.size());
    py::array_t<double> Tout(n);
    std::memcpy(Tout.mutable_data(), T.data(), sizeof(double) * n);
    double ms;
    {
      py::gil_scoped_release nogil;
      ms = chem_fast_run_host(name, y.mutable_data(), rho.data(), e.data(), Tout.mutable_data(), n, dt, nsub, repeats);
    }
    return py::make_tuple(y, Tout, ms);
  });
  // run-time specialised kinetics (chem_rtc.hip): name = built-in name, *.mech path or mechanism text
  auto mech_of = [](const std::string& name) {
    return name.find('\n') == std::string::npos ? load_mechanism(name) : parse_mechanism(name);
  };
  m.def("mech_struct_source", [mech_of](const std::string& name) { return mech_struct_source(mech_of(name)->data); });
  m.def("chem_rtc_program", [mech_of](const std::string& name) { return chem_rtc_program(mech_of(name)->data); });
  m.def("chem_rtc_cache_dir", &chem_rtc_cache_dir);
  m.def("chem_rtc_compile", [mech_of](const std::string& name) {
    // hiprtc compile of the mechanism's kernels (host only): (code bytes, cached, log)
    std::string why;
    bool cached = false;
    long n;
    {
      auto mi = mech_of(name);
      py::gil_scoped_release nogil;
      n = chem_rtc_compile(mi->data, &why, &cached);
    }
    return py::make_tuple(n, cached, why);
  });
  m.def("chem_rtc_run", [mech_of](const std::string& name, py::array_t<double, py::array::c_style | py::array::forcecast> rhoY,
                                  py::array_t<double, py::array::c_style | py::array::forcecast> rho,
                                  py::array_t<double, py::array::c_style | py::array::forcecast> e,
                                  py::array_t<double, py::array::c_style | py::array::forcecast> T, double dt, int nsub,
                                  int repeats) {
    // hiprtc-specialised kinetics kernel on the GPU: returns (rhoY, T, mean ms, code object was cached)
    auto mi = mech_of(name);
    const long n = (long)rho.size();
    if (rhoY.ndim() != 2 || rhoY.shape(0) != mi->data.ns || rhoY.shape(1) != n || e.size() != n || T.size() != n)
      throw std::runtime_error("chem_rtc_run: shapes [ns, n], [n], [n], [n]");
    py::array_t<double> y({(long)rhoY.shape(0), n});
    std::memcpy(y.mutable_data(), rhoY.data(), sizeof(double) * rhoY.size());
    py::array_t<double> Tout(n);
    std::memcpy(Tout.mutable_data(), T.data(), sizeof(double) * n);
    double ms;
    {
      py::gil_scoped_release nogil;
      ms = chem_rtc_run_host(mi->data, y.mutable_data(), rho.data(), e.data(), Tout.mutable_data(), n, dt, nsub,
                             repeats);
    }
    return py::make_tuple(y, Tout, ms, chem_rtc_last_cached());
  });
  m.def("mech_thermo_host", [](const std::string& name, std::vector<double> Y, double T) {
    auto mi = load_mechanism(name);
    double e, cv, R, cp, mu, lam;
    mech_mix_thermo<MECH_MAXSP>(mi->data, Y.data(), T, &e, &cv, &R, &cp);
    mech_transport<MECH_MAXSP>(mi->data, Y.data(), T, &mu, &lam);
    py::dict d;
    d["e"] = e;
    d["cv"] = cv;
    d["R"] = R;
    d["cp"] = cp;
    d["mu"] = mu;
    d["lam"] = lam;
    d["T_from_e"] = mech_T_from_e<MECH_MAXSP>(mi->data, Y.data(), e, 1000.0);
    return d;
  });

  py::class_<RefSolver, SolverBase>(m, "RefSolver").def(py::init<Case&>(), py::keep_alive<1, 2>());

  py::class_<LocalGroup, std::shared_ptr<LocalGroup>>(m, "LocalGroup")
      .def(py::init([](int n) { return make_local_group(n); }), py::arg("n"));

  py::class_<DeviceSolver, SolverBase>(m, "DeviceSolver")
      .def("init_local", &DeviceSolver::init_local, py::arg("group"), py::arg("rank"))
      .def(py::init<Case&, int, int, int>(), py::arg("case"), py::arg("device") = 0, py::arg("gi0") = 0,
           py::arg("gi1") = -1, py::keep_alive<1, 2>())
      .def_static("nccl_unique_id", []() { return py::bytes(DeviceSolver::nccl_unique_id()); })
      .def("init_comm", [](DeviceSolver& s, py::bytes uid, int r, int n) { s.init_comm(std::string(uid), r, n); })
      .def("p2p_loopback", &DeviceSolver::p2p_loopback, py::arg("rank"), py::arg("nranks"))
      .def("p2p_export", [](DeviceSolver& s, int r, int n) { return py::bytes(s.p2p_export(r, n)); },
           py::arg("rank"), py::arg("nranks"))
      .def("p2p_import",
           [](DeviceSolver& s, const std::vector<py::bytes>& d) {
             std::vector<std::string> v;
             for (const auto& b : d) v.push_back(std::string(b));
             s.p2p_import(v);
           })
      .def("fx_trace",
           [](DeviceSolver& s) {
             std::vector<unsigned long long> v;
             {
               py::gil_scoped_release nogil;
               v = s.fx_trace();
             }
             return v;
           })
      .def("p2p_probe",
           [](DeviceSolver& s) {
             std::string b;
             {
               py::gil_scoped_release rel;   // waits for the peers' exchange
               b = s.p2p_probe();
             }
             return py::bytes(b);
           },
           "p2p self-validation blob (collective; see p2p_probe_ok)")
      .def_static("p2p_probe_ok",
                  [](const std::vector<py::bytes>& d, int rank) {
                    std::vector<std::string> v;
                    for (const auto& b : d) v.push_back(std::string(b));
                    std::string why;
                    const bool ok = DeviceSolver::p2p_probe_ok(v, rank, &why);
                    return py::make_tuple(ok, why);
                  },
                  py::arg("blobs"), py::arg("rank"))
      .def("p2p_fallback", &DeviceSolver::p2p_fallback, py::call_guard<py::gil_scoped_release>())
      .def_property("p2p_active", &DeviceSolver::p2p_active, &DeviceSolver::p2p_set)
      .def_readwrite("p2p_fuse", &DeviceSolver::p2p_fuse)
      .def_readwrite("p2p_queue_check", &DeviceSolver::p2p_queue_check)
      .def_readwrite("dt_read_mode", &DeviceSolver::dt_read_mode)
      .def_readwrite("tile_skip_same", &DeviceSolver::tile_skip_same)
      .def_readwrite("lns_ghost_prologue", &DeviceSolver::lns_ghost_prologue)
      .def_readonly("lns_prologue_steps", &DeviceSolver::lns_prologue_steps)
      .def_readwrite("fill_occ", &DeviceSolver::fill_occ)
      .def_readwrite("split_xcd", &DeviceSolver::split_xcd)
      .def_readwrite("grad_every", &DeviceSolver::grad_every)
      .def_readwrite("chem_compact", &DeviceSolver::chem_compact)
      .def_readwrite("comm_overlap", &DeviceSolver::comm_overlap)
      .def_readwrite("lnm_overlap", &DeviceSolver::lnm_overlap)
      .def_readwrite("host_tail", &DeviceSolver::host_tail)
      .def_readwrite("lean_ns", &DeviceSolver::lean_ns)
      .def_readwrite("lns_occ", &DeviceSolver::lns_occ)
      .def_readonly("lns_ok", &DeviceSolver::lns_ok)
      .def_readonly("lns_why", &DeviceSolver::lns_why)
      .def_readonly("lns_state", &DeviceSolver::lns_state)
      .def_readonly("lns_steps", &DeviceSolver::lns_steps)
      .def_readonly("lns_turb", &DeviceSolver::lns_turb)
      .def_readwrite("lean_mech", &DeviceSolver::lean_mech)
      .def_readonly("lnm_ok", &DeviceSolver::lnm_ok)
      .def_readonly("lnm_why", &DeviceSolver::lnm_why)
      .def_readonly("lnm_turb", &DeviceSolver::lnm_turb)
      .def_readonly("lnm_steps", &DeviceSolver::lnm_steps)
      .def_readwrite("lnm_ti", &DeviceSolver::lnm_ti)
      .def_readwrite("lnm_timing", &DeviceSolver::lnm_timing)
      .def_property(
          "lnm_phase_ms",
          [](const DeviceSolver& s) {
            return std::vector<double>(s.lnm_phase_ms, s.lnm_phase_ms + 4);
          },
          [](DeviceSolver& s, const std::vector<double>& v) {
            for (int q = 0; q < 4; q++) s.lnm_phase_ms[q] = q < (int)v.size() ? v[q] : 0.0;
          })
      .def("lnm_trace_fetch", &DeviceSolver::lnm_trace_fetch, py::call_guard<py::gil_scoped_release>())
      .def_readonly("overlap_steps", &DeviceSolver::overlap_steps)
      .def_readonly("lns_fx_steps", &DeviceSolver::lns_fx_steps)
      .def_readonly("p2p_mwg_exchanges", &DeviceSolver::p2p_mwg_exchanges)
      .def("comm_rank", &DeviceSolver::comm_rank)
      .def("comm_size", &DeviceSolver::comm_size)
      .def("synchronize", &DeviceSolver::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("autotune", &DeviceSolver::autotune, py::arg("steps") = 120, py::call_guard<py::gil_scoped_release>())
      .def("trace_tile", &DeviceSolver::trace_tile, py::arg("steps") = 20,
           "one phase-traced lean tile step: per workgroup [entry, staged, wave0 computed, reduced, dt atomic done "
           "(s_memrealtime, 100 MHz), HW_ID, XCC_ID, blockIdx]")
      .def_readwrite("fused", &DeviceSolver::fused)
      .def_readwrite("lean", &DeviceSolver::lean)
      .def_readwrite("lean_tile", &DeviceSolver::lean_tile)
      .def_readwrite("lean_sg", &DeviceSolver::lean_sg)
      .def_readwrite("lean_tj", &DeviceSolver::lean_tj)
      .def_readwrite("tile_stagger", &DeviceSolver::tile_stagger)
      .def_readwrite("lean_occ", &DeviceSolver::lean_occ)
      .def_readwrite("push_per", &DeviceSolver::push_per)
      .def_readwrite("lean_wgcu", &DeviceSolver::lean_wgcu)
      .def_readwrite("use_graph", &DeviceSolver::use_graph)
      .def_readwrite("chem_fast", &DeviceSolver::chem_fast)
      .def_readwrite("chem_kernel", &DeviceSolver::chem_kernel)
      .def_readwrite("chem_rtc", &DeviceSolver::chem_rtc)
      .def_readonly("chem_rtc_ok", &DeviceSolver::chem_rtc_ok)
      .def_readonly("chem_rtc_why", &DeviceSolver::chem_rtc_why)
      .def_readonly("chem_kernel_used", &DeviceSolver::chem_kernel_used)
      .def_readonly("chem_fast_ok", &DeviceSolver::chem_fast_ok)
      .def_readonly("graph_launches", &DeviceSolver::graph_launches)
      .def_readwrite("lean_cpt", &DeviceSolver::lean_cpt)
      .def_readwrite("lean_nt", &DeviceSolver::lean_nt)
      .def_readwrite("sgl", &DeviceSolver::sgl)
      .def_readonly("sgl_ok", &DeviceSolver::sgl_ok)
      .def_readonly("sgl_why", &DeviceSolver::sgl_why)
      .def_readonly("sk_mode", &DeviceSolver::sk_mode)
      .def_readonly("lean_sg_ok", &DeviceSolver::lean_sg_ok)
      .def_readonly("lean_has_cauchy_x", &DeviceSolver::lean_has_cauchy_x)
      .def_readwrite("halo_compact", &DeviceSolver::halo_compact)
      .def_readonly("any_cauchy_x", &DeviceSolver::any_cauchy_x)
      .def("halo_field_count", [](const DeviceSolver& d, int group, bool full) {
        std::vector<real*> f;
        d.halo_fields(group, f, full);
        return (int)f.size();
      }, py::arg("group"), py::arg("full") = false)
      .def_property("lean_plain", [](const DeviceSolver& d) { return d.lean_plain; },
                    [](DeviceSolver& d, bool on) { d.set_lean_plain(on); })
      .def_readonly("lean_ok", &DeviceSolver::lean_ok)
      .def_readonly("lean_why", &DeviceSolver::lean_why)
      .def_readonly("gi0", &DeviceSolver::gi0)
      .def_readonly("gi1", &DeviceSolver::gi1)
      .def_property_readonly("stream", [](const DeviceSolver& s) { return (uintptr_t)s.stream(); });
}
