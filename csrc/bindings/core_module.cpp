// Torch-free Python bindings of the native core (channel_gpu_amd._core).
//
// Config, grid, plan, Solver, I/O, bootstrap and communicator entry points, built with pybind11
// only (no libtorch): a process that imports just this module runs on the ROCm runtime and RCCL
// of /opt/rocm, exactly like the C++ driver binary.  bench.py and the Python driver use it that
// way; the torch extension (_C, bindings.cpp) re-exports everything here and adds the tensor
// kernel entry points used by the tests.
#include <pybind11/complex.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <complex>
#include <map>
#include <memory>

#include "channel/bootstrap.hpp"
#include "channel/comm.hpp"
#include "channel/common.hpp"
#include "channel/config.hpp"
#include "channel/grid.hpp"
#include "channel/io.hpp"
#include "channel/kernels.hpp"
#include "channel/plan.hpp"
#include "channel/solver.hpp"

namespace py = pybind11;
using namespace channel;

namespace {

py::array_t<double> vec(const std::vector<double>& v) {
  py::array_t<double> a(v.size());
  std::copy(v.begin(), v.end(), a.mutable_data());
  return a;
}

py::bytes new_uid() { return py::bytes(Comm::new_unique_id()); }

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // namespace

PYBIND11_MODULE(_core, m) {
  m.doc() = "channel_gpu_amd native core, torch-free bindings (gfx950 HIP kernels, RCCL, HDF5 I/O)";
  py::register_exception<channel::Error>(m, "ChannelError", PyExc_RuntimeError);
  py::class_<Config>(m, "Config")
      .def(py::init<>())
      .def_static("from_file", &Config::from_file, py::arg("path"), py::arg("overrides") = std::vector<std::string>())
      .def_static("from_string",
                  [](const std::string& text, const std::vector<std::string>& overrides) {
                    ConfigTree t = ConfigTree::parse_string(text);
                    for (const auto& o : overrides) {
                      auto eq = o.find('=');
                      CH_CHECK(eq != std::string::npos, "override must be key=value");
                      std::string k = o.substr(0, eq);
                      if (t.has("application." + k)) k = "application." + k;
                      t.set(k, o.substr(eq + 1));
                    }
                    return Config::from_tree(t);
                  },
                  py::arg("text"), py::arg("overrides") = std::vector<std::string>())
      .def("to_string", &Config::to_string)
      .def("validate", &Config::validate)
      .def_property_readonly("nzp", &Config::nzp)
#define RW(f) .def_readwrite(#f, &Config::f)
      RW(NX) RW(NY) RW(NZ) RW(in_G) RW(in_DDV) RW(in_UMEAN) RW(out_G) RW(out_DDV) RW(out_UMEAN) RW(path) RW(Re) RW(Q)
      RW(LX) RW(LZ) RW(stretch) RW(nsteps) RW(t_end) RW(cfl) RW(dt_fixed) RW(dt_max) RW(cfl_mode) RW(stats_every)
      RW(symmetry_every) RW(checkpoint_every) RW(log_every) RW(precision) RW(decomposition) RW(pr) RW(pc) RW(seed)
      RW(ic) RW(ic_amplitude) RW(forcing) RW(influence) RW(explicit_d2) RW(checkpoint_async) RW(health_check) RW(health_every) RW(on_nan) RW(snapshot_every)
      RW(max_rollbacks) RW(rollback_cfl_factor) RW(spectra_every) RW(spectra_planes) RW(log_json);
#undef RW

  m.def("parse_config_tree", [](const std::string& text) { return ConfigTree::parse_string(text).items(); });

  py::class_<YGrid>(m, "YGrid")
      .def_static("build", &YGrid::build, py::arg("N"), py::arg("stretch") = 2.0)
      .def_readonly("N", &YGrid::N)
      .def_property_readonly("y", [](const YGrid& g) { return vec(g.y); })
      .def_property_readonly("d1_lo", [](const YGrid& g) { return vec(g.d1_lo); })
      .def_property_readonly("d1_up", [](const YGrid& g) { return vec(g.d1_up); })
      .def_property_readonly("d1_rm", [](const YGrid& g) { return vec(g.d1_rm); })
      .def_property_readonly("d1_rc", [](const YGrid& g) { return vec(g.d1_rc); })
      .def_property_readonly("d1_rp", [](const YGrid& g) { return vec(g.d1_rp); })
      .def_property_readonly("d1_w0", [](const YGrid& g) { return std::vector<double>(g.d1_w0, g.d1_w0 + 3); })
      .def_property_readonly("d1_wN", [](const YGrid& g) { return std::vector<double>(g.d1_wN, g.d1_wN + 3); })
      .def_property_readonly("m_lo", [](const YGrid& g) { return vec(g.m_lo); })
      .def_property_readonly("m_up", [](const YGrid& g) { return vec(g.m_up); })
      .def_property_readonly("k_lo", [](const YGrid& g) { return vec(g.k_lo); })
      .def_property_readonly("k_c", [](const YGrid& g) { return vec(g.k_c); })
      .def_property_readonly("k_up", [](const YGrid& g) { return vec(g.k_up); })
      .def_property_readonly("trap", [](const YGrid& g) { return vec(g.trap); })
      .def_property_readonly("d2_w0", [](const YGrid& g) { return std::vector<double>(g.d2_w0, g.d2_w0 + 3); })
      .def_property_readonly("d2_wN", [](const YGrid& g) { return std::vector<double>(g.d2_wN, g.d2_wN + 3); })
      .def_readonly("d2_w0_up", &YGrid::d2_w0_up)
      .def_readonly("d2_wN_lo", &YGrid::d2_wN_lo);

  py::class_<Split>(m, "Split")
      .def_static("balanced", &Split::balanced)
      .def_readonly("start", &Split::start)
      .def_readonly("count", &Split::count)
      .def("owner", &Split::owner);

  py::class_<Plan>(m, "Plan")
      .def_static("make", &Plan::make)
#define RO(f) .def_readonly(#f, &Plan::f)
      RO(NX) RO(NY) RO(NZ) RO(Nzp) RO(Kx) RO(nkx) RO(Kz) RO(nkz) RO(P) RO(rank) RO(kx_split) RO(y_split) RO(nkx_loc)
      RO(kx0) RO(ny_loc) RO(y0) RO(R) RO(ax) RO(az) RO(Pr) RO(Pc) RO(prow) RO(pcol) RO(kz_split) RO(x_split)
      RO(nkz_loc) RO(kz0) RO(nx_loc) RO(x0)
#undef RO
      .def("lines_loc", &Plan::lines_loc)
      .def("pencil", &Plan::pencil)
      .def("owns_mean", &Plan::owns_mean)
      .def("kx_of", &Plan::kx_of)
      .def("kx_fft_pos", &Plan::kx_fft_pos);

  m.def("yline_supported_R", &yline_supported_R);


  m.def("new_unique_id", &new_uid);
  m.def("hdf5_available", &hdf5_available);
  m.def("set_debug_sync", &set_debug_sync);
  m.def("set_lds_poison", &set_lds_poison);
  m.def("lds_poison_enabled", &lds_poison_enabled);
  m.def("install_crash_handler", &install_crash_handler, "native backtrace on fatal signals (stderr)");
  m.def("h5_create_field", &h5_create_field, py::arg("path"), py::arg("NX"), py::arg("NY"), py::arg("NZ"),
        py::arg("fp64") = false, py::arg("Kx") = -1);
  m.def("h5_write_planes", &h5_write_planes);
  m.def("h5_read_planes", [](const std::string& p, const std::vector<int>& planes) {
    std::vector<double> d;
    int dims[3];
    h5_read_planes(p, planes, d, dims);
    return std::make_pair(vec(d), std::vector<int>(dims, dims + 3));
  });
  m.def("h5_write_attrs", &h5_write_attrs);
  m.def("h5_write_vector", &h5_write_vector);
  m.def("h5_read_vector", [](const std::string& p, const std::string& name) {
    std::vector<double> v;
    const bool ok = h5_read_vector(p, name, v);
    return py::make_tuple(ok, vec(v));
  });
  m.def("h5_read_attrs", &h5_read_attrs);
  m.def("umean_write", &umean_write);
  m.def("umean_read", &umean_read);

  py::class_<StepLog>(m, "StepLog")
#define LG(f) .def_readonly(#f, &StepLog::f)
      LG(step) LG(time) LG(dt) LG(dt_c) LG(dt_v) LG(umax) LG(vmax) LG(wmax) LG(cflsum) LG(dUdy_lo) LG(dUdy_hi) LG(flux)
      LG(dpdx) LG(utau_lo) LG(utau_hi) LG(utau) LG(health);
#undef LG

  py::class_<Solver>(m, "Solver")
      .def(py::init([](const Config& cfg, int rank, int nranks, int device, py::bytes uid) {
             return std::make_unique<Solver>(cfg, rank, nranks, device, std::string(uid));
           }),
           py::arg("cfg"), py::arg("rank") = 0, py::arg("nranks") = 1, py::arg("device") = 0,
           py::arg("uid") = py::bytes(""))
      .def_property_readonly("plan", &Solver::plan, py::return_value_policy::reference_internal)
      .def_property_readonly("grid", &Solver::grid, py::return_value_policy::reference_internal)
      .def_property_readonly("config", &Solver::config, py::return_value_policy::reference_internal)
      .def("set_state",
           [](Solver& s, py::array_t<std::complex<double>, py::array::c_style | py::array::forcecast> phi,
              py::array_t<std::complex<double>, py::array::c_style | py::array::forcecast> om,
              py::array_t<double, py::array::c_style | py::array::forcecast> U) {
             const size_t n = s.plan().spec_elems();
             CH_CHECK(static_cast<size_t>(phi.size()) == n && static_cast<size_t>(om.size()) == n,
                         "state arrays must have NY*nkx_loc*nkz_loc elements");
             CH_CHECK(U.size() == s.plan().NY, "U must have NY elements");
             py::gil_scoped_release r;
             s.set_state(phi.data(), om.data(), U.data());
           })
      .def("get_state",
           [](Solver& s) {
             const Plan& p = s.plan();
             py::array_t<std::complex<double>> phi({p.NY, p.nkx_loc, p.nkz_loc}), om({p.NY, p.nkx_loc, p.nkz_loc});
             py::array_t<double> U(p.NY);
             s.get_state(phi.mutable_data(), om.mutable_data(), U.mutable_data());
             return py::make_tuple(phi, om, U);
           })
      .def("init_ic", &Solver::init_ic, py::call_guard<py::gil_scoped_release>())
      .def("prepare", &Solver::prepare, py::call_guard<py::gil_scoped_release>())
      .def("step", &Solver::step, py::arg("stats_for_next") = false, py::call_guard<py::gil_scoped_release>())
      .def("run", &Solver::run, py::arg("nsteps"), py::arg("verbose") = true, py::call_guard<py::gil_scoped_release>())
      .def("synchronize", &Solver::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("log", &Solver::log, py::call_guard<py::gil_scoped_release>())
      .def("stats", [](Solver& s) { return vec(s.stats()); })
      .def("kblocks", &Solver::kblocks)
      .def("bwd_blocks_issued", &Solver::bwd_blocks_issued)
      .def("captured_compute_streams", &Solver::captured_compute_streams)
      .def("spec_kzb", &Solver::spec_kzb)
      .def("combine", &Solver::combine)
      .def("mean_profile", [](Solver& s) { return vec(s.mean_profile()); })
      .def("health", &Solver::health)
      .def("time", &Solver::time)
      .def("steps_done", &Solver::steps_done)
      .def("set_time", &Solver::set_time)
      .def("set_use_graph", &Solver::set_use_graph)
      .def("set_phase_timing", &Solver::set_phase_timing, py::call_guard<py::gil_scoped_release>())
      .def("phase_times_ms", &Solver::phase_times_ms)
      .def("reset_phase_times", &Solver::reset_phase_times)
      .def("set_step_timing", &Solver::set_step_timing)
      .def("step_times_ms", &Solver::step_times_ms, py::call_guard<py::gil_scoped_release>())
      .def("graph_active", &Solver::graph_active)
      .def("comm_kind", &Solver::comm_kind)
      .def("kspec_profile", &Solver::kspec_profile)
      .def("symmetrize", &Solver::symmetrize)
      .def("substep_debug", &Solver::substep_debug, py::call_guard<py::gil_scoped_release>())
      .def("transforms_debug", &Solver::transforms_debug, py::call_guard<py::gil_scoped_release>())
      .def("write_restart", &Solver::write_restart, py::call_guard<py::gil_scoped_release>())
      .def("read_restart", &Solver::read_restart, py::call_guard<py::gil_scoped_release>())
      .def("checkpoint_async", &Solver::checkpoint_async, py::call_guard<py::gil_scoped_release>())
      .def("wait_checkpoint", &Solver::wait_checkpoint, py::call_guard<py::gil_scoped_release>())
      .def("barrier", &Solver::barrier, py::call_guard<py::gil_scoped_release>())
      .def("max_over_ranks", &Solver::max_over_ranks, py::call_guard<py::gil_scoped_release>())
      .def("take_snapshot", &Solver::take_snapshot, py::call_guard<py::gil_scoped_release>())
      .def("rollback", &Solver::rollback, py::call_guard<py::gil_scoped_release>())
      .def("rollbacks", &Solver::rollbacks)
      .def("snapshot_step", &Solver::snapshot_step)
      .def("cfl", &Solver::cfl)
      .def("inject_nan", &Solver::inject_nan, py::arg("field") = 0)
      .def("spectra",
           [](Solver& s) {
             Solver::Spectra sp;
             {
               py::gil_scoped_release r;
               sp = s.spectra();
             }
             const Plan& p = s.plan();
             const int np = static_cast<int>(sp.planes.size());
             auto arr = [](const std::vector<double>& v, std::vector<py::ssize_t> shape) {
               py::array_t<double> a(shape);
               std::copy(v.begin(), v.end(), a.mutable_data());
               return a;
             };
             py::dict d;
             d["planes"] = sp.planes;
             d["ekx"] = arr(sp.ekx, {3, np, p.Kx + 1});
             d["ekz"] = arr(sp.ekz, {3, np, p.nkz});
             d["map"] = arr(sp.map, {3, p.nkx, p.nkz});
             return d;
           },
           "energy spectra of u, v, w of the current state at cfg.spectra_planes (global)");

  py::class_<ProcInfo>(m, "ProcInfo")
      .def(py::init<>())
      .def_static("from_env", &ProcInfo::from_env)
      .def_readwrite("rank", &ProcInfo::rank)
      .def_readwrite("size", &ProcInfo::size)
      .def_readwrite("local_rank", &ProcInfo::local_rank);
  m.def(
      "tcp_broadcast",
      [](const ProcInfo& pi, py::bytes payload, int timeout_s) {
        std::string in = payload;
        std::string out;
        {
          py::gil_scoped_release r;
          out = tcp_broadcast(pi, in, timeout_s);
        }
        return py::bytes(out);
      },
      py::arg("pi"), py::arg("payload"), py::arg("timeout_s") = 300,
      "rank 0's payload on every rank (TCP rendezvous at MASTER_ADDR:MASTER_PORT+11)");
  m.def("device_count", &device_count, "visible HIP devices (does not create a context)");
}
