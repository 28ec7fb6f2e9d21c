// PyTorch-ROCm bindings of the native core (channel_gpu_amd._C).
// Every kernel is exposed individually (taking torch tensors on the current HIP stream) so the
// tests can check it against a NumPy/PyTorch fp64 reference of the same operator.
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPStream.h>
#include <pybind11/complex.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

#include <complex>
#include <map>
#include <memory>

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

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_dev_tensor(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

bool is_fp64_complex(const torch::Tensor& t) {
  TORCH_CHECK(t.scalar_type() == torch::kComplexFloat || t.scalar_type() == torch::kComplexDouble,
              "expected complex64/complex128 tensor");
  return t.scalar_type() == torch::kComplexDouble;
}

py::array_t<double> vec(const std::vector<double>& v) {
  py::array_t<double> a(v.size());
  std::copy(v.begin(), v.end(), a.mutable_data());
  return a;
}

// y-line operator tables for a given grid (test entry)
struct YLineOps {
  YGrid grid;
  YTablesDev tab;
  YLineOps(int NY, double stretch) : grid(YGrid::build(NY, stretch)) {
    tab.upload(grid, yline_supported_R(NY), cur_stream());
  }
  torch::Tensor apply(int op, torch::Tensor in, py::object k2, double c) {
    check_dev_tensor(in, "in");
    const bool f64 = is_fp64_complex(in);
    TORCH_CHECK(in.dim() == 2 && in.size(0) == grid.N, "in must be [NY, lines]");
    const int lines = static_cast<int>(in.size(1));
    auto out = torch::zeros_like(in);
    torch::Tensor k2t;
    const double* k2p = nullptr;
    if (!k2.is_none()) {
      k2t = k2.cast<torch::Tensor>().to(in.device(), torch::kFloat64).contiguous();
      TORCH_CHECK(k2t.numel() == lines, "k2 must have one entry per line");
      k2p = k2t.data_ptr<double>();
    }
    yline_test(tab, op, in.data_ptr(), out.data_ptr(), lines, k2p, c, f64, cur_stream());
    return out;
  }
};

std::map<std::pair<int, bool>, std::unique_ptr<Twiddles>>& tw_cache() {
  static std::map<std::pair<int, bool>, std::unique_ptr<Twiddles>> c;
  return c;
}
const Twiddles& twiddles(int n, bool f64) {
  auto& c = tw_cache();
  auto key = std::make_pair(n, f64);
  auto it = c.find(key);
  if (it == c.end()) {
    auto t = std::make_unique<Twiddles>();
    t->build(n, f64);
    it = c.emplace(key, std::move(t)).first;
  }
  return *it->second;
}

torch::Tensor fft_c2c(torch::Tensor x, int dir) {
  check_dev_tensor(x, "x");
  const bool f64 = is_fp64_complex(x);
  auto y = x.clone();
  const int n = static_cast<int>(x.size(-1));
  const int batch = static_cast<int>(x.numel() / n);
  fft_c2c_test(y.data_ptr(), n, batch, dir, twiddles(n, f64), f64, cur_stream());
  return y;
}

// x-direction backward/forward transforms on a single-rank layout (tests)
torch::Tensor xfft_b(torch::Tensor spec, int NX, int Kx) {
  check_dev_tensor(spec, "spec");
  const bool f64 = is_fp64_complex(spec);
  TORCH_CHECK(spec.dim() == 4, "spec must be [F, ny, nkx, nkz]");
  const int F = spec.size(0), ny = spec.size(1), nkx = spec.size(2), nkz = spec.size(3);
  TORCH_CHECK(nkx == 2 * Kx + 1, "nkx != 2Kx+1");
  auto phys = torch::zeros({F, ny, NX, nkz}, spec.options());
  XArgs a;
  a.NX = NX; a.nkx = nkx; a.Kx = Kx; a.nkz = nkz; a.ny = ny; a.nfields = F;
  a.field_stride_spec = static_cast<long long>(ny) * nkx * nkz;
  a.field_stride_phys = static_cast<long long>(ny) * NX * nkz;
  XSrc s;
  s.base = spec.data_ptr();
  s.nsrc = 1;
  s.kx_start[0] = 0;
  s.kx_start[1] = nkx;
  xfft_backward(a, s, phys.data_ptr(), twiddles(NX, f64), f64, cur_stream());
  return phys;
}

torch::Tensor xfft_f(torch::Tensor phys, int Kx) {
  check_dev_tensor(phys, "phys");
  const bool f64 = is_fp64_complex(phys);
  TORCH_CHECK(phys.dim() == 4, "phys must be [F, ny, NX, nkz]");
  const int F = phys.size(0), ny = phys.size(1), NX = phys.size(2), nkz = phys.size(3);
  const int nkx = 2 * Kx + 1;
  auto spec = torch::zeros({F, ny, nkx, nkz}, phys.options());
  XArgs a;
  a.NX = NX; a.nkx = nkx; a.Kx = Kx; a.nkz = nkz; a.ny = ny; a.nfields = F;
  a.field_stride_spec = static_cast<long long>(ny) * nkx * nkz;
  a.field_stride_phys = static_cast<long long>(ny) * NX * nkz;
  XDst d;
  d.base = spec.data_ptr();
  d.ndst = 1;
  d.kx_start[0] = 0;
  d.kx_start[1] = nkx;
  xfft_forward(a, phys.data_ptr(), d, twiddles(NX, f64), f64, cur_stream());
  return spec;
}

// z physical stage (tests): fields [6, ny, NX, nkz] -> H [3, ny, NX, nkz], maxima [4]
std::pair<torch::Tensor, torch::Tensor> zphys_op(torch::Tensor fields, int Nzp, torch::Tensor inv_dy, double cx, double cz) {
  check_dev_tensor(fields, "fields");
  const bool f64 = is_fp64_complex(fields);
  TORCH_CHECK(fields.dim() == 4 && fields.size(0) == 6, "fields must be [6, ny, NX, nkz]");
  auto f = fields.clone();
  const int ny = f.size(1), NX = f.size(2), nkz = f.size(3);
  auto maxima = torch::zeros({4}, fields.options().dtype(torch::kFloat32));
  auto idy = inv_dy.to(fields.device(), torch::kFloat64).contiguous();
  ZArgs a;
  a.NX = NX; a.Nzp = Nzp; a.nkz = nkz; a.ny = ny; a.y0 = 0;
  a.field_stride = static_cast<long long>(ny) * NX * nkz;
  a.scale = 1.0 / (static_cast<double>(NX) * Nzp);
  a.inv_dy = idy.data_ptr<double>();
  a.cx = cx; a.cz = cz;
  a.maxima = maxima.data_ptr<float>();
  zphys(a, f.data_ptr(), twiddles(Nzp, f64), f64, cur_stream());
  return {f.narrow(0, 0, 3).contiguous(), maxima};
}

py::bytes new_uid() { return py::bytes(Comm::new_unique_id()); }

torch::Tensor field_tensor(Solver& s, int f) {
  const Plan& p = s.plan();
  auto opts = torch::TensorOptions()
                  .dtype(s.fp64() ? torch::kComplexDouble : torch::kComplexFloat)
                  .device(torch::kCUDA, c10::hip::current_device());
  return torch::from_blob(s.field_ptr(f), {p.NY, p.nkx_loc, p.nkz_loc}, opts);
}

torch::Tensor phys_tensor(Solver& s) {
  const Plan& p = s.plan();
  auto opts = torch::TensorOptions()
                  .dtype(s.fp64() ? torch::kComplexDouble : torch::kComplexFloat)
                  .device(torch::kCUDA, c10::hip::current_device());
  return torch::from_blob(s.phys_ptr(), {6, p.ny_loc, p.NX, p.nkz_loc}, opts);
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "channel_gpu_amd native core (gfx950 HIP kernels, RCCL, HDF5 I/O)";
  py::register_exception<channel::Error>(m, "ChannelError", PyExc_RuntimeError);

  py::class_<Config>(m, "Config")
      .def(py::init<>())
      .def_static("from_file", &Config::from_file, py::arg("path"), py::arg("overrides") = std::vector<std::string>())
      .def_static("from_string",
                  [](const std::string& text, const std::vector<std::string>& overrides) {
                    ConfigTree t = ConfigTree::parse_string(text);
                    for (const auto& o : overrides) {
                      auto eq = o.find('=');
                      TORCH_CHECK(eq != std::string::npos, "override must be key=value");
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
      RW(ic) RW(ic_amplitude) RW(forcing) RW(health_check) RW(health_every) RW(on_nan) RW(snapshot_every)
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

  py::class_<YLineOps>(m, "YLineOps")
      .def(py::init<int, double>(), py::arg("NY"), py::arg("stretch") = 2.0)
      .def("apply", &YLineOps::apply, py::arg("op"), py::arg("x"), py::arg("k2") = py::none(), py::arg("c") = 0.0);

  m.def("fft_c2c", &fft_c2c, "batched in-LDS C2C FFT along the last axis; dir=+1 inverse (unnormalised)");
  m.def("xfft_backward", &xfft_b);
  m.def("xfft_forward", &xfft_f);
  m.def("zphys", &zphys_op);
  m.def("new_unique_id", &new_uid);
  m.def("hdf5_available", &hdf5_available);
  m.def("set_debug_sync", &set_debug_sync);
  m.def("h5_create_field", &h5_create_field);
  m.def("h5_write_planes", &h5_write_planes);
  m.def("h5_read_planes", [](const std::string& p, const std::vector<int>& planes) {
    std::vector<double> d;
    int dims[3];
    h5_read_planes(p, planes, d, dims);
    return std::make_pair(vec(d), std::vector<int>(dims, dims + 3));
  });
  m.def("h5_write_attrs", &h5_write_attrs);
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
             TORCH_CHECK(static_cast<size_t>(phi.size()) == n && static_cast<size_t>(om.size()) == n,
                         "state arrays must have NY*nkx_loc*nkz_loc elements");
             TORCH_CHECK(U.size() == s.plan().NY, "U must have NY elements");
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
      .def("barrier", &Solver::barrier, py::call_guard<py::gil_scoped_release>())
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
           "energy spectra of u, v, w of the current state at cfg.spectra_planes (global)")
      .def("field", &field_tensor, "zero-copy torch view of a device field [NY, nkx_loc, nkz]")
      .def("phys", &phys_tensor, "zero-copy torch view of the physical-stage buffer [6, ny_loc, NX, nkz]");
}
