// PyTorch-ROCm bindings of the native core (channel_gpu_amd._C).
// Every kernel is exposed individually (taking torch tensors on the current HIP stream) so the
// tests can check it against a NumPy/PyTorch fp64 reference of the same operator.  Everything
// that needs no tensors lives in the torch-free module _core (core_module.cpp) and is re-exported
// here, so `_C.Solver is _core.Solver` (one pybind11 type registry: both modules are built
// against the same pybind11 headers).
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

// y-line operator tables for a given grid (test entry)
struct YLineOps {
  YGrid grid;
  YTablesDev tab;
  YLineOps(int NY, double stretch, int halves) : grid(YGrid::build(NY, stretch)) {
    // halves = 2: lines over two waves of R = 4 (K-SPEC's geometry for 258 < NY <= 512)
    tab.upload(grid, halves == 2 ? 4 : yline_supported_R(NY), cur_stream(), halves);
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
  // the dense-D1 MFMA kernel (complex128 only)
  DenseD1Dev dense;
  torch::Tensor d1_mfma(torch::Tensor in) {
    check_dev_tensor(in, "in");
    TORCH_CHECK(is_fp64_complex(in), "d1_mfma: complex128 input");
    TORCH_CHECK(in.dim() == 2 && in.size(0) == grid.N, "in must be [NY, lines]");
    if (!dense.d) dense.upload(grid, cur_stream());
    auto out = torch::zeros_like(in);
    d1_dense_mfma(dense, in.data_ptr(), out.data_ptr(), static_cast<int>(in.size(1)), cur_stream());
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
// combine = 1: spec holds the five K-SPEC outputs (D1 v, v, D1 omega, omega, phi) and the six
// physical-stage fields u, v, w, omega_x, omega_y, omega_z are formed per element (XArgs::combine;
// ax, az = 2 pi / LX, 2 pi / LZ, kz0 = global kz of local kz 0)
void set_combine(XArgs& a, XSrc& s, const char* base, long long fstride, size_t esz, int combine, double ax, double az,
                 int kz0) {
  a.combine = combine;
  a.ax = ax;
  a.az = az;
  a.kz_glob0 = kz0;
  if (combine) {
    a.nfields = 6;
    for (int j = 0; j < 5; ++j) s.fld[j] = base + static_cast<size_t>(j) * fstride * esz;
  }
}

torch::Tensor xfft_b(torch::Tensor spec, int NX, int Kx, int combine, double ax, double az, int kz0) {
  check_dev_tensor(spec, "spec");
  const bool f64 = is_fp64_complex(spec);
  TORCH_CHECK(spec.dim() == 4, "spec must be [F, ny, nkx, nkz]");
  const int F = spec.size(0), ny = spec.size(1), nkx = spec.size(2), nkz = spec.size(3);
  TORCH_CHECK(nkx == 2 * Kx + 1, "nkx != 2Kx+1");
  TORCH_CHECK(!combine || F == 5, "combine mode: five input fields");
  auto phys = torch::zeros({combine ? 6 : F, ny, NX, nkz}, spec.options());
  XArgs a;
  a.NX = NX; a.nkx = nkx; a.Kx = Kx; a.nkz = nkz; a.ny = ny; a.nfields = F;
  a.field_stride_spec = static_cast<long long>(ny) * nkx * nkz;
  a.field_stride_phys = static_cast<long long>(ny) * NX * nkz;
  XSrc s;
  s.base = spec.data_ptr();
  s.nsrc = 1;
  s.kx_start[0] = 0;
  s.kx_start[1] = nkx;
  set_combine(a, s, static_cast<const char*>(spec.data_ptr()), a.field_stride_spec, spec.element_size(), combine, ax, az, kz0);
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

// x transforms on the one-rank blocked spectral layout (spec_index, kzb = 8; tests): the variants the
// headline grid runs -- plane tiles (fp32 NX = 512 / 1024), 16-byte accesses (even nkz),
// non-temporal spectral accesses (nt) -- on planes y0 .. y0 + ny - 1 of F fields of `rows` planes.
// specb: 1-D complex buffer of F * spec_rows(rows) * nkx * nkzs elements (nkzs = nkz rounded up to 8)
torch::Tensor xfft_b_blocked(torch::Tensor specb, int F, int rows, int y0, int ny, int NX, int Kx, int nkz, int nt,
                             int zero_mean_field, int combine, double ax, double az) {
  check_dev_tensor(specb, "specb");
  const bool f64 = is_fp64_complex(specb);
  const int nkx = 2 * Kx + 1, nkzs = (nkz + kSpecKzBlock - 1) / kSpecKzBlock * kSpecKzBlock;
  const long long fstride = static_cast<long long>(spec_rows(kSpecKzBlock, rows)) * nkx * nkzs;
  TORCH_CHECK(specb.dim() == 1 && specb.numel() == F * fstride, "specb must hold F blocked fields");
  TORCH_CHECK(y0 >= 0 && ny > 0 && y0 + ny <= rows, "plane range outside the fields");
  TORCH_CHECK(!combine || F == 5, "combine mode: five input fields");
  auto phys = torch::zeros({combine ? 6 : F, ny, NX, nkz}, specb.options());
  XArgs a;
  a.NX = NX; a.nkx = nkx; a.Kx = Kx; a.nkz = nkz; a.ny = ny; a.nfields = F;
  a.field_stride_spec = fstride;
  a.field_stride_phys = static_cast<long long>(ny) * NX * nkz;
  a.kzb = kSpecKzBlock; a.nkzs = nkzs; a.spec_y0 = y0; a.nt = nt;
  a.zero_mean_field = zero_mean_field;
  XSrc s;
  s.base = specb.data_ptr();
  s.nsrc = 1;
  s.kx_start[0] = 0;
  s.kx_start[1] = nkx;
  set_combine(a, s, static_cast<const char*>(specb.data_ptr()), fstride, specb.element_size(), combine, ax, az, 0);
  xfft_backward(a, s, phys.data_ptr(), twiddles(NX, f64), f64, cur_stream());
  return phys;
}

// forward counterpart: phys [F, ny, NX, nkz] -> planes y0 .. y0 + ny - 1 of specb (updated in place)
torch::Tensor xfft_f_blocked(torch::Tensor phys, torch::Tensor specb, int rows, int y0, int Kx, int nt) {
  check_dev_tensor(phys, "phys");
  check_dev_tensor(specb, "specb");
  const bool f64 = is_fp64_complex(phys);
  TORCH_CHECK(phys.dim() == 4, "phys must be [F, ny, NX, nkz]");
  const int F = phys.size(0), ny = phys.size(1), NX = phys.size(2), nkz = phys.size(3);
  const int nkx = 2 * Kx + 1, nkzs = (nkz + kSpecKzBlock - 1) / kSpecKzBlock * kSpecKzBlock;
  const long long fstride = static_cast<long long>(spec_rows(kSpecKzBlock, rows)) * nkx * nkzs;
  TORCH_CHECK(specb.dim() == 1 && specb.numel() == F * fstride && is_fp64_complex(specb) == f64, "specb mismatch");
  TORCH_CHECK(y0 >= 0 && y0 + ny <= rows, "plane range outside the fields");
  XArgs a;
  a.NX = NX; a.nkx = nkx; a.Kx = Kx; a.nkz = nkz; a.ny = ny; a.nfields = F;
  a.field_stride_spec = fstride;
  a.field_stride_phys = static_cast<long long>(ny) * NX * nkz;
  a.kzb = kSpecKzBlock; a.nkzs = nkzs; a.spec_y0 = y0; a.nt = nt;
  XDst d;
  d.base = specb.data_ptr();
  d.ndst = 1;
  d.kx_start[0] = 0;
  d.kx_start[1] = nkx;
  xfft_forward(a, phys.data_ptr(), d, twiddles(NX, f64), f64, cur_stream());
  return specb;
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

torch::Tensor field_tensor(Solver& s, int f) {
  const Plan& p = s.plan();
  // a [y][kx][kz] view only exists for the plain layout (kx sub-blocks: use get_state)
  CH_CHECK(s.kblocks() == 1, "field(): the spectral fields are stored as " << s.kblocks() << " kx sub-blocks");
  CH_CHECK(s.spec_kzb() == 0, "field(): the spectral fields are blocked by kz lines (use get_state)");
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
  m.doc() = "channel_gpu_amd native core (gfx950 HIP kernels, RCCL, HDF5 I/O) with torch tensor entry points";
  py::module_ core = py::module_::import("channel_gpu_amd._core");
  for (auto item : core.attr("__dict__").cast<py::dict>()) {
    const std::string k = py::str(item.first);
    if (k.rfind("__", 0) == 0) continue;
    m.attr(item.first) = item.second;
  }

  py::class_<YLineOps>(m, "YLineOps")
      .def(py::init<int, double, int>(), py::arg("NY"), py::arg("stretch") = 2.0, py::arg("halves") = 1)
      .def("apply", &YLineOps::apply, py::arg("op"), py::arg("x"), py::arg("k2") = py::none(), py::arg("c") = 0.0)
      .def("d1_mfma", &YLineOps::d1_mfma, py::arg("x"));

  m.def("fft_c2c", &fft_c2c, "batched in-LDS C2C FFT along the last axis; dir=+1 inverse (unnormalised)");
  m.def("xfft_backward", &xfft_b, py::arg("spec"), py::arg("NX"), py::arg("Kx"), py::arg("combine") = 0,
        py::arg("ax") = 1.0, py::arg("az") = 2.0, py::arg("kz0") = 0);
  m.def("xfft_forward", &xfft_f);
  m.def("xfft_backward_blocked", &xfft_b_blocked, py::arg("specb"), py::arg("F"), py::arg("rows"), py::arg("y0"),
        py::arg("ny"), py::arg("NX"), py::arg("Kx"), py::arg("nkz"), py::arg("nt") = 0, py::arg("zero_mean_field") = -1,
        py::arg("combine") = 0, py::arg("ax") = 1.0, py::arg("az") = 2.0);
  m.def("xfft_forward_blocked", &xfft_f_blocked, py::arg("phys"), py::arg("specb"), py::arg("rows"), py::arg("y0"),
        py::arg("Kx"), py::arg("nt") = 0);
  m.def("zphys", &zphys_op);
  m.def("xfft_last_variant", [] { return xfft_last_variant(); },
        "template arguments of the last x-transform launch (rocprofv3 kernel-name form)");
  m.def("xfft_last_backward_variant", [] { return xfft_last_backward_variant(); },
        "template arguments of the last x-backward launch (rocprofv3 kernel-name form)");

  // tensor views of a Solver's device buffers, attached to the _core Solver class
  py::object cls = core.attr("Solver");
  cls.attr("field") = py::cpp_function(&field_tensor, py::name("field"), py::is_method(cls),
                                       "zero-copy torch view of a device field [NY, nkx_loc, nkz]");
  cls.attr("phys") = py::cpp_function(&phys_tensor, py::name("phys"), py::is_method(cls),
                                      "zero-copy torch view of the physical-stage buffer [6, ny_loc, NX, nkz]");
}
