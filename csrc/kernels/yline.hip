// Wall-normal (y-line) kernels: coefficient tables, the D1 factorisation and a per-operator test
// entry point.  The fused spectral substep kernel (K-SPEC) is in kspec.hip.
//
// K-SPEC fuses, per (kx,kz) line, everything the reference does in y between two FFT rounds
// (SURVEY §7.3 K-SPEC-A/B):
//   calcHvg/calcHvv (nonLinear_kernels.cu:94-190), rk_step_1/2 (RK3_kernels.cu:6-153),
//   implicitSolver_double x2 (implicitStep_nu_double.cu:227-247), bilaplaSolver_double
//   (bilplacSolver_double.cu:320-348: implicit phi, Helmholtz v, D1 v, influence matrix),
//   meanURKstep_1/2 + forcing (meanUevol.c:201-221, 439-567, on the device for line (0,0)),
//   calcUW (nonLinear_kernels.cu:8-92), the wz/wx D1 calls and calcOmega
//   (convolution.c:7-20, convolution_kernels.cu:7-66), calcSt plane sums (statistics.cu:7-95).
// The reference runs these as ~50 launches + 44 cusparse calls + 8 D2D copies per substep with
// float<->double casts through HBM.  Here one launch reads 7 fields and writes 10, all y-work is
// fp64 in registers, and the wall-normal operators are applied in "M-form" (the compact D2 mass
// matrix multiplies the equation), so the explicit viscous term needs no solve at all.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "channel/common.hpp"
#include "channel/kernels.hpp"
#include "channel/yline_device.hpp"
#include "channel/kspec_config.hpp"

namespace channel {

using namespace dev;

int yline_supported_R(int NY) {
  static const int supported[] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 16, 24};
  for (int r : supported)
    if (64 * r >= NY) return r;
  CH_CHECK(false, "NY=" << NY << " too large for the y-line kernels (max 1536)");
}

// ------------------------------------------------------------------------------------------
template <int R>
__global__ void __launch_bounds__(64) d1_factor_kernel(YTab t, double* out) {
  const int lane = __lane_id();
  PFac<R> F;
  CoefD1 cd{t, lane};
  pfactor<R, kXlDpp>(F, cd, Xl<kXlDpp>{}, lane);
  pfac_store<R>(F, out, lane);
}

void YTablesDev::upload(const YGrid& g, int R_, hipStream_t stream) {
  release();
  R = R_;
  const int N = g.N;
  CH_CHECK(64 * R >= N, "R too small for NY");
  const int rows = 64 * R;
  // lane-major reorder: index r*64+lane <- row lane*R + r
  auto lm = [&](const std::vector<double>& v) {
    std::vector<double> o(rows, 0.0);
    for (int lane = 0; lane < 64; ++lane)
      for (int r = 0; r < R; ++r) {
        const int j = lane * R + r;
        o[r * 64 + lane] = j < N ? v[j] : 0.0;
      }
    return o;
  };
  std::vector<double> mask(N, 0.0);
  for (int j = 1; j < N - 1; ++j) mask[j] = 1.0;
  // first and last rows of the dense D1 = A1^-1 B1: row_w = B1^T g, A1^T g = e_w (Thomas on A1^T)
  auto d1_row = [&](int wall) {
    std::vector<double> a(N, 0.0), b(N, 1.0), c(N, 0.0), d(N, 0.0);
    for (int j = 0; j < N; ++j) {
      a[j] = j > 0 ? g.d1_up[j - 1] : 0.0;      // (A1^T)[j][j-1] = A1[j-1][j]
      c[j] = j < N - 1 ? g.d1_lo[j + 1] : 0.0;  // (A1^T)[j][j+1] = A1[j+1][j]
    }
    d[wall] = 1.0;
    std::vector<double> cp(N), dp(N);
    cp[0] = c[0] / b[0];
    dp[0] = d[0] / b[0];
    for (int j = 1; j < N; ++j) {
      const double m = b[j] - a[j] * cp[j - 1];
      cp[j] = c[j] / m;
      dp[j] = (d[j] - a[j] * dp[j - 1]) / m;
    }
    std::vector<double> gv(N);
    gv[N - 1] = dp[N - 1];
    for (int j = N - 2; j >= 0; --j) gv[j] = dp[j] - cp[j] * gv[j + 1];
    std::vector<double> row(N, 0.0);
    for (int i = 1; i < N - 1; ++i) {
      row[i - 1] += gv[i] * g.d1_rm[i];
      row[i] += gv[i] * g.d1_rc[i];
      row[i + 1] += gv[i] * g.d1_rp[i];
    }
    for (int k = 0; k < 3; ++k) {
      row[k] += gv[0] * g.d1_w0[k];
      row[N - 1 - k] += gv[N - 1] * g.d1_wN[k];
    }
    return row;
  };
  // D1 right-hand side B1 with the one-sided wall closures folded into rows 0 and N-1 (their
  // third points w0[2], wN[2] are applied separately, see d1_rhs)
  std::vector<double> rm = g.d1_rm, rc = g.d1_rc, rp = g.d1_rp;
  rc[0] = g.d1_w0[0];
  rp[0] = g.d1_w0[1];
  rc[N - 1] = g.d1_wN[0];
  rm[N - 1] = g.d1_wN[1];
  // order = YTab fields d1_lo .. d1rowN (kYTabRowTables, staged into LDS by K-SPEC), then the D1
  // factorisation, then trap
  std::vector<std::vector<double>> tabs = {lm(g.d1_lo), lm(g.d1_up), lm(rm),    lm(rc),     lm(rp),
                                           lm(g.m_lo),  lm(g.m_up),  lm(g.k_lo), lm(g.k_c),  lm(g.k_up),
                                           lm(mask),    lm(d1_row(0)), lm(d1_row(N - 1))};
  static_assert(kYTabRowTables == 13, "table order");
  int nf = 0;
  CH_DISPATCH_R(R, nf = PFac<R>::kNumFields);
  const size_t nrow = tabs.size() * rows;
  const size_t n = nrow + static_cast<size_t>(nf) * 64 + rows;
  bytes = n * sizeof(double);
  HIP_CHECK(hipMalloc(&buf, bytes));
  std::vector<double> host(n, 0.0);
  for (size_t i = 0; i < tabs.size(); ++i) std::copy(tabs[i].begin(), tabs[i].end(), host.begin() + i * rows);
  {
    const std::vector<double> tr = lm(g.trap);
    std::copy(tr.begin(), tr.end(), host.begin() + nrow + static_cast<size_t>(nf) * 64);
  }
  HIP_CHECK(hipMemcpyAsync(buf, host.data(), bytes, hipMemcpyHostToDevice, stream));
  const double* p = buf;
  tab.d1_lo = p + 0 * rows;
  tab.d1_up = p + 1 * rows;
  tab.d1_rm = p + 2 * rows;
  tab.d1_rc = p + 3 * rows;
  tab.d1_rp = p + 4 * rows;
  tab.m_lo = p + 5 * rows;
  tab.m_up = p + 6 * rows;
  tab.k_lo = p + 7 * rows;
  tab.k_c = p + 8 * rows;
  tab.k_up = p + 9 * rows;
  tab.mask = p + 10 * rows;
  tab.d1row0 = p + 11 * rows;
  tab.d1rowN = p + 12 * rows;
  double* fac = buf + nrow;
  tab.d1fac = fac;
  tab.trap = fac + static_cast<size_t>(nf) * 64;
  for (int i = 0; i < 3; ++i) {
    tab.w0[i] = g.d1_w0[i];
    tab.wN[i] = g.d1_wN[i];
  }
  tab.N = N;
  CH_DISPATCH_R(R, hipLaunchKernelGGL(d1_factor_kernel<R>, dim3(1), dim3(64), 0, stream, tab, fac));
  HIP_LAUNCH_CHECK(stream);
  HIP_CHECK(hipStreamSynchronize(stream));
}

void YTablesDev::release() {
  if (buf) (void)hipFree(buf);
  buf = nullptr;
  bytes = 0;
}

// ------------------------------------------------------------------------------------------
// test kernel: one wave per line, data [y][line] complex, direct global access; the cross-lane
// policy is the one K-SPEC uses at this R (kspec_xmode), so the operator tests cover it
template <int R, typename T>
__global__ void __launch_bounds__(256) yline_test_kernel(YTab t, int op, const void* vin, void* vout, int lines,
                                                         const double* k2s, double c) {
  using T2 = typename Cplx<T>::type;
  constexpr int XM = kspec_xmode<R, T>();
  __shared__ double xs[4][xl_scratch_doubles(4)];
  const T2* in = static_cast<const T2*>(vin);
  T2* out = static_cast<T2*>(vout);
  const int lane = __lane_id();
  const int line = blockIdx.x * 4 + threadIdx.x / 64;
  if (line >= lines) return;  // whole wave exits together
  const Xl<XM> xl{xs[threadIdx.x / 64]};
  const int N = t.N;
  double x[2][R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int j = lane * R + r;
    T2 v = j < N ? in[static_cast<size_t>(j) * lines + line] : T2{0, 0};
    x[0][r] = j < N ? static_cast<double>(v.x) : 0.0;
    x[1][r] = j < N ? static_cast<double>(v.y) : 0.0;
  }
  const double k2 = k2s ? k2s[line] : 0.0;
  double m[2][R];
  if (op == YOP_D1) {
    d1_apply_to<R, 2, XM>(t, x, m, xl, lane);
  } else if (op == YOP_HELM) {
    apply_M<R, 2, XM>(t, x, m, lane);
    PFac<R> F;
    CoefHelm ch{t, lane, k2};
    pfactor<R, XM>(F, ch, xl, lane);
    psolve<R, 2, XM>(F, ch, m, xl, lane);
  } else if (op == YOP_IMPL) {
    apply_M<R, 2, XM>(t, x, m, lane);
    PFac<R> F;
    CoefImpl ci{t, lane, 1.0 + c * k2, c};
    pfactor<R, XM>(F, ci, xl, lane);
    psolve<R, 2, XM>(F, ci, m, xl, lane);
  } else if (op == YOP_MAPPLY) {
    apply_M<R, 2, XM>(t, x, m, lane);
  } else {
    apply_K<R, 2, XM>(t, x, m, lane);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int j = lane * R + r;
    if (j < N) out[static_cast<size_t>(j) * lines + line] = T2{static_cast<T>(m[0][r]), static_cast<T>(m[1][r])};
  }
}

void yline_test(const YTablesDev& t, int op, const void* in, void* out, int lines, const double* k2, double c,
                bool fp64, hipStream_t stream) {
  dim3 grid((lines + 3) / 4), block(256);
  if (fp64) {
    CH_DISPATCH_R(t.R, hipLaunchKernelGGL((yline_test_kernel<R, double>), grid, block, 0, stream, t.tab, op, in, out,
                                          lines, k2, c));
  } else {
    CH_DISPATCH_R(t.R, hipLaunchKernelGGL((yline_test_kernel<R, float>), grid, block, 0, stream, t.tab, op, in, out,
                                          lines, k2, c));
  }
  HIP_LAUNCH_CHECK(stream);
}

}  // namespace channel
