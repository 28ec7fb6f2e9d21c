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
#include <cstdlib>
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

void kspec_geometry(int NY, bool fp64, int& R, int& H) {
  // opt-in (CHANNEL_KSPEC_HALVES=1): measured slower than one wave per line at 1024x385x1024
  // (6.85 vs 4.2 ms per K-SPEC; profiles/r04/README.md); solver-level oracle test:
  // tests/test_solver_gpu.py::test_kspec_halves_matches_oracle
  // (read per Solver: a test process can construct solvers with and without it)
  const char* e = std::getenv("CHANNEL_KSPEC_HALVES");
  const bool on = e && std::atoi(e) == 1;
  // two waves of R = 4 per line where one wave would need R = 5..8 (one wave per SIMD at more
  // than 256 registers); rows N-3 .. N-1 must share a half (the D1 wall closure)
  if (on && !fp64 && NY > 256 + 2 && NY <= 512) {
    R = 4;
    H = 2;
    return;
  }
  R = yline_supported_R(NY);
  H = 1;
}

// ------------------------------------------------------------------------------------------
// the constant D1 factorisation (per half for two-wave lines, with the halves' coupling dropped)
// and, for two halves, each half's spike (response to its coupling coefficient)
template <int R, int H>
__global__ void __launch_bounds__(64 * H) d1_factor_kernel(YTab t, double* out, double* spk) {
  const int lane = __lane_id(), h = threadIdx.x / 64;
  YTab th = t;
  th.d1_lo = t.d1_lo + h * R * 64;
  th.d1_up = t.d1_up + h * R * 64;
  PFac<R> F;
  const CoefD1 cd{th, lane};
  const CutLo<CoefD1> cc{cd, H == 2 && h == 1 && lane == 0};
  pfactor<R, kXlDpp>(F, cc, Xl<kXlDpp>{}, lane);
  pfac_store<R>(F, out + h * PFac<R>::kNumFields * 64, lane);
  if constexpr (H == 2) {
    double z[1][R];
    LineG<2> gh;
    gh.h = h;
    spike_rhs<R>(z[0], cd, gh, lane);
    psolve<R, 1, kXlDpp>(F, cd, z, Xl<kXlDpp>{}, lane);
#pragma unroll
    for (int r = 0; r < R; ++r) spk[(h * R + r) * 64 + lane] = z[0][r];
  }
}

void YTablesDev::upload(const YGrid& g, int R_, hipStream_t stream, int H_) {
  release();
  R = R_;
  H = H_;
  const int N = g.N;
  CH_CHECK(H == 1 || H == 2, "lines over 1 or 2 waves");
  CH_CHECK(64 * R * H >= N, "R too small for NY");
  CH_CHECK(H == 1 || (N > 64 * R + 2 && R == 4), "two-wave lines: R = 4 and rows N-3 .. N-1 in the second half");
  const int rows = 64 * R * H, HR = 64 * R;
  // lane-major reorder: index (h R + r) 64 + lane <- row h HR + lane R + r
  auto lm = [&](const std::vector<double>& v) {
    std::vector<double> o(rows, 0.0);
    for (int h = 0; h < H; ++h)
      for (int lane = 0; lane < 64; ++lane)
        for (int r = 0; r < R; ++r) {
          const int j = h * HR + lane * R + r;
          o[(h * R + r) * 64 + lane] = j < N ? v[j] : 0.0;
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
  // [13 row tables][D1 factorisation per half][D1 spikes (two halves)][trap]
  const size_t nrow = tabs.size() * rows;
  const size_t nfac = static_cast<size_t>(nf) * 64 * H, nspk = H == 2 ? rows : 0;
  const size_t n = nrow + nfac + nspk + rows;
  bytes = n * sizeof(double);
  HIP_CHECK(hipMalloc(&buf, bytes));
  std::vector<double> host(n, 0.0);
  for (size_t i = 0; i < tabs.size(); ++i) std::copy(tabs[i].begin(), tabs[i].end(), host.begin() + i * rows);
  {
    const std::vector<double> tr = lm(g.trap);
    std::copy(tr.begin(), tr.end(), host.begin() + nrow + nfac + nspk);
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
  tab.d1spk = H == 2 ? fac + nfac : nullptr;
  tab.trap = fac + nfac + nspk;
  for (int i = 0; i < 3; ++i) {
    tab.w0[i] = g.d1_w0[i];
    tab.wN[i] = g.d1_wN[i];
  }
  tab.N = N;
  if (H == 2) {
    hipLaunchKernelGGL((d1_factor_kernel<4, 2>), dim3(1), dim3(128), 0, stream, tab, fac, fac + nfac);
  } else {
    CH_DISPATCH_R(R, hipLaunchKernelGGL((d1_factor_kernel<R, 1>), dim3(1), dim3(64), 0, stream, tab, fac, nullptr));
  }
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

// the same operators on lines over two waves (K-SPEC's H = 2 geometry): one line per workgroup,
// wave h holding rows h 64R + lane R + r
template <int R, typename T>
__global__ void __launch_bounds__(128) yline_test2_kernel(YTab t, int op, const void* vin, void* vout, int lines,
                                                          const double* k2s, double c) {
  using T2 = typename Cplx<T>::type;
  constexpr int XM = kspec_xmode<R, T>();
  __shared__ double xs[2][xl_scratch_doubles(4)];
  __shared__ double lxb[4 * LineG<2>::kXK];
  __shared__ int lxf[2];
  const T2* in = static_cast<const T2*>(vin);
  T2* out = static_cast<T2*>(vout);
  const int lane = __lane_id(), h = threadIdx.x / 64;
  const int line = blockIdx.x;
  if (threadIdx.x < 2) lxf[threadIdx.x] = 0;
  __syncthreads();
  LineG<2> g;
  g.h = h;
  g.buf = lxb;
  g.flag = lxf;
  const Xl<XM> xl{xs[h]};
  const int N = t.N, off = h * R * 64;
  YTab th = t;
  for (const double** p : {&th.d1_lo, &th.d1_up, &th.d1_rm, &th.d1_rc, &th.d1_rp, &th.m_lo, &th.m_up, &th.k_lo, &th.k_c,
                           &th.k_up, &th.mask, &th.d1row0, &th.d1rowN, &th.trap, &th.d1spk})
    *p += off;
  th.d1fac = t.d1fac + h * PFac<R>::kNumFields * 64;
  double x[2][R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int j = h * 64 * R + lane * R + r;
    T2 v = j < N ? in[static_cast<size_t>(j) * lines + line] : T2{0, 0};
    x[0][r] = j < N ? static_cast<double>(v.x) : 0.0;
    x[1][r] = j < N ? static_cast<double>(v.y) : 0.0;
  }
  const double k2 = k2s ? k2s[line] : 0.0;
  double m[3][R];  // two right-hand sides + the half's spike
  auto& m2 = reinterpret_cast<double (&)[2][R]>(m);
  if (op == YOP_D1) {
    d1_apply_to<R, 2, XM>(th, x, m2, xl, lane, g);
  } else if (op == YOP_HELM || op == YOP_IMPL) {
    apply_M<R, 2, XM>(th, x, m2, lane, g);
    PFac<R> F;
    if (op == YOP_HELM) {
      const CoefHelm ch{th, lane, k2};
      pfactor<R, XM>(F, CutLo<CoefHelm>{ch, h == 1 && lane == 0}, xl, lane);
      spike_rhs<R>(m[2], ch, g, lane);
      psolve<R, 3, XM>(F, ch, m, xl, lane);
    } else {
      const CoefImpl ci{th, lane, 1.0 + c * k2, c};
      pfactor<R, XM>(F, CutLo<CoefImpl>{ci, h == 1 && lane == 0}, xl, lane);
      spike_rhs<R>(m[2], ci, g, lane);
      psolve<R, 3, XM>(F, ci, m, xl, lane);
    }
    spike_join<R, 2, 3>(m, m[2], g, lane);
  } else if (op == YOP_MAPPLY) {
    apply_M<R, 2, XM>(th, x, m2, lane, g);
  } else {
    apply_K<R, 2, XM>(th, x, m2, lane, g);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int j = h * 64 * R + lane * R + r;
    if (j < N) out[static_cast<size_t>(j) * lines + line] = T2{static_cast<T>(m[0][r]), static_cast<T>(m[1][r])};
  }
}

void yline_test(const YTablesDev& t, int op, const void* in, void* out, int lines, const double* k2, double c,
                bool fp64, hipStream_t stream) {
  if (t.H == 2) {
    CH_CHECK(t.R == 4, "two-wave lines: R = 4");
    if (fp64)
      hipLaunchKernelGGL((yline_test2_kernel<4, double>), dim3(lines), dim3(128), 0, stream, t.tab, op, in, out, lines, k2, c);
    else
      hipLaunchKernelGGL((yline_test2_kernel<4, float>), dim3(lines), dim3(128), 0, stream, t.tab, op, in, out, lines, k2, c);
    HIP_LAUNCH_CHECK(stream);
    return;
  }
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
