#include "channel/grid.hpp"

#include <cmath>

#include "channel/common.hpp"

namespace channel {

YGrid YGrid::build(int N, double stretch) {
  CH_CHECK(N >= 5, "NY must be >= 5");
  YGrid g;
  g.N = N;
  g.stretch = stretch;
  g.y.resize(N);
  const double dy = 2.0 / (N - 1);
  const double ts = std::tanh(stretch);
  for (int j = 0; j < N; ++j) g.y[j] = std::tanh(stretch * (j * dy - 1.0)) / ts;
  g.y[0] = -1.0;
  g.y[N - 1] = 1.0;
  const auto& y = g.y;

  g.d1_lo.assign(N, 0.0); g.d1_up.assign(N, 0.0);
  g.d1_rm.assign(N, 0.0); g.d1_rc.assign(N, 0.0); g.d1_rp.assign(N, 0.0);
  g.m_lo.assign(N, 0.0); g.m_up.assign(N, 0.0);
  g.k_lo.assign(N, 0.0); g.k_c.assign(N, 0.0); g.k_up.assign(N, 0.0);
  g.trap.assign(N, 0.0);

  for (int j = 1; j < N - 1; ++j) {
    const double a = y[j + 1] - y[j];  // > 0
    const double b = y[j - 1] - y[j];  // < 0
    // compact D1 (derivatives_nu_double.cu:60-65, 227-232)
    const double amb2 = (a - b) * (a - b);
    g.d1_up[j] = b * b / amb2;
    g.d1_lo[j] = a * a / amb2;
    const double A1 = 2.0 * (2.0 * a * b * b - b * b * b) / ((a * a - a * b) * amb2);
    const double B1 = 2.0 * (2.0 * b * a * a - a * a * a) / ((b * b - a * b) * amb2);
    g.d1_rp[j] = A1;
    g.d1_rm[j] = B1;
    g.d1_rc[j] = -A1 - B1;
    // compact D2 (hemholzt_nu_double.cu:58-62, 136-145)
    const double den = a * a * a - b * b * b - 4.0 * a * a * b + 4.0 * b * b * a;
    const double A2 = -12.0 * b / den;
    const double B2 = 12.0 * a / den;
    const double den2 = a * a * a - 4.0 * a * a * b + 4.0 * a * b * b - b * b * b;
    g.m_up[j] = -(-b * b * b - a * b * b + a * a * b) / den2;
    g.m_lo[j] = -(a * a * a + b * a * a - b * b * a) / den2;
    g.k_up[j] = A2;
    g.k_lo[j] = B2;
    g.k_c[j] = -A2 - B2;
  }
  // D1 wall closure (derivatives_nu_double.cu:85-112 RHS, 247-274 LHS)
  {
    double a = y[1] - y[0], b = y[2] - y[1];
    g.d1_up[0] = (a + b) / b;
    g.d1_w0[0] = -(3.0 * a + 2.0 * b) / (a * a + a * b);
    g.d1_w0[1] = ((a + b) * (2.0 * b - a)) / (a * b * b);
    g.d1_w0[2] = a * a / (b * b * a + b * b * b);
    a = y[N - 2] - y[N - 1];
    b = y[N - 3] - y[N - 2];
    g.d1_lo[N - 1] = (a + b) / b;
    g.d1_wN[0] = -(3.0 * a + 2.0 * b) / (a * a + a * b);
    g.d1_wN[1] = ((a + b) * (2.0 * b - a)) / (a * b * b);
    g.d1_wN[2] = a * a / (b * b * a + b * b * b);
  }
  // D2 wall closure (meanUevol.c:254-274, 301-329)
  {
    double a = y[1] - y[0], b = y[2] - y[0];
    g.d2_w0_up = (a + b) / (2.0 * a - b);
    double A = 6.0 / ((a - b) * (2.0 * a - b));
    double B = -6.0 * a / ((a * b - b * b) * (2.0 * a - b));
    g.d2_w0[0] = -A - B; g.d2_w0[1] = A; g.d2_w0[2] = B;
    a = y[N - 2] - y[N - 1];
    b = y[N - 3] - y[N - 1];
    g.d2_wN_lo = (a + b) / (2.0 * a - b);
    A = 6.0 / ((a - b) * (2.0 * a - b));
    B = -6.0 * a / ((a * b - b * b) * (2.0 * a - b));
    g.d2_wN[0] = -A - B; g.d2_wN[1] = A; g.d2_wN[2] = B;
  }
  // Flux quadrature: on each interval [y_j, y_{j+1}] integrate the cubic Lagrange interpolant
  // through 4 neighbouring points (shifted at the walls) with 2-point Gauss-Legendre (exact for
  // cubics).  4th-order accurate and exact for the laminar parabola, so the constant-flux
  // constraint does not bias U (the reference used a trapezoid starting at j=10).
  for (int j = 0; j < N - 1; ++j) {
    int s = j - 1;
    if (s < 0) s = 0;
    if (s + 3 > N - 1) s = N - 4;
    const double a = y[j], b = y[j + 1];
    const double gq[2] = {0.5 * (a + b) - 0.5 * (b - a) / std::sqrt(3.0), 0.5 * (a + b) + 0.5 * (b - a) / std::sqrt(3.0)};
    for (int q = 0; q < 2; ++q) {
      for (int m = 0; m < 4; ++m) {
        double l = 1.0;
        for (int n = 0; n < 4; ++n)
          if (n != m) l *= (gq[q] - y[s + n]) / (y[s + m] - y[s + n]);
        g.trap[s + m] += 0.5 * (b - a) * l;
      }
    }
  }
  return g;
}

}  // namespace channel
