// Wall-normal grid and compact finite-difference coefficient tables (fp64).
//
// Reproduces the reference discretisation:
//  * grid  y_j = tanh(s (j*dy - 1)) / tanh(s), dy = 2/(NY-1), s = 2  (channel.h:21, 50-51)
//  * compact D1: interior  beta f'_{j-1} + f'_j + alpha f'_{j+1} = B f_{j-1} + C f_j + A f_{j+1}
//    (derivatives_nu_double.cu:60-65, 227-232), 3-point one-sided wall closure (:85-112, 247-274)
//  * compact D2: interior  beta f''_{j-1} + f''_j + alpha f''_{j+1} = B f_{j-1} + C f_j + A f_{j+1}
//    (hemholzt_nu_double.cu:58-62, 136-145); the mass matrix M = tridiag(beta,1,alpha) and the
//    stencil K = tridiag(B,C,A) are kept separately because every implicit/Helmholtz system is
//    solved in "M-form": [K - k^2 M] v = M phi,  [(1+c k^2) M - c K] q = M rhs.
//  * D2 wall closure (used by the mean-flow solver in the reference, meanUevol.c:254-329); kept
//    for the parity/oracle path.
#pragma once

#include <vector>

namespace channel {

struct YGrid {
  int N = 0;
  double stretch = 2.0;
  std::vector<double> y;       // N points, y[0] = -1, y[N-1] = +1

  // compact D1 (LHS rows: lo*f'_{j-1} + f'_j + up*f'_{j+1}); lo[0]=0, up[N-1]=0
  std::vector<double> d1_lo, d1_up;
  // D1 RHS stencil on interior rows (zero on wall rows); wall rows use w0 / wN below
  std::vector<double> d1_rm, d1_rc, d1_rp;
  double d1_w0[3] = {0, 0, 0};  // row 0:    w0[0] f0 + w0[1] f1 + w0[2] f2
  double d1_wN[3] = {0, 0, 0};  // row N-1:  wN[0] f_{N-1} + wN[1] f_{N-2} + wN[2] f_{N-3}

  // compact D2 interior rows 1..N-2 (zero on wall rows)
  std::vector<double> m_lo, m_up;        // M = tridiag(m_lo, 1, m_up)
  std::vector<double> k_lo, k_c, k_up;   // K = tridiag(k_lo, k_c, k_up)
  // D2 wall closure (reference mean flow): LHS off-diagonals and RHS (E,A,B) at the walls
  double d2_w0_up = 0, d2_wN_lo = 0;
  double d2_w0[3] = {0, 0, 0};  // row 0:   E f0 + A f1 + B f2
  double d2_wN[3] = {0, 0, 0};  // row N-1: E f_{N-1} + A f_{N-2} + B f_{N-3}

  std::vector<double> trap;     // trapezoid quadrature weights (sum = 2)

  static YGrid build(int N, double stretch = 2.0);
};

}  // namespace channel
