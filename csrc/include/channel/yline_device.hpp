// Device-side building blocks of the y-line (wall-normal) kernels.
//
// One 64-lane wavefront owns one (kx,kz) line of NY points; lane l holds rows j = l*R + r,
// r = 0..R-1, in registers (rows >= NY are identity padding).  Tridiagonal systems are solved by a
// register-resident partitioned algorithm:
//   1. each lane eliminates its R-1 interior rows (Thomas, fp64), expressing them through the
//      separator rows of its own and its left neighbour (the lane's last row is a separator);
//   2. the 64 separator unknowns form a tridiagonal system across lanes, solved by parallel cyclic
//      reduction (6 levels of cross-lane exchange, ds_bpermute);
//   3. each lane back-substitutes its interior rows.
// The factorisation (elimination multipliers + PCR multipliers) is separated from the solve so
// that several right-hand sides share one factorisation (complex data = 2 real RHS; the implicit
// phi/omega solves share one; the influence-matrix homogeneous solutions add 2 more).
//
// This replaces the reference's cusparseZgtsvStridedBatch + per-call diagonal kernels
// (derivatives_nu_double.cu:209-285, 390-415; hemholzt_nu_double.cu:98-251;
// implicitStep_nu_double.cu:98-247), which wrote three double2 diagonal fields to HBM per solve.
// Nothing here touches HBM: the k-independent D1 factorisation is a 64-lane constant table, the
// k-dependent ones are formed in registers from per-row coefficient tables.
#pragma once

#include <hip/hip_runtime.h>

namespace channel {
namespace dev {

constexpr int kWave = 64;
constexpr int kPcrLevels = 6;  // log2(64)

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ double bperm(double v, int src_lane) {
  const int addr = src_lane << 2;
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __builtin_amdgcn_ds_bpermute(addr, lo);
  hi = __builtin_amdgcn_ds_bpermute(addr, hi);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ float bperm(float v, int src_lane) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src_lane << 2, __float_as_int(v)));
}
// value of lane-s (0 for lanes < s)
template <typename V>
__device__ __forceinline__ V shfl_up_z(V v, int s, int lane) {
  V r = bperm(v, (lane - s) & 63);
  return lane >= s ? r : V(0);
}
// value of lane+s (0 for lanes >= 64-s)
template <typename V>
__device__ __forceinline__ V shfl_down_z(V v, int s, int lane) {
  V r = bperm(v, (lane + s) & 63);
  return lane + s < 64 ? r : V(0);
}
// 1/x to full double precision: hardware reciprocal estimate + two Newton steps (each doubles the
// correct bits).  Replaces IEEE division (~10 dependent instructions incl. scale/fixup) on the
// sequential factorisation chains; pivots here are O(1) and never denormal or zero.
__device__ __forceinline__ double fast_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-x, r, 1.0);
  return __builtin_fma(r, e, r);
}

__device__ __forceinline__ double bcast(double v, int src_lane) {
  return bperm(v, src_lane);
}

// Per-row coefficient tables, lane-major: tab[r*64 + lane] is row j = lane*R + r.
struct YTab {
  const double* d1_lo;   // D1 LHS (incl. wall closure rows)
  const double* d1_up;
  const double* d1_rm;   // D1 RHS stencil, interior rows (0 on walls/pad)
  const double* d1_rc;
  const double* d1_rp;
  const double* m_lo;    // compact D2 mass matrix M (interior rows)
  const double* m_up;
  const double* k_lo;    // compact D2 stencil K (interior rows)
  const double* k_c;
  const double* k_up;
  const double* mask;    // 1 on interior rows, 0 on walls and padding
  const double* trap;    // trapezoid weights (0 on padding)
  const double* d1fac;   // D1 factorisation table [nf][64]
  const double* d1row0;  // first row of the dense D1 = A1^-1 B1 (wall derivative at y=-1)
  const double* d1rowN;  // last row (wall derivative at y=+1)
  double w0[3], wN[3];   // D1 wall closures
  int N;
};

__device__ __forceinline__ double tab(const double* __restrict__ p, int r, int lane) {
  return p[r * 64 + lane];
}

template <int R>
struct PFac {
  static constexpr int NI = (R > 1 ? R - 1 : 1);
  double inv[NI], cp[NI];
  double a0, cR2, as, cs;
  double k1[kPcrLevels], k2[kPcrLevels];
  double invB;
  static constexpr int kNumFields = 2 * NI + 4 + 2 * kPcrLevels + 1;
};

// ---- coefficient providers: abc(r, a, b, c) and a(r) for row j = lane*R + r ----------------
struct CoefD1 {
  const YTab& t;
  int lane;
  __device__ void abc(int r, double& a, double& b, double& c) const {
    a = tab(t.d1_lo, r, lane);
    b = 1.0;
    c = tab(t.d1_up, r, lane);
  }
  __device__ double a(int r) const { return tab(t.d1_lo, r, lane); }
};

// (1 + c k^2) M - c K on interior rows, identity on walls/padding  (implicitStep_nu_double.cu:156-163)
struct CoefImpl {
  const YTab& t;
  int lane;
  double g, c;  // g = 1 + c k^2
  __device__ void abc(int r, double& a, double& b, double& cc) const {
    a = tab(t.m_lo, r, lane) * g - c * tab(t.k_lo, r, lane);
    cc = tab(t.m_up, r, lane) * g - c * tab(t.k_up, r, lane);
    const double m = tab(t.mask, r, lane);
    b = 1.0 + m * (g - 1.0 - c * tab(t.k_c, r, lane));
  }
  __device__ double a(int r) const { return tab(t.m_lo, r, lane) * g - c * tab(t.k_lo, r, lane); }
};

// K - k^2 M on interior rows, identity on walls/padding  (hemholzt_nu_double.cu:156-185)
struct CoefHelm {
  const YTab& t;
  int lane;
  double k2;
  __device__ void abc(int r, double& a, double& b, double& c) const {
    a = tab(t.k_lo, r, lane) - k2 * tab(t.m_lo, r, lane);
    c = tab(t.k_up, r, lane) - k2 * tab(t.m_up, r, lane);
    const double m = tab(t.mask, r, lane);
    b = 1.0 + m * (tab(t.k_c, r, lane) - k2 - 1.0);
  }
  __device__ double a(int r) const { return tab(t.k_lo, r, lane) - k2 * tab(t.m_lo, r, lane); }
};

// ---- factorisation -----------------------------------------------------------------------
template <int R, class Coef>
__device__ void pfactor(PFac<R>& F, const Coef& coef, int lane) {
  double A, B, C;
  if constexpr (R == 1) {
    coef.abc(0, A, B, C);
    F.a0 = 0.0; F.cR2 = 0.0; F.as = A; F.cs = C;
    F.inv[0] = 1.0; F.cp[0] = 0.0;
  } else {
    double pc = 0.0;
#pragma unroll
    for (int r = 0; r < R - 1; ++r) {
      double a, b, c;
      coef.abc(r, a, b, c);
      if (r == 0) F.a0 = a;
      if (r == R - 2) F.cR2 = c;
      const double den = b - a * pc;
      F.inv[r] = fast_rcp(den);
      F.cp[r] = c * F.inv[r];
      pc = F.cp[r];
    }
    // left spike L (rhs = -a0 e_0) and right spike U (rhs = -cR2 e_{R-2})
    double dl[R - 1];
    dl[0] = -F.a0 * F.inv[0];
#pragma unroll
    for (int r = 1; r < R - 1; ++r) dl[r] = -coef.a(r) * dl[r - 1] * F.inv[r];
    const double L_last = dl[R - 2];
    double Lr = dl[R - 2];
#pragma unroll
    for (int r = R - 3; r >= 0; --r) Lr = dl[r] - F.cp[r] * Lr;
    const double L_first = Lr;
    const double U_last = -F.cR2 * F.inv[R - 2];
    double Ur = U_last;
#pragma unroll
    for (int r = R - 3; r >= 0; --r) Ur = -F.cp[r] * Ur;
    const double U_first = Ur;
    double as, bs, cs;
    coef.abc(R - 1, as, bs, cs);
    F.as = as;
    F.cs = cs;
    const double L0n = shfl_down_z(L_first, 1, lane);
    const double U0n = shfl_down_z(U_first, 1, lane);
    A = as * L_last;
    B = bs + as * U_last + cs * L0n;
    C = cs * U0n;
  }
#pragma unroll
  for (int t = 0; t < kPcrLevels; ++t) {
    const int s = 1 << t;
    // each lane inverts its own pivot once and the neighbours receive 1/B (one reciprocal per
    // level instead of two divisions)
    const double iB = fast_rcp(B);
    const double Am = shfl_up_z(A, s, lane), iBm = shfl_up_z(iB, s, lane), Cm = shfl_up_z(C, s, lane);
    const double Ap = shfl_down_z(A, s, lane), iBp = shfl_down_z(iB, s, lane), Cp = shfl_down_z(C, s, lane);
    const bool hm = lane >= s, hp = lane + s < 64;
    const double k1 = hm ? A * iBm : 0.0;
    const double k2 = hp ? C * iBp : 0.0;
    const double nA = -Am * k1;
    const double nC = -Cp * k2;
    const double nB = B - Cm * k1 - Ap * k2;
    A = nA; B = nB; C = nC;
    F.k1[t] = k1;
    F.k2[t] = k2;
  }
  F.invB = fast_rcp(B);
}

template <int R>
__device__ void pfac_store(const PFac<R>& F, double* __restrict__ out, int lane) {
  int f = 0;
#pragma unroll
  for (int r = 0; r < PFac<R>::NI; ++r) out[(f++) * 64 + lane] = F.inv[r];
#pragma unroll
  for (int r = 0; r < PFac<R>::NI; ++r) out[(f++) * 64 + lane] = F.cp[r];
  out[(f++) * 64 + lane] = F.a0;
  out[(f++) * 64 + lane] = F.cR2;
  out[(f++) * 64 + lane] = F.as;
  out[(f++) * 64 + lane] = F.cs;
#pragma unroll
  for (int t = 0; t < kPcrLevels; ++t) out[(f++) * 64 + lane] = F.k1[t];
#pragma unroll
  for (int t = 0; t < kPcrLevels; ++t) out[(f++) * 64 + lane] = F.k2[t];
  out[(f++) * 64 + lane] = F.invB;
}

template <int R>
__device__ void pfac_load(PFac<R>& F, const double* __restrict__ in, int lane) {
  int f = 0;
#pragma unroll
  for (int r = 0; r < PFac<R>::NI; ++r) F.inv[r] = in[(f++) * 64 + lane];
#pragma unroll
  for (int r = 0; r < PFac<R>::NI; ++r) F.cp[r] = in[(f++) * 64 + lane];
  F.a0 = in[(f++) * 64 + lane];
  F.cR2 = in[(f++) * 64 + lane];
  F.as = in[(f++) * 64 + lane];
  F.cs = in[(f++) * 64 + lane];
#pragma unroll
  for (int t = 0; t < kPcrLevels; ++t) F.k1[t] = in[(f++) * 64 + lane];
#pragma unroll
  for (int t = 0; t < kPcrLevels; ++t) F.k2[t] = in[(f++) * 64 + lane];
  F.invB = in[(f++) * 64 + lane];
}

// ---- solve K right-hand sides in place ----------------------------------------------------
template <int R, int K, class Coef>
__device__ void psolve(const PFac<R>& F, const Coef& coef, double (&d)[K][R], int lane) {
  double D[K];
  if constexpr (R == 1) {
#pragma unroll
    for (int k = 0; k < K; ++k) D[k] = d[k][0];
  } else {
    double P0[K], PL[K];
    {
      double dp[K][R - 1];
#pragma unroll
      for (int k = 0; k < K; ++k) dp[k][0] = d[k][0] * F.inv[0];
#pragma unroll
      for (int r = 1; r < R - 1; ++r) {
        const double a = coef.a(r);
#pragma unroll
        for (int k = 0; k < K; ++k) dp[k][r] = (d[k][r] - a * dp[k][r - 1]) * F.inv[r];
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        double P = dp[k][R - 2];
        PL[k] = P;
#pragma unroll
        for (int r = R - 3; r >= 0; --r) P = dp[k][r] - F.cp[r] * P;
        P0[k] = P;
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) D[k] = d[k][R - 1] - F.as * PL[k] - F.cs * shfl_down_z(P0[k], 1, lane);
  }
#pragma unroll
  for (int t = 0; t < kPcrLevels; ++t) {
    const int s = 1 << t;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double Dm = shfl_up_z(D[k], s, lane);
      const double Dp = shfl_down_z(D[k], s, lane);
      D[k] = D[k] - F.k1[t] * Dm - F.k2[t] * Dp;
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double y = D[k] * F.invB;
    if constexpr (R == 1) {
      d[k][0] = y;
    } else {
      const double yl = shfl_up_z(y, 1, lane);
      d[k][0] -= F.a0 * yl;
      d[k][R - 2] -= F.cR2 * y;
      // interior solve with the separator values known
      double dp[R - 1];
      dp[0] = d[k][0] * F.inv[0];
#pragma unroll
      for (int r = 1; r < R - 1; ++r) dp[r] = (d[k][r] - coef.a(r) * dp[r - 1]) * F.inv[r];
      double x = dp[R - 2];
      d[k][R - 2] = x;
#pragma unroll
      for (int r = R - 3; r >= 0; --r) {
        x = dp[r] - F.cp[r] * x;
        d[k][r] = x;
      }
      d[k][R - 1] = y;
    }
  }
}

// ---- stencils ----------------------------------------------------------------------------
// value at global row j (wave-uniform j); returns 0 if j out of range
template <int R>
__device__ __forceinline__ double row_value(const double (&x)[R], int j, int lane) {
  const int src = j / R, rr = j - src * R;
  double v = 0.0;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (r == rr) v = x[r];
  return bcast(v, src);
}

template <int R, int K>
__device__ __forceinline__ void halo(const double (&x)[K][R], double (&left)[K], double (&right)[K], int lane) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    left[k] = shfl_up_z(x[k][R - 1], 1, lane);
    right[k] = shfl_down_z(x[k][0], 1, lane);
  }
}

// out = tridiag(lo, c, up) * x with per-row tables (c may be null => mask)
template <int R, int K>
__device__ void apply_tri(const double* __restrict__ lo, const double* __restrict__ cc, const double* __restrict__ up,
                          const double (&x)[K][R], double (&out)[K][R], int lane) {
  double L[K], Rt[K];
  halo<R, K>(x, L, Rt, lane);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const double a = tab(lo, r, lane), b = tab(cc, r, lane), c = tab(up, r, lane);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double xm = (r == 0) ? L[k] : x[k][r - 1];
      const double xp = (r == R - 1) ? Rt[k] : x[k][r + 1];
      out[k][r] = a * xm + b * x[k][r] + c * xp;
    }
  }
}

// D1 right-hand side B1 f (interior stencil + 3-point one-sided wall closures)
template <int R, int K>
__device__ void d1_rhs(const YTab& t, const double (&x)[K][R], double (&out)[K][R], int lane) {
  apply_tri<R, K>(t.d1_rm, t.d1_rc, t.d1_rp, x, out, lane);
  const int N = t.N;
  const int jN = N - 1, lN = jN / R, rN = jN - lN * R;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double f1 = row_value<R>(x[k], 1, lane), f2 = row_value<R>(x[k], 2, lane);
    const double g1 = row_value<R>(x[k], N - 2, lane), g2 = row_value<R>(x[k], N - 3, lane);
    const double f0 = row_value<R>(x[k], 0, lane), g0 = row_value<R>(x[k], N - 1, lane);
    if (lane == 0) out[k][0] = t.w0[0] * f0 + t.w0[1] * f1 + t.w0[2] * f2;
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (lane == lN && r == rN) out[k][r] = t.wN[0] * g0 + t.wN[1] * g1 + t.wN[2] * g2;
  }
}

template <int K>
__device__ __forceinline__ void wave_sum_n(double (&v)[K]) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1)
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += bperm(v[k], (__lane_id() ^ s));
}

template <int R>
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) v += bperm(v, (__lane_id() ^ s));
  return v;
}

}  // namespace dev
}  // namespace channel
