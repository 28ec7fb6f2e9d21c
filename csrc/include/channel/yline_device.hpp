// Device-side building blocks of the y-line (wall-normal) kernels.
//
// One 64-lane wavefront owns one (kx,kz) line of NY points; lane l holds rows j = l*R + r,
// r = 0..R-1, in registers (rows >= NY are identity padding).  Tridiagonal systems are solved by a
// register-resident partitioned algorithm:
//   1. each lane eliminates its R-1 interior rows (Thomas, fp64), expressing them through the
//      separator rows of its own and its left neighbour (the lane's last row is a separator);
//   2. the 64 separator unknowns form a tridiagonal system across lanes, solved by parallel cyclic
//      reduction (6 levels of cross-lane exchange in the VALU: DPP and permlane swaps);
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

// ---- cross-lane shifts in the VALU (no LDS) -------------------------------------------------
// The solver's communication is fixed-stride shifts (PCR strides 1..32, halos, wave sums).  A
// ds_bpermute is an LDS round trip (~100+ cycles) on the dependent chain of every PCR level and,
// at one wave per SIMD, nothing hides it; it also competes with the staging tiles for LDS.  Here:
//   stride 1      DPP wave_shr:1 / wave_shl:1 (one VALU op per dword)
//   stride 2, 4   chains of stride-1 DPP moves
//   stride 8      DPP row_shr/row_shl inside 16-lane rows + row_ror fed through a 16-lane shift
//   stride 16     v_permlane16_swap + v_permlane32_swap (CDNA4), both directions at once
//   stride 32     v_permlane32_swap, both directions at once
// XV = false selects the ds_bpermute versions (kernels that spill VGPRs keep them: see xl_valu()).
constexpr int kDppRowShl = 0x100, kDppRowShr = 0x110, kDppRowRor = 0x120, kDppWaveShl1 = 0x130,
              kDppWaveShr1 = 0x138;
template <int CTRL>
__device__ __forceinline__ int dpp_z(int v) {  // lanes whose source is out of range read 0
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}
// f of lane-16 (0 in rows 0) and of lane+16 (0 in row 3)
__device__ __forceinline__ void xl_updn16(int f, int& up, int& dn) {
  const int row = __lane_id() >> 4;
  // p = {[f0 f0 f2 f2], [f1 f1 f3 f3]} (rows), q = {[f0 f0 f1 f1], [f2 f2 f3 f3]}
  const auto p = __builtin_amdgcn_permlane16_swap(f, f, false, false);
  const auto q = __builtin_amdgcn_permlane32_swap(p[0], p[1], false, false);
  up = row == 0 ? 0 : static_cast<int>(row == 3 ? p[0] : q[0]);
  dn = row == 3 ? 0 : static_cast<int>(row == 0 ? p[1] : q[1]);
}
// v of lane-S (0 for lanes < S) and of lane+S (0 for lanes >= 64-S); S is a compile-time constant
// after unrolling at every call site
__device__ __forceinline__ void xl_updn(int v, int s, int& up, int& dn) {
  const int lane = __lane_id(), l16 = lane & 15;
  switch (s) {
    case 1:
      up = dpp_z<kDppWaveShr1>(v);
      dn = dpp_z<kDppWaveShl1>(v);
      break;
    case 2:
      up = dpp_z<kDppWaveShr1>(dpp_z<kDppWaveShr1>(v));
      dn = dpp_z<kDppWaveShl1>(dpp_z<kDppWaveShl1>(v));
      break;
    case 4:
      up = dpp_z<kDppWaveShr1>(dpp_z<kDppWaveShr1>(dpp_z<kDppWaveShr1>(dpp_z<kDppWaveShr1>(v))));
      dn = dpp_z<kDppWaveShl1>(dpp_z<kDppWaveShl1>(dpp_z<kDppWaveShl1>(dpp_z<kDppWaveShl1>(v))));
      break;
    case 8: {
      const int a = dpp_z<kDppRowShr + 8>(v), b = dpp_z<kDppRowShl + 8>(v), f = dpp_z<kDppRowRor + 8>(v);
      int u16, d16;
      xl_updn16(f, u16, d16);
      up = l16 >= 8 ? a : u16;
      dn = l16 < 8 ? b : d16;
      break;
    }
    case 16:
      xl_updn16(v, up, dn);
      break;
    default: {  // 32
      const auto q = __builtin_amdgcn_permlane32_swap(v, v, false, false);  // {[v0 v1 v0 v1], [v2 v3 v2 v3]}
      up = lane >= 32 ? static_cast<int>(q[0]) : 0;
      dn = lane < 32 ? static_cast<int>(q[1]) : 0;
    }
  }
}
template <bool XV>
__device__ __forceinline__ void xl_updn(double v, int s, double& up, double& dn) {
  if constexpr (!XV) {
    const int lane = __lane_id();
    const double u = bperm(v, (lane - s) & 63), d = bperm(v, (lane + s) & 63);
    up = lane >= s ? u : 0.0;
    dn = lane + s < 64 ? d : 0.0;
  } else {
    int ul, uh, dl, dh;
    xl_updn(__double2loint(v), s, ul, dl);
    xl_updn(__double2hiint(v), s, uh, dh);
    up = __hiloint2double(uh, ul);
    dn = __hiloint2double(dh, dl);
  }
}
// value of lane-s (0 for lanes < s)
template <bool XV>
__device__ __forceinline__ double shfl_up_z(double v, int s, int lane) {
  if constexpr (XV) {
    if (s == 1)
      return __hiloint2double(dpp_z<kDppWaveShr1>(__double2hiint(v)), dpp_z<kDppWaveShr1>(__double2loint(v)));
  }
  double up, dn;
  xl_updn<XV>(v, s, up, dn);
  return up;
}
// value of lane+s (0 for lanes >= 64-s)
template <bool XV>
__device__ __forceinline__ double shfl_down_z(double v, int s, int lane) {
  if constexpr (XV) {
    if (s == 1)
      return __hiloint2double(dpp_z<kDppWaveShl1>(__double2hiint(v)), dpp_z<kDppWaveShl1>(__double2loint(v)));
  }
  double up, dn;
  xl_updn<XV>(v, s, up, dn);
  return dn;
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

// value of lane src_lane (wave-uniform) in every lane
template <bool XV>
__device__ __forceinline__ double bcast(double v, int src_lane) {
  if constexpr (!XV)
    return bperm(v, src_lane);
  else
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), src_lane),
                            __builtin_amdgcn_readlane(__double2loint(v), src_lane));
}

// sum over the wave, bitwise identical in every lane: rotations inside 16-lane rows (each lane
// pairs with a partner that forms the same sum), then the row pairs and halves via permlane swaps
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  return __hiloint2double(dpp_z<CTRL>(__double2hiint(v)), dpp_z<CTRL>(__double2loint(v)));
}
__device__ __forceinline__ double xl_swap16(double v) {  // value of lane ^ 16
  const int row = __lane_id() >> 4;
  const auto ph = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
  const auto pl = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
  return (row & 1) ? __hiloint2double(ph[0], pl[0]) : __hiloint2double(ph[1], pl[1]);
}
__device__ __forceinline__ double xl_swap32(double v) {  // value of lane ^ 32
  const bool lo = __lane_id() < 32;
  const auto qh = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
  const auto ql = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
  return lo ? __hiloint2double(qh[1], ql[1]) : __hiloint2double(qh[0], ql[0]);
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
template <int R, bool XV, class Coef>
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
    const double L0n = shfl_down_z<XV>(L_first, 1, lane);
    const double U0n = shfl_down_z<XV>(U_first, 1, lane);
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
    double Am, iBm, Cm, Ap, iBp, Cp;
    xl_updn<XV>(A, s, Am, Ap);
    xl_updn<XV>(iB, s, iBm, iBp);
    xl_updn<XV>(C, s, Cm, Cp);
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
template <int R, int K, bool XV, class Coef>
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
    for (int k = 0; k < K; ++k) D[k] = d[k][R - 1] - F.as * PL[k] - F.cs * shfl_down_z<XV>(P0[k], 1, lane);
  }
#pragma unroll
  for (int t = 0; t < kPcrLevels; ++t) {
    const int s = 1 << t;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      double Dm, Dp;
      xl_updn<XV>(D[k], s, Dm, Dp);
      D[k] = D[k] - F.k1[t] * Dm - F.k2[t] * Dp;
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double y = D[k] * F.invB;
    if constexpr (R == 1) {
      d[k][0] = y;
    } else {
      const double yl = shfl_up_z<XV>(y, 1, lane);
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
template <int R, bool XV>
__device__ __forceinline__ double row_value(const double (&x)[R], int j, int lane) {
  const int src = j / R, rr = j - src * R;
  double v = 0.0;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (r == rr) v = x[r];
  return bcast<XV>(v, src);
}

template <int R, int K, bool XV>
__device__ __forceinline__ void halo(const double (&x)[K][R], double (&left)[K], double (&right)[K], int lane) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    left[k] = shfl_up_z<XV>(x[k][R - 1], 1, lane);
    right[k] = shfl_down_z<XV>(x[k][0], 1, lane);
  }
}

// out = tridiag(lo, c, up) * x with per-row tables (c may be null => mask)
template <int R, int K, bool XV>
__device__ void apply_tri(const double* __restrict__ lo, const double* __restrict__ cc, const double* __restrict__ up,
                          const double (&x)[K][R], double (&out)[K][R], int lane) {
  double L[K], Rt[K];
  halo<R, K, XV>(x, L, Rt, lane);
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
template <int R, int K, bool XV>
__device__ void d1_rhs(const YTab& t, const double (&x)[K][R], double (&out)[K][R], int lane) {
  apply_tri<R, K, XV>(t.d1_rm, t.d1_rc, t.d1_rp, x, out, lane);
  const int N = t.N;
  const int jN = N - 1, lN = jN / R, rN = jN - lN * R;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double f1 = row_value<R, XV>(x[k], 1, lane), f2 = row_value<R, XV>(x[k], 2, lane);
    const double g1 = row_value<R, XV>(x[k], N - 2, lane), g2 = row_value<R, XV>(x[k], N - 3, lane);
    const double f0 = row_value<R, XV>(x[k], 0, lane), g0 = row_value<R, XV>(x[k], N - 1, lane);
    if (lane == 0) out[k][0] = t.w0[0] * f0 + t.w0[1] * f1 + t.w0[2] * f2;
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (lane == lN && r == rN) out[k][r] = t.wN[0] * g0 + t.wN[1] * g1 + t.wN[2] * g2;
  }
}

template <int K, bool XV>
__device__ __forceinline__ void wave_sum_n(double (&v)[K]) {
  if constexpr (!XV) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1)
#pragma unroll
      for (int k = 0; k < K; ++k) v[k] += bperm(v[k], (__lane_id() ^ s));
    return;
  }
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_d<kDppRowRor + 8>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_d<kDppRowRor + 4>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_d<kDppRowRor + 2>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_d<kDppRowRor + 1>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += xl_swap16(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += xl_swap32(v[k]);
}

template <int R, bool XV>
__device__ __forceinline__ double wave_sum(double v) {
  double a[1] = {v};
  wave_sum_n<1, XV>(a);
  return a[0];
}

}  // namespace dev
}  // namespace channel
