// Device-side building blocks of the y-line (wall-normal) kernels.
//
// One 64-lane wavefront owns one (kx,kz) line of NY points; lane l holds rows j = l*R + r,
// r = 0..R-1, in registers (rows >= NY are identity padding).  Tridiagonal systems are solved by a
// register-resident partitioned algorithm:
//   1. each lane eliminates its R-1 interior rows (Thomas, fp64), expressing them through the
//      separator rows of its own and its left neighbour (the lane's last row is a separator);
//   2. the 64 separator unknowns form a tridiagonal system across lanes, solved by parallel cyclic
//      reduction (6 levels of cross-lane exchange, strides 1..32);
//   3. each lane back-substitutes its interior rows.
// The factorisation (elimination multipliers + PCR multipliers) is separated from the solve so
// that several right-hand sides share one factorisation (complex data = 2 real RHS; the implicit
// phi/omega solves share one; the influence-matrix homogeneous solutions add 2 more).
//
// Cross-lane exchange policies (template parameter XM):
//   kXlBperm  ds_bpermute for every stride (LDS crossbar, no LDS storage)
//   kXlDpp    VALU only: DPP wave_shr/shl, row_shr/shl/ror and v_permlane16/32_swap
//   kXlLds    strides 1, 2 by DPP; strides >= 4 by one ds_write_b64 + two ds_read_b64 per value
//             through a per-wave LDS scratch line.  The DPP forms of the long strides cost 11-22
//             VALU instructions per double (8 of them v_cndmask) against 3 LDS instructions, and
//             the LDS pipe runs beside the VALU.  Out-of-range neighbours read a clamped lane:
//             the PCR multipliers that consume them are exactly zero there (A = 0 on lanes < s,
//             C = 0 on lanes >= 64 - s at level s), so the results equal the zero-filled forms.
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
constexpr int kXlBperm = 0, kXlDpp = 1, kXlLds = 2;
// doubles of per-wave LDS scratch the kXlLds policy needs for K values exchanged at once
constexpr int xl_scratch_doubles(int kmax) { return kmax * kWave; }

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
//   stride 1      DPP wave_shr:1 / wave_shl:1 (one VALU op per dword)
//   stride 2, 4   chains of stride-1 DPP moves
//   stride 8      DPP row_shr/row_shl inside 16-lane rows + row_ror fed through a 16-lane shift
//   stride 16     v_permlane16_swap + v_permlane32_swap (CDNA4), both directions at once
//   stride 32     v_permlane32_swap, both directions at once
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
__device__ __forceinline__ void xl_updn_i(int v, int s, int& up, int& dn) {
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
__device__ __forceinline__ void xl_updn_dpp(double v, int s, double& up, double& dn) {
  int ul, uh, dl, dh;
  xl_updn_i(__double2loint(v), s, ul, dl);
  xl_updn_i(__double2hiint(v), s, uh, dh);
  up = __hiloint2double(uh, ul);
  dn = __hiloint2double(dh, dl);
}
__device__ __forceinline__ void xl_updn_bperm(double v, int s, double& up, double& dn) {
  const int lane = __lane_id();
  const double u = bperm(v, (lane - s) & 63), d = bperm(v, (lane + s) & 63);
  up = lane >= s ? u : 0.0;
  dn = lane + s < 64 ? d : 0.0;
}

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  return __hiloint2double(dpp_z<CTRL>(__double2hiint(v)), dpp_z<CTRL>(__double2loint(v)));
}
// value of lane-1 (0 in lane 0) / lane+1 (0 in lane 63): one DPP move per dword in every policy
// except kXlBperm
template <int XM>
__device__ __forceinline__ double shfl_up1(double v) {
  if constexpr (XM == kXlBperm) {
    double u, d;
    xl_updn_bperm(v, 1, u, d);
    return u;
  } else {
    return dpp_d<kDppWaveShr1>(v);
  }
}
template <int XM>
__device__ __forceinline__ double shfl_dn1(double v) {
  if constexpr (XM == kXlBperm) {
    double u, d;
    xl_updn_bperm(v, 1, u, d);
    return d;
  } else {
    return dpp_d<kDppWaveShl1>(v);
  }
}

// Cross-lane exchange of K values at stride s.  kXlLds: buf = this wave's scratch (K*64 doubles);
// the neighbours outside the wave are clamped reads (see the header comment), the DPP/bpermute
// forms zero-fill them.
template <int XM>
struct Xl {
  double* buf = nullptr;
  template <int K>
  __device__ __forceinline__ void updn(const double (&v)[K], int s, double (&up)[K], double (&dn)[K]) const {
    if constexpr (XM == kXlLds) {
      if (s >= 4) {
        const int lane = __lane_id();
#pragma unroll
        for (int k = 0; k < K; ++k) buf[k * kWave + lane] = v[k];
        // a wave's LDS instructions execute in order: the reads below see these writes, and the
        // next exchange's writes cannot overtake them (the compiler keeps the aliasing order)
        const int lu = lane >= s ? lane - s : lane;
        const int ld = lane + s < kWave ? lane + s : lane;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          up[k] = buf[k * kWave + lu];
          dn[k] = buf[k * kWave + ld];
        }
        return;
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if constexpr (XM == kXlBperm) xl_updn_bperm(v[k], s, up[k], dn[k]);
      else xl_updn_dpp(v[k], s, up[k], dn[k]);
    }
  }
};

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
template <int XM>
__device__ __forceinline__ double bcast(double v, int src_lane) {
  if constexpr (XM == kXlBperm)
    return bperm(v, src_lane);
  else
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), src_lane),
                            __builtin_amdgcn_readlane(__double2loint(v), src_lane));
}

// sum over the wave, bitwise identical in every lane: rotations inside 16-lane rows (each lane
// pairs with a partner that forms the same sum), then the row pairs and halves via permlane swaps
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
  const double* d1_rm;   // D1 RHS stencil B1: interior rows, wall closures folded in at rows 0, N-1
  const double* d1_rc;
  const double* d1_rp;
  const double* m_lo;    // compact D2 mass matrix M (interior rows)
  const double* m_up;
  const double* k_lo;    // compact D2 stencil K (interior rows)
  const double* k_c;
  const double* k_up;
  const double* mask;    // 1 on interior rows, 0 on walls and padding
  const double* d1row0;  // first row of the dense D1 = A1^-1 B1 (wall derivative at y=-1)
  const double* d1rowN;  // last row (wall derivative at y=+1)
  const double* d1fac;   // D1 factorisation table [nf][64]
  const double* trap;    // trapezoid weights (0 on padding; mean line only, never staged in LDS)
  const double* d1spk;   // lines over two waves: this half's D1 spike (response to its coupling row)
  double w0[3], wN[3];   // D1 wall closures (w0[2], wN[2]: the third points, see d1_rhs)
  int N;
};
// The table buffer (YTablesDev::upload) is contiguous: kYTabRowTables per-row tables of 64*R
// doubles in the YTab field order d1_lo .. d1rowN, then d1fac, then trap.
constexpr int kYTabRowTables = 13;

__device__ __forceinline__ double tab(const double* __restrict__ p, int r, int lane) {
  return p[r * 64 + lane];
}

// ---- lines over H waves ---------------------------------------------------------------------
// H = 1: a line is one wave (lane l holds rows l R .. l R + R - 1).  H = 2: a line is two waves of
// one workgroup, wave half h holding rows h HR + l R + r (HR = 64 R).  Every tridiagonal system is
// solved per half with the coupling between rows HR - 1 and HR dropped (the per-wave SPIKE/PCR
// solver below, unchanged), plus one extra right-hand side per half, the spike (the half's response
// to its coupling coefficient); the halves then meet in a 2 x 2 interface solve (the two-partition
// SPIKE form).  Stencils exchange one halo row per side, line sums add the two halves.  The two
// waves of a line exchange values through a small LDS area with a per-line flag pair (no workgroup
// barrier: only the partner is waited for, and line-dependent branches such as the mean line's stay
// legal).  At NY = 385 this gives R = 4 (two waves per SIMD) instead of one wave of R = 7 per line.
template <int H>
struct LineG;
template <>
struct LineG<1> {
  static constexpr int kH = 1;
  int h = 0;
};
template <>
struct LineG<2> {
  static constexpr int kH = 2;
  static constexpr int kXK = 16;  // doubles per exchange slot
  int h = 0;
  double* buf = nullptr;  // [2 parity][2 halves][kXK] of this line (LDS)
  int* flag = nullptr;    // [2 halves] exchange generation of each half (LDS, zeroed at start)
  mutable int gen = 0;
  // uniform values of this half -> the partner's; the generation parity double-buffers the slots
  // (a half can be at most one exchange ahead: it waits for the partner's flag of its generation)
  // this half's slot of the next exchange: the caller's lanes write their values into it, then
  // post() publishes them (the generation parity double-buffers the slots: a half can be at most
  // one exchange ahead, it waits for the partner's flag of its generation)
  __device__ __forceinline__ double* slot() const { return buf + (((gen + 1) & 1) * 2 + h) * kXK; }
  // publish this half's slot, wait for the partner's; returns the partner's slot
  __device__ __forceinline__ const double* post() const {
    ++gen;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // every lane's slot writes first
    if (__lane_id() == 0) __hip_atomic_store(flag + h, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    // bounded wait (every wave must be able to finish: a broken pairing yields wrong results, which
    // the oracle tests catch, never a hung kernel); the partner is normally a few hundred cycles away
    for (int it = 0; it < (1 << 16) &&
                     __hip_atomic_load(flag + (1 - h), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < gen;
         ++it)
      __builtin_amdgcn_s_sleep(1);
    return buf + ((gen & 1) * 2 + (1 - h)) * kXK;
  }
  // wave-uniform values of this half -> the partner's
  template <int K>
  __device__ __forceinline__ void exch(const double (&mine)[K], double (&theirs)[K]) const {
    static_assert(K <= kXK, "exchange slot too small");
    double* sl = slot();
    if (__lane_id() == 0)
#pragma unroll
      for (int k = 0; k < K; ++k) sl[k] = mine[k];
    const double* rb = post();
#pragma unroll
    for (int k = 0; k < K; ++k) theirs[k] = rb[k];
  }
};

__device__ __forceinline__ double readlane_d(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}

// factorisation coefficients of one half: the lower coupling of the half's first row (row HR,
// lane 0 of half 1) is dropped (the upper one of row HR - 1 drops out by itself: lane 63 has no
// right neighbour in the wave)
template <class Coef>
struct CutLo {
  const Coef& c;
  bool cut;
  __device__ void abc(int r, double& a, double& b, double& cc) const {
    c.abc(r, a, b, cc);
    if (cut && r == 0) a = 0.0;
  }
  __device__ double a(int r) const { return (cut && r == 0) ? 0.0 : c.a(r); }
};

// ---- factorisations: registers (k-dependent) or a 64-lane table (the constant D1) -------------
// Per lane: the interior Thomas multipliers (inv, cp) of rows 0..R-2, the spikes Ls / Us (the
// interior rows' responses to the left neighbour's and to the own separator unknown), the
// separator row's coupling (as, cs), the PCR multipliers and the final pivot.
template <int R>
struct PFac {
  static constexpr int NI = (R > 1 ? R - 1 : 1);
  double inv_[NI], cp_[NI], ls_[NI], us_[NI];
  double as_, cs_;
  double k1_[kPcrLevels], k2_[kPcrLevels];
  double invB_;
  static constexpr int kNumFields = 4 * NI + 2 + 2 * kPcrLevels + 1;
  __device__ __forceinline__ double inv(int r) const { return inv_[r]; }
  __device__ __forceinline__ double cp(int r) const { return cp_[r]; }
  __device__ __forceinline__ double ls(int r) const { return ls_[r]; }
  __device__ __forceinline__ double us(int r) const { return us_[r]; }
  __device__ __forceinline__ double as() const { return as_; }
  __device__ __forceinline__ double cs() const { return cs_; }
  __device__ __forceinline__ double k1(int t) const { return k1_[t]; }
  __device__ __forceinline__ double k2(int t) const { return k2_[t]; }
  __device__ __forceinline__ double invB() const { return invB_; }
};
// the same fields read from the table written by pfac_store (field f of lane l at p[f*64 + l]):
// no registers held across the solve
template <int R>
struct TFac {
  static constexpr int NI = PFac<R>::NI;
  const double* __restrict__ p;
  int lane;
  __device__ __forceinline__ double at(int f) const { return p[f * 64 + lane]; }
  __device__ __forceinline__ double inv(int r) const { return at(r); }
  __device__ __forceinline__ double cp(int r) const { return at(NI + r); }
  __device__ __forceinline__ double ls(int r) const { return at(2 * NI + r); }
  __device__ __forceinline__ double us(int r) const { return at(3 * NI + r); }
  __device__ __forceinline__ double as() const { return at(4 * NI); }
  __device__ __forceinline__ double cs() const { return at(4 * NI + 1); }
  __device__ __forceinline__ double k1(int t) const { return at(4 * NI + 2 + t); }
  __device__ __forceinline__ double k2(int t) const { return at(4 * NI + 2 + kPcrLevels + t); }
  __device__ __forceinline__ double invB() const { return at(4 * NI + 2 + 2 * kPcrLevels); }
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
template <int R, int XM, class Coef>
__device__ void pfactor(PFac<R>& F, const Coef& coef, const Xl<XM>& xl, int lane) {
  double A, B, C;
  if constexpr (R == 1) {
    coef.abc(0, A, B, C);
    F.as_ = A; F.cs_ = C;
    F.inv_[0] = 1.0; F.cp_[0] = 0.0; F.ls_[0] = 0.0; F.us_[0] = 0.0;
  } else {
    double pc = 0.0, a0 = 0.0, cR2 = 0.0;
#pragma unroll
    for (int r = 0; r < R - 1; ++r) {
      double a, b, c;
      coef.abc(r, a, b, c);
      if (r == 0) a0 = a;
      if (r == R - 2) cR2 = c;
      const double den = b - a * pc;
      F.inv_[r] = fast_rcp(den);
      F.cp_[r] = c * F.inv_[r];
      pc = F.cp_[r];
    }
    // left spike (interior response to the left separator: rhs -a0 e_0) and right spike (to the
    // own separator: rhs -cR2 e_{R-2}), both fully back-substituted
    F.ls_[0] = -a0 * F.inv_[0];
#pragma unroll
    for (int r = 1; r < R - 1; ++r) F.ls_[r] = -coef.a(r) * F.ls_[r - 1] * F.inv_[r];
#pragma unroll
    for (int r = R - 3; r >= 0; --r) F.ls_[r] -= F.cp_[r] * F.ls_[r + 1];
    F.us_[R - 2] = -cR2 * F.inv_[R - 2];
#pragma unroll
    for (int r = R - 3; r >= 0; --r) F.us_[r] = -F.cp_[r] * F.us_[r + 1];
    double as, bs, cs;
    coef.abc(R - 1, as, bs, cs);
    F.as_ = as;
    F.cs_ = cs;
    const double L0n = shfl_dn1<XM>(F.ls_[0]);
    const double U0n = shfl_dn1<XM>(F.us_[0]);
    A = as * F.ls_[R - 2];
    B = bs + as * F.us_[R - 2] + cs * L0n;
    C = cs * U0n;
  }
#pragma unroll
  for (int t = 0; t < kPcrLevels; ++t) {
    const int s = 1 << t;
    // each lane inverts its own pivot once and the neighbours receive 1/B (one reciprocal per
    // level instead of two divisions).  A is exactly 0 on lanes < s and C on lanes >= 64 - s, so
    // the multipliers vanish there whatever the (zero-filled or clamped) neighbour values are.
    const double v[3] = {A, fast_rcp(B), C};
    double m[3], p[3];
    xl.template updn<3>(v, s, m, p);
    const double k1 = A * m[1];
    const double k2 = C * p[1];
    const double nA = -m[0] * k1;
    const double nC = -p[2] * k2;
    const double nB = B - m[2] * k1 - p[0] * k2;
    A = nA; B = nB; C = nC;
    F.k1_[t] = k1;
    F.k2_[t] = k2;
  }
  F.invB_ = fast_rcp(B);
}

template <int R>
__device__ void pfac_store(const PFac<R>& F, double* __restrict__ out, int lane) {
  constexpr int NI = PFac<R>::NI;
  int f = 0;
#pragma unroll
  for (int r = 0; r < NI; ++r) out[(f++) * 64 + lane] = F.inv_[r];
#pragma unroll
  for (int r = 0; r < NI; ++r) out[(f++) * 64 + lane] = F.cp_[r];
#pragma unroll
  for (int r = 0; r < NI; ++r) out[(f++) * 64 + lane] = F.ls_[r];
#pragma unroll
  for (int r = 0; r < NI; ++r) out[(f++) * 64 + lane] = F.us_[r];
  out[(f++) * 64 + lane] = F.as_;
  out[(f++) * 64 + lane] = F.cs_;
#pragma unroll
  for (int t = 0; t < kPcrLevels; ++t) out[(f++) * 64 + lane] = F.k1_[t];
#pragma unroll
  for (int t = 0; t < kPcrLevels; ++t) out[(f++) * 64 + lane] = F.k2_[t];
  out[(f++) * 64 + lane] = F.invB_;
}

// ---- solve K right-hand sides in place (F: PFac in registers or TFac from a table) -----------
// SPIKE form: interior Thomas in place, the separator system by PCR, then every interior row adds
// its two spike responses (two independent FMAs per row instead of a second elimination pass).
template <int R, int K, int XM, class Fac, class Coef>
__device__ void psolve(const Fac& F, const Coef& coef, double (&d)[K][R], const Xl<XM>& xl, int lane) {
  double D[K];
  if constexpr (R == 1) {
#pragma unroll
    for (int k = 0; k < K; ++k) D[k] = d[k][0];
  } else {
    {
      const double i0 = F.inv(0);
#pragma unroll
      for (int k = 0; k < K; ++k) d[k][0] *= i0;
    }
#pragma unroll
    for (int r = 1; r < R - 1; ++r) {
      const double a = coef.a(r), ir = F.inv(r);
#pragma unroll
      for (int k = 0; k < K; ++k) d[k][r] = (d[k][r] - a * d[k][r - 1]) * ir;
    }
#pragma unroll
    for (int r = R - 3; r >= 0; --r) {
      const double c = F.cp(r);
#pragma unroll
      for (int k = 0; k < K; ++k) d[k][r] -= c * d[k][r + 1];
    }
    const double as = F.as(), cs = F.cs();
#pragma unroll
    for (int k = 0; k < K; ++k) D[k] = d[k][R - 1] - as * d[k][R - 2] - cs * shfl_dn1<XM>(d[k][0]);
  }
#pragma unroll
  for (int t = 0; t < kPcrLevels; ++t) {
    const int s = 1 << t;
    double Dm[K], Dp[K];
    xl.template updn<K>(D, s, Dm, Dp);
    const double k1 = F.k1(t), k2 = F.k2(t);
#pragma unroll
    for (int k = 0; k < K; ++k) D[k] = D[k] - k1 * Dm[k] - k2 * Dp[k];
  }
  const double invB = F.invB();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double y = D[k] * invB;
    if constexpr (R == 1) {
      d[k][0] = y;
    } else {
      const double yl = shfl_up1<XM>(y);
#pragma unroll
      for (int r = 0; r < R - 1; ++r) d[k][r] += yl * F.ls(r) + y * F.us(r);
      d[k][R - 1] = y;
    }
  }
}

// ---- two-wave lines: spike right-hand side and interface -----------------------------------
// this half's spike right-hand side: its coupling coefficient at its boundary row (half 0: the
// upper coefficient of row HR - 1, lane 63; half 1: the lower coefficient of row HR, lane 0)
template <int R, class Coef, class G>
__device__ __forceinline__ void spike_rhs(double (&z)[R], const Coef& coef, const G& g, int lane) {
#pragma unroll
  for (int r = 0; r < R; ++r) z[r] = 0.0;
  if (g.h == 0) {
    if (lane == 63) {
      double a, b, c;
      coef.abc(R - 1, a, b, c);
      z[R - 1] = c;
    }
  } else if (lane == 0) {
    z[0] = coef.a(0);
  }
}
// rows 0 .. K-1 of d hold this half's local solutions, spk its spike: solve the 2 x 2 interface
// system for x(HR - 1), x(HR) and subtract the spike times the partner's interface unknown.  Both
// halves form the same numbers in the same order, so the interface values are bitwise shared.
template <int R, int K, int KT, class G>
__device__ void spike_join(double (&d)[KT][R], const double (&spk)[R], const G& g, int lane) {
  static_assert(K <= KT, "rows");
  if constexpr (G::kH == 2) {
    static_assert(K + 1 <= LineG<2>::kXK, "exchange slot too small");
    // the boundary lane writes its rows straight into the slot (no cross-lane broadcast)
    double* mine = g.slot();
    if (lane == (g.h == 0 ? 63 : 0)) {
#pragma unroll
      for (int k = 0; k < K; ++k) mine[k] = g.h == 0 ? d[k][R - 1] : d[k][0];
      mine[K] = g.h == 0 ? spk[R - 1] : spk[0];
    }
    const double* theirs = g.post();
    const double ts = theirs[K], ms = mine[K];
    const double v = g.h == 0 ? ms : ts, w = g.h == 0 ? ts : ms;
    const double idet = 1.0 / (1.0 - v * w);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double tk = theirs[k], mk = mine[k];
      const double a0 = g.h == 0 ? mk : tk, b0 = g.h == 0 ? tk : mk;
      const double xl = (a0 - v * b0) * idet;  // row HR - 1
      const double xf = b0 - w * xl;           // row HR
      const double cc = g.h == 0 ? xf : xl;
#pragma unroll
      for (int r = 0; r < R; ++r) d[k][r] -= cc * spk[r];
    }
  }
  (void)lane;
}
// 3-point stencils across the half boundary, in split phases so that the partner's latency hides
// behind the stencil: stage (lane 0 publishes the half's first rows, lane 63 its last rows), the
// stencil itself with zero neighbours at the half boundary (the in-wave shifts zero-fill), then
// finish: row HR (lane 0 of half 1) adds its lower coefficient times the partner's last row, row
// HR - 1 (lane 63 of half 0) its upper coefficient times the partner's first row.
template <int R, int K, class G>
__device__ __forceinline__ void halo_stage(const double (&x)[K][R], const G& g, int lane) {
  if constexpr (G::kH == 2) {
    static_assert(2 * K <= LineG<2>::kXK, "exchange slot too small");
    double* mine = g.slot();
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < K; ++k) mine[k] = x[k][0];
    if (lane == 63)
#pragma unroll
      for (int k = 0; k < K; ++k) mine[K + k] = x[k][R - 1];
  }
  (void)x, (void)lane;
}
template <int R, int K, class G>
__device__ __forceinline__ void halo_finish(double (&out)[K][R], double a0, double cl, const G& g, int lane) {
  if constexpr (G::kH == 2) {
    const double* theirs = g.post();
    if (g.h == 1 && lane == 0)
#pragma unroll
      for (int k = 0; k < K; ++k) out[k][0] += a0 * theirs[K + k];
    if (g.h == 0 && lane == 63)
#pragma unroll
      for (int k = 0; k < K; ++k) out[k][R - 1] += cl * theirs[k];
  }
  (void)out, (void)a0, (void)cl, (void)lane;
}

// ---- stencils ----------------------------------------------------------------------------
// value at global row j (wave-uniform j); returns 0 if j out of range
template <int R, int XM>
__device__ __forceinline__ double row_value(const double (&x)[R], int j, int lane) {
  const int src = j / R, rr = j - src * R;
  double v = 0.0;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (r == rr) v = x[r];
  return bcast<XM>(v, src);
}

// out = tridiag(lo, c, up) * x with per-row tables (c = mask for M); cl, cc, cu scale the three
// diagonals of a second table set added on top (fused (cA A + cB B) x, see apply_tri2)
template <int R, int K, int XM, class G = LineG<1>>
__device__ void apply_tri(const double* __restrict__ lo, const double* __restrict__ cc, const double* __restrict__ up,
                          const double (&x)[K][R], double (&out)[K][R], int lane, const G& g = G{}) {
  double L[K], Rt[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    L[k] = shfl_up1<XM>(x[k][R - 1]);
    Rt[k] = shfl_dn1<XM>(x[k][0]);
  }
  halo_stage<R, K>(x, g, lane);
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
  if constexpr (G::kH == 2) halo_finish<R, K>(out, tab(lo, 0, lane), tab(up, R - 1, lane), g, lane);
}

// out = (sA A + sB B) x for two tridiagonal table sets A = (alo, ac, aup), B = (blo, bc, bup)
// (the explicit RK3 operator (1 - dt a nu k^2) M + dt a nu K in one pass, no M x / K x temporaries)
template <int R, int K, int XM, class G = LineG<1>>
__device__ void apply_tri2(const double* __restrict__ alo, const double* __restrict__ ac,
                           const double* __restrict__ aup, double sA, const double* __restrict__ blo,
                           const double* __restrict__ bc, const double* __restrict__ bup, double sB,
                           const double (&x)[K][R], double (&out)[K][R], int lane, const G& g = G{}) {
  double L[K], Rt[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    L[k] = shfl_up1<XM>(x[k][R - 1]);
    Rt[k] = shfl_dn1<XM>(x[k][0]);
  }
  halo_stage<R, K>(x, g, lane);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const double a = sA * tab(alo, r, lane) + sB * tab(blo, r, lane);
    const double b = sA * tab(ac, r, lane) + sB * tab(bc, r, lane);
    const double c = sA * tab(aup, r, lane) + sB * tab(bup, r, lane);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double xm = (r == 0) ? L[k] : x[k][r - 1];
      const double xp = (r == R - 1) ? Rt[k] : x[k][r + 1];
      out[k][r] = a * xm + b * x[k][r] + c * xp;
    }
  }
  if constexpr (G::kH == 2)
    halo_finish<R, K>(out, sA * tab(alo, 0, lane) + sB * tab(blo, 0, lane), sA * tab(aup, R - 1, lane) + sB * tab(bup, R - 1, lane),
                      g, lane);
}

// D1 right-hand side B1 f: the 3-point interior stencil with the one-sided wall closures folded
// into rows 0 and N-1 of the tables; the closures' third points are f_2 (row 0: lane 0's own
// register when R >= 3) and f_{N-3} (row N-1 at the wave-uniform slot rN: one scalar branch)
template <int R, int K, int XM, class G = LineG<1>>
__device__ void d1_rhs(const YTab& t, const double (&x)[K][R], double (&out)[K][R], int lane, const G& g = G{}) {
  apply_tri<R, K, XM>(t.d1_rm, t.d1_rc, t.d1_rp, x, out, lane, g);
  const int N = t.N;
  // row N - 1 in its half (two-wave lines: the host keeps rows N - 3 .. N - 1 in one half)
  const int hN = (N - 1) / (64 * R), jN = (N - 1) - hN * 64 * R;
  const int lN = jN / R, rN = jN - lN * R;  // wave-uniform
  static_assert(G::kH == 1 || R >= 3, "two-wave lines need R >= 3");
  if constexpr (R >= 3) {
    const double cp2 = (lane == 0 && g.h == 0) ? t.w0[2] : 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) out[k][0] += cp2 * x[k][2];
    const double cm2 = (lane == lN && g.h == hN) ? t.wN[2] : 0.0;
    switch (rN) {
#define CH_D1_RM2(RR)                                                                  \
  case RR:                                                                             \
    if constexpr (RR < R) {                                                            \
      _Pragma("unroll") for (int k = 0; k < K; ++k) {                                  \
        const double xm2 = RR >= 2 ? x[k][RR >= 2 ? RR - 2 : 0]                        \
                                   : shfl_up1<XM>(x[k][RR == 1 ? R - 1 : R - 2]);      \
        out[k][RR] += cm2 * xm2;                                                       \
      }                                                                                \
    }                                                                                  \
    break;
      CH_D1_RM2(0) CH_D1_RM2(1) CH_D1_RM2(2) CH_D1_RM2(3) CH_D1_RM2(4) CH_D1_RM2(5) CH_D1_RM2(6)
      CH_D1_RM2(7) CH_D1_RM2(8) CH_D1_RM2(9) CH_D1_RM2(10) CH_D1_RM2(11) CH_D1_RM2(12)
      CH_D1_RM2(13) CH_D1_RM2(14) CH_D1_RM2(15) CH_D1_RM2(16) CH_D1_RM2(17) CH_D1_RM2(18)
      CH_D1_RM2(19) CH_D1_RM2(20) CH_D1_RM2(21) CH_D1_RM2(22) CH_D1_RM2(23)
#undef CH_D1_RM2
      default: break;
    }
  } else {
    // R <= 2 (NY <= 128): the closure points straddle lanes; broadcast them
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double f2 = row_value<R, XM>(x[k], 2, lane), g2 = row_value<R, XM>(x[k], N - 3, lane);
      if (lane == 0) out[k][0] += t.w0[2] * f2;
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (lane == lN && r == rN) out[k][r] += t.wN[2] * g2;
    }
  }
}

template <int K, int XM>
__device__ __forceinline__ void wave_sum_n(double (&v)[K]) {
  if constexpr (XM == kXlBperm) {
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

template <int XM>
__device__ __forceinline__ double wave_sum(double v) {
  double a[1] = {v};
  wave_sum_n<1, XM>(a);
  return a[0];
}
// sums over the whole line (both halves, added in the same order in each)
template <int K, int XM, class G>
__device__ __forceinline__ void line_sum_n(double (&v)[K], const G& g) {
  wave_sum_n<K, XM>(v);
  if constexpr (G::kH == 2) {
    double t[K];
    g.template exch<K>(v, t);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = g.h == 0 ? v[k] + t[k] : t[k] + v[k];
  }
}
template <int XM, class G>
__device__ __forceinline__ double line_sum(double v, const G& g) {
  double a[1] = {v};
  line_sum_n<1, XM>(a, g);
  return a[0];
}
// value at global row j of the line (wave-uniform j) in every lane of both halves
template <int R, int XM, class G>
__device__ __forceinline__ double line_row_value(const double (&x)[R], int j, const G& g, int lane) {
  if constexpr (G::kH == 1) {
    return row_value<R, XM>(x, j, lane);
  } else {
    const int hj = j / (64 * R);
    double m[1] = {hj == g.h ? row_value<R, XM>(x, j - hj * 64 * R, lane) : 0.0}, t[1];
    g.template exch<1>(m, t);
    return hj == g.h ? m[0] : t[0];
  }
}

// ---- operators on whole lines ------------------------------------------------------------
// out = D1 x (compact first derivative): B1 x, then the constant factorisation from its table
template <int R, int K, int XM, class G = LineG<1>>
__device__ __forceinline__ void d1_apply_to(const YTab& t, const double (&x)[K][R], double (&out)[K][R],
                                            const Xl<XM>& xl, int lane, const G& g = G{}) {
  d1_rhs<R, K, XM>(t, x, out, lane, g);
  const TFac<R> F{t.d1fac, lane};
  const CoefD1 cd{t, lane};
  psolve<R, K, XM>(F, cd, out, xl, lane);
  if constexpr (G::kH == 2) {
    double spk[R];
#pragma unroll
    for (int r = 0; r < R; ++r) spk[r] = tab(t.d1spk, r, lane);
    spike_join<R, K, K>(out, spk, g, lane);
  }
}
template <int R, int K, int XM, class G = LineG<1>>
__device__ __forceinline__ void apply_M(const YTab& t, const double (&x)[K][R], double (&o)[K][R], int lane,
                                        const G& g = G{}) {
  apply_tri<R, K, XM>(t.m_lo, t.mask, t.m_up, x, o, lane, g);
}
template <int R, int K, int XM, class G = LineG<1>>
__device__ __forceinline__ void apply_K(const YTab& t, const double (&x)[K][R], double (&o)[K][R], int lane,
                                        const G& g = G{}) {
  apply_tri<R, K, XM>(t.k_lo, t.k_c, t.k_up, x, o, lane, g);
}

}  // namespace dev
}  // namespace channel
