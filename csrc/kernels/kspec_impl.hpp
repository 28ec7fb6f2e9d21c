// K-SPEC: the fused spectral (y-line) substep kernel.
//
// Per (kx,kz) line it does everything the reference does in y between two FFT rounds
// (SURVEY §7.3 K-SPEC-A/B):
//   calcHvg/calcHvv (nonLinear_kernels.cu:94-190), rk_step_1/2 (RK3_kernels.cu:6-153),
//   implicitSolver_double x2 (implicitStep_nu_double.cu:227-247), bilaplaSolver_double
//   (bilplacSolver_double.cu:320-348: implicit phi, Helmholtz v, D1 v, influence matrix),
//   meanURKstep_1/2 + forcing (meanUevol.c:201-221, 439-567, on the device for line (0,0)),
//   calcUW (nonLinear_kernels.cu:8-92), the wz/wx D1 calls and calcOmega
//   (convolution.c:7-20, convolution_kernels.cu:7-66), calcSt plane sums (statistics.cu:7-95).
// The reference runs these as ~50 launches + 44 cusparse calls + 8 D2D copies per substep with
// float<->double casts through HBM.  Here one launch reads 7 fields (5 on the first substep) and
// writes the states phi and omega, R_phi and R_omega (not on the last substep: the next one has
// zeta = 0) and the physical-stage inputs: u, v, w, omega_x, omega_z (the six-output mode, one
// rank and P >= 5: 9 stores, 7 on the last substep; the omega state is the omega_y field) or v,
// D1 v, D1 omega, from which the x-backward forms the six fields (XArgs::combine, P = 2..4: 7
// stores, 5 on the last substep).  All y-work is fp64 in registers, and the wall-normal
// operators are applied in "M-form" (the compact D2 mass matrix multiplies the equation), so the
// explicit viscous term needs no solve at all.
//
// Layout: one wave per line (lane l holds rows l*R .. l*R+R-1), W lines per workgroup, one
// persistent workgroup per CU walking tiles of W lines.  Per CU the LDS holds the coefficient
// tables (staged once), two staging tiles [r][lane][line] (pitch W+1: conflict-free column
// reads; global side: W consecutive complex values per y row) and one cross-lane scratch line per
// wave for the PCR strides >= 4 (yline_device.hpp, kXlLds).  The register budget is laid out for
// 2 waves per SIMD at 8 lines (fp32, R <= 8): the solves work in place (SPIKE form), the constant
// D1 factorisation is read from LDS where it is used, and only NS input fields are prefetched into
// registers (distance NS in the input sequence; the next tile's first inputs are issued before the
// last solve of the current one).
// This header holds the kernel template; kspec.hip (PAR = 0) and kspec_par*.hip (the parity
// variants) instantiate it in separate translation units so they compile in parallel.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "channel/common.hpp"
#include "channel/fft_device.hpp"
#include "channel/kernels.hpp"
#include "channel/kspec_config.hpp"
#include "channel/yline_device.hpp"

namespace channel {

using namespace dev;

// async global->LDS staging of the inputs where it applies (R > 8 with two tiles); compile with
// -DCH_KSPEC_GLDS=0 for the address-only A/B
constexpr bool kspec_glds_enabled() {
#if defined(CH_KSPEC_GLDS) && CH_KSPEC_GLDS == 0
  return false;
#else
  return true;
#endif
}

// ------------------------------------------------------------------------------------------
// Staging of W lines through an LDS tile (double-buffered where tile2 is set) with NS register
// prefetch slots (or address-only slots where registers are short: R > 8).
// Tile layout: y-major, row y at y*PITCH + (y/R)*G (W lines + 1 pad slot per row).  A wave's
// column read (rows lane*R + r) then strides R*PITCH + G slots between lanes, an odd number of
// 8-B words, which spreads the 32 lanes of each ds_read_b64 half over all 64 banks; G = 1 fixes
// the parity for even R.  Thread t of the cooperative copies handles rows t/W + 64 q of line t%W,
// so both the LDS and the global addresses are one base plus compile-time / scalar offsets.
//
// R > 8 (the VGPR cap leaves no room for register slots) with two tiles: the prefetch is an
// asynchronous global->LDS copy (global_load_lds_dword, no VGPRs) of the W lines' rows into the
// spare tile in their global order [y][W lines] (8 lanes per row, one dword each: the rows start
// at 8-byte boundaries only, lines = nkx_loc * nkz may be odd); commit() waits for it and reads
// the column from that raw image (4-way LDS bank conflicts on the column read, against an HBM
// round trip per field that the address-only slots exposed: 60 % of the R = 10 kernel's cycles
// sat in the input phases).  Lines past the end (the last tile) copy the last line, rows >= N
// are not copied and read as zero.  One field ahead only (one spare tile), and the next tile's
// first field goes out after the output stores, which use both tiles; at R <= 8 the register
// slots (two fields ahead, the next tile's issued during the D1 solve) measured faster
// (profiles/r03s3/ab_kspec_glds_r7.txt).
// H = 2 (lines over two waves): the tile holds 64 R H rows, wave half h reads rows h 64R + lane R + r.
template <int R, typename T, int W, int NS, bool GL = false, int H = 1>
struct Stage {
  using T2 = typename Cplx<T>::type;
  static constexpr int PITCH = W + 1;
  static constexpr int G = (R * PITCH) % 2 == 1 ? 0 : 1;
  static constexpr int TILE = 64 * R * H * PITCH + (G ? 64 * H : 0);
  static constexpr int RPB = 64 * H;  // rows per copy pass: W * 64 H threads / W lines
  static_assert(!GL || H == 1, "async LDS staging: one wave per line");
  static constexpr bool kRegSlots = R <= 8;
  static constexpr int DPE = static_cast<int>(sizeof(T2)) / 4;  // dwords per element
  static constexpr int DPR = W * DPE;                             // dwords per raw row
  static constexpr bool kGldsOk = 64 % DPR == 0;
  static_assert(!GL || (kGldsOk && kspec_glds_enabled()), "async LDS staging needs 64 % (W * dwords) == 0");
  T2* tile;   // buffer of the last staging (column() reads it)
  T2* tile2;  // the other buffer (nullptr: single-buffered)
  int N, lines, line0, w, lane;
  // spectral layout (spec_index): element (y, line) at rowoff(y) + lineoff(line); rows y and y + 64
  // are 64 * rs = 64 * lines elements apart in either layout
  int kzb = 0;
  unsigned rs = 0;
  int h = 0;  // this wave's half of its line (H = 2)
  // Per-thread element offset of (row y0 = tid / W, line line0 + tid % W) and of one 64-row pass:
  // re-derived per tile through an opaque copy, so the per-field addresses are formed at their
  // use (a 64-bit field base + a 32-bit offset: global_load/store saddr forms) instead of being
  // hoisted out of the tile loop into ~2 registers per field
  unsigned toff = 0, pstride = 0;
  T2 pend[kRegSlots ? NS : 1][R];
  const T2* dsrc[kRegSlots || GL ? 1 : NS];
  unsigned doff[kRegSlots || GL ? 1 : NS];

  static __device__ __forceinline__ int row_off(int y) { return y * PITCH + (G ? (y / R) : 0); }
  // row of this thread in a copy pass, laundered like toff: the per-q row masks and clamped offsets
  // derived from it are loop invariants the compiler would otherwise keep live (or spill) across
  // the whole tile loop
  static __device__ __forceinline__ int copy_row() {
    int y0 = static_cast<int>(threadIdx.x) / W;
    asm volatile("" : "+v"(y0));
    return y0;
  }
  __device__ __forceinline__ void set_layout(int kzb_) {
    kzb = kzb_;
    rs = static_cast<unsigned>(lines);
  }
  __device__ __forceinline__ unsigned lineoff(int line) const { return static_cast<unsigned>(spec_line_off(kzb, line)); }
  __device__ __forceinline__ unsigned rowoff(int y) const { return static_cast<unsigned>(spec_row_off(kzb, lines, y)); }
  __device__ __forceinline__ unsigned thread_off(int l0) const {
    const int y0 = threadIdx.x / W, l = threadIdx.x % W;
    unsigned o = rowoff(y0) + lineoff(min(l0 + l, lines - 1));
    asm volatile("" : "+v"(o));
    return o;
  }
  __device__ __forceinline__ void set_line0(int l0) {
    line0 = l0;
    toff = thread_off(l0);
  }
  __device__ __forceinline__ void next_tile() {
    if (tile2) {
      T2* t = tile2;
      tile2 = tile;
      tile = t;
    } else {
      lds_barrier();  // single buffer: the previous staging's reads must be done
    }
  }
  // Issue the global loads of a field (rows y0 + 64 q, q < R, of this thread's line) without
  // waiting.  Unconditional loads (a guarded load becomes a branch and a vmcnt(0) wait per
  // element): rows >= N read row N-1 (never committed), lines >= lines read the last line (staged
  // but never stored).
  template <int S>
  __device__ __forceinline__ void prefetch_at(const T2* __restrict__ src, int l0) {
    const unsigned o = thread_off(l0);
    if constexpr (GL) {
      // rows y = RPI k + lane / DPR, dword lane % DPR of the row (line l0 + dw / DPE clamped to the
      // last line: lines >= lines are staged but never stored); instruction k (wave k % W) writes
      // LDS dwords 64 k .. 64 k + 63 of the spare tile
      constexpr int RPI = 64 / DPR;  // rows per instruction
      const int lane = __lane_id();
      const int ry = lane / DPR, dw = lane % DPR;
      const unsigned base = lineoff(min(l0 + dw / DPE, lines - 1)) * DPE + dw % DPE;
      const unsigned* srcd = reinterpret_cast<const unsigned*>(src);
      unsigned* dstd = reinterpret_cast<unsigned*>(tile2);
      const int ninst = (N + RPI - 1) / RPI;
      for (int k = w; k < ninst; k += W) {
        const int y = k * RPI + ry;
        if (y < N)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(srcd + (base + rowoff(y) * DPE)),
                                           (__attribute__((address_space(3))) void*)(dstd + 64 * k), 4, 0, 0);
      }
      (void)o;
    } else if constexpr (!kRegSlots) {
      dsrc[S] = src;
      doff[S] = o;
    } else {
      const int y0 = copy_row(), l = threadIdx.x % W;
      // rows >= N read row N-1 of the same (clamped) line
      const unsigned last = rowoff(N - 1) + lineoff(min(l0 + l, lines - 1));
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const unsigned oq = y0 + RPB * q < N ? o + static_cast<unsigned>(RPB * q) * rs : last;
        pend[S][q] = src[oq];
      }
    }
  }
  // Stage the prefetched field through the LDS tile and return this wave's line.  Rows >= N of
  // both tiles are zero from the start and never written (the solves keep padding rows at exactly
  // zero), so the column read needs no masks.
  template <int S>
  __device__ __forceinline__ void commit(double (&x)[2][R]) {
    next_tile();
    if constexpr (GL) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's share of the copy landed
      lds_barrier();                                   // ... and every other wave's
      const T2* c = tile + w;
      int ln = lane;  // (laundered: see copy_row)
      asm volatile("" : "+v"(ln));
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int y = ln * R + r;
        const T2 v = c[(y < N ? y : 0) * W];  // raw image: rows >= N were never written
        x[0][r] = y < N ? static_cast<double>(v.x) : 0.0;
        x[1][r] = y < N ? static_cast<double>(v.y) : 0.0;
      }
      return;
    }
    const int y0 = copy_row(), l = threadIdx.x % W;
    T2* const tb = tile + row_off(y0) + l;  // (G = 0: row q at a compile-time LDS offset from it)
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int y = y0 + RPB * q;
      if (y < N) {
        T2& dstl = G ? tile[row_off(y) + l] : tb[RPB * q * PITCH];
        if constexpr (kRegSlots) {
          dstl = pend[S][q];
        } else {
          dstl = dsrc[S][doff[S] + static_cast<unsigned>(RPB * q) * rs];
        }
      }
    }
    lds_barrier();
    column(x);
  }
  // This wave's line as it sits in the tile.  After store() the tile still holds the stored
  // field, so a value just written out can be re-read from LDS (at storage precision) without
  // a global round trip, as long as no staging has happened since.
  __device__ __forceinline__ void column(double (&x)[2][R]) const {
    const T2* c = tile + row_off(h * 64 * R + lane * R) + w;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const T2 v = c[r * PITCH];
      x[0][r] = static_cast<double>(v.x);
      x[1][r] = static_cast<double>(v.y);
    }
  }
  __device__ __forceinline__ void load(const T2* __restrict__ src, double (&x)[2][R]) {
    prefetch_at<0>(src, line0);
    commit<0>(x);
  }
  // rows >= N are written too: the operators keep them at exactly zero
  __device__ __forceinline__ void store(T2* __restrict__ dst, const double (&x)[2][R]) { store(dst, x[0], x[1]); }
  // Two fields stored through two given tiles behind ONE barrier (instead of one barrier per field).
  // The caller picks tiles whose previous readers have all passed a barrier since (STORE2).
  __device__ __forceinline__ void store2_into(T2* ta, T2* tb, T2* __restrict__ da, const double (&ra)[R],
                                              const double (&ia)[R], T2* __restrict__ db, const double (&rb)[R],
                                              const double (&ib)[R]) {
    {
      T2* ca = ta + row_off(h * 64 * R + lane * R) + w;
      T2* cb = tb + row_off(h * 64 * R + lane * R) + w;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        ca[r * PITCH] = T2{static_cast<T>(ra[r]), static_cast<T>(ia[r])};
        cb[r * PITCH] = T2{static_cast<T>(rb[r]), static_cast<T>(ib[r])};
      }
    }
    lds_barrier();
    const int y0 = copy_row(), l = threadIdx.x % W;
    const T2* const pa = ta + row_off(y0) + l;
    const T2* const pb = tb + row_off(y0) + l;
    if (line0 + l < lines) {
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const int y = y0 + RPB * q;
        if (y < N) {
          const unsigned o = toff + static_cast<unsigned>(RPB * q) * rs;
          da[o] = G ? ta[row_off(y) + l] : pa[RPB * q * PITCH];
          db[o] = G ? tb[row_off(y) + l] : pb[RPB * q * PITCH];
        }
      }
    }
  }
  // one field through a given tile (same rule)
  __device__ __forceinline__ void store_into(T2* t, T2* __restrict__ dst, const double (&re)[R], const double (&im)[R]) {
    {
      T2* c = t + row_off(h * 64 * R + lane * R) + w;
#pragma unroll
      for (int r = 0; r < R; ++r) c[r * PITCH] = T2{static_cast<T>(re[r]), static_cast<T>(im[r])};
    }
    lds_barrier();
    const int y0 = copy_row(), l = threadIdx.x % W;
    const T2* const tb = t + row_off(y0) + l;
    if (line0 + l < lines) {
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const int y = y0 + RPB * q;
        if (y < N) dst[toff + static_cast<unsigned>(RPB * q) * rs] = G ? t[row_off(y) + l] : tb[RPB * q * PITCH];
      }
    }
  }
  // (re, im) rows of a line, optionally scaled (wave-uniform)
  __device__ __forceinline__ void store(T2* __restrict__ dst, const double (&re)[R], const double (&im)[R],
                                        double sc = 1.0) {
    next_tile();
    {
      T2* c = tile + row_off(h * 64 * R + lane * R) + w;
#pragma unroll
      for (int r = 0; r < R; ++r) c[r * PITCH] = T2{static_cast<T>(sc * re[r]), static_cast<T>(sc * im[r])};
    }
    lds_barrier();
    const int y0 = copy_row(), l = threadIdx.x % W;
    const T2* const tb = tile + row_off(y0) + l;  // (G = 0: row q at a compile-time LDS offset from it)
    if (line0 + l < lines) {
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const int y = y0 + RPB * q;
        if (y < N) dst[toff + static_cast<unsigned>(RPB * q) * rs] = G ? tile[row_off(y) + l] : tb[RPB * q * PITCH];
      }
    }
  }
};

template <int R>
__device__ __forceinline__ void czero(double (&x)[2][R]) {
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int r = 0; r < R; ++r) x[k][r] = 0.0;
}

// overflow-safe cosh(l y)/cosh(l) and sinh(l y)/sinh(l) (and their y-derivatives), |y| <= 1, l > 0
__device__ __forceinline__ void chs_profiles(double l, double y, double& C, double& S, double& dC, double& dS) {
  const double ep = exp(l * (y - 1.0)), em = exp(-l * (y + 1.0)), e2 = exp(-2.0 * l);
  C = (ep + em) / (1.0 + e2);
  S = (ep - em) / (1.0 - e2);
  dC = l * (ep - em) / (1.0 + e2);
  dS = l * (ep + em) / (1.0 - e2);
}

// per-wave exchange scratch (kXlLds)
template <int R, int W, int H = 1>
constexpr int kspec_scratch_doubles() {
  return kspec_xmode<R, float>() == kXlLds ? W * H * xl_scratch_doubles(kKspecXK + (H == 2 ? 1 : 0)) : 1;
}
// staged tables: 13 row tables, the D1 factorisation (per half) and, for two halves, the D1 spikes
template <int R, typename T, int W, int H = 1>
constexpr int kspec_lds_tables_doubles() {
  return kYTabRowTables * 64 * R * H + PFac<R>::kNumFields * 64 * H + (H == 2 ? 64 * R * H : 0);
}
// stage the tables when tables + two tiles + the exchange scratch fit the 160 KB LDS; fp64 storage
// from R = 8 (whose double tiles alone take 82-102 KB): tables + ONE tile, the tables' per-row reads
// from LDS instead of L2 (read from global memory they were hoisted into registers: 74 / 143 spilled
// VGPRs at R = 8 / 10)
template <int R, typename T, int W, int H = 1>
constexpr bool kspec_tables_in_lds() {
  constexpr int tiles = (sizeof(T) == 8 && R >= 8) ? 1 : 2;
  return kspec_lds_tables_doubles<R, T, W, H>() * 8 +
             tiles * Stage<R, T, W, 1, false, H>::TILE * static_cast<int>(sizeof(typename Cplx<T>::type)) +
             kspec_scratch_doubles<R, W, H>() * 8 <=
         158 * 1024;
}
template <int R, typename T, int W, int H = 1>
constexpr bool kspec_double_tile() {
  return (kspec_tables_in_lds<R, T, W, H>() ? kspec_lds_tables_doubles<R, T, W, H>() * 8 : 0) +
             2 * Stage<R, T, W, 1, false, H>::TILE * static_cast<int>(sizeof(typename Cplx<T>::type)) +
             kspec_scratch_doubles<R, W, H>() * 8 <=
         158 * 1024;
}

// two extra store tiles (STORE2: paired output stores behind one barrier) where the LDS has room
template <int R, typename T, int W, int H = 1>
constexpr bool kspec_store2_tiles() {
  return H == 1 && kspec_double_tile<R, T, W, H>() &&
         (kspec_tables_in_lds<R, T, W, H>() ? kspec_lds_tables_doubles<R, T, W, H>() * 8 : 0) +
                 4 * Stage<R, T, W, 1, false, H>::TILE * static_cast<int>(sizeof(typename Cplx<T>::type)) +
                 kspec_scratch_doubles<R, W, H>() * 8 <=
             158 * 1024;
}

// Reference-parity variants (compile-time, PAR bits): kParDD = explicit viscous D2 as D1 o D1
// (RK3_kernels.cu:160-164, derivatives_nu_double.cu:440-446); kParAnalytic = analytic influence
// functions (bilplacSolver_double.cu:56-250, l1/l2 typo fixed).  The default (PAR = 0) is the
// compact D2 and discrete Green's functions; the parity code paths would otherwise set the
// register allocation of the default kernel.
constexpr int kParDD = 1, kParAnalytic = 2;

// GLM: 0 = async LDS staging where the registers are short (R > 8, two tiles), 1 = also at R <= 8
// in place of the register slots (one field ahead instead of NS)
// (A/B record, not kept: direct register->global stores instead of the tile transposes, 9 % slower
// at R = 7, profiles/r03s3/ab_kspec_ns7.txt)
// SPLIT: 0 = the whole substep in this kernel; 1 = stop after the phi / v stores (the D1 of v and
// omega, the statistics and the u, w, omega_x, omega_z outputs run in kspec_out_kernel)
// H = 2: every line runs on two waves of the workgroup (LineG<2>, yline_device.hpp), waves 0 .. W-1
// holding the first halves of the W lines and waves W .. 2W-1 the second halves
template <int R, typename T, int W, int NS, int XM, int PAR, int GLM = 0, int SPLIT = 0, int H = 1>
__global__ void __launch_bounds__(W * 64 * H) kspec_kernel(YTab tg, SpecArgs a) {
  using T2 = typename Cplx<T>::type;
  constexpr bool kGldsTile = H == 1 && (GLM == 1 || !Stage<R, T, W, 1>::kRegSlots) && Stage<R, T, W, 1>::kGldsOk &&
                             kspec_double_tile<R, T, W>() && kspec_glds_enabled();
  using St = Stage<R, T, W, NS, kGldsTile, H>;
  constexpr int HR = 64 * R;        // rows of one wave
  constexpr int ROWS = 64 * R * H;  // rows of a line (table stride)
  constexpr int NT = W * 64 * H;
  constexpr int NF = PFac<R>::kNumFields;
  // fp64 storage from R = 10 runs the six-output mode only (the solver never selects the combine
  // mode there): without the combine branch the register allocation of these spill-prone kernels
  // does not have to cover both output stages
  constexpr bool kSixOnly = sizeof(T) == 8 && R >= 10;
  const bool out6 = kSixOnly || a.out6;
  constexpr bool TLDS = kspec_tables_in_lds<R, T, W, H>();
  constexpr int NTAB = kspec_lds_tables_doubles<R, T, W, H>();
  constexpr bool kDoubleTile = kspec_double_tile<R, T, W, H>();
  constexpr int XS = xl_scratch_doubles(kKspecXK + (H == 2 ? 1 : 0));  // (+ the spike column)
  // LEAN: two waves per SIMD at R >= 5 (8 one-wave lines per workgroup, <= 256 registers): the
  // multi-RHS solves run two real right-hand sides (one complex field) at a time on the same
  // factorisation, so the 6- and 4-RHS working sets and their cross-lane temporaries are never
  // live at once (CHANNEL_KSPEC_W8, A/B)
  constexpr bool LEAN = H == 1 && W >= 8 && R >= 5;
  static_assert(H == 1 || (SPLIT == 0 && GLM == 0), "two-wave lines: the fused kernel");
  __shared__ double tab_lds[TLDS ? NTAB : 1];
  // STORE2: paired stores of the R fields and the outputs through two extra tiles (not with the
  // async staging, which fills the spare tile during the output stores; not in the split kernel)
  constexpr bool kStore2 = kspec_store2_tiles<R, T, W, H>() && !kGldsTile && SPLIT == 0;
  constexpr int NTILES = kStore2 ? 4 : (kDoubleTile ? 2 : 1);
  __shared__ T2 tile_mem[NTILES * St::TILE];
  __shared__ double xs_mem[kspec_scratch_doubles<R, W, H>()];
  __shared__ double lx_buf[H == 2 ? W * 4 * LineG<2>::kXK : 1];
  __shared__ int lx_flag[H == 2 ? W * 2 : 1];
  int lane = __lane_id();  // (re-laundered per tile in the LEAN variant: see the tile loop)
  const int wv = threadIdx.x / 64;
  const int w = wv % W;   // line slot of the tile
  const int hh = wv / W;  // half of the line (H = 2)
  const int N = a.N;
  if (a.lds_poison) {
    lds_poison_fill(tab_lds, sizeof(tab_lds));
    lds_poison_fill(tile_mem, sizeof(tile_mem));
    lds_poison_fill(xs_mem, sizeof(xs_mem));
    __syncthreads();
  }
  if constexpr (TLDS) {
    // coefficient tables (13 per-row tables + the D1 factorisation, contiguous from d1_lo) staged
    // once per block: every solve step reads them, and from L2 each read is a dependent load
    const double* src = tg.d1_lo;
    for (int i = threadIdx.x; i < NTAB; i += NT) tab_lds[i] = src[i];
  }
  LineG<H> g;
  if constexpr (H == 2) {
    g.h = hh;
    g.buf = lx_buf + w * 4 * LineG<2>::kXK;
    g.flag = lx_flag + w * 2;
    if (threadIdx.x < W * 2) lx_flag[threadIdx.x] = 0;
  }
  // this half's rows: the half's table is the one-wave table of its rows (YTablesDev::upload)
  const int thalf = hh * R * 64;
  // Table pointers re-derived at each phase from a laundered zero offset: the table reads are
  // loop-invariant, and without this LICM/GVN hoist every one of them out of the tile loop and
  // keep them live across all phases (13 tables x R + the D1 factor: ~260 registers at R = 7).
  // Within a phase the compiler still shares and schedules them freely.
  YTab t = tg;
  auto fresh = [&]() {
    int z = 0;
    asm volatile("" : "+v"(z));
    if constexpr (TLDS) {
      const double* b = tab_lds + z + thalf;
      t.d1_lo = b + 0 * ROWS;
      t.d1_up = b + 1 * ROWS;
      t.d1_rm = b + 2 * ROWS;
      t.d1_rc = b + 3 * ROWS;
      t.d1_rp = b + 4 * ROWS;
      t.m_lo = b + 5 * ROWS;
      t.m_up = b + 6 * ROWS;
      t.k_lo = b + 7 * ROWS;
      t.k_c = b + 8 * ROWS;
      t.k_up = b + 9 * ROWS;
      t.mask = b + 10 * ROWS;
      t.d1row0 = b + 11 * ROWS;
      t.d1rowN = b + 12 * ROWS;
      const double* f = tab_lds + z + kYTabRowTables * ROWS;
      t.d1fac = f + hh * NF * 64;
      if constexpr (H == 2) t.d1spk = f + H * NF * 64 + thalf;
    } else {
      t.d1_lo = tg.d1_lo + z + thalf;
      t.d1_up = tg.d1_up + z + thalf;
      t.d1_rm = tg.d1_rm + z + thalf;
      t.d1_rc = tg.d1_rc + z + thalf;
      t.d1_rp = tg.d1_rp + z + thalf;
      t.m_lo = tg.m_lo + z + thalf;
      t.m_up = tg.m_up + z + thalf;
      t.k_lo = tg.k_lo + z + thalf;
      t.k_c = tg.k_c + z + thalf;
      t.k_up = tg.k_up + z + thalf;
      t.mask = tg.mask + z + thalf;
      t.d1row0 = tg.d1row0 + z + thalf;
      t.d1rowN = tg.d1rowN + z + thalf;
      t.d1fac = tg.d1fac + z + hh * NF * 64;
      if constexpr (H == 2) t.d1spk = tg.d1spk + z + thalf;
    }
    t.trap = tg.trap + z + thalf;  // (the mean line's weights: otherwise R 64-bit addresses live across the tile loop)
  };
  // zero tiles: rows >= N stay zero for the whole kernel (Stage::commit)
  for (int i = threadIdx.x; i < NTILES * St::TILE; i += NT) tile_mem[i] = T2{0, 0};
  __syncthreads();
  const Xl<XM> xl{xs_mem + wv * XS};
  // statistics reduction [4][64 R] in the staging tiles: between the phi store and the output
  // stores nothing reads them, and the output stores rewrite every slot a column read uses
  // (padding rows included, with zeros) before the next staging
  double* sred = reinterpret_cast<double*>(tile_mem);
  static_assert(St::TILE * sizeof(T2) >= 4 * ROWS * sizeof(double), "tile too small for the statistics reduction");

  // Persistent blocks: the grid is the resident capacity and each block walks tiles of W lines.
  // XCD-aware order: at each iteration the blocks of one XCD take consecutive tiles, which share
  // partial 128-B lines in that L2.
  const int ntiles = (a.lines + W - 1) / W;
  const int lb = static_cast<int>(xcd_remap(blockIdx.x, gridDim.x));
  St st{tile_mem, kDoubleTile ? tile_mem + St::TILE : nullptr, N, a.lines, lb * W, w, lane};
  T2* const xt0 = tile_mem + 2 * St::TILE;  // (STORE2 only)
  T2* const xt1 = tile_mem + 3 * St::TILE;
  st.set_layout(a.kzb);
  st.h = hh;
  // global row of (lane, r) in this wave
  auto row = [&](int r) { return hh * HR + lane * R + r; };
  T2* phi = static_cast<T2*>(a.phi);
  T2* omega = static_cast<T2*>(a.omega);
  T2* Rphi = static_cast<T2*>(a.Rphi);
  T2* Romega = static_cast<T2*>(a.Romega);
  const bool zprev = a.rk_z != 0.0;
  // input sequence of mode 1: 0 H_x, 1 H_z, 2 H_y, 3 phi, 4 omega, 5 R_phi, 6 R_omega (5, 6 only
  // when the substep uses the previous nonlinear term); input i goes to slot i % NS and is
  // prefetched when input i - NS is committed
  constexpr int D = kGldsTile ? 1 : NS;  // (one spare tile: one field ahead)
  static_assert(D >= 1 && D <= 7, "prefetch distance: the first D inputs of a tile are issued explicitly");
  const int nin = zprev ? 7 : 5;
  auto src_of = [&](int i) -> const T2* {
    switch (i) {
      case 0: return static_cast<const T2*>(a.out[0]);
      case 1: return static_cast<const T2*>(a.out[2]);
      case 2: return static_cast<const T2*>(a.out[1]);
      case 3: return phi;
      case 4: return omega;
      case 5: return Rphi;
      default: return Romega;
    }
  };
  auto ahead = [&](auto ic, int l0) {
    constexpr int I = decltype(ic)::value;
    if constexpr (I < 7) {
      if (I < nin) st.template prefetch_at<I % NS>(src_of(I), l0);
    }
  };
  // the first D inputs of the tile starting at line l0
  auto ahead_first = [&](int l0) {
    ahead(std::integral_constant<int, 0>{}, l0);
    if constexpr (D > 1) ahead(std::integral_constant<int, 1>{}, l0);
    if constexpr (D > 2) ahead(std::integral_constant<int, 2>{}, l0);
    if constexpr (D > 3) ahead(std::integral_constant<int, 3>{}, l0);
    if constexpr (D > 4) ahead(std::integral_constant<int, 4>{}, l0);
    if constexpr (D > 5) ahead(std::integral_constant<int, 5>{}, l0);
    if constexpr (D > 6) ahead(std::integral_constant<int, 6>{}, l0);
  };
  if (a.mode == 1 && lb < ntiles) {
    ahead_first(lb * W);
  }
  // optional per-phase shader-clock accounting (CHANNEL_KSPEC_PROF)
  const bool prof_on = a.prof != nullptr;
  unsigned long long tprev = prof_on ? __builtin_amdgcn_s_memtime() : 0;
#define KSPEC_STAMP(k)                                            \
  if (prof_on) {                                                  \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    if (lane == 0) atomicAdd(&a.prof[k], now_ - tprev);           \
    tprev = now_;                                                 \
  }
  for (int tile = lb; tile < ntiles; tile += gridDim.x) {
    // the per-row masks and offsets derived from the lane (row < N, j == 0, ...) are loop
    // invariants; hoisted out of the tile loop they stay live across every phase (at the
    // 256-register cap of two waves per SIMD they were spilled)
    if constexpr (LEAN) asm volatile("" : "+v"(lane));
    const int line0 = tile * W;
    st.set_line0(line0);
    const int line = line0 + w;
    const bool valid = line < a.lines;
    const int next_line0 = (tile + static_cast<int>(gridDim.x)) * W;
    const bool has_next = a.mode == 1 && next_line0 < a.lines;

    const int ikx = valid ? line / a.nkz : 0;
    const int kz = valid ? a.kz0 + (line - ikx * a.nkz) : 0;
    const int ig = a.kx0 + ikx;
    const int kx = ig <= a.Kx ? ig : ig - a.nkx;
    const double al = a.ax * kx, be = a.az * kz;
    const double k2 = al * al + be * be;
    const bool is_mean = valid && kx == 0 && kz == 0;
    const double inv_k2 = k2 > 0.0 ? 1.0 / k2 : 0.0;
    // the mean line (al = be = 0) differs only by these terms: wave-uniform multipliers instead
    // of per-element selects
    const double mf = is_mean ? 1.0 : 0.0;

    double ph[2][R];  // phi (state)
    double vo[4][R];  // v (0, 1) and omega (2, 3; U(y) on the mean line): the final D1's operands
    double mean_diag_flux = 0.0, mean_C = 0.0;

    if (a.mode == 1) {
      const double dt = *a.dt;
      double RPn[2][R], RWn[2][R];
      fresh();
      // ---------------- nonlinear terms h_v, h_g in M-form ---------------------------------
      {
        double X[2][R], G[2][R];
        {
          double Hc[2][R];
          st.template commit<0 % NS>(Hc);  // H_x
          ahead(std::integral_constant<int, D>{}, line0);
#pragma unroll
          for (int r = 0; r < R; ++r) {
            X[0][r] = al * Hc[1][r];  // -i al Hx
            X[1][r] = -al * Hc[0][r];
            G[0][r] = mf * Hc[0][r] - be * Hc[1][r];  // i be Hx ; mean line: N(y) = Re Hx(0,0)
            G[1][r] = be * Hc[0][r];
          }
          st.template commit<1 % NS>(Hc);  // H_z
          ahead(std::integral_constant<int, 1 + D>{}, line0);
#pragma unroll
          for (int r = 0; r < R; ++r) {
            X[0][r] += be * Hc[1][r];  // -i be Hz
            X[1][r] -= be * Hc[0][r];
            G[0][r] += al * Hc[1][r];  // -i al Hz
            G[1][r] -= al * Hc[0][r];
          }
        }
        double Y[2][R];
        fresh();
        d1_apply_to<R, 2, XM>(t, X, Y, xl, lane, g);  // D(-i al Hx - i be Hz)
        st.template commit<2 % NS>(X);              // H_y (X is free)
        ahead(std::integral_constant<int, 2 + D>{}, line0);
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int r = 0; r < R; ++r) Y[k][r] -= k2 * X[k][r];
        fresh();
        apply_M<R, 2, XM>(t, Y, RPn, lane, g);
        apply_M<R, 2, XM>(t, G, RWn, lane, g);
        KSPEC_STAMP(0)
        if (a.mean_diag && is_mean) {
          int z = 0;  // (laundered like the tables: keeps the addresses out of the loop preheader)
          asm volatile("" : "+v"(z));
          double* md = a.mean_diag + N + z;
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int j = row(r);
            if (j < N) md[j] = G[0][r];
          }
        }
      }
      // ---------------- explicit part of the RK3 substep in M-form -------------------------
      // M rhs = M q + dt [ a_n nu (K q - k^2 M q) + g_n R_now + z_n R_prev ]
      double rhsP[2][R], rhsW[2][R];
      {
        const double cM = 1.0 - dt * a.rk_a * a.nu * k2, cK = dt * a.rk_a * a.nu, cg = dt * a.rk_g;
        auto explicit_op = [&](const double (&q)[2][R], double (&o)[2][R]) {
          if ((PAR & kParDD) && !is_mean) {
            // reference parity (RK3_kernels.cu:160-164, derivatives_nu_double.cu:440-446): the
            // explicit viscous D2 of the fluctuations as D1 o D1, M (cM q + cK D1 D1 q)
            double D1q[2][R], DD[2][R];
            d1_apply_to<R, 2, XM>(t, q, D1q, xl, lane, g);
            d1_apply_to<R, 2, XM>(t, D1q, DD, xl, lane, g);
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
              for (int r = 0; r < R; ++r) DD[k][r] = cM * q[k][r] + cK * DD[k][r];
            apply_M<R, 2, XM>(t, DD, o, lane, g);
          } else {
            apply_tri2<R, 2, XM>(t.m_lo, t.mask, t.m_up, cM, t.k_lo, t.k_c, t.k_up, cK, q, o, lane, g);
          }
        };
        double q[2][R];
        fresh();
        st.template commit<3 % NS>(q);  // phi
        ahead(std::integral_constant<int, 3 + D>{}, line0);
        explicit_op(q, rhsP);
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int r = 0; r < R; ++r) rhsP[k][r] += cg * RPn[k][r];
        fresh();
        st.template commit<4 % NS>(q);  // omega
        ahead(std::integral_constant<int, 4 + D>{}, line0);
        explicit_op(q, rhsW);
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int r = 0; r < R; ++r) rhsW[k][r] += cg * RWn[k][r];
        if (zprev) {
          const double cz = dt * a.rk_z;
          st.template commit<5 % NS>(q);  // R_phi
          ahead(std::integral_constant<int, 5 + D>{}, line0);
#pragma unroll
          for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int r = 0; r < R; ++r) rhsP[k][r] += cz * q[k][r];
          st.template commit<6 % NS>(q);  // R_omega
#pragma unroll
          for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int r = 0; r < R; ++r) rhsW[k][r] += cz * q[k][r];
        }
      }
      KSPEC_STAMP(1)
      if (a.store_r) {  // (the last substep's R is never read: the next substep has zeta = 0)
        if constexpr (kStore2) {
          st.store2_into(xt0, xt1, Rphi, RPn[0], RPn[1], Romega, RWn[0], RWn[1]);
        } else {
          st.store(Rphi, RPn);
          st.store(Romega, RWn);
        }
      }
      KSPEC_STAMP(2)

      // ---------------- implicit viscous solves (phi, omega share one factorisation) -------
      const double c = a.rk_b * dt * a.nu;
      double pp[4][R];  // phi particular (0, 1) and the two homogeneous phi solutions (2, 3)
      fresh();
      {
        PFac<R> F;
        const CoefImpl ci{t, lane, 1.0 + c * k2, c};
        // (two-wave lines: each half factors its own rows, the coupling to the other half dropped)
        pfactor<R, XM>(F, CutLo<CoefImpl>{ci, H == 2 && hh == 1 && lane == 0}, xl, lane);
        constexpr int KS = H == 2 ? 1 : 0;  // + the half's spike right-hand side
        if constexpr (LEAN) {
          psolve<R, 2, XM>(F, ci, rhsW, xl, lane);
          psolve<R, 2, XM>(F, ci, rhsP, xl, lane);
          int zl = 0;  // (laundered: the loop-invariant unit columns would otherwise be hoisted)
          asm volatile("" : "+v"(zl));
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int j = row(r) + zl;
            pp[0][r] = rhsP[0][r];
            pp[1][r] = rhsP[1][r];
            pp[2][r] = (j == 0) ? 1.0 : 0.0;
            pp[3][r] = (j == N - 1) ? 1.0 : 0.0;
          }
          psolve<R, 2, XM>(F, ci, *reinterpret_cast<double (*)[2][R]>(&pp[2][0]), xl, lane);
        } else {
          // omega, phi and the two homogeneous phi solutions (k=0 -> phi(-1)=1, k=1 -> phi(+1)=1)
          // share the factorisation: one solve with 6 real right-hand sides
          double Z[6 + KS][R];
          int zl = 0;  // (laundered: the loop-invariant unit columns would otherwise be hoisted)
          asm volatile("" : "+v"(zl));
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int j = row(r) + zl;
            Z[0][r] = rhsW[0][r];
            Z[1][r] = rhsW[1][r];
            Z[2][r] = rhsP[0][r];
            Z[3][r] = rhsP[1][r];
            Z[4][r] = (j == 0) ? 1.0 : 0.0;
            Z[5][r] = (j == N - 1) ? 1.0 : 0.0;
          }
          if constexpr (H == 2) spike_rhs<R>(Z[6], ci, g, lane);
          psolve<R, 6 + KS, XM>(F, ci, Z, xl, lane);
          spike_join<R, 6, 6 + KS>(Z, Z[6 + KS - 1], g, lane);
#pragma unroll
          for (int r = 0; r < R; ++r) {
            rhsW[0][r] = Z[0][r];
            rhsW[1][r] = Z[1][r];
            pp[0][r] = Z[2][r];
            pp[1][r] = Z[3][r];
            pp[2][r] = Z[4][r];
            pp[3][r] = Z[5][r];
          }
        }
        if (is_mean) {
          // constant flow rate: U += C * U1, U1 = response to a unit mean pressure gradient
          double fU = 0.0;
#pragma unroll
          for (int r = 0; r < R; ++r) fU += tab(t.trap, r, lane) * rhsW[0][r];
          fU = line_sum<XM>(fU, g);
          if (a.forcing == 0) {
            double one[1][R], U1[1 + KS][R];
            int zl = 0;  // (laundered: the loop-invariant 0/1 column would otherwise be hoisted)
            asm volatile("" : "+v"(zl));
#pragma unroll
            for (int r = 0; r < R; ++r) one[0][r] = (row(r) + zl < N) ? 1.0 : 0.0;
            apply_tri<R, 1, XM>(t.m_lo, t.mask, t.m_up, one, reinterpret_cast<double (&)[1][R]>(U1), lane, g);
            if constexpr (H == 2) spike_rhs<R>(U1[1], ci, g, lane);
            psolve<R, 1 + KS, XM>(F, ci, U1, xl, lane);
            spike_join<R, 1, 1 + KS>(U1, U1[KS], g, lane);
            double f1 = 0.0;
#pragma unroll
            for (int r = 0; r < R; ++r) f1 += tab(t.trap, r, lane) * U1[0][r];
            f1 = line_sum<XM>(f1, g);
            mean_C = f1 != 0.0 ? (a.Q - fU) / f1 : 0.0;
#pragma unroll
            for (int r = 0; r < R; ++r) rhsW[0][r] += mean_C * U1[0][r];
          } else {
            // reference forcing (meanUevol.c:201-221): constant added to interior points
            mean_C = (a.Q - fU) / 2.0;
#pragma unroll
            for (int r = 0; r < R; ++r) rhsW[0][r] += mean_C * tab(t.mask, r, lane);
          }
#pragma unroll
          for (int r = 0; r < R; ++r) rhsW[1][r] = 0.0;
          mean_diag_flux = fU;
        }
      }
      KSPEC_STAMP(3)
      st.store(omega, rhsW);
      KSPEC_STAMP(4)

      // ---------------- velocity recovery + influence matrix (v(+-1) = v'(+-1) = 0) --------
      fresh();
      {
        PFac<R> F;
        const CoefHelm chm{t, lane, k2};
        pfactor<R, XM>(F, CutLo<CoefHelm>{chm, H == 2 && hh == 1 && lane == 0}, xl, lane);
        constexpr int KS = H == 2 ? 1 : 0;
        double Y[4 + KS][R];  // v particular (0, 1), homogeneous v (2, 3) [, the half's spike]
        if constexpr (LEAN) {
          for (int hf = 0; hf < 2; ++hf) {  // (not unrolled: one copy of the solve)
            double(&Yh)[2][R] = *reinterpret_cast<double (*)[2][R]>(&Y[2 * hf][0]);
            apply_M<R, 2, XM>(t, *reinterpret_cast<const double (*)[2][R]>(&pp[2 * hf][0]), Yh, lane, g);
            psolve<R, 2, XM>(F, chm, Yh, xl, lane);
          }
        } else {
          apply_M<R, 4, XM>(t, pp, reinterpret_cast<double (&)[4][R]>(Y), lane, g);
          if constexpr (H == 2) spike_rhs<R>(Y[4], chm, g, lane);
          psolve<R, 4 + KS, XM>(F, chm, Y, xl, lane);
          spike_join<R, 4, 4 + KS>(Y, Y[4 + KS - 1], g, lane);
        }
        fresh();
        // wall derivatives v'(+-1) = first / last row of the dense D1 applied to v (no solves)
        double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const double g0 = tab(t.d1row0, r, lane), gN = tab(t.d1rowN, r, lane);
          acc[0] += g0 * Y[0][r];
          acc[1] += g0 * Y[1][r];
          acc[2] += gN * Y[0][r];
          acc[3] += gN * Y[1][r];
          acc[4] += g0 * Y[2][r];
          acc[5] += gN * Y[2][r];
          acc[6] += g0 * Y[3][r];
          acc[7] += gN * Y[3][r];
        }
        line_sum_n<8, XM>(acc, g);
        const double p0r = acc[0], p0i = acc[1], pNr = acc[2], pNi = acc[3];
        double h10 = acc[4], h1N = acc[5], h20 = acc[6], h2N = acc[7];
        if ((PAR & kParAnalytic) && k2 > 0.0 && dt > 1e-14) {
          // reference parity (bilplacSolver_double.cu:56-217): phi1,2 = (C_l1 -+ S_l1)/2,
          // v1,2 = D [(C_l1 -+ S_l1)/2 - (C_l2 -+ S_l2)/2], l1^2 = k^2 + Re/(beta dt), l2 = k,
          // D = 1/(l1^2 - l2^2); wall derivatives analytic, the particular one discrete
          const double l2 = sqrt(k2), l1 = sqrt(k2 + 1.0 / (a.rk_b * dt * a.nu)), Dd = 1.0 / (l1 * l1 - l2 * l2);
          double dh[2][2];  // [solution][wall]
#pragma unroll
          for (int wall = 0; wall < 2; ++wall) {
            const double yw = wall == 0 ? -1.0 : 1.0;
            double C1_, S1_, dC1, dS1, C2_, S2_, dC2, dS2;
            chs_profiles(l1, yw, C1_, S1_, dC1, dS1);
            chs_profiles(l2, yw, C2_, S2_, dC2, dS2);
            dh[0][wall] = Dd * (0.5 * (dC1 - dS1) - 0.5 * (dC2 - dS2));
            dh[1][wall] = Dd * (0.5 * (dC1 + dS1) - 0.5 * (dC2 + dS2));
          }
          h10 = dh[0][0];
          h1N = dh[0][1];
          h20 = dh[1][0];
          h2N = dh[1][1];
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int j = row(r);
            const bool in = j < N;
            const double yj = in ? a.ygrid[j] : 0.0;
            double C1_, S1_, dC1, dS1, C2_, S2_, dC2, dS2;
            chs_profiles(l1, yj, C1_, S1_, dC1, dS1);
            chs_profiles(l2, yj, C2_, S2_, dC2, dS2);
            pp[2][r] = in ? 0.5 * (C1_ - S1_) : 0.0;
            pp[3][r] = in ? 0.5 * (C1_ + S1_) : 0.0;
            Y[2][r] = in ? Dd * (0.5 * (C1_ - S1_) - 0.5 * (C2_ - S2_)) : 0.0;
            Y[3][r] = in ? Dd * (0.5 * (C1_ + S1_) - 0.5 * (C2_ + S2_)) : 0.0;
          }
        }
        const double det = h10 * h2N - h20 * h1N;
        const bool apply = !is_mean && k2 > 0.0 && dt > 1e-14 && det != 0.0;
        const double id = apply ? 1.0 / det : 0.0;
        // [h10 h20; h1N h2N] [C1; C2] = -[p0; pN]
        const double C1r = (-p0r * h2N + h20 * pNr) * id, C1i = (-p0i * h2N + h20 * pNi) * id;
        const double C2r = (-h10 * pNr + h1N * p0r) * id, C2i = (-h10 * pNi + h1N * p0i) * id;
        const double nz = (is_mean || k2 == 0.0) ? 0.0 : 1.0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          ph[0][r] = nz * (pp[0][r] + C1r * pp[2][r] + C2r * pp[3][r]);
          ph[1][r] = nz * (pp[1][r] + C1i * pp[2][r] + C2i * pp[3][r]);
          vo[0][r] = nz * (Y[0][r] + C1r * Y[2][r] + C2r * Y[3][r]);
          vo[1][r] = nz * (Y[1][r] + C1i * Y[2][r] + C2i * Y[3][r]);
        }
      }
      KSPEC_STAMP(5)
      {
        // omega was the last field staged (store above): re-read it from the tile, not from HBM
        double om[2][R];
        st.column(om);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          vo[2][r] = om[0][r];
          vo[3][r] = om[1][r];
        }
      }
      // (STORE2 with the combine outputs: phi goes out at the end, paired with D1 omega)
      if (!kStore2 || out6) st.store(phi, ph);
      KSPEC_STAMP(6)
      // the next tile's first inputs load during the D1 solve and the output stores (the async
      // LDS copies go out after the output stores instead: those use both tiles)
      if (!kGldsTile && has_next) {
        ahead_first(next_line0);
      }
    } else {
      // ---------------- prepare only: fields from the state --------------------------------
      fresh();
      double om[2][R];
      st.load(phi, ph);
      st.load(omega, om);
      PFac<R> F;
      const CoefHelm chm{t, lane, k2};
      pfactor<R, XM>(F, CutLo<CoefHelm>{chm, H == 2 && hh == 1 && lane == 0}, xl, lane);
      constexpr int KS = H == 2 ? 1 : 0;
      double v[2 + KS][R];
      apply_M<R, 2, XM>(t, ph, reinterpret_cast<double (&)[2][R]>(v), lane, g);
      if constexpr (H == 2) spike_rhs<R>(v[2], chm, g, lane);
      psolve<R, 2 + KS, XM>(F, chm, v, xl, lane);
      spike_join<R, 2, 2 + KS>(v, v[2 + KS - 1], g, lane);
      const double nz = (is_mean || k2 == 0.0) ? 0.0 : 1.0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        ph[0][r] = nz * ph[0][r];
        ph[1][r] = nz * ph[1][r];
        vo[0][r] = nz * v[0][r];
        vo[1][r] = nz * v[1][r];
        vo[2][r] = om[0][r];
        vo[3][r] = om[1][r];
      }
    }

    // ---------------- health check (non-finite state) ---------------------------------------
    if (a.health) {
      bool bad = false;
#pragma unroll
      for (int r = 0; r < R; ++r)
        bad |= !isfinite(ph[0][r]) || !isfinite(ph[1][r]) || !isfinite(vo[2][r]) || !isfinite(vo[3][r]);
      if (__any(bad) && lane == 0) atomicOr(a.health, 1u);
    }

    if constexpr (SPLIT == 1) {
      // the output stage reads v from out[1], omega and phi from the state
      st.store(static_cast<T2*>(a.out[1]), vo[0], vo[1]);
      if (a.mean_diag && is_mean && lane == 0) {
        a.mean_diag[3 * N + 2] = mean_diag_flux;
        a.mean_diag[3 * N + 3] = mean_C;
      }
      KSPEC_STAMP(9)
      if (kGldsTile && has_next) {
        ahead_first(next_line0);
      }
      continue;
    }
    // ---------------- prepare velocity / vorticity for the physical-space stage --------------
    fresh();
    double dvo[4][R];  // D1 v (0, 1), D1 omega (2, 3): one 4-RHS solve
    if constexpr (LEAN) {
      d1_apply_to<R, 2, XM>(t, *reinterpret_cast<const double (*)[2][R]>(&vo[0][0]),
                            *reinterpret_cast<double (*)[2][R]>(&dvo[0][0]), xl, lane, g);
      d1_apply_to<R, 2, XM>(t, *reinterpret_cast<const double (*)[2][R]>(&vo[2][0]),
                            *reinterpret_cast<double (*)[2][R]>(&dvo[2][0]), xl, lane, g);
    } else {
      d1_apply_to<R, 4, XM>(t, vo, dvo, xl, lane, g);
    }
    KSPEC_STAMP(7)
    // velocities u = i (al dv - be om)/k2, w = i (be dv + al om)/k2 (nonLinear_kernels.cu:55-72),
    // for the plane statistics (the x-backward forms them for the physical-space stage)
    auto vel_u = [&](int r, double& re, double& im) {
      const double ar = (al * dvo[0][r] - be * vo[2][r]) * inv_k2, ai = (al * dvo[1][r] - be * vo[3][r]) * inv_k2;
      re = mf * vo[2][r] - ai;  // mean line: U(y)
      im = ar;
    };
    auto vel_w = [&](int r, double& re, double& im) {
      const double br = (be * dvo[0][r] + al * vo[2][r]) * inv_k2, bi = (be * dvo[1][r] + al * vo[3][r]) * inv_k2;
      re = -bi;
      im = br;
    };
    // plane statistics (statistics.cu:7-95), fluctuations only, weight 2 for kz > 0
    if (a.stats) {
      __syncthreads();  // every wave is done with the tiles (last use: the phi store or the omega column)
      for (int i = threadIdx.x; i < 4 * ROWS; i += NT) sred[i] = 0.0;
      __syncthreads();
      if (valid && !is_mean) {
        const double wgt = kz == 0 ? 1.0 : 2.0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int idx = (hh * R + r) * 64 + lane;
          double ur, ui, wr, wi;
          vel_u(r, ur, ui);
          vel_w(r, wr, wi);
          atomicAdd(&sred[0 * ROWS + idx], wgt * (ur * ur + ui * ui));
          atomicAdd(&sred[1 * ROWS + idx], wgt * (vo[0][r] * vo[0][r] + vo[1][r] * vo[1][r]));
          atomicAdd(&sred[2 * ROWS + idx], wgt * (wr * wr + wi * wi));
          atomicAdd(&sred[3 * ROWS + idx], wgt * (ur * vo[0][r] + ui * vo[1][r]));
        }
      }
      __syncthreads();
      for (int i = threadIdx.x; i < 4 * ROWS; i += NT) {
        const int s = i / ROWS, rem = i - s * ROWS, hr = rem / 64, l = rem - hr * 64;
        const int j = (hr / R) * HR + l * R + hr % R;
        if (j < N) atomicAdd(&a.stats[s * N + j], sred[i]);
      }
      __syncthreads();  // sred is a staging tile again
    }
    KSPEC_STAMP(8)
    // Outputs for the physical-space stage: v, D1 v and D1 omega (+ the omega and phi states).  The
    // x-backward forms u, w, omega_x, omega_z from them per element (XArgs::combine): u, w from
    // (D1 v, omega) as above, and with D2 v = phi + k2 v (the Helmholtz identity of the compact D2
    // operator) omega_x = Dw - i be v = i (be phi + al D1 omega)/k2 and omega_z = i al v - Du =
    // i (be D1 omega - al phi)/k2 (convolution_kernels.cu:46-53; mean line: u = U, omega_z = -dU/dy).
    // Three field stores instead of five per substep, and the exchange of P > 1 moves five fields.
    if (out6) {
      // The six physical-stage fields themselves (u, v, w, omega_x, omega_z; omega_y is the omega
      // state): the x-backward then reads one field per tile (two planes of a kz block, whole 128-B
      // lines), while K-SPEC takes the same time with 9 or 7 stores (32.53 vs 32.54 ms/step at one
      // rank: profiles/r06/ab_start_combine_forcecomm.txt, kspec_write_size_combine.txt)
      // wx = Dw - i be v = i (be phi + al D1 omega)/k2 - (v terms that cancel), written as in the
      // reference's calcOmega with D(dv) = D2 v = phi + k2 v (convolution_kernels.cu:46-53)
      auto omx = [&](int r, double& re, double& im) {
        const double DDr = ph[0][r] + k2 * vo[0][r], DDi = ph[1][r] + k2 * vo[1][r];
        const double br = (be * DDr + al * dvo[2][r]) * inv_k2, bi = (be * DDi + al * dvo[3][r]) * inv_k2;
        re = -bi + be * vo[1][r];
        im = br - be * vo[0][r];
      };
      auto omz = [&](int r, double& re, double& im) {  // wz = i al v - Du ; mean line: -dU/dy
        const double DDr = ph[0][r] + k2 * vo[0][r], DDi = ph[1][r] + k2 * vo[1][r];
        const double ar = (al * DDr - be * dvo[2][r]) * inv_k2, ai = (al * DDi - be * dvo[3][r]) * inv_k2;
        re = -al * vo[1][r] + ai - mf * dvo[2][r];
        im = al * vo[0][r] - ar;
      };
      double x[2][R], x2[2][R];
      if constexpr (kStore2) {
        // v and u, then w and omega_x, behind one barrier each (tiles: the extra pair, then the
        // staging pair, whose last readers (the phi store) passed the first pair's barrier), then
        // omega_z through the extra tile of the first pair (its readers passed the second barrier)
#pragma unroll
        for (int r = 0; r < R; ++r) vel_u(r, x[0][r], x[1][r]);
        st.store2_into(xt0, xt1, static_cast<T2*>(a.out[1]), vo[0], vo[1], static_cast<T2*>(a.out[0]), x[0], x[1]);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          vel_w(r, x[0][r], x[1][r]);
          omx(r, x2[0][r], x2[1][r]);
        }
        st.store2_into(st.tile, st.tile2, static_cast<T2*>(a.out[2]), x[0], x[1], static_cast<T2*>(a.out[3]), x2[0], x2[1]);
#pragma unroll
        for (int r = 0; r < R; ++r) omz(r, x[0][r], x[1][r]);
        st.store_into(xt0, static_cast<T2*>(a.out[5]), x[0], x[1]);
      } else {
        st.store(static_cast<T2*>(a.out[1]), vo[0], vo[1]);  // v
#pragma unroll
        for (int r = 0; r < R; ++r) vel_u(r, x[0][r], x[1][r]);
        st.store(static_cast<T2*>(a.out[0]), x[0], x[1]);
#pragma unroll
        for (int r = 0; r < R; ++r) vel_w(r, x[0][r], x[1][r]);
        st.store(static_cast<T2*>(a.out[2]), x[0], x[1]);
#pragma unroll
        for (int r = 0; r < R; ++r) omx(r, x[0][r], x[1][r]);
        st.store(static_cast<T2*>(a.out[3]), x[0], x[1]);
#pragma unroll
        for (int r = 0; r < R; ++r) omz(r, x[0][r], x[1][r]);
        st.store(static_cast<T2*>(a.out[5]), x[0], x[1]);
      }
      goto outputs_done;
    }
    if constexpr (kStore2) {
      if (a.mode == 1) {
        // phi and D1 omega, then v and D1 v, behind one barrier each (tiles: the extra pair, whose
        // last readers (the R stores) passed the omega store's barrier; then the staging pair, whose
        // last readers (the omega column) passed the first pair's barrier); the closing barrier
        // keeps the next tile's first staging behind the second pair's copy-out
        st.store2_into(xt0, xt1, phi, ph[0], ph[1], static_cast<T2*>(a.out[2]), dvo[2], dvo[3]);
        st.store2_into(st.tile, st.tile2, static_cast<T2*>(a.out[1]), vo[0], vo[1], static_cast<T2*>(a.out[0]), dvo[0],
                       dvo[1]);
        lds_barrier();
        goto outputs_done;
      }
    }
    st.store(static_cast<T2*>(a.out[1]), vo[0], vo[1]);    // v
    st.store(static_cast<T2*>(a.out[0]), dvo[0], dvo[1]);  // D1 v
    st.store(static_cast<T2*>(a.out[2]), dvo[2], dvo[3]);  // D1 omega (mean line: dU/dy)
  outputs_done:
    if (a.mean_diag && is_mean) {
      const double d0 = line_row_value<R, XM>(dvo[2], 0, g, lane), dN = line_row_value<R, XM>(dvo[2], N - 1, g, lane);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int j = row(r);
        if (j < N) a.mean_diag[j] = vo[2][r];
      }
      if (lane == 0 && hh == 0) {
        a.mean_diag[3 * N + 0] = d0;
        a.mean_diag[3 * N + 1] = dN;
        a.mean_diag[3 * N + 2] = mean_diag_flux;
        a.mean_diag[3 * N + 3] = mean_C;
      }
    }
    KSPEC_STAMP(9)
    if (kGldsTile && has_next) {
      ahead_first(next_line0);
    }
  }  // tile loop
#undef KSPEC_STAMP
}

// K-SPEC output stage (split mode, after kspec_kernel<..., SPLIT = 1>): per line, v (out[1]) and
// omega in, D1 of omega and of v (two 2-RHS solves on the constant factorisation), the plane
// statistics (statistics.cu:7-95) and the D1 v / D1 omega outputs the x-backward forms u, w,
// omega_x, omega_z from (nonLinear_kernels.cu:8-92, convolution_kernels.cu:7-66).  Without the advance's registers (the
// k-dependent factorisations, the 6-RHS implicit solve) a line fits in <= 256 VGPRs at R <= 8, so
// W = 8 lines per workgroup run two waves per SIMD: the output half of the substep was the
// latency-bound half at one wave per SIMD (it reads 2 fields more than the fused kernel).
template <int R, typename T, int W, int XM>
__global__ void __launch_bounds__(W * 64) kspec_out_kernel(YTab tg, SpecArgs a) {
  using T2 = typename Cplx<T>::type;
  constexpr int NS = 3;  // register slots 0 (omega) and 2 (v)
  using St = Stage<R, T, W, NS, false>;
  constexpr int ROWS = 64 * R;
  constexpr bool TLDS = kspec_tables_in_lds<R, T, W>();
  constexpr int NTAB = kspec_lds_tables_doubles<R, T, W>();
  constexpr bool kDoubleTile = kspec_double_tile<R, T, W>();
  constexpr int XS = xl_scratch_doubles(4);
  __shared__ double tab_lds[TLDS ? NTAB : 1];
  __shared__ T2 tile_mem[(kDoubleTile ? 2 : 1) * St::TILE];
  __shared__ double xs_mem[XM == kXlLds ? W * XS : 1];
  const int lane = __lane_id();
  const int w = threadIdx.x / 64;
  const int N = a.N;
  if (a.lds_poison) {
    lds_poison_fill(tab_lds, sizeof(tab_lds));
    lds_poison_fill(tile_mem, sizeof(tile_mem));
    lds_poison_fill(xs_mem, sizeof(xs_mem));
    __syncthreads();
  }
  if constexpr (TLDS) {
    const double* src = tg.d1_lo;
    for (int i = threadIdx.x; i < NTAB; i += W * 64) tab_lds[i] = src[i];
  }
  YTab t = tg;
  auto fresh = [&]() {
    int z = 0;
    asm volatile("" : "+v"(z));
    if constexpr (TLDS) {
      const double* b = tab_lds + z;
      t.d1_lo = b + 0 * ROWS;
      t.d1_up = b + 1 * ROWS;
      t.d1_rm = b + 2 * ROWS;
      t.d1_rc = b + 3 * ROWS;
      t.d1_rp = b + 4 * ROWS;
      t.d1fac = b + kYTabRowTables * ROWS;
    } else {
      t.d1_lo = tg.d1_lo + z;
      t.d1_up = tg.d1_up + z;
      t.d1_rm = tg.d1_rm + z;
      t.d1_rc = tg.d1_rc + z;
      t.d1_rp = tg.d1_rp + z;
      t.d1fac = tg.d1fac + z;
    }
  };
  for (int i = threadIdx.x; i < (kDoubleTile ? 2 : 1) * St::TILE; i += W * 64) tile_mem[i] = T2{0, 0};
  __syncthreads();
  const Xl<XM> xl{xs_mem + w * XS};
  double* sred = reinterpret_cast<double*>(tile_mem);
  static_assert(St::TILE * sizeof(T2) >= 4 * ROWS * sizeof(double), "tile too small for the statistics reduction");

  const int ntiles = (a.lines + W - 1) / W;
  const int lb = static_cast<int>(xcd_remap(blockIdx.x, gridDim.x));
  St st{tile_mem, kDoubleTile ? tile_mem + St::TILE : nullptr, N, a.lines, lb * W, w, lane};
  st.set_layout(a.kzb);
  const T2* vin = static_cast<const T2*>(a.out[1]);
  const T2* omega = static_cast<const T2*>(a.omega);
  // inputs: omega (slot 0), v (slot 2); each slot is refilled with the next tile's field right
  // after its commit
  if (lb < ntiles) {
    st.template prefetch_at<0>(omega, lb * W);
    st.template prefetch_at<2>(vin, lb * W);
  }
  for (int tile = lb; tile < ntiles; tile += gridDim.x) {
    const int line0 = tile * W;
    st.set_line0(line0);
    const int line = line0 + w;
    const bool valid = line < a.lines;
    const int next_line0 = (tile + static_cast<int>(gridDim.x)) * W;
    const bool has_next = next_line0 < a.lines;
    const int ikx = valid ? line / a.nkz : 0;
    const int kz = valid ? a.kz0 + (line - ikx * a.nkz) : 0;
    const int ig = a.kx0 + ikx;
    const int kx = ig <= a.Kx ? ig : ig - a.nkx;
    const double al = a.ax * kx, be = a.az * kz;
    const double k2 = al * al + be * be;
    const bool is_mean = valid && kx == 0 && kz == 0;
    const double inv_k2 = k2 > 0.0 ? 1.0 / k2 : 0.0;
    const double mf = is_mean ? 1.0 : 0.0;

    // D1 omega (mean line: dU/dy), then D1 v: the outputs of the physical-space stage besides v and
    // the states (the x-backward forms u, w, omega_x, omega_z from them, kspec_kernel)
    double om[2][R], v[2][R], d[2][R];
    st.template commit<0>(om);
    if (has_next) st.template prefetch_at<0>(omega, next_line0);
    fresh();
    d1_apply_to<R, 2, XM>(t, om, d, xl, lane);
    double dU0 = 0.0, dUN = 0.0;
    if (a.mean_diag && is_mean) {
      dU0 = row_value<R, XM>(d[0], 0, lane);
      dUN = row_value<R, XM>(d[0], N - 1, lane);
    }
    st.store(static_cast<T2*>(a.out[2]), d[0], d[1]);
    st.template commit<2>(v);
    if (has_next) st.template prefetch_at<2>(vin, next_line0);
    fresh();
    d1_apply_to<R, 2, XM>(t, v, d, xl, lane);  // D1 v
    auto vel_u = [&](int r, double& re, double& im) {
      const double ar = (al * d[0][r] - be * om[0][r]) * inv_k2, ai = (al * d[1][r] - be * om[1][r]) * inv_k2;
      re = mf * om[0][r] - ai;  // mean line: U(y)
      im = ar;
    };
    auto vel_w = [&](int r, double& re, double& im) {
      const double br = (be * d[0][r] + al * om[0][r]) * inv_k2, bi = (be * d[1][r] + al * om[1][r]) * inv_k2;
      re = -bi;
      im = br;
    };
    if (a.stats) {
      __syncthreads();
      for (int i = threadIdx.x; i < 4 * ROWS; i += W * 64) sred[i] = 0.0;
      __syncthreads();
      if (valid && !is_mean) {
        const double wgt = kz == 0 ? 1.0 : 2.0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int idx = r * 64 + lane;
          double ur, ui, wr, wi;
          vel_u(r, ur, ui);
          vel_w(r, wr, wi);
          atomicAdd(&sred[0 * ROWS + idx], wgt * (ur * ur + ui * ui));
          atomicAdd(&sred[1 * ROWS + idx], wgt * (v[0][r] * v[0][r] + v[1][r] * v[1][r]));
          atomicAdd(&sred[2 * ROWS + idx], wgt * (wr * wr + wi * wi));
          atomicAdd(&sred[3 * ROWS + idx], wgt * (ur * v[0][r] + ui * v[1][r]));
        }
      }
      __syncthreads();
      for (int i = threadIdx.x; i < 4 * ROWS; i += W * 64) {
        const int s = i / ROWS, rem = i - s * ROWS, r = rem / 64, l = rem - r * 64;
        const int j = l * R + r;
        if (j < N) atomicAdd(&a.stats[s * N + j], sred[i]);
      }
      __syncthreads();
    }
    st.store(static_cast<T2*>(a.out[0]), d[0], d[1]);
    if (a.mean_diag && is_mean) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int j = lane * R + r;
        if (j < N) a.mean_diag[j] = om[0][r];
      }
      if (lane == 0) {
        a.mean_diag[3 * N + 0] = dU0;
        a.mean_diag[3 * N + 1] = dUN;
      }
    }
  }
}

// Split (advance kernel + output kernel), CHANNEL_KSPEC_SPLIT=1, at R = 5..7 (A/B; off by default:
// at the headline grid the two kernels took 3.30 + 1.08 ms per substep against 4.17 ms fused, the
// output kernel's 3 extra field reads costing more than its second wave per SIMD gains)
static int kspec_split_env() {
  static const int v = [] {
    const char* e = std::getenv("CHANNEL_KSPEC_SPLIT");
    return e ? std::atoi(e) : -1;
  }();
  return v;
}
template <int R, typename T>
constexpr bool kspec_split_default() {
  // the instantiated split: fp32 storage, R = 5..7, where the output kernel is spill-free at two
  // waves per SIMD (R = 8 and the fp64 slots spill at 256 VGPRs)
  return sizeof(T) == 4 && R >= 5 && R <= 7;
}
template <int R, typename T>
constexpr int kspec_out_lines() {
  return 8;
}

// CHANNEL_KSPEC_GLDS7=1: the R = 7 fp32 kernel (headline grid) with async LDS staging instead of
// its two register slots (A/B)
static bool kspec_glds7() {
  static const bool on = [] {
    const char* e = std::getenv("CHANNEL_KSPEC_GLDS7");
    return e && std::atoi(e) == 1;
  }();
  return on;
}

// CHANNEL_KSPEC_NS7=3: the R = 7 fp32 kernel with three register prefetch slots (A/B)
static int kspec_ns7() {
  static const int ns = [] {
    const char* e = std::getenv("CHANNEL_KSPEC_NS7");
    return e ? std::atoi(e) : 0;
  }();
  return ns;
}

// CHANNEL_KSPEC_W8=1: the R = 7 fp32 kernel at 8 lines per workgroup, two waves per SIMD (LEAN
// solves, async LDS staging instead of register slots; A/B against the one-wave-per-SIMD default)
static bool kspec_w8() {
  static const bool on = [] {
    const char* e = std::getenv("CHANNEL_KSPEC_W8");
    return e && std::atoi(e) == 1;
  }();
  return on;
}

// CHANNEL_KSPEC_VAR = w4 | ns2 | ns5 | ns7 (A/B at R = 3, the small grids): 4 lines per block
// instead of 8, or 2 / 5 / 7 register prefetch slots (5 and 7: every input of a tile issued at
// its start, one exposed memory latency instead of one per prefetch window)
static int kspec_var_env() {
  static const int v = [] {
    const char* e = std::getenv("CHANNEL_KSPEC_VAR");
    if (!e) return 0;
    const std::string s(e);
    return s == "w4" ? 1 : (s == "ns2" ? 2 : (s == "ns7" ? 3 : (s == "ns5" ? 4 : 0)));
  }();
  return v;
}

template <int R, typename T, int PAR = 0>
static void kspec_launch_t(const YTablesDev& t, const SpecArgs& a, hipStream_t stream) {
  if constexpr (R == 3 && PAR == 0) {
    if (const int v = kspec_var_env()) {
      constexpr int W3 = 4;
      auto k = v == 1   ? kspec_kernel<3, T, W3, 1, kspec_xmode<3, T>(), 0>
               : v == 3 ? kspec_kernel<3, T, 8, 7, kspec_xmode<3, T>(), 0>
               : v == 4 ? kspec_kernel<3, T, 8, 5, kspec_xmode<3, T>(), 0>
                        : kspec_kernel<3, T, 8, 2, kspec_xmode<3, T>(), 0>;
      const int w = v == 1 ? W3 : 8;
      const int nt = (a.lines + w - 1) / w;
      dim3 grid(std::min(nt, resident_blocks(reinterpret_cast<const void*>(k), w * 64))), block(w * 64);
      hipLaunchKernelGGL(k, grid, block, 0, stream, t.tab, a);
      return;
    }
  }
  if constexpr (R == 4 && sizeof(T) == 4) {
    if (t.H == 2) {
      // lines over two waves: 4 lines x 2 halves = 8 waves per workgroup (two per SIMD)
      constexpr int W2 = 4;
      auto k = kspec_kernel<4, float, W2, kspec_slots<4, float>(), kspec_xmode<4, float>(), PAR, 0, 0, 2>;
      const int nt = (a.lines + W2 - 1) / W2;
      dim3 grid(std::min(nt, resident_blocks(reinterpret_cast<const void*>(k), W2 * 128))), block(W2 * 128);
      hipLaunchKernelGGL(k, grid, block, 0, stream, t.tab, a);
      return;
    }
  }
  CH_CHECK(t.H == 1, "kspec: lines over two waves are instantiated for R = 4, fp32 storage");
  constexpr int W = kspec_lines<R, T>();
  auto kern = kspec_kernel<R, T, W, kspec_slots<R, T>(), kspec_xmode<R, T>(), PAR>;
  if constexpr (R == 7 && sizeof(T) == 4 && PAR == 0) {
    if (kspec_glds7()) kern = kspec_kernel<R, T, W, kspec_slots<R, T>(), kspec_xmode<R, T>(), PAR, 1>;
    if (kspec_ns7() == 3) kern = kspec_kernel<R, T, W, 3, kspec_xmode<R, T>(), PAR>;
    if (kspec_w8()) {
      constexpr int W8 = 8;
      auto k = kspec_kernel<R, T, W8, kspec_slots<R, T>(), kspec_xmode<R, T>(), PAR, 1>;
      const int nt = (a.lines + W8 - 1) / W8;
      dim3 grid(std::min(nt, resident_blocks(reinterpret_cast<const void*>(k), W8 * 64))), block(W8 * 64);
      hipLaunchKernelGGL(k, grid, block, 0, stream, t.tab, a);
      return;
    }
  }
  const int sp = kspec_split_env();
  if constexpr (kspec_split_default<R, T>()) {
    if (sp == 1 && !a.out6) {  // (the output kernel writes the combine outputs)
      auto k1 = kspec_kernel<R, T, W, kspec_slots<R, T>(), kspec_xmode<R, T>(), PAR, 0, 1>;
      const int nt1 = (a.lines + W - 1) / W;
      dim3 g1(std::min(nt1, resident_blocks(reinterpret_cast<const void*>(k1), W * 64))), b1(W * 64);
      hipLaunchKernelGGL(k1, g1, b1, 0, stream, t.tab, a);
      constexpr int W2 = kspec_out_lines<R, T>();
      auto k2 = kspec_out_kernel<R, T, W2, kspec_xmode<R, T>()>;
      const int nt2 = (a.lines + W2 - 1) / W2;
      dim3 g2(std::min(nt2, resident_blocks(reinterpret_cast<const void*>(k2), W2 * 64))), b2(W2 * 64);
      hipLaunchKernelGGL(k2, g2, b2, 0, stream, t.tab, a);
      return;
    }
  }
  // persistent grid: as many blocks as can be resident at once
  const int ntiles = (a.lines + W - 1) / W;
  dim3 grid(std::min(ntiles, resident_blocks(reinterpret_cast<const void*>(kern), W * 64))), block(W * 64);
  hipLaunchKernelGGL(kern, grid, block, 0, stream, t.tab, a);
}

// all rows-per-lane and storage instantiations of one parity variant
template <int PAR>
void kspec_launch_par(const YTablesDev& t, const SpecArgs& a, bool fp64, hipStream_t stream) {
#ifdef CH_KSPEC_ISA_ONLY  // one instantiation, for ISA inspection builds
  CH_CHECK(t.R == CH_KSPEC_ISA_ONLY && !fp64, "ISA build");
  kspec_launch_t<CH_KSPEC_ISA_ONLY, float, PAR>(t, a, stream);
#else
  if (fp64) {
    CH_DISPATCH_R(t.R, (kspec_launch_t<R, double, PAR>(t, a, stream)));
  } else {
    CH_DISPATCH_R(t.R, (kspec_launch_t<R, float, PAR>(t, a, stream)));
  }
#endif
}
extern template void kspec_launch_par<0>(const YTablesDev&, const SpecArgs&, bool, hipStream_t);
extern template void kspec_launch_par<1>(const YTablesDev&, const SpecArgs&, bool, hipStream_t);
extern template void kspec_launch_par<2>(const YTablesDev&, const SpecArgs&, bool, hipStream_t);
extern template void kspec_launch_par<3>(const YTablesDev&, const SpecArgs&, bool, hipStream_t);

}  // namespace channel
