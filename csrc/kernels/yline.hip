// Wall-normal (y-line) kernels: coefficient tables, the fused spectral substep kernel (K-SPEC) and
// a per-operator test entry point.
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
#include "channel/fft_device.hpp"

namespace channel {

using namespace dev;

template <typename T>
struct Cplx;
template <>
struct Cplx<float> {
  using type = float2;
};
template <>
struct Cplx<double> {
  using type = double2;
};

int yline_supported_R(int NY) {
  static const int supported[] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 16, 24};
  for (int r : supported)
    if (64 * r >= NY) return r;
  CH_CHECK(false, "NY=" << NY << " too large for the y-line kernels (max 1536)");
}

#define CH_DISPATCH_R(R_, ...)                       \
  switch (R_) {                                      \
    case 1: { constexpr int R = 1; __VA_ARGS__; } break;    \
    case 2: { constexpr int R = 2; __VA_ARGS__; } break;    \
    case 3: { constexpr int R = 3; __VA_ARGS__; } break;    \
    case 4: { constexpr int R = 4; __VA_ARGS__; } break;    \
    case 5: { constexpr int R = 5; __VA_ARGS__; } break;    \
    case 6: { constexpr int R = 6; __VA_ARGS__; } break;    \
    case 7: { constexpr int R = 7; __VA_ARGS__; } break;    \
    case 8: { constexpr int R = 8; __VA_ARGS__; } break;    \
    case 10: { constexpr int R = 10; __VA_ARGS__; } break;  \
    case 12: { constexpr int R = 12; __VA_ARGS__; } break;  \
    case 16: { constexpr int R = 16; __VA_ARGS__; } break;  \
    case 24: { constexpr int R = 24; __VA_ARGS__; } break;  \
    default: CH_CHECK(false, "unsupported R=" << R_); \
  }

// Cross-lane exchanges go through the VALU (DPP / permlane swaps, yline_device.hpp) in the
// instantiations that fit their registers.  The ones that spill VGPRs keep ds_bpermute: the VALU
// variant of kspec_kernel<10, float> (48 spilled VGPRs) faulted on MI355X with a memory aperture
// violation, and so did a DPP-only variant (no permlane swaps) of kspec_kernel<10, double> (104
// spilled VGPRs) while the DPP-only <10, float> passed its oracle test: the fault follows the
// spilling kernels, not one instruction; not root-caused.  The spill-free kernels are the ones
// where the exchange latency matters (one wave per SIMD, no spill traffic to hide it).
template <int R, typename T, int PAR = 0>
constexpr bool xl_valu() {
  if (PAR != 0) return false;
  return sizeof(T) == 4 ? (R <= 3 || (R >= 5 && R <= 7)) : (R <= 3 || R == 5);
}

// ------------------------------------------------------------------------------------------
template <int R>
__global__ void __launch_bounds__(64) d1_factor_kernel(YTab t, double* out) {
  constexpr bool XV = true;  // one wave, no register pressure
  const int lane = __lane_id();
  PFac<R> F;
  CoefD1 cd{t, lane};
  pfactor<R, XV>(F, cd, lane);
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
  std::vector<std::vector<double>> tabs = {lm(g.d1_lo), lm(g.d1_up), lm(g.d1_rm), lm(g.d1_rc), lm(g.d1_rp),
                                           lm(g.m_lo),  lm(g.m_up),  lm(g.k_lo),  lm(g.k_c),   lm(g.k_up),
                                           lm(mask),    lm(g.trap),  lm(d1_row(0)), lm(d1_row(N - 1))};
  int nf = 0;
  CH_DISPATCH_R(R, nf = PFac<R>::kNumFields);
  const size_t n = tabs.size() * rows + static_cast<size_t>(nf) * 64;
  bytes = n * sizeof(double);
  HIP_CHECK(hipMalloc(&buf, bytes));
  std::vector<double> host(n, 0.0);
  for (size_t i = 0; i < tabs.size(); ++i) std::copy(tabs[i].begin(), tabs[i].end(), host.begin() + i * rows);
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
  tab.trap = p + 11 * rows;
  tab.d1row0 = p + 12 * rows;
  tab.d1rowN = p + 13 * rows;
  double* fac = buf + tabs.size() * rows;
  tab.d1fac = fac;
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

// ---- shared helpers for line kernels --------------------------------------------------------
template <int R, int K, bool XV>
__device__ void d1_apply(const YTab& t, double (&x)[K][R], int lane) {
  double rhs[K][R];
  d1_rhs<R, K, XV>(t, x, rhs, lane);
  PFac<R> F;
  pfac_load<R>(F, t.d1fac, lane);
  CoefD1 cd{t, lane};
  psolve<R, K, XV>(F, cd, rhs, lane);
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int r = 0; r < R; ++r) x[k][r] = rhs[k][r];
}

template <int R, int K, bool XV>
__device__ __forceinline__ void apply_M(const YTab& t, const double (&x)[K][R], double (&o)[K][R], int lane) {
  apply_tri<R, K, XV>(t.m_lo, t.mask, t.m_up, x, o, lane);
}
template <int R, int K, bool XV>
__device__ __forceinline__ void apply_K(const YTab& t, const double (&x)[K][R], double (&o)[K][R], int lane) {
  apply_tri<R, K, XV>(t.k_lo, t.k_c, t.k_up, x, o, lane);
}

// value of complex line at row j (wave-uniform), returned in re/im
template <int R, bool XV>
__device__ __forceinline__ void row_cplx(const double (&x)[2][R], int j, int lane, double& re, double& im) {
  re = row_value<R, XV>(x[0], j, lane);
  im = row_value<R, XV>(x[1], j, lane);
}

// ------------------------------------------------------------------------------------------
// test kernel: one wave per line, data [y][line] complex, direct global access
template <int R, typename T>
__global__ void __launch_bounds__(256) yline_test_kernel(YTab t, int op, const void* vin, void* vout, int lines,
                                                         const double* k2s, double c) {
  using T2 = typename Cplx<T>::type;
  constexpr bool XV = xl_valu<R, T>();
  const T2* in = static_cast<const T2*>(vin);
  T2* out = static_cast<T2*>(vout);
  const int lane = __lane_id();
  const int line = blockIdx.x * 4 + threadIdx.x / 64;
  if (line >= lines) return;  // whole wave exits together
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
  if (op == YOP_D1) {
    d1_apply<R, 2, XV>(t, x, lane);
  } else if (op == YOP_HELM) {
    double m[2][R];
    apply_M<R, 2, XV>(t, x, m, lane);
    PFac<R> F;
    CoefHelm ch{t, lane, k2};
    pfactor<R, XV>(F, ch, lane);
    psolve<R, 2, XV>(F, ch, m, lane);
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int r = 0; r < R; ++r) x[k][r] = m[k][r];
  } else if (op == YOP_IMPL) {
    double m[2][R];
    apply_M<R, 2, XV>(t, x, m, lane);
    PFac<R> F;
    CoefImpl ci{t, lane, 1.0 + c * k2, c};
    pfactor<R, XV>(F, ci, lane);
    psolve<R, 2, XV>(F, ci, m, lane);
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int r = 0; r < R; ++r) x[k][r] = m[k][r];
  } else if (op == YOP_MAPPLY) {
    double m[2][R];
    apply_M<R, 2, XV>(t, x, m, lane);
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int r = 0; r < R; ++r) x[k][r] = m[k][r];
  } else if (op == YOP_KAPPLY) {
    double m[2][R];
    apply_K<R, 2, XV>(t, x, m, lane);
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int r = 0; r < R; ++r) x[k][r] = m[k][r];
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int j = lane * R + r;
    if (j < N) out[static_cast<size_t>(j) * lines + line] = T2{static_cast<T>(x[0][r]), static_cast<T>(x[1][r])};
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

// ------------------------------------------------------------------------------------------
// K-SPEC: W lines per workgroup (one wave per line); fields staged through an LDS tile
// [r][lane][line] (pitch W+1 => conflict-free column reads), global access = W consecutive
// complex values per y row.
template <int R, typename T, int W, int NS = 1>
struct SpecTile {
  using T2 = typename Cplx<T>::type;
  static constexpr int PITCH = W + 1;
  // r-planes padded by one slot so consecutive y rows (consecutive r) of a staging store differ in bank
  static constexpr int PLANE = 64 * PITCH + 1;
  // Register slots hold R values per field per thread: at R <= 8 seven slots fit next to the
  // solver state, at R = 10 they pushed the kernel to 970 spilled VGPRs (130 ms/substep at
  // 2048x633x2048).  Above R = 8 a slot only records the field's address and commit() issues the
  // loads (all R per thread back to back, then the LDS stores).
  // R = 3, 4 (W = 8 lines per block) spill with register slots too: address-only there
  // (128x129x128 fp64 1.18 -> 0.84 ms/step); register slots at R = 5..8 despite some spills
  // (1024x385x1024 fp64: 99.4 ms vs 105.7 ms address-only)
  static constexpr bool kRegSlots = R <= 2 || (R >= 5 && R <= 8);
  T2* tile;             // the buffer of the last staging (column() reads it)
  int N, lines, line0, w, lane;
  // Double buffering (tile2 != nullptr): consecutive stagings alternate between two buffers, so a
  // staging's writes cannot race the previous staging's cross-wave reads and only the barrier
  // between its own writes and reads remains.  (Two stagings back, the buffer was freed by the
  // intervening staging's barrier: every wave drains its LDS reads, lgkmcnt(0), before it.)
  T2* tile2 = nullptr;
  __device__ T2* next_tile() {
    if (tile2) {
      T2* t = tile2;
      tile2 = tile;
      tile = t;
    } else {
      lds_barrier();  // single buffer: the previous staging's reads must be done
    }
    return tile;
  }
  T2 pend[kRegSlots ? NS : 1][R];  // prefetch slots: this thread's share of fields whose loads are in flight
  const T2* dsrc[kRegSlots ? 1 : NS];
  int dl0[kRegSlots ? 1 : NS];

  // Issue the global loads of a field (N*W <= 64*R*W => at most R per thread) without waiting:
  // the kernel prefetches field k+1 before computing on field k, so at one wave per SIMD the HBM
  // latency of each staging overlaps the fp64 line solves instead of stalling the whole block.
  template <int S = 0>
  __device__ void prefetch(const T2* __restrict__ src) { prefetch_at<S>(src, line0); }
  template <int S = 0>
  __device__ void prefetch_at(const T2* __restrict__ src, int l0) {
    if constexpr (!kRegSlots) {
      dsrc[S] = src;
      dl0[S] = l0;
      return;
    }
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int e = threadIdx.x + q * W * 64;
      const int y = e / W, l = e - y * W;
      pend[S][q] = T2{0, 0};
      if (e < N * W && l0 + l < lines) pend[S][q] = src[static_cast<size_t>(y) * lines + l0 + l];
    }
  }
  // Stage the prefetched field through the LDS tile and return this wave's line.
  template <int S = 0>
  __device__ void commit(double (&x)[2][R]) {
    next_tile();
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int e = threadIdx.x + q * W * 64;
      if (e < N * W) {
        const int y = e / W, l = e - y * W;
        const int ly = y / R, r = y - ly * R;
        if constexpr (kRegSlots) {
          tile[r * PLANE + ly * PITCH + l] = pend[S][q];
        } else {
          const int l0 = dl0[S];
          tile[r * PLANE + ly * PITCH + l] =
              l0 + l < lines ? dsrc[S][static_cast<size_t>(y) * lines + l0 + l] : T2{0, 0};
        }
      }
    }
    lds_barrier();
    column(x);
  }
  // This wave's line as it sits in the tile.  After store() the tile still holds the stored
  // field, so a value just written out can be re-read from LDS (at storage precision) without
  // a global round trip, as long as no staging has happened since.
  __device__ void column(double (&x)[2][R]) const {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int j = lane * R + r;
      const T2 v = tile[r * PLANE + lane * PITCH + w];
      x[0][r] = j < N ? static_cast<double>(v.x) : 0.0;
      x[1][r] = j < N ? static_cast<double>(v.y) : 0.0;
    }
  }
  __device__ void load(const T2* __restrict__ src, double (&x)[2][R]) {
    prefetch(src);
    commit(x);
  }
  __device__ void store(T2* __restrict__ dst, const double (&x)[2][R]) {
    next_tile();
#pragma unroll
    for (int r = 0; r < R; ++r) tile[r * PLANE + lane * PITCH + w] = T2{static_cast<T>(x[0][r]), static_cast<T>(x[1][r])};
    lds_barrier();
    for (int e = threadIdx.x; e < N * W; e += W * 64) {
      const int y = e / W, l = e - y * W;
      if (line0 + l < lines) {
        const int ly = y / R, r = y - ly * R;
        dst[static_cast<size_t>(y) * lines + line0 + l] = tile[r * PLANE + ly * PITCH + l];
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

// Reference-parity variants (compile-time, PAR bits): kParDD = explicit viscous D2 as D1 o D1
// (RK3_kernels.cu:160-164, derivatives_nu_double.cu:440-446); kParAnalytic = analytic influence
// functions (bilplacSolver_double.cu:56-250, l1/l2 typo fixed).  The default (PAR = 0) is the
// compact D2 and discrete Green's functions.
constexpr int kParDD = 1, kParAnalytic = 2;

// overflow-safe cosh(l y)/cosh(l) and sinh(l y)/sinh(l) (and their y-derivatives), |y| <= 1, l > 0
__device__ __forceinline__ void chs_profiles(double l, double y, double& C, double& S, double& dC, double& dS) {
  const double ep = exp(l * (y - 1.0)), em = exp(-l * (y + 1.0)), e2 = exp(-2.0 * l);
  C = (ep + em) / (1.0 + e2);
  S = (ep - em) / (1.0 - e2);
  dC = l * (ep - em) / (1.0 + e2);
  dS = l * (ep + em) / (1.0 - e2);
}

template <int R, typename T, int W, int PAR = 0>
__global__ void __launch_bounds__(W * 64) kspec_kernel(YTab tg, SpecArgs a) {
  using T2 = typename Cplx<T>::type;
  constexpr bool XV = xl_valu<R, T, PAR>();
  // Coefficient tables (14 per-row tables + the D1 factorisation) are staged into LDS once per
  // block when they fit: every solve step reads them, and from L2 each read is a dependent
  // ~500-cycle load at one wave per SIMD.  Offsets are compile-time so the reads stay ds_read.
  constexpr int ROWS = 64 * R;
  constexpr int NTAB = 14 * ROWS + PFac<R>::kNumFields * 64;
  // stage when tables + the staging tile fit the 160 KB LDS with headroom (one block per CU at
  // this register budget, so LDS does not limit occupancy): R <= 12 in fp32
  constexpr bool TLDS = NTAB * 8 + R * (64 * (W + 1) + 1) * static_cast<int>(sizeof(T2)) <= 144 * 1024;
  __shared__ double tab_lds[TLDS ? NTAB : 1];
  YTab t = tg;
  if constexpr (TLDS) {
    const double* src = tg.d1_lo;  // the table buffer is contiguous, d1_lo first (YTablesDev::upload)
    for (int i = threadIdx.x; i < NTAB; i += W * 64) tab_lds[i] = src[i];
    t.d1_lo = tab_lds + 0 * ROWS;
    t.d1_up = tab_lds + 1 * ROWS;
    t.d1_rm = tab_lds + 2 * ROWS;
    t.d1_rc = tab_lds + 3 * ROWS;
    t.d1_rp = tab_lds + 4 * ROWS;
    t.m_lo = tab_lds + 5 * ROWS;
    t.m_up = tab_lds + 6 * ROWS;
    t.k_lo = tab_lds + 7 * ROWS;
    t.k_c = tab_lds + 8 * ROWS;
    t.k_up = tab_lds + 9 * ROWS;
    t.mask = tab_lds + 10 * ROWS;
    t.trap = tab_lds + 11 * ROWS;
    t.d1row0 = tab_lds + 12 * ROWS;
    t.d1rowN = tab_lds + 13 * ROWS;
    t.d1fac = tab_lds + 14 * ROWS;
    __syncthreads();
  }
  constexpr int TILE = R * (64 * (W + 1) + 1);
  // a second staging buffer where it fits next to the tables at this kernel's blocks per CU
  // (W = 8: two blocks per CU, W = 4: one)
  constexpr int kLdsBudget = (W == 8 ? 78 : 150) * 1024;
  constexpr bool kDoubleTile = (TLDS ? NTAB * 8 : 0) + 2 * TILE * static_cast<int>(sizeof(T2)) <= kLdsBudget;
  __shared__ T2 tile_mem[(kDoubleTile ? 2 : 1) * TILE];
  double* sred = reinterpret_cast<double*>(tile_mem);  // stats reduction reuses the staging tile
  static_assert(sizeof(T2) * (W + 1) >= 4 * sizeof(double), "tile too small for the stats reduction");
  const int lane = __lane_id();
  const int w = threadIdx.x / 64;
  const int N = a.N;
  // Persistent blocks: the grid is sized to the resident capacity (one block per CU at the R=7
  // register budget) and each block walks tiles of W lines, so the coefficient tables are staged
  // into LDS once per block instead of once per tile, and the first field of the next tile is
  // prefetched while the current tile's outputs drain.  XCD-aware order: at each iteration the
  // blocks of one XCD take consecutive tiles, which share partial 128-B lines in that L2.
  const int ntiles = (a.lines + W - 1) / W;
  const int lb = static_cast<int>(xcd_remap(blockIdx.x, gridDim.x));
  SpecTile<R, T, W, 7> st{tile_mem, N, a.lines, lb * W, w, lane};
  if constexpr (kDoubleTile) st.tile2 = tile_mem + TILE;
  T2* phi = static_cast<T2*>(a.phi);
  T2* omega = static_cast<T2*>(a.omega);
  T2* Rphi = static_cast<T2*>(a.Rphi);
  T2* Romega = static_cast<T2*>(a.Romega);
  T2* out[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) out[i] = static_cast<T2*>(a.out[i]);
  const bool zprev = a.rk_z != 0.0;
  // Input staging of mode 1 is software-pipelined across tiles: the 7 input fields of the NEXT
  // tile are loaded into register slots during the long solve phases of the current one (slots:
  // 0 H_x, 1 H_z, 2 H_y, 3 phi, 4 omega, 5 R_phi, 6 R_omega), so at one wave per SIMD the HBM
  // latency is hidden behind fp64 work instead of stalling each staging step.
  auto pre_H = [&](int l0) {
    st.template prefetch_at<0>(out[0], l0);
    st.template prefetch_at<1>(out[2], l0);
    st.template prefetch_at<2>(out[1], l0);
  };
  auto pre_S = [&](int l0) {
    st.template prefetch_at<3>(phi, l0);
    st.template prefetch_at<4>(omega, l0);
  };
  auto pre_R = [&](int l0) {
    if (zprev) {
      st.template prefetch_at<5>(Rphi, l0);
      st.template prefetch_at<6>(Romega, l0);
    }
  };
  if (a.mode == 1 && lb < ntiles) {
    pre_H(lb * W);
    pre_S(lb * W);
    pre_R(lb * W);
  }
  // optional per-phase shader-clock accounting (wave-uniform, SGPRs only)
  const bool prof_on = a.prof != nullptr;
  unsigned long long pacc[kKspecPhases] = {};
  unsigned long long tprev = prof_on ? __builtin_amdgcn_s_memtime() : 0;
#define KSPEC_STAMP(k)                                           \
  if (prof_on) {                                                 \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    pacc[k] += now_ - tprev;                                     \
    tprev = now_;                                                \
  }
  for (int tile = lb; tile < ntiles; tile += gridDim.x) {
  const int line0 = tile * W;
  st.line0 = line0;
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

  double om[2][R];   // omega (state), U(y) on the mean line
  double ph[2][R];   // phi (state)
  double v[2][R];    // wall-normal velocity
  double dv[2][R];   // dv/dy
  double mean_diag_flux = 0.0, mean_C = 0.0;

  if (a.mode == 1) {
    const double dt = *a.dt;
    double RPn[2][R], RWn[2][R];
    // ---------------- nonlinear terms h_v, h_g in M-form -----------------------------------
    {
      double X[2][R], G[2][R];
      {
        double H[2][R];
        st.template commit<0>(H);  // H_x
#pragma unroll
        for (int r = 0; r < R; ++r) {
          X[0][r] = al * H[1][r];   // -i al Hx
          X[1][r] = -al * H[0][r];
          G[0][r] = is_mean ? H[0][r] : -be * H[1][r];  // i be Hx ; mean line: N(y) = Re Hx(0,0)
          G[1][r] = is_mean ? 0.0 : be * H[0][r];
        }
        st.template commit<1>(H);  // H_z
#pragma unroll
        for (int r = 0; r < R; ++r) {
          X[0][r] += be * H[1][r];  // -i be Hz
          X[1][r] -= be * H[0][r];
          G[0][r] += al * H[1][r];  // -i al Hz
          G[1][r] -= al * H[0][r];
        }
      }
      d1_apply<R, 2, XV>(t, X, lane);  // D(-i al Hx - i be Hz)
      {
        double Hy[2][R];
        st.template commit<2>(Hy);
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int r = 0; r < R; ++r) X[k][r] -= k2 * Hy[k][r];
      }
      apply_M<R, 2, XV>(t, X, RPn, lane);
      apply_M<R, 2, XV>(t, G, RWn, lane);
      KSPEC_STAMP(0)
      if (a.mean_diag && is_mean) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int j = lane * R + r;
          if (j < N) a.mean_diag[N + j] = G[0][r];
        }
      }
    }
    // ---------------- explicit part of the RK3 substep in M-form ---------------------------
    // M rhs = M q + dt [ a_n nu (K q - k^2 M q) + g_n R_now + z_n R_prev ]
    double rhsP[2][R], rhsW[2][R];
    {
      double q[2][R], Mq[2][R], Kq[2][R];
      auto explicit_d2 = [&](double (&qq)[2][R]) {
        if constexpr ((PAR & kParDD) != 0) {
          if (!is_mean) {  // fluctuations: M (D1 o D1) q; the mean profile keeps the compact D2
            double DD[2][R];
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
              for (int r = 0; r < R; ++r) DD[k][r] = qq[k][r];
            d1_apply<R, 2, XV>(t, DD, lane);
            d1_apply<R, 2, XV>(t, DD, lane);
            apply_M<R, 2, XV>(t, DD, Kq, lane);
            return;
          }
        }
        apply_K<R, 2, XV>(t, qq, Kq, lane);
      };
      st.template commit<3>(q);  // phi
      apply_M<R, 2, XV>(t, q, Mq, lane);
      explicit_d2(q);
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int r = 0; r < R; ++r)
          rhsP[k][r] = Mq[k][r] + dt * (a.rk_a * a.nu * (Kq[k][r] - k2 * Mq[k][r]) + a.rk_g * RPn[k][r]);
      st.template commit<4>(q);  // omega
      apply_M<R, 2, XV>(t, q, Mq, lane);
      explicit_d2(q);
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int r = 0; r < R; ++r)
          rhsW[k][r] = Mq[k][r] + dt * (a.rk_a * a.nu * (Kq[k][r] - k2 * Mq[k][r]) + a.rk_g * RWn[k][r]);
      if (zprev) {
        st.template commit<5>(q);  // R_phi
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int r = 0; r < R; ++r) rhsP[k][r] += dt * a.rk_z * q[k][r];
        st.template commit<6>(q);  // R_omega
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int r = 0; r < R; ++r) rhsW[k][r] += dt * a.rk_z * q[k][r];
      }
    }
    KSPEC_STAMP(1)
    st.store(Rphi, RPn);
    st.store(Romega, RWn);
    KSPEC_STAMP(2)
    if (has_next) pre_H(next_line0);

    // ---------------- implicit viscous solves (phi, omega share one factorisation) ---------
    const double c = a.rk_b * dt * a.nu;
    double phH[2][R];  // homogeneous phi solutions (real): k=0 -> phi(-1)=1, k=1 -> phi(+1)=1
    {
      PFac<R> F;
      CoefImpl ci{t, lane, 1.0 + c * k2, c};
      pfactor<R, XV>(F, ci, lane);
      {
        // omega, phi and the two homogeneous phi solutions share the factorisation: one solve
        // with 6 real right-hand sides keeps 6 independent chains in flight per PCR level
        double Z[6][R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int j = lane * R + r;
          Z[0][r] = rhsW[0][r];
          Z[1][r] = rhsW[1][r];
          Z[2][r] = rhsP[0][r];
          Z[3][r] = rhsP[1][r];
          Z[4][r] = (j == 0) ? 1.0 : 0.0;
          Z[5][r] = (j == N - 1) ? 1.0 : 0.0;
        }
        psolve<R, 6, XV>(F, ci, Z, lane);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          rhsW[0][r] = Z[0][r];
          rhsW[1][r] = Z[1][r];
          rhsP[0][r] = Z[2][r];
          rhsP[1][r] = Z[3][r];
          phH[0][r] = Z[4][r];
          phH[1][r] = Z[5][r];
        }
      }
      if (is_mean) {
        // constant flow rate: U += C * U1, U1 = response to a unit mean pressure gradient
        const double fU = wave_sum<R, XV>([&] {
          double s = 0;
#pragma unroll
          for (int r = 0; r < R; ++r) s += tab(t.trap, r, lane) * rhsW[0][r];
          return s;
        }());
        if (a.forcing == 0) {
          double U1[1][R], one[1][R], M1[1][R];
#pragma unroll
          for (int r = 0; r < R; ++r) one[0][r] = (lane * R + r < N) ? 1.0 : 0.0;
          apply_tri<R, 1, XV>(t.m_lo, t.mask, t.m_up, one, M1, lane);
#pragma unroll
          for (int r = 0; r < R; ++r) U1[0][r] = M1[0][r];
          psolve<R, 1, XV>(F, ci, U1, lane);
          const double f1 = wave_sum<R, XV>([&] {
            double s = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) s += tab(t.trap, r, lane) * U1[0][r];
            return s;
          }());
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
    if (has_next) pre_S(next_line0);

    // ---------------- velocity recovery + influence matrix (v(+-1) = v'(+-1) = 0) ----------
    {
      PFac<R> F;
      CoefHelm chm{t, lane, k2};
      pfactor<R, XV>(F, chm, lane);
      double vH[2][R];
      {
        double Y[4][R], Z[4][R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          Z[0][r] = rhsP[0][r];
          Z[1][r] = rhsP[1][r];
          Z[2][r] = phH[0][r];
          Z[3][r] = phH[1][r];
        }
        apply_M<R, 4, XV>(t, Z, Y, lane);
        psolve<R, 4, XV>(F, chm, Y, lane);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          v[0][r] = Y[0][r];
          v[1][r] = Y[1][r];
          vH[0][r] = Y[2][r];
          vH[1][r] = Y[3][r];
        }
      }
      // wall derivatives v'(+-1) = first / last row of the dense D1 applied to v (no solves)
      double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double g0 = tab(t.d1row0, r, lane), gN = tab(t.d1rowN, r, lane);
        acc[0] += g0 * v[0][r];
        acc[1] += g0 * v[1][r];
        acc[2] += gN * v[0][r];
        acc[3] += gN * v[1][r];
        acc[4] += g0 * vH[0][r];
        acc[5] += gN * vH[0][r];
        acc[6] += g0 * vH[1][r];
        acc[7] += gN * vH[1][r];
      }
      wave_sum_n<8, XV>(acc);
      const double p0r = acc[0], p0i = acc[1], pNr = acc[2], pNi = acc[3];
      double h10 = acc[4], h1N = acc[5], h20 = acc[6], h2N = acc[7];
      if constexpr ((PAR & kParAnalytic) != 0) {
        // analytic homogeneous solutions (bilplacSolver_double.cu:56-217): phi1,2 = (C_l1 -+ S_l1)/2,
        // v1,2 = D [(C_l1 -+ S_l1)/2 - (C_l2 -+ S_l2)/2], l1^2 = k^2 + Re/(beta dt), l2 = k,
        // D = 1/(l1^2 - l2^2); wall derivatives analytic, the particular one discrete
        if (k2 > 0.0 && dt > 1e-14) {
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
            const int j = lane * R + r;
            const double yj = j < N ? a.ygrid[j] : 0.0;
            double C1_, S1_, dC1, dS1, C2_, S2_, dC2, dS2;
            chs_profiles(l1, yj, C1_, S1_, dC1, dS1);
            chs_profiles(l2, yj, C2_, S2_, dC2, dS2);
            const bool in = j < N;
            phH[0][r] = in ? 0.5 * (C1_ - S1_) : 0.0;
            phH[1][r] = in ? 0.5 * (C1_ + S1_) : 0.0;
            vH[0][r] = in ? Dd * (0.5 * (C1_ - S1_) - 0.5 * (C2_ - S2_)) : 0.0;
            vH[1][r] = in ? Dd * (0.5 * (C1_ + S1_) - 0.5 * (C2_ + S2_)) : 0.0;
          }
        }
      }
      const double det = h10 * h2N - h20 * h1N;
      const bool apply = !is_mean && k2 > 0.0 && dt > 1e-14 && det != 0.0;
      const double id = apply ? 1.0 / det : 0.0;
      // [h10 h20; h1N h2N] [C1; C2] = -[p0; pN]
      const double C1r = (-p0r * h2N + h20 * pNr) * id, C1i = (-p0i * h2N + h20 * pNi) * id;
      const double C2r = (-h10 * pNr + h1N * p0r) * id, C2i = (-h10 * pNi + h1N * p0i) * id;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        ph[0][r] = rhsP[0][r] + C1r * phH[0][r] + C2r * phH[1][r];
        ph[1][r] = rhsP[1][r] + C1i * phH[0][r] + C2i * phH[1][r];
        v[0][r] += C1r * vH[0][r] + C2r * vH[1][r];
        v[1][r] += C1i * vH[0][r] + C2i * vH[1][r];
      }
      if (is_mean || k2 == 0.0) {
        czero<R>(ph);
        czero<R>(v);
      }
    }
    KSPEC_STAMP(5)
    // omega was the last field staged (store above): re-read it from the tile, not from HBM
    st.column(om);
    st.store(phi, ph);
    KSPEC_STAMP(6)
    if (has_next) pre_R(next_line0);
  } else {
    // ---------------- prepare only: fields from the state ----------------------------------
    st.load(phi, ph);
    st.load(omega, om);
    PFac<R> F;
    CoefHelm chm{t, lane, k2};
    pfactor<R, XV>(F, chm, lane);
    apply_M<R, 2, XV>(t, ph, v, lane);
    psolve<R, 2, XV>(F, chm, v, lane);
    if (is_mean || k2 == 0.0) {
      czero<R>(ph);
      czero<R>(v);
    }
  }

  // ---------------- health check (non-finite state) -----------------------------------------
  if (a.health) {
    bool bad = false;
#pragma unroll
    for (int r = 0; r < R; ++r) bad |= !isfinite(ph[0][r]) || !isfinite(ph[1][r]) || !isfinite(om[0][r]) || !isfinite(om[1][r]);
    if (__any(bad) && lane == 0) atomicOr(a.health, 1u);
  }

  // ---------------- prepare velocity / vorticity for the physical-space stage ----------------
  double Dom[2][R];
  {
    // D1 of v and omega in one 4-RHS solve
    double Z[4][R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      Z[0][r] = v[0][r];
      Z[1][r] = v[1][r];
      Z[2][r] = om[0][r];
      Z[3][r] = om[1][r];
    }
    d1_apply<R, 4, XV>(t, Z, lane);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      dv[0][r] = Z[0][r];
      dv[1][r] = Z[1][r];
      Dom[0][r] = Z[2][r];
      Dom[1][r] = Z[3][r];
    }
  }

  KSPEC_STAMP(7)
  double fu[2][R], fw[2][R];
  // u = i (al dv - be om)/k2 ; w = i (be dv + al om)/k2   (nonLinear_kernels.cu:55-72)
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const double ar = (al * dv[0][r] - be * om[0][r]) * inv_k2, ai = (al * dv[1][r] - be * om[1][r]) * inv_k2;
    const double br = (be * dv[0][r] + al * om[0][r]) * inv_k2, bi = (be * dv[1][r] + al * om[1][r]) * inv_k2;
    fu[0][r] = -ai; fu[1][r] = ar;
    fw[0][r] = -bi; fw[1][r] = br;
  }
  if (is_mean) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      fu[0][r] = om[0][r];  // U(y)
      fu[1][r] = 0.0;
      fw[0][r] = 0.0;
      fw[1][r] = 0.0;
    }
  }
  // plane statistics (statistics.cu:7-95), fluctuations only, weight 2 for kz > 0
  if (a.stats) {
    __syncthreads();  // the tile may still be read by the previous staging store
    for (int i = threadIdx.x; i < 4 * 64 * R; i += W * 64) sred[i] = 0.0;
    __syncthreads();
    if (valid && !is_mean) {
      const double wgt = kz == 0 ? 1.0 : 2.0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int idx = r * 64 + lane;
        atomicAdd(&sred[0 * 64 * R + idx], wgt * (fu[0][r] * fu[0][r] + fu[1][r] * fu[1][r]));
        atomicAdd(&sred[1 * 64 * R + idx], wgt * (v[0][r] * v[0][r] + v[1][r] * v[1][r]));
        atomicAdd(&sred[2 * 64 * R + idx], wgt * (fw[0][r] * fw[0][r] + fw[1][r] * fw[1][r]));
        atomicAdd(&sred[3 * 64 * R + idx], wgt * (fu[0][r] * v[0][r] + fu[1][r] * v[1][r]));
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 4 * 64 * R; i += W * 64) {
      const int s = i / (64 * R), rem = i - s * 64 * R, r = rem / 64, l = rem - r * 64;
      const int j = l * R + r;
      if (j < N) atomicAdd(&a.stats[s * N + j], sred[i]);
    }
  }
  KSPEC_STAMP(8)
  st.store(out[0], fu);
  st.store(out[1], v);
  st.store(out[2], fw);
  // vorticity: wx = Dw - i be v ; wy = omega ; wz = i al v - Du   (convolution_kernels.cu:46-53)
  // D(dv) = D2 v = phi + k2 v (Helmholtz identity, consistent with the compact D2 operator)
  {
    double wx[2][R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double DDr = ph[0][r] + k2 * v[0][r], DDi = ph[1][r] + k2 * v[1][r];
      const double br = (be * DDr + al * Dom[0][r]) * inv_k2, bi = (be * DDi + al * Dom[1][r]) * inv_k2;
      wx[0][r] = -bi + be * v[1][r];
      wx[1][r] = br - be * v[0][r];
      if (is_mean) { wx[0][r] = 0.0; wx[1][r] = 0.0; }
    }
    st.store(out[3], wx);
  }
  {
    double wy[2][R];  // omega_y; zero on the mean line (whose omega slot holds U)
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int r = 0; r < R; ++r) wy[k][r] = is_mean ? 0.0 : om[k][r];
    st.store(out[4], wy);  // every wave reaches every staging barrier
  }
  {
    double wz[2][R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double DDr = ph[0][r] + k2 * v[0][r], DDi = ph[1][r] + k2 * v[1][r];
      const double ar = (al * DDr - be * Dom[0][r]) * inv_k2, ai = (al * DDi - be * Dom[1][r]) * inv_k2;
      // Du = i(ar + i ai) = -ai + i ar ; wz = i al v - Du
      wz[0][r] = -al * v[1][r] + ai;
      wz[1][r] = al * v[0][r] - ar;
      if (is_mean) { wz[0][r] = -Dom[0][r]; wz[1][r] = 0.0; }
    }
    st.store(out[5], wz);
  }
  if (a.mean_diag && is_mean) {
    const double d0 = row_value<R, XV>(Dom[0], 0, lane), dN = row_value<R, XV>(Dom[0], N - 1, lane);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int j = lane * R + r;
      if (j < N) a.mean_diag[j] = om[0][r];
    }
    if (lane == 0) {
      a.mean_diag[3 * N + 0] = d0;
      a.mean_diag[3 * N + 1] = dN;
      a.mean_diag[3 * N + 2] = mean_diag_flux;
      a.mean_diag[3 * N + 3] = mean_C;
    }
  }
  KSPEC_STAMP(9)
  }  // tile loop
#undef KSPEC_STAMP
  if (prof_on && lane == 0)
    for (int k = 0; k < kKspecPhases; ++k) atomicAdd(&a.prof[k], pacc[k]);
}

template <int R, typename T>
constexpr int kspec_waves() {
  return (R <= 4 && 64 * R * 9 * 2 * sizeof(T) <= 64 * 1024) ? 8 : 4;
}

template <int R, typename T, int PAR = 0>
static void kspec_launch_t(const YTablesDev& t, const SpecArgs& a, hipStream_t stream) {
  constexpr int W = kspec_waves<R, T>();
  auto kern = kspec_kernel<R, T, W, PAR>;
  // persistent grid: as many blocks as can be resident at once
  const int ntiles = (a.lines + W - 1) / W;
  dim3 grid(std::min(ntiles, resident_blocks(reinterpret_cast<const void*>(kern), W * 64))), block(W * 64);
  hipLaunchKernelGGL(kern, grid, block, 0, stream, t.tab, a);
}

template <int PAR>
static void kspec_launch_par(const YTablesDev& t, const SpecArgs& a, bool fp64, hipStream_t stream) {
  switch (t.R) {
#define CH_PAR_R(RR)                                                  \
  case RR:                                                            \
    if (fp64) kspec_launch_t<RR, double, PAR>(t, a, stream);          \
    else kspec_launch_t<RR, float, PAR>(t, a, stream);                \
    break;
    CH_PAR_R(1) CH_PAR_R(2) CH_PAR_R(3) CH_PAR_R(4)
#undef CH_PAR_R
    default: CH_CHECK(false, "reference-parity modes (influence=analytic, explicit_d2=dd) support NY <= 256");
  }
}

void kspec_launch(const YTablesDev& t, const SpecArgs& a, bool fp64, hipStream_t stream) {
  CH_CHECK(a.N == t.tab.N, "kspec: NY mismatch with tables");
  const int par = (a.explicit_dd ? kParDD : 0) | (a.analytic_influence ? kParAnalytic : 0);
  if (par) {
    CH_CHECK(!a.analytic_influence || a.ygrid, "kspec: analytic influence needs the y grid");
    if (par == kParDD) kspec_launch_par<kParDD>(t, a, fp64, stream);
    else if (par == kParAnalytic) kspec_launch_par<kParAnalytic>(t, a, fp64, stream);
    else kspec_launch_par<kParDD | kParAnalytic>(t, a, fp64, stream);
    HIP_LAUNCH_CHECK(stream);
    return;
  }
  if (fp64) {
    CH_DISPATCH_R(t.R, kspec_launch_t<R, double>(t, a, stream));
  } else {
    CH_DISPATCH_R(t.R, kspec_launch_t<R, float>(t, a, stream));
  }
  HIP_LAUNCH_CHECK(stream);
}

}  // namespace channel
