// Small device kernels: time-step control, kz=0 Hermitian symmetrisation, field utilities.
#include <hip/hip_runtime.h>

#include <cmath>

#include "channel/common.hpp"
#include "channel/kernels.hpp"

namespace channel {

// Device-resident time-step control (RK3.c:64-109, calcDt).  The reference computed the CFL
// maxima with cublasIsamax + D2H copies + 6 MPI_Allreduce on the host and applied the new dt one
// step late (RK3.c:144, 179).  Here zphys reduces the maxima on the device (and the
// solver all-reduces them over RCCL) and this 1-thread kernel computes dt for the CURRENT step.
__global__ void dt_update_kernel(DtArgs a) {
  const double umax = a.maxima[0], vmax = a.maxima[1], wmax = a.maxima[2], csum = a.maxima[3];
  const double two_pi = 2.0 * 3.14159265358979323846;
  double dt_c, dt_v;
  if (a.parity) {
    // reference formula (RK3.c:86-89), including its NX for the z term
    const double c = (a.NX / (two_pi * a.LX)) * umax + vmax / a.dy_uniform + (a.NX / (two_pi * a.LZ)) * wmax;
    dt_c = c > 0.0 ? a.cfl / c : a.dt_max;
    const double kx = a.NX / (3.0 * a.LX), kz = a.NZ / (3.0 * a.LZ);
    dt_v = a.cfl * a.Re / (1.0 / (a.dy_uniform * a.dy_uniform) + kx * kx + kz * kz);
  } else {
    dt_c = csum > 0.0 ? a.cfl / csum : a.dt_max;
    dt_v = a.dt_max;  // viscous terms are implicit
  }
  double dt = fmin(fmin(dt_c, dt_v), a.dt_max);
  if (a.dt_fixed > 0.0) dt = a.dt_fixed;
  // health bit 1: the CFL inputs are not finite or dt collapsed (a blow-up that stays finite in the
  // fields can still overflow the fp32 maxima and freeze the run at dt = 0)
  if (a.health && (!isfinite(csum) || !isfinite(umax) || !isfinite(vmax) || !isfinite(wmax) || !(dt > 1e-12)))
    atomicOr(a.health, 2u);
  *a.dt = dt;
  *a.time += dt;
  if (a.dt_log) {
    a.dt_log[0] = umax;
    a.dt_log[1] = vmax;
    a.dt_log[2] = wmax;
    a.dt_log[3] = csum;
    a.dt_log[4] = dt_c;
    a.dt_log[5] = dt_v;
    a.dt_log[6] = dt;
    a.dt_log[7] = *a.time;
  }
  for (int i = 0; i < 4; ++i) a.maxima[i] = 0.0f;
}

void dt_update(const DtArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(dt_update_kernel, dim3(1), dim3(1), 0, s, a);
  HIP_LAUNCH_CHECK(s);
}

// kz = 0 plane Hermitian symmetry q(-kx) = conj q(kx) for a field held entirely by one rank
// (imposeSymetry.c:5-18 did this with a full FFT round trip).  lines are [y][kx][kz].
template <typename T2>
__global__ void symmetrize_kernel(T2* q, int N, int nkx, int nkzs, int Kx, int kzb) {
  const int y = blockIdx.x;
  for (int i = threadIdx.x + 1; i <= Kx; i += blockDim.x) {
    const int im = nkx - i;  // index of -kx
    T2* a = q + spec_index(kzb, nkx, nkzs, y, i, 0);
    T2* b = q + spec_index(kzb, nkx, nkzs, y, im, 0);
    const T2 va = *a, vb = *b;
    const T2 m{static_cast<decltype(va.x)>(0.5 * (va.x + vb.x)), static_cast<decltype(va.x)>(0.5 * (va.y - vb.y))};
    *a = m;
    *b = T2{m.x, -m.y};
  }
  if (threadIdx.x == 0) {
    T2* z = q + spec_index(kzb, nkx, nkzs, y, 0, 0);
    z->y = 0;
  }
}

void symmetrize_kz0(void* q, int N, int nkx, int nkzs, int Kx, int kzb, bool fp64, hipStream_t s) {
  if (fp64)
    hipLaunchKernelGGL(symmetrize_kernel<double2>, dim3(N), dim3(128), 0, s, static_cast<double2*>(q), N, nkx, nkzs, Kx, kzb);
  else
    hipLaunchKernelGGL(symmetrize_kernel<float2>, dim3(N), dim3(128), 0, s, static_cast<float2*>(q), N, nkx, nkzs, Kx, kzb);
  HIP_LAUNCH_CHECK(s);
}

// Distributed kz = 0 symmetrisation (any P, slab or pencil): the kx lines are spread over the ranks
// of a process row, so every rank first publishes its kz = 0 column [y][kx_loc] (pack), the
// columns are exchanged (the solver's all-to-all; each rank receives every block of its row), and
// each rank replaces its lines by 0.5 (q(kx) + conj q(-kx)) from the pre-symmetrisation copy, so
// the two owners of a +-kx pair write conjugate values without further communication.  The
// reference re-imposed the symmetry with a full backward+forward FFT round trip of both fields
// through the global transposes (imposeSymetry.c:5-18).
template <typename T2>
__global__ void kz0_pack_kernel(const T2* q, T2* col, int N, int nkx_loc, int nkz_loc, int kzb) {
  const int y = blockIdx.x;
  for (int i = threadIdx.x; i < nkx_loc; i += blockDim.x)
    col[static_cast<size_t>(y) * nkx_loc + i] = q[spec_index(kzb, nkx_loc, nkz_loc, y, i, 0)];
}

template <typename T2>
__global__ void kz0_sym_dist_kernel(T2* q, const T2* col, Kz0SymArgs a) {
  const int y = blockIdx.x;
  for (int i = threadIdx.x; i < a.nkx_loc; i += blockDim.x) {
    const int ig = a.kx0 + i;
    const int igp = ig == 0 ? 0 : a.nkx - ig;  // index of -kx
    int c = 0;
    for (int r = 1; r < a.nblk; ++r)
      if (igp >= a.kx_start[r]) c = r;
    const int cnt = a.kx_start[c + 1] - a.kx_start[c];
    const T2 vp = col[static_cast<size_t>(a.N) * a.kx_start[c] + static_cast<size_t>(y) * cnt + (igp - a.kx_start[c])];
    T2* dst = q + spec_index(a.kzb, a.nkx_loc, a.nkz_loc, y, i, 0);
    const T2 v = *dst;
    *dst = T2{static_cast<decltype(v.x)>(0.5 * (v.x + vp.x)), static_cast<decltype(v.x)>(0.5 * (v.y - vp.y))};
  }
}

void kz0_pack(const void* q, void* col, int N, int nkx_loc, int nkz_loc, int kzb, bool fp64, hipStream_t s) {
  if (fp64)
    hipLaunchKernelGGL(kz0_pack_kernel<double2>, dim3(N), dim3(128), 0, s, static_cast<const double2*>(q),
                       static_cast<double2*>(col), N, nkx_loc, nkz_loc, kzb);
  else
    hipLaunchKernelGGL(kz0_pack_kernel<float2>, dim3(N), dim3(128), 0, s, static_cast<const float2*>(q),
                       static_cast<float2*>(col), N, nkx_loc, nkz_loc, kzb);
  HIP_LAUNCH_CHECK(s);
}

void kz0_symmetrize_dist(void* q, const void* col_all, const Kz0SymArgs& a, bool fp64, hipStream_t s) {
  CH_CHECK(a.nblk >= 1 && a.nblk <= kMaxSeg && a.kx_start[0] == 0 && a.kx_start[a.nblk] == a.nkx,
           "kz0 symmetrisation: bad kx block table");
  if (fp64)
    hipLaunchKernelGGL(kz0_sym_dist_kernel<double2>, dim3(a.N), dim3(128), 0, s, static_cast<double2*>(q),
                       static_cast<const double2*>(col_all), a);
  else
    hipLaunchKernelGGL(kz0_sym_dist_kernel<float2>, dim3(a.N), dim3(128), 0, s, static_cast<float2*>(q),
                       static_cast<const float2*>(col_all), a);
  HIP_LAUNCH_CHECK(s);
}

// Energy spectra of u, v, w at selected y planes (the reference's calcSpectra, statistics.cu:245-326,
// is dead code that dumped |q|^2 of one plane; here it is a live, device-side diagnostic).
// One block per (local kx, plane); fluctuations only (the (0,0) line carries U(y)).  The kz = 0
// column counts once and kz > 0 twice (the -kz half), so E_kx sums to the plane energy.
template <typename T2>
__global__ void __launch_bounds__(256) spectra_kernel(SpectraArgs a) {
  const int ikx = blockIdx.x, pl = blockIdx.y;
  const int j = a.planes[pl];
  const int ig = a.kx0 + ikx;
  const int kx = ig <= a.Kx ? ig : ig - a.nkx;
  const int akx = kx < 0 ? -kx : kx;
  const T2* dv = static_cast<const T2*>(a.dv);
  const T2* vv = static_cast<const T2*>(a.v);
  const T2* om = static_cast<const T2*>(a.om);
  const double al = a.ax * kx;
  double sx[3] = {0.0, 0.0, 0.0};
  for (int kl = threadIdx.x; kl < a.nkz_loc; kl += blockDim.x) {
    const int kz = a.kz0 + kl;
    const size_t idx = spec_index(a.kzb, a.nkx_loc, a.nkzs, j, ikx, kl);
    const double wgt = (kx == 0 && kz == 0) ? 0.0 : (kz == 0 ? 1.0 : 2.0);
    const double be = a.az * kz, k2 = al * al + be * be, r = k2 > 0.0 ? 1.0 / k2 : 0.0;
    double ur, ui, wr, wi;
    if (a.combine) {
      const T2 d = dv[idx], o = om[idx];
      // |u|^2 = |al D1v - be om|^2 / k2^2, |w|^2 = |be D1v + al om|^2 / k2^2 (nonLinear_kernels.cu:55-72)
      ur = (al * d.x - be * o.x) * r;
      ui = (al * d.y - be * o.y) * r;
      wr = (be * d.x + al * o.x) * r;
      wi = (be * d.y + al * o.y) * r;
    } else {
      const T2 cu = static_cast<const T2*>(a.u)[idx], cw = static_cast<const T2*>(a.w)[idx];
      ur = cu.x;
      ui = cu.y;
      wr = cw.x;
      wi = cw.y;
    }
    const T2 c1 = vv[idx];
    const double en[3] = {ur * ur + ui * ui, static_cast<double>(c1.x) * c1.x + static_cast<double>(c1.y) * c1.y,
                          wr * wr + wi * wi};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const double e = en[q];
      sx[q] += wgt * e;
      atomicAdd(&a.ekz[(static_cast<size_t>(q) * a.nplanes + pl) * a.nkz + kz], wgt * e);
      if (pl == 0 && a.map) a.map[(static_cast<size_t>(q) * a.nkx + ig) * a.nkz + kz] = (kx == 0 && kz == 0) ? 0.0 : e;
    }
  }
  __shared__ double red[3][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    double v = sx[q];
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) red[q][w] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int q = threadIdx.x;
    double v = 0.0;
    for (int i = 0; i < static_cast<int>(blockDim.x >> 6); ++i) v += red[q][i];
    atomicAdd(&a.ekx[(static_cast<size_t>(q) * a.nplanes + pl) * (a.Kx + 1) + akx], v);
  }
}

void spectra_accumulate(const SpectraArgs& a, bool fp64, hipStream_t s) {
  CH_CHECK(a.nplanes > 0 && a.nkx_loc > 0 && a.nkz_loc > 0, "spectra: empty");
  dim3 grid(a.nkx_loc, a.nplanes);
  if (fp64) hipLaunchKernelGGL(spectra_kernel<double2>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(spectra_kernel<float2>, grid, dim3(256), 0, s, a);
  HIP_LAUNCH_CHECK(s);
}

// fault injection (tests): overwrite one element of a field with NaN
__global__ void poison_kernel(float* p) { p[0] = __int_as_float(0x7fc00000); }

void inject_nan(void* field, size_t elem, bool fp64, hipStream_t s) {
  char* b = static_cast<char*>(field) + elem * (fp64 ? 16 : 8);
  if (fp64) {
    const double nanv = std::nan("");
    HIP_CHECK(hipMemcpyAsync(b, &nanv, sizeof(double), hipMemcpyHostToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));
  } else {
    hipLaunchKernelGGL(poison_kernel, dim3(1), dim3(1), 0, s, reinterpret_cast<float*>(b));
    HIP_LAUNCH_CHECK(s);
  }
}

}  // namespace channel
