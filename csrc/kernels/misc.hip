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
__global__ void symmetrize_kernel(T2* q, int N, int nkx, int nkz, int Kx) {
  const int y = blockIdx.x;
  for (int i = threadIdx.x + 1; i <= Kx; i += blockDim.x) {
    const int im = nkx - i;  // index of -kx
    T2* a = q + (static_cast<size_t>(y) * nkx + i) * nkz;
    T2* b = q + (static_cast<size_t>(y) * nkx + im) * nkz;
    const T2 va = *a, vb = *b;
    const T2 m{static_cast<decltype(va.x)>(0.5 * (va.x + vb.x)), static_cast<decltype(va.x)>(0.5 * (va.y - vb.y))};
    *a = m;
    *b = T2{m.x, -m.y};
  }
  if (threadIdx.x == 0) {
    T2* z = q + static_cast<size_t>(y) * nkx * nkz;
    z->y = 0;
  }
}

void symmetrize_kz0(void* q, int N, int nkx, int nkz, int Kx, bool fp64, hipStream_t s) {
  if (fp64)
    hipLaunchKernelGGL(symmetrize_kernel<double2>, dim3(N), dim3(128), 0, s, static_cast<double2*>(q), N, nkx, nkz, Kx);
  else
    hipLaunchKernelGGL(symmetrize_kernel<float2>, dim3(N), dim3(128), 0, s, static_cast<float2*>(q), N, nkx, nkz, Kx);
  HIP_LAUNCH_CHECK(s);
}

}  // namespace channel
