// Transform stages between spectral and physical space (SURVEY §7.3 K-XB, K-PHYS, K-XF).
//
//  * xfft_backward: for each local y plane and a chunk of C kz columns, gather the retained kx
//    modes (directly from the all-to-all receive blocks; zero-padded to NX in LDS), inverse C2C of
//    length NX, write [y][x][kz].  Replaces the x-part of the reference's 2-D cufftExecC2R and the
//    transposeYZX2XYZ local transposes + dealias (fft.c:54-78, channel_cuda_mpi.c:95-128).
//  * zphys: per (y,x) row, the six fields u,v,w,wx,wy,wz are paired into three complex rows
//    (z = a + i b), zero-padded from the retained kz to 2NZ-2 points, inverse FFT'd, the
//    rotational nonlinear term H = u x omega is formed in registers (rotorkernel,
//    convolution_kernels.cu:69-148) with the CFL maxima (the cublasIsamax calls of fft.c:143-200),
//    and H is forward transformed (Hx+iHy and pairs of Hz rows) and truncated to the retained kz.
//    Physical fields never leave LDS/registers.
//  * xfft_forward: forward C2C along x and truncation to the retained kx, written straight into
//    the per-destination all-to-all send blocks (or, for P=1, into the spectral H arrays).
#include <hip/hip_runtime.h>

#include <cmath>
#include <vector>

#include "channel/common.hpp"
#include "channel/fft_device.hpp"
#include "channel/kernels.hpp"

namespace channel {

using namespace dev;

void Twiddles::build(int n_, bool fp64_) {
  release();
  n = n_;
  fp64 = fp64_;
  const double two_pi = 2.0 * std::acos(-1.0);
  if (fp64) {
    std::vector<double2> h(n);
    for (int m = 0; m < n; ++m) h[m] = double2{std::cos(two_pi * m / n), -std::sin(two_pi * m / n)};
    HIP_CHECK(hipMalloc(&buf, n * sizeof(double2)));
    HIP_CHECK(hipMemcpy(buf, h.data(), n * sizeof(double2), hipMemcpyHostToDevice));
  } else {
    std::vector<float2> h(n);
    for (int m = 0; m < n; ++m)
      h[m] = float2{static_cast<float>(std::cos(two_pi * m / n)), static_cast<float>(-std::sin(two_pi * m / n))};
    HIP_CHECK(hipMalloc(&buf, n * sizeof(float2)));
    HIP_CHECK(hipMemcpy(buf, h.data(), n * sizeof(float2), hipMemcpyHostToDevice));
  }
}

void Twiddles::release() {
  if (buf) (void)hipFree(buf);
  buf = nullptr;
}

// ---- x-direction -------------------------------------------------------------------------
template <int NX, typename T>
struct XCfg {
  static constexpr int C = sizeof(T) == 4 ? (NX >= 1024 ? 8 : 16) : (NX >= 1024 ? 4 : 8);
  static constexpr int NT = 256;
  // row pitch: padded FFT row + 1 or 2 slots so that the transposing global->LDS stores (lanes =
  // C consecutive kz columns x consecutive x) hit distinct banks (pitch*c spreads over 16 slots)
  static constexpr int PITCH = FftPitch<NX>::value + (sizeof(T) == 4 ? (C >= 16 ? 1 : 2) : (C >= 8 ? 1 : 2));
};

__device__ __forceinline__ int find_block(const int* start, int n, int i) {
  int s = 0;
  for (int q = 1; q < n; ++q)
    if (i >= start[q]) s = q;
  return s;
}

template <int NX, typename T>
__global__ void __launch_bounds__(256) xfft_backward_kernel(XArgs a, XSrc src, typename C2<T>::type* phys,
                                                            const typename C2<T>::type* tw) {
  using T2 = typename C2<T>::type;
  using Cfg = XCfg<NX, T>;
  constexpr int C = Cfg::C, NT = Cfg::NT, PITCH = Cfg::PITCH;
  __shared__ T2 s[C * PITCH];
  const int nkzc = (a.nkz + C - 1) / C;
  const unsigned t = xcd_remap(blockIdx.x, gridDim.x);  // adjacent kz chunks of one (y, f) share an XCD
  const int kz0 = static_cast<int>(t % nkzc) * C;
  const int rest = static_cast<int>(t / nkzc);
  const int y = rest % a.ny, f = rest / a.ny;
  const int tid = threadIdx.x;
  const T2* base = static_cast<const T2*>(src.base) + f * a.field_stride_spec;
  // issue every global load of this thread before touching LDS (one latency, not EPT of them)
  constexpr int EPT = (NX * C + NT - 1) / NT;
  T2 v[EPT];
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    const int e = tid + q * NT;
    const int x = e / C, c = e - x * C;
    const int kz = kz0 + c;
    int i = -1;
    if (x <= a.Kx) i = x;
    else if (x >= NX - a.Kx) i = a.nkx - (NX - x);
    v[q] = T2{0, 0};
    if (e < NX * C && i >= 0 && kz < a.nkz) {
      const int sb = find_block(src.kx_start, src.nsrc, i);
      const int nk = src.kx_start[sb + 1] - src.kx_start[sb];
      v[q] = base[src.off[sb] + (static_cast<long long>(y) * nk + (i - src.kx_start[sb])) * a.nkz + kz];
    }
  }
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    const int e = tid + q * NT;
    const int x = e / C, c = e - x * C;
    if (e < NX * C) s[c * PITCH + fft_pidx(x)] = v[q];
  }
  __syncthreads();
  lds_fft<NX, C, PITCH, NT, true>(s, tw, tid);
  T2* out = phys + f * a.field_stride_phys;
  for (int e = tid; e < NX * C; e += NT) {
    const int x = e / C, c = e - x * C;
    const int kz = kz0 + c;
    if (kz < a.nkz) out[(static_cast<long long>(y) * NX + x) * a.nkz + kz] = s[c * PITCH + fft_pidx(x)];
  }
}

template <int NX, typename T>
__global__ void __launch_bounds__(256) xfft_forward_kernel(XArgs a, const typename C2<T>::type* phys, XDst dst,
                                                           const typename C2<T>::type* tw) {
  using T2 = typename C2<T>::type;
  using Cfg = XCfg<NX, T>;
  constexpr int C = Cfg::C, NT = Cfg::NT, PITCH = Cfg::PITCH;
  __shared__ T2 s[C * PITCH];
  const int nkzc = (a.nkz + C - 1) / C;
  const unsigned t = xcd_remap(blockIdx.x, gridDim.x);
  const int kz0 = static_cast<int>(t % nkzc) * C;
  const int rest = static_cast<int>(t / nkzc);
  const int y = rest % a.ny, f = rest / a.ny;
  const int tid = threadIdx.x;
  const T2* in = phys + f * a.field_stride_phys;
  constexpr int EPT = (NX * C + NT - 1) / NT;
  T2 v[EPT];
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    const int e = tid + q * NT;
    const int x = e / C, c = e - x * C;
    const int kz = kz0 + c;
    v[q] = T2{0, 0};
    if (e < NX * C && kz < a.nkz) v[q] = in[(static_cast<long long>(y) * NX + x) * a.nkz + kz];
  }
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    const int e = tid + q * NT;
    const int x = e / C, c = e - x * C;
    if (e < NX * C) s[c * PITCH + fft_pidx(x)] = v[q];
  }
  __syncthreads();
  lds_fft<NX, C, PITCH, NT, false>(s, tw, tid);
  T2* outb = static_cast<T2*>(dst.base) + f * a.field_stride_spec;
  for (int e = tid; e < a.nkx * C; e += NT) {
    const int i = e / C, c = e - i * C;
    const int kz = kz0 + c;
    if (kz < a.nkz) {
      const int x = i <= a.Kx ? i : NX - (a.nkx - i);
      const int d = find_block(dst.kx_start, dst.ndst, i);
      const int nk = dst.kx_start[d + 1] - dst.kx_start[d];
      outb[dst.off[d] + (static_cast<long long>(y) * nk + (i - dst.kx_start[d])) * a.nkz + kz] = s[c * PITCH + fft_pidx(x)];
    }
  }
}

#define CH_DISPATCH_N(N_, ...)                          \
  switch (N_) {                                         \
    case 16: { constexpr int NN = 16; __VA_ARGS__; } break;    \
    case 32: { constexpr int NN = 32; __VA_ARGS__; } break;    \
    case 64: { constexpr int NN = 64; __VA_ARGS__; } break;    \
    case 128: { constexpr int NN = 128; __VA_ARGS__; } break;  \
    case 256: { constexpr int NN = 256; __VA_ARGS__; } break;  \
    case 512: { constexpr int NN = 512; __VA_ARGS__; } break;  \
    case 1024: { constexpr int NN = 1024; __VA_ARGS__; } break; \
    case 2048: { constexpr int NN = 2048; __VA_ARGS__; } break; \
    default: CH_CHECK(false, "unsupported FFT length " << N_); \
  }

template <typename T>
static void xb_launch(const XArgs& a, const XSrc& src, void* phys, const Twiddles& tw, hipStream_t s) {
  using T2 = typename C2<T>::type;
  CH_DISPATCH_N(a.NX, {
    constexpr int C = XCfg<NN, T>::C;
    dim3 grid(static_cast<unsigned>(a.ny) * ((a.nkz + C - 1) / C) * a.nfields);
    hipLaunchKernelGGL((xfft_backward_kernel<NN, T>), grid, dim3(256), 0, s, a, src, static_cast<T2*>(phys),
                       static_cast<const T2*>(tw.buf));
  });
  HIP_LAUNCH_CHECK(s);
}

template <typename T>
static void xf_launch(const XArgs& a, const void* phys, const XDst& dst, const Twiddles& tw, hipStream_t s) {
  using T2 = typename C2<T>::type;
  CH_DISPATCH_N(a.NX, {
    constexpr int C = XCfg<NN, T>::C;
    dim3 grid(static_cast<unsigned>(a.ny) * ((a.nkz + C - 1) / C) * a.nfields);
    hipLaunchKernelGGL((xfft_forward_kernel<NN, T>), grid, dim3(256), 0, s, a, static_cast<const T2*>(phys), dst,
                       static_cast<const T2*>(tw.buf));
  });
  HIP_LAUNCH_CHECK(s);
}

void xfft_backward(const XArgs& a, const XSrc& src, void* phys, const Twiddles& tw, bool fp64, hipStream_t s) {
  CH_CHECK(tw.n == a.NX && tw.fp64 == fp64, "xfft_backward: twiddle table mismatch");
  CH_CHECK(a.ny > 0 && a.nkz > 0, "xfft_backward: empty");
  if (fp64) xb_launch<double>(a, src, phys, tw, s);
  else xb_launch<float>(a, src, phys, tw, s);
}

void xfft_forward(const XArgs& a, const void* phys, const XDst& dst, const Twiddles& tw, bool fp64, hipStream_t s) {
  CH_CHECK(tw.n == a.NX && tw.fp64 == fp64, "xfft_forward: twiddle table mismatch");
  if (fp64) xf_launch<double>(a, phys, dst, tw, s);
  else xf_launch<float>(a, phys, dst, tw, s);
}

// ---- z-direction physical stage -------------------------------------------------------------
template <int NZP, typename T>
struct ZCfg {
  static constexpr int NR = sizeof(T) == 4 ? (2048 / NZP > 2 ? 2048 / NZP : 2) : (1024 / NZP > 2 ? 1024 / NZP : 2);
  static constexpr int NT = 256;
};

__device__ __forceinline__ void atomic_max_pos(float* p, float v) {
  atomicMax(reinterpret_cast<unsigned int*>(p), __float_as_uint(v));
}

template <int NZP, typename T>
__global__ void __launch_bounds__(256) zphys_kernel(ZArgs a, typename C2<T>::type* fields,
                                                    const typename C2<T>::type* tw) {
  using T2 = typename C2<T>::type;
  using Cfg = ZCfg<NZP, T>;
  constexpr int NR = Cfg::NR, NT = Cfg::NT;
  constexpr int E = NR * NZP / NT > 0 ? NR * NZP / NT : 1;
  static_assert(NR % 2 == 0, "NR must be even");
  constexpr int PITCH = FftPitch<NZP>::value;
  __shared__ T2 s[3 * NR * PITCH];
  __shared__ float red[4][NT / 64];
  const int tid = threadIdx.x;
  const long long nrows = static_cast<long long>(a.ny) * a.NX;
  const long long row0 = static_cast<long long>(blockIdx.x) * NR;
  const int Kz = a.nkz - 1;
  const long long fs = a.field_stride;

  // gather, pass 1: each retained coefficient is loaded exactly once, all loads of a field issued
  // before its LDS stores.  Field 2p of row q -> slots [0, Kz] of LDS row (q,p); field 2p+1 -> slot
  // N-k (k >= 1) and N/2 (k = 0; the Nyquist slot, unused since Kz < N/2).  The rows of one field
  // are contiguous, so element e covers (row0 + e / nkz, e % nkz): tracked incrementally.
  {
    constexpr int MAXE = (NR * (NZP / 2) + NT - 1) / NT;  // nkz <= NZP/2
    const int tot = NR * a.nkz;
    const long long nvalid = (nrows - row0 < NR ? nrows - row0 : NR) * a.nkz;
    const int qr0 = tid / a.nkz, k0 = tid - qr0 * a.nkz;
    const int dq = NT / a.nkz, dk = NT - dq * a.nkz;
#pragma unroll
    for (int f = 0; f < 6; ++f) {
      const T2* src = fields + f * fs + row0 * a.nkz;
      T2 v[MAXE];
#pragma unroll
      for (int q = 0; q < MAXE; ++q) {
        const int e = tid + q * NT;
        v[q] = (e < tot && e < nvalid) ? src[e] : T2{0, 0};
      }
      int qr = qr0, k = k0;
      const int p = f >> 1;
#pragma unroll
      for (int q = 0; q < MAXE; ++q) {
        const int e = tid + q * NT;
        if (e < tot) {
          const int slot = (f & 1) == 0 ? k : (k == 0 ? NZP / 2 : NZP - k);
          s[(qr * 3 + p) * PITCH + fft_pidx(slot)] = v[q];
        }
        qr += dq;
        k += dk;
        if (k >= a.nkz) { k -= a.nkz; ++qr; }
      }
    }
  }
  __syncthreads();
  // pass 2: Z_k = A_k + i B_k, Z_{N-k} = conj(A_k) + i conj(B_k), zero padding in between
  for (int e = tid; e < 3 * NR * (NZP / 2); e += NT) {
    const int rr = e / (NZP / 2), k = e - rr * (NZP / 2);
    T2* row = s + rr * PITCH;
    if (k == 0) {
      const T2 A = row[fft_pidx(0)], B = row[fft_pidx(NZP / 2)];
      row[fft_pidx(0)] = T2{A.x, B.x};
      row[fft_pidx(NZP / 2)] = T2{0, 0};
    } else if (k <= Kz) {
      const T2 A = row[fft_pidx(k)], B = row[fft_pidx(NZP - k)];
      row[fft_pidx(k)] = T2{A.x - B.y, A.y + B.x};
      row[fft_pidx(NZP - k)] = T2{A.x + B.y, B.x - A.y};
    } else {
      row[fft_pidx(k)] = T2{0, 0};
      row[fft_pidx(NZP - k)] = T2{0, 0};
    }
  }
  __syncthreads();
  lds_fft<NZP, 3 * NR, PITCH, NT, true>(s, tw, tid);

  // H = u x omega, CFL maxima
  T hx[E], hy[E], hz[E];
  float mu = 0.f, mv = 0.f, mw = 0.f, mc = 0.f;
#pragma unroll
  for (int b = 0; b < E; ++b) {
    const int e = tid + b * NT;
    const int q = e / NZP, n = e - q * NZP;
    const int pn = fft_pidx(n);
    const T2 z0 = s[(q * 3 + 0) * PITCH + pn], z1 = s[(q * 3 + 1) * PITCH + pn], z2 = s[(q * 3 + 2) * PITCH + pn];
    const T u = z0.x, v = z0.y, w = z1.x, wx = z1.y, wy = z2.x, wz = z2.y;
    hx[b] = v * wz - w * wy;
    hy[b] = w * wx - u * wz;
    hz[b] = u * wy - v * wx;
    const long long row = row0 + q;
    if (row < nrows) {
      const int yl = static_cast<int>(row / a.NX);
      const float au = fabsf(static_cast<float>(u)), av = fabsf(static_cast<float>(v)), aw = fabsf(static_cast<float>(w));
      mu = fmaxf(mu, au);
      mv = fmaxf(mv, av);
      mw = fmaxf(mw, aw);
      mc = fmaxf(mc, static_cast<float>(au * a.cx + av * a.inv_dy[a.y0 + yl] + aw * a.cz));
    }
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < E; ++b) {
    const int e = tid + b * NT;
    const int q = e / NZP, n = e - q * NZP;
    const int pn = fft_pidx(n);
    s[q * PITCH + pn] = T2{hx[b], hy[b]};
    reinterpret_cast<T*>(&s[(NR + q / 2) * PITCH + pn])[q & 1] = hz[b];
  }
  // block maxima
  for (int o = 32; o >= 1; o >>= 1) {
    mu = fmaxf(mu, __shfl_xor(mu, o));
    mv = fmaxf(mv, __shfl_xor(mv, o));
    mw = fmaxf(mw, __shfl_xor(mw, o));
    mc = fmaxf(mc, __shfl_xor(mc, o));
  }
  if ((tid & 63) == 0) {
    red[0][tid / 64] = mu;
    red[1][tid / 64] = mv;
    red[2][tid / 64] = mw;
    red[3][tid / 64] = mc;
  }
  __syncthreads();
  if (tid < 4 && a.maxima) {
    float m = 0.f;
    for (int i = 0; i < NT / 64; ++i) m = fmaxf(m, red[tid][i]);
    atomic_max_pos(&a.maxima[tid], m);
  }
  lds_fft<NZP, 3 * NR / 2, PITCH, NT, false>(s, tw, tid);

  // extract retained kz, normalise, write H_x, H_y, H_z over fields 0..2
  const T sc = static_cast<T>(0.5 * a.scale);
  const int dq2 = NT / a.nkz, dk2 = NT - dq2 * a.nkz;
  int q = tid / a.nkz, k = tid - q * a.nkz;
  for (int e = tid; e < NR * a.nkz; e += NT, q += dq2, k += dk2) {
    if (k >= a.nkz) { k -= a.nkz; ++q; }
    const long long row = row0 + q;
    if (row >= nrows) continue;
    const int km = (NZP - k) & (NZP - 1);
    const T2 Z = s[q * PITCH + fft_pidx(k)], Zm = s[q * PITCH + fft_pidx(km)];
    // X = (Z + conj Zm)/2, Y = (Z - conj Zm)/(2i)
    const T2 X{(Z.x + Zm.x) * sc, (Z.y - Zm.y) * sc};
    const T2 Y{(Z.y + Zm.y) * sc, -(Z.x - Zm.x) * sc};
    const T2 P = s[(NR + q / 2) * PITCH + fft_pidx(k)], Pm = s[(NR + q / 2) * PITCH + fft_pidx(km)];
    const T2 Hz = (q & 1) == 0 ? T2{(P.x + Pm.x) * sc, (P.y - Pm.y) * sc} : T2{(P.y + Pm.y) * sc, -(P.x - Pm.x) * sc};
    fields[0 * fs + row * a.nkz + k] = X;
    fields[1 * fs + row * a.nkz + k] = Y;
    fields[2 * fs + row * a.nkz + k] = Hz;
  }
}

template <typename T>
static void zphys_launch(const ZArgs& a, void* fields, const Twiddles& tw, hipStream_t s) {
  using T2 = typename C2<T>::type;
  CH_DISPATCH_N(a.Nzp, {
    if constexpr (sizeof(T) == 8 && NN > 1024) {
      CH_CHECK(false, "fp64 storage supports 2NZ-2 <= 1024");
    } else {
      constexpr int NR = ZCfg<NN, T>::NR;
      const long long nrows = static_cast<long long>(a.ny) * a.NX;
      dim3 grid(static_cast<unsigned>((nrows + NR - 1) / NR));
      hipLaunchKernelGGL((zphys_kernel<NN, T>), grid, dim3(256), 0, s, a, static_cast<T2*>(fields),
                         static_cast<const T2*>(tw.buf));
    }
  });
  HIP_LAUNCH_CHECK(s);
}

void zphys(const ZArgs& a, void* fields, const Twiddles& tw, bool fp64, hipStream_t s) {
  CH_CHECK(tw.n == a.Nzp && tw.fp64 == fp64, "zphys: twiddle table mismatch");
  CH_CHECK(a.nkz - 1 < a.Nzp / 2, "zphys: retained kz must be below Nyquist");
  if (a.ny == 0) return;
  if (fp64) zphys_launch<double>(a, fields, tw, s);
  else zphys_launch<float>(a, fields, tw, s);
}

// ---- standalone batched C2C (tests) ----------------------------------------------------------
template <int N, typename T, bool INV>
__global__ void __launch_bounds__(256) fft_test_kernel(typename C2<T>::type* data, int batch,
                                                       const typename C2<T>::type* tw) {
  using T2 = typename C2<T>::type;
  constexpr int ROWS = N >= 1024 ? 2 : 2048 / N;
  constexpr int PITCH = FftPitch<N>::value;
  __shared__ T2 s[ROWS * PITCH];
  const long long r0 = static_cast<long long>(blockIdx.x) * ROWS;
  for (int e = threadIdx.x; e < ROWS * N; e += 256) {
    const int q = e / N, x = e - q * N;
    s[q * PITCH + fft_pidx(x)] = (r0 + q < batch) ? data[r0 * N + e] : T2{0, 0};
  }
  __syncthreads();
  lds_fft<N, ROWS, PITCH, 256, INV>(s, tw, threadIdx.x);
  for (int e = threadIdx.x; e < ROWS * N; e += 256) {
    const int q = e / N, x = e - q * N;
    if (r0 + q < batch) data[r0 * N + e] = s[q * PITCH + fft_pidx(x)];
  }
}

template <typename T>
static void fft_test_launch(void* data, int n, int batch, int dir, const Twiddles& tw, hipStream_t s) {
  using T2 = typename C2<T>::type;
  CH_DISPATCH_N(n, {
    constexpr int ROWS = NN >= 1024 ? 2 : 2048 / NN;
    if constexpr (sizeof(T) == 8 && NN > 1024) {
      CH_CHECK(false, "fp64 test FFT supports n <= 1024");
    } else {
      dim3 grid((batch + ROWS - 1) / ROWS);
      if (dir > 0)
        hipLaunchKernelGGL((fft_test_kernel<NN, T, true>), grid, dim3(256), 0, s, static_cast<T2*>(data), batch,
                           static_cast<const T2*>(tw.buf));
      else
        hipLaunchKernelGGL((fft_test_kernel<NN, T, false>), grid, dim3(256), 0, s, static_cast<T2*>(data), batch,
                           static_cast<const T2*>(tw.buf));
    }
  });
  HIP_LAUNCH_CHECK(s);
}

void fft_c2c_test(void* data, int n, int batch, int dir, const Twiddles& tw, bool fp64, hipStream_t s) {
  CH_CHECK(tw.n == n && tw.fp64 == fp64, "fft_c2c_test: twiddle table mismatch");
  if (fp64) fft_test_launch<double>(data, n, batch, dir, tw, s);
  else fft_test_launch<float>(data, n, batch, dir, tw, s);
}

}  // namespace channel
