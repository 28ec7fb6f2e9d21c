// In-LDS batched complex FFT (Stockham autosort, radix-4 passes + one radix-2 pass when log2 N is
// odd).  All threads of the workgroup cooperate on ROWS rows of length N held in LDS; each pass
// gathers its butterfly inputs into registers, synchronises, and writes the outputs back to the
// same LDS rows (in-place through registers), so a tile needs only one LDS buffer.
// Twiddles come from a global table W_N^m = exp(-2 pi i m / N) (L1/L2 resident).
//
// Replaces the reference's cuFFT 2-D plans (fft.c:17-23); length is a compile-time power of two.
#pragma once

#include <hip/hip_runtime.h>

namespace channel {
namespace dev {

template <typename T>
struct C2;
template <>
struct C2<float> {
  using type = float2;
};
template <>
struct C2<double> {
  using type = double2;
};

template <typename T2>
__device__ __forceinline__ T2 cmul(T2 a, T2 b) {
  return T2{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
template <typename T2>
__device__ __forceinline__ T2 cadd(T2 a, T2 b) {
  return T2{a.x + b.x, a.y + b.y};
}
template <typename T2>
__device__ __forceinline__ T2 csub(T2 a, T2 b) {
  return T2{a.x - b.x, a.y - b.y};
}

constexpr int ilog2(int n) { return n <= 1 ? 0 : 1 + ilog2(n / 2); }

template <bool INV, typename T2>
__device__ __forceinline__ void radix4(T2 (&v)[4]) {
  const T2 a0 = cadd(v[0], v[2]), a1 = csub(v[0], v[2]);
  const T2 a2 = cadd(v[1], v[3]);
  const T2 d = csub(v[1], v[3]);
  // forward: a3 = -i d ; inverse: a3 = +i d
  const T2 a3 = INV ? T2{-d.y, d.x} : T2{d.y, -d.x};
  v[0] = cadd(a0, a2);
  v[1] = cadd(a1, a3);
  v[2] = csub(a0, a2);
  v[3] = csub(a1, a3);
}

template <int N, int ROWS, int NT, bool INV, typename T2>
__device__ void lds_fft(T2* __restrict__ buf, int pitch, const T2* __restrict__ tw, int tid) {
  constexpr int LOG = ilog2(N);
  constexpr int Q = N / 4;
  constexpr int NB4 = ROWS * Q;
  constexpr int B4 = (NB4 + NT - 1) / NT;
#pragma unroll
  for (int pass = 0; pass < LOG / 2; ++pass) {
    const int Ns = 1 << (2 * pass);
    T2 v[B4][4];
#pragma unroll
    for (int b = 0; b < B4; ++b) {
      const int idx = tid + b * NT;
      if (NB4 % NT == 0 || idx < NB4) {
        const int row = idx / Q, j = idx - row * Q;
        const T2* p = buf + row * pitch + j;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[b][r] = p[r * Q];
      }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < B4; ++b) {
      const int idx = tid + b * NT;
      if (NB4 % NT == 0 || idx < NB4) {
        const int row = idx / Q, j = idx - row * Q;
        const int k = j & (Ns - 1);
        if (pass > 0) {
          const int stride = N / (4 * Ns);
#pragma unroll
          for (int r = 1; r < 4; ++r) {
            T2 w = tw[k * r * stride];
            if (INV) w.y = -w.y;
            v[b][r] = cmul(v[b][r], w);
          }
        }
        radix4<INV>(v[b]);
        T2* p = buf + row * pitch + (j - k) * 4 + k;
#pragma unroll
        for (int r = 0; r < 4; ++r) p[r * Ns] = v[b][r];
      }
    }
    __syncthreads();
  }
  if constexpr (LOG % 2 == 1) {
    constexpr int H = N / 2;
    constexpr int NB2 = ROWS * H;
    constexpr int B2 = (NB2 + NT - 1) / NT;
    constexpr int Ns = N / 2;  // final radix-2 pass
    T2 v[B2][2];
#pragma unroll
    for (int b = 0; b < B2; ++b) {
      const int idx = tid + b * NT;
      if (NB2 % NT == 0 || idx < NB2) {
        const int row = idx / H, j = idx - row * H;
        v[b][0] = buf[row * pitch + j];
        v[b][1] = buf[row * pitch + j + H];
      }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < B2; ++b) {
      const int idx = tid + b * NT;
      if (NB2 % NT == 0 || idx < NB2) {
        const int row = idx / H, j = idx - row * H;
        const int k = j & (Ns - 1);  // = j
        T2 w = tw[k];
        if (INV) w.y = -w.y;
        const T2 x1 = cmul(v[b][1], w);
        buf[row * pitch + k] = cadd(v[b][0], x1);
        buf[row * pitch + k + Ns] = csub(v[b][0], x1);
      }
    }
    __syncthreads();
  }
}

}  // namespace dev
}  // namespace channel
