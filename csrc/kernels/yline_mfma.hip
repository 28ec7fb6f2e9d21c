// Dense wall-normal first derivative on the matrix cores (v_mfma_f64_16x16x4_f64): the MFMA
// experiment for the one GEMM-shaped y operator.
//
// The compact D1 is D = A1^-1 B1 with k-independent A1 (tridiagonal) and B1 (tridiagonal interior
// stencil + 3-point one-sided wall closures) — what the reference rebuilds and solves with cuSPARSE
// on every call (derivatives_nu_double.cu:209-285, 390-415).  K-SPEC applies it as a partitioned
// Thomas + PCR solve in registers (O(NY) per line).  Here the dense NY x NY matrix (precomputed on
// the host) multiplies a block of lines as a GEMM: Y[NP x 16] = D[NP x NP] X[NP x 16], the 16
// columns being 8 lines x (re, im), 16 x 16 output tiles accumulated over NP/4 k-steps.
//
// Measured A/B on MI355X (profiles/r02_mfma_d1_ab.md, 65,536 complex fp64 lines): MFMA / PCR time
// = 0.91 at NY = 33, 1.15 at 65, 2.02 at 129, 2.13 at 192 — the fp64 matrix rate equals the fp64
// vector rate on this part, and the dense product does NY^2 multiply-adds per real line against
// O(NY) for the solve.  K-SPEC therefore keeps the PCR solve on every BASELINE grid (NY >= 129);
// the kernel and its oracle test stay as the measured alternative.
#include <hip/hip_runtime.h>

#include <vector>

#include "channel/common.hpp"
#include "channel/kernels.hpp"

namespace channel {

namespace {
constexpr int kMaxNP = 192;  // NY <= 192 (R <= 3 in the y-line kernels)
}

void DenseD1Dev::upload(const YGrid& g, hipStream_t stream) {
  release();
  N = g.N;
  CH_CHECK(N >= 4 && N <= kMaxNP, "dense D1: NY must be in [4, " << kMaxNP << "]");
  NP = (N + 15) / 16 * 16;
  // column c of D = A1^-1 (B1 e_c): B1 column, then a Thomas solve with A1 (unit diagonal)
  std::vector<double> D(static_cast<size_t>(NP) * NP, 0.0);
  std::vector<double> b(N), cp(N), dp(N), x(N);
  for (int c = 0; c < N; ++c) {
    std::fill(b.begin(), b.end(), 0.0);
    for (int i = 1; i < N - 1; ++i) {
      if (c == i - 1) b[i] += g.d1_rm[i];
      if (c == i) b[i] += g.d1_rc[i];
      if (c == i + 1) b[i] += g.d1_rp[i];
    }
    for (int k = 0; k < 3; ++k) {
      if (c == k) b[0] += g.d1_w0[k];
      if (c == N - 1 - k) b[N - 1] += g.d1_wN[k];
    }
    // A1 x = b: A1[j][j-1] = d1_lo[j], A1[j][j] = 1, A1[j][j+1] = d1_up[j]
    cp[0] = g.d1_up[0];
    dp[0] = b[0];
    for (int j = 1; j < N; ++j) {
      const double m = 1.0 - g.d1_lo[j] * cp[j - 1];
      cp[j] = j < N - 1 ? g.d1_up[j] / m : 0.0;
      dp[j] = (b[j] - g.d1_lo[j] * dp[j - 1]) / m;
    }
    x[N - 1] = dp[N - 1];
    for (int j = N - 2; j >= 0; --j) x[j] = dp[j] - cp[j] * x[j + 1];
    for (int r = 0; r < N; ++r) D[static_cast<size_t>(r) * NP + c] = x[r];
  }
  HIP_CHECK(hipMalloc(&d, D.size() * sizeof(double)));
  HIP_CHECK(hipMemcpyAsync(d, D.data(), D.size() * sizeof(double), hipMemcpyHostToDevice, stream));
  HIP_CHECK(hipStreamSynchronize(stream));
}

void DenseD1Dev::release() {
  if (d) (void)hipFree(d);
  d = nullptr;
}

// 4 waves, 8 lines per block.  MFMA operand maps (f64 16x16x4): A lane l = A[l&15][k = l>>4],
// B lane l = B[k = l>>4][l&15], C/D register i of lane l = C[(l>>4) + 4 i][l&15].
__global__ void __launch_bounds__(256) d1_dense_mfma_kernel(const double* __restrict__ D, const double2* __restrict__ in,
                                                            double2* __restrict__ out, int N, int NP, int lines) {
  using d4 = double __attribute__((ext_vector_type(4)));
  __shared__ double xs[kMaxNP * 16];  // [row][col], col = 2 * line + (re, im)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int line0 = blockIdx.x * 8;
  for (int e = tid; e < NP * 8; e += 256) {
    const int y = e >> 3, l = e & 7;
    double2 v{0.0, 0.0};
    if (y < N && line0 + l < lines) v = in[static_cast<size_t>(y) * lines + line0 + l];
    xs[y * 16 + 2 * l] = v.x;
    xs[y * 16 + 2 * l + 1] = v.y;
  }
  __syncthreads();
  const int NT = NP / 16, NK = NP / 4;
  const int col = lane & 15, l = col >> 1;
  for (int t = w; t < NT; t += 4) {
    // two accumulators (even / odd k-steps): two independent MFMA chains in flight
    d4 acc = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    const double* drow = D + static_cast<size_t>(t * 16 + (lane & 15)) * NP + (lane >> 4);
    const double* xcol = xs + (lane >> 4) * 16 + col;
    int kk = 0;
    for (; kk + 1 < NK; kk += 2) {
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(drow[4 * kk], xcol[64 * kk], acc, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(drow[4 * kk + 4], xcol[64 * kk + 64], acc1, 0, 0, 0);
    }
    if (kk < NK) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(drow[4 * kk], xcol[64 * kk], acc, 0, 0, 0);
    acc += acc1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = t * 16 + (lane >> 4) + 4 * i;
      if (row < N && line0 + l < lines)
        reinterpret_cast<double*>(out + static_cast<size_t>(row) * lines + line0 + l)[col & 1] = acc[i];
    }
  }
}

void d1_dense_mfma(const DenseD1Dev& m, const void* in, void* out, int lines, hipStream_t stream) {
  CH_CHECK(m.d != nullptr && lines > 0, "dense D1: not uploaded");
  dim3 grid((lines + 7) / 8), block(256);
  hipLaunchKernelGGL(d1_dense_mfma_kernel, grid, block, 0, stream, m.d, static_cast<const double2*>(in),
                     static_cast<double2*>(out), m.N, m.NP, lines);
  HIP_LAUNCH_CHECK(stream);
}

}  // namespace channel
