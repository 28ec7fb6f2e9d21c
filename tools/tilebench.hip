// HBM ceiling of the K-SPEC tile access pattern: fields stored [y][line] (complex fp32), a tile =
// W consecutive lines x all NY rows, persistent workgroups walking tiles with the XCD-aware order.
// Each tile reads NIN fields and writes NOUT fields (copy + scale, no LDS, no compute), so the
// time is the data-movement floor of that pattern for a given W / threads / occupancy.
// Build: hipcc --offload-arch=gfx950 -O3 tools/tilebench.hip -o bin/tilebench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                   \
  do {                                                          \
    hipError_t e = (x);                                         \
    if (e != hipSuccess) {                                      \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e)); \
      std::exit(1);                                             \
    }                                                           \
  } while (0)

__device__ __forceinline__ unsigned xcd_remap(unsigned b, unsigned n) {
  const unsigned per = n / 8, rem = n % 8, x = b % 8, k = b / 8;
  return (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + k;
}

struct Fields {
  const float2* in[8];
  float2* out[8];
};

// THREADS threads per block, W lines per tile: thread t copies rows t/W + (THREADS/W) q of line t%W
// B = 0: [y][line]; B > 0: blocked [line / B][y][line % B] (a tile of W <= B lines inside a block)
template <int W, int THREADS, int NIN, int NOUT, int B = 0>
__global__ void __launch_bounds__(THREADS) tile_copy(Fields f, int N, int lines, int sink) {
  constexpr int RPP = THREADS / W;  // rows per pass
  const int ntiles = (lines + W - 1) / W;
  const int lb = static_cast<int>(xcd_remap(blockIdx.x, gridDim.x));
  const int y0 = threadIdx.x / W, l = threadIdx.x % W;
  for (int tile = lb; tile < ntiles; tile += gridDim.x) {
    const int line = tile * W + l;
    if (line >= lines) continue;
    auto at = [&](int y) -> size_t {
      if constexpr (B == 0) return static_cast<size_t>(y) * lines + line;
      else return (static_cast<size_t>(line / B) * N + y) * B + line % B;
    };
    // field by field, as K-SPEC stages them: every row of the tile for one field, then the next
    float2 acc = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < NIN; ++i) {
#pragma unroll 8
      for (int y = y0; y < N; y += RPP) {
        const float2 v = f.in[i][at(y)];
        acc.x += v.x;
        acc.y += v.y;
      }
    }
    if (sink) f.out[7][line] = acc;
#pragma unroll
    for (int i = 0; i < NOUT; ++i) {
#pragma unroll 8
      for (int y = y0; y < N; y += RPP) f.out[i][at(y)] = float2{acc.x + y, acc.y};
    }
  }
}

// K-SPEC-like: Q rows per thread fully unrolled, field i+1 (and i+2) loaded before field i is used
template <int W, int THREADS, int NIN, int NOUT, int B, int Q>
__global__ void __launch_bounds__(THREADS) tile_pipe(Fields f, int N, int lines, int sink) {
  constexpr int RPP = THREADS / W;
  const int ntiles = (lines + W - 1) / W;
  const int lb = static_cast<int>(xcd_remap(blockIdx.x, gridDim.x));
  const int y0 = threadIdx.x / W, l = threadIdx.x % W;
  for (int tile = lb; tile < ntiles; tile += gridDim.x) {
    const int line = min(tile * W + l, lines - 1);
    auto at = [&](int q) -> size_t {
      const int y = min(y0 + RPP * q, N - 1);
      if constexpr (B == 0) return static_cast<size_t>(y) * lines + line;
      else return (static_cast<size_t>(line / B) * N + y) * B + line % B;
    };
    float2 p0[Q], p1[Q], acc = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < Q; ++q) p0[q] = f.in[0][at(q)];
#pragma unroll
    for (int i = 0; i < NIN; ++i) {
      if (i + 1 < NIN) {
#pragma unroll
        for (int q = 0; q < Q; ++q) p1[q] = f.in[i + 1][at(q)];
      }
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        acc.x += p0[q].x;
        acc.y += p0[q].y;
      }
#pragma unroll
      for (int q = 0; q < Q; ++q) p0[q] = p1[q];
    }
    if (sink) f.out[7][line] = acc;
#pragma unroll
    for (int i = 0; i < NOUT; ++i) {
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (y0 + RPP * q < N) f.out[i][at(q)] = float2{acc.x + q, acc.y};
    }
  }
}

template <int W, int THREADS, int NIN, int NOUT, int B, int Q>
static void runp(const Fields& f, int N, int lines, int blocks_per_cu, int cus, double bytes) {
  auto k = tile_pipe<W, THREADS, NIN, NOUT, B, Q>;
  const int grid = std::min((lines + W - 1) / W, blocks_per_cu * cus);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(grid), dim3(THREADS), 0, 0, f, N, lines, 0);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int it = 0; it < 5; ++it) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k, dim3(grid), dim3(THREADS), 0, 0, f, N, lines, 0);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = std::min(best, ms);
  }
  std::printf("pipe B=%3d W=%3d threads=%4d blocks/CU=%d in=%d out=%d : %8.3f ms  %6.2f TB/s\n", B, W, THREADS, blocks_per_cu,
              NIN, NOUT, best, bytes / best / 1e9);
}

template <int W, int THREADS, int NIN, int NOUT, int B = 0>
static void run(const Fields& f, int N, int lines, int blocks_per_cu, int cus, double bytes) {
  auto k = tile_copy<W, THREADS, NIN, NOUT, B>;
  const int grid = std::min((lines + W - 1) / W, blocks_per_cu * cus);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(grid), dim3(THREADS), 0, 0, f, N, lines, 0);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int it = 0; it < 5; ++it) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k, dim3(grid), dim3(THREADS), 0, 0, f, N, lines, 0);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = std::min(best, ms);
  }
  std::printf("B=%3d W=%3d threads=%4d blocks/CU=%d in=%d out=%d : %8.3f ms  %6.2f TB/s\n", B, W, THREADS, blocks_per_cu, NIN, NOUT,
              best, bytes / best / 1e9);
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? std::atoi(argv[1]) : 385;
  const int lines = argc > 2 ? std::atoi(argv[2]) : 683 * 342;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t n = static_cast<size_t>(N) * lines;
  Fields f{};
  for (int i = 0; i < 8; ++i) {
    float2 *p, *q;
    CK(hipMalloc(&p, n * sizeof(float2)));
    CK(hipMalloc(&q, n * sizeof(float2)));
    CK(hipMemset(p, 0, n * sizeof(float2)));
    f.in[i] = p;
    f.out[i] = q;
  }
  const double fb = static_cast<double>(n) * sizeof(float2);
  std::printf("N=%d lines=%d field=%.1f MB CUs=%d\n", N, lines, fb / 1e6, cus);
  runp<4, 256, 7, 8, 0, 7>(f, N, lines, 1, cus, 15 * fb);
  runp<4, 256, 7, 8, 4, 7>(f, N, lines, 1, cus, 15 * fb);
  runp<4, 256, 7, 8, 8, 7>(f, N, lines, 1, cus, 15 * fb);
  runp<4, 256, 7, 8, 16, 7>(f, N, lines, 1, cus, 15 * fb);
  runp<4, 256, 7, 8, 0, 7>(f, N, lines, 2, cus, 15 * fb);
  runp<4, 256, 7, 8, 4, 7>(f, N, lines, 2, cus, 15 * fb);
  runp<4, 256, 7, 8, 8, 7>(f, N, lines, 2, cus, 15 * fb);
  runp<4, 256, 7, 8, 16, 7>(f, N, lines, 2, cus, 15 * fb);
  runp<8, 512, 7, 8, 0, 7>(f, N, lines, 1, cus, 15 * fb);
  runp<8, 512, 7, 8, 8, 7>(f, N, lines, 1, cus, 15 * fb);
  runp<8, 512, 7, 8, 16, 7>(f, N, lines, 1, cus, 15 * fb);
  runp<4, 256, 7, 0, 0, 7>(f, N, lines, 1, cus, 7 * fb);
  runp<4, 256, 7, 0, 8, 7>(f, N, lines, 1, cus, 7 * fb);
  runp<4, 256, 0, 8, 0, 7>(f, N, lines, 1, cus, 8 * fb);
  runp<4, 256, 0, 8, 8, 7>(f, N, lines, 1, cus, 8 * fb);
  return 0;
}
