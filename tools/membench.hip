// HBM bandwidth calibration for the access patterns the transform kernels use.
//   contiguous : float4 copy, grid-stride
//   seg<S>     : copy where each group of S bytes is contiguous and groups are `stride` bytes
//                apart on the read side and written contiguously (and the reverse), i.e. the
//                [y][x][kz] <-> chunked patterns of the x-transforms with S = C * 8 bytes.
// Build: hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o bin/membench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e));         \
      std::exit(1);                                                     \
    }                                                                   \
  } while (0)

__global__ void copy4(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// element = float2 (8 B).  rows of `rowlen` elements, chunk of C elements per row is gathered:
// gather (READ strided, WRITE contiguous) when dir=0, scatter when dir=1.
template <int C>
__global__ void seg_copy(const float2* __restrict__ a, float2* __restrict__ b, int nrows, int rowlen, int dir) {
  const int nchunks = rowlen / C;
  const size_t total = (size_t)nrows * rowlen;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    // e enumerates the chunked layout [chunk][row][c]
    const int c = e % C;
    const size_t rest = e / C;
    const int row = rest % nrows;
    const int chunk = rest / nrows;
    const size_t rowmajor = (size_t)row * rowlen + chunk * C + c;
    if (dir == 0) b[e] = a[rowmajor];
    else b[rowmajor] = a[e];
  }
  (void)nchunks;
}

int main() {
  const size_t bytes = size_t(2) << 30;  // 2 GiB per buffer
  void *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int reps = 10;
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    std::printf("%-40s %8.3f ms  %7.2f TB/s (read+write)\n", name, ms, 2.0 * bytes / (ms * 1e-3) / 1e12);
  };
  timeit("contiguous float4 copy", [&] { copy4<<<256 * 64, 256>>>((const float4*)a, (float4*)b, bytes / 16); });
  const int rowlen = 342;  // nkz
  const int nrows = (int)(bytes / 8 / 344);
  char name[128];
#define SEG(CC)                                                                                        \
  for (int dir = 0; dir < 2; ++dir) {                                                                   \
    std::snprintf(name, sizeof name, "%d-B segments (%s)", CC * 8, dir ? "strided write" : "strided read"); \
    timeit(name, [&] { seg_copy<CC><<<256 * 64, 256>>>((const float2*)a, (float2*)b, nrows, (rowlen / CC) * CC, dir); }); \
  }
  SEG(2)
  SEG(4)
  SEG(8)
  SEG(16)
  SEG(38)
  return 0;
}
