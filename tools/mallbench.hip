// Infinity Cache (MALL) vs HBM bandwidth for streaming reads, writes and copies, by footprint.
// The transform stage keeps its x-expanded intermediates (~100 MB per y-chunk) resident in the
// 256 MiB Infinity Cache; this measures what bandwidth that residency can buy on MI355X, i.e. the
// floor the stage is accounted against.
//
//   hipcc --offload-arch=gfx950 -O3 tools/mallbench.hip -o /tmp/mallbench && /tmp/mallbench
//
// Each kernel is persistent-free grid-stride, 16-B accesses, 8 waves per CU; each size is timed
// over 50 back-to-back launches after 5 warm-ups (the footprint is re-touched every launch, so
// footprints below ~256 MiB are served from the cache after the first pass).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                   \
  do {                                                          \
    hipError_t e_ = (x);                                        \
    if (e_ != hipSuccess) {                                     \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_)); \
      std::exit(1);                                             \
    }                                                           \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(512) rd(const f4* __restrict__ a, size_t n, float* __restrict__ sink) {
  f4 acc = {0, 0, 0, 0};
  const size_t st = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i + 3 * st < n; i += 4 * st) acc += a[i] + a[i + st] + a[i + 2 * st] + a[i + 3 * st];
  for (; i < n; i += st) acc += a[i];
  if (acc.x + acc.y + acc.z + acc.w == 1.2345f) sink[0] = acc.x;  // keeps the loads alive
}

__global__ void __launch_bounds__(512) wr(f4* __restrict__ a, size_t n, float v) {
  const size_t st = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += st) a[i] = f4{v, v, v, v};
}

__global__ void __launch_bounds__(512) cp(const f4* __restrict__ a, f4* __restrict__ b, size_t n) {
  const size_t st = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i + st < n; i += 2 * st) {
    const f4 x = a[i], y = a[i + st];
    b[i] = x;
    b[i + st] = y;
  }
  for (; i < n; i += st) b[i] = a[i];
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t maxb = size_t(2) << 30;
  f4 *a, *b;
  float* sink;
  CK(hipMalloc(&a, maxb));
  CK(hipMalloc(&b, maxb));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 0, maxb));
  CK(hipMemset(b, 0, maxb));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = cus * 4;  // 512-thread blocks, 4 per CU = 32 waves per CU
  const size_t mbs[] = {16, 32, 64, 100, 128, 160, 192, 224, 256, 320, 512, 2048};
  std::printf("%8s %12s %12s %12s   (TB/s; copy counts read + write bytes)\n", "MB", "read", "write", "copy");
  for (size_t mb : mbs) {
    const size_t bytes = mb << 20, n = bytes / 16;
    const int reps = 50;
    float t[3];
    for (int k = 0; k < 3; ++k) {
      auto launch = [&] {
        if (k == 0) hipLaunchKernelGGL(rd, dim3(grid), dim3(512), 0, 0, a, n, sink);
        else if (k == 1) hipLaunchKernelGGL(wr, dim3(grid), dim3(512), 0, 0, a, n, 1.0f);
        else hipLaunchKernelGGL(cp, dim3(grid), dim3(512), 0, 0, a, b, n / 2);  // footprint = mb
      };
      for (int w = 0; w < 5; ++w) launch();
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[k] = ms / reps;
    }
    const double gb = bytes / 1e9;
    std::printf("%8zu %12.2f %12.2f %12.2f\n", mb, gb / t[0], gb / t[1], gb / t[2]);
  }
  return 0;
}
