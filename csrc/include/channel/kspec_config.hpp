// Compile-time configuration of the fused spectral kernel (K-SPEC, kernels/kspec.hip) per
// (R = rows per lane, storage type): lines per workgroup, cross-lane policy, prefetch slots.
#pragma once

#include "channel/common.hpp"
#include "channel/yline_device.hpp"

namespace channel {

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

// Lines (= waves) per workgroup.  One workgroup per CU holds the coefficient tables in LDS once.
// From R = 5 a line needs more than 256 registers (one wave per SIMD: 4 lines); up to R = 4, 8
// lines make 2 waves per SIMD.
template <int R, typename T>
constexpr int kspec_lines() {
#ifdef CH_KSPEC_W7
  if (R == 7) return CH_KSPEC_W7;
#endif
  return R <= 4 ? 8 : 4;
}

// Cross-lane policy: strides >= 4 through LDS wherever the scratch fits beside the tables.
template <int R, typename T>
constexpr int kspec_xmode() {
  return R <= 12 ? dev::kXlLds : dev::kXlDpp;
}

// register prefetch slots for the input fields (prefetch distance); three at R = 7 measured the
// same as two (profiles/r03s3/ab_kspec_ns7.txt)
template <int R, typename T>
constexpr int kspec_slots() {
  // fp64 R = 3 (Re_tau~180, 3.7k lines: two rounds of waves, latency-bound): two slots measured
  // 0.470 ms/step at 128x129x128 against 0.475 / 0.502 with one (same box, run-to-run spread ~5 %;
  // profiles/r04/ab_small_grid.txt); fp32 R = 3: no difference
  return R <= 4 ? ((R == 3 && sizeof(T) == 8) ? 2 : 1) : (R <= 8 ? 2 : 1);
}

// dispatch a runtime R to the instantiated rows-per-lane values
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

// values exchanged at once by one wave (the 6-RHS implicit solve)
constexpr int kKspecXK = 6;

}  // namespace channel
