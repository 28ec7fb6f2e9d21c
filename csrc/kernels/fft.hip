// Transform stages between spectral and physical space: host API, twiddle tables and the length
// dispatch.  The kernels (x transforms, z physical stage, test C2C) are in fft_impl.hpp and are
// instantiated per length family in fft_pow2.hip and fft_r{3,5,7,9,11,13,15}.hip.
#include "fft_impl.hpp"

namespace channel {

using namespace dev;

static void build_reg_twiddles(int n, bool fp64, void** out);

XVariant& xfft_variant_slot() {
  static thread_local XVariant v;
  return v;
}
static thread_local XVariant g_last_backward;
static std::string xfft_variant_string(const XVariant& v);
std::string xfft_last_variant() { return xfft_variant_string(xfft_variant_slot()); }
std::string xfft_last_backward_variant() { return xfft_variant_string(g_last_backward); }
static std::string xfft_variant_string(const XVariant& v) {
  std::string s = std::string(v.kernel) + "<" + std::to_string(v.nn) + ", " + (v.f64 ? "double" : "float") + ", " +
                  (v.seg ? "true" : "false") + ", " + std::to_string(v.wide) + ", " + std::to_string(v.sm) + ", " +
                  std::to_string(v.v) + ", " + std::to_string(v.sl);
  if (v.cmb >= 0) s += v.cmb ? ", true" : ", false";
  return s + ">";
}

void Twiddles::build(int n_, bool fp64_) {
  release();
  n = n_;
  fp64 = fp64_;
  const double two_pi = 2.0 * std::acos(-1.0);
  // N-point tables, then the z stage's real-signal half-transform tables (HalfPlan<n>)
  const int sz0 = fft_twiddle_size(n);
  const int szh = fft_half_twiddle_size(n);
  // n = 1024: the z stage's 4 x 16 x 16 tables follow (fft1024_4x16x16): [15][64] W_1024^(j r),
  // then [15][4] W_64^(k r) = W_1024^(16 k r)
  const int sz = sz0 + szh + (n == 1024 ? kR4TwSize : 0);
  std::vector<double2> h(sz, double2{1.0, 0.0});
  auto w = [&](int m) { return double2{std::cos(two_pi * m / n), -std::sin(two_pi * m / n)}; };
  fft_twiddle_fill(n, [&](int i, int m) { h[i] = w(m); });
  fft_half_twiddle_fill(n, [&](int i, int m) { h[sz0 + i] = w(m); });
  if (n == 1024) {
    const int o = sz0 + szh;
    for (int r = 1; r < 16; ++r) {
      for (int j = 0; j < 64; ++j) h[o + (r - 1) * 64 + j] = w(j * r);
      for (int k = 0; k < 4; ++k) h[o + kR4Tw2 + (r - 1) * 4 + k] = w(16 * k * r);
    }
  }
  if (fp64) {
    HIP_CHECK(hipMalloc(&buf, sz * sizeof(double2)));
    HIP_CHECK(hipMemcpy(buf, h.data(), sz * sizeof(double2), hipMemcpyHostToDevice));
  } else {
    std::vector<float2> hf(sz);
    for (int i = 0; i < sz; ++i) hf[i] = float2{static_cast<float>(h[i].x), static_cast<float>(h[i].y)};
    HIP_CHECK(hipMalloc(&buf, sz * sizeof(float2)));
    HIP_CHECK(hipMemcpy(buf, hf.data(), sz * sizeof(float2), hipMemcpyHostToDevice));
  }
  if (n == 1024) build_reg_twiddles(n, fp64, &reg);
}

void Twiddles::release() {
  if (buf) (void)hipFree(buf);
  if (reg) (void)hipFree(reg);
  buf = reg = nullptr;
}

// transform lengths with kernels: 2^k (16..2048), 3*2^k (48..1536), 5*2^k (80..1280),
// 7*2^k (112..1792), 9*2^k (144..1152), 15*2^k (240..1920), 11*2^k (176..1408), 13*2^k (208..1664)
#define CH_CASE_N(V, ...) \
  case V: { constexpr int NN = V; __VA_ARGS__; } break;
#define CH_DISPATCH_N(N_, ...)                                                                              \
  switch (N_) {                                                                                             \
    CH_CASE_N(16, __VA_ARGS__) CH_CASE_N(32, __VA_ARGS__) CH_CASE_N(64, __VA_ARGS__)                        \
    CH_CASE_N(128, __VA_ARGS__) CH_CASE_N(256, __VA_ARGS__) CH_CASE_N(512, __VA_ARGS__)                     \
    CH_CASE_N(1024, __VA_ARGS__) CH_CASE_N(2048, __VA_ARGS__)                                               \
    CH_CASE_N(48, __VA_ARGS__) CH_CASE_N(96, __VA_ARGS__) CH_CASE_N(192, __VA_ARGS__)                       \
    CH_CASE_N(384, __VA_ARGS__) CH_CASE_N(768, __VA_ARGS__) CH_CASE_N(1536, __VA_ARGS__)                    \
    CH_CASE_N(80, __VA_ARGS__) CH_CASE_N(160, __VA_ARGS__) CH_CASE_N(320, __VA_ARGS__)                      \
    CH_CASE_N(640, __VA_ARGS__) CH_CASE_N(1280, __VA_ARGS__)                                                \
    CH_CASE_N(112, __VA_ARGS__) CH_CASE_N(224, __VA_ARGS__) CH_CASE_N(448, __VA_ARGS__)                     \
    CH_CASE_N(896, __VA_ARGS__) CH_CASE_N(1792, __VA_ARGS__)                                                \
    CH_CASE_N(144, __VA_ARGS__) CH_CASE_N(288, __VA_ARGS__) CH_CASE_N(576, __VA_ARGS__)                     \
    CH_CASE_N(1152, __VA_ARGS__) CH_CASE_N(240, __VA_ARGS__) CH_CASE_N(480, __VA_ARGS__)                    \
    CH_CASE_N(960, __VA_ARGS__) CH_CASE_N(1920, __VA_ARGS__)                                                \
    CH_CASE_N(176, __VA_ARGS__) CH_CASE_N(352, __VA_ARGS__) CH_CASE_N(704, __VA_ARGS__)                     \
    CH_CASE_N(1408, __VA_ARGS__) CH_CASE_N(208, __VA_ARGS__) CH_CASE_N(416, __VA_ARGS__)                    \
    CH_CASE_N(832, __VA_ARGS__) CH_CASE_N(1664, __VA_ARGS__)                                                \
    default: CH_CHECK(false, "unsupported FFT length " << N_);                                              \
  }

// one segment: plain [y][x][kz]; otherwise the table must tile [0, NX)
static XArgs norm_pseg(const XArgs& in) {
  XArgs a = in;
  a.diag = fft_diag();
  if (a.npseg <= 1) {
    a.npseg = 1;
    a.x_start[0] = 0;
    a.x_start[1] = a.NX;
    a.poff[0] = 0;
  }
  CH_CHECK(a.npseg <= 8 && a.x_start[0] == 0 && a.x_start[a.npseg] == a.NX, "x transform: bad x segment table");
  return a;
}

void xfft_backward(const XArgs& a_in, const XSrc& src, void* phys, const Twiddles& tw, bool fp64, hipStream_t s) {
  const XArgs a = norm_pseg(a_in);
  CH_CHECK(tw.n == a.NX && tw.fp64 == fp64, "xfft_backward: twiddle table mismatch");
  CH_CHECK(a.ny > 0 && a.nkz > 0, "xfft_backward: empty");
  // the first pass skips the zero band of the 2/3 rule at compile time (wave_pass ZB)
  CH_CHECK(a.Kx == a.NX / 3 && a.nkx == 2 * a.Kx + 1, "xfft_backward: retained kx must be the 2/3 rule's (Kx = NX/3)");
  CH_CHECK(a.field_stride_spec < (1LL << 32), "xfft_backward: per-field spectral block exceeds 32-bit offsets");
  if (a.combine) {
    for (int j = 0; j < kCmbInputs; ++j)
      CH_CHECK(src.fld[j] && (src.self_seg < 0 || src.self_fld[j]), "xfft_backward: combine mode input field " << j << " missing");
  }
  CH_CHECK(static_cast<long long>(a.ny) * a.NX * a.nkz < (1LL << 32), "xfft_backward: per-field plane block exceeds 32-bit offsets");
  // one-source / blocked-layout paths address with 32-bit BYTE offsets (fft_impl.hpp at_byte)
  const long long esz = fp64 ? 16 : 8;
  CH_CHECK(static_cast<long long>(a.ny) * a.NX * a.nkz * esz < (1LL << 32),
           "xfft_backward: a field's x-expanded chunk exceeds 4 GiB (use smaller y chunks)");
  CH_CHECK(!a.kzb || (a.combine ? static_cast<long long>(spec_rows(kSpecKzBlock, a.spec_y0 + a.ny)) * a.nkx * a.nkzs
                               : a.field_stride_spec) * esz < (1LL << 32),
           "xfft_backward: blocked spectral field exceeds 4 GiB");
  CH_CHECK(src.nsrc > 1 || src.self_seg >= 0 || static_cast<long long>(a.ny) * a.nkx * a.nkz * esz < (1LL << 32),
           "xfft_backward: a field's spectral chunk exceeds 4 GiB (use smaller y chunks)");
  CH_DISPATCH_N(a.NX, fft_xb_len<NN>(a, src, phys, tw, fp64, s));
  g_last_backward = xfft_variant_slot();
  HIP_LAUNCH_CHECK(s);
}

void xfft_forward(const XArgs& a_in, const void* phys, const XDst& dst, const Twiddles& tw, bool fp64, hipStream_t s) {
  const XArgs a = norm_pseg(a_in);
  CH_CHECK(tw.n == a.NX && tw.fp64 == fp64, "xfft_forward: twiddle table mismatch");
  CH_CHECK(a.Kx == a.NX / 3 && a.nkx == 2 * a.Kx + 1, "xfft_forward: retained kx must be the 2/3 rule's (Kx = NX/3)");
  CH_CHECK(static_cast<long long>(a.ny) * a.NX * a.nkz < (1LL << 32), "xfft_forward: per-field plane block exceeds 32-bit offsets");
  CH_CHECK(static_cast<long long>(a.ny) * a.nkx * a.nkz < (1LL << 32), "xfft_forward: per-field spectral block exceeds 32-bit offsets");
  const long long esz = fp64 ? 16 : 8;
  CH_CHECK(static_cast<long long>(a.ny) * a.NX * a.nkz * esz < (1LL << 32),
           "xfft_forward: a field's x-expanded chunk exceeds 4 GiB (use smaller y chunks)");
  CH_CHECK(!a.kzb || a.field_stride_spec * esz < (1LL << 32), "xfft_forward: blocked spectral field exceeds 4 GiB");
  CH_CHECK(dst.ndst > 1 || dst.self_seg >= 0 || static_cast<long long>(a.ny) * a.nkx * a.nkz * esz < (1LL << 32),
           "xfft_forward: a field's spectral chunk exceeds 4 GiB (use smaller y chunks)");
  CH_DISPATCH_N(a.NX, fft_xf_len<NN>(a, phys, dst, tw, fp64, s));
  HIP_LAUNCH_CHECK(s);
}

// twiddles of the register z stage: [M][64] W_N^(n1 k2) then [4][16] W_64^(a c) (forward sign)
static void build_reg_twiddles(int n, bool fp64, void** out) {
  const int M = n / 64;
  const double two_pi = 2.0 * std::acos(-1.0);
  std::vector<double2> h(n + 64);
  for (int n1 = 0; n1 < M; ++n1)
    for (int k2 = 0; k2 < 64; ++k2) {
      const double ang = -two_pi * static_cast<double>(n1 * k2) / n;
      h[n1 * 64 + k2] = double2{std::cos(ang), std::sin(ang)};
    }
  for (int aa = 0; aa < 4; ++aa)
    for (int c = 0; c < 16; ++c) {
      const double ang = -two_pi * static_cast<double>(aa * c) / 64.0;
      h[n + aa * 16 + c] = double2{std::cos(ang), std::sin(ang)};
    }
  if (fp64) {
    HIP_CHECK(hipMalloc(out, h.size() * sizeof(double2)));
    HIP_CHECK(hipMemcpy(*out, h.data(), h.size() * sizeof(double2), hipMemcpyHostToDevice));
  } else {
    std::vector<float2> hf(h.size());
    for (size_t i = 0; i < h.size(); ++i) hf[i] = float2{static_cast<float>(h[i].x), static_cast<float>(h[i].y)};
    HIP_CHECK(hipMalloc(out, hf.size() * sizeof(float2)));
    HIP_CHECK(hipMemcpy(*out, hf.data(), hf.size() * sizeof(float2), hipMemcpyHostToDevice));
  }
}

void zphys(const ZArgs& a_in, void* fields, const Twiddles& tw, bool fp64, hipStream_t s) {
  ZArgs a = a_in;
  a.diag = fft_diag();
  if (a.nseg <= 1) {
    a.nseg = 1;
    a.kz_start[0] = 0;
    a.kz_start[1] = a.nkz;
    a.off[0] = 0;
  }
  CH_CHECK(a.nseg <= 8 && a.kz_start[0] == 0 && a.kz_start[a.nseg] == a.nkz, "zphys: bad kz segment table");
  CH_CHECK(tw.n == a.Nzp && tw.fp64 == fp64, "zphys: twiddle table mismatch");
  CH_CHECK(a.nkz - 1 < a.Nzp / 2, "zphys: retained kz must be below Nyquist");
  if (a.ny == 0) return;
  if (a.Nzp == 1024 && zreg_enabled()) {
    CH_CHECK(tw.reg, "zphys: register-FFT twiddles missing");
    const long long nrows = static_cast<long long>(a.ny) * a.NX;
    dim3 grid(static_cast<unsigned>((nrows + ZW - 1) / ZW));
    if (fp64) {
      if (a.nseg > 1)
        hipLaunchKernelGGL((zphys_reg_kernel<16, double, true>), grid, dim3(256), 0, s, a, static_cast<double2*>(fields),
                           static_cast<const double2*>(tw.reg));
      else
        hipLaunchKernelGGL((zphys_reg_kernel<16, double, false>), grid, dim3(256), 0, s, a,
                           static_cast<double2*>(fields), static_cast<const double2*>(tw.reg));
    } else {
      if (a.nseg > 1)
        hipLaunchKernelGGL((zphys_reg_kernel<16, float, true>), grid, dim3(256), 0, s, a, static_cast<float2*>(fields),
                           static_cast<const float2*>(tw.reg));
      else
        hipLaunchKernelGGL((zphys_reg_kernel<16, float, false>), grid, dim3(256), 0, s, a, static_cast<float2*>(fields),
                           static_cast<const float2*>(tw.reg));
    }
    HIP_LAUNCH_CHECK(s);
    return;
  }
  CH_DISPATCH_N(a.Nzp, fft_zp_len<NN>(a, fields, tw, fp64, s));
  HIP_LAUNCH_CHECK(s);
}

void fft_c2c_test(void* data, int n, int batch, int dir, const Twiddles& tw, bool fp64, hipStream_t s) {
  CH_CHECK(tw.n == n && tw.fp64 == fp64, "fft_c2c_test: twiddle table mismatch");
  CH_DISPATCH_N(n, fft_test_len<NN>(data, batch, dir, tw, fp64, s));
  HIP_LAUNCH_CHECK(s);
}

}  // namespace channel
