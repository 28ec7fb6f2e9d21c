// In-LDS batched complex FFT (Stockham autosort, mixed radix 16/15/12/10/9/8/7/6/5/4/3/2, radix 16 first).
//
// All threads of the workgroup cooperate on ROWS rows of length N held in LDS.  Each pass gathers
// its butterfly inputs into registers, synchronises, applies the inter-pass twiddles and an R-point
// DFT in registers, and writes the outputs back in place.  LDS addresses are padded by one slot per
// 16 elements (fft_pidx): with radix-16 first passes every store lane-stride becomes 17 elements
// (34 dwords), which is conflict-free for ds_write_b64, and the strided reads stay contiguous.
// Radix plans (fft_radices): powers of two 16, 16x2, ..., 16x16x8 (N = 16 ... 2048), and the
// lengths 3*2^k and 5*2^k from 48 / 80 with the odd factor in the last pass (e.g. 96 = 16x6,
// 384 = 16x8x3, 768 = 16x16x3, 1536 = 16x16x6, 1280 = 16x16x5): at most three LDS round trips per
// transform (the radix-4-only version needed log4 N + 1).
// Twiddles come from per-pass tables (FftPlan::T1/T2, built by fft_twiddle_fill), staged in LDS.
//
// Replaces the reference's cuFFT 2-D plans (fft.c:17-23), which take any NX and 2NZ-2; the length
// is a compile-time constant of the form 2^a 3^b 5^c with b + c <= 1.
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
// fp32: the same operations on the native 2-vector, so each complex add/sub is one v_pk_add_f32
// and a complex product one v_pk_mul_f32 + one v_pk_fma_f32 with operand swizzles (component-wise
// code left the pairing to the SLP vectoriser, which built its pairs with v_mov shuffles)
typedef float f2v_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v_t v2(float2 a) { return __builtin_bit_cast(f2v_t, a); }
__device__ __forceinline__ float2 c2v(f2v_t a) { return __builtin_bit_cast(float2, a); }
template <>
__device__ __forceinline__ float2 cadd<float2>(float2 a, float2 b) {
  return c2v(v2(a) + v2(b));
}
template <>
__device__ __forceinline__ float2 csub<float2>(float2 a, float2 b) {
  return c2v(v2(a) - v2(b));
}
template <>
__device__ __forceinline__ float2 cmul<float2>(float2 a, float2 b) {
  const f2v_t x = v2(a), y = v2(b);
  const f2v_t yr = {-y.y, y.x};
  return c2v(__builtin_elementwise_fma(x.yy, yr, x.xx * y));
}

// complex product by a twiddle loaded at run time: fp32 as v_pk_mul_f32 + v_pk_fma_f32 with the
// broadcasts and the swap in op_sel / op_sel_hi (the compiler built those operand pairs with two
// v_mov_b32 each)
template <bool CONJ, typename T2>
__device__ __forceinline__ T2 cmul_tw(T2 a, T2 b) {  // a * b, or a * conj(b)
  if constexpr (sizeof(T2) == 8) {
    const f2v_t x = v2(a), y = v2(b);
    f2v_t t, r;
    if constexpr (!CONJ) {
      // t = (ax*bx, ax*by); r = (-ay*by + t.x, ay*bx + t.y)
      asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(x), "v"(y));
      asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
          : "=v"(r) : "v"(x), "v"(y), "v"(t));
    } else {
      // t = (ax*bx, -ax*by); r = (ay*by + t.x, ay*bx + t.y)
      asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(t) : "v"(x), "v"(y));
      asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(x), "v"(y), "v"(t));
    }
    return c2v(r);
  } else {
    if constexpr (CONJ) b.y = -b.y;
    return cmul(a, b);
  }
}

// multiply by -i (forward) or +i (inverse)
template <bool INV, typename T2>
__device__ __forceinline__ T2 mul_mi(T2 d) {
  if constexpr (sizeof(T2) == 8) {  // float2: a swizzle + sign the packed adds can absorb
    const f2v_t v = v2(d);
    return c2v(INV ? f2v_t{-v.y, v.x} : f2v_t{v.y, -v.x});
  } else {
    return INV ? T2{-d.y, d.x} : T2{d.y, -d.x};
  }
}

// a + w b with w = -i (forward) or +i (inverse), and a - w b.  fp32: ONE v_pk_add_f32 each, the
// swap of b's halves and the sign riding on op_sel / neg (a separate mul_mi materialised the
// swapped value with a v_xor + v_mov pair per complex before the add: ~100 VALU per 1024-point
// z-stage row, tools/isa_mix.py)
__device__ __forceinline__ float2 pk_add_swap_nhi(float2 a, float2 b) {  // (ax + by, ay - bx)
  f2v_t r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(v2(a)), "v"(v2(b)));
  return c2v(r);
}
__device__ __forceinline__ float2 pk_add_swap_nlo(float2 a, float2 b) {  // (ax - by, ay + bx)
  f2v_t r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(v2(a)), "v"(v2(b)));
  return c2v(r);
}
template <bool INV, typename T2>
__device__ __forceinline__ T2 add_w(T2 a, T2 b) {  // a + (-+i) b
  if constexpr (sizeof(T2) == 8) return INV ? pk_add_swap_nlo(a, b) : pk_add_swap_nhi(a, b);
  else return cadd(a, mul_mi<INV>(b));
}
template <bool INV, typename T2>
__device__ __forceinline__ T2 sub_w(T2 a, T2 b) {  // a - (-+i) b
  if constexpr (sizeof(T2) == 8) return INV ? pk_add_swap_nhi(a, b) : pk_add_swap_nlo(a, b);
  else return csub(a, mul_mi<INV>(b));
}


// padded LDS index of logical element p of a row: one pad slot per 2^SH elements.  SH = 4 (the
// default): the stride-16 stores of a radix-16 first pass are conflict-free for ds_write_b64 and a
// contiguous 32-lane ds_read_b64 half meets one 2-way conflict (its 32 elements span 33 slots).
// SH = 5 (the 1024-point z stage): contiguous 32-lane reads are conflict-free (2 LDS cycles instead
// of 4) and the first pass's stride-16 stores take 2-way conflicts (8 cycles instead of 6), which
// nets fewer LDS cycles where a transform reads more than it writes at stride 16.
template <int SH = 4>
__device__ __forceinline__ constexpr int fft_pidx_s(int p) { return p + (p >> SH); }
__device__ __forceinline__ constexpr int fft_pidx(int p) { return fft_pidx_s<4>(p); }
template <int N>
struct FftPitch {
  static constexpr int value = N + N / 16 + (N >= 16 ? 0 : 1);
};

// ---- register DFTs (in place, natural order) --------------------------------------------------
template <bool INV, typename T2>
__device__ __forceinline__ void dft2(T2* v) {
  const T2 a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}

// compile-time zero (the pruned inputs of a zero-padded first pass): after inlining the compiler
// folds the test, so the butterflies below drop the terms instead of adding zeros through asm
template <typename T2>
__device__ __forceinline__ bool is_czero(T2 x) {
  return __builtin_constant_p(x.x) && __builtin_constant_p(x.y) && x.x == 0 && x.y == 0;
}

template <bool INV, typename T2>
__device__ __forceinline__ void dft4(T2* v) {
  const T2 a0 = cadd(v[0], v[2]), a1 = csub(v[0], v[2]);
  const T2 a2 = cadd(v[1], v[3]);
  T2 o1, o3;
  if (is_czero(v[1])) {  // d = -v3
    o1 = sub_w<INV>(a1, v[3]);
    o3 = add_w<INV>(a1, v[3]);
  } else if (is_czero(v[3])) {
    o1 = add_w<INV>(a1, v[1]);
    o3 = sub_w<INV>(a1, v[1]);
  } else {
    const T2 d = csub(v[1], v[3]);
    o1 = add_w<INV>(a1, d);
    o3 = sub_w<INV>(a1, d);
  }
  v[0] = cadd(a0, a2);
  v[1] = o1;
  v[2] = csub(a0, a2);
  v[3] = o3;
}
// dft4 whose input v[2] still has to be multiplied by w = -i (forward) / +i (inverse): the product
// folds into the first butterfly
template <bool INV, typename T2>
__device__ __forceinline__ void dft4_w2(T2* v) {
  const T2 a0 = add_w<INV>(v[0], v[2]), a1 = sub_w<INV>(v[0], v[2]);
  const T2 a2 = cadd(v[1], v[3]), d = csub(v[1], v[3]);
  v[0] = cadd(a0, a2);
  v[1] = add_w<INV>(a1, d);
  v[2] = csub(a0, a2);
  v[3] = sub_w<INV>(a1, d);
}
// x W_8^1 (forward sign; inverse: conjugate) = h (x + w x), x W_8^3 = -h (x - w x)
template <bool INV, typename T2>
__device__ __forceinline__ T2 mul_w8_1(T2 x) {
  using T = decltype(x.x);
  const T h = static_cast<T>(0.70710678118654752440);
  const T2 t = add_w<INV>(x, x);
  return T2{h * t.x, h * t.y};
}
template <bool INV, typename T2>
__device__ __forceinline__ T2 mul_w8_3(T2 x) {
  using T = decltype(x.x);
  const T h = static_cast<T>(-0.70710678118654752440);
  const T2 t = sub_w<INV>(x, x);
  return T2{h * t.x, h * t.y};
}

// DFT of length 4*Q computed as Q-point... (generic two-level decomposition R = 4 x S)
template <bool INV, typename T2>
__device__ __forceinline__ void dft8(T2* v) {
  using T = decltype(v[0].x);
  const T h = static_cast<T>(0.70710678118654752440);
  // stage 1: DFT4 over n = 2 n1 + n2 for fixed n2
  T2 a[2][4];
#pragma unroll
  for (int n2 = 0; n2 < 2; ++n2) {
#pragma unroll
    for (int n1 = 0; n1 < 4; ++n1) a[n2][n1] = v[2 * n1 + n2];
    dft4<INV>(a[n2]);
  }
  // twiddles W8^(n2*k1) for n2 = 1
  // k1=1: W8^1 = (h, -h) fwd ; k1=2: -i (folded into the radix-2 below) ; k1=3: W8^3 = (-h, -h)
  (void)h;
  a[1][1] = mul_w8_1<INV>(a[1][1]);
  a[1][3] = mul_w8_3<INV>(a[1][3]);
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    if (k1 == 2) {
      v[2] = add_w<INV>(a[0][2], a[1][2]);
      v[6] = sub_w<INV>(a[0][2], a[1][2]);
    } else {
      v[k1] = cadd(a[0][k1], a[1][k1]);
      v[k1 + 4] = csub(a[0][k1], a[1][k1]);
    }
  }
}

template <bool INV, typename T2>
__device__ __forceinline__ void dft16(T2* v) {
  using T = decltype(v[0].x);
  // n = 4 n1 + n2, k = k1 + 4 k2
  T2 a[4][4];
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) {
#pragma unroll
    for (int n1 = 0; n1 < 4; ++n1) a[n2][n1] = v[4 * n1 + n2];
    dft4<INV>(a[n2]);
  }
  // twiddles W16^(n2*k1)
  const T c1 = static_cast<T>(0.92387953251128675613), s1 = static_cast<T>(0.38268343236508977173);
  const T h = static_cast<T>(0.70710678118654752440);
  const T sg = INV ? T(1) : T(-1);  // sign of the sine part
  const T cs[10] = {T(1), c1, h, s1, T(0), -s1, -h, -c1, T(-1), -c1};
  const T sn[10] = {T(0), s1, h, c1, T(1), c1, h, s1, T(0), -s1};
  // m = 2, 6: h (x +- w x) (one packed add + one packed multiply); m = 4: w, folded into the
  // second-stage butterfly of k1 = 2 (dft4_w2)
#pragma unroll
  for (int n2 = 1; n2 < 4; ++n2)
#pragma unroll
    for (int k1 = 1; k1 < 4; ++k1) {
      const int m = n2 * k1;
      if (m == 2) {
        a[n2][k1] = mul_w8_1<INV>(a[n2][k1]);
      } else if (m == 6) {
        a[n2][k1] = mul_w8_3<INV>(a[n2][k1]);
      } else if (m != 4) {
        const T2 w{cs[m], sg * sn[m]};
        a[n2][k1] = cmul(a[n2][k1], w);
      }
    }
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    T2 b[4] = {a[0][k1], a[1][k1], a[2][k1], a[3][k1]};
    if (k1 == 2) dft4_w2<INV>(b);
    else dft4<INV>(b);
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) v[k1 + 4 * k2] = b[k2];
  }
}

// odd radices (forward sign e^{-2 pi i nk/R}; INV flips it)
template <bool INV, typename T2>
__device__ __forceinline__ void dft3(T2* v) {
  using T = decltype(v[0].x);
  const T s = static_cast<T>(0.86602540378443864676);  // sin 60
  const T2 t1 = cadd(v[1], v[2]), d = csub(v[1], v[2]);
  const T2 t2{v[0].x - T(0.5) * t1.x, v[0].y - T(0.5) * t1.y};
  const T2 m = mul_mi<INV>(T2{s * d.x, s * d.y});  // -i s d (forward)
  v[0] = cadd(v[0], t1);
  v[1] = cadd(t2, m);
  v[2] = csub(t2, m);
}
template <bool INV, typename T2>
__device__ __forceinline__ void dft5(T2* v) {
  using T = decltype(v[0].x);
  const T c1 = static_cast<T>(0.30901699437494742410), c2 = static_cast<T>(-0.80901699437494742410);
  const T s1 = static_cast<T>(0.95105651629515357212), s2 = static_cast<T>(0.58778525229247312917);
  const T2 t1 = cadd(v[1], v[4]), t2 = cadd(v[2], v[3]), t3 = csub(v[1], v[4]), t4 = csub(v[2], v[3]);
  const T2 a1{v[0].x + c1 * t1.x + c2 * t2.x, v[0].y + c1 * t1.y + c2 * t2.y};
  const T2 a2{v[0].x + c2 * t1.x + c1 * t2.x, v[0].y + c2 * t1.y + c1 * t2.y};
  const T2 b1 = mul_mi<INV>(T2{s1 * t3.x + s2 * t4.x, s1 * t3.y + s2 * t4.y});  // -i b1 (forward)
  const T2 b2 = mul_mi<INV>(T2{s2 * t3.x - s1 * t4.x, s2 * t3.y - s1 * t4.y});
  v[0] = cadd(v[0], cadd(t1, t2));
  v[1] = cadd(a1, b1);
  v[4] = csub(a1, b1);
  v[2] = cadd(a2, b2);
  v[3] = csub(a2, b2);
}

// W_R^m = exp(-2 pi i m / R) (forward sign) for the composite radices, compile-time tables
template <int R>
struct RootTable;
template <>
struct RootTable<7> {
  static constexpr double c[7] = {1.0, 0.62348980185873353053, -0.22252093395631440429, -0.90096886790241912624,
                                  -0.90096886790241912624, -0.22252093395631440429, 0.62348980185873353053};
  static constexpr double s[7] = {0.0, 0.78183148246802980871, 0.97492791218182360702, 0.43388373911755812048,
                                  -0.43388373911755812048, -0.97492791218182360702, -0.78183148246802980871};
};
template <>
struct RootTable<9> {
  static constexpr double c[9] = {1.0, 0.76604444311897803520, 0.17364817766693034885, -0.5, -0.93969262078590838405,
                                  -0.93969262078590838405, -0.5, 0.17364817766693034885, 0.76604444311897803520};
  static constexpr double s[9] = {0.0, 0.64278760968653932632, 0.98480775301220805936, 0.86602540378443864676,
                                  0.34202014332566873304, -0.34202014332566873304, -0.86602540378443864676,
                                  -0.98480775301220805936, -0.64278760968653932632};
};
template <>
struct RootTable<15> {
  static constexpr double c[15] = {1.0, 0.91354545764260089550, 0.66913060635885821383, 0.30901699437494742410,
                                   -0.10452846326765347140, -0.5, -0.80901699437494742410, -0.97814760073380563793,
                                   -0.97814760073380563793, -0.80901699437494742410, -0.5, -0.10452846326765347140,
                                   0.30901699437494742410, 0.66913060635885821383, 0.91354545764260089550};
  static constexpr double s[15] = {0.0, 0.40673664307580020775, 0.74314482547739423501, 0.95105651629515357212,
                                   0.99452189536827333692, 0.86602540378443864676, 0.58778525229247312917,
                                   0.20791169081775933710, -0.20791169081775933710, -0.58778525229247312917,
                                   -0.86602540378443864676, -0.99452189536827333692, -0.95105651629515357212,
                                   -0.74314482547739423501, -0.40673664307580020775};
};

// odd prime radix P = 7, 11, 13 (forward sign; INV flips it): X_k = a_k - i b_k,
// X_{P-k} = a_k + i b_k with a_k = v0 + sum_j cos(2 pi jk/P) (v_j + v_{P-j}),
// b_k = sum_j sin(2 pi jk/P) (v_j - v_{P-j}), j, k = 1 .. (P-1)/2: (P-1)^2/2 real multiply-adds
// per component instead of P^2
template <int P, bool INV, typename T2>
__device__ __forceinline__ void dft_odd(T2* v) {
  using T = decltype(v[0].x);
  using RT = RootTable<P>;
  constexpr int H = (P - 1) / 2;
  T2 t[H + 1], d[H + 1];
#pragma unroll
  for (int j = 1; j <= H; ++j) {
    t[j] = cadd(v[j], v[P - j]);
    d[j] = csub(v[j], v[P - j]);
  }
  const T2 v0 = v[0];
  T2 s0 = t[H];
#pragma unroll
  for (int j = H - 1; j >= 1; --j) s0 = cadd(t[j], s0);
  v[0] = cadd(v0, s0);
#pragma unroll
  for (int k = 1; k <= H; ++k) {
    T2 a = v0, b{T(0), T(0)};
#pragma unroll
    for (int j = 1; j <= H; ++j) {
      const T c = static_cast<T>(RT::c[(j * k) % P]), sn = static_cast<T>(RT::s[(j * k) % P]);
      a = T2{a.x + c * t[j].x, a.y + c * t[j].y};
      b = T2{b.x + sn * d[j].x, b.y + sn * d[j].y};
    }
    const T2 m = mul_mi<INV>(b);  // -i b (forward)
    v[k] = cadd(a, m);
    v[P - k] = csub(a, m);
  }
}
template <bool INV, typename T2>
__device__ __forceinline__ void dft7(T2* v) {
  dft_odd<7, INV>(v);
}
template <>
struct RootTable<11> {
  static constexpr double c[11] = {1.0, 0.84125353283118120551, 0.41541501300188643508, -0.1423148382732850048,
                                   -0.65486073394528498959, -0.95949297361449736865, -0.95949297361449736865,
                                   -0.65486073394528498959, -0.1423148382732850048, 0.41541501300188643508,
                                   0.84125353283118120551};
  static constexpr double s[11] = {0.0, 0.54064081745559755543, 0.90963199535451833011, 0.98982144188093279524,
                                   0.7557495743542582689, 0.28173255684142967104, -0.28173255684142967104,
                                   -0.7557495743542582689, -0.98982144188093279524, -0.90963199535451833011,
                                   -0.54064081745559755543};
};
template <>
struct RootTable<13> {
  static constexpr double c[13] = {1.0, 0.88545602565320991051, 0.56806474673115592289, 0.12053668025532300601,
                                   -0.35460488704253545489, -0.74851074817110119231, -0.9709418174260520118,
                                   -0.9709418174260520118, -0.74851074817110119231, -0.35460488704253545489,
                                   0.12053668025532300601, 0.56806474673115592289, 0.88545602565320991051};
  static constexpr double s[13] = {0.0, 0.46472317204376850652, 0.82298386589365635224, 0.99270887409805397272,
                                   0.93501624268541483342, 0.66312265824079519305, 0.23931566428755768339,
                                   -0.23931566428755768339, -0.66312265824079519305, -0.93501624268541483342,
                                   -0.99270887409805397272, -0.82298386589365635224, -0.46472317204376850652};
};
template <>
struct RootTable<6> {
  static constexpr double c[6] = {1.0, 0.5, -0.5, -1.0, -0.5, 0.5};
  static constexpr double s[6] = {0.0, 0.86602540378443864676, 0.86602540378443864676, 0.0,
                                  -0.86602540378443864676, -0.86602540378443864676};
};
template <>
struct RootTable<10> {
  static constexpr double c[10] = {1.0, 0.80901699437494742410, 0.30901699437494742410, -0.30901699437494742410,
                                   -0.80901699437494742410, -1.0, -0.80901699437494742410, -0.30901699437494742410,
                                   0.30901699437494742410, 0.80901699437494742410};
  static constexpr double s[10] = {0.0, 0.58778525229247312917, 0.95105651629515357212, 0.95105651629515357212,
                                   0.58778525229247312917, 0.0, -0.58778525229247312917, -0.95105651629515357212,
                                   -0.95105651629515357212, -0.58778525229247312917};
};
template <>
struct RootTable<12> {
  static constexpr double c[12] = {1.0, 0.86602540378443864676, 0.5, 0.0, -0.5, -0.86602540378443864676,
                                   -1.0, -0.86602540378443864676, -0.5, 0.0, 0.5, 0.86602540378443864676};
  static constexpr double s[12] = {0.0, 0.5, 0.86602540378443864676, 1.0, 0.86602540378443864676, 0.5,
                                   0.0, -0.5, -0.86602540378443864676, -1.0, -0.86602540378443864676, -0.5};
};

template <int R, bool INV, typename T2>
__device__ __forceinline__ void dftR(T2* v);

// R = A * B in two levels (the dft8 / dft16 pattern): n = B n1 + n2, k = k1 + A k2; A-point DFTs
// over n1, twiddles W_R^(n2 k1), B-point DFTs over n2
template <int A, int B, bool INV, typename T2>
__device__ __forceinline__ void dft_ab(T2* v) {
  using T = decltype(v[0].x);
  constexpr int R = A * B;
  T2 a[B][A];
#pragma unroll
  for (int n2 = 0; n2 < B; ++n2) {
#pragma unroll
    for (int n1 = 0; n1 < A; ++n1) a[n2][n1] = v[B * n1 + n2];
    dftR<A, INV>(a[n2]);
  }
#pragma unroll
  for (int n2 = 1; n2 < B; ++n2)
#pragma unroll
    for (int k1 = 1; k1 < A; ++k1) {
      const int m = (n2 * k1) % R;
      const T2 w{static_cast<T>(RootTable<R>::c[m]), static_cast<T>((INV ? 1.0 : -1.0) * RootTable<R>::s[m])};
      a[n2][k1] = cmul(a[n2][k1], w);
    }
#pragma unroll
  for (int k1 = 0; k1 < A; ++k1) {
    T2 b[B];
#pragma unroll
    for (int n2 = 0; n2 < B; ++n2) b[n2] = a[n2][k1];
    dftR<B, INV>(b);
#pragma unroll
    for (int k2 = 0; k2 < B; ++k2) v[k1 + A * k2] = b[k2];
  }
}

template <int R, bool INV, typename T2>
__device__ __forceinline__ void dftR(T2* v) {
  if constexpr (R == 2) dft2<INV>(v);
  else if constexpr (R == 3) dft3<INV>(v);
  else if constexpr (R == 4) dft4<INV>(v);
  else if constexpr (R == 5) dft5<INV>(v);
  else if constexpr (R == 6) dft_ab<3, 2, INV>(v);
  else if constexpr (R == 7) dft7<INV>(v);
  else if constexpr (R == 8) dft8<INV>(v);
  else if constexpr (R == 9) dft_ab<3, 3, INV>(v);
  else if constexpr (R == 10) dft_ab<5, 2, INV>(v);
  else if constexpr (R == 11) dft_odd<11, INV>(v);
  else if constexpr (R == 12) dft_ab<4, 3, INV>(v);
  else if constexpr (R == 13) dft_odd<13, INV>(v);
  else if constexpr (R == 15) dft_ab<5, 3, INV>(v);
  else {
    static_assert(R == 16, "unsupported radix");
    dft16<INV>(v);
  }
}

// radix plan: 16 first, then 16 or the rest, the odd factor (3, 5, 7, 9 or 15, possibly inside a
// 6, 10 or 12) in the last pass.  Host and device share this function (twiddle tables, kernels).
struct Radices {
  int r0, r1, r2;
};
__host__ __device__ constexpr bool fft_radix_ok(int r) {
  return r == 1 || r == 2 || r == 3 || r == 4 || r == 5 || r == 6 || r == 7 || r == 8 || r == 9 || r == 10 ||
         r == 11 || r == 12 || r == 13 || r == 15 || r == 16;
}
__host__ __device__ constexpr Radices fft_radices(int n) {
  if (n <= 16) return Radices{n, 1, 1};
  const int rem = n / 16;
  if (n % 16 != 0) return Radices{0, 0, 0};
  if (fft_radix_ok(rem)) return Radices{16, rem, 1};
  if (rem % 16 == 0 && fft_radix_ok(rem / 16)) return Radices{16, 16, rem / 16};
  const int odd = rem % 3 == 0 ? 3 : (rem % 5 == 0 ? 5 : 1);
  if (odd > 1 && fft_radix_ok(rem / odd)) return Radices{16, rem / odd, odd};
  // 7, 9, 11, 13, 15 * 2^k: the whole odd factor in the last pass
  const int odds[5] = {7, 9, 11, 13, 15};
  for (int i = 0; i < 5; ++i)
    if (rem % odds[i] == 0 && fft_radix_ok(rem / odds[i])) return Radices{16, rem / odds[i], odds[i]};
  return Radices{0, 0, 0};
}
__host__ __device__ constexpr bool fft_length_ok(int n) {
  const Radices r = fft_radices(n);
  return n >= 2 && r.r0 > 0 && fft_radix_ok(r.r0) && fft_radix_ok(r.r1) && fft_radix_ok(r.r2) && r.r0 * r.r1 * r.r2 == n;
}

template <int N>
struct FftPlan {
  static constexpr Radices RR = fft_radices(N);
  static constexpr int R0 = RR.r0;
  static constexpr int R1 = RR.r1;
  static constexpr int R2 = RR.r2;
  static_assert(fft_length_ok(N), "unsupported FFT length");
  // per-pass twiddle tables, [r-1][k] (k = butterfly phase, fastest): for a fixed r the lanes of a
  // wave read consecutive entries, which is bank-conflict free (the former single W_N^m table
  // was read at k*r*stride, up to 16-way conflicts for even r)
  static constexpr int T1 = R1 > 1 ? (R1 - 1) * R0 : 0;         // pass 2: NS = R0
  static constexpr int T2 = R2 > 1 ? (R2 - 1) * R0 * R1 : 0;    // pass 3: NS = R0*R1
  static constexpr int TSIZE = T1 + T2 > 0 ? T1 + T2 : 1;
};

// host-side table builder: entry [(r-1)*NS + k] of a pass = W_N^(k*r*N/(R*NS)) = exp(-2 pi i ...)
inline int fft_twiddle_size(int n) {
  const Radices r = fft_radices(n);
  int t = (r.r1 > 1 ? (r.r1 - 1) * r.r0 : 0) + (r.r2 > 1 ? (r.r2 - 1) * r.r0 * r.r1 : 0);
  return t > 0 ? t : 1;
}
template <typename F>
inline void fft_twiddle_fill(int n, F&& put) {  // put(index, m): entry index holds W_n^m
  const Radices rr = fft_radices(n);
  int off = 0;
  auto pass = [&](int R, int NS) {
    const int stride = n / (R * NS);
    for (int r = 1; r < R; ++r)
      for (int k = 0; k < NS; ++k) put(off + (r - 1) * NS + k, k * r * stride);
    off += (R - 1) * NS;
  };
  if (rr.r1 > 1) pass(rr.r1, rr.r0);
  if (rr.r2 > 1) pass(rr.r2, rr.r0 * rr.r1);
}

// ---- real-signal forward transform of the z stage (N = 1024, 2048) -------------------------
// A real row x of length N is packed as z_m = x_2m + i x_2m+1 and transformed at length H = N/2;
// X_k = E_k + W_N^k O_k with E_k = (Z_k + conj Z_{H-k})/2, O_k = (Z_k - conj Z_{H-k})/(2i).
// Radices of the half transform: 512 = 8x8x8 and 1024 = 16x16x4, so every pass gives each of the
// 64 lanes exactly one butterfly (a 16x16x2 plan of 512 would idle half the wave in two passes).
// Its tables are appended to the N-point table: [post W_N^k, k < N/2][pass 2][pass 3].
template <int N>
struct HalfPlan {
  static constexpr bool ok = N == 1024 || N == 2048;
  static constexpr int H = N / 2;
  static constexpr int R0 = H == 512 ? 8 : 16, R1 = R0, R2 = H / (R0 * R1);
  static constexpr int POST = H;                    // post-processing twiddles W_N^k
  static constexpr int P2 = POST;                   // offset of pass 2 (R1, NS = R0)
  static constexpr int P3 = P2 + (R1 - 1) * R0;     // offset of pass 3 (R2, NS = R0*R1)
  static constexpr int SIZE = ok ? P3 + (R2 - 1) * R0 * R1 : 0;
};
inline int fft_half_twiddle_size(int n) {
  if (n != 1024 && n != 2048) return 0;
  const int h = n / 2, r0 = h == 512 ? 8 : 16, r2 = h / (r0 * r0);
  return h + (r0 - 1) * r0 + (r2 - 1) * r0 * r0;
}
template <typename F>
inline void fft_half_twiddle_fill(int n, F&& put) {  // put(index, m): entry holds W_n^m
  if (fft_half_twiddle_size(n) == 0) return;
  const int h = n / 2, r0 = h == 512 ? 8 : 16, r2 = h / (r0 * r0);
  for (int k = 0; k < h; ++k) put(k, k);
  int off = h;
  auto pass = [&](int R, int NS) {  // W_h^(k r h/(R NS)) = W_n^(2 k r h/(R NS))
    const int stride = h / (R * NS);
    for (int r = 1; r < R; ++r)
      for (int k = 0; k < NS; ++k) put(off + (r - 1) * NS + k, 2 * k * r * stride);
    off += (R - 1) * NS;
  };
  pass(r0, r0);
  pass(r2, r0 * r0);
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() also waits for vmcnt(0), i.e. for
// every outstanding global load AND store of the wave (CDNA counts both on vmcnt), which
// serialises a staging pipeline: each field's stores would have to be acknowledged by HBM before
// the next field could be staged, and prefetched loads would be drained early.  Here only this
// wave's LDS operations are waited for (lgkmcnt(0)) before s_barrier; the "memory" clobber keeps
// the compiler from moving memory accesses across it.  Valid wherever the barrier only orders
// LDS writes/reads between waves (global data exchanged between waves needs __syncthreads()).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Ordering of a row's LDS accesses between its threads: one wave (TPR = 64) only needs the
// compiler to keep program order; a row shared by several waves needs the block barrier (every
// thread of the block must then reach it).
template <int TPR>
__device__ __forceinline__ void row_sync() {
  if constexpr (TPR == 64) __builtin_amdgcn_wave_barrier();
  else lds_barrier();
}

// ---- wave-owned variant -------------------------------------------------------------------
// One wavefront transforms RW rows it owns.  A wave's LDS instructions are processed in order,
// so the pass structure (all reads of a pass, then all writes) needs no s_barrier: the only
// requirement is that the compiler keeps the program order of the (possibly aliasing) LDS
// accesses, which wave_barrier() pins.  Blocks then need barriers only around cooperative
// global<->LDS staging, not per pass.
// TPR threads (64: one wave; 128: two waves of one block) share the rows; lane = thread index
// within them
// Zero band of a 2/3-dealiased spectral row of length N (kx = N/3 + 1 .. N - N/3 - 1 are zero):
// for the first pass (NS = 1) of an inverse x transform, input block r (elements Q r .. Q r + Q - 1)
// is entirely in the band when zero_block() holds; those inputs are never read (compile-time zeros,
// so the DFT drops their terms) and never need to be written
template <int N, int Q>
__host__ __device__ constexpr bool zero_block(int r) {
  return Q * r >= N / 3 + 1 && Q * r + Q - 1 <= N - N / 3 - 1;
}

template <int N, int R, int NS, int RW, int PITCH, bool INV, int TPR = 64, bool ZB = false, bool TR = false,
          int SH = 4, typename T2>
__device__ __forceinline__ void wave_pass(T2* __restrict__ buf, const T2* __restrict__ tw, int lane) {
  // tw: this pass's [R-1][NS] twiddle table; ZB: first pass of a zero-band input (zero_block);
  // TR: last pass of a forward x transform whose outputs in the 2/3-rule band are discarded (not
  // written back)
  constexpr int Q = N / R;
  constexpr int NB = RW * Q;
  constexpr int B = (NB + TPR - 1) / TPR;
  static_assert(!ZB || NS == 1, "zero-band pruning applies to the first pass");
  // Power-of-two lengths: every index split of a pass satisfies fft_pidx(a + b) = fft_pidx(a) +
  // fft_pidx(b) (reads: a = j < Q, b = r Q; writes: a = base, b = r NS, with (a % 16) + (b % 16) <
  // 16 for radix-16-first plans), so each butterfly column is ONE address register plus
  // compile-time LDS offsets (the per-element p + (p >> 4) cost ~150 VALU per 1024-point z row)
  // (SH = 5: the same holds with (a % 32) + (b % 32) < 32 for the z stage's plans, 16x16x4 and the
  // half-length 8x8x8, checked case by case; other plans keep SH = 4)
  static_assert(SH == 4 || N == 1024 || N == 512, "pad shift 5: the z stage's plans only");
  constexpr bool LIN = (N & (N - 1)) == 0;
  T2 v[B][R];
#pragma unroll
  for (int b = 0; b < B; ++b) {
    const int idx = lane + b * TPR;
    if (NB % TPR == 0 || idx < NB) {
      const int row = idx / Q, j = idx - row * Q;
      const T2* p = buf + row * PITCH + (LIN ? fft_pidx_s<SH>(j) : 0);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (ZB && zero_block<N, Q>(r)) v[b][r] = T2{0, 0};
        else v[b][r] = LIN ? p[fft_pidx_s<SH>(r * Q)] : p[fft_pidx_s<SH>(j + r * Q)];
      }
    }
  }
  row_sync<TPR>();
#pragma unroll
  for (int b = 0; b < B; ++b) {
    const int idx = lane + b * TPR;
    if (NB % TPR == 0 || idx < NB) {
      const int row = idx / Q, j = idx - row * Q;
      const int k = j % NS;
      if constexpr (NS > 1) {
#pragma unroll
        for (int r = 1; r < R; ++r) {
          v[b][r] = cmul_tw<INV>(v[b][r], tw[(r - 1) * NS + k]);
        }
      }
      dftR<R, INV>(v[b]);
      const int base = (j - k) * R + k;
      T2* p = buf + row * PITCH + (LIN ? fft_pidx_s<SH>(base) : 0);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int pos = base + r * NS;
        if (!TR || pos <= N / 3 || pos >= N - N / 3) {
          if constexpr (LIN) p[fft_pidx_s<SH>(r * NS)] = v[b][r];
          else p[fft_pidx_s<SH>(pos)] = v[b][r];
        }
      }
    }
  }
  row_sync<TPR>();
}

template <int N, int RW, int PITCH, bool INV, int TPR = 64, bool ZB = false, bool TR = false, typename T2>
__device__ __forceinline__ void wave_fft(T2* __restrict__ buf, const T2* __restrict__ tw, int lane) {
  using Pl = FftPlan<N>;
  constexpr bool L0 = Pl::R1 == 1, L1 = Pl::R1 > 1 && Pl::R2 == 1;  // which pass is the last
  wave_pass<N, Pl::R0, 1, RW, PITCH, INV, TPR, ZB, TR && L0>(buf, tw, lane);
  if constexpr (Pl::R1 > 1) wave_pass<N, Pl::R1, Pl::R0, RW, PITCH, INV, TPR, false, TR && L1>(buf, tw, lane);
  if constexpr (Pl::R2 > 1) wave_pass<N, Pl::R2, Pl::R0 * Pl::R1, RW, PITCH, INV, TPR, false, TR>(buf, tw + Pl::T1, lane);
}

// ---- register-edge passes (one butterfly column per lane: N / R0 == TPR) ------------------------
// When the first pass has exactly one butterfly per lane (Q = N/R0 = TPR), lane j's inputs are the
// elements j + r Q, which is the "point n = lane + TPR i" register layout the z stage keeps its
// physical rows in; and when the last pass has NS = N/R a multiple of TPR, its outputs j + r NS
// (j = lane + TPR b) are that layout again.  So a transform can start from and end in registers,
// saving the gather-to-LDS and the read-back round trips of the LDS-only version.
template <int N>
struct FftLast {  // radix and stride of the last pass
  static constexpr int R = FftPlan<N>::R2 > 1 ? FftPlan<N>::R2 : FftPlan<N>::R1;
  static constexpr int NS = N / R;
  static constexpr int TOFF = FftPlan<N>::R2 > 1 ? FftPlan<N>::T1 : 0;  // its twiddle table
};
template <int N, int TPR>
constexpr bool fft_reg_edges_ok() {
  return FftPlan<N>::R0 * TPR == N && FftPlan<N>::R1 > 1 && FftLast<N>::NS % TPR == 0;
}
// first pass (NS = 1) from registers: x[r] = element j + r N/R0 (j = lane); writes its output
template <int N, bool INV, int SH = 4, typename T2>
__device__ __forceinline__ void wave_pass_first_reg(T2* __restrict__ buf, T2 (&x)[FftPlan<N>::R0], int j) {
  constexpr int R = FftPlan<N>::R0;
  dftR<R, INV>(x);
  T2* p = buf + fft_pidx_s<SH>(j * R);  // (j R + r, r < R = 16: one address register, immediate offsets)
#pragma unroll
  for (int r = 0; r < R; ++r) p[r] = x[r];
}
// middle pass (the second of a three-pass plan) through LDS
template <int N, int PITCH, bool INV, int TPR, int SH = 4, typename T2>
__device__ __forceinline__ void wave_pass_middle(T2* __restrict__ buf, const T2* __restrict__ tw, int lane) {
  using Pl = FftPlan<N>;
  static_assert(Pl::R2 > 1, "middle pass of a three-pass plan");
  wave_pass<N, Pl::R1, Pl::R0, 1, PITCH, INV, TPR, false, false, SH>(buf, tw, lane);
}
// The same pass (one butterfly per lane: N / R1 == 64) with its twiddles held in registers: butterfly
// j = lane uses W^(k r), k = lane % R0, for every row and both directions (twr, loaded once per
// kernel by middle_twiddles), instead of R1 - 1 LDS reads per transform
template <int N>
struct MidTw {
  static constexpr int R = FftPlan<N>::R1, NS = FftPlan<N>::R0;
  static constexpr bool ok = N / R == 64 && FftPlan<N>::R2 > 1;
};
template <int N, typename T2>
__device__ __forceinline__ void middle_twiddles(const T2* __restrict__ tw, T2 (&twr)[MidTw<N>::R - 1], int lane) {
  constexpr int NS = MidTw<N>::NS;
#pragma unroll
  for (int r = 1; r < MidTw<N>::R; ++r) twr[r - 1] = tw[(r - 1) * NS + lane % NS];
}
template <int N, int PITCH, bool INV, int SH = 4, typename T2>
__device__ __forceinline__ void wave_pass_middle_rt(T2* __restrict__ buf, const T2 (&twr)[MidTw<N>::R - 1], int lane) {
  constexpr int R = MidTw<N>::R, NS = MidTw<N>::NS, Q = N / R;
  static_assert(MidTw<N>::ok && (N & (N - 1)) == 0, "register-twiddle middle pass: one butterfly per lane");
  T2 v[R];
  const T2* p = buf + fft_pidx_s<SH>(lane);
#pragma unroll
  for (int r = 0; r < R; ++r) v[r] = p[fft_pidx_s<SH>(r * Q)];
  row_sync<64>();
#pragma unroll
  for (int r = 1; r < R; ++r) v[r] = cmul_tw<INV>(v[r], twr[r - 1]);
  dftR<R, INV>(v);
  const int k = lane % NS, base = (lane - k) * R + k;
  T2* q = buf + fft_pidx_s<SH>(base);
#pragma unroll
  for (int r = 0; r < R; ++r) q[fft_pidx_s<SH>(r * NS)] = v[r];
  row_sync<64>();
}
// last pass into registers: out[b + r B] = element j + r NS, j = lane + TPR b, B = NS / TPR
template <int N, bool INV, int TPR, int SH = 4, typename T2>
__device__ __forceinline__ void wave_pass_last_reg(const T2* __restrict__ buf, const T2* __restrict__ tw,
                                                   T2 (&out)[N / TPR], int lane) {
  constexpr int R = FftLast<N>::R, NS = FftLast<N>::NS, B = NS / TPR;
  const T2* t = tw + FftLast<N>::TOFF;
  T2 v[B][R];
  const T2* p = buf + fft_pidx_s<SH>(lane);  // (TPR b + r NS: multiples of 64 added to lane < 64)
#pragma unroll
  for (int b = 0; b < B; ++b)
#pragma unroll
    for (int r = 0; r < R; ++r) v[b][r] = p[fft_pidx_s<SH>(TPR * b + r * NS)];
#pragma unroll
  for (int b = 0; b < B; ++b) {
    const int j = lane + TPR * b;
#pragma unroll
    for (int r = 1; r < R; ++r) v[b][r] = cmul_tw<INV>(v[b][r], t[(r - 1) * NS + j]);
    dftR<R, INV>(v[b]);
#pragma unroll
    for (int r = 0; r < R; ++r) out[b + r * B] = v[b][r];
  }
}

// length-N/2 transform of HalfPlan<N>; htw points at the appended tables (post twiddles first)
template <int N, int PITCH, bool INV, int TPR = 64, int SH = 4, typename T2>
__device__ __forceinline__ void wave_fft_half(T2* __restrict__ buf, const T2* __restrict__ htw, int lane) {
  using Hp = HalfPlan<N>;
  static_assert(Hp::ok, "no half plan for this length");
  wave_pass<Hp::H, Hp::R0, 1, 1, PITCH, INV, TPR, false, false, SH>(buf, htw, lane);
  wave_pass<Hp::H, Hp::R1, Hp::R0, 1, PITCH, INV, TPR, false, false, SH>(buf, htw + Hp::P2, lane);
  wave_pass<Hp::H, Hp::R2, Hp::R0 * Hp::R1, 1, PITCH, INV, TPR, false, false, SH>(buf, htw + Hp::P3, lane);
}


// LDS poison fill (debug): every 32-bit word of [p, p + bytes) becomes 0xFFFFFFFF, a
// NaN as float and as double, so data read from a slot the kernel never wrote propagates as NaN.
// Block-cooperative; the caller synchronises before the first real use.
__device__ __forceinline__ void lds_poison_fill(void* p, int bytes) {
  unsigned* w = static_cast<unsigned*>(p);
  for (int i = threadIdx.x; i < bytes / 4; i += blockDim.x) w[i] = 0xFFFFFFFFu;
}

// XCD-aware block remap (cdna_hip_programming.md T1): blocks b and b+8 share an XCD under the
// observed round-robin dispatch, so logical tiles that are adjacent in memory are given to blocks
// on the same XCD (their partial cache lines then merge in one L2).  Bijective for any n.
__device__ __forceinline__ unsigned xcd_remap(unsigned b, unsigned n) {
  const unsigned q = n / 8, r = n % 8, x = b % 8, i = b / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

}  // namespace dev
}  // namespace channel
