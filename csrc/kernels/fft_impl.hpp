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
// Kernel templates of the transform stages; fft.hip holds the host API and the length dispatch,
// fft_pow2.hip / fft_r3.hip / fft_r5.hip instantiate the kernels per length family (parallel
// compilation).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

#include "channel/common.hpp"
#include "channel/fft_device.hpp"
#include "channel/kernels.hpp"

namespace channel {

using namespace dev;

constexpr int pow2_floor(int n) { return n < 2 ? 1 : 2 * pow2_floor(n / 2); }
constexpr int pow2_ceil(int n) { return pow2_floor(n) < n ? 2 * pow2_floor(n) : pow2_floor(n); }

// ---- x-direction -------------------------------------------------------------------------
// fp64 at NX = 2048: 2 columns per tile (the 4-column tile plus the twiddles would exceed the
// 160 KB of LDS), one wave per column
constexpr int xcfg_c(int nx, int tsz) {
  return tsz == 4 ? (nx > 512 ? 8 : 16) : (nx > 1024 ? 2 : (nx > 512 ? 4 : (nx >= 512 ? 8 : 16)));
}
// WIDE = 1: twice the kz columns per tile (128-B row segments) with 512 threads and one block per
// CU (the same 8 waves per CU); WIDE = 0: 64-B segments, 256 threads, two blocks per CU.
constexpr int xcfg_nt(int wide, int c = 4) { return wide ? 512 : (c >= 4 ? 256 : 64 * c); }
constexpr int xcfg_minb(int wide) { return wide ? 1 : 2; }
template <int NX, typename T, int WIDE = 0>
struct XCfg {
  // kz columns per tile
  static constexpr int C = xcfg_c(NX, sizeof(T)) * (WIDE ? 2 : 1);
  // fp32 at 2048 points: the LDS holds one 8-column tile per CU, so that tile gets 8 waves, two per
  // row (TPR = 128, block barriers between the passes; 2 waves per SIMD without spills) instead of
  // 4 waves of 2 rows at one wave per SIMD
  // (fp64 from 1024 points likewise: 4 columns x 2 waves at 1024, 2 x 2 at 2048)
  static constexpr bool BIG = NX >= (sizeof(T) == 4 ? 2048 : 1024) && !WIDE;
  static constexpr int NT = BIG ? 128 * (C < 4 ? C : 4) : xcfg_nt(WIDE, C);
  static constexpr int MINB = BIG ? 1 : xcfg_minb(WIDE);
  static constexpr int TPR = BIG ? 128 : 64;  // threads per transformed row
  // row pitch: padded FFT row + 1 or 2 slots so that the transposing global->LDS stores (lanes =
  // C consecutive kz columns x consecutive x) hit distinct banks (pitch*c spreads over 16 slots)
  static constexpr int PITCH = FftPitch<NX>::value + (sizeof(T) == 4 ? (C >= 16 ? 1 : 2) : (C >= 8 ? 1 : 2));
};

// CHANNEL_FFT_DIAG=1 skips the in-LDS transforms (timing diagnosis only: results are wrong)
static int fft_diag() {
  static const int d = [] {
    const char* e = std::getenv("CHANNEL_FFT_DIAG");
    return e ? std::atoi(e) : 0;
  }();
  return d;
}

// blocked spectral layout: the wide x tiles as plane tiles (SL = 2); CHANNEL_XPLANES=0 keeps the
// 8-column one-plane tiles (A/B)
static bool xplanes_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("CHANNEL_XPLANES");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}

// CHANNEL_XSEGROWS=0: the per-element segment lookups of the exchange-segment x kernels (A/B of
// the per-thread row table, kSegRows)
static bool xsegrows_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("CHANNEL_XSEGROWS");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}

static bool xwide_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("CHANNEL_XWIDE");
    return e && std::atoi(e) == 1;
  }();
  return on;
}

// Segment lookup in a small split table (at most MAXS segments) without dynamic indexing.
// Indexing a by-value kernel-argument array with a per-lane index makes hipcc gather the entries
// from the kernarg segment with per-lane global loads, each followed by s_waitcnt vmcnt(0): that
// drained every in-flight prefetch load and store of the wave at every element and serialised
// the x transforms.  Unrolled over the compile-time capacity the entries are wave-uniform
// (SGPR) values and the lookup is a chain of compares and selects.
struct SegPos {
  int start;      // first index of the segment
  int count;      // its length
  long long off;  // element offset of its block
  int idx;        // segment index
};
template <int MAXS = 8>
__device__ __forceinline__ SegPos seg_find(const int* start, const long long* off, int n, int i) {
  SegPos p{start[0], start[1] - start[0], off[0], 0};
#pragma unroll
  for (int q = 1; q < MAXS; ++q)
    if (q < n && i >= start[q]) p = SegPos{start[q], start[q + 1] - start[q], off[q], q};
  return p;
}

// Segment of i for i in the wave-uniform window [lo, lo + span) when every segment is at least
// span long (checked on the host): the window meets at most two segments, found with scalar
// lookups of its two ends, and each lane picks one with a single compare.
template <int MAXS = 8>
__device__ __forceinline__ SegPos seg_find_win(const int* start, const long long* off, int n, int lo, int span, int i) {
  const SegPos a = seg_find<MAXS>(start, off, n, lo);
  const SegPos b = seg_find<MAXS>(start, off, n, lo + span - 1);
  return i >= b.start ? b : a;
}
// kx segment addressing of the x kernels: kSegOne = one block, no self block (one rank);
// kSegWin = window lookup (seg_find_win); kSegFull = per-element lookup; kSegRows = per-thread row
// table: a thread's kx rows are the same in every tile, so their segments are looked up once per
// launch (SegRows) and a tile's access is one 32-bit multiply-add per element (the per-element
// lookups of the other modes spilled 375-402 SGPRs into VGPR lanes at 1024 points)
constexpr int kSegOne = 0, kSegWin = 1, kSegFull = 2, kSegRows = 3;
constexpr int kSegRowsMax = 24;  // rows per thread with a table (longer rows keep the lookups)
// kSegRows: element offset of row i at y = 0 (off + (i - start) S), the y stride of its segment
// (count S), and whether the segment is a self block, for the K rows i = (tid + k NT) / CW of a
// thread (clamped to the last row like the accesses).  S = nkz for [y][kx][kz] segments; blocked
// segments (XArgs::segblk: [y/8][line/8][y%8][line%8], line = kx * nkzs + kz) take S = 8 nkzs and
// the access coordinates (Y, KZ) of seg_yk.
// x-expanded segments (the pencil's x rows) keep S = nkz.
template <int K>
struct SegRows {
  unsigned a[K], b[K];
  unsigned self = 0;
  template <int NT, int CW, int NROW, int MAXS = kMaxSeg>
  __device__ __forceinline__ void build(const int* start, const long long* off, int n, int self_seg, int nself, int nkz,
                                        int tid) {
    static_assert(NT % CW == 0, "rows tid / CW + k NT / CW");
    build_at<NROW, MAXS>(start, off, n, self_seg, nself, nkz, tid / CW, NT / CW);
  }
  // rows i = r0 + k di (the plane tiles' quad lane map: r0 = quad_row(tid))
  template <int NROW, int MAXS = kMaxSeg>
  __device__ __forceinline__ void build_at(const int* start, const long long* off, int n, int self_seg, int nself,
                                           int nkz, int r0, int di) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = min(r0 + k * di, NROW - 1);
      const SegPos sp = seg_find<MAXS>(start, off, n, i);
      a[k] = static_cast<unsigned>(sp.off) + static_cast<unsigned>(i - sp.start) * static_cast<unsigned>(nkz);
      b[k] = static_cast<unsigned>(sp.count) * static_cast<unsigned>(nkz);
      if (static_cast<unsigned>(sp.idx - self_seg) < static_cast<unsigned>(nself)) self |= 1u << k;
    }
  }
  // rows i = r0 + k di from a host-built row table (XSrc::rowtab): two loads per row instead of
  // a segment lookup per row (whose unrolled compare / select chains over kMaxSeg segments cost
  // ~500 VALU instructions per wave and launch, against ~4 tiles per wave per launch)
  template <int NROW>
  __device__ __forceinline__ void load_at(const unsigned* tab, int y0, int r0, int di) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = min(r0 + k * di, NROW - 1);
      const uint2 e = *reinterpret_cast<const uint2*>(tab + 2 * i);
      b[k] = e.y & 0x7fffffffu;
      a[k] = e.x + static_cast<unsigned>(y0) * b[k];
      if (e.y >> 31) self |= 1u << k;
    }
  }
  __device__ __forceinline__ unsigned at(int k, unsigned Y, unsigned KZ) const { return a[k] + Y * b[k] + KZ; }
  __device__ __forceinline__ bool is_self(int k) const { return (self >> k) & 1u; }
};
// (Y, KZ) of element (y, kz) of an exchange segment or self block (y: the chunk's row plus
// XArgs::seg_yoff, the first row of a part of an exchange chunk) (offset = segment row base +
// Y * (rows stride) + KZ): plain [y][kx][kz] Y = y, KZ = kz; blocked (XArgs::segblk) Y = y / 8,
// KZ = (y % 8) 8 + (kz / 8) 64 + kz % 8.  seg_stride: S of SegRows / the per-element lookups.
__device__ __forceinline__ void seg_yk(int segblk, int y, int kz, unsigned& Y, unsigned& KZ) {
  if (segblk) {
    Y = static_cast<unsigned>(y) >> 3;
    KZ = ((static_cast<unsigned>(y) & 7u) << 3) + ((static_cast<unsigned>(kz) >> 3) << 6) + (static_cast<unsigned>(kz) & 7u);
  } else {
    Y = static_cast<unsigned>(y);
    KZ = static_cast<unsigned>(kz);
  }
}
__host__ __device__ inline int seg_stride(const XArgs& a) { return a.segblk ? kSpecKzBlock * a.nkzs : a.nkz; }

template <int NT, int C>
inline int seg_mode(int n, const int* start, int self_seg, long long off0) {
  if (n == 1 && self_seg < 0 && off0 == 0) return kSegOne;
  int m = 1 << 30;
  for (int q = 0; q < n; ++q) m = std::min(m, start[q + 1] - start[q]);
  return m >= NT / C ? kSegWin : kSegFull;
}

// element offset of (row y of the chunk, retained kx i, kz) in a blocked spectral field (spec_index
// with kzb = 8; XArgs::spec_y0 / nkzs); consecutive kx rows are nkzs * 8 elements apart
__device__ __forceinline__ unsigned spec_blk_off(const XArgs& a, int y, int i, int kz) {
  return static_cast<unsigned>(spec_row_off(kSpecKzBlock, a.nkx * a.nkzs, a.spec_y0 + y) +
                               spec_line_off(kSpecKzBlock, i * a.nkzs + kz));
}

// V consecutive complex values moved by one global access (V = 2 for fp32: 16-byte loads and
// stores, half the instructions of 8-byte ones; the stores of the x kernels were issue-bound)
template <typename T2, int V>
struct alignas(sizeof(T2) * V) CVec {
  T2 c[V];
};
// Lane map of the global<->LDS transposes of the 16-column plane tiles (SL = 2, two planes x one
// 8-wide kz block, V = 2): a ds_write_b64 is banked per 16 contiguous lanes modulo 32 dwords and a
// ds_read_b64 per 32 lanes modulo 64, so no row pitch serves both with the same lane map (pitch
// = 1 mod 16: writes conflict-free, reads 2-way; = 2 mod 16: the reverse).  With the pitch at
// 2 mod 16 the global->LDS side takes quads of 4 lanes = one plane's 64-B kz piece, 8 rows per
// half-wave, plane 0 in lanes 0-31 and plane 1 in 32-63 (16 lanes = 4 rows x 4 kz pairs of one
// plane: conflict-free), and the LDS->global side keeps 8 lanes per row (2 planes x 4 kz pairs,
// 4 rows per half-wave: conflict-free).  quad_col / quad_row: the column pair and the row of
// thread tid within each group of NT / 8 rows.
template <int NX, typename T, int WIDE, int SL, int V>
struct XQuad {
  static constexpr bool on = SL == 2 && V == 2 && XCfg<NX, T, WIDE>::C == 16 && FftPitch<NX>::value % 16 == 0;
  static constexpr int PITCH = on ? FftPitch<NX>::value + 2 : XCfg<NX, T, WIDE>::PITCH;
};
__device__ __forceinline__ int quad_col(int tid) { return (tid & 3) | ((tid >> 3) & 4); }
__device__ __forceinline__ int quad_row(int tid) { return ((tid >> 2) & 7) | ((tid >> 6) << 3); }

// element at a 32-bit BYTE offset from a wave-uniform base: the global access then takes the base
// in SGPRs and the offset in one VGPR (saddr form) instead of 64-bit address arithmetic per
// element; every caller's span is checked below 4 GiB on the host
template <typename P>
__device__ __forceinline__ P& at_byte(P* base, unsigned off) {
  return *reinterpret_cast<P*>(reinterpret_cast<char*>(base) + off);
}
template <typename P>
__device__ __forceinline__ const P& at_byte(const P* base, unsigned off) {
  return *reinterpret_cast<const P*>(reinterpret_cast<const char*>(base) + off);
}
// streaming (non-temporal) access of the spectral fields, which the x kernels read or write once
// per substep (XArgs::nt): they then do not displace the x-expanded intermediates of the chunks in
// flight from the Infinity Cache
template <typename P>
__device__ __forceinline__ P ld_nt(const P& r) {
  static_assert(sizeof(P) == 8 || sizeof(P) == 16, "8- or 16-byte accesses");
  typedef unsigned int v2u __attribute__((ext_vector_type(2)));
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  P out;
  if constexpr (sizeof(P) == 16) {
    const v4u x = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(&r));
    __builtin_memcpy(&out, &x, 16);
  } else {
    const v2u x = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(&r));
    __builtin_memcpy(&out, &x, 8);
  }
  return out;
}
template <typename P>
__device__ __forceinline__ void st_nt(P& r, const P& v) {
  static_assert(sizeof(P) == 8 || sizeof(P) == 16, "8- or 16-byte accesses");
  typedef unsigned int v2u __attribute__((ext_vector_type(2)));
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  if constexpr (sizeof(P) == 16) {
    v4u x;
    __builtin_memcpy(&x, &v, 16);
    __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(&r));
  } else {
    v2u x;
    __builtin_memcpy(&x, &v, 8);
    __builtin_nontemporal_store(x, reinterpret_cast<v2u*>(&r));
  }
}

// Combine mode of the x-backward (XArgs::combine): K-SPEC writes v, D1 v, D1 omega next to the
// states omega and phi, and the gather forms the six fields of the physical-space stage in
// registers, per element (kspec_kernel; nonLinear_kernels.cu:55-72, convolution_kernels.cu:46-53):
//   u  = i (al D1v - be om)/k2        w  = i (be D1v + al om)/k2
//   wx = i (be phi + al D1om)/k2      wz = i (be D1om - al phi)/k2   (D2 v = phi + k2 v)
//   v = v, wy = om; on the mean line (kx = kz = 0) u = U = Re om, wz = -dU/dy, wy = 0.
// A tile of group g holds two output fields (kCmbOutA/B[g], CL columns each) formed from two input
// fields (kCmbInP/Q[g]) loaded at the same elements.  Input fields: 0 D1 v, 1 v, 2 D1 omega,
// 3 omega, 4 phi (XSrc::fld).
// Groups 0 (u, w from D1 v, omega) and 1 (v, omega_y from v, omega) are adjacent in the tile order,
// so the second read of omega's chunk follows the first (from the Infinity Cache).
constexpr int kCmbGroups = 3, kCmbInputs = 5;
__host__ __device__ constexpr int cmb_in_p(int g) { return g == 0 ? 0 : (g == 1 ? 1 : 4); }
__host__ __device__ constexpr int cmb_in_q(int g) { return g == 2 ? 2 : 3; }
__host__ __device__ constexpr int cmb_out_a(int g) { return g == 0 ? 0 : (g == 1 ? 1 : 3); }
__host__ __device__ constexpr int cmb_out_b(int g) { return g == 0 ? 2 : (g == 1 ? 4 : 5); }
template <typename T>
__device__ __forceinline__ T cmb_rcp(T k2) {
  if constexpr (sizeof(T) == 4) return k2 > 0.f ? __builtin_amdgcn_rcpf(k2) : 0.f;
  else return k2 > 0.0 ? 1.0 / k2 : 0.0;
}
template <typename T2, typename T>
__device__ __forceinline__ void cmb_pair(int g, T2 P, T2 Q, T al, T be, T r, bool mean, T2& A, T2& B) {
  if (g == 0) {  // u, w from (D1 v, omega)
    A = T2{-(al * P.y - be * Q.y) * r + (mean ? Q.x : T(0)), (al * P.x - be * Q.x) * r};
    B = T2{-(be * P.y + al * Q.y) * r, (be * P.x + al * Q.x) * r};
  } else if (g == 2) {  // omega_x, omega_z from (phi, D1 omega)
    A = T2{-(be * P.y + al * Q.y) * r, (be * P.x + al * Q.x) * r};
    B = T2{-(be * Q.y - al * P.y) * r - (mean ? Q.x : T(0)), (be * Q.x - al * P.x) * r};
  } else {  // v, omega_y from (v, omega)
    A = P;
    B = mean ? T2{0, 0} : Q;
  }
}

// Both x kernels are persistent: the grid is the resident capacity (2 blocks per CU, bounded by
// LDS) and each block walks (field, y, kz-chunk) tiles.  The next tile's global loads are issued
// into registers right after the current tile is staged into LDS, so they are in flight during
// the FFT and the stores; one block per tile (the previous design) left HBM idle for most of each
// block's lifetime (SQ_WAIT_ANY ~73 % of wave cycles at ~2 TB/s).  Twiddles are staged once.
// SM (kSegOne / kSegWin / kSegFull): how the kx source blocks are addressed; a per-element 8-way
// compare/select lookup costs 22 chains per tile and spilled ~330 SGPRs
// SL = 1: blocked spectral layout (XArgs::kzb, one rank: SM = kSegOne); tiles then walk y fastest,
// so the tiles of one XCD share the 128-byte lines two planes of a kz block fill.  SL = 2: the
// same layout with the C columns of a tile taken as C / 8 planes x one 8-wide kz block: each
// retained kx then contributes one contiguous piece of C / 8 rows of the block (128 bytes, a whole
// line, for the 16-column tiles) instead of 64-byte halves read by two tiles.
// CMB: combine mode (above): a tile is one group, CL = C / 2 columns of each of its two outputs,
// each thread loading its elements of both inputs (SL = 2: one plane x one 8-wide kz block; the
// neighbouring plane's tile, the next one in the XCD's order, reads the other half of the lines).
template <int NX, typename T, bool SEG, int WIDE, int SM = kSegFull, int V = 1, int SL = 0, bool CMB = false>
__global__ void __launch_bounds__((XCfg<NX, T, WIDE>::NT), (XCfg<NX, T, WIDE>::MINB))
    xfft_backward_kernel(XArgs a, XSrc src, typename C2<T>::type* phys, const typename C2<T>::type* tw) {
  using T2 = typename C2<T>::type;
  using Cfg = XCfg<NX, T, WIDE>;
  using CV = CVec<T2, V>;
  using QM = XQuad<NX, T, WIDE, CMB ? 0 : SL, V>;
  constexpr int C = Cfg::C, NT = Cfg::NT, PITCH = QM::PITCH;
  constexpr int CL = CMB ? C / 2 : C;  // loaded columns per input field
  static_assert(!CMB || (C % (2 * V) == 0), "combine mode: two halves of whole accesses");
  constexpr int CW = CL / V;  // accesses per tile row and input (V kz columns each; the host checks nkz % V == 0)
  // only the retained kx are loaded (nkx*CL elements per input); the zero padding is re-written in LDS
  constexpr int NKMAX = 2 * (NX / 3) + 1;
  constexpr int NKX = NKMAX, KXH = NX / 3;  // retained kx: the 2/3 rule's (checked on the host)
  constexpr int EPT = (NKMAX * CW + NT - 1) / NT;
  constexpr int NIN = CMB ? 2 : 1;  // input fields per tile
  __shared__ T2 s[C * PITCH];
  constexpr int TS = FftPlan<NX>::TSIZE;
  __shared__ T2 tws[TS];
  if (a.lds_poison) {
    lds_poison_fill(s, sizeof(s));
    lds_poison_fill(tws, sizeof(tws));
    __syncthreads();
  }
  for (int i = threadIdx.x; i < TS; i += NT) tws[i] = tw[i];
  // tile = YP planes x KC kz columns (column c: plane y0 + c / KC, kz kz0 + c % KC; CMB: c % CL)
  constexpr int KC = SL == 2 ? kSpecKzBlock : CL, YP = CL / KC;
  static_assert(SL != 2 || CL % kSpecKzBlock == 0, "plane tiles need whole kz blocks");
  const int nkzc = (a.nkz + KC - 1) / KC, nyt = (a.ny + YP - 1) / YP;
  const int nf = CMB ? kCmbGroups : a.nfields;
  const int ntiles = nyt * nkzc * nf;
  const int G = static_cast<int>(gridDim.x);
  const int tid = threadIdx.x;
  const int nload = NKX * CW;
  CV v[NIN][EPT];
  // SL with SM = kSegRows: the P > 1 exchange segments and self blocks in the blocked layout
  // (XArgs::segblk), read as plane tiles like the one-rank field
  static_assert(SL == 0 || SM == kSegOne || SM == kSegRows, "blocked spectral layout: one source block or row tables");
  static_assert(SM != kSegRows || (NT % CW == 0 && EPT <= kSegRowsMax), "row table: a thread's rows repeat per access");
  SegRows<SM == kSegRows ? EPT : 1> rt;
  if constexpr (SM == kSegRows) {
    if (src.rowtab)
      rt.template load_at<NKX>(src.rowtab, a.seg_y0, QM::on ? quad_row(tid) : tid / CW, NT / CW);
    else
      rt.template build_at<NKX>(src.kx_start, src.off, src.nsrc, src.self_seg, src.nself, seg_stride(a),
                                QM::on ? quad_row(tid) : tid / CW, NT / CW);
  }
  // SEG (pencil: the x-expanded output blocked by x range) with row tables: the thread's x rows
  // x = (tid + k NT) / CWO of the store passes, looked up once like the kx rows
  constexpr int CWO = C / V;  // store accesses per x row (both halves in CMB mode)
  constexpr int KXS = (NX * CWO + NT - 1) / NT;
  constexpr bool kXRows = SEG && SM == kSegRows;
  static_assert(!kXRows || KXS <= kSegRowsMax, "x row table too long");
  SegRows<kXRows ? KXS : 1> xt;
  if constexpr (kXRows) xt.template build<NT, CWO, NX, 8>(a.x_start, a.poff, a.npseg, -1, 0, a.nkz, tid);
  // tile t -> (f, y0, kz0); at each iteration the blocks of one XCD take consecutive tiles
  auto decode = [&](int t, int& f, int& y, int& kz0) {
    if constexpr (SL) {
      y = (t % nyt) * YP;
      const int rest = t / nyt;
      kz0 = (rest % nkzc) * KC;
      f = rest / nkzc;
    } else {
      kz0 = (t % nkzc) * CL;
      const int rest = t / nkzc;
      y = rest % a.ny;
      f = rest / a.ny;
    }
  };
  // spectral base of input k (0: P, 1: Q) of tile field / group f, and of its self blocks
  auto in_base = [&](int f, int k) -> const T2* {
    if constexpr (CMB) return static_cast<const T2*>(src.fld[k ? cmb_in_q(f) : cmb_in_p(f)]);
    else return static_cast<const T2*>(src.base) + f * a.field_stride_spec;
  };
  auto in_self = [&](int f, int k) -> const T2* {
    if constexpr (CMB) return static_cast<const T2*>(src.self_fld[k ? cmb_in_q(f) : cmb_in_p(f)]);
    else return static_cast<const T2*>(src.self_base) + f * src.self_field_stride;
  };
  auto fetch = [&](int t) {
    int f, y, kz0;
    decode(t, f, y, kz0);
#pragma unroll
    for (int k = 0; k < NIN; ++k) {
      const T2* base = in_base(f, k);
      if constexpr (SL) {
        // each thread keeps one column (plane, kz) and walks kx rows i0 + q NT/CW, one block column
        // stride apart; the retained kx count is NKMAX (checked on the host), so only the rows of
        // the last accesses can pass it
        static_assert(NT % CW == 0, "a thread's column must be the same for every access");
        constexpr int DI = NT / CW;
        const int c = (QM::on ? quad_col(tid) : tid % CW) * V, r0 = QM::on ? quad_row(tid) : tid / CW;
        if constexpr (SM == kSegRows) {
          // rows r0 + q DI from the row table (exchange segment or own block per row)
          const T2* sbase = in_self(f, k);
          unsigned Y, KZ;
          seg_yk(1, min(y + c / KC, a.ny - 1) + a.seg_yoff, min(kz0 + c % KC, a.nkz - V), Y, KZ);
#pragma unroll
          for (int q = 0; q < EPT; ++q) {
            const CV& r = *reinterpret_cast<const CV*>((rt.is_self(q) ? sbase : base) + rt.at(q, Y, KZ));
            v[k][q] = a.nt ? ld_nt(r) : r;
          }
          continue;
        }
        const unsigned bt = spec_blk_off(a, min(y + c / KC, a.ny - 1), 0, min(kz0 + c % KC, a.nkz - V)) *
                            static_cast<unsigned>(sizeof(T2));
        const unsigned rs = static_cast<unsigned>(a.nkzs) * kSpecYBlock * static_cast<unsigned>(sizeof(T2));
        const CV* bv = reinterpret_cast<const CV*>(base);
        if (a.nt) {
#pragma unroll
          for (int q = 0; q < EPT; ++q) {
            int i = r0 + q * DI;
            if ((q + 1) * DI > NKMAX) i = min(i, NKMAX - 1);
            v[k][q] = ld_nt(at_byte(bv, bt + static_cast<unsigned>(i) * rs));
          }
        } else {
#pragma unroll
          for (int q = 0; q < EPT; ++q) {
            int i = r0 + q * DI;
            if ((q + 1) * DI > NKMAX) i = min(i, NKMAX - 1);
            v[k][q] = at_byte(bv, bt + static_cast<unsigned>(i) * rs);
          }
        }
        continue;
      }
      // this rank's own block is read in place from its spectral field (no self exchange)
      const T2* sbase = src.self_seg >= 0 ? in_self(f, k) : base;
#pragma unroll
      for (int q = 0; q < EPT; ++q) {
        const int e = tid + q * NT;
        // unconditional load from a clamped valid address: rows i >= nkx are never staged,
        // columns kz >= nkz are transformed (independently) but never stored
        const int i = min(e / CW, NKX - 1);
        const int c = (e % CW) * V;
        const int kz = min(kz0 + c % KC, a.nkz - V);
        if constexpr (SM == kSegOne) {
          const CV& r = at_byte(reinterpret_cast<const CV*>(base),
                                (static_cast<unsigned>(y * NKX + i) * static_cast<unsigned>(a.nkz) + static_cast<unsigned>(kz)) *
                                    static_cast<unsigned>(sizeof(T2)));
          v[k][q] = a.nt ? ld_nt(r) : r;
        } else if constexpr (SM == kSegRows) {
          unsigned Y, KZ;
          seg_yk(a.segblk, y + a.seg_yoff, kz, Y, KZ);
          v[k][q] = *reinterpret_cast<const CV*>((rt.is_self(q) ? sbase : base) + rt.at(q, Y, KZ));
        } else {
          const SegPos sp = SM == kSegWin ? seg_find_win<kMaxSeg>(src.kx_start, src.off, src.nsrc, (q * NT) / CW, NT / CW, i)
                                          : seg_find<kMaxSeg>(src.kx_start, src.off, src.nsrc, i);
          const T2* b = static_cast<unsigned>(sp.idx - src.self_seg) < static_cast<unsigned>(src.nself) ? sbase : base;
          unsigned Y, KZ;
          seg_yk(a.segblk, y + a.seg_yoff, kz, Y, KZ);
          const long long S = seg_stride(a);
          // 32-bit offsets (checked on the host) keep the address in one VGPR: base in SGPRs
          v[k][q] = *reinterpret_cast<const CV*>(
              b + static_cast<unsigned>(sp.off + (static_cast<long long>(Y) * sp.count + (i - sp.start)) * S + KZ));
        }
      }
    }
  };
  int t = static_cast<int>(xcd_remap(blockIdx.x, gridDim.x));
  if (t < ntiles) fetch(t);
  for (; t < ntiles; t += G) {
    int f, y, kz0;
    decode(t, f, y, kz0);
    lds_barrier();  // previous tile's stores have finished reading s
    // element (kx 0, kz 0) of field zero_mean_field reads as 0 (the omega_y source is the omega
    // state, whose mean line holds U(y)); it is kx row i = 0, the kz-0 column of each plane
    const bool zmean = !CMB && f == a.zero_mean_field && kz0 + a.kz_glob0 == 0;
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + q * NT;
      const int i = QM::on ? quad_row(tid) + q * (NT / CW) : (SL ? tid / CW + q * (NT / CW) : e / CW);
      const int c = (QM::on ? quad_col(tid) : (SL ? tid % CW : e - (e / CW) * CW)) * V;
      const int x = i <= KXH ? i : NX - (NKX - i);
      if (QM::on || SL ? i < NKX : e < nload) {
        if constexpr (CMB) {
          // the two outputs of the group from the two inputs (wavenumbers of this element)
          const int kxs = i <= KXH ? i : i - NKX;
          const T al = static_cast<T>(a.ax * kxs);
#pragma unroll
          for (int u = 0; u < V; ++u) {
            const int kzg = a.kz_glob0 + kz0 + (c + u) % KC;
            const T be = static_cast<T>(a.az * kzg);
            const T r = cmb_rcp<T>(al * al + be * be);
            T2 A, B;
            cmb_pair<T2, T>(f, v[0][q].c[u], v[1][q].c[u], al, be, r, i == 0 && kzg == 0, A, B);
            s[(c + u) * PITCH + fft_pidx(x)] = A;
            s[(CL + c + u) * PITCH + fft_pidx(x)] = B;
          }
        } else {
#pragma unroll
          for (int u = 0; u < V; ++u)
            s[(c + u) * PITCH + fft_pidx(x)] = (zmean && i == 0 && (c + u) % KC == 0) ? T2{0, 0} : v[0][q].c[u];
        }
      }
    }
    // zero padding: only the band elements the first pass reads (its input blocks that straddle
    // the band edges; the blocks inside the band are compile-time zeros, wave_pass ZB)
    {
      constexpr int Q0 = NX / FftPlan<NX>::R0, KX = NX / 3;
      constexpr int ZLO = KX + 1, ZHI = NX - KX - 1;                    // band [ZLO, ZHI]
      constexpr int E1 = ZLO % Q0 ? std::min(ZHI, Q0 * (ZLO / Q0 + 1) - 1) : ZLO - 1;  // [ZLO, E1]
      constexpr int S2 = (ZHI + 1) % Q0 ? std::max(ZLO, Q0 * (ZHI / Q0)) : ZHI + 1;    // [S2, ZHI]
      constexpr int N1 = E1 - ZLO + 1, N2 = (S2 > E1 ? ZHI - S2 + 1 : 0);
      for (int e = tid; e < (N1 + N2) * C; e += NT) {
        const int j = e / C, c = e - j * C;
        s[c * PITCH + fft_pidx(j < N1 ? ZLO + j : S2 + (j - N1))] = T2{0, 0};
      }
    }
    lds_barrier();
    if (t + G < ntiles) fetch(t + G);
    {
      constexpr int TPR = Cfg::TPR;
      constexpr int RW = C / (NT / TPR);  // rows (kz columns) owned by each wave (or wave pair)
      // one row at a time from 1024 points (the prefetched next tile already holds EPT registers);
      // shorter rows RB at a time, so a radix-16 pass has 64 butterflies for the 64 lanes
      // (a power of two, so it divides RW: the last call must not run into the next wave's rows)
      constexpr int RB = pow2_floor(1024 / NX < 1 ? 1 : (1024 / NX < RW ? 1024 / NX : RW));
      if (!(a.diag & 1))
#pragma unroll 1
        for (int rr = 0; rr < RW; rr += RB)
          wave_fft<NX, RB, PITCH, true, TPR, true>(s + ((tid / TPR) * RW + rr) * PITCH, tws, tid % TPR);
    }
    lds_barrier();
    // output field of LDS column c (CMB: the group's two outputs) and its kz / plane
    const int fa = CMB ? cmb_out_a(f) : f, fb = CMB ? cmb_out_b(f) : f;
    T2* outa = phys + fa * a.field_stride_phys;
    T2* outb = phys + fb * a.field_stride_phys;
    if constexpr (kXRows) {
#pragma unroll
      for (int k = 0; k < KXS; ++k) {
        const int e = tid + k * NT;
        const int x = e / CWO, c = (e - x * CWO) * V;
        const int cc = c % CL;
        const int kz = kz0 + cc % KC, yy = y + cc / KC;
        if (e < NX * CWO && kz < a.nkz && yy < a.ny) {
          CV w;
#pragma unroll
          for (int u = 0; u < V; ++u) w.c[u] = s[(c + u) * PITCH + fft_pidx(x)];
          *reinterpret_cast<CV*>((c < CL ? outa : outb) + xt.at(k, yy, kz)) = w;
        }
      }
      continue;
    }
    for (int e = tid; e < NX * CWO; e += NT) {
      const int x = e / CWO, c = (e - x * CWO) * V;
      const int cc = c % CL;
      const int kz = kz0 + cc % KC, yy = y + cc / KC;
      if (kz < a.nkz && yy < a.ny) {
        CV w;
#pragma unroll
        for (int u = 0; u < V; ++u) w.c[u] = s[(c + u) * PITCH + fft_pidx(x)];
        T2* out = c < CL ? outa : outb;
        if constexpr (SEG) {
          const SegPos sp = seg_find(a.x_start, a.poff, a.npseg, x);
          *reinterpret_cast<CV*>(out + sp.off + (static_cast<long long>(yy) * sp.count + (x - sp.start)) * a.nkz + kz) = w;
        } else {
          at_byte(reinterpret_cast<CV*>(out), (static_cast<unsigned>(yy * NX + x) * static_cast<unsigned>(a.nkz) +
                                               static_cast<unsigned>(kz)) * static_cast<unsigned>(sizeof(T2))) = w;
        }
      }
    }
  }
}

template <int NX, typename T, bool SEG, int WIDE, int SM = kSegFull, int V = 1, int SL = 0>
__global__ void __launch_bounds__((XCfg<NX, T, WIDE>::NT), (XCfg<NX, T, WIDE>::MINB))
    xfft_forward_kernel(XArgs a, const typename C2<T>::type* phys, XDst dst, const typename C2<T>::type* tw) {
  using T2 = typename C2<T>::type;
  using Cfg = XCfg<NX, T, WIDE>;
  using CV = CVec<T2, V>;
  using QM = XQuad<NX, T, WIDE, SL, V>;
  constexpr int C = Cfg::C, NT = Cfg::NT, PITCH = QM::PITCH;
  constexpr int CW = C / V;
  constexpr int EPT = (NX * CW + NT - 1) / NT;
  static_assert(!QM::on || NT % CW == 0, "quad lane map: a thread's column is the same for every access");
  constexpr int NKX = 2 * (NX / 3) + 1, KXH = NX / 3;  // retained kx: the 2/3 rule's (checked on the host)
  __shared__ T2 s[C * PITCH];
  constexpr int TS = FftPlan<NX>::TSIZE;
  __shared__ T2 tws[TS];
  if (a.lds_poison) {
    lds_poison_fill(s, sizeof(s));
    lds_poison_fill(tws, sizeof(tws));
    __syncthreads();
  }
  for (int i = threadIdx.x; i < TS; i += NT) tws[i] = tw[i];
  constexpr int KC = SL == 2 ? kSpecKzBlock : C, YP = C / KC;
  static_assert(SL != 2 || C % kSpecKzBlock == 0, "plane tiles need whole kz blocks");
  const int nkzc = (a.nkz + KC - 1) / KC, nyt = (a.ny + YP - 1) / YP;
  const int ntiles = nyt * nkzc * a.nfields;
  const int G = static_cast<int>(gridDim.x);
  const int tid = threadIdx.x;
  CV v[EPT];
  static_assert(SL == 0 || SM == kSegOne || SM == kSegRows, "blocked spectral layout: one destination block or row tables");
  constexpr int KE = (NKX * CW + NT - 1) / NT;  // store passes over the retained kx rows
  static_assert(SM != kSegRows || (NT % CW == 0 && KE <= kSegRowsMax), "row table: a thread's rows repeat per pass");
  SegRows<SM == kSegRows ? KE : 1> rt;
  if constexpr (SM == kSegRows) {
    if (dst.rowtab) rt.template load_at<NKX>(dst.rowtab, a.seg_y0, tid / CW, NT / CW);
    else rt.template build<NT, CW, NKX>(dst.kx_start, dst.off, dst.ndst, dst.self_seg, dst.nself, seg_stride(a), tid);
  }
  // SEG (pencil: the x-expanded input blocked by x range) with row tables: the thread's x rows of
  // the fetch (x = (tid + q NT) / CW, clamped), looked up once
  constexpr bool kXRows = SEG && SM == kSegRows;
  static_assert(!kXRows || (EPT <= kSegRowsMax && !QM::on), "x row table too long");
  SegRows<kXRows ? EPT : 1> xt;
  if constexpr (kXRows) xt.template build<NT, CW, NX, 8>(a.x_start, a.poff, a.npseg, -1, 0, a.nkz, tid);
  auto decode = [&](int t, int& f, int& y, int& kz0) {
    if constexpr (SL) {
      y = (t % nyt) * YP;
      const int rest = t / nyt;
      kz0 = (rest % nkzc) * KC;
      f = rest / nkzc;
    } else {
      kz0 = (t % nkzc) * C;
      const int rest = t / nkzc;
      y = rest % a.ny;
      f = rest / a.ny;
    }
  };
  auto fetch = [&](int t) {
    int f, y, kz0;
    decode(t, f, y, kz0);
    const T2* in = phys + f * a.field_stride_phys;
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + q * NT;
      const int x = min(QM::on ? quad_row(tid) + q * (NT / CW) : e / CW, NX - 1);
      const int c = (QM::on ? quad_col(tid) : e % CW) * V;
      const int kz = min(kz0 + c % KC, a.nkz - V), yy = min(y + c / KC, a.ny - 1);
      if constexpr (kXRows) {
        v[q] = *reinterpret_cast<const CV*>(in + xt.at(q, yy, kz));
      } else if constexpr (SEG) {
        const SegPos sp = seg_find(a.x_start, a.poff, a.npseg, x);
        v[q] = *reinterpret_cast<const CV*>(in + static_cast<unsigned>(sp.off) +
                                            static_cast<unsigned>(yy * sp.count + x - sp.start) * static_cast<unsigned>(a.nkz) +
                                            static_cast<unsigned>(kz));
      } else {
        v[q] = at_byte(reinterpret_cast<const CV*>(in), (static_cast<unsigned>(yy * NX + x) * static_cast<unsigned>(a.nkz) +
                                                         static_cast<unsigned>(kz)) * static_cast<unsigned>(sizeof(T2)));
      }
    }
  };
  int t = static_cast<int>(xcd_remap(blockIdx.x, gridDim.x));
  if (t < ntiles) fetch(t);
  for (; t < ntiles; t += G) {
    int f, y, kz0;
    decode(t, f, y, kz0);
    lds_barrier();
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + q * NT;
      const int x = QM::on ? quad_row(tid) + q * (NT / CW) : e / CW;
      const int c = (QM::on ? quad_col(tid) : e - (e / CW) * CW) * V;
      if (QM::on ? x < NX : e < NX * CW)
#pragma unroll
        for (int u = 0; u < V; ++u) s[(c + u) * PITCH + fft_pidx(x)] = v[q].c[u];
    }
    lds_barrier();
    if (t + G < ntiles) fetch(t + G);
    {
      constexpr int TPR = Cfg::TPR;
      constexpr int RW = C / (NT / TPR);  // rows (kz columns) owned by each wave (or wave pair)
      // one row at a time from 1024 points (the prefetched next tile already holds EPT registers);
      // shorter rows RB at a time, so a radix-16 pass has 64 butterflies for the 64 lanes
      // (a power of two, so it divides RW: the last call must not run into the next wave's rows)
      constexpr int RB = pow2_floor(1024 / NX < 1 ? 1 : (1024 / NX < RW ? 1024 / NX : RW));
      if (!(a.diag & 1))
#pragma unroll 1
        for (int rr = 0; rr < RW; rr += RB)
          wave_fft<NX, RB, PITCH, false, TPR, false, true>(s + ((tid / TPR) * RW + rr) * PITCH, tws, tid % TPR);
    }
    lds_barrier();
    T2* outb = static_cast<T2*>(dst.base) + f * a.field_stride_spec;
    if constexpr (SL && SM != kSegRows) {
      // one column per thread (NT % CW == 0), kx rows one block-column stride apart
      static_assert(NT % CW == 0, "a thread's column must be the same for every access");
      const int c = (tid % CW) * V;
      const int kz = kz0 + c % KC, yy = y + c / KC;
      if (kz < a.nkz && yy < a.ny) {
        const unsigned ot = spec_blk_off(a, yy, 0, kz) * static_cast<unsigned>(sizeof(T2));
        const unsigned rs = static_cast<unsigned>(a.nkzs) * kSpecYBlock * static_cast<unsigned>(sizeof(T2));
        CV* ov = reinterpret_cast<CV*>(outb);
        for (int i = tid / CW; i < NKX; i += NT / CW) {
          const int x = i <= KXH ? i : NX - (NKX - i);
          CV w;
#pragma unroll
          for (int u = 0; u < V; ++u) w.c[u] = s[(c + u) * PITCH + fft_pidx(x)];
          if (a.nt) st_nt(at_byte(ov, ot + static_cast<unsigned>(i) * rs), w);
          else at_byte(ov, ot + static_cast<unsigned>(i) * rs) = w;
        }
      }
      continue;
    }
    // this rank's own block goes straight into its spectral field (no self exchange)
    T2* soutb = dst.self_seg >= 0 ? static_cast<T2*>(dst.self_base) + f * dst.self_field_stride : outb;
    if constexpr (SM == kSegRows) {
#pragma unroll
      for (int k = 0; k < KE; ++k) {
        const int e = k * NT + tid;
        const int i = e / CW, c = (e - i * CW) * V;
        const int kz = kz0 + c % KC, yy = y + c / KC;
        if (e < NKX * CW && kz < a.nkz && yy < a.ny) {
          const int x = i <= KXH ? i : NX - (NKX - i);
          CV w;
#pragma unroll
          for (int u = 0; u < V; ++u) w.c[u] = s[(c + u) * PITCH + fft_pidx(x)];
          unsigned Y, KZ;
          seg_yk(a.segblk, yy + a.seg_yoff, kz, Y, KZ);
          CV& r = *reinterpret_cast<CV*>((rt.is_self(k) ? soutb : outb) + rt.at(k, Y, KZ));
          if (SL && a.nt) st_nt(r, w);
          else r = w;
        }
      }
      continue;
    }
    for (int e0 = 0; e0 < NKX * CW; e0 += NT) {
      const int e = e0 + tid;
      const int i = e / CW, c = (e - i * CW) * V;
      const int kz = kz0 + c % KC, yy = y + c / KC;
      if (e < NKX * CW && kz < a.nkz && yy < a.ny) {
        const int x = i <= KXH ? i : NX - (NKX - i);
        CV w;
#pragma unroll
        for (int u = 0; u < V; ++u) w.c[u] = s[(c + u) * PITCH + fft_pidx(x)];
        if constexpr (SM == kSegOne) {
          CV& r = at_byte(reinterpret_cast<CV*>(outb), (static_cast<unsigned>(y * NKX + i) * static_cast<unsigned>(a.nkz) +
                                                        static_cast<unsigned>(kz)) * static_cast<unsigned>(sizeof(T2)));
          if (a.nt) st_nt(r, w);
          else r = w;
        } else {
          const SegPos sp = SM == kSegWin ? seg_find_win<kMaxSeg>(dst.kx_start, dst.off, dst.ndst, e0 / CW, NT / CW, i)
                                          : seg_find<kMaxSeg>(dst.kx_start, dst.off, dst.ndst, i);
          T2* ob = static_cast<unsigned>(sp.idx - dst.self_seg) < static_cast<unsigned>(dst.nself) ? soutb : outb;
          unsigned Y, KZ;
          seg_yk(a.segblk, y + a.seg_yoff, kz, Y, KZ);
          *reinterpret_cast<CV*>(ob + sp.off + (static_cast<long long>(Y) * sp.count + (i - sp.start)) * seg_stride(a) + KZ) = w;
        }
      }
    }
  }
}

// The template arguments of the last x-transform launch of this thread, as in the rocprofv3 kernel
// names ("xfft_backward_kernel<1024, float, false, 1, 0, 2, 2, true>"): tests assert that they
// exercise the variant the headline grid runs.  Recorded as plain values on the launch path and
// formatted only when asked for (xfft_last_variant).
struct XVariant {
  const char* kernel = "";
  int nn = 0, wide = 0, sm = 0, v = 0, sl = 0;
  bool f64 = false, seg = false;
  int cmb = -1;  // -1: the kernel has no combine argument (the forward)
};
XVariant& xfft_variant_slot();
inline void xfft_note_variant(const char* k, int nn, bool f64, bool seg, int wide, int sm, int v, int sl, int cmb = -1) {
  xfft_variant_slot() = XVariant{k, nn, wide, sm, v, sl, f64, seg, cmb};
}

// Persistent grid of a transform kernel: the resident capacity, or fewer blocks per CU when
// CHANNEL_<NAME>_BPC sets it (A/B: room beside it for a concurrent kernel of the other stream)
inline int persist_blocks(const void* kern, int threads, const char* env) {
  int cap = resident_blocks(kern, threads);
  if (const char* e = std::getenv(env)) {
    const int bpc = std::atoi(e);
    int dev = 0, cus = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (bpc > 0) cap = std::min(cap, bpc * cus);
  }
  return std::max(1, cap);
}

// 16-byte accesses (two fp32 complex per lane) need every element offset of a tile row even:
// nkz even (rows start at multiples of nkz) and every block offset and field stride even
inline bool xvec_ok(const XArgs& a, const long long* off, int n, long long self_stride, long long self_off) {
  if (a.nkz % 2 || a.field_stride_spec % 2 || a.field_stride_phys % 2 || self_stride % 2 || self_off % 2) return false;
  for (int i = 0; i < n; ++i)
    if (off[i] % 2) return false;
  for (int i = 0; i < a.npseg; ++i)
    if (a.poff[i] % 2) return false;
  static const bool off_env = [] {
    const char* e = std::getenv("CHANNEL_XVEC");
    return e && std::atoi(e) == 0;
  }();
  return !off_env;
}

template <int NN, typename T, int WIDE, int V = 1>
static void xb_launch_cfg(const XArgs& a, const XSrc& src, void* phys, const Twiddles& tw, hipStream_t s) {
  using T2 = typename C2<T>::type;
  using Cfg = XCfg<NN, T, WIDE>;
  if constexpr (V == 1 && sizeof(T) == 4 && Cfg::C % 4 == 0) {
    bool ok = xvec_ok(a, src.off, src.nsrc, src.self_field_stride, 0);
    if (a.combine)  // (every input field pointer 16-byte aligned)
      for (int j = 0; j < kCmbInputs; ++j)
        ok = ok && reinterpret_cast<uintptr_t>(src.fld[j]) % 16 == 0 &&
             (src.self_seg < 0 || reinterpret_cast<uintptr_t>(src.self_fld[j]) % 16 == 0);
    if (ok) return xb_launch_cfg<NN, T, WIDE, 2>(a, src, phys, tw, s);
  }
  // combine mode: two halves of C / 2 columns (the loaded columns per input field)
  constexpr int CL = Cfg::C / 2;
  constexpr int CWC = CL / V;
  // (no window variant here: the fetch is unrolled over the tile, and the scalar lookups of all
  // its windows, computed up front, spilled ~640 SGPRs)
  const int sm = seg_mode<Cfg::NT, CWC>(src.nsrc, src.kx_start, src.self_seg, src.off[0]);
  CH_CHECK(!a.kzb || (sm == kSegOne && a.npseg == 1 && a.nkzs % kSpecKzBlock == 0),
           "xfft_backward: the blocked spectral layout needs one source block");
  // blocked layout: plane tiles when wide (combine: one plane of one 8-wide kz block per half)
  constexpr int SLB = (WIDE && Cfg::C % kSpecKzBlock == 0) ? 2 : 1;
  constexpr int SLC = (WIDE && CL % kSpecKzBlock == 0) ? 2 : 1;
  // (row tables where a thread has at most kSegRowsMax rows: 2 VGPRs per row)
  constexpr int kRowsK = ((2 * (NN / 3) + 1) * CWC + Cfg::NT - 1) / Cfg::NT;
  constexpr int SMR = (kRowsK <= kSegRowsMax && Cfg::NT % CWC == 0) ? kSegRows : kSegFull;
  const bool rows = SMR == kSegRows && xsegrows_enabled();
  constexpr int kXRowsK = (NN * (Cfg::C / V) + Cfg::NT - 1) / Cfg::NT;
  constexpr int SMX = (SMR == kSegRows && kXRowsK <= kSegRowsMax) ? kSegRows : kSegFull;
  decltype(&xfft_backward_kernel<NN, T, false, WIDE, kSegOne, V, 0, true>) kern;
  int smv = kSegOne, slv = 0;
  if (a.combine) {
    CH_CHECK(a.nfields == 6, "xfft_backward: the combine mode forms the six physical-stage fields");
    if (a.kzb) {
      kern = xfft_backward_kernel<NN, T, false, WIDE, kSegOne, V, SLC, true>;
      slv = SLC;
    } else if (a.segblk && a.npseg == 1 && rows && SMR == kSegRows) {
      // P > 1, blocked exchange segments: plane tiles through the row table
      kern = xfft_backward_kernel<NN, T, false, WIDE, (SMR == kSegRows ? kSegRows : kSegOne), V, (SMR == kSegRows ? SLC : 0), true>;
      smv = kSegRows;
      slv = SLC;
    } else if (a.npseg > 1) {
      kern = rows ? xfft_backward_kernel<NN, T, true, WIDE, SMX, V, 0, true> : xfft_backward_kernel<NN, T, true, WIDE, kSegFull, V, 0, true>;
      smv = rows ? SMX : kSegFull;
    } else if (sm == kSegOne) {
      kern = xfft_backward_kernel<NN, T, false, WIDE, kSegOne, V, 0, true>;
    } else {
      kern = rows ? xfft_backward_kernel<NN, T, false, WIDE, SMR, V, 0, true> : xfft_backward_kernel<NN, T, false, WIDE, kSegFull, V, 0, true>;
      smv = rows ? kSegRows : kSegFull;
    }
  } else {
    // one field per tile (K-SPEC's six-output mode)
    constexpr int CW1 = Cfg::C / V;
    const int sm1 = seg_mode<Cfg::NT, CW1>(src.nsrc, src.kx_start, src.self_seg, src.off[0]);
    constexpr int kRowsK1 = ((2 * (NN / 3) + 1) * CW1 + Cfg::NT - 1) / Cfg::NT;
    constexpr int SMR1 = (kRowsK1 <= kSegRowsMax && Cfg::NT % CW1 == 0) ? kSegRows : kSegFull;
    const bool rows1 = SMR1 == kSegRows && xsegrows_enabled();
    constexpr int SMX1 = (SMR1 == kSegRows && kXRowsK <= kSegRowsMax) ? kSegRows : kSegFull;
    if (a.kzb) {
      kern = xfft_backward_kernel<NN, T, false, WIDE, kSegOne, V, SLB, false>;
      slv = SLB;
    } else if (a.segblk && a.npseg == 1 && rows1 && SMR1 == kSegRows) {
      kern = xfft_backward_kernel<NN, T, false, WIDE, (SMR1 == kSegRows ? kSegRows : kSegOne), V, (SMR1 == kSegRows ? SLB : 0), false>;
      smv = kSegRows;
      slv = SLB;
    } else if (a.npseg > 1) {
      kern = rows1 ? xfft_backward_kernel<NN, T, true, WIDE, SMX1, V, 0, false> : xfft_backward_kernel<NN, T, true, WIDE, kSegFull, V, 0, false>;
      smv = rows1 ? SMX1 : kSegFull;
    } else if (sm1 == kSegOne) {
      kern = xfft_backward_kernel<NN, T, false, WIDE, kSegOne, V, 0, false>;
    } else {
      kern = rows1 ? xfft_backward_kernel<NN, T, false, WIDE, SMR1, V, 0, false> : xfft_backward_kernel<NN, T, false, WIDE, kSegFull, V, 0, false>;
      smv = rows1 ? kSegRows : kSegFull;
    }
  }
  const int cl = a.combine ? CL : Cfg::C;
  const int kc = slv == 2 ? kSpecKzBlock : cl, yp = cl / kc;
  const int ntiles = (a.ny + yp - 1) / yp * ((a.nkz + kc - 1) / kc) * (a.combine ? kCmbGroups : a.nfields);
  xfft_note_variant("xfft_backward_kernel", NN, sizeof(T) == 8, !a.kzb && !slv && a.npseg > 1, WIDE, smv, V, slv, a.combine ? 1 : 0);
  dim3 grid(std::min(ntiles, persist_blocks(reinterpret_cast<const void*>(kern), Cfg::NT, "CHANNEL_XB_BPC")));
  hipLaunchKernelGGL(kern, grid, dim3(Cfg::NT), 0, s, a, src, static_cast<T2*>(phys), static_cast<const T2*>(tw.buf));
}

template <int NN, typename T, int WIDE, int V = 1>
static void xf_launch_cfg(const XArgs& a, const void* phys, const XDst& dst, const Twiddles& tw, hipStream_t s) {
  using T2 = typename C2<T>::type;
  using Cfg = XCfg<NN, T, WIDE>;
  if constexpr (V == 1 && sizeof(T) == 4 && Cfg::C % 2 == 0) {
    if (xvec_ok(a, dst.off, dst.ndst, dst.self_field_stride, 0)) return xf_launch_cfg<NN, T, WIDE, 2>(a, phys, dst, tw, s);
  }
  const int sm = seg_mode<Cfg::NT, Cfg::C / V>(dst.ndst, dst.kx_start, dst.self_seg, dst.off[0]);
  CH_CHECK(!a.kzb || (sm == kSegOne && a.npseg == 1 && a.nkzs % kSpecKzBlock == 0),
           "xfft_forward: the blocked spectral layout needs one destination block");
  constexpr int SLB = (WIDE && Cfg::C % kSpecKzBlock == 0) ? 2 : 1;
  constexpr int kRowsK = ((2 * (NN / 3) + 1) * (Cfg::C / V) + Cfg::NT - 1) / Cfg::NT;
  constexpr int SMR = (kRowsK <= kSegRowsMax && Cfg::NT % (Cfg::C / V) == 0) ? kSegRows : kSegFull;
  const bool rows = SMR == kSegRows && xsegrows_enabled();
  constexpr int kXRowsK = (NN * (Cfg::C / V) + Cfg::NT - 1) / Cfg::NT;
  constexpr int SMX = (SMR == kSegRows && kXRowsK <= kSegRowsMax) ? kSegRows : kSegFull;
  const bool segsl = !a.kzb && a.segblk && a.npseg == 1 && rows && SMR == kSegRows;  // P > 1 plane tiles
  auto kern = a.kzb                   ? xfft_forward_kernel<NN, T, false, WIDE, kSegOne, V, SLB>
              : segsl                 ? xfft_forward_kernel<NN, T, false, WIDE, (SMR == kSegRows ? kSegRows : kSegOne), V, (SMR == kSegRows ? SLB : 0)>
              : a.npseg > 1           ? (rows ? xfft_forward_kernel<NN, T, true, WIDE, SMX, V>
                                              : xfft_forward_kernel<NN, T, true, WIDE, kSegFull, V>)
              : sm == kSegOne ? xfft_forward_kernel<NN, T, false, WIDE, kSegOne, V>
              : rows          ? xfft_forward_kernel<NN, T, false, WIDE, SMR, V>
              : sm == kSegWin ? xfft_forward_kernel<NN, T, false, WIDE, kSegWin, V>
                              : xfft_forward_kernel<NN, T, false, WIDE, kSegFull, V>;
  const int kc = ((a.kzb || segsl) && SLB == 2) ? kSpecKzBlock : Cfg::C, yp = Cfg::C / kc;
  const int ntiles = (a.ny + yp - 1) / yp * ((a.nkz + kc - 1) / kc) * a.nfields;
  xfft_note_variant("xfft_forward_kernel", NN, sizeof(T) == 8, (a.kzb || segsl) ? 0 : (a.npseg > 1), WIDE,
                    a.kzb ? kSegOne : segsl ? kSegRows : (a.npseg > 1 ? (rows ? SMX : kSegFull) : (sm != kSegOne && rows ? kSegRows : sm)), V,
                    (a.kzb || segsl) ? SLB : 0);
  dim3 grid(std::min(ntiles, persist_blocks(reinterpret_cast<const void*>(kern), Cfg::NT, "CHANNEL_XF_BPC")));
  hipLaunchKernelGGL(kern, grid, dim3(Cfg::NT), 0, s, a, static_cast<const T2*>(phys), dst,
                     static_cast<const T2*>(tw.buf));
}

// ---- 1024-point row transform, 4 x 16 x 16 (z stage, fp32) -----------------------------------
// In and out in the row layout of the z stage (lane t, slot s: element t + 64 s), Stockham DIT:
//  P1 (R = 4, NS = 1): butterfly j = t + 64 g takes slots g, g + 4, g + 8, g + 12 of lane t -- all in
//     the lane's registers, no twiddles; output y1[4 t + 256 g + b] lands in slot 4 g + b;
//  a 4 x 4 transpose of (lane row t / 16, slot index b) for each g, by v_permlane32_swap (row bit 1
//     <-> b bit 1) and v_permlane16_swap (row bit 0 <-> b bit 0): lane u = a + 16 k2 then holds the
//     16 inputs r = 4 g + c of the P2 butterfly j2 = 4 a + k2, in slot r;
//  P2 (R = 16, NS = 4): twiddles W_64^(k2 r) (tw2, registers) and a radix-16 DFT; the outputs go to
//     LDS positions 64 a + k2 + 4 r' (one pad slot per 64 elements: 65 a + k2 + 4 r', conflict-free
//     for the stride-64 ds_write_b64 groups);
//  P3 (R = 16, NS = 64): lane j3 reads j3 + 64 r (65 r + j3: contiguous, conflict-free), twiddles
//     W_1024^(j3 r) (tw3 table in LDS), radix-16 DFT; output r' is element j3 + 64 r' (the layout of
//     the input).
// One LDS round trip per transform instead of two (the 16 x 16 x 4 plan's first and last passes
// run in registers but its middle pass reads and writes LDS both ways), for +32 permlane moves.
// tw3: [15][64] W_1024^(j r) then (kR4Tw2) [15][4] W_64^(k r), forward sign; INV conjugates.
constexpr int kR4Tw2 = 15 * 64, kR4TwSize = 15 * 64 + 15 * 4;
__device__ __forceinline__ void permlane32_swap_c(float2& a, float2& b) {
  const auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.x), __float_as_uint(b.x), false, false);
  const auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.y), __float_as_uint(b.y), false, false);
  a = float2{__uint_as_float(rx[0]), __uint_as_float(ry[0])};
  b = float2{__uint_as_float(rx[1]), __uint_as_float(ry[1])};
}
__device__ __forceinline__ void permlane16_swap_c(float2& a, float2& b) {
  const auto rx = __builtin_amdgcn_permlane16_swap(__float_as_uint(a.x), __float_as_uint(b.x), false, false);
  const auto ry = __builtin_amdgcn_permlane16_swap(__float_as_uint(a.y), __float_as_uint(b.y), false, false);
  a = float2{__uint_as_float(rx[0]), __uint_as_float(ry[0])};
  b = float2{__uint_as_float(rx[1]), __uint_as_float(ry[1])};
}
template <bool INV>
__device__ __forceinline__ void fft1024_4x16x16(float2 (&x)[16], float2* __restrict__ buf, const float2 (&tw2)[15],
                                                const float2* __restrict__ tw3, int lane) {
  // P1: radix-4 inside the lane
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    float2 v[4] = {x[g], x[g + 4], x[g + 8], x[g + 12]};
    dft4<INV>(v);
    float2 y[4] = {v[0], v[1], v[2], v[3]};
    // slot 4 g + b holds output b (written after all four loads of this g: slots g + 4 r overlap)
    x[g] = y[0];
    x[g + 4] = y[1];
    x[g + 8] = y[2];
    x[g + 12] = y[3];
  }
  // (P1 left output b of group g in slot g + 4 b; the transpose below works on slot 4 g + b, so
  // relabel: z[4 g + b] = x[g + 4 b])
  float2 z[16];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int b = 0; b < 4; ++b) z[4 * g + b] = x[g + 4 * b];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    permlane32_swap_c(z[4 * g + 0], z[4 * g + 2]);
    permlane32_swap_c(z[4 * g + 1], z[4 * g + 3]);
    permlane16_swap_c(z[4 * g + 0], z[4 * g + 1]);
    permlane16_swap_c(z[4 * g + 2], z[4 * g + 3]);
  }
  // P2: slot r = input r of butterfly 4 a + k2 (a = lane % 16, k2 = lane / 16)
#pragma unroll
  for (int r = 1; r < 16; ++r) z[r] = cmul_tw<INV>(z[r], tw2[r - 1]);
  dft16<INV>(z);
  {
    float2* q = buf + 65 * (lane & 15) + (lane >> 4);
#pragma unroll
    for (int r = 0; r < 16; ++r) q[4 * r] = z[r];
  }
  __builtin_amdgcn_wave_barrier();
  // P3: butterfly j3 = lane
  {
    const float2* p = buf + lane;
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = p[65 * r];
  }
  __builtin_amdgcn_wave_barrier();  // (the reads precede the row's next writes)
#pragma unroll
  for (int r = 1; r < 16; ++r) x[r] = cmul_tw<INV>(x[r], tw3[(r - 1) * 64 + lane]);
  dft16<INV>(x);
}

// ---- z-direction physical stage -------------------------------------------------------------
__device__ __forceinline__ void atomic_max_pos(float* p, float v) {
  atomicMax(reinterpret_cast<unsigned int*>(p), __float_as_uint(v));
}

// One wave per (y,x) row up to 1024 points; a block holds ZWT rows and each wave owns one LDS row
// buffer, so there is no block barrier between the gather, the five FFTs, the product and the
// extraction.  The six physical fields stay in registers (thread t of a row owns points
// n = t + TPR i).  2048-point rows take two waves (TPR = 128) with block barriers between the
// passes: at one wave per row the 6 x 32 points per lane needed ~430 registers (one wave per
// SIMD; 180 spilled VGPRs in fp64), at two waves the register budget of the 1024-point kernel.
// Below 1024 points a wave holds several rows (TPR < 64 threads per row): every thread keeps 16
// (fp32) or 8 (fp64) points per field, and the wave's transforms cover all its rows at once, so a
// 128-point row no longer leaves 56 of 64 lanes idle in its first radix-16 pass.
constexpr int ZW = 4;
// threads per row: 16 (fp32) / 8 (fp64) points per thread, rounded up to a power of two so a
// wave holds a whole number of rows (lengths 3*2^k, 5*2^k: 12 / 10 points per thread)
template <int NZP>
constexpr int zphys_tpr(int esz = 4) {
  return esz == 4 ? (NZP >= 16 ? pow2_ceil((NZP + 15) / 16) : 1)
                  : (NZP >= 1024 ? 128 : (NZP >= 16 ? pow2_ceil((NZP + 7) / 8) : 1));
}
// rows per block: 2 above 1536 points (two row buffers + the twiddles fit twice per CU in fp32;
// four fp64 rows of 1792 points and their twiddles would exceed the LDS); 4 waves' worth of rows
// below 64 threads per row
template <int NZP, typename T, int TPR = zphys_tpr<NZP>(sizeof(T))>
constexpr int zphys_rows() {
  return TPR < 64 ? ZW * 64 / TPR : (NZP > 1536 || (sizeof(T) == 4 && TPR == 128) ? 2 : ZW);
}

template <int NZP, typename T, bool SEG, bool ZH = true, int TPRT = zphys_tpr<NZP>(sizeof(T)),
          int ZWT = zphys_rows<NZP, T, TPRT>(), int WPE = 2, int ZF = 3>
__global__ void __launch_bounds__(ZWT * TPRT) __attribute__((amdgpu_waves_per_eu(WPE), target("no-load-store-opt"))) zphys_kernel(ZArgs a, typename C2<T>::type* fields,
                                                         const typename C2<T>::type* tw) {
  using T2 = typename C2<T>::type;
  // register-edge transforms (first pass from and last pass into registers, fft_device.hpp) where
  // one wave owns a row and the plan has one first-pass butterfly per lane (NZP = 1024: 16x16x4)
  constexpr int kEP = (NZP + TPRT - 1) / TPRT, kMK = (NZP / 3 + 1 + TPRT - 1) / TPRT;
  constexpr bool kRegEdge = TPRT == 64 && kEP == 16 && FftPlan<NZP>::R0 == 16 && FftPlan<NZP>::R2 > 1 &&
                            fft_reg_edges_ok<NZP, 64>() && 2 * kMK <= 16;
  // row layout: one pad slot per 32 elements for the fp32 register-edge rows (their LDS traffic is
  // mostly contiguous 64-lane reads: conflict-free ds_read_b64, kept unmerged by the kernel's
  // no-load-store-opt attribute), per 16 elsewhere (fft_pidx_s)
  constexpr int SH = kRegEdge && sizeof(T) == 4 ? 5 : 4;
  // ZF (fp32 register-edge rows): 0 = three passes 16 x 16 x 4, middle-pass twiddles from LDS;
  // 1 = the same with those twiddles in registers; 2 = 4 x 16 x 16 with one LDS round trip
  // (fft1024_4x16x16: pad one slot per 64 elements, its own twiddle tables after the half plan's)
  // ZF = 3: the same plan, and H_z through it as a complex transform of (Hz, 0) (its outputs k < nkz
  // are the spectrum directly: no mirror, no half-length plan, one LDS round trip)
  // ZF = 4: the same, with the H_z of two consecutive rows of the wave transformed together as
  // (Hz_a + i Hz_b) and split like Hx / Hy (one 1024-point transform per two rows instead of two)
  constexpr bool kR4 = kRegEdge && sizeof(T) == 4 && NZP == 1024 && ZF >= 2;
  constexpr bool kR4Hz = kR4 && ZF >= 3;
  constexpr bool kPairHz = kR4 && ZF == 4;
  constexpr int PITCH = kR4 ? 1040 : (SH == 5 ? NZP + NZP / 32 : FftPitch<NZP>::value);
  constexpr int TPR = TPRT;  // threads per row
  constexpr int NWB = ZWT * TPR / 64;     // waves per block
  constexpr int TPRF = TPR < 64 ? 64 : TPR;  // threads per transform call (one wave or a row)
  constexpr int RWW = TPR < 64 ? 64 / TPR : 1;  // rows per transform call
  constexpr int EP = (NZP + TPR - 1) / TPR;  // points per thread
  __shared__ T2 s[ZWT * PITCH];
  constexpr int TS = FftPlan<NZP>::TSIZE;
  // real H_z: half-length complex transform + post twiddles (HalfPlan) where one exists
  using Hp = HalfPlan<NZP>;
  constexpr bool kHalf = ZH && Hp::ok;
  constexpr int TSA = TS + ((kHalf || kR4) ? Hp::SIZE : 0) + (kR4 ? kR4TwSize : 0);
  __shared__ T2 tws[TSA];  // twiddles staged once per block: LDS latency instead of L2 in the passes
  __shared__ float red[4][NWB];
  // lane: wave lane (reductions); t: thread within the row; w: row within the block
  const int tid = threadIdx.x, lane = tid & 63;
  int t = tid % TPR, w = tid / TPR;
  if (a.lds_poison) {
    lds_poison_fill(s, sizeof(s));
    lds_poison_fill(tws, sizeof(tws));
    lds_poison_fill(red, sizeof(red));
    __syncthreads();
  }
  for (int i = tid; i < TSA; i += ZWT * TPR) tws[i] = tw[i];
  __syncthreads();
  T2* row = s + w * PITCH;
  T2* frow = s + (tid / TPRF) * RWW * PITCH;  // first row of this thread's transform group
  int ft = tid % TPRF;
  const long long nrows = static_cast<long long>(a.ny) * a.NX;
  const long long ngroups = (nrows + ZWT - 1) / ZWT;
  // one segment holds every retained kz (Nzp/3 + 1: the launcher checks it), a compile-time count,
  // so only the last of a thread's kz slots needs a bound check
  const int nkz = SEG ? a.nkz : NZP / 3 + 1, Kz = nkz - 1;
  const long long fs = a.field_stride;
  float mu = 0.f, mv = 0.f, mw = 0.f, mc = 0.f;
  // element offset of (row r, kz) in the kz-blocked row layout (one block: r * nkz + kz, 32-bit:
  // one segment runs only when a field's rows fit 4 GiB (zphys_launch_tpr), so a field's accesses
  // are a uniform 64-bit base plus a 32-bit lane byte offset -- no 64-bit arithmetic per element)
  auto zaddr = [&](long long r, int k) -> long long {
    if constexpr (SEG) {
      const SegPos sp = seg_find(a.kz_start, a.off, a.nseg, k);
      return sp.off + r * sp.count + (k - sp.start);
    } else {
      return static_cast<long long>(static_cast<unsigned>(r) * static_cast<unsigned>(nkz) + static_cast<unsigned>(k));
    }
  };
  // retained kz per thread: nkz = Nzp/3 + 1 (2/3 rule; checked on the host)
  constexpr int MK = (NZP / 3 + 1 + TPR - 1) / TPR;
  auto fetch = [&](long long r, int p, T2 (&va)[MK], T2 (&vb)[MK]) {
    const bool rv = TPR < 64 ? r < nrows : true;
    const T2* A = fields + (2 * p) * fs;
    const T2* B = fields + (2 * p + 1) * fs;
    if constexpr (!SEG) {
      // unconditional loads at a clamped (in-bounds) index, zeros selected afterwards: a guarded
      // load is a branch, an exec-mask save/restore and a zero move per element
      const unsigned rb = static_cast<unsigned>(rv ? r : nrows - 1) * static_cast<unsigned>(nkz);
#pragma unroll
      for (int i = 0; i < MK; ++i) {
        const int k = t + TPR * i;
        const bool ld = k < nkz && rv;
        const unsigned o = (rb + static_cast<unsigned>(min(k, nkz - 1))) * static_cast<unsigned>(sizeof(T2));
        const T2 x = *reinterpret_cast<const T2*>(reinterpret_cast<const char*>(A) + o);
        const T2 y = *reinterpret_cast<const T2*>(reinterpret_cast<const char*>(B) + o);
        va[i] = ld ? x : T2{0, 0};
        vb[i] = ld ? y : T2{0, 0};
      }
    } else {
#pragma unroll
      for (int i = 0; i < MK; ++i) {
        const int k = t + TPR * i;
        const bool ld = k < nkz && rv;
        const long long o = ld ? zaddr(r, k) : 0;
        va[i] = ld ? A[o] : T2{0, 0};
        vb[i] = ld ? B[o] : T2{0, 0};
      }
    }
  };
  // store of field f at element offset o (one segment: a 32-bit byte offset from the field base)
  auto zstore = [&](int f, long long o, T2 v) {
    if constexpr (!SEG) {
      *reinterpret_cast<T2*>(reinterpret_cast<char*>(fields + f * fs) +
                             static_cast<unsigned>(o) * static_cast<unsigned>(sizeof(T2))) = v;
    } else {
      fields[f * fs + o] = v;
    }
  };
  // The next pair's loads are in flight during each transform where the registers fit (fp32,
  // <= 1024 points, one segment); elsewhere each pair is loaded right before its transform.
  // Persistent launch (grid = resident capacity, the block walks row groups g, g + G, ...): the
  // NEXT row's first pair is loaded during this row's forward transforms, so no row starts on an
  // exposed load latency (the one-shot launch exposed it once per row: with the
  // transforms skipped the stage still took 55 of its 88 us per 8-plane chunk).
  constexpr bool kPrefetch = sizeof(T) == 4 && NZP <= 1024 && !SEG;
  T2 pa[kPrefetch ? MK : 1], pb[kPrefetch ? MK : 1];
  // the middle pass's twiddles in registers (fp32 register-edge rows: 30 VGPRs against 15 LDS reads
  // per transform; only in the CHANNEL_ZFFT=1 plan -- ZFFT=0 keeps the LDS reads, A/B)
  constexpr bool kMidReg = kRegEdge && MidTw<NZP>::ok && sizeof(T) == 4 && ZF == 1;
  T2 twm[kMidReg || kR4 ? 15 : 1];
  if constexpr (kMidReg) middle_twiddles<NZP>(tws, twm, lane);
  // 4 x 16 x 16: the second pass's twiddles W_64^(k2 r), k2 = lane / 16, in registers; the third
  // pass's W_1024^(lane r) are read from the LDS table
  const T2* tw3 = tws + TS + Hp::SIZE;  // (Twiddles::build: after the half plan's tables at n = 1024)
  if constexpr (kR4) {
#pragma unroll
    for (int r = 1; r < 16; ++r) twm[r - 1] = tw3[kR4Tw2 + (r - 1) * 4 + lane / 16];
  }
  // (not kept: a second buffer issuing pair 2 two transforms ahead and the next row's pair 1 a
  // row ahead: 28 spilled VGPRs, 39.4 vs 37.7 ms/step, profiles/r03s3/ab_zphys_prefetch2.txt)
  long long g = blockIdx.x;
  if constexpr (kPrefetch) {
    if (g < ngroups) fetch(g * ZWT + w, 0, pa, pb);
  }
  // kPairHz: H_z of the wave's previous row, waiting for its partner (wave-uniform state), parked
  // in a per-wave LDS area (slot pair i / 2 of lane l at (i / 2) * 64 + l: conflict-free b64
  // accesses) instead of 16 registers held across the next row's inverse transforms
  __shared__ T2 hzbuf[kPairHz ? ZWT * EP / 2 * 64 : 1];
  long long rprev = 0;
  bool held = false;
  const T scz = static_cast<T>(0.5 * a.scale);
  // H_z^(k) of rows ra (the real part of the packed row) and rb (the imaginary part) from the
  // transform zh of (Hz_ra + i Hz_rb); rb < 0: a single row, zh the transform of (Hz_ra, 0)
  auto hz_split_store = [&](T2 (&zh)[EP], long long ra, long long rb, int tt) {
    const int src = (64 - tt) & 63;
#pragma unroll
    for (int i = 0; i < MK; ++i) {
      const int k = tt + TPR * i;
      const T2 pm{__shfl(zh[15 - i].x, src), __shfl(zh[15 - i].y, src)};
      const T2 Zm = tt != 0 ? pm : zh[(16 - i) & 15];
      if (k < nkz) {
        const T2 Z = zh[i];
        zstore(2, zaddr(ra, k), T2{(Z.x + Zm.x) * scz, (Z.y - Zm.y) * scz});
        if (rb >= 0) zstore(2, zaddr(rb, k), T2{(Z.y + Zm.y) * scz, -(Z.x - Zm.x) * scz});
      }
    }
  };
  // Rows past the end (TPR < 64 only: the host checks nrows % ZWT == 0 otherwise) run the
  // transforms on zeros and skip every global access.  The loop is block-uniform.
  for (; g < ngroups; g += gridDim.x) {
    {
      // the thread's lane-dependent addresses are re-derived per row from an opaque copy of the
      // thread id: hoisted out of the row loop, the LDS and global address offsets of every pass
      // stayed live across it (256 VGPRs + 74 spilled instead of 224 without the loop)
      int tl = threadIdx.x;
      asm volatile("" : "+v"(tl));
      t = tl % TPR;
      w = tl / TPR;
      ft = tl % TPRF;
      row = s + w * PITCH;
      frow = s + (tl / TPRF) * RWW * PITCH;
    }
    const T2* twl = tws;
    const long long r = g * ZWT + w;
    const bool rv = TPR < 64 ? r < nrows : true;  // (TPR >= 64: the host checks nrows % ZWT == 0)
    const long long rnext = (g + gridDim.x) * ZWT + w;
    const bool more = g + gridDim.x < ngroups;
    T2 ph[3][EP];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      T2 va[MK], vb[MK];
      if constexpr (kPrefetch) {
#pragma unroll
        for (int i = 0; i < MK; ++i) {
          va[i] = pa[i];
          vb[i] = pb[i];
        }
      } else {
        fetch(r, p, va, vb);
      }
      // Z_k = A_k + i B_k, Z_{N-k} = conj(A_k) + i conj(B_k); the kz=0 imaginary parts are dropped
      // (a real z-row has a real mean), zero padding between Kz and N-Kz.
      if constexpr (kRegEdge) {
        // First pass straight from the loaded registers: lane t's butterfly takes Z at t + 64 r,
        // r < MK directly (the lane's own modes) and, for r >= 16 - MK, the mirror Z_{N-k} of mode
        // k = 64 (15 - r) + (64 - t) held by lane 64 - t (lane 0: its own mode 64 (16 - r)); the
        // band between is the zero padding.  The mirror values cross lanes by ds_bpermute, 2
        // dwords per slot, instead of a row gather through LDS.
        T2 d[MK], m[MK];
#pragma unroll
        for (int i = 0; i < MK; ++i) {
          const int k = t + TPR * i;
          const bool ok = k < nkz;
          d[i] = ok ? (k == 0 ? T2{va[i].x, vb[i].x} : T2{va[i].x - vb[i].y, va[i].y + vb[i].x}) : T2{0, 0};
          m[i] = ok && k > 0 ? T2{va[i].x + vb[i].y, vb[i].x - va[i].y} : T2{0, 0};
        }
        if constexpr (kPrefetch) {
          if (p < 2) fetch(r, p + 1, pa, pb);
        }
        const int src = (64 - t) & 63;
        T2 x[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          if (q < MK) {
            x[q] = d[q];
          } else if (q < 16 - MK) {
            x[q] = T2{0, 0};
          } else {
            const T2 pm{__shfl(m[15 - q].x, src), __shfl(m[15 - q].y, src)};
            x[q] = t != 0 ? pm : (16 - q < MK ? m[16 - q] : T2{0, 0});
          }
        }
        if (!(a.diag & 1)) {
          if constexpr (kR4) {
            fft1024_4x16x16<true>(x, row, twm, tw3, t);
#pragma unroll
            for (int i = 0; i < EP; ++i) ph[p][i] = x[i];
          } else {
            wave_pass_first_reg<NZP, true, SH>(row, x, t);
            row_sync<64>();
            if constexpr (kMidReg) wave_pass_middle_rt<NZP, PITCH, true, SH>(row, twm, t);
            else wave_pass_middle<NZP, PITCH, true, 64, SH>(row, twl, t);
            wave_pass_last_reg<NZP, true, 64, SH>(row, twl, ph[p], t);
          }
        } else {
#pragma unroll
          for (int i = 0; i < EP; ++i) ph[p][i] = x[i];
        }
        row_sync<64>();  // the last pass's reads precede the next pair's first-pass writes
      } else {
#pragma unroll
      for (int i = 0; i < MK; ++i) {
        const int k = t + TPR * i;
        if (k < nkz) {
          if (k == 0) {
            row[fft_pidx(0)] = T2{va[i].x, vb[i].x};
          } else {
            row[fft_pidx(k)] = T2{va[i].x - vb[i].y, va[i].y + vb[i].x};
            row[fft_pidx(NZP - k)] = T2{va[i].x + vb[i].y, vb[i].x - va[i].y};
          }
        }
      }
      for (int k = Kz + 1 + t; k < NZP - Kz; k += TPR) row[fft_pidx(k)] = T2{0, 0};
      if constexpr (kPrefetch) {
        if (p < 2) fetch(r, p + 1, pa, pb);
      }
      row_sync<TPRF>();
      if (!(a.diag & 1)) wave_fft<NZP, RWW, PITCH, true, TPRF>(frow, twl, ft);
#pragma unroll
      for (int i = 0; i < EP; ++i) {
        const int n = t + TPR * i;
        ph[p][i] = n < NZP ? row[fft_pidx(n)] : T2{0, 0};
      }
      row_sync<TPRF>();
      }
    }
    // rotational product H = u x omega (convolution_kernels.cu:125-131) and CFL maxima
    const int yl = rv ? static_cast<int>(r / a.NX) : 0;
    const float idy = static_cast<float>(a.inv_dy[a.y0 + yl]);
    // (the CFL sum in fp32: a double kx_max promoted every point's sum to fp64, 2 cvt + 2 FMA64 per point)
    const float cxf = static_cast<float>(a.cx), czf = static_cast<float>(a.cz);
    T hz[EP];
    T2 hxy[kRegEdge ? EP : 1];
#pragma unroll
    for (int i = 0; i < EP; ++i) {
      const T u = ph[0][i].x, v = ph[0][i].y, ww = ph[1][i].x, wx = ph[1][i].y, wy = ph[2][i].x, wz = ph[2][i].y;
      const T hx = v * wz - ww * wy, hy = ww * wx - u * wz;
      hz[i] = u * wy - v * wx;
      const float au = fabsf(static_cast<float>(u)), av = fabsf(static_cast<float>(v)), aw = fabsf(static_cast<float>(ww));
      mu = fmaxf(mu, au);
      mv = fmaxf(mv, av);
      mw = fmaxf(mw, aw);
      mc = fmaxf(mc, au * cxf + av * idy + aw * czf);
      const int n = t + TPR * i;
      if constexpr (kRegEdge) hxy[i] = T2{hx, hy};
      else if (n < NZP) row[fft_pidx(n)] = T2{hx, hy};
    }
    const T sc = static_cast<T>(0.5 * a.scale);
    // (Hx + i Hy)^_k = Z_k: Hx_k = (Z_k + conj Z_{N-k})/2, Hy_k = (Z_k - conj Z_{N-k})/(2i)
    // (unrolled: all LDS reads are issued before the global stores)
    constexpr int MKO = MK;  // retained kz per thread (nkz <= NZP/3 + 1)
    if constexpr (kRegEdge) {
      // first pass from the product registers, last pass into registers; Z_{N-k} of the lane's
      // mode k = t + 64 i sits in lane 64 - t at slot 15 - i (lane 0: its own slot 16 - i)
      T2 z[EP];
      if (!(a.diag & 1)) {
        if constexpr (kR4) {
#pragma unroll
          for (int i = 0; i < EP; ++i) z[i] = hxy[i];
          fft1024_4x16x16<false>(z, row, twm, tw3, t);
        } else {
          wave_pass_first_reg<NZP, false, SH>(row, hxy, t);
          row_sync<64>();
          if constexpr (kMidReg) wave_pass_middle_rt<NZP, PITCH, false, SH>(row, twm, t);
          else wave_pass_middle<NZP, PITCH, false, 64, SH>(row, twl, t);
          wave_pass_last_reg<NZP, false, 64, SH>(row, twl, z, t);
        }
      } else {
#pragma unroll
        for (int i = 0; i < EP; ++i) z[i] = hxy[i];
      }
      const int src = (64 - t) & 63;
#pragma unroll
      for (int i = 0; i < MKO; ++i) {
        const int k = t + TPR * i;
        const T2 pm{__shfl(z[15 - i].x, src), __shfl(z[15 - i].y, src)};
        const T2 Zm = t != 0 ? pm : z[(16 - i) & 15];
        if (k < nkz) {
          const T2 Z = z[i];
          const long long o = zaddr(r, k);
          zstore(0, o, T2{(Z.x + Zm.x) * sc, (Z.y - Zm.y) * sc});
          zstore(1, o, T2{(Z.y + Zm.y) * sc, -(Z.x - Zm.x) * sc});
        }
      }
    } else {
    row_sync<TPRF>();
    if (!(a.diag & 1)) wave_fft<NZP, RWW, PITCH, false, TPRF>(frow, twl, ft);
    {
      T2 z0[MKO] = {}, z1[MKO] = {};  // (zero-initialised: conditionally set arrays became loop-carried)
#pragma unroll
      for (int i = 0; i < MKO; ++i) {
        const int k = t + TPR * i;
        if (k < nkz) {
          z0[i] = row[fft_pidx(k)];
          z1[i] = row[fft_pidx(k == 0 ? 0 : NZP - k)];
        }
      }
#pragma unroll
      for (int i = 0; i < MKO; ++i) {
        const int k = t + TPR * i;
        if (k < nkz && rv) {
          const T2 Z = z0[i], Zm = z1[i];
          const long long o = zaddr(r, k);
          zstore(0, o, T2{(Z.x + Zm.x) * sc, (Z.y - Zm.y) * sc});
          zstore(1, o, T2{(Z.y + Zm.y) * sc, -(Z.x - Zm.x) * sc});
        }
      }
    }
    }
    // the next row's first pair: in flight during this row's H_z transform and stores (and the
    // next row's start); issued here, after the Hx/Hy stores, it adds nothing to the register peak
    if constexpr (kPrefetch) {
      if (more) fetch(rnext, 0, pa, pb);
    }
    row_sync<TPRF>();
    if constexpr (kPairHz) {
      T2* hb = hzbuf + w * (EP / 2) * 64 + t;
      if (!held) {
#pragma unroll
        for (int i = 0; i < EP / 2; ++i) hb[i * 64] = T2{hz[2 * i], hz[2 * i + 1]};
        rprev = r;
        held = true;
      } else {
        T2 zh[EP];
#pragma unroll
        for (int i = 0; i < EP / 2; ++i) {
          const T2 hp = hb[i * 64];
          zh[2 * i] = T2{hp.x, hz[2 * i]};
          zh[2 * i + 1] = T2{hp.y, hz[2 * i + 1]};
        }
        if (!(a.diag & 1)) fft1024_4x16x16<false>(zh, row, twm, tw3, t);
        hz_split_store(zh, rprev, r, t);
        held = false;
      }
    } else if constexpr (kR4Hz) {
      T2 zh[EP];
#pragma unroll
      for (int i = 0; i < EP; ++i) zh[i] = T2{hz[i], T(0)};
      if (!(a.diag & 1)) fft1024_4x16x16<false>(zh, row, twm, tw3, t);
      const T s2 = 2 * sc;  // (sc carries the 1/2 of the Hx / Hy split)
#pragma unroll
      for (int i = 0; i < MKO; ++i) {
        const int k = t + TPR * i;
        if (k < nkz && rv) zstore(2, zaddr(r, k), T2{zh[i].x * s2, zh[i].y * s2});
      }
    } else if constexpr (kHalf) {
      // H_z is real: z_m = Hz_2m + i Hz_2m+1 (scalar LDS stores, conflict-free), an N/2-point
      // transform, then Hz_k = E_k + W_N^k O_k (one N-point complex transform per row saved)
      T* rowf = reinterpret_cast<T*>(row);
#pragma unroll
      for (int i = 0; i < EP; ++i) {
        const int n = t + TPR * i;
        if (n < NZP) rowf[2 * fft_pidx_s<SH>(n >> 1) + (n & 1)] = hz[i];
      }
      row_sync<TPRF>();
      const T2* htw = twl + TS;
      if (!(a.diag & 1)) wave_fft_half<NZP, PITCH, false, TPRF, SH>(row, htw, ft);
      T2 z0[MKO] = {}, z1[MKO] = {}, wk[MKO] = {};
#pragma unroll
      for (int i = 0; i < MKO; ++i) {
        const int k = t + TPR * i;
        if (k < nkz) {
          z0[i] = row[fft_pidx_s<SH>(k)];
          z1[i] = row[fft_pidx_s<SH>((Hp::H - k) & (Hp::H - 1))];
          wk[i] = htw[k];
        }
      }
#pragma unroll
      for (int i = 0; i < MKO; ++i) {
        const int k = t + TPR * i;
        if (k < nkz && rv) {
          // 2E = Z_k + conj Z_{H-k}; 2O = (Z_k - conj Z_{H-k}) / i
          const T2 E2{z0[i].x + z1[i].x, z0[i].y - z1[i].y};
          const T2 O2{z0[i].y + z1[i].y, z1[i].x - z0[i].x};
          const T2 X = cadd(E2, cmul_tw<false>(O2, wk[i]));
          zstore(2, zaddr(r, k), T2{X.x * sc, X.y * sc});
        }
      }
    } else {
#pragma unroll
    for (int i = 0; i < EP; ++i) {
      const int n = t + TPR * i;
      if (n < NZP) row[fft_pidx(n)] = T2{hz[i], T(0)};
    }
    row_sync<TPRF>();
    if (!(a.diag & 1)) wave_fft<NZP, RWW, PITCH, false, TPRF>(frow, twl, ft);
    {
      T2 z0[MKO] = {}, z1[MKO] = {};
#pragma unroll
      for (int i = 0; i < MKO; ++i) {
        const int k = t + TPR * i;
        if (k < nkz) {
          z0[i] = row[fft_pidx(k)];
          z1[i] = row[fft_pidx(k == 0 ? 0 : NZP - k)];
        }
      }
#pragma unroll
      for (int i = 0; i < MKO; ++i) {
        const int k = t + TPR * i;
        if (k < nkz && rv) zstore(2, zaddr(r, k), T2{(z0[i].x + z1[i].x) * sc, (z0[i].y - z1[i].y) * sc});
      }
    }
    }
    row_sync<TPRF>();  // this row's last LDS reads precede the next row's writes
  }
  if constexpr (kPairHz) {
    // an odd count of rows: the last one's H_z alone (the (Hz, 0) transform, split as a pair)
    if (held) {
      int tl = threadIdx.x;
      asm volatile("" : "+v"(tl));
      t = tl % TPR;
      row = s + (tl / TPR) * PITCH;
      const T2* hb = hzbuf + (tl / TPR) * (EP / 2) * 64 + t;
      T2 zh[EP];
#pragma unroll
      for (int i = 0; i < EP / 2; ++i) {
        const T2 hp = hb[i * 64];
        zh[2 * i] = T2{hp.x, T(0)};
        zh[2 * i + 1] = T2{hp.y, T(0)};
      }
      if (!(a.diag & 1)) fft1024_4x16x16<false>(zh, row, twm, tw3, t);
      hz_split_store(zh, rprev, -1, t);
    }
  }
  // block maxima -> one atomicMax per block and quantity
  for (int o = 32; o >= 1; o >>= 1) {
    mu = fmaxf(mu, __shfl_xor(mu, o));
    mv = fmaxf(mv, __shfl_xor(mv, o));
    mw = fmaxf(mw, __shfl_xor(mw, o));
    mc = fmaxf(mc, __shfl_xor(mc, o));
  }
  if (lane == 0) {
    red[0][tid >> 6] = mu;
    red[1][tid >> 6] = mv;
    red[2][tid >> 6] = mw;
    red[3][tid >> 6] = mc;
  }
  __syncthreads();
  if (tid < 4 && a.maxima) {
    float m = 0.f;
    for (int i = 0; i < NWB; ++i) m = fmaxf(m, red[tid][i]);
    atomic_max_pos(&a.maxima[tid], m);
  }
}

// ---- register-resident z stage (NZP = 64 M, M = 16: the 1024-point rows of the headline grid) --
// The LDS-pass FFT above makes 4 LDS round trips per transform (gather, 3 Stockham passes) and is
// latency-bound at 2 waves/SIMD.  Here each transform is a four-step FFT N = M x 64 held in the
// wave's registers: lane k2 owns Z[k2 + 64 k1] (loaded straight from global memory, conjugate
// mirror included), an M-point DFT in registers, a twiddle, ONE LDS transpose, a 16-point DFT in
// registers, a twiddle and a 4-point DFT across the lanes of a quad (DPP quad_perm, no LDS).  The
// physical row stays in registers in the permuted order n = n1 + M (c + 16 br(a)), which is exactly
// the input order of the reverse network used for the forward transforms of H.
constexpr int kQuadXor1 = 0xB1;  // DPP quad_perm [1,0,3,2]
constexpr int kQuadXor2 = 0x4E;  // DPP quad_perm [2,3,0,1]
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(b & 0xffffffffll), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}
template <int CTRL, typename T2>
__device__ __forceinline__ T2 quad_swap(T2 v) {
  return T2{dpp_mov<CTRL>(v.x), dpp_mov<CTRL>(v.y)};
}
// one radix-2 stage across a lane pair: low lane a + b, high lane a - b (b = partner's value)
template <int CTRL, typename T2>
__device__ __forceinline__ T2 quad_bfly(T2 v, bool high) {
  using T = decltype(v.x);
  const T2 p = quad_swap<CTRL>(v);
  const T s = high ? T(-1) : T(1);
  return T2{p.x + s * v.x, p.y + s * v.y};
}
// natural order in (lane a of the quad holds y_a) -> lane a holds Y[br(a)] (br swaps 1 and 2)
template <bool INV, typename T2>
__device__ __forceinline__ T2 quad_dft4_nat_in(T2 v, int a) {
  v = quad_bfly<kQuadXor2>(v, (a & 2) != 0);
  if (a == 3) v = mul_mi<INV>(v);
  return quad_bfly<kQuadXor1>(v, (a & 1) != 0);
}
// bit-reversed order in (lane a holds y_br(a)) -> natural order out (lane a holds Y[a])
template <bool INV, typename T2>
__device__ __forceinline__ T2 quad_dft4_br_in(T2 v, int a) {
  v = quad_bfly<kQuadXor1>(v, (a & 1) != 0);
  if (a == 3) v = mul_mi<INV>(v);
  return quad_bfly<kQuadXor2>(v, (a & 2) != 0);
}
template <typename T2>
__device__ __forceinline__ T2 cmulc(T2 a, T2 w) {  // a * conj(w)
  return T2{a.x * w.x + a.y * w.y, a.y * w.x - a.x * w.y};
}

constexpr int kRegPitch = 68;  // transpose row pitch (64 + 4): conflict-free b64 column reads

// Inverse transform of one spectral row held as z[k1] = Z[lane + 64 k1] (unnormalised, +i sign);
// on return z[c] = x[n1 + M (c + 16 br(a))], lane = 4 g + a, n1 = g (M = 16).
// buf: this wave's M x kRegPitch transpose buffer; tw1: [M][64] W_N^(n1 k2); tw64: [4][16] W_64^(a c).
template <int M, typename T2>
__device__ __forceinline__ void reg_fft_inv(T2 (&z)[M], T2* buf, const T2* tw1, const T2* tw64, int lane) {
  static_assert(M == 16, "register z-stage FFT: M = 16 (N = 1024)");
  dft16<true>(z);  // over k1 -> n1
#pragma unroll
  for (int n1 = 1; n1 < M; ++n1) z[n1] = cmulc(z[n1], tw1[n1 * 64 + lane]);
#pragma unroll
  for (int n1 = 0; n1 < M; ++n1) buf[n1 * kRegPitch + lane] = z[n1];
  __builtin_amdgcn_wave_barrier();
  const int g = lane >> 2, a = lane & 3;
#pragma unroll
  for (int b = 0; b < 16; ++b) z[b] = buf[g * kRegPitch + a + 4 * b];
  __builtin_amdgcn_wave_barrier();
  dft16<true>(z);  // over b -> c
#pragma unroll
  for (int c = 1; c < 16; ++c)
    if (a != 0) z[c] = cmulc(z[c], tw64[a * 16 + c]);
#pragma unroll
  for (int c = 0; c < 16; ++c) z[c] = quad_dft4_nat_in<true>(z[c], a);
}

// Forward transform of a physical row in the register order produced by reg_fft_inv; on return
// z[k1] = Z[lane + 64 k1] (unnormalised, -i sign).
template <int M, typename T2>
__device__ __forceinline__ void reg_fft_fwd(T2 (&z)[M], T2* buf, const T2* tw1, const T2* tw64, int lane) {
  static_assert(M == 16, "register z-stage FFT: M = 16 (N = 1024)");
  const int g = lane >> 2, a = lane & 3;
#pragma unroll
  for (int c = 0; c < 16; ++c) z[c] = quad_dft4_br_in<false>(z[c], a);  // over d -> e = a
#pragma unroll
  for (int c = 1; c < 16; ++c)
    if (a != 0) z[c] = cmul(z[c], tw64[a * 16 + c]);
  dft16<false>(z);  // over c -> f
#pragma unroll
  for (int f = 0; f < 16; ++f) buf[g * kRegPitch + a + 4 * f] = z[f];
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int n1 = 0; n1 < M; ++n1) z[n1] = buf[n1 * kRegPitch + lane];
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int n1 = 1; n1 < M; ++n1) z[n1] = cmul(z[n1], tw1[n1 * 64 + lane]);
  dft16<false>(z);  // over n1 -> k1
}

template <int M, typename T, bool SEG>
__global__ void __launch_bounds__(256) zphys_reg_kernel(ZArgs a, typename C2<T>::type* fields,
                                                        const typename C2<T>::type* tw) {
  using T2 = typename C2<T>::type;
  constexpr int NZP = 64 * M;
  __shared__ T2 tbuf[ZW][M * kRegPitch];
  __shared__ T2 tws[NZP + 64];  // [M][64] W_N^(n1 k2), then [4][16] W_64^(a c)
  __shared__ float red[4][ZW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < NZP + 64; i += ZW * 64) tws[i] = tw[i];
  __syncthreads();
  const T2* tw1 = tws;
  const T2* tw64 = tws + NZP;
  T2* buf = tbuf[w];
  const long long nrows = static_cast<long long>(a.ny) * a.NX;
  const long long r = static_cast<long long>(blockIdx.x) * ZW + w;
  const int nkz = a.nkz;
  const long long fs = a.field_stride;
  float mu = 0.f, mv = 0.f, mw = 0.f, mc = 0.f;
  auto zaddr = [&](int k) -> long long {
    if constexpr (SEG) {
      const SegPos sp = seg_find(a.kz_start, a.off, a.nseg, k);
      return sp.off + r * sp.count + (k - sp.start);
    } else {
      return r * nkz + k;
    }
  };

  if (r < nrows) {  // wave-uniform
    T2 ph[3][M];
    // Only the retained half is loaded (slot i = mode lane + 64 i, i < M/2); the conjugate mirror
    // Z_{N-k} comes from lane 64 - lane (slot M-1-k1; lane 0: its own slot M-k1) by a lane
    // permute.  The loads of field pair p+1 are issued before the transform of pair p.
    constexpr int MH = M / 2;
    T2 la[2][MH], lb[2][MH];
    auto load_pair = [&](int p, T2 (&va)[MH], T2 (&vb)[MH]) {
      const T2* A = fields + (2 * p) * fs;
      const T2* B = fields + (2 * p + 1) * fs;
#pragma unroll
      for (int i = 0; i < MH; ++i) {
        const int k = lane + 64 * i;
        const bool ok = k < nkz;
        const long long o = ok ? zaddr(k) : 0;
        va[i] = ok ? A[o] : T2{0, 0};
        vb[i] = ok ? B[o] : T2{0, 0};
      }
    };
    load_pair(0, la[0], lb[0]);
    const int src = (64 - lane) & 63;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const int cur = p & 1;
      if (p < 2) load_pair(p + 1, la[cur ^ 1], lb[cur ^ 1]);
      // Z_k = A_k + i B_k (k < nkz), Z_{N-k} = conj(A_k) + i conj(B_k); kz = 0 imaginary parts dropped
#pragma unroll
      for (int k1 = 0; k1 < MH; ++k1) {
        const T2 A = la[cur][k1], B = lb[cur][k1];
        ph[p][k1] = (lane == 0 && k1 == 0) ? T2{A.x, B.x} : T2{A.x - B.y, A.y + B.x};
      }
#pragma unroll
      for (int k1 = MH; k1 < M; ++k1) {
        T2 A{__shfl(la[cur][M - 1 - k1].x, src), __shfl(la[cur][M - 1 - k1].y, src)};
        T2 B{__shfl(lb[cur][M - 1 - k1].x, src), __shfl(lb[cur][M - 1 - k1].y, src)};
        if (lane == 0) {  // N - k = 64 (M - k1): own slot M - k1 (k1 = M/2 is the Nyquist mode: zero)
          A = k1 > MH ? la[cur][(M - k1) % MH] : T2{0, 0};
          B = k1 > MH ? lb[cur][(M - k1) % MH] : T2{0, 0};
        }
        ph[p][k1] = T2{A.x + B.y, B.x - A.y};
      }
      if (!(a.diag & 1)) reg_fft_inv<M>(ph[p], buf, tw1, tw64, lane);
    }
    // rotational product H = u x omega (convolution_kernels.cu:125-131) and CFL maxima
    const int yl = static_cast<int>(r / a.NX);
    const float idy = static_cast<float>(a.inv_dy[a.y0 + yl]);
    // (the CFL sum in fp32: a double kx_max promoted every point's sum to fp64, 2 cvt + 2 FMA64 per point)
    const float cxf = static_cast<float>(a.cx), czf = static_cast<float>(a.cz);
    T2 hxy[M], hz[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const T u = ph[0][i].x, v = ph[0][i].y, ww = ph[1][i].x, wx = ph[1][i].y, wy = ph[2][i].x, wz = ph[2][i].y;
      hxy[i] = T2{v * wz - ww * wy, ww * wx - u * wz};
      hz[i] = T2{u * wy - v * wx, T(0)};
      const float au = fabsf(static_cast<float>(u)), av = fabsf(static_cast<float>(v)), aw = fabsf(static_cast<float>(ww));
      mu = fmaxf(mu, au);
      mv = fmaxf(mv, av);
      mw = fmaxf(mw, aw);
      mc = fmaxf(mc, au * cxf + av * idy + aw * czf);
    }
    if (!(a.diag & 1)) {
      reg_fft_fwd<M>(hxy, buf, tw1, tw64, lane);
      reg_fft_fwd<M>(hz, buf, tw1, tw64, lane);
    }
    // (Hx + i Hy)^_k = Z_k: Hx_k = (Z_k + conj Z_{N-k})/2, Hy_k = (Z_k - conj Z_{N-k})/(2i); Z_{N-k}
    // lives in lane 64 - lane at k1' = M-1-k1 (lane 0: its own k1' = M - k1)
    const T sc = static_cast<T>(0.5 * a.scale), sz = static_cast<T>(a.scale);
    constexpr int MKO = (NZP / 2 + 63) / 64;
#pragma unroll
    for (int k1 = 0; k1 < MKO; ++k1) {
      const int k = lane + 64 * k1;
      const int src = (64 - lane) & 63;
      T2 zm{__shfl(hxy[M - 1 - k1].x, src), __shfl(hxy[M - 1 - k1].y, src)};
      if (lane == 0) zm = hxy[(M - k1) % M];
      if (k < nkz) {
        const T2 Z = hxy[k1];
        const long long o = zaddr(k);
        fields[0 * fs + o] = T2{(Z.x + zm.x) * sc, (Z.y - zm.y) * sc};
        fields[1 * fs + o] = T2{(Z.y + zm.y) * sc, -(Z.x - zm.x) * sc};
        fields[2 * fs + o] = T2{hz[k1].x * sz, hz[k1].y * sz};
      }
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    mu = fmaxf(mu, __shfl_xor(mu, o));
    mv = fmaxf(mv, __shfl_xor(mv, o));
    mw = fmaxf(mw, __shfl_xor(mw, o));
    mc = fmaxf(mc, __shfl_xor(mc, o));
  }
  if (lane == 0) {
    red[0][w] = mu;
    red[1][w] = mv;
    red[2][w] = mw;
    red[3][w] = mc;
  }
  __syncthreads();
  if (tid < 4 && a.maxima) {
    float m = 0.f;
    for (int i = 0; i < ZW; ++i) m = fmaxf(m, red[tid][i]);
    atomic_max_pos(&a.maxima[tid], m);
  }
}

// CHANNEL_ZREG=1 selects the register-resident z stage at Nzp = 1024.  Measured at 1024x385x1024
// fp32 (r2p): 3.5x fewer LDS instructions than the LDS-pass kernel but +17 % VALU and +65 %
// wave-parked cycles (one transpose wait + per-FFT twiddle reads per transform at 2 waves/SIMD):
// 51.2 vs 50.0 ms/step, so the LDS-pass kernel stays the default.
inline bool zreg_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("CHANNEL_ZREG");
    return e && std::atoi(e) != 0;
  }();
  return on;
}

// CHANNEL_ZFFT = 0 | 1 | 2 | 3 | 4: the 1024-point fp32 z-stage row transforms (zphys_kernel ZF, A/B).
// Default 3 (4 x 16 x 16 for all five transforms of a row); measured per 8-plane chunk alone at
// 1024x385x1024: 60.9 / 58.5 / 57.9 / 56.9 us, bench 33.13 (ZF 1) / 32.97 / 32.79 ms/step
// (gpurun_out/g10_*, profiles/r05/zfft_ab.txt)
inline int zfft_mode() {
  static const int v = [] {
    const char* e = std::getenv("CHANNEL_ZFFT");
    return e ? std::atoi(e) : 3;
  }();
  return v;
}

// CHANNEL_ZHALF=0: H_z through a full-length complex transform (A/B of the half-length path)
inline bool zhalf_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("CHANNEL_ZHALF");
    return !e || std::atoi(e) != 0;
  }();
  return on;
}

// CHANNEL_ZPERS=0: one-shot z-stage grid (one row group per block) instead of the persistent one (A/B)
inline bool zpers_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("CHANNEL_ZPERS");
    return !e || std::atoi(e) != 0;
  }();
  return on;
}

template <int NN, typename T, int TPR, int WPE = 2>
static void zphys_launch_tpr(const ZArgs& a, void* fields, const Twiddles& tw, hipStream_t s, bool zh) {
  using T2 = typename C2<T>::type;
  constexpr int ZR = zphys_rows<NN, T, TPR>();
  const long long nrows = static_cast<long long>(a.ny) * a.NX;
  // (one segment with 32-bit byte offsets when a field's rows fit 4 GiB; the segment path otherwise)
  const bool seg = a.nseg > 1 || a.nkz != NN / 3 + 1 ||
                   static_cast<unsigned long long>(nrows) * a.nkz * sizeof(T2) >= (1ull << 32);
  auto kern = seg ? (zh ? zphys_kernel<NN, T, true, true, TPR, ZR, WPE> : zphys_kernel<NN, T, true, false, TPR, ZR, WPE>)
                  : (zh ? zphys_kernel<NN, T, false, true, TPR, ZR, WPE> : zphys_kernel<NN, T, false, false, TPR, ZR, WPE>);
  if constexpr (sizeof(T) == 4 && NN == 1024 && TPR == 64 && WPE == 2) {
    const int zf = zfft_mode();
    if (!seg && zh && zf == 0) kern = zphys_kernel<NN, T, false, true, TPR, ZR, WPE, 0>;
    if (!seg && zh && zf == 1) kern = zphys_kernel<NN, T, false, true, TPR, ZR, WPE, 1>;
    if (!seg && zh && zf == 2) kern = zphys_kernel<NN, T, false, true, TPR, ZR, WPE, 2>;
    if (!seg && zh && zf == 4) kern = zphys_kernel<NN, T, false, true, TPR, ZR, WPE, 4>;
  }
  const long long ngroups = (nrows + ZR - 1) / ZR;
  const long long cap = zpers_enabled() ? persist_blocks(reinterpret_cast<const void*>(kern), ZR * TPR, "CHANNEL_Z_BPC") : ngroups;
  dim3 grid(static_cast<unsigned>(std::min(ngroups, cap)));
  CH_CHECK(a.nkz <= NN / 3 + 1, "zphys: more retained kz than the 2/3 rule allows");
  CH_CHECK(TPR < 64 || nrows % ZR == 0, "zphys: rows per plane must be a multiple of the rows per block");
  hipLaunchKernelGGL(kern, grid, dim3(ZR * TPR), 0, s, a, static_cast<T2*>(fields), static_cast<const T2*>(tw.buf));
}

// CHANNEL_ZTPR=64|128: threads per 1024-point fp32 row (A/B; see zphys_tpr for the default).  Two
// waves per row take 152 instead of 218 VGPRs (3 waves/SIMD) but pay a block barrier per pass:
// measured 48.8 vs 46.3 ms/step on the headline grid, so one wave per row stays the default.
// CHANNEL_ZWPE=3: the one-wave-per-row 1024-point fp32 kernel compiled for 3 waves per SIMD (168
// VGPRs, ~20 spilled) instead of 2 (216 VGPRs, no spills) (A/B).  Measured on the headline grid,
// same box, alternating: 47.4 vs 45.5 ms/step, so 2 waves per SIMD without spills stays the default
inline int zwpe_env() {
  static const int v = [] {
    const char* e = std::getenv("CHANNEL_ZWPE");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}
inline int ztpr_env() {
  static const int v = [] {
    const char* e = std::getenv("CHANNEL_ZTPR");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

// ---- standalone batched C2C (tests) ----------------------------------------------------------
template <int N, typename T, bool INV>
__global__ void __launch_bounds__(256) fft_test_kernel(typename C2<T>::type* data, int batch,
                                                       const typename C2<T>::type* tw) {
  using T2 = typename C2<T>::type;
  constexpr int PITCH = FftPitch<N>::value;
  __shared__ T2 s[4 * PITCH];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long rw = static_cast<long long>(blockIdx.x) * 4 + w;
  if (rw >= batch) return;  // wave-uniform; no block barriers below
  T2* row = s + w * PITCH;
  for (int x = lane; x < N; x += 64) row[fft_pidx(x)] = data[rw * N + x];
  __builtin_amdgcn_wave_barrier();
  wave_fft<N, 1, PITCH, INV>(row, tw, lane);
  for (int x = lane; x < N; x += 64) data[rw * N + x] = row[fft_pidx(x)];
}

// ---- per-length entry points (instantiated by the length-family translation units) ----------
template <int NN>
void fft_xb_len(const XArgs& a, const XSrc& src, void* phys, const Twiddles& tw, bool fp64, hipStream_t s) {
  if (fp64) {
    xb_launch_cfg<NN, double, 0>(a, src, phys, tw, s);
  } else if constexpr (NN == 512 || NN == 1024) {
    if (xwide_enabled() || ((a.kzb || a.segblk) && xplanes_enabled())) xb_launch_cfg<NN, float, 1>(a, src, phys, tw, s);
    else xb_launch_cfg<NN, float, 0>(a, src, phys, tw, s);
  } else {
    xb_launch_cfg<NN, float, 0>(a, src, phys, tw, s);
  }
}
template <int NN>
void fft_xf_len(const XArgs& a, const void* phys, const XDst& dst, const Twiddles& tw, bool fp64, hipStream_t s) {
  if (fp64) {
    xf_launch_cfg<NN, double, 0>(a, phys, dst, tw, s);
  } else if constexpr (NN == 512 || NN == 1024) {
    if (xwide_enabled() || ((a.kzb || a.segblk) && xplanes_enabled())) xf_launch_cfg<NN, float, 1>(a, phys, dst, tw, s);
    else xf_launch_cfg<NN, float, 0>(a, phys, dst, tw, s);
  } else {
    xf_launch_cfg<NN, float, 0>(a, phys, dst, tw, s);
  }
}
template <int NN, typename T>
void fft_zp_len_t(const ZArgs& a, void* fields, const Twiddles& tw, hipStream_t s) {
  const bool zh = zhalf_enabled();
  constexpr int DEF = zphys_tpr<NN>(sizeof(T));
  if constexpr (sizeof(T) == 4 && NN == 1024) {
    constexpr int ALT = DEF == 64 ? 128 : 64;
    if (ztpr_env() == ALT) zphys_launch_tpr<NN, T, ALT>(a, fields, tw, s, zh);
    else if (DEF == 64 && zwpe_env() == 3) zphys_launch_tpr<NN, T, DEF, 3>(a, fields, tw, s, zh);
    else zphys_launch_tpr<NN, T, DEF>(a, fields, tw, s, zh);
  } else {
    zphys_launch_tpr<NN, T, DEF>(a, fields, tw, s, zh);
  }
}
template <int NN>
void fft_zp_len(const ZArgs& a, void* fields, const Twiddles& tw, bool fp64, hipStream_t s) {
  if (fp64) fft_zp_len_t<NN, double>(a, fields, tw, s);
  else fft_zp_len_t<NN, float>(a, fields, tw, s);
}
template <int NN>
void fft_test_len(void* data, int batch, int dir, const Twiddles& tw, bool fp64, hipStream_t s) {
  dim3 grid((batch + 3) / 4);
  if (fp64) {
    if (dir > 0) hipLaunchKernelGGL((fft_test_kernel<NN, double, true>), grid, dim3(256), 0, s, static_cast<double2*>(data), batch, static_cast<const double2*>(tw.buf));
    else hipLaunchKernelGGL((fft_test_kernel<NN, double, false>), grid, dim3(256), 0, s, static_cast<double2*>(data), batch, static_cast<const double2*>(tw.buf));
  } else {
    if (dir > 0) hipLaunchKernelGGL((fft_test_kernel<NN, float, true>), grid, dim3(256), 0, s, static_cast<float2*>(data), batch, static_cast<const float2*>(tw.buf));
    else hipLaunchKernelGGL((fft_test_kernel<NN, float, false>), grid, dim3(256), 0, s, static_cast<float2*>(data), batch, static_cast<const float2*>(tw.buf));
  }
}

// the lengths with kernels: 2^k (16..2048), 3*2^k (48..1536), 5*2^k (80..1280), 7*2^k (112..1792),
// 9*2^k (144..1152), 15*2^k (240..1920), 11*2^k (176..1408), 13*2^k (208..1664)
#define CH_FFT_POW2_LENGTHS(X) X(16) X(32) X(64) X(128) X(256) X(512) X(1024) X(2048)
#define CH_FFT_R3_LENGTHS(X) X(48) X(96) X(192) X(384) X(768) X(1536)
#define CH_FFT_R5_LENGTHS(X) X(80) X(160) X(320) X(640) X(1280)
#define CH_FFT_R7_LENGTHS(X) X(112) X(224) X(448) X(896) X(1792)
#define CH_FFT_R9_LENGTHS(X) X(144) X(288) X(576) X(1152)
#define CH_FFT_R15_LENGTHS(X) X(240) X(480) X(960) X(1920)
#define CH_FFT_R11_LENGTHS(X) X(176) X(352) X(704) X(1408)
#define CH_FFT_R13_LENGTHS(X) X(208) X(416) X(832) X(1664)
#define CH_FFT_INSTANTIATE(NN)                                                                              \
  template void fft_xb_len<NN>(const XArgs&, const XSrc&, void*, const Twiddles&, bool, hipStream_t);      \
  template void fft_xf_len<NN>(const XArgs&, const void*, const XDst&, const Twiddles&, bool, hipStream_t); \
  template void fft_zp_len<NN>(const ZArgs&, void*, const Twiddles&, bool, hipStream_t);                    \
  template void fft_test_len<NN>(void*, int, int, const Twiddles&, bool, hipStream_t);
// (extern declarations per entry point: an extern template covers one declaration)
#define CH_FFT_EXTERN_ALL(NN)                                                                                   \
  extern template void fft_xb_len<NN>(const XArgs&, const XSrc&, void*, const Twiddles&, bool, hipStream_t);      \
  extern template void fft_xf_len<NN>(const XArgs&, const void*, const XDst&, const Twiddles&, bool, hipStream_t); \
  extern template void fft_zp_len<NN>(const ZArgs&, void*, const Twiddles&, bool, hipStream_t);                    \
  extern template void fft_test_len<NN>(void*, int, int, const Twiddles&, bool, hipStream_t);
CH_FFT_POW2_LENGTHS(CH_FFT_EXTERN_ALL)
CH_FFT_R3_LENGTHS(CH_FFT_EXTERN_ALL)
CH_FFT_R5_LENGTHS(CH_FFT_EXTERN_ALL)
CH_FFT_R7_LENGTHS(CH_FFT_EXTERN_ALL)
CH_FFT_R9_LENGTHS(CH_FFT_EXTERN_ALL)
CH_FFT_R15_LENGTHS(CH_FFT_EXTERN_ALL)
CH_FFT_R11_LENGTHS(CH_FFT_EXTERN_ALL)
CH_FFT_R13_LENGTHS(CH_FFT_EXTERN_ALL)

}  // namespace channel
