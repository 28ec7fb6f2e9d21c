// Host-side launchers for the HIP kernels (implemented in csrc/kernels/*.hip).
#pragma once

#include <string>

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "channel/grid.hpp"
#include "channel/yline_device.hpp"

namespace channel {

// R values the y-line kernels are instantiated for (64*R >= NY).
int yline_supported_R(int NY);
// K-SPEC line geometry for NY: R rows per lane on H waves per line.  Default H = 1 (one wave per
// line, 64 R >= NY); CHANNEL_KSPEC_HALVES=1 opts in to lines over two waves (H = 2, 64 R H >= NY),
// measured slower at the headline grid and checked against the oracle by
// tests/test_solver_gpu.py::test_kspec_halves_matches_oracle
void kspec_geometry(int NY, bool fp64, int& R, int& H);

// Device copies of the per-row coefficient tables (lane-major, see yline_device.hpp).  H = 2: row
// j = h 64R + lane R + r of half h at index (h R + r) 64 + lane (a half's table is the one-wave
// table of its rows), the D1 factorisation per half, and the halves' D1 spikes.
struct YTablesDev {
  double* buf = nullptr;     // single allocation
  size_t bytes = 0;
  dev::YTab tab{};
  int R = 1, H = 1;
  void upload(const YGrid& g, int R, hipStream_t stream, int H = 1);
  void release();
  ~YTablesDev() { release(); }
};

// Debug/test entry point: apply one y-line operator to `lines` complex lines stored [y][line].
enum YLineOp : int {
  YOP_D1 = 0,        // out = D1 in (compact first derivative)
  YOP_HELM = 1,      // out = (K - k^2 M)^{-1} M in, out(+-1) = 0 (velocity recovery)
  YOP_IMPL = 2,      // out = ((1+c k^2) M - c K)^{-1} M in, out(+-1)=0 (implicit viscous step)
  YOP_MAPPLY = 3,    // out = M in (interior rows, 0 on walls)
  YOP_KAPPLY = 4,    // out = K in (interior rows, 0 on walls)
};
void yline_test(const YTablesDev& t, int op, const void* in, void* out, int lines, const double* k2, double c,
                bool fp64, hipStream_t stream);

// Dense D1 = A1^-1 B1 (NY <= 192) applied to [y][line] complex fp64 lines on the matrix cores
// (yline_mfma.hip): the measured MFMA alternative to the PCR D1 solve.
struct DenseD1Dev {
  double* d = nullptr;  // [NP][NP] row-major, zero-padded
  int N = 0, NP = 0;
  void upload(const YGrid& g, hipStream_t stream);
  void release();
  ~DenseD1Dev() { release(); }
};
void d1_dense_mfma(const DenseD1Dev& m, const void* in, void* out, int lines, hipStream_t stream);

// ---- spectral field layout ----------------------------------------------------------------------
// Element (y, line) of a spectral field, line = local kx * nkzs + local kz (nkzs: the kz line
// stride), lines = nkx_loc * nkzs.  kzb = 0: [y][line], every y plane contiguous (the exchange
// blocks of P > 1 are row ranges).  kzb = 8 (one rank, nkzs a multiple of 8, rows padded to a
// multiple of 8): tiles of 8 planes x 8 kz lines, [y / 8][line / 8][y % 8][line % 8], i.e. a 512-B
// (fp32) piece per (8-plane chunk, kz block).  The spectral fields are read in two shapes: K-SPEC
// tiles (4 lines x all y: 49 such pieces instead of 385 rows of 32 B, 1.9 MB apart) and the
// x transforms (2 planes x 8 kz x all kx: 128-B lines, the kx rows of one chunk 22 KB apart);
// tools/tilebench.hip: K-SPEC's pattern 2.5 -> 4.2 TB/s blocked.  Blocking all NY rows of a kz
// block instead ([kz/8][kx][y][8]) gave K-SPEC whole-tile contiguity but spread an x tile over
// 16.8 MB and the chunk's tiles over the whole field: the x-backward's average read latency rose
// from 950 to 1670 cycles (TCP_TCC_READ_REQ_LATENCY, gpurun_out/r4g*), 62 -> 71 us per chunk.
// Row and line parts of the offset are separable: offset = spec_row_off(y) + spec_line_off(line),
// and spec_row_off(y + 64) = spec_row_off(y) + 64 lines in both layouts.
constexpr int kSpecKzBlock = 8, kSpecYBlock = 8;
__host__ __device__ inline size_t spec_row_off(int kzb, int lines, int y) {
  return kzb ? static_cast<size_t>(y / kSpecYBlock) * kSpecYBlock * lines + (y % kSpecYBlock) * kSpecKzBlock
             : static_cast<size_t>(y) * lines;
}
__host__ __device__ inline size_t spec_line_off(int kzb, int line) {
  return kzb ? static_cast<size_t>(line / kSpecKzBlock) * (kSpecYBlock * kSpecKzBlock) + line % kSpecKzBlock
             : static_cast<size_t>(line);
}
__host__ __device__ inline size_t spec_index(int kzb, int nkx, int nkzs, int y, int ikx, int kz) {
  return spec_row_off(kzb, nkx * nkzs, y) + spec_line_off(kzb, ikx * nkzs + kz);
}
// rows allocated per spectral field (kzb: whole 8-plane chunks)
__host__ __device__ inline int spec_rows(int kzb, int N) { return kzb ? (N + kSpecYBlock - 1) / kSpecYBlock * kSpecYBlock : N; }

// ---- the fused spectral (y-line) substep kernel ---------------------------------------------
struct SpecArgs {
  // geometry
  int N = 0;              // NY
  int lines = 0;          // local lines = nkx_loc * nkz, line = ikx_local * nkz + kz
  int nkz = 0, kx0 = 0, nkx = 0, Kx = 0;   // nkz = local kz line stride (pencil: a kz range; kzb: padded to 8)
  int kzb = 0;            // spectral layout (spec_index)
  int kz0 = 0;            // first local kz (pencil)
  double ax = 1, az = 2;  // 2 pi / LX, 2 pi / LZ
  double nu = 1.0 / 3250.0;
  // RK3 substep (mode 1)
  int mode = 0;           // 0 = prepare only (fields from state), 1 = advance + prepare
  double rk_a = 0, rk_b = 0, rk_g = 0, rk_z = 0;
  const double* dt = nullptr;   // device scalar
  // mean flow forcing
  double Q = 1.8;
  int forcing = 0;        // 0 implicit (exact flux), 1 parity (constant add)
  // reference-parity switches (config influence / explicit_d2; every NY)
  bool explicit_dd = false;          // explicit viscous D2 = D1 o D1
  bool analytic_influence = false;   // cosh/sinh influence functions
  const double* ygrid = nullptr;     // [N] y_j (analytic influence)
  // fields (T2* cast to void*)
  void* phi = nullptr;
  void* omega = nullptr;  // line (0,0) holds U(y)
  void* Rphi = nullptr;
  void* Romega = nullptr;
  void* out[6] = {};      // out6 = 1: u, v, w, omega_x, -, omega_z (out[4] == omega: the state is the
                          // omega_y source, the x-backward zeroes its mean line); out6 = 0 (the
                          // combine mode of P > 1): D1 v, v, D1 omega in out[0..2], out[3], out[5]
                          // unused (XArgs::combine forms u, w, omega_x, omega_z from D1 v, omega,
                          // phi, D1 omega).  out[0..2] double as the H_x, H_y, H_z inputs.
  int out6 = 1;
  int store_r = 1;        // 0: skip the R_phi/R_omega stores (last substep: the next one has zeta = 0)
  int lds_poison = 0;     // debug: fill the LDS with NaN before use (CHANNEL_LDS_POISON)
  // diagnostics
  double* stats = nullptr;   // [4][N] plane sums (uu, vv, ww, uv) when non-null
  double* mean_diag = nullptr;  // [3N + 8]: U, Nx, dU/dy(walls), flux, pressure gradient ...
  unsigned* health = nullptr;   // bit 0: non-finite state
  unsigned long long* prof = nullptr;  // [kKspecPhases] shader-clock sums per phase (debug, CHANNEL_KSPEC_PROF)
};
constexpr int kKspecPhases = 10;
void kspec_launch(const YTablesDev& t, const SpecArgs& a, bool fp64, hipStream_t stream);

// ---- FFT stages ---------------------------------------------------------------------------
// Per-pass FFT twiddle tables for length n (FftPlan T1/T2 layout, fft_device.hpp), fp32 or fp64.
struct Twiddles {
  void* buf = nullptr;
  void* reg = nullptr;  // n = 1024: [M][64] W_N^(n1 k2), [4][16] W_64^(a c) of the register z stage
  int n = 0;
  bool fp64 = false;
  void build(int n, bool fp64);
  void release();
  ~Twiddles() { release(); }
};
// Source of a spectral field for the backward x-transform: for P ranks the blocks received from
// each source rank s hold [y_local][nkx_s][nkz] starting at element offset off[s].
// Blocks self_seg .. self_seg + nself - 1 (this rank's own kx range, if self_seg >= 0; several when
// the rank's spectral fields are stored as kx sub-blocks, Solver::nkb_) live at self_base + f *
// self_field_stride + off[s] instead (the spectral field itself: no self exchange, no copy).
// exchange segments of the x transforms: P ranks x kx sub-blocks (slab8 with 2 sub-blocks: 16)
constexpr int kMaxSeg = 16;
struct XSrc {
  const void* base = nullptr;
  // combine mode (XArgs::combine): input field j (0 D1 v, 1 v, 2 D1 omega, 3 omega, 4 phi) at fld[j]
  // (the exchange blocks or the spectral field: base is unused) and its self blocks at self_fld[j]
  const void* fld[5] = {};
  const void* self_fld[5] = {};
  int nsrc = 1;
  int kx_start[kMaxSeg + 1] = {0};   // global retained-kx start of source s (kx_start[nsrc] = nkx)
  long long off[kMaxSeg] = {0};      // element offset of source block s
  int self_seg = -1;
  int nself = 1;
  const void* self_base = nullptr;
  long long self_field_stride = 0;
  // per-row table of the exchange segments (row-table modes, optional): for each retained kx row i,
  // rowtab[2 i] = element offset of row i at segment row Y = 0 of the FIRST chunk (y0 = 0),
  // rowtab[2 i + 1] = its segment's Y stride | 0x80000000 for a self block.  Chunk rows then add
  // XArgs::seg_y0 to Y.  Built once per run on the host (Solver::build_rowtab) instead of per launch.
  const unsigned* rowtab = nullptr;
};
struct XDst {             // destination blocks for the forward x-transform (per destination rank)
  void* base = nullptr;
  int ndst = 1;
  int kx_start[kMaxSeg + 1] = {0};
  long long off[kMaxSeg] = {0};
  int self_seg = -1;
  int nself = 1;
  void* self_base = nullptr;
  long long self_field_stride = 0;
  const unsigned* rowtab = nullptr;  // as XSrc::rowtab
};

struct XArgs {
  int NX = 0, nkx = 0, Kx = 0, nkz = 0, ny = 0;   // ny = local y planes, nkz = local kz count
  int nfields = 1;
  long long field_stride_spec = 0;   // element stride between fields in the spectral buffers
  long long field_stride_phys = 0;   // element stride between fields in the physical buffers
  // x-expanded buffer blocked by x range (pencil B exchange): x in [x_start[d], x_start[d+1]) lives
  // at poff[d] + (y * nx_d + x - x_start[d]) * nkz.  One segment = plain [y][x][kz].
  int npseg = 1;
  int x_start[9] = {0};
  long long poff[8] = {0};
  int diag = 0;                      // bit 0: skip the transforms (timing diagnosis, CHANNEL_FFT_DIAG)
  // backward only: field zero_mean_field's (kx = 0, kz = 0) element is read as 0 (omega_y: the
  // spectral source is the omega state, whose mean line holds U(y)); kz_glob0 = global kz of local
  // kz 0 (pencil rows)
  int zero_mean_field = -1;
  int kz_glob0 = 0;
  int lds_poison = 0;                // debug: fill the LDS with NaN before use
  // blocked spectral layout (one rank, one source block; spec_index with kzb = 8): rows spec_y0 ..
  // spec_y0 + ny - 1 of fields of line stride nkzs (lines = nkx * nkzs)
  int kzb = 0, nkzs = 0, spec_y0 = 0;
  // P > 1: the exchange segments and self blocks hold the blocked layout too (spec_index with
  // kzb = 8 within each segment: [y/8][line/8][y%8][line%8], line = kx in segment * nkzs + kz;
  // chunk rows start on 8-plane tiles).  fft_impl.hpp seg_yk / seg_stride
  int segblk = 0;
  int seg_y0 = 0;                    // with XSrc / XDst::rowtab: the chunk's first segment row Y
  int seg_yoff = 0;                  // rows of the exchange chunk before this launch's first row (the
                                     // second part of a chunk split over two compute streams)
  int nt = 0;                        // streaming (non-temporal) spectral accesses (solver default 1;
                                     // CHANNEL_XNT=0 off: 35.0 vs 34.75 ms/step, profiles/r04/ab_xnt.txt)
  // backward only: combine mode -- the six output fields u, v, w, omega_x, omega_y, omega_z are
  // formed per element from the five inputs XSrc::fld (D1 v, v, D1 omega, omega, phi; fft_impl.hpp
  // cmb_pair); ax, az = 2 pi / LX, 2 pi / LZ (the kx of retained row i, the kz of kz_glob0 + kz)
  int combine = 0;
  double ax = 1.0, az = 2.0;
};
// backward: spectral (truncated kx) -> [y][x][kz] complex, zero padding kx
void xfft_backward(const XArgs& a, const XSrc& src, void* phys, const Twiddles& tw, bool fp64, hipStream_t s);
// forward: [y][x][kz] -> spectral truncated kx (unnormalised)
void xfft_forward(const XArgs& a, const void* phys, const XDst& dst, const Twiddles& tw, bool fp64, hipStream_t s);
// template arguments of this thread's last x-transform launch, in rocprofv3's kernel-name form (tests)
std::string xfft_last_variant();
// the same for this thread's last x-backward launch (a solver step ends with forward transforms)
std::string xfft_last_backward_variant();

struct ZArgs {
  int NX = 0, Nzp = 0, nkz = 0, ny = 0, y0 = 0;   // NX = local x count (rows = ny * NX)
  // rows blocked by kz range (pencil B exchange): kz in [kz_start[s], kz_start[s+1]) of row r lives
  // at off[s] + r * nkz_s + kz - kz_start[s].  One segment = plain [row][kz].
  int nseg = 1;
  int kz_start[9] = {0};
  long long off[8] = {0};
  int diag = 0;                      // bit 0: skip the transforms (timing diagnosis)
  long long field_stride = 0;        // element stride between the 6 input fields
  double scale = 1.0;                // forward normalisation 1/(NX*Nzp)
  const double* inv_dy = nullptr;    // [NY] 1/local spacing for the CFL estimate
  double cx = 0, cz = 0;             // kx_max, kz_max for the CFL estimate
  float* maxima = nullptr;           // [4]: |u|max, |v|max, |w|max, cfl sum max (atomicMax)
  int lds_poison = 0;                // debug: fill the LDS with NaN before use
};
// physical-space stage: 6 fields (u,v,w,wx,wy,wz) [y][x][kz] -> z C2R -> H = u x omega -> z R2C
// -> truncated H_x,H_y,H_z written in place over fields 0..2.
void zphys(const ZArgs& a, void* fields, const Twiddles& tw, bool fp64, hipStream_t s);

// standalone FFT entry points for tests: batched C2C along the contiguous axis
void fft_c2c_test(void* data, int n, int batch, int dir, const Twiddles& tw, bool fp64, hipStream_t s);

// ---- small kernels ---------------------------------------------------------------------------
struct DtArgs {
  float* maxima = nullptr;   // [4] from zphys; reset to 0 after use
  double* dt = nullptr;      // output dt (device)
  double* time = nullptr;    // accumulated time (device)
  double* dt_log = nullptr;  // [8]: umax vmax wmax cflsum dt_c dt_v dt ...
  unsigned* health = nullptr;  // bit 1 set on non-finite CFL maxima or dt collapse
  double cfl = 0.5, dt_max = 0.05, dt_fixed = 0.0;
  int parity = 0;
  double NX = 0, NZ = 0, LX = 0, LZ = 0, Re = 0, dy_uniform = 0;
};
void dt_update(const DtArgs& a, hipStream_t s);

// kz=0 plane Hermitian symmetrisation of a [y][nkx][nkz] field held entirely by one rank
void symmetrize_kz0(void* q, int N, int nkx, int nkzs, int Kx, int kzb, bool fp64, hipStream_t s);
// distributed version: pack the local kz=0 column [y][kx_loc], exchange, symmetrise from the
// gathered columns (blocks [c][y][nkx_c] of the ranks of this process row)
struct Kz0SymArgs {
  int N = 0, nkx_loc = 0, nkz_loc = 0, kx0 = 0, nkx = 0;
  int kzb = 0;  // spectral layout of q (spec_index; nkz_loc is then the padded line stride nkzs)
  int nblk = 1;
  int kx_start[kMaxSeg + 1] = {0};
};
void kz0_pack(const void* q, void* col, int N, int nkx_loc, int nkz_loc, int kzb, bool fp64, hipStream_t s);
void kz0_symmetrize_dist(void* q, const void* col_all, const Kz0SymArgs& a, bool fp64, hipStream_t s);

// ---- diagnostics ---------------------------------------------------------------------------
struct SpectraArgs {
  // spectral [NY][lines] fields, lines = nkx_loc*nkz_loc: the K-SPEC outputs D1 v, v and the omega
  // state; u = i (al D1v - be om)/k2 and w = i (be D1v + al om)/k2 are formed per element
  const void *dv = nullptr, *v = nullptr, *om = nullptr;
  double ax = 1.0, az = 2.0;
  // combine = 0 (K-SPEC's six-output mode): u and w are stored fields themselves
  int combine = 1;
  const void *u = nullptr, *w = nullptr;
  int lines = 0, nkx_loc = 0, kx0 = 0, nkz_loc = 0, kz0 = 0;
  int nkzs = 0, kzb = 0;              // line stride in kz, layout (spec_index)
  int nkx = 0, Kx = 0, nkz = 0;       // global retained counts
  const int* planes = nullptr;        // device [nplanes] y indices
  int nplanes = 0;
  double* ekx = nullptr;              // [3][nplanes][Kx+1]  (|kx| bins, summed over kz)
  double* ekz = nullptr;              // [3][nplanes][nkz]   (summed over kx)
  double* map = nullptr;              // [3][nkx][nkz] |q|^2 at planes[0] (may be null)
};
// accumulates (+=) into ekx/ekz; map is overwritten for the local block
void spectra_accumulate(const SpectraArgs& a, bool fp64, hipStream_t s);
// fault injection (tests): element `elem` of a complex field becomes NaN
void inject_nan(void* field, size_t elem, bool fp64, hipStream_t s);

}  // namespace channel
