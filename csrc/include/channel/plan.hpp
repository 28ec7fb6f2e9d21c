// Decomposition plan: retained-mode sets, slab split tables and local buffer sizes.
//
// Reference: 1-D slab, spectral kx-slabs of NX/P planes and physical y-slabs of NY/P planes
// (channel.h:71-76), valid only for NX==NY, NY%P==0, NX/P%64==0.
// Here:
//  * only the 2/3-rule retained modes are stored: |kx| <= Kx = floor(NX/3), 0 <= kz <= Kz =
//    floor((2NZ-2)/3) (the dealias mask of dealias.cu:37), 44.5 % of the reference's storage;
//  * retained kx are kept in compact FFT order  i -> kx = (i <= Kx ? i : i - nkx);
//  * every split is balanced (counts differ by at most one), so any P <= min(nkx, NY) works,
//    including NY = 385 at P = 8;
//  * spectral layout per rank: [y][kx_local][kz] (y outermost, kz fastest): the all-to-all block
//    for peer p is the contiguous row range y in Y_p, so no local transposes are needed
//    (the reference ran 5 cublasCgeam passes per transpose, channel_cuda_mpi.c:64-128);
//  * physical/intermediate layout per rank: [y_local][x][kz].
//
// Pencil (decomposition = "pencil"): P = Pr x Pc ranks, rank = prow * Pc + pcol.
//  * spectral   [y (all)][kx in KX_pcol][kz in KZ_prow]       (kx split over Pc, kz split over Pr)
//  * A exchange (column group: same prow, Pc ranks): kx <-> y  -> [y in Y_pcol][kx (all)][kz in KZ_prow]
//  * x transform                                               -> [y in Y_pcol][x (all)][kz in KZ_prow]
//  * B exchange (row group: same pcol, Pr ranks):    kz <-> x  -> [y in Y_pcol][x in X_prow][kz (all)]
//  * z physical stage on full z rows, then the same exchanges in reverse.
// The slab is the Pr = 1 special case (no B exchange).  Neither exchange needs a communicator
// split: both are variable all-to-alls on the world communicator with zero counts outside the group.
#pragma once

#include <cstddef>
#include <vector>

#include "channel/config.hpp"

namespace channel {

struct Split {
  int n = 0, parts = 1;
  std::vector<int> start, count;
  static Split balanced(int n, int parts);
  // groups of a items (the last one may be partial), balanced over the parts (Plan::align_y)
  static Split aligned(int n, int parts, int a);
  int owner(int idx) const;
  int max_count() const;
};

struct Plan {
  int NX = 0, NY = 0, NZ = 0, Nzp = 0;
  int Kx = 0, nkx = 0, Kz = 0, nkz = 0;
  int P = 1, rank = 0;
  int Pr = 1, Pc = 1;         // process grid (slab: Pr = 1, Pc = P)
  int prow = 0, pcol = 0;     // rank = prow * Pc + pcol
  Split kx_split, y_split;    // over Pc (column index)
  Split kz_split, x_split;    // over Pr (row index)
  int nkx_loc = 0, kx0 = 0;   // local retained-kx range [kx0, kx0 + nkx_loc)
  int nkz_loc = 0, kz0 = 0;   // local retained-kz range [kz0, kz0 + nkz_loc) (slab: all)
  int ny_loc = 0, y0 = 0;     // local physical y range
  int nx_loc = 0, x0 = 0;     // local physical x range of the z stage (slab: all)
  int R = 1;                  // rows per lane of the 64-lane y-line solver: 64 * R >= NY
  double ax = 1.0, az = 2.0;  // 2*pi/LX, 2*pi/LZ

  int yalign = 1;             // y split in whole groups of yalign planes (align_y)

  static Plan make(const Config& cfg, int P, int rank);
  // y split in groups of a planes: the blocked spectral layout at P > 1 (Solver) keeps each
  // rank's y range whole 8-plane tiles, so the exchange blocks stay contiguous
  void align_y(int a);

  bool pencil() const { return Pr > 1; }
  int rank_of(int row, int col) const { return row * Pc + col; }
  int lines_loc() const { return nkx_loc * nkz_loc; }
  size_t spec_elems() const { return static_cast<size_t>(NY) * lines_loc(); }
  // x-expanded intermediate [y_loc][x][kz_loc] (pencil: blocked by destination x range)
  size_t phys_elems() const { return static_cast<size_t>(ny_loc) * NX * nkz_loc; }
  // z-stage rows [y_loc][x_loc][kz] (pencil only; blocked by source kz range)
  size_t zrow_elems() const { return static_cast<size_t>(ny_loc) * nx_loc * nkz; }
  // automatic pencil grid: the most square Pr x Pc with Pr <= Pc
  static void auto_grid(int P, int NX, int NY, int nkx, int nkz, int& Pr, int& Pc);
  // integer wavenumbers
  int kx_of(int i_global) const { return i_global <= Kx ? i_global : i_global - nkx; }
  // position of retained kx index in an NX-point FFT array
  int kx_fft_pos(int i_global) const { return i_global <= Kx ? i_global : NX - (nkx - i_global); }
  bool owns_mean() const { return kx0 == 0 && kz0 == 0; }
};

}  // namespace channel
