#include "channel/plan.hpp"

#include <algorithm>
#include <cmath>

#include "channel/common.hpp"

namespace channel {

Split Split::balanced(int n, int parts) {
  CH_CHECK(parts >= 1 && n >= parts, "cannot split " << n << " items over " << parts << " parts");
  Split s;
  s.n = n;
  s.parts = parts;
  s.start.resize(parts);
  s.count.resize(parts);
  int base = n / parts, rem = n % parts, off = 0;
  for (int p = 0; p < parts; ++p) {
    s.count[p] = base + (p < rem ? 1 : 0);
    s.start[p] = off;
    off += s.count[p];
  }
  return s;
}

// n items in groups of a (the last group may be partial) over `parts`: whole groups balanced, the
// extra groups on the LAST parts, so the partial group lands on a part with an extra group (NY =
// 385 in groups of 8 over 8 parts: 48 x 7 + 49, the balanced split's maximum).  Every part gets at
// least one group (the caller checks ceil(n / a) >= parts).
Split Split::aligned(int n, int parts, int a) {
  const int ng = (n + a - 1) / a;
  CH_CHECK(parts >= 1 && ng >= parts, "cannot split " << ng << " groups of " << a << " over " << parts << " parts");
  Split s;
  s.n = n;
  s.parts = parts;
  s.start.resize(parts);
  s.count.resize(parts);
  const int base = ng / parts, rem = ng % parts;
  int off = 0;
  for (int p = 0; p < parts; ++p) {
    const int g = base + (p >= parts - rem ? 1 : 0);
    s.start[p] = off;
    s.count[p] = std::min(g * a, n - off);
    off += s.count[p];
  }
  return s;
}

void Plan::align_y(int a) {
  y_split = Split::aligned(NY, Pc, a);
  ny_loc = y_split.count[pcol];
  y0 = y_split.start[pcol];
  yalign = a;
}

int Split::owner(int idx) const {
  for (int p = parts - 1; p >= 0; --p)
    if (idx >= start[p]) return p;
  return 0;
}

// The pencil grid with the fewest bytes on the busiest xGMI link.  Per substep a rank sends each
// column-group peer (A exchange, kx <-> y) (NY/Pc)(nkx/Pc)(nkz/Pr) and each row-group peer (B
// exchange, kz <-> x, on x-EXPANDED rows) (NY/Pc)(NX/Pr)(nkz/Pr) complex values, every peer over
// its own link: at 8 ranks of the 1024 x 385 x 1024 grid 4 x 2 puts 1.22 GB per step on a link
// against 1.83 GB for 2 x 4 (the most square grid), because B carries NX rather than nkx = 2NX/3.
// Ties go to the squarer grid with Pr <= Pc.  (The slab, Pr = 1, moves 0.31 GB per link: the
// pencil is for grids where the slab cannot split, e.g. NY < P.)
void Plan::auto_grid(int P, int NX, int NY, int nkx, int nkz, int& Pr, int& Pc) {
  Pr = 1;
  Pc = P;
  double best = -1.0;
  for (int r = 2; r <= 8 && r < P; ++r) {
    if (P % r) continue;
    const int c = P / r;
    if (c > 8 || c > nkx || c > NY || r > nkz || r > NX) continue;
    const double ny = static_cast<double>(NY) / c, kz = static_cast<double>(nkz) / r;
    const double a = c > 1 ? ny * (static_cast<double>(nkx) / c) * kz : 0.0;
    const double b = ny * (static_cast<double>(NX) / r) * kz;
    const double link = std::max(a, b);
    const bool squarer = std::abs(r - c) < std::abs(Pr - Pc) || (std::abs(r - c) == std::abs(Pr - Pc) && r <= c);
    if (best < 0 || link < best * (1.0 - 1e-9) || (link <= best * (1.0 + 1e-9) && squarer)) {
      best = link;
      Pr = r;
      Pc = c;
    }
  }
}

int Split::max_count() const { return *std::max_element(count.begin(), count.end()); }

Plan Plan::make(const Config& cfg, int P, int rank) {
  cfg.validate();
  Plan p;
  p.NX = cfg.NX;
  p.NY = cfg.NY;
  p.NZ = cfg.NZ;
  p.Nzp = cfg.nzp();
  p.Kx = p.NX / 3;
  p.nkx = 2 * p.Kx + 1;
  p.Kz = p.Nzp / 3;
  p.nkz = p.Kz + 1;
  CH_CHECK(p.nkz <= p.NZ, "internal: nkz > NZ");
  p.P = P;
  p.rank = rank;
  CH_CHECK(rank >= 0 && rank < P, "bad rank " << rank << " of " << P);
  if (cfg.decomposition == "pencil") {
    if (cfg.pr > 0 || cfg.pc > 0) {
      p.Pr = cfg.pr > 0 ? cfg.pr : P / std::max(1, cfg.pc);
      p.Pc = cfg.pc > 0 ? cfg.pc : P / std::max(1, cfg.pr);
    } else {
      auto_grid(P, p.NX, p.NY, p.nkx, p.nkz, p.Pr, p.Pc);
    }
    CH_CHECK(p.Pr * p.Pc == P, "pencil grid pr x pc = " << p.Pr << " x " << p.Pc << " does not match " << P << " ranks");
  } else {
    p.Pr = 1;
    p.Pc = P;
  }
  CH_CHECK(p.Pc <= 8 && p.Pr <= 8, "each exchange group holds at most 8 ranks (pr, pc <= 8)");
  CH_CHECK(p.Pc <= p.nkx && p.Pc <= p.NY,
           "pc=" << p.Pc << " exceeds retained kx (" << p.nkx << ") or NY (" << p.NY << ")");
  CH_CHECK(p.Pr <= p.nkz && p.Pr <= p.NX,
           "pr=" << p.Pr << " exceeds retained kz (" << p.nkz << ") or NX (" << p.NX << ")");
  p.prow = rank / p.Pc;
  p.pcol = rank % p.Pc;
  p.kx_split = Split::balanced(p.nkx, p.Pc);
  p.y_split = Split::balanced(p.NY, p.Pc);
  p.kz_split = Split::balanced(p.nkz, p.Pr);
  p.x_split = Split::balanced(p.NX, p.Pr);
  p.nkx_loc = p.kx_split.count[p.pcol];
  p.kx0 = p.kx_split.start[p.pcol];
  p.ny_loc = p.y_split.count[p.pcol];
  p.y0 = p.y_split.start[p.pcol];
  p.nkz_loc = p.kz_split.count[p.prow];
  p.kz0 = p.kz_split.start[p.prow];
  p.nx_loc = p.x_split.count[p.prow];
  p.x0 = p.x_split.start[p.prow];
  p.R = (p.NY + 63) / 64;
  CH_CHECK(p.R <= 24, "NY too large for the y-line solver (max 1536)");
  const double two_pi = 2.0 * std::acos(-1.0);
  p.ax = two_pi / cfg.LX;
  p.az = two_pi / cfg.LZ;
  return p;
}

}  // namespace channel
