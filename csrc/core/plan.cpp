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

int Split::owner(int idx) const {
  for (int p = parts - 1; p >= 0; --p)
    if (idx >= start[p]) return p;
  return 0;
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
  CH_CHECK(P <= p.nkx && P <= p.NY, "P=" << P << " exceeds retained kx (" << p.nkx << ") or NY (" << p.NY << ")");
  p.kx_split = Split::balanced(p.nkx, P);
  p.y_split = Split::balanced(p.NY, P);
  p.nkx_loc = p.kx_split.count[rank];
  p.kx0 = p.kx_split.start[rank];
  p.ny_loc = p.y_split.count[rank];
  p.y0 = p.y_split.start[rank];
  p.R = (p.NY + 63) / 64;
  CH_CHECK(p.R <= 16, "NY too large for the y-line solver (max 1024)");
  const double two_pi = 2.0 * std::acos(-1.0);
  p.ax = two_pi / cfg.LX;
  p.az = two_pi / cfg.LZ;
  return p;
}

}  // namespace channel
