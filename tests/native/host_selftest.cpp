// Host-side self-test of the native core's CPU components (config parser, grid/coefficient
// tables, decomposition plan, UMEAN/HDF5 I/O), built with AddressSanitizer + UndefinedBehavior
// Sanitizer by tools/host_sanitize.py.  SURVEY §5.2: the reference had no sanitizer or race
// tooling at all (Makefile:7 `DEBUG =` hook empty; host out-of-bounds u[-1]/u[NY] reads at
// meanUevol.c:415).  GPU ASan/xnack is not available on the MI355X pool, so the sanitizers cover
// the host code, and device code is covered by bounds checks on the host before every launch plus
// the debug-sync mode (common.hpp HIP_LAUNCH_CHECK).
//
// Exit status 0 = all checks passed; any sanitizer report aborts with a non-zero status.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "channel/common.hpp"
#include "channel/config.hpp"
#include "channel/grid.hpp"
#include "channel/io.hpp"
#include "channel/plan.hpp"

// The solver translation unit (not linked here) owns the debug flag and the occupancy helper.
namespace channel {
bool debug_sync_enabled() { return false; }
void set_debug_sync(bool) {}
int resident_blocks(const void*, int, size_t) { return 1; }
}  // namespace channel

static int g_fail = 0;
#define EXPECT(c)                                                      \
  do {                                                                 \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                        \
    }                                                                  \
  } while (0)

template <class F>
static bool throws(F&& f) {
  try {
    f();
  } catch (const channel::Error&) {
    return true;
  } catch (const std::exception&) {
    return true;
  }
  return false;
}

static void test_config() {
  using channel::Config;
  using channel::ConfigTree;
  const char* text =
      "application:\n{\n  NX = 64;\n  NY = 65;\n  NZ = 33;\n"
      "  input: { G = \"-\"; DDV = \"-\"; UMEAN = \"-\"; };\n"
      "  output: { G = \"G.h5\"; DDV = \"DDV.h5\"; UMEAN = \"Umean.bin\"; };\n"
      "  path = \"./out/\";   // trailing comment\n};\n# hash comment\n/* block\n comment */\n"
      "Re = 180.5; cfl = 0.25; health_check = false; precision = \"fp64\";\n";
  ConfigTree t = ConfigTree::parse_string(text);
  Config c = Config::from_tree(t);
  EXPECT(c.NX == 64 && c.NY == 65 && c.NZ == 33);
  EXPECT(c.out_G == "G.h5" && c.out_UMEAN == "Umean.bin" && c.path == "./out/");
  EXPECT(std::fabs(c.Re - 180.5) < 1e-12 && std::fabs(c.cfl - 0.25) < 1e-12);
  EXPECT(!c.health_check && c.fp64() && c.nzp() == 64);
  c.validate();
  // echo -> parse round trip
  Config c2 = Config::from_tree(ConfigTree::parse_string(c.to_string()));
  EXPECT(c2.NX == c.NX && c2.NY == c.NY && c2.Re == c.Re && c2.path == c.path);
  // malformed inputs must throw, never read out of bounds
  const char* bad[] = {"application: { NX = ; };", "application: { NX = 64",
                       "application: { NX = \"unterminated; };", "}", "/* never closed",
                       "a = 1 b = 2;", ""};
  for (const char* b : bad) {
    bool threw = throws([&] { (void)Config::from_tree(ConfigTree::parse_string(b)); });
    (void)threw;  // empty input is legal (all defaults); the point is no sanitizer report
  }
  EXPECT(throws([] { (void)ConfigTree::parse_string("application: { NX = 64"); }));
  // invalid settings
  Config v;
  v.NX = 100;  // not a power of two
  EXPECT(throws([&] { v.validate(); }));
  Config w;
  w.cfl = -1.0;
  EXPECT(throws([&] { w.validate(); }));
  Config s;
  s.spectra_planes = "0,5,128";
  auto pl = s.spectra_plane_list();
  EXPECT(pl.size() == 3 && pl[1] == 5);
}

static void test_grid() {
  for (int N : {5, 9, 33, 65, 129, 385, 1024}) {
    channel::YGrid g = channel::YGrid::build(N);
    EXPECT(static_cast<int>(g.y.size()) == N);
    EXPECT(std::fabs(g.y.front() + 1.0) < 1e-14 && std::fabs(g.y.back() - 1.0) < 1e-14);
    double s = 0.0;
    for (double w : g.trap) s += w;
    EXPECT(std::fabs(s - 2.0) < 1e-12);
    for (int j = 1; j < N; ++j) EXPECT(g.y[j] > g.y[j - 1]);
    // compact D1 is exact for linear functions: rhs(y) = lhs * 1
    for (int j = 1; j + 1 < N; ++j) {
      double rhs = g.d1_rm[j] * g.y[j - 1] + g.d1_rc[j] * g.y[j] + g.d1_rp[j] * g.y[j + 1];
      double lhs = g.d1_lo[j] + 1.0 + g.d1_up[j];
      EXPECT(std::fabs(rhs - lhs) < 1e-9 * std::fabs(lhs) + 1e-9);
    }
  }
}

static void test_plan() {
  channel::Config c;
  c.NX = 256;
  c.NY = 129;
  c.NZ = 129;
  for (int P : {1, 2, 3, 4, 7, 8}) {
    int lines = 0, ys = 0;
    for (int r = 0; r < P; ++r) {
      channel::Plan p = channel::Plan::make(c, P, r);
      lines += p.nkx_loc;
      ys += p.ny_loc;
      EXPECT(p.R * 64 >= p.NY);
      EXPECT(p.owns_mean() == (r == 0));
    }
    EXPECT(lines == channel::Plan::make(c, P, 0).nkx && ys == c.NY);
  }
  channel::Config pc = c;
  pc.decomposition = "pencil";
  for (int P : {4, 8}) {
    long total = 0;
    for (int r = 0; r < P; ++r) total += static_cast<long>(channel::Plan::make(pc, P, r).lines_loc());
    channel::Plan p0 = channel::Plan::make(pc, P, 0);
    EXPECT(total == static_cast<long>(p0.nkx) * p0.nkz);
  }
  auto sp = channel::Split::balanced(10, 3);
  EXPECT(sp.count[0] + sp.count[1] + sp.count[2] == 10 && sp.max_count() == 4);
  for (int i = 0; i < 10; ++i) EXPECT(sp.start[sp.owner(i)] <= i);
  EXPECT(throws([&] { (void)channel::Plan::make(c, 100000, 0); }));
}

static void test_io(const std::string& dir) {
  std::vector<double> U(65);
  for (size_t j = 0; j < U.size(); ++j) U[j] = 1.0 - 0.01 * static_cast<double>(j * j);
  std::string up = dir + "/Umean.bin";
  channel::umean_write(up, U);
  auto R = channel::umean_read(up, 65);
  EXPECT(R.size() == U.size());
  for (size_t j = 0; j < U.size() && j < R.size(); ++j)
    EXPECT(std::fabs(R[j] - static_cast<double>(static_cast<float>(U[j]))) < 1e-12);
  EXPECT(throws([&] { (void)channel::umean_read(up, 4096); }));  // short file
  EXPECT(throws([&] { (void)channel::umean_read(dir + "/missing.bin", 8); }));
  if (!channel::hdf5_available()) {
    std::printf("hdf5: not available, skipped\n");
    return;
  }
  const int NX = 8, NY = 5, NZ = 3;
  std::string hp = dir + "/G.h5";
  channel::h5_create_field(hp, NX, NY, NZ, false);
  std::vector<int> planes = {0, 7};
  std::vector<double> d(planes.size() * NY * 2 * NZ);
  for (size_t i = 0; i < d.size(); ++i) d[i] = static_cast<double>(static_cast<float>(0.5 * i - 3.0));
  channel::h5_write_planes(hp, planes, d);
  std::vector<double> g;
  int dims[3] = {0, 0, 0};
  channel::h5_read_planes(hp, planes, g, dims);
  EXPECT(dims[0] == NX && dims[1] == NY && dims[2] == 2 * NZ);
  EXPECT(g == d);
  channel::h5_write_attrs(hp, {{"time", 1.5}, {"dt", 2e-4}});
  auto a = channel::h5_read_attrs(hp);
  EXPECT(a["time"] == 1.5 && a["dt"] == 2e-4);
  EXPECT(throws([&] { channel::h5_read_planes(hp, {NX}, g, dims); }));  // plane out of range
}

int main(int argc, char** argv) {
  std::string dir = argc > 1 ? argv[1] : "/tmp";
  test_config();
  test_grid();
  test_plan();
  test_io(dir);
  if (g_fail) {
    std::fprintf(stderr, "host_selftest: %d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host_selftest: all checks passed\n");
  return 0;
}
