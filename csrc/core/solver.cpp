#include "channel/solver.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <chrono>
#include <functional>
#include <mutex>
#include <sstream>
#include <thread>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "channel/common.hpp"
#include "channel/io.hpp"

namespace channel {

namespace {
bool g_debug_sync = false;

template <typename T2>
void to_dev_type(const std::complex<double>* src, size_t n, std::vector<T2>& dst) {
  dst.resize(n);
  for (size_t i = 0; i < n; ++i) {
    dst[i].x = static_cast<decltype(dst[i].x)>(src[i].real());
    dst[i].y = static_cast<decltype(dst[i].x)>(src[i].imag());
  }
}

// deterministic uniform [-1, 1) from a 64-bit key (splitmix64)
double urand(unsigned long long key) {
  unsigned long long z = key + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  z = z ^ (z >> 31);
  return (static_cast<double>(z >> 11) / 9007199254740992.0) * 2.0 - 1.0;
}

// Thomas for complex RHS with real tridiagonal matrix (host, IC construction)
void thomas(const std::vector<double>& a, const std::vector<double>& b, const std::vector<double>& c,
            std::vector<std::complex<double>>& d) {
  const int n = static_cast<int>(d.size());
  std::vector<double> cp(n);
  std::vector<std::complex<double>> dp(n);
  cp[0] = c[0] / b[0];
  dp[0] = d[0] / b[0];
  for (int i = 1; i < n; ++i) {
    const double m = b[i] - a[i] * cp[i - 1];
    cp[i] = c[i] / m;
    dp[i] = (d[i] - a[i] * dp[i - 1]) / m;
  }
  d[n - 1] = dp[n - 1];
  for (int i = n - 2; i >= 0; --i) d[i] = dp[i] - cp[i] * d[i + 1];
}
}  // namespace

namespace {
void crash_handler(int sig) {
  static const char msg[] = "\n[channel] fatal signal; native backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  void* frames[64];
  const int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
struct CrashTraceAtLoad {
  CrashTraceAtLoad() {
    const char* e = std::getenv("CHANNEL_CRASH_TRACE");
    if (e && std::atoi(e) == 1) install_crash_handler();
  }
} g_crash_trace_at_load;
}  // namespace

void install_crash_handler() {
  for (int sig : {SIGSEGV, SIGBUS, SIGABRT, SIGILL, SIGFPE}) signal(sig, crash_handler);
}

int hip_runtime_version() {
  static const int v = [] {
    int r = 0;
    if (hipRuntimeGetVersion(&r) != hipSuccess) {
      (void)hipGetLastError();
      r = 0;
    }
    return r;
  }();
  return v;
}

bool debug_sync_enabled() { return g_debug_sync; }
void set_debug_sync(bool on) { g_debug_sync = on; }
bool g_lds_poison = [] {
  const char* e = std::getenv("CHANNEL_LDS_POISON");
  return e && std::atoi(e) != 0;
}();
bool lds_poison_enabled() { return g_lds_poison; }
void set_lds_poison(bool on) { g_lds_poison = on; }

int resident_blocks(const void* kernel, int threads, size_t dyn_lds) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, int> cache;
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find({dev, kernel});
  if (it != cache.end()) return it->second;
  int cus = 0, per_cu = 0;
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, dyn_lds));
  const int n = std::max(1, cus) * std::max(1, per_cu);
  cache[{dev, kernel}] = n;
  return n;
}

Solver::Solver(const Config& cfg, int rank, int nranks, int device, const std::string& nccl_uid)
    : cfg_(cfg), plan_(Plan::make(cfg, nranks, rank)), grid_(YGrid::build(cfg.NY, cfg.stretch)), device_(device) {
  fp64_ = cfg_.fp64();
  esz_ = fp64_ ? 16 : 8;
  HIP_CHECK(hipSetDevice(device_));
  // cache the runtime version outside any stream capture: transforms_slab first asks for it inside
  // a capture, where hipRuntimeGetVersion fails and left the cached value 0 (the two-compute-stream
  // pipeline then silently stayed off in every captured step)
  (void)hip_runtime_version();
  HIP_CHECK(hipStreamCreateWithFlags(&s_comp_, hipStreamNonBlocking));
  HIP_CHECK(hipStreamCreateWithFlags(&s_comm_, hipStreamNonBlocking));
  // A communicator exists for P > 1, and also at P = 1 when a unique id is passed: that runs the
  // distributed (exchange-based) pipeline on one rank, e.g. a real 1-rank RCCL communicator on a
  // one-GPU box, so the RCCL data plane and its graph capture are exercised on any machine.
  if (nranks > 1 || !nccl_uid.empty()) {
    CH_CHECK(!nccl_uid.empty(), "P > 1 requires an RCCL unique id");
    comm_ = Comm::create(rank, nranks, nccl_uid, device_);
    // per-run nonce shared by all ranks without a collective: FNV-1a of the communicator id
    run_nonce_ = 1469598103934665603ULL;
    for (unsigned char ch : nccl_uid) run_nonce_ = (run_nonce_ ^ ch) * 1099511628211ULL;
    // RCCL exchanges are captured into the step graph like everything else (the first step runs
    // eagerly so RCCL sets up its peer connections outside capture); CHANNEL_GRAPH_MULTI=0 keeps
    // multi-rank steps eager.  The host-staged ShmComm is never capturable.
    const char* gm = std::getenv("CHANNEL_GRAPH_MULTI");
    if (!comm_->graph_capturable() || (gm && std::atoi(gm) == 0)) use_graph_ = false;
    if (const char* t = std::getenv("CHANNEL_COMM_TIMEOUT_S")) comm_timeout_s_ = std::atof(t);
    if (const char* m = std::getenv("CHANNEL_MARKERS")) markers_ = std::atoi(m) == 1;
    if (plan_.pencil()) {
      // one communicator per decomposition axis (collective: same call order on every rank)
      std::vector<int> col, row;
      for (int c = 0; c < plan_.Pc; ++c) col.push_back(plan_.rank_of(plan_.prow, c));
      for (int r = 0; r < plan_.Pr; ++r) row.push_back(plan_.rank_of(r, plan_.pcol));
      comm_col_ = comm_->group(col);
      comm_row_ = comm_->group(row);
    }
  }
  {
    int R = 1, H = 1;
    kspec_geometry(cfg_.NY, fp64_, R, H);
    ytab_.upload(grid_, R, s_comp_, H);
  }
  tw_x_.build(plan_.NX, fp64_);
  tw_z_.build(plan_.Nzp, fp64_);
  choose_layout();
  alloc();
}

// Spectral layout: blocked [y/8][line/8][y%8][line%8] (kzb_ = 8, spec_index) where it measured
// faster: R = 7, 8 (1024x385x1024: 39.5 -> 35.8 ms/step at one rank); the plain layout stays at
// R = 5 (512x257x512: 7.37 vs 7.63) and R = 10 (2048x633x2048: 315 vs 323; profiles/r04/
// ab_layout_grids.txt).  CHANNEL_SPEC_KZB=0/1 forces it off/on (A/B).  At P > 1 the exchange blocks
// are row ranges of every line, so the y split is taken in whole 8-plane tiles (Plan::align_y: NY =
// 385 over 8 ranks is 48 x 7 + 49, the balanced split's maximum) and every block stays contiguous;
// the x kernels address the exchange segments in the same tiles (XArgs::segblk).  The same choice
// on every rank (a function of the grid, the precision and the environment).
void Solver::choose_layout() {
  const Plan& p = plan_;
  // The physical-stage fields: at P > 1 K-SPEC writes D1 v, v, D1 omega and the x-backward forms
  // u, w, omega_x, omega_z from them (combine): the backward exchange moves 5 fields instead of 6.
  // At one rank (no exchange, also the 1-rank RCCL communicator) K-SPEC writes the six fields (the
  // combine mode measured the same there, 32.54 vs 32.53 ms/step: K-SPEC takes the same time with 7
  // or 9 stores; profiles/r06/ab_start_combine_forcecomm.txt).  Where the exchange sets the pace
  // (the busiest-link model of BASELINE.md §3: P = 2 and 4 at the headline, exchange >= compute) one
  // sixth fewer backward bytes pay for the combine mode's two-input x-backward tiles (34.98 vs 33.78
  // ms/step of per-rank work at the headline on one GPU); at P >= 5 the step is compute-bound and
  // the six-output mode stays.  CHANNEL_COMBINE=0/1 forces either.
  combine_ = comm_ && p.P > 1 && p.P <= 4;
  if (const char* e = std::getenv("CHANNEL_COMBINE")) combine_ = std::atoi(e) != 0;
  {
    // fp64 storage from R = 10: K-SPEC is built for the six-output mode only (kspec_impl.hpp kSixOnly)
    int R = 1, H = 1;
    kspec_geometry(cfg_.NY, fp64_, R, H);
    if (combine_ && fp64_ && R >= 10) {
      if (std::getenv("CHANNEL_COMBINE")) std::fprintf(stderr, "[channel] CHANNEL_COMBINE ignored: fp64 at R >= 10 runs the six-output mode\n");
      combine_ = false;
    }
  }
  kzb_ = (p.R >= 7 && p.R <= 8) ? kSpecKzBlock : 0;
  if (const char* e = std::getenv("CHANNEL_SPEC_KZB")) kzb_ = std::atoi(e) != 0 ? kSpecKzBlock : 0;
  // (the x transforms address a blocked field with 32-bit byte offsets: above 4 GiB per field the
  // plain layout is used, also when CHANNEL_SPEC_KZB=1 asks for the blocked one)
  if (kzb_ && static_cast<unsigned long long>(spec_rows(kSpecKzBlock, p.NY)) * p.nkx_loc *
                      ((p.nkz_loc + kSpecKzBlock - 1) / kSpecKzBlock * kSpecKzBlock) * (fp64_ ? 16 : 8) >= (1ull << 32)) {
    if (std::getenv("CHANNEL_SPEC_KZB")) std::fprintf(stderr, "[channel] CHANNEL_SPEC_KZB ignored: a blocked field would exceed 4 GiB\n");
    kzb_ = 0;
  }
  if (comm_ && kzb_) {
    // every column-group rank needs a whole tile of planes; the round-1 per-field pencil exchange
    // (A/B) keeps the plain layout
    if ((p.NY + kSpecYBlock - 1) / kSpecYBlock < p.Pc || std::getenv("CHANNEL_PENCIL_UNCHUNKED")) kzb_ = 0;
    else plan_.align_y(kSpecYBlock);
  }
}

Solver::~Solver() {
  try {
    wait_checkpoint();
  } catch (const std::exception& e) {
    std::cerr << "[channel] background checkpoint failed: " << e.what() << "\n";
  }
  try {
    if (s_comp_) (void)hipStreamSynchronize(s_comp_);
    if (s_comm_) (void)hipStreamSynchronize(s_comm_);
  } catch (...) {
  }
  free_all();
  comm_row_.reset();
  comm_col_.reset();
  comm_.reset();
  if (s_comp_) (void)hipStreamDestroy(s_comp_);
  if (s_comm_) (void)hipStreamDestroy(s_comm_);
}

void Solver::alloc() {
  const Plan& p = plan_;
  // (kzb_: choose_layout)
  nkzs_ = kzb_ ? (p.nkz_loc + kzb_ - 1) / kzb_ * kzb_ : p.nkz_loc;
  canon_ = p.spec_elems();
  spec_ = static_cast<size_t>(spec_rows(kzb_, p.NY)) * p.nkx_loc * nkzs_;
  // streaming (non-temporal) spectral accesses in the x transforms only where the spectral fields
  // cannot stay in the 256 MB Infinity Cache anyway (a small grid's fields, written by K-SPEC, are
  // read back from it); CHANNEL_XNT=0/1 forces it (read per Solver)
  xnt_ = 6ull * spec_ * esz_ > (256ull << 20) ? 1 : 0;
  if (const char* e = std::getenv("CHANNEL_XNT")) xnt_ = std::atoi(e) != 0 ? 1 : 0;
  physn_ = p.phys_elems();
  // kx sub-blocks (K-SPEC / exchange overlap): slab with a communicator only; the same count on
  // every rank (a function of Pc and the environment), at most kMaxSeg exchange segments in total
  nkb_ = 1;
  if (comm_) {  // (pencil: the column group's A exchange, kx <-> y, is the slab's)
    int want = p.Pc <= 2 ? 4 : 2;
    if (const char* e = std::getenv("CHANNEL_KBLOCKS")) want = std::atoi(e);
    int minc = p.nkx;
    for (int c = 0; c < p.Pc; ++c) minc = std::min(minc, p.kx_split.count[c]);
    nkb_ = std::max(1, std::min({want, kMaxSeg / p.Pc, minc}));
    // the round-1 per-field pencil exchange (A/B) addresses whole rank blocks
    if (p.pencil() && std::getenv("CHANNEL_PENCIL_UNCHUNKED")) nkb_ = 1;
  }
  {
    const Split kb = Split::balanced(p.nkx_loc, nkb_);
    kb_start_ = kb.start;
    kb_cnt_ = kb.count;
    kb_off_.assign(nkb_, 0);
    // (each block a [y][lines_b] region, blocked like the whole field when kzb_: spec_index)
    for (int b = 1; b < nkb_; ++b)
      kb_off_[b] = kb_off_[b - 1] + static_cast<size_t>(spec_rows(kzb_, p.NY)) * kb_cnt_[b - 1] * nkzs_;
    ev_kb_.resize(nkb_);
    for (auto& e : ev_kb_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ev_fb_.resize(nkb_);
    for (auto& e : ev_fb_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&ev_cfl_, hipEventDisableTiming));
    // CHANNEL_FWD_SPLIT=0: the whole forward exchange completes before K-SPEC (A/B)
    if (const char* e = std::getenv("CHANNEL_FWD_SPLIT")) fwd_split_ = std::atoi(e) != 0;
  }
  // exchange receive buffer per field: segments [src column][y_loc][kx of the segment][kz] (blocked
  // like the spectral fields when kzb_: rows padded to whole 8-plane tiles, kz lines to nkzs_)
  xstride_ = static_cast<size_t>(spec_rows(kzb_, p.ny_loc)) * p.nkx * nkzs_;
  zstride_ = p.pencil() ? p.zrow_elems() : 0;
  // state_ = phi, R_phi, R_omega; the omega state is out_ field 4 (it IS the omega_y output of
  // K-SPEC, which then stores one field less per substep; the x transform zeroes its mean line)
  HIP_CHECK(hipMalloc(&state_, 3 * spec_ * esz_));
  HIP_CHECK(hipMalloc(&out_, 6 * spec_ * esz_));
  HIP_CHECK(hipMalloc(&phys_, std::max<size_t>(6 * physn_, 1) * esz_));
  HIP_CHECK(hipMemset(state_, 0, 3 * spec_ * esz_));
  HIP_CHECK(hipMemset(out_, 0, 6 * spec_ * esz_));
  if (comm_) {
    HIP_CHECK(hipMalloc(&xbuf_, 6 * xstride_ * esz_));
    HIP_CHECK(hipMemset(xbuf_, 0, 6 * xstride_ * esz_));
  }
  if (p.pencil()) {
    HIP_CHECK(hipMalloc(&zbuf_, 6 * zstride_ * esz_));
    HIP_CHECK(hipMemset(zbuf_, 0, 6 * zstride_ * esz_));
  }
  const int N = p.NY;
  // scalars: dt, time, dtlog[8], stats[4N], mean[3N+8], invdy[N], host-reduction scratch,
  // maxima[4] (float), health
  const size_t nd = 2 + 8 + 4 * N + (3 * N + 8) + N + 1;
  const size_t nbytes = nd * sizeof(double) + 32 + kKspecPhases * sizeof(unsigned long long);
  HIP_CHECK(hipMalloc(&dscal_, nbytes));
  HIP_CHECK(hipMemset(dscal_, 0, nbytes));
  double* d = static_cast<double*>(dscal_);
  d_dt_ = d;
  d_time_ = d + 1;
  d_dtlog_ = d + 2;
  d_stats_ = d + 10;
  d_mean_ = d_stats_ + 4 * N;
  d_invdy_ = d_mean_ + 3 * N + 8;
  d_red_ = d_invdy_ + N;
  d_max_ = reinterpret_cast<float*>(d_red_ + 1);
  d_health_ = reinterpret_cast<unsigned*>(d_max_ + 4);
  d_kprof_ = reinterpret_cast<unsigned long long*>(static_cast<char*>(dscal_) + nd * sizeof(double) + 32);
  kprof_on_ = std::getenv("CHANNEL_KSPEC_PROF") != nullptr;
  // y planes per x->z->x chunk (P = 1): 16 planes of 6 fp32 fields at NX = Nzp = 1024 are ~270 MB,
  // about the Infinity Cache; measured 57.9 -> 52.3 ms/step at 1024x385x1024 (4..64 swept, 16 best
  // on one stream); alternating two streams with 8-plane chunks: 50.6 ms/step.  The chunk is sized
  // in bytes (~144 MiB of x-expanded intermediates per stream), which the sweeps confirm across
  // grids: 512x257x512 best at 32 planes (11.2 -> 10.1 ms), 1024^2 fp64 at 4, 2048x633x2048 at 2
  // (gpurun_out/yc_*, profiles/r01_v18_ychunk_sweep.log).  Two streams keep two chunks in flight,
  // so at P = 1 each gets ~104 MiB (the pair stays inside the 256 MB cache): 6 planes at
  // 1024x385x1024, 35.9 -> 35.2 ms/step (profiles/r04/ab_ychunk.txt)
  ystreams_ = 2;
  if (const char* ys = std::getenv("CHANNEL_YSTREAMS")) ystreams_ = std::max(1, std::min(8, std::atoi(ys)));
  const size_t plane = 6ull * static_cast<size_t>(plan_.NX) * plan_.nkz * (fp64_ ? 16 : 8);
  // (no plane cap below the byte budget: a small grid whose whole x-expanded buffer fits is one
  // chunk, 3 launches per substep; 128x129x128 fp64: 0.537 -> 0.505 ms/step against 64 planes)
  auto planes_in = [&](size_t mib) { return static_cast<int>(std::max<size_t>(1, std::min<size_t>(1 << 16, (mib << 20) / plane))); };
  ychunk_ = ystreams_ >= 2 ? std::max(2, planes_in(104)) : planes_in(144);  // (2048x633x2048: 2 planes, 300.8 vs 310.7 ms at 1)
  // P > 1 slab: ~144 MiB per chunk; each chunk is also one batched exchange per direction, so the
  // exchange of chunk k+1 (and the return of chunk k-1) overlaps the transforms of chunk k
  // (several chunks keep the exchange pipelined); each chunk's transforms run as two parts on two
  // compute streams (transforms_slab), each part with the one-stream chunk's budget (~144 MiB: 8
  // planes at the headline): with a 1-rank RCCL communicator 35.9 (one stream, 8-plane chunks) ->
  // 34.2 (4 + 4-plane parts) -> 33.4 ms/step (8 + 8) against the 32.0 fast path; the 4-plane parts'
  // kernels ran mostly partial rounds of tiles (x-forward: 258 tiles for 256 CUs).  At slab8 (48-49
  // planes per rank) that is 4 chunks, and the exchange of a chunk's last kx sub-block is ~0.1 ms
  // (profiles/r06/ab_p_gt_1_plane_tiles.txt).  CHANNEL_PSTREAMS=1 keeps one stream
  pstreams_ = 2;
  if (const char* ps = std::getenv("CHANNEL_PSTREAMS")) pstreams_ = std::max(1, std::min(2, std::atoi(ps)));
  ychunk_p_ = std::min(64, planes_in(pstreams_ >= 2 && !plan_.pencil() ? 288 : 144));  // (the pencil: one stream)
  if (const char* yc = std::getenv("CHANNEL_YCHUNK")) ychunk_ = ychunk_p_ = std::atoi(yc);
  // blocked layout at P > 1: exchange chunks of whole 8-plane tiles (contiguous blocks)
  if (comm_ && kzb_ && ychunk_p_ > 0) ychunk_p_ = std::max(kSpecYBlock, ychunk_p_ / kSpecYBlock * kSpecYBlock);
  // CHANNEL_A2A_SELF = direct (default: the x transforms access the own block in place) | copy
  // (D2D copy inside the exchange) | rccl (through ncclSend/ncclRecv; RcclComm reads it too)
  if (const char* sm = std::getenv("CHANNEL_A2A_SELF")) self_direct_ = std::string(sm) == "direct";
  if (comm_ && pstreams_ >= 2) {
    HIP_CHECK(hipStreamCreateWithFlags(&s_comp2_, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&ev_comp2_, hipEventDisableTiming));
  }
  for (int i = 2; i < ystreams_; ++i) {
    hipStream_t st;
    HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    s_extra_.push_back(st);
  }
  ev_join_.resize(std::max(2, ystreams_));
  for (auto& e : ev_join_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  std::vector<double> invdy(N);
  const auto& y = grid_.y;
  for (int j = 0; j < N; ++j) {
    const double h = (j == 0) ? y[1] - y[0] : (j == N - 1 ? y[N - 1] - y[N - 2] : 0.5 * (y[j + 1] - y[j - 1]));
    invdy[j] = 1.0 / h;
  }
  HIP_CHECK(hipMemcpy(d_invdy_, invdy.data(), N * sizeof(double), hipMemcpyHostToDevice));
  HIP_CHECK(hipMalloc(&d_y_, N * sizeof(double)));
  HIP_CHECK(hipMemcpy(d_y_, y.data(), N * sizeof(double), hipMemcpyHostToDevice));
  ev_a2a_.resize(6);
  ev_xf_.resize(6);
  ev_b_.resize(6);
  ev_bb_.resize(3);
  for (auto* v : {&ev_a2a_, &ev_xf_, &ev_b_, &ev_bb_})
    for (auto& e : *v) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&ev_spec_, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&ev_phys_, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&ev_fwd_done_, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&ev_red_, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&ev_stats_, hipEventDisableTiming));
  for (auto& e : ev_dtf_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  ph_ms_.assign(8, 0.0);
  if (comm_ && !p.pencil()) build_rowtab();
}

// Row table of the slab exchange segments (XSrc / XDst::rowtab): for retained kx row i of segment
// s = c * nkb_ + b (rank c's kx sub-block b), the element offset of row i at the first chunk (y0 = 0)
// and the segment's Y stride (rows of 8 planes in the blocked layout, planes in the plain one), with
// the self-block bit for this rank's own blocks (read / written in place in the spectral fields).
// A chunk at y0 adds (y0 / 8 or y0) Y strides (XArgs::seg_y0): the offsets of transforms_slab's
// per-chunk segment tables, without a lookup per launch.
void Solver::build_rowtab() {
  const Plan& p = plan_;
  const int NB = nkb_;
  const long long ny_pad = spec_rows(kzb_, p.ny_loc);
  const long long S = kzb_ ? static_cast<long long>(kSpecKzBlock) * nkzs_ : nkzs_;  // seg_stride
  std::vector<unsigned> h(2 * static_cast<size_t>(p.nkx));
  for (int c = 0; c < p.Pc; ++c)
    for (int b = 0; b < NB; ++b) {
      const bool self = self_direct_ && c == p.pcol;
      const long long start = kb_gstart(c, b), count = kb_gcount(c, b);
      const long long off0 = self ? static_cast<long long>(kb_off_[b]) + static_cast<long long>(p.y0) * kb_cnt_[b] * nkzs_
                                  : ny_pad * start * nkzs_;
      for (long long i = start; i < start + count; ++i) {
        const long long a = off0 + (i - start) * S, st = count * S;
        CH_CHECK(a + (ny_pad / (kzb_ ? kSpecKzBlock : 1)) * st < (1ll << 32) && st < (1ll << 31),
                 "exchange segment offsets exceed 32 bits");
        h[2 * i] = static_cast<unsigned>(a);
        h[2 * i + 1] = static_cast<unsigned>(st) | (self ? 0x80000000u : 0u);
      }
    }
  HIP_CHECK(hipMalloc(&d_rowtab_, h.size() * sizeof(unsigned)));
  HIP_CHECK(hipMemcpy(d_rowtab_, h.data(), h.size() * sizeof(unsigned), hipMemcpyHostToDevice));
}

void Solver::free_all() {
  for (int i = 0; i < 2; ++i)
    if (gexec_[i]) (void)hipGraphExecDestroy(gexec_[i]);
  for (auto* v : {&ev_a2a_, &ev_xf_, &ev_b_, &ev_bb_})
    for (auto e : *v) (void)hipEventDestroy(e);
  for (auto e : tev_pool_) (void)hipEventDestroy(e);
  for (auto e : ev_join_) (void)hipEventDestroy(e);
  for (auto st : s_extra_) (void)hipStreamDestroy(st);
  if (s_comp2_) (void)hipStreamDestroy(s_comp2_);
  if (ev_comp2_) (void)hipEventDestroy(ev_comp2_);
  s_comp2_ = nullptr;
  ev_comp2_ = nullptr;
  ev_join_.clear();
  s_extra_.clear();
  for (auto* v : {&ev_cb_, &ev_cc_, &ev_cc2_, &ev_kb_, &ev_fb_})
    for (auto e : *v) (void)hipEventDestroy(e);
  ev_kb_.clear();
  ev_fb_.clear();
  for (auto& v : ev_pen_) {
    for (auto e : v) (void)hipEventDestroy(e);
    v.clear();
  }
  for (auto& pr : step_ev_) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  tev_pool_.clear();
  ev_cb_.clear();
  ev_cc_.clear();
  ev_cc2_.clear();
  step_ev_.clear();
  for (auto e : {ev_spec_, ev_phys_, ev_fwd_done_, ev_red_, ev_cfl_, ev_stats_, ev_tdt_[0], ev_tdt_[1], ev_dtf_[0], ev_dtf_[1]})
    if (e) (void)hipEventDestroy(e);
  if (h_tdt_) (void)hipHostFree(h_tdt_);
  h_tdt_ = nullptr;
  for (void* p : {state_, out_, phys_, xbuf_, zbuf_, dscal_, snap_, d_spec_, d_sym_, static_cast<void*>(d_y_),
                  static_cast<void*>(d_rowtab_)})
    if (p) (void)hipFree(p);
  state_ = out_ = phys_ = xbuf_ = zbuf_ = dscal_ = snap_ = d_spec_ = d_sym_ = nullptr;
  d_rowtab_ = nullptr;
  d_y_ = nullptr;
}

void* Solver::field_ptr(int f) const {
  char* st = static_cast<char*>(state_);
  char* ou = static_cast<char*>(out_);
  if (f == OMEGA) f = OUT4;
  if (f == PHI) return st;
  if (f == RPHI || f == ROMEGA) return st + static_cast<size_t>(f - RPHI + 1) * spec_ * esz_;
  if (f >= OUT0 && f <= OUT5) return ou + static_cast<size_t>(f - OUT0) * spec_ * esz_;
  CH_CHECK(false, "bad field index " << f);
}

// Input j of the x-backward's combine mode (XArgs::combine): 0 D1 v, 1 v, 2 D1 omega, 3 omega, 4 phi
// -- what K-SPEC leaves for the physical-space stage; the backward exchange of P > 1 moves these
// five fields (the forward one the three H fields)
// (six-output mode: the six fields u, v, w, omega_x, omega_y (the omega state), omega_z)
void* Solver::in_field(int j) const {
  static const Field kIn[5] = {OUT0, OUT1, OUT2, OMEGA, PHI};
  CH_CHECK(j >= 0 && j < bwd_fields(), "bad backward field " << j);
  return combine_ ? field_ptr(kIn[j]) : field_ptr(OUT0 + j);
}

int Solver::kb_gstart(int c, int b) const {
  return plan_.kx_split.start[c] + Split::balanced(plan_.kx_split.count[c], nkb_).start[b];
}
int Solver::kb_gcount(int c, int b) const { return Split::balanced(plan_.kx_split.count[c], nkb_).count[b]; }
size_t Solver::kb_index(int y, int ikx, int kz) const {
  int b = nkb_ - 1;
  while (b > 0 && ikx < kb_start_[b]) --b;
  return kb_off_[b] + spec_index(kzb_, kb_cnt_[b], nkzs_, y, ikx - kb_start_[b], kz);
}
size_t Solver::dev_index(int y, int ikx, int kz) const { return kb_index(y, ikx, kz); }

// ---- state ------------------------------------------------------------------------------------
void Solver::set_state(const std::complex<double>* phi, const std::complex<double>* omega, const double* U) {
  const Plan& p = plan_;
  const int lines = p.lines_loc();
  std::vector<std::complex<double>> om(omega, omega + canon_);
  if (p.owns_mean()) {
    for (int j = 0; j < p.NY; ++j) om[static_cast<size_t>(j) * lines] = std::complex<double>(U ? U[j] : 0.0, 0.0);
  }
  std::vector<std::complex<double>> phb;
  if (nkb_ > 1 || kzb_) {  // [y][kx_local][kz] -> kx sub-blocks / kz line blocks (padding: 0)
    phb.assign(spec_, 0.0);
    std::vector<std::complex<double>> omb(spec_, 0.0);
    for (int y = 0; y < p.NY; ++y)
      for (int i = 0; i < p.nkx_loc; ++i)
        for (int k = 0; k < p.nkz_loc; ++k) {
          const size_t src = (static_cast<size_t>(y) * p.nkx_loc + i) * p.nkz_loc + k, dst = dev_index(y, i, k);
          phb[dst] = phi[src];
          omb[dst] = om[src];
        }
    om.swap(omb);
    phi = phb.data();
  }
  HIP_CHECK(hipStreamSynchronize(s_comp_));
  if (fp64_) {
    std::vector<double2> h;
    to_dev_type(phi, spec_, h);
    HIP_CHECK(hipMemcpy(field_ptr(PHI), h.data(), spec_ * esz_, hipMemcpyHostToDevice));
    to_dev_type(om.data(), spec_, h);
    HIP_CHECK(hipMemcpy(field_ptr(OMEGA), h.data(), spec_ * esz_, hipMemcpyHostToDevice));
  } else {
    std::vector<float2> h;
    to_dev_type(phi, spec_, h);
    HIP_CHECK(hipMemcpy(field_ptr(PHI), h.data(), spec_ * esz_, hipMemcpyHostToDevice));
    to_dev_type(om.data(), spec_, h);
    HIP_CHECK(hipMemcpy(field_ptr(OMEGA), h.data(), spec_ * esz_, hipMemcpyHostToDevice));
  }
  HIP_CHECK(hipMemset(field_ptr(RPHI), 0, 2 * spec_ * esz_));
  prepared_ = false;
}

void Solver::get_state(std::complex<double>* phi, std::complex<double>* omega, double* U) const {
  const Plan& p = plan_;
  HIP_CHECK(hipStreamSynchronize(s_comp_));
  // device layout -> canonical [y][kx_local][kz]
  auto fetch = [&](int f, std::complex<double>* dst) {
    std::vector<std::complex<double>> t(spec_);
    if (fp64_) {
      std::vector<double2> h(spec_);
      HIP_CHECK(hipMemcpy(h.data(), field_ptr(f), spec_ * esz_, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < spec_; ++i) t[i] = {h[i].x, h[i].y};
    } else {
      std::vector<float2> h(spec_);
      HIP_CHECK(hipMemcpy(h.data(), field_ptr(f), spec_ * esz_, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < spec_; ++i) t[i] = {h[i].x, h[i].y};
    }
    if (nkb_ == 1 && !kzb_) {
      std::copy(t.begin(), t.end(), dst);
      return;
    }
    for (int y = 0; y < p.NY; ++y)
      for (int i = 0; i < p.nkx_loc; ++i)
        for (int k = 0; k < p.nkz_loc; ++k) dst[(static_cast<size_t>(y) * p.nkx_loc + i) * p.nkz_loc + k] = t[dev_index(y, i, k)];
  };
  fetch(PHI, phi);
  fetch(OMEGA, omega);
  const int lines = p.lines_loc();
  for (int j = 0; j < p.NY; ++j) {
    if (p.owns_mean()) {
      if (U) U[j] = omega[static_cast<size_t>(j) * lines].real();
      omega[static_cast<size_t>(j) * lines] = 0.0;
    } else if (U) {
      U[j] = 0.0;
    }
  }
}

void Solver::init_ic() {
  const Plan& p = plan_;
  const int N = p.NY, lines = p.lines_loc();
  std::vector<std::complex<double>> phi(canon_), om(canon_);
  std::vector<double> U(N);
  const auto& y = grid_.y;
  for (int j = 0; j < N; ++j) U[j] = (cfg_.ic == "zero") ? 0.0 : 0.75 * cfg_.Q * (1.0 - y[j] * y[j]);
  if (cfg_.ic == "random") {
    // full compact D2 with wall closure (reference secondDerivative, meanUevol.c:223-345)
    std::vector<double> la(N, 0), lb(N, 1), lc(N, 0);
    for (int j = 1; j < N - 1; ++j) { la[j] = grid_.m_lo[j]; lc[j] = grid_.m_up[j]; }
    lc[0] = grid_.d2_w0_up;
    la[N - 1] = grid_.d2_wN_lo;
    std::vector<std::complex<double>> v(N), w(N);
    const double amp = cfg_.ic_amplitude;
    // smooth in y: each line's profile is a random combination of the Chebyshev polynomials
    // T_0 .. T_{M-1} (weights 1/(1+m)) times the wall factors, so phi = D2 v - k2 v is a resolved
    // field (independent draws per grid point made grid-scale noise that D2 amplified by 1/dy^2)
    constexpr int kIcModes = 8;
    std::vector<double> cheb(static_cast<size_t>(N) * kIcModes);
    for (int j = 0; j < N; ++j) {
      double* T = &cheb[static_cast<size_t>(j) * kIcModes];
      T[0] = 1.0;
      T[1] = y[j];
      for (int m = 2; m < kIcModes; ++m) T[m] = 2.0 * y[j] * T[m - 1] - T[m - 2];
    }
    for (int ikx = 0; ikx < p.nkx_loc; ++ikx) {
      const int ig = p.kx0 + ikx;
      const int kx = p.kx_of(ig);
      for (int kzl = 0; kzl < p.nkz_loc; ++kzl) {
        const int kz = p.kz0 + kzl;
        const int line = ikx * p.nkz_loc + kzl;
        if (kx == 0 && kz == 0) continue;
        const double al = p.ax * kx, be = p.az * kz, k2 = al * al + be * be;
        const double env = std::exp(-k2 / 32.0);
        const bool cj = (kz == 0 && kx < 0);
        const unsigned long long base =
            (cfg_.seed * 1000003ULL + static_cast<unsigned long long>(std::abs(kx))) * 1000033ULL + kz;
        std::complex<double> cv[kIcModes], co[kIcModes];
        for (int m = 0; m < kIcModes; ++m) {
          const unsigned long long key = base * 4099ULL + m;
          const double wm = 1.0 / (1.0 + m);
          cv[m] = wm * std::complex<double>(urand(key * 4 + 0), urand(key * 4 + 1));
          co[m] = wm * std::complex<double>(urand(key * 4 + 2), urand(key * 4 + 3));
          if (cj) { cv[m] = std::conj(cv[m]); co[m] = std::conj(co[m]); }
        }
        for (int j = 0; j < N; ++j) {
          const double w1 = 1.0 - y[j] * y[j];
          const double* T = &cheb[static_cast<size_t>(j) * kIcModes];
          std::complex<double> vr = 0.0, orr = 0.0;
          for (int m = 0; m < kIcModes; ++m) {
            vr += cv[m] * T[m];
            orr += co[m] * T[m];
          }
          v[j] = amp * env * w1 * w1 * vr;
          w[j] = amp * env * w1 * orr;
        }
        v[0] = v[N - 1] = 0.0;
        w[0] = w[N - 1] = 0.0;
        // phi = D2 v - k2 v
        std::vector<std::complex<double>> d2(N);
        d2[0] = grid_.d2_w0[0] * v[0] + grid_.d2_w0[1] * v[1] + grid_.d2_w0[2] * v[2];
        d2[N - 1] = grid_.d2_wN[0] * v[N - 1] + grid_.d2_wN[1] * v[N - 2] + grid_.d2_wN[2] * v[N - 3];
        for (int j = 1; j < N - 1; ++j) d2[j] = grid_.k_lo[j] * v[j - 1] + grid_.k_c[j] * v[j] + grid_.k_up[j] * v[j + 1];
        thomas(la, lb, lc, d2);
        for (int j = 0; j < N; ++j) {
          phi[static_cast<size_t>(j) * lines + line] = d2[j] - k2 * v[j];
          om[static_cast<size_t>(j) * lines + line] = w[j];
        }
      }
    }
  } else {
    CH_CHECK(cfg_.ic == "laminar" || cfg_.ic == "zero", "init_ic: ic='" << cfg_.ic << "' needs set_state / read_restart");
  }
  set_state(phi.data(), om.data(), U.data());
  double zero2[2] = {0.0, 0.0};
  HIP_CHECK(hipMemcpy(d_dt_, zero2, 2 * sizeof(double), hipMemcpyHostToDevice));
  nstep_ = 0;
}

void Solver::set_time(double t, double dt) {
  double v[2] = {dt, t};
  HIP_CHECK(hipMemcpy(d_dt_, v, 2 * sizeof(double), hipMemcpyHostToDevice));
}

double Solver::time() const {
  // the step runs on the non-blocking compute stream: wait for it before reading the device time
  HIP_CHECK(hipStreamSynchronize(s_comp_));
  double t = 0;
  HIP_CHECK(hipMemcpy(&t, d_time_, sizeof(double), hipMemcpyDeviceToHost));
  return t;
}

// ---- pipeline ----------------------------------------------------------------------------------
void Solver::kspec(int mode, int n, bool stats) {
  const Plan& p = plan_;
  SpecArgs a;
  a.N = p.NY;
  a.lines = p.nkx_loc * nkzs_;
  a.nkz = nkzs_;
  a.kzb = kzb_;
  a.kz0 = p.kz0;
  a.kx0 = p.kx0;
  a.nkx = p.nkx;
  a.Kx = p.Kx;
  a.ax = p.ax;
  a.az = p.az;
  a.nu = 1.0 / cfg_.Re;
  a.mode = mode;
  if (mode == 1) {
    a.rk_a = RK3Coef::alpha[n];
    a.rk_b = RK3Coef::beta[n];
    a.rk_g = RK3Coef::gamma[n];
    a.rk_z = RK3Coef::zeta[n];
    a.store_r = n < 2 ? 1 : 0;  // R of the last substep is never read (zeta[0] = 0)
  }
  a.dt = d_dt_;
  a.Q = cfg_.Q;
  a.forcing = cfg_.forcing == "parity" ? 1 : 0;
  a.explicit_dd = cfg_.explicit_d2 == "dd";
  a.analytic_influence = cfg_.influence == "analytic";
  a.ygrid = d_y_;
  a.phi = field_ptr(PHI);
  a.omega = field_ptr(OMEGA);
  a.Rphi = field_ptr(RPHI);
  a.Romega = field_ptr(ROMEGA);
  for (int i = 0; i < 6; ++i) a.out[i] = field_ptr(OUT0 + i);
  a.stats = stats ? d_stats_ : nullptr;
  a.mean_diag = p.owns_mean() ? d_mean_ : nullptr;
  a.health = cfg_.health_check ? d_health_ : nullptr;
  a.prof = kprof_on_ ? d_kprof_ : nullptr;
  a.lds_poison = lds_poison_enabled() ? 1 : 0;
  a.out6 = combine_ ? 0 : 1;
  if (stats) HIP_CHECK(hipMemsetAsync(d_stats_, 0, 4 * p.NY * sizeof(double), s_comp_));
  ev(0, false);
  // (measured r2s: splitting this fused pass into an advance kernel and a prepare kernel frees no
  // occupancy at R = 7 -- 481 and 348 registers -- and costs 10.2 vs 7.2 ms per substep)
  if (nkb_ == 1) {
    join_forward();
    kspec_launch(ytab_, a, fp64_, s_comp_);
  } else {
    // kx sub-block b: the lines of local kx [kb_start_[b], +kb_cnt_[b]), a [y][lines_b] region of
    // every field; ev_kb_[b] lets the comm stream send block b while block b+1 is solved
    for (int b = 0; b < nkb_; ++b) {
      if (fwd_pending_) HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_fb_[b], 0));  // block b's returned rows
      SpecArgs ab = a;
      const size_t off = kb_off_[b] * esz_;
      auto sh = [&](void* q) { return static_cast<void*>(static_cast<char*>(q) + off); };
      ab.lines = kb_cnt_[b] * nkzs_;
      ab.kx0 = p.kx0 + kb_start_[b];
      ab.phi = sh(a.phi);
      ab.omega = sh(a.omega);
      ab.Rphi = sh(a.Rphi);
      ab.Romega = sh(a.Romega);
      for (int i = 0; i < 6; ++i) ab.out[i] = sh(a.out[i]);
      ab.mean_diag = b == 0 ? a.mean_diag : nullptr;  // (kx = 0 is local kx 0: block 0)
      kspec_launch(ytab_, ab, fp64_, s_comp_);
      HIP_CHECK(hipEventRecord(ev_kb_[b], s_comp_));
    }
    fwd_pending_ = false;  // (the last wait joined the comm stream's forward exchange back)
  }
  ev(0, true);
  if (stats && comm_) {
    HIP_CHECK(hipEventRecord(ev_stats_, s_comp_));
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_stats_, 0));
    comm_->allreduce_sum_f64(d_stats_, 4 * p.NY, s_comm_);
    HIP_CHECK(hipEventRecord(ev_stats_, s_comm_));
    HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_stats_, 0));
  }
}

// A exchange (column group: the Pc ranks of this process row), kx <-> y.
// spectral [y][kx_loc][kz_loc]: the block for column c is the contiguous row range Y_c;
// received blocks are [src column][y_loc][nkx_src][kz_loc] (the x transform gathers from them).
void Solver::a2a_spec(const void* spec, void* xb, bool to_phys) {
  const Plan& p = plan_;
  const int lines = p.lines_loc();
  std::vector<size_t> sc(p.P, 0), so(p.P, 0), rc(p.P, 0), ro(p.P, 0);
  for (int c = 0; c < p.Pc; ++c) {
    const int g = p.rank_of(p.prow, c);
    const size_t yo = static_cast<size_t>(p.y_split.start[c]) * lines * esz_;
    const size_t yc = static_cast<size_t>(p.y_split.count[c]) * lines * esz_;
    const size_t xo = static_cast<size_t>(p.ny_loc) * p.kx_split.start[c] * p.nkz_loc * esz_;
    const size_t xc = static_cast<size_t>(p.ny_loc) * p.kx_split.count[c] * p.nkz_loc * esz_;
    if (to_phys) { so[g] = yo; sc[g] = yc; ro[g] = xo; rc[g] = xc; }
    else { so[g] = xo; sc[g] = xc; ro[g] = yo; rc[g] = yc; }
  }
  if (to_phys) comm_->alltoallv(spec, sc, so, xb, rc, ro, s_comm_);
  else comm_->alltoallv(xb, sc, so, const_cast<void*>(spec), rc, ro, s_comm_);
}

// B exchange (row group: the Pr ranks of this process column), kz <-> x (pencil only).
// x-expanded [dst row][y_loc][x_r][kz_loc] <-> z rows [src row][y_loc][x_loc][kz_r].
void Solver::a2a_rows(void* xexp, void* zrows, bool to_z) {
  const Plan& p = plan_;
  std::vector<size_t> sc(p.P, 0), so(p.P, 0), rc(p.P, 0), ro(p.P, 0);
  for (int r = 0; r < p.Pr; ++r) {
    const int g = p.rank_of(r, p.pcol);
    const size_t xo = static_cast<size_t>(p.ny_loc) * p.x_split.start[r] * p.nkz_loc * esz_;
    const size_t xc = static_cast<size_t>(p.ny_loc) * p.x_split.count[r] * p.nkz_loc * esz_;
    const size_t zo = static_cast<size_t>(p.ny_loc) * p.nx_loc * p.kz_split.start[r] * esz_;
    const size_t zc = static_cast<size_t>(p.ny_loc) * p.nx_loc * p.kz_split.count[r] * esz_;
    if (to_z) { so[g] = xo; sc[g] = xc; ro[g] = zo; rc[g] = zc; }
    else { so[g] = zo; sc[g] = zc; ro[g] = xo; rc[g] = xc; }
  }
  if (to_z) comm_->alltoallv(xexp, sc, so, zrows, rc, ro, s_comm_);
  else comm_->alltoallv(zrows, sc, so, xexp, rc, ro, s_comm_);
}

void Solver::ev(int phase, bool end, hipStream_t s) {
  // roctx ranges name the phases in rocprofv3 --marker-trace timelines (host-side, no-ops otherwise)
  static const char* kPhaseNames[8] = {"kspec", "x_backward", "z_physical", "x_forward", "a2a", "reduce", "io", "other"};
  if (end) roctxRangePop();
  else roctxRangePushA(kPhaseNames[phase & 7]);
  if (!phase_timing_) return;
  hipEvent_t e = timing_event();
  HIP_CHECK(hipEventRecord(e, s ? s : s_comp_));
  if (!end) topen_[phase & 7] = e;
  else tpairs_.push_back({phase & 7, topen_[phase & 7], e});
}

hipEvent_t Solver::timing_event() {
  if (tev_used_ == tev_pool_.size()) {
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));
    tev_pool_.push_back(e);
  }
  return tev_pool_[tev_used_++];
}

void Solver::flush_phase_events() {
  if (!tpairs_.empty()) {
    synchronize();
    // intervals on a common clock (relative to the first event of the step): durations per phase,
    // and in slot 7 the time K-SPEC (phase 0, compute stream) and the exchanges (phase 4, comm
    // stream) actually ran at once (the K-SPEC / exchange overlap of the kx sub-blocks)
    std::vector<std::pair<float, float>> ks, ex;
    for (const auto& t : tpairs_) {
      float ms = 0, a0 = 0, b0 = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, t.a, t.b));
      ph_ms_[t.phase] += ms;
      if (t.phase == 0 || t.phase == 4) {
        HIP_CHECK(hipEventElapsedTime(&a0, tpairs_[0].a, t.a));
        HIP_CHECK(hipEventElapsedTime(&b0, tpairs_[0].a, t.b));
        (t.phase == 0 ? ks : ex).push_back({a0, b0});
      }
    }
    double ov = 0.0;
    for (const auto& k : ks)
      for (const auto& e : ex) ov += std::max(0.0f, std::min(k.second, e.second) - std::max(k.first, e.first));
    ph_ms_[7] += ov;
  }
  tpairs_.clear();
  tev_used_ = 0;
}

void Solver::set_phase_timing(bool on) {
  if (on && !phase_timing_) synchronize();
  phase_timing_ = on;
}

std::vector<double> Solver::phase_times_ms() { return ph_ms_; }

void Solver::reset_phase_times() { ph_ms_.assign(8, 0.0); }

std::vector<double> Solver::step_times_ms() {
  synchronize();
  std::vector<double> out;
  for (size_t i = 0; i < step_ev_used_; ++i) {
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, step_ev_[i].first, step_ev_[i].second));
    out.push_back(ms);
  }
  step_ev_used_ = 0;
  return out;
}

bool Solver::graph_active() const { return use_graph_ && (gexec_[0] != nullptr || gexec_[1] != nullptr); }

std::string Solver::comm_kind() const { return comm_ ? comm_->kind() : "none"; }

std::vector<double> Solver::kspec_profile() {
  std::vector<unsigned long long> h(kKspecPhases, 0);
  HIP_CHECK(hipStreamSynchronize(s_comp_));
  HIP_CHECK(hipMemcpy(h.data(), d_kprof_, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return std::vector<double>(h.begin(), h.end());
}

void Solver::transforms(int n, bool /*stats*/) {
  const Plan& p = plan_;
  XArgs xa;
  xa.NX = p.NX;
  xa.nkx = p.nkx;
  xa.Kx = p.Kx;
  xa.nkz = p.nkz;
  xa.ny = p.ny_loc;
  xa.field_stride_phys = static_cast<long long>(physn_);
  // u, v, w, omega_x, omega_y, omega_z: read (omega_y's source is the omega state, whose mean line
  // holds U: read as 0) or formed per element from the five combine-mode outputs
  xa.combine = combine_ ? 1 : 0;
  xa.zero_mean_field = combine_ ? -1 : 4;
  xa.ax = p.ax;
  xa.az = p.az;
  xa.kz_glob0 = p.kz0;
  xa.lds_poison = lds_poison_enabled() ? 1 : 0;
  xa.nt = xnt_;
  ZArgs za;
  za.lds_poison = xa.lds_poison;
  za.NX = p.NX;
  za.Nzp = p.Nzp;
  za.nkz = p.nkz;
  za.ny = p.ny_loc;
  za.y0 = p.y0;
  za.field_stride = static_cast<long long>(physn_);
  za.scale = 1.0 / (static_cast<double>(p.NX) * p.Nzp);
  za.inv_dy = d_invdy_;
  za.cx = p.ax * p.Kx;
  za.cz = p.az * p.Kz;
  // CFL maxima of the current state only (substep 0, as calcDt at RK3.c:143-145); substeps 1, 2 skip them
  za.maxima = n == 0 ? d_max_ : nullptr;
  DtArgs da;
  da.maxima = d_max_;
  da.dt = d_dt_;
  da.time = d_time_;
  da.dt_log = d_dtlog_;
  da.health = cfg_.health_check ? d_health_ : nullptr;
  da.cfl = cfg_.cfl;
  da.dt_max = cfg_.dt_max;
  da.dt_fixed = cfg_.dt_fixed;
  da.parity = cfg_.cfl_mode == "parity" ? 1 : 0;
  da.NX = p.NX;
  da.NZ = p.NZ;
  da.LX = cfg_.LX;
  da.LZ = cfg_.LZ;
  da.Re = cfg_.Re;
  da.dy_uniform = 2.0 / (p.NY - 1);

  if (!comm_) {
    // one rank: the spectral fields are blocked by 8 kz lines (kzb_, spec_index); the x transforms
    // address rows spec_y0 .. of the full fields
    xa.kzb = kzb_;
    xa.nkzs = nkzs_;
    xa.spec_y0 = 0;
    XSrc src;
    src.base = out_;
    src.nsrc = 1;
    src.kx_start[0] = 0;
    src.kx_start[1] = p.nkx;
    if (combine_)
      for (int j = 0; j < kCmbIn; ++j) src.fld[j] = in_field(j);
    xa.nfields = 6;
    xa.field_stride_spec = static_cast<long long>(spec_);
    XDst dst;
    dst.base = out_;
    dst.ndst = 1;
    dst.kx_start[0] = 0;
    dst.kx_start[1] = p.nkx;
    if (ychunk_ > 0 && ychunk_ < p.ny_loc) {
      // y-chunked x -> z -> x pipeline: the physical intermediates of one chunk of y planes
      // (9 fields x chunk x NX x nkz) are produced and consumed back to back, so they are served
      // from the 256 MB Infinity Cache instead of making a full HBM round trip per stage
      // chunks alternate between the compute and the (idle at P = 1) comm stream, so one chunk's
      // launch tail overlaps the next chunk's transforms (chunks are independent; the CFL maxima
      // are atomic)
      // (phase timing serialises the chunks on one stream so the stage times add up to the step)
      const int nst = phase_timing_ ? 1 : std::max(1, ystreams_);
      std::vector<hipStream_t> streams = {s_comp_, s_comm_};
      for (auto e : s_extra_) streams.push_back(e);
      roctxRangePushA("xzx_ychunked");
      if (nst > 1) {
        HIP_CHECK(hipEventRecord(ev_spec_, s_comp_));
        for (int i = 1; i < nst; ++i) HIP_CHECK(hipStreamWaitEvent(streams[i], ev_spec_, 0));
      }
      int ci = 0;
      for (int y0 = 0; y0 < p.ny_loc; y0 += ychunk_, ++ci) {
        const int ny = std::min(ychunk_, p.ny_loc - y0);
        hipStream_t cs = streams[ci % nst];
        const size_t so = kzb_ ? 0 : static_cast<size_t>(y0) * p.nkx * p.nkz * esz_;
        char* ph = static_cast<char*>(phys_) + static_cast<size_t>(y0) * p.NX * p.nkz * esz_;
        XArgs xc = xa;
        xc.ny = ny;
        if (kzb_) xc.spec_y0 = y0;
        XSrc sc = src;
        sc.base = static_cast<char*>(out_) + so;
        if (combine_)
          for (int j = 0; j < kCmbIn; ++j) sc.fld[j] = static_cast<const char*>(src.fld[j]) + so;
        xc.nfields = 6;
        ev(1, false, cs);
        xfft_backward(xc, sc, ph, tw_x_, fp64_, cs);
        ev(1, true, cs);
        ZArgs zc = za;
        zc.ny = ny;
        zc.y0 = p.y0 + y0;
        ev(2, false, cs);
        zphys(zc, ph, tw_z_, fp64_, cs);
        ev(2, true, cs);
        XDst dc = dst;
        dc.base = static_cast<char*>(out_) + so;
        xc.nfields = 3;
        ev(3, false, cs);
        xfft_forward(xc, ph, dc, tw_x_, fp64_, cs);
        ev(3, true, cs);
      }
      for (int i = 1; i < nst; ++i) {
        HIP_CHECK(hipEventRecord(ev_join_[i], streams[i]));
        HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_join_[i], 0));
      }
      if (n == 0) dt_update(da, s_comp_);
      roctxRangePop();
      return;
    }
    ev(1, false);
    xfft_backward(xa, src, phys_, tw_x_, fp64_, s_comp_);
    ev(1, true);
    ev(2, false);
    zphys(za, phys_, tw_z_, fp64_, s_comp_);
    ev(2, true);
    // dt from the CFL maxima on the (idle at P = 1) comm stream, beside the x-forward: only the next
    // K-SPEC needs it (one ~5 us kernel less on the critical path of a small grid's step; phase
    // timing keeps it in line)
    const bool fork_dt = n == 0 && !phase_timing_;
    if (fork_dt) {
      HIP_CHECK(hipEventRecord(ev_dtf_[0], s_comp_));
      HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_dtf_[0], 0));
      dt_update(da, s_comm_);
      HIP_CHECK(hipEventRecord(ev_dtf_[1], s_comm_));
    } else if (n == 0) {
      dt_update(da, s_comp_);
    }
    xa.nfields = 3;
    ev(3, false);
    xfft_forward(xa, phys_, dst, tw_x_, fp64_, s_comp_);
    ev(3, true);
    if (fork_dt) HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_dtf_[1], 0));
    return;
  }
  if (!p.pencil()) {
    transforms_slab(n, xa, za, da);
    return;
  }
  if (std::getenv("CHANNEL_PENCIL_UNCHUNKED") == nullptr) {
    transforms_pencil(n, xa, za, da);
    return;
  }
  // ---- pencil: per-field exchanges on the comm stream, overlapped with the x transforms ----
  const int Pc = p.Pc, Pr = p.Pr;
  const bool pen = p.pencil();
  XSrc src;
  src.base = xbuf_;
  src.nsrc = Pc;
  XDst dst;
  dst.base = xbuf_;
  dst.ndst = Pc;
  for (int c = 0; c < Pc; ++c) {
    src.kx_start[c] = dst.kx_start[c] = p.kx_split.start[c];
    src.off[c] = dst.off[c] = static_cast<long long>(p.ny_loc) * p.kx_split.start[c] * p.nkz_loc;
  }
  src.kx_start[Pc] = dst.kx_start[Pc] = p.nkx;
  xa.nkz = p.nkz_loc;
  xa.nfields = 6;
  xa.field_stride_spec = static_cast<long long>(xstride_);
  if (pen) {  // x-expanded output blocked by destination row (x range)
    xa.npseg = Pr;
    for (int r = 0; r < Pr; ++r) {
      xa.x_start[r] = p.x_split.start[r];
      xa.poff[r] = static_cast<long long>(p.ny_loc) * p.x_split.start[r] * p.nkz_loc;
    }
    xa.x_start[Pr] = p.NX;
    // z stage over [src row][y_loc][x_loc][kz_r]
    za.NX = p.nx_loc;
    za.field_stride = static_cast<long long>(zstride_);
    za.nseg = Pr;
    for (int r = 0; r < Pr; ++r) {
      za.kz_start[r] = p.kz_split.start[r];
      za.off[r] = static_cast<long long>(p.ny_loc) * p.nx_loc * p.kz_split.start[r];
    }
    za.kz_start[Pr] = p.nkz;
  }
  auto fld = [&](void* base, size_t stride, int f) { return static_cast<char*>(base) + static_cast<size_t>(f) * stride * esz_; };
  HIP_CHECK(hipEventRecord(ev_spec_, s_comp_));
  HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_spec_, 0));
  for (int f = 0; f < bwd_fields(); ++f) {
    ev(4, false, s_comm_);
    a2a_spec(in_field(f), fld(xbuf_, xstride_, f), true);
    ev(4, true, s_comm_);
  }
  HIP_CHECK(hipEventRecord(ev_a2a_[0], s_comm_));
  HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_a2a_[0], 0));
  ev(1, false);
  {
    XSrc sf = src;
    if (combine_)
      for (int j = 0; j < kCmbIn; ++j) sf.fld[j] = fld(xbuf_, xstride_, j);
    else
      xa.zero_mean_field = 4;
    xfft_backward(xa, sf, phys_, tw_x_, fp64_, s_comp_);
  }
  if (pen) {  // ship the x-blocks of the six fields to the row group
    HIP_CHECK(hipEventRecord(ev_b_[0], s_comp_));
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_b_[0], 0));
    for (int f = 0; f < 6; ++f) {
      ev(4, false, s_comm_);
      a2a_rows(fld(phys_, physn_, f), fld(zbuf_, zstride_, f), true);
      ev(4, true, s_comm_);
    }
  }
  ev(1, true);
  void* zf = phys_;
  if (pen) {
    HIP_CHECK(hipEventRecord(ev_fwd_done_, s_comm_));
    HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_fwd_done_, 0));
    zf = zbuf_;
  }
  ev(2, false);
  zphys(za, zf, tw_z_, fp64_, s_comp_);
  ev(2, true);
  if (n == 0) {
    HIP_CHECK(hipEventRecord(ev_phys_, s_comp_));
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_phys_, 0));
    ev(5, false, s_comm_);
    comm_->allreduce_max_f32(d_max_, 4, s_comm_);
    ev(5, true, s_comm_);
    HIP_CHECK(hipEventRecord(ev_red_, s_comm_));
    HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_red_, 0));
    dt_update(da, s_comp_);
  }
  if (pen) {
    HIP_CHECK(hipEventRecord(ev_phys_, s_comp_));
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_phys_, 0));
    for (int f = 0; f < 3; ++f) {
      ev(4, false, s_comm_);
      a2a_rows(fld(phys_, physn_, f), fld(zbuf_, zstride_, f), false);
      ev(4, true, s_comm_);
      HIP_CHECK(hipEventRecord(ev_bb_[f], s_comm_));
    }
  }
  ev(3, false);
  xa.nfields = 1;  // (one field per forward call)
  for (int f = 0; f < 3; ++f) {
    if (pen) HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_bb_[f], 0));
    XDst df = dst;
    df.base = fld(xbuf_, xstride_, f);
    xfft_forward(xa, fld(phys_, physn_, f), df, tw_x_, fp64_, s_comp_);
    HIP_CHECK(hipEventRecord(ev_xf_[f], s_comp_));
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_xf_[f], 0));
    ev(4, false, s_comm_);
    a2a_spec(field_ptr(OUT0 + f), fld(xbuf_, xstride_, f), false);
    ev(4, true, s_comm_);
  }
  ev(3, true);
  HIP_CHECK(hipEventRecord(ev_fwd_done_, s_comm_));
  HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_fwd_done_, 0));
}

// Exchange of y chunk k over the column group (the slab: every rank; the pencil: the Pc ranks of
// this process row, A exchange kx <-> y): chunk k holds rows [k*ch, (k+1)*ch) of EVERY
// rank's y range, so the chunk count is the same on all ranks (uneven splits send empty blocks
// at the end).  Backward (to_phys): my spectral rows Y_c[k] of fields 0..nf-1 go to rank c and
// land in c's receive block [src][y_loc][nkx_src][kz] at row k*ch; forward: the transformed rows
// of my chunk go back into the owners' spectral rows.  Both sides are contiguous in memory, so
// there is no pack/unpack pass (the reference ran 5 cublasCgeam passes around each host-staged
// MPI_Alltoall, channel_cuda_mpi.c:64-128).
void Solver::a2a_slab_chunk(int k, int ch, bool to_phys, int nf) { a2a_slab_rows(k * ch, ch, to_phys, nf, 0, nkb_); }

// Rows [r0, r0 + nr) of every rank's y range, kx sub-blocks [blo, bhi): one op per (field, block),
// each with one contiguous piece per peer (block b of the spectral field is [y][lines_b]; the
// receive segment (c, b) of xbuf is [y_loc][kx in block b of rank c][kz] in global kx order).
void Solver::a2a_slab_rows(int r0, int nr, bool to_phys, int nf, int blo, int bhi) {
  const Plan& p = plan_;
  const int P = p.Pc;  // column group (slab: the world)
  const size_t nr_me = static_cast<size_t>(std::max(0, std::min(nr, p.ny_loc - r0)));
  std::vector<A2ABlock> ops;
  ops.reserve(static_cast<size_t>(nf) * (bhi - blo));
  if (to_phys) bwd_blocks_issued_ += bhi - blo;  // (host-side count of issued backward block exchanges)
  // blocked layout (kzb_): rows go in whole 8-plane tiles (r0 and every rank's first row are tile
  // aligned; a rank's last tile may be partial and is sent whole: padding rows of the fields)
  auto rows_pad = [&](size_t n) { return kzb_ ? (n + kSpecYBlock - 1) / kSpecYBlock * kSpecYBlock : n; };
  const size_t ny_pad = rows_pad(static_cast<size_t>(p.ny_loc));
  for (int f = 0; f < nf; ++f)
    for (int b = blo; b < bhi; ++b) {
      ops.emplace_back();
      A2ABlock& o = ops.back();
      o.scount.assign(P, 0);
      o.soff.assign(P, 0);
      o.rcount.assign(P, 0);
      o.roff.assign(P, 0);
      char* spec = static_cast<char*>(to_phys ? in_field(f) : field_ptr(OUT0 + f));
      char* xb = static_cast<char*>(xbuf_) + static_cast<size_t>(f) * xstride_ * esz_;
      const size_t lines_b = static_cast<size_t>(kb_cnt_[b]) * nkzs_;
      for (int c = 0; c < P; ++c) {
        if (self_direct_ && c == p.pcol) continue;  // read/written in place by the x transforms
        const size_t nr_c = rows_pad(static_cast<size_t>(std::max(0, std::min(nr, p.y_split.count[c] - r0))));
        const size_t yo = (kb_off_[b] + (static_cast<size_t>(p.y_split.start[c]) + r0) * lines_b) * esz_;
        const size_t yc = nr_c * lines_b * esz_;
        const size_t gs = static_cast<size_t>(kb_gstart(c, b)), gc = static_cast<size_t>(kb_gcount(c, b));
        const size_t xo = (ny_pad * gs + static_cast<size_t>(r0) * gc) * nkzs_ * esz_;
        const size_t xc = rows_pad(nr_me) * gc * nkzs_ * esz_;
        if (to_phys) {
          o.soff[c] = yc ? yo : 0;
          o.scount[c] = yc;
          o.roff[c] = xc ? xo : 0;
          o.rcount[c] = xc;
        } else {
          o.soff[c] = xc ? xo : 0;
          o.scount[c] = xc;
          o.roff[c] = yc ? yo : 0;
          o.rcount[c] = yc;
        }
      }
      o.send = to_phys ? static_cast<const void*>(spec) : static_cast<const void*>(xb);
      o.recv = to_phys ? static_cast<void*>(xb) : static_cast<void*>(spec);
    }
  col_comm()->alltoallv_batch(ops, s_comm_);
}

// P > 1 slab substep transforms, y-chunked and pipelined over two streams:
//   comm:  B(0) B(1) F(0) B(2) F(1) ... F(nch-1) [CFL allreduce]
//   comp:       x->z->x(0)  x->z->x(1) ...
// B(k) = backward exchange of chunk k (6 fields, one batched group), F(k) = forward exchange of
// chunk k (3 fields).  While chunk k is transformed, chunk k+1 arrives and chunk k-1 returns, and
// the x-expanded intermediates of a chunk are produced and consumed back to back (served from the
// Infinity Cache).  The arithmetic is identical to the unchunked sequence (bitwise).
void Solver::transforms_slab(int n, const XArgs& xa0, const ZArgs& za0, const DtArgs& da) {
  const Plan& p = plan_;
  const int P = p.P;
  const int maxrows = p.y_split.max_count();
  const int ch = (ychunk_p_ > 0 && ychunk_p_ < maxrows) ? ychunk_p_ : maxrows;
  const int nch = (maxrows + ch - 1) / ch;
  while (static_cast<int>(ev_cb_.size()) < nch) {
    hipEvent_t a, b;
    HIP_CHECK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
    ev_cb_.push_back(a);
    ev_cc_.push_back(b);
  }
  XArgs xa = xa0;
  xa.nkz = p.nkz_loc;
  xa.nkzs = nkzs_;
  xa.segblk = kzb_ ? 1 : 0;
  xa.field_stride_spec = static_cast<long long>(xstride_);
  const long long ny_pad = spec_rows(kzb_, p.ny_loc);
  // exchange segments: block b of rank c is segment c * nkb_ + b (global kx order)
  const int NB = nkb_, NS = P * NB;
  CH_CHECK(NS <= kMaxSeg, "at most " << kMaxSeg << " exchange segments");
  XSrc src;
  src.base = xbuf_;
  src.nsrc = NS;
  XDst dst;
  dst.base = xbuf_;
  dst.ndst = NS;
  for (int c = 0; c < P; ++c)
    for (int b = 0; b < NB; ++b) src.kx_start[c * NB + b] = dst.kx_start[c * NB + b] = kb_gstart(c, b);
  src.kx_start[NS] = dst.kx_start[NS] = p.nkx;
  src.rowtab = dst.rowtab = d_rowtab_;  // (the same rows as the per-chunk off[] below, at y0 = 0)
  if (self_direct_) {  // own kx blocks: straight from / into the spectral fields
    src.self_seg = dst.self_seg = p.rank * NB;
    src.nself = dst.nself = NB;
    src.self_base = out_;
    dst.self_base = out_;
    src.self_field_stride = dst.self_field_stride = static_cast<long long>(spec_);
    CH_CHECK(spec_ < (1ull << 32), "spectral field exceeds 32-bit element offsets");
  }
  // combine inputs: received blocks in the exchange buffer (five fields), own blocks in place
  if (combine_)
    for (int j = 0; j < kCmbIn; ++j) {
      src.fld[j] = static_cast<const char*>(xbuf_) + static_cast<size_t>(j) * xstride_ * esz_;
      if (self_direct_) src.self_fld[j] = in_field(j);
    }

  roctxRangePushA("xzx_slab_chunked");
  // K-SPEC / exchange overlap: blocks 0 .. NB-2 of the previous substep's K-SPEC go out whole as
  // soon as each is solved (while the next block runs on the compute stream); the last block is
  // sent chunk by chunk ahead of the transforms.  Substep 0 of a step starts without the overlap:
  // its K-SPEC belongs to the previous step (another graph launch), whose events this step's
  // capture cannot wait on.
  const bool overlap = NB > 1 && n > 0;
  const bool present = NB > 1 && n == 0 && presend_done_;  // blocks 0 .. NB-2 already sent
  presend_done_ = false;
  const int bchunk = (overlap || present) ? NB - 1 : 0;  // blocks still to send per chunk: [bchunk, NB)
  const bool fsplit = NB > 1 && fwd_split_;
  join_forward();  // (normally consumed by the K-SPEC in between)
  if (overlap) {
    for (int b = 0; b + 1 < NB; ++b) {
      HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_kb_[b], 0));
      ev(4, false, s_comm_);
      a2a_slab_rows(0, maxrows, true, bwd_fields(), b, b + 1);
      ev(4, true, s_comm_);
    }
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_kb_[NB - 1], 0));
  } else {
    HIP_CHECK(hipEventRecord(ev_spec_, s_comp_));
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_spec_, 0));
  }
  auto backward = [&](int k) {
    ev(4, false, s_comm_);
    a2a_slab_rows(k * ch, ch, true, bwd_fields(), bchunk, NB);
    ev(4, true, s_comm_);
    HIP_CHECK(hipEventRecord(ev_cb_[k], s_comm_));
  };
  backward(0);
  // a chunk's transforms may run as two parts on two compute streams (below; each part waits for its
  // chunk's backward exchange, which follows K-SPEC on the comm stream; parts touch disjoint phys
  // planes and exchange rows; the CFL maxima are atomic); phase timing keeps one stream so the stage
  // times add up
  // (not inside a stream capture on a HIP runtime older than 7.2: a process that imports torch
  // binds torch's bundled HIP 7.0 runtime and RCCL (same sonames), and there a captured step with the
  // second compute stream forked next to the RCCL exchanges segfaults in the runtime; eager steps and
  // /opt/rocm's 7.2 runtime -- bench.py and the drivers are torch-free -- capture it fine)
  // (CHANNEL_PSTREAMS_CAPTURE=1 lifts the runtime-version gate: diagnosis of the 7.0 crash)
  hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
  if (s_comp2_) HIP_CHECK(hipStreamIsCapturing(s_comp_, &cst));
  static const bool cap_force = [] {
    const char* e = std::getenv("CHANNEL_PSTREAMS_CAPTURE");
    return e && std::atoi(e) == 1;
  }();
  const bool two = s_comp2_ != nullptr && !phase_timing_ && nch > 1 &&
                   (cst == hipStreamCaptureStatusNone || hip_runtime_version() >= 70200000 || cap_force);
  // two compute streams: each exchange chunk's transforms run as two parts of (about) half its rows,
  // one per stream, both waiting for the chunk's backward exchange (the pair of parts in flight is
  // one chunk's intermediates, as at P = 1, where alternating whole 8-plane chunks kept two chunks'
  // intermediates in flight and overflowed the Infinity Cache); parts start on plane pairs (the
  // plane tiles) and address their rows of the chunk's exchange blocks through XArgs::seg_yoff
  while (static_cast<int>(ev_cc2_.size()) < nch) {
    hipEvent_t e;
    HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ev_cc2_.push_back(e);
  }
  if (cst != hipStreamCaptureStatusNone) captured_streams_ = two ? 2 : 1;
  if (markers_ && cst != hipStreamCaptureStatusNone && n == 0)
    marker(two ? "capture: transforms on two compute streams" : "capture: transforms on one compute stream");
  // CHANNEL_PSPLIT=0: whole chunks alternate between the two streams instead (A/B)
  static const bool psplit = [] {
    const char* e = std::getenv("CHANNEL_PSPLIT");
    return !(e && std::atoi(e) == 0);
  }();
  const int nparts = two && psplit ? 2 : 1;
  const int part = nparts > 1 ? ((ch + 3) / 4) * 2 : ch;  // rows of the first part (even)
  for (int k = 0; k < nch; ++k) {
    if (k + 1 < nch) backward(k + 1);
    const int y0 = k * ch, ny = std::max(0, std::min(ch, p.ny_loc - y0));
    for (int c = 0; c < P; ++c)
      for (int b = 0; b < NB; ++b)
        src.off[c * NB + b] = dst.off[c * NB + b] =
            (ny_pad * kb_gstart(c, b) + static_cast<long long>(y0) * kb_gcount(c, b)) * nkzs_;
    if (self_direct_)  // rows y0.. of this rank's y range in its own spectral fields (block b)
      for (int b = 0; b < NB; ++b)
        src.off[p.rank * NB + b] = dst.off[p.rank * NB + b] =
            static_cast<long long>(kb_off_[b]) + (static_cast<long long>(p.y0) + y0) * kb_cnt_[b] * nkzs_;
    for (int h = 0; h < nparts; ++h) {
      hipStream_t cs = (h || (two && !psplit && (k & 1))) ? s_comp2_ : s_comp_;
      HIP_CHECK(hipStreamWaitEvent(cs, ev_cb_[k], 0));
      const int r0 = h ? std::min(part, ny) : 0;
      const int nr = nparts > 1 ? (h ? ny - r0 : std::min(part, ny)) : ny;
      if (nr > 0) {
        XArgs xc = xa;
        xc.ny = nr;
        xc.nfields = 6;
        xc.seg_y0 = kzb_ ? y0 / kSpecYBlock : y0;
        xc.seg_yoff = r0;
        char* ph = static_cast<char*>(phys_) + static_cast<size_t>(y0 + r0) * p.NX * p.nkz_loc * esz_;
        ev(1, false, cs);
        xfft_backward(xc, src, ph, tw_x_, fp64_, cs);
        ev(1, true, cs);
        ZArgs zc = za0;
        zc.ny = nr;
        zc.y0 = p.y0 + y0 + r0;
        ev(2, false, cs);
        zphys(zc, ph, tw_z_, fp64_, cs);
        ev(2, true, cs);
        xc.nfields = 3;
        ev(3, false, cs);
        xfft_forward(xc, ph, dst, tw_x_, fp64_, cs);
        ev(3, true, cs);
      }
      HIP_CHECK(hipEventRecord(h ? ev_cc2_[k] : ev_cc_[k], cs));
      HIP_CHECK(hipStreamWaitEvent(s_comm_, h ? ev_cc2_[k] : ev_cc_[k], 0));
    }
    if (fsplit && k == nch - 1) {
      // forward-path overlap: the CFL maxima first (every z stage is done), then the last chunk's
      // rows block by block; K-SPEC block b waits only for ev_fb_[b] (kspec())
      if (n == 0) {
        ev(5, false, s_comm_);
        comm_->allreduce_max_f32(d_max_, 4, s_comm_);
        ev(5, true, s_comm_);
        HIP_CHECK(hipEventRecord(ev_cfl_, s_comm_));
      }
      for (int b = 0; b < NB; ++b) {
        ev(4, false, s_comm_);
        a2a_slab_rows(k * ch, ch, false, 3, b, b + 1);
        ev(4, true, s_comm_);
        HIP_CHECK(hipEventRecord(ev_fb_[b], s_comm_));
      }
      continue;
    }
    ev(4, false, s_comm_);
    a2a_slab_chunk(k, ch, false, 3);
    ev(4, true, s_comm_);
  }
  if (two) {  // join the second compute stream (also reached through the forward exchange)
    HIP_CHECK(hipEventRecord(ev_comp2_, s_comp2_));
    HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_comp2_, 0));
  }
  if (fsplit) {
    if (n == 0) HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_cfl_, 0));
    fwd_pending_ = true;
  } else {
    if (n == 0) {  // every chunk's z stage precedes ev_cc_[nch-1], which the comm stream waited on
      ev(5, false, s_comm_);
      comm_->allreduce_max_f32(d_max_, 4, s_comm_);
      ev(5, true, s_comm_);
    }
    HIP_CHECK(hipEventRecord(ev_fwd_done_, s_comm_));
    HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_fwd_done_, 0));
  }
  if (n == 0) dt_update(da, s_comp_);
  roctxRangePop();
}

// B exchange of y chunk k over the row group (the Pr ranks of this process column, x <-> kz):
// the x-expanded rows of the chunk, blocked by destination row r ([r][y_loc][x_r][kz_loc]), go to
// row peer r and land in its z-row buffer [src][y_loc][x_loc][kz_src] at row k*ch (to_z), and the
// z stage's H rows come back the same way (!to_z).  Every block is contiguous: no packing.
void Solver::b2b_pencil_chunk(int k, int ch, bool to_z, int nf) {
  const Plan& p = plan_;
  const int Pr = p.Pr;
  const size_t y0 = static_cast<size_t>(k) * ch;
  const size_t nr = static_cast<size_t>(std::max(0, std::min(ch, p.ny_loc - k * ch)));
  std::vector<A2ABlock> ops(nf);
  for (int f = 0; f < nf; ++f) {
    A2ABlock& o = ops[f];
    o.scount.assign(Pr, 0);
    o.soff.assign(Pr, 0);
    o.rcount.assign(Pr, 0);
    o.roff.assign(Pr, 0);
    char* xe = static_cast<char*>(phys_) + static_cast<size_t>(f) * physn_ * esz_;
    char* zr = static_cast<char*>(zbuf_) + static_cast<size_t>(f) * zstride_ * esz_;
    for (int r = 0; r < Pr; ++r) {
      const size_t xo = (static_cast<size_t>(p.ny_loc) * p.x_split.start[r] + y0 * p.x_split.count[r]) * p.nkz_loc * esz_;
      const size_t xc = nr * p.x_split.count[r] * p.nkz_loc * esz_;
      const size_t zo = (static_cast<size_t>(p.ny_loc) * p.nx_loc * p.kz_split.start[r] + y0 * p.nx_loc * p.kz_split.count[r]) * esz_;
      const size_t zc = nr * p.nx_loc * p.kz_split.count[r] * esz_;
      if (to_z) {
        o.soff[r] = xc ? xo : 0;
        o.scount[r] = xc;
        o.roff[r] = zc ? zo : 0;
        o.rcount[r] = zc;
      } else {
        o.soff[r] = zc ? zo : 0;
        o.scount[r] = zc;
        o.roff[r] = xc ? xo : 0;
        o.rcount[r] = xc;
      }
    }
    o.send = to_z ? static_cast<const void*>(xe) : static_cast<const void*>(zr);
    o.recv = to_z ? static_cast<void*>(zr) : static_cast<void*>(xe);
  }
  comm_row_->alltoallv_batch(ops, s_comm_);
}

// P = Pr x Pc pencil substep transforms: the slab's y-chunked pipeline with the row-group B
// exchange between the x transforms and the z stage, as a software pipeline over two streams.
// Per chunk k the stages are A-in(k) -> x-backward(k) -> B-in(k) -> z(k) -> B-out(k) ->
// x-forward(k) -> A-out(k); in issue step t the comm stream runs A-in(t), B-in(t-2), B-out(t-4),
// A-out(t-6) and the compute stream x-backward(t-1), z(t-3), x-forward(t-5), each waiting only on
// the event its predecessor recorded in step t-1.  Every exchange is one batched group on its
// axis communicator (RCCL: ncclCommSplit), the chunk's intermediates are produced and consumed
// back to back (Infinity Cache), and the whole schedule is captured in the step graph.  The
// arithmetic is the unchunked sequence's (bitwise).
void Solver::transforms_pencil(int n, const XArgs& xa0, const ZArgs& za0, const DtArgs& da) {
  const Plan& p = plan_;
  const int Pc = p.Pc, Pr = p.Pr;
  const int maxrows = p.y_split.max_count();
  const int ch = (ychunk_p_ > 0 && ychunk_p_ < maxrows) ? ychunk_p_ : maxrows;
  const int nch = (maxrows + ch - 1) / ch;
  for (auto& v : ev_pen_)
    while (static_cast<int>(v.size()) < nch) {
      hipEvent_t e;
      HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      v.push_back(e);
    }
  enum { E_A = 0, E_XB, E_B, E_Z, E_BF, E_XF };
  XArgs xa = xa0;
  xa.nkz = p.nkz_loc;
  xa.nkzs = nkzs_;
  xa.segblk = kzb_ ? 1 : 0;
  xa.field_stride_spec = static_cast<long long>(xstride_);
  const long long ny_pad = spec_rows(kzb_, p.ny_loc);
  xa.npseg = Pr;
  for (int r = 0; r < Pr; ++r) xa.x_start[r] = p.x_split.start[r];
  xa.x_start[Pr] = p.NX;
  // A-exchange segments: kx sub-block b of column c is segment c * nkb_ + b (global kx order)
  const int NB = nkb_, NSG = Pc * NB;
  CH_CHECK(NSG <= kMaxSeg, "at most " << kMaxSeg << " exchange segments");
  XSrc src;
  src.base = xbuf_;
  src.nsrc = NSG;
  XDst dst;
  dst.base = xbuf_;
  dst.ndst = NSG;
  for (int c = 0; c < Pc; ++c)
    for (int b = 0; b < NB; ++b) src.kx_start[c * NB + b] = dst.kx_start[c * NB + b] = kb_gstart(c, b);
  src.kx_start[NSG] = dst.kx_start[NSG] = p.nkx;
  if (self_direct_) {  // own column blocks: straight from / into the spectral fields
    src.self_seg = dst.self_seg = p.pcol * NB;
    src.nself = dst.nself = NB;
    src.self_base = out_;
    dst.self_base = out_;
    src.self_field_stride = dst.self_field_stride = static_cast<long long>(spec_);
    CH_CHECK(spec_ < (1ull << 32), "spectral field exceeds 32-bit element offsets");
  }
  // combine inputs: received blocks in the exchange buffer (five fields), own blocks in place
  if (combine_)
    for (int j = 0; j < kCmbIn; ++j) {
      src.fld[j] = static_cast<const char*>(xbuf_) + static_cast<size_t>(j) * xstride_ * esz_;
      if (self_direct_) src.self_fld[j] = in_field(j);
    }
  ZArgs za = za0;
  za.NX = p.nx_loc;
  za.field_stride = static_cast<long long>(zstride_);
  za.nseg = Pr;
  for (int r = 0; r < Pr; ++r) za.kz_start[r] = p.kz_split.start[r];
  za.kz_start[Pr] = p.nkz;
  // chunk-dependent offsets
  auto chunk_rows = [&](int k) { return std::max(0, std::min(ch, p.ny_loc - k * ch)); };
  auto set_x = [&](int k, XArgs& x, XSrc& sc, XDst& dc) {
    const long long y0 = static_cast<long long>(k) * ch;
    x.ny = chunk_rows(k);
    for (int r = 0; r < Pr; ++r)
      x.poff[r] = (static_cast<long long>(p.ny_loc) * p.x_split.start[r] + y0 * p.x_split.count[r]) * p.nkz_loc;
    for (int c = 0; c < Pc; ++c)
      for (int b = 0; b < NB; ++b)
        sc.off[c * NB + b] = dc.off[c * NB + b] = (ny_pad * kb_gstart(c, b) + y0 * kb_gcount(c, b)) * nkzs_;
    if (self_direct_)
      for (int b = 0; b < NB; ++b)
        sc.off[p.pcol * NB + b] = dc.off[p.pcol * NB + b] =
            static_cast<long long>(kb_off_[b]) + (static_cast<long long>(p.y0) + y0) * kb_cnt_[b] * nkzs_;
  };
  auto xbw = [&](int k) {
    if (chunk_rows(k) > 0) {
      XArgs x = xa;
      XSrc sc = src;
      XDst dc = dst;
      set_x(k, x, sc, dc);
      x.nfields = 6;
      ev(1, false);
      xfft_backward(x, sc, phys_, tw_x_, fp64_, s_comp_);
      ev(1, true);
    }
    HIP_CHECK(hipEventRecord(ev_pen_[E_XB][k], s_comp_));
  };
  auto zst = [&](int k) {
    if (chunk_rows(k) > 0) {
      ZArgs z = za;
      const long long y0 = static_cast<long long>(k) * ch;
      z.ny = chunk_rows(k);
      z.y0 = p.y0 + static_cast<int>(y0);
      for (int r = 0; r < Pr; ++r)
        z.off[r] = static_cast<long long>(p.ny_loc) * p.nx_loc * p.kz_split.start[r] + y0 * p.nx_loc * p.kz_split.count[r];
      ev(2, false);
      zphys(z, zbuf_, tw_z_, fp64_, s_comp_);
      ev(2, true);
    }
    HIP_CHECK(hipEventRecord(ev_pen_[E_Z][k], s_comp_));
  };
  auto xfw = [&](int k) {
    if (chunk_rows(k) > 0) {
      XArgs x = xa;
      XSrc sc = src;
      XDst dc = dst;
      set_x(k, x, sc, dc);
      x.nfields = 3;
      ev(3, false);
      xfft_forward(x, phys_, dc, tw_x_, fp64_, s_comp_);
      ev(3, true);
    }
    HIP_CHECK(hipEventRecord(ev_pen_[E_XF][k], s_comp_));
  };
  auto comm_op = [&](int k, int wait_ev, int rec_ev, const std::function<void()>& f) {
    if (wait_ev >= 0) HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_pen_[wait_ev][k], 0));
    ev(4, false, s_comm_);
    f();
    ev(4, true, s_comm_);
    if (rec_ev >= 0) HIP_CHECK(hipEventRecord(ev_pen_[rec_ev][k], s_comm_));
  };

  roctxRangePushA("xzx_pencil_chunked");
  // K-SPEC / A-exchange overlap over kx sub-blocks, as in transforms_slab
  const bool overlap = NB > 1 && n > 0;
  const bool present = NB > 1 && n == 0 && presend_done_;
  presend_done_ = false;
  const int bchunk = (overlap || present) ? NB - 1 : 0;
  if (overlap) {
    for (int b = 0; b + 1 < NB; ++b) {
      HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_kb_[b], 0));
      ev(4, false, s_comm_);
      a2a_slab_rows(0, maxrows, true, bwd_fields(), b, b + 1);
      ev(4, true, s_comm_);
    }
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_kb_[NB - 1], 0));
  } else {
    HIP_CHECK(hipEventRecord(ev_spec_, s_comp_));
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_spec_, 0));
  }
  for (int t = 0; t < nch + 6; ++t) {
    if (t < nch) comm_op(t, -1, E_A, [&] { a2a_slab_rows(t * ch, ch, true, bwd_fields(), bchunk, NB); });
    if (t - 2 >= 0 && t - 2 < nch) comm_op(t - 2, E_XB, E_B, [&] { b2b_pencil_chunk(t - 2, ch, true, 6); });
    if (t - 4 >= 0 && t - 4 < nch) comm_op(t - 4, E_Z, E_BF, [&] { b2b_pencil_chunk(t - 4, ch, false, 3); });
    if (t - 6 >= 0 && t - 6 < nch) comm_op(t - 6, E_XF, -1, [&] { a2a_slab_chunk(t - 6, ch, false, 3); });
    if (t - 1 >= 0 && t - 1 < nch) {
      HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_pen_[E_A][t - 1], 0));
      xbw(t - 1);
    }
    if (t - 3 >= 0 && t - 3 < nch) {
      HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_pen_[E_B][t - 3], 0));
      zst(t - 3);
    }
    if (t - 5 >= 0 && t - 5 < nch) {
      HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_pen_[E_BF][t - 5], 0));
      xfw(t - 5);
    }
  }
  if (n == 0) {  // every z stage precedes the last A-out on the comm stream (E_Z -> E_BF -> E_XF)
    ev(5, false, s_comm_);
    comm_->allreduce_max_f32(d_max_, 4, s_comm_);
    ev(5, true, s_comm_);
  }
  HIP_CHECK(hipEventRecord(ev_fwd_done_, s_comm_));
  HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_fwd_done_, 0));
  if (n == 0) dt_update(da, s_comp_);
  roctxRangePop();
}

void Solver::prepare() {
  presend_done_ = false;  // the outputs are recomputed: a pre-sent exchange is stale
  kspec(0, 0, cfg_.stats_every > 0);
  stats_pending_ = cfg_.stats_every > 0;
  prepared_ = true;
}

void Solver::step_body(bool stats) {
  for (int n = 0; n < 3; ++n) {
    transforms(n, false);
    kspec(1, n, stats && n == 2);
    CH_CHECK(!capture_fail_test_, "capture failure injected (CHANNEL_TEST_CAPTURE_FAIL)");
  }
  // the next step's substep-0 backward exchange of blocks 0 .. NB-2, behind this step's last
  // K-SPEC blocks (joined back into the compute stream: a captured graph must end there)
  if (kb_overlap()) presend_backward(true);
}

// Backward exchange of kx sub-blocks 0 .. nkb_-2 (all rows) for the coming substep 0.
// wait_blocks: each waits for its K-SPEC block (ev_kb_); otherwise for everything queued on the
// compute stream so far.  The comm stream is joined back into the compute stream.
void Solver::presend_backward(bool wait_blocks) {
  const int maxrows = plan_.y_split.max_count();
  if (!wait_blocks) {
    HIP_CHECK(hipEventRecord(ev_spec_, s_comp_));
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_spec_, 0));
  }
  for (int b = 0; b + 1 < nkb_; ++b) {
    if (wait_blocks) HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_kb_[b], 0));
    ev(4, false, s_comm_);
    a2a_slab_rows(0, maxrows, true, bwd_fields(), b, b + 1);
    ev(4, true, s_comm_);
  }
  HIP_CHECK(hipEventRecord(ev_fwd_done_, s_comm_));
  HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_fwd_done_, 0));
  presend_done_ = true;
}

void Solver::marker(const char* what) {
  const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_created_).count();
  std::fprintf(stderr, "[channel] rank %d/%d: %s (step %ld, %.2f s after setup)\n", plan_.rank, plan_.P, what, nstep_, t);
  std::fflush(stderr);
}

// A capture that threw: end it on the origin stream and make sure no stream forked into it is
// left in capture mode (a later collective on such a stream would fail on this rank only and strand
// its peers in the capture agreement below).
void Solver::end_failed_capture() {
  fwd_pending_ = false;  // (the captured forward exchange is discarded with the graph)
  hipGraph_t junk = nullptr;
  (void)hipStreamEndCapture(s_comp_, &junk);
  if (junk) (void)hipGraphDestroy(junk);
  std::vector<hipStream_t> forked = {s_comm_};
  for (auto st : s_extra_) forked.push_back(st);
  if (s_comp2_) forked.push_back(s_comp2_);
  for (auto st : forked) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
      hipGraph_t j2 = nullptr;
      (void)hipStreamEndCapture(st, &j2);
      if (j2) (void)hipGraphDestroy(j2);
    }
  }
  (void)hipGetLastError();
}

void Solver::step(bool stats_for_next) {
  if (!prepared_) prepare();
  const int gi = stats_for_next ? 1 : 0;
  bool done = false;
  const bool warmup_step = comm_ && !comm_warm_;
  bool captured_now = false;
  if (step_timing_) {
    if (step_ev_used_ == step_ev_.size()) {
      hipEvent_t a, b;
      HIP_CHECK(hipEventCreate(&a));
      HIP_CHECK(hipEventCreate(&b));
      step_ev_.emplace_back(a, b);
    }
    HIP_CHECK(hipEventRecord(step_ev_[step_ev_used_].first, s_comp_));
  }
  // substep 0 relies on blocks 0 .. NB-2 having been sent (the previous step's tail does it)
  if (kb_overlap() && !presend_done_) presend_backward(false);
  // P > 1: the first step runs eagerly so RCCL connects its peers outside stream capture
  const bool warm = !comm_ || comm_warm_;
  if (use_graph_ && warm && !debug_sync_enabled() && !phase_timing_) {
    if (!gexec_[gi] && !graph_ok_[gi]) {
      const long long blocks_saved = bwd_blocks_issued_;
      try {
        hipGraph_t g = nullptr;
        // thread-local capture with a communicator: RCCL's proxy thread keeps making HIP calls
        hipStreamCaptureMode mode = comm_ ? hipStreamCaptureModeThreadLocal : hipStreamCaptureModeGlobal;
        if (const char* m = std::getenv("CHANNEL_CAPTURE_MODE")) {
          const std::string ms(m);
          mode = ms == "global" ? hipStreamCaptureModeGlobal
                                : (ms == "relaxed" ? hipStreamCaptureModeRelaxed : hipStreamCaptureModeThreadLocal);
        }
        // test-only (CHANNEL_TEST_CAPTURE_FAIL=<rank>): that rank's capture fails after the first
        // substep has been recorded, to drive the cross-rank agreement below
        const char* tf = std::getenv("CHANNEL_TEST_CAPTURE_FAIL");
        const bool inject = tf && std::atoi(tf) == plan_.rank;
        // capturing records the step without running it, but step_body() still updates the host
        // pipeline state (presend_done_: which kx sub-blocks of substep 0 the coming step resends).
        // A graph that is abandoned (here or after the cross-rank agreement below) must leave that
        // state as it was, or this rank's eager step would exchange other blocks than its peers'.
        presend_saved_ = presend_done_;
        // (CHANNEL_MARKERS=1: one line per capture phase, to place a failure inside the runtime)
        if (markers_) marker("capture: begin");
        HIP_CHECK(hipStreamBeginCapture(s_comp_, mode));
        try {
          capture_fail_test_ = inject;
          step_body(stats_for_next);
          capture_fail_test_ = false;
          if (markers_) marker("capture: step recorded");
        } catch (...) {
          capture_fail_test_ = false;
          end_failed_capture();
          presend_done_ = presend_saved_;
          bwd_blocks_issued_ = blocks_saved;
          throw;
        }
        HIP_CHECK(hipStreamEndCapture(s_comp_, &g));
        if (markers_) marker("capture: ended");
        // CHANNEL_GRAPH_DOT=<prefix>: the captured step graph as <prefix>_r<rank>_g<gi>.dot (topology
        // diagnosis: which nodes and cross-stream edges a replay has to honour)
        if (const char* dp = std::getenv("CHANNEL_GRAPH_DOT")) {
          const std::string path = std::string(dp) + "_r" + std::to_string(plan_.rank) + "_g" + std::to_string(gi) + ".dot";
          if (hipGraphDebugDotPrint(g, path.c_str(), 0) != hipSuccess) (void)hipGetLastError();
        }
        HIP_CHECK(hipGraphInstantiate(&gexec_[gi], g, nullptr, nullptr, 0));
        if (markers_) marker("capture: instantiated");
        (void)hipGraphDestroy(g);
      } catch (const Error& e) {
        std::cerr << "[channel] hipGraph capture failed, running eagerly: " << e.what() << "\n";
        (void)hipGetLastError();
        gexec_[gi] = nullptr;
        use_graph_ = false;
      }
      graph_ok_[gi] = true;
      captured_now = true;
      if (comm_) {
        // every rank must replay the same exchange sequence: if capture failed anywhere, all ranks
        // drop their graphs and step eagerly (no rank may launch a captured RCCL sequence that a
        // peer runs eagerly in a different order).  An error here aborts every communicator, so
        // the peers waiting in this allreduce fail too instead of hanging.
        unsigned* flag = d_health_ + 1;
        const unsigned mine = gexec_[gi] ? 0u : 1u;
        unsigned any = 0;
        try {
          HIP_CHECK(hipMemcpyAsync(flag, &mine, sizeof(unsigned), hipMemcpyHostToDevice, s_comm_));
          comm_->allreduce_max_u32(flag, 1, s_comm_);
          HIP_CHECK(hipMemcpyAsync(&any, flag, sizeof(unsigned), hipMemcpyDeviceToHost, s_comm_));
          wait(s_comm_);
        } catch (...) {
          abort_comms();
          throw;
        }
        HIP_CHECK(hipMemsetAsync(flag, 0, sizeof(unsigned), s_comm_));
        if (any) {
          if (gexec_[gi]) {
            (void)hipGraphExecDestroy(gexec_[gi]);
            gexec_[gi] = nullptr;
            std::cerr << "[channel] hipGraph capture failed on a peer rank: every rank runs eagerly\n";
          }
          presend_done_ = presend_saved_;  // the dropped graph never ran its pre-send
          bwd_blocks_issued_ = blocks_saved;
          use_graph_ = false;
        }
      }
    }
    if (gexec_[gi]) {
      HIP_CHECK(hipGraphLaunch(gexec_[gi], s_comp_));
      if (markers_ && !replayed_[gi]) marker("graph launched");
      done = true;
    }
  }
  if (!done) step_body(stats_for_next);
  comm_warm_ = true;
  if (markers_) {
    if (warmup_step) {
      synchronize();
      marker("eager warm-up step done (RCCL peers connected)");
    }
    if (captured_now) marker(gexec_[gi] ? "step graph captured" : "step graph not captured: stepping eagerly");
    // eager steps (no graph, e.g. the host-driven loopback transport): one line per step issued
    if (!done && !warmup_step) marker("eager step issued");
    if (done && !replayed_[gi]) {
      synchronize();
      replayed_[gi] = true;
      marker(gi ? "first replay of the statistics step graph done" : "first replay of the step graph done");
    }
  }
  if (step_timing_) HIP_CHECK(hipEventRecord(step_ev_[step_ev_used_++].second, s_comp_));
  if (phase_timing_) flush_phase_events();
  if (stats_for_next) stats_pending_ = true;
  ++nstep_;
}

void Solver::substep_debug(int n) {
  if (!prepared_) prepare();
  transforms(n, false);
  kspec(1, n, false);
}

void Solver::transforms_debug(bool dt_upd) {
  transforms(dt_upd ? 0 : 1, false);
  join_forward();
}

// the compute stream waits for every block of a split forward exchange (no K-SPEC follows)
void Solver::join_forward() {
  if (!fwd_pending_) return;
  HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_fb_.back(), 0));
  fwd_pending_ = false;
}

// P > 1: poll instead of blocking so that a dead or hung peer (RCCL async error, or no progress
// for CHANNEL_COMM_TIMEOUT_S seconds) aborts the communicator and raises on every surviving rank
// instead of hanging the job (the reference's exit(1) left peers blocked in MPI, check.cu:67-79).
void Solver::wait(hipStream_t s) {
  if (!comm_) {
    HIP_CHECK(hipStreamSynchronize(s));
    return;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (int it = 0;; ++it) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) HIP_CHECK(e);
    if (comm_failed()) {
      abort_comms();
      CH_CHECK(false, "communicator failure on rank " << plan_.rank << " (peer died or network error)");
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (comm_timeout_s_ > 0 && el > comm_timeout_s_) {
      abort_comms();
      CH_CHECK(false, "rank " << plan_.rank << ": no progress for " << comm_timeout_s_ << " s; communicator aborted");
    }
    if (it > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

void Solver::abort_comms() {
  if (comm_row_) comm_row_->abort();
  if (comm_col_) comm_col_->abort();
  if (comm_) comm_->abort();
}

bool Solver::comm_failed() {
  return comm_->async_error() || (comm_col_ && comm_col_->async_error()) || (comm_row_ && comm_row_->async_error());
}

void Solver::wait_event(hipEvent_t e) {
  if (!comm_) {
    HIP_CHECK(hipEventSynchronize(e));
    return;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (int it = 0;; ++it) {
    const hipError_t r = hipEventQuery(e);
    if (r == hipSuccess) return;
    if (r != hipErrorNotReady) HIP_CHECK(r);
    if (comm_failed()) {
      abort_comms();
      CH_CHECK(false, "communicator failure on rank " << plan_.rank << " (peer died or network error)");
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (comm_timeout_s_ > 0 && el > comm_timeout_s_) {
      abort_comms();
      CH_CHECK(false, "rank " << plan_.rank << ": no progress for " << comm_timeout_s_ << " s; communicator aborted");
    }
    if (it > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

void Solver::synchronize() {
  wait(s_comp_);
  wait(s_comm_);
}

void Solver::barrier() {
  if (comm_) {
    // tiny allreduce as a device barrier, then host sync
    comm_->allreduce_max_u32(d_health_, 1, s_comm_);
    wait(s_comm_);
  }
  synchronize();
}

double Solver::max_over_ranks(double v) {
  if (!comm_) return v;
  synchronize();
  HIP_CHECK(hipMemcpy(d_red_, &v, sizeof(double), hipMemcpyHostToDevice));
  comm_->allreduce_max_f64(d_red_, 1, s_comm_);
  wait(s_comm_);
  HIP_CHECK(hipMemcpy(&v, d_red_, sizeof(double), hipMemcpyDeviceToHost));
  return v;
}

StepLog Solver::log() {
  synchronize();
  StepLog L;
  double dl[8];
  HIP_CHECK(hipMemcpy(dl, d_dtlog_, sizeof(dl), hipMemcpyDeviceToHost));
  L.step = nstep_;
  L.umax = dl[0];
  L.vmax = dl[1];
  L.wmax = dl[2];
  L.cflsum = dl[3];
  L.dt_c = dl[4];
  L.dt_v = dl[5];
  L.dt = dl[6];
  L.time = dl[7];
  const int N = plan_.NY;
  if (plan_.owns_mean()) {
    double md[4];
    HIP_CHECK(hipMemcpy(md, d_mean_ + 3 * N, sizeof(md), hipMemcpyDeviceToHost));
    L.dUdy_lo = md[0];
    L.dUdy_hi = md[1];
    L.flux = md[2];
    L.dpdx = md[3];
    const double nu = 1.0 / cfg_.Re;
    L.utau_lo = std::sqrt(nu * std::fabs(L.dUdy_lo));
    L.utau_hi = std::sqrt(nu * std::fabs(L.dUdy_hi));
    L.utau = std::sqrt(0.5 * (L.utau_lo * L.utau_lo + L.utau_hi * L.utau_hi));
  }
  L.health = health();
  return L;
}

unsigned Solver::health() {
  if (comm_) {
    comm_->allreduce_max_u32(d_health_, 1, s_comm_);
    wait(s_comm_);
  }
  unsigned h = 0;
  HIP_CHECK(hipMemcpy(&h, d_health_, sizeof(h), hipMemcpyDeviceToHost));
  return h;
}

std::vector<double> Solver::stats() {
  synchronize();
  std::vector<double> s(4 * plan_.NY);
  HIP_CHECK(hipMemcpy(s.data(), d_stats_, s.size() * sizeof(double), hipMemcpyDeviceToHost));
  return s;
}

std::vector<double> Solver::mean_profile() {
  synchronize();
  std::vector<double> U(plan_.NY, 0.0);
  if (plan_.owns_mean()) HIP_CHECK(hipMemcpy(U.data(), d_mean_, U.size() * sizeof(double), hipMemcpyDeviceToHost));
  return U;
}

void Solver::symmetrize() {
  const Plan& p = plan_;
  if (!comm_) {
    symmetrize_kz0(field_ptr(PHI), p.NY, p.nkx, nkzs_, p.Kx, kzb_, fp64_, s_comp_);
    symmetrize_kz0(field_ptr(OMEGA), p.NY, p.nkx, nkzs_, p.Kx, kzb_, fp64_, s_comp_);
    prepared_ = false;
    return;
  }
  // distributed: the kz = 0 column lives on the ranks of process row 0 (slab: every rank)
  const bool has_kz0 = p.kz0 == 0;
  const size_t loc = static_cast<size_t>(p.NY) * p.nkx_loc, all = static_cast<size_t>(p.NY) * p.nkx;
  if (!d_sym_) HIP_CHECK(hipMalloc(&d_sym_, 2 * (loc + all) * esz_));
  char* col_loc = static_cast<char*>(d_sym_);
  char* col_all = col_loc + 2 * loc * esz_;
  std::vector<A2ABlock> ops(2);
  for (int f = 0; f < 2; ++f) {
    A2ABlock& o = ops[f];
    o.scount.assign(p.P, 0);
    o.soff.assign(p.P, 0);
    o.rcount.assign(p.P, 0);
    o.roff.assign(p.P, 0);
    o.send = col_loc + f * loc * esz_;
    o.recv = col_all + f * all * esz_;
    if (has_kz0) {
      for (int c = 0; c < p.Pc; ++c) {
        const int g = p.rank_of(p.prow, c);
        o.scount[g] = loc * esz_;
        o.rcount[g] = static_cast<size_t>(p.NY) * p.kx_split.count[c] * esz_;
        o.roff[g] = static_cast<size_t>(p.NY) * p.kx_split.start[c] * esz_;
      }
    }
    if (has_kz0)  // per kx sub-block: col_loc = [b][y][kx in b], i.e. global kx order again
      for (int b = 0; b < nkb_; ++b)
        kz0_pack(static_cast<char*>(field_ptr(f == 0 ? PHI : OMEGA)) + kb_off_[b] * esz_,
                 col_loc + (f * loc + static_cast<size_t>(p.NY) * kb_start_[b]) * esz_, p.NY, kb_cnt_[b], nkzs_, kzb_,
                 fp64_, s_comp_);
  }
  HIP_CHECK(hipEventRecord(ev_stats_, s_comp_));
  HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_stats_, 0));
  comm_->alltoallv_batch(ops, s_comm_);
  HIP_CHECK(hipEventRecord(ev_stats_, s_comm_));
  HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_stats_, 0));
  if (has_kz0) {
    Kz0SymArgs a;
    a.N = p.NY;
    a.nkz_loc = nkzs_;  // (the line stride)
    a.kzb = kzb_;
    a.nkx = p.nkx;
    a.nblk = p.Pc * nkb_;  // gathered blocks (c, b) in global kx order
    for (int c = 0; c < p.Pc; ++c)
      for (int b = 0; b < nkb_; ++b) a.kx_start[c * nkb_ + b] = kb_gstart(c, b);
    a.kx_start[a.nblk] = p.nkx;
    for (int f = 0; f < 2; ++f)
      for (int b = 0; b < nkb_; ++b) {
        a.nkx_loc = kb_cnt_[b];
        a.kx0 = p.kx0 + kb_start_[b];
        kz0_symmetrize_dist(static_cast<char*>(field_ptr(f == 0 ? PHI : OMEGA)) + kb_off_[b] * esz_,
                            col_all + f * all * esz_, a, fp64_, s_comp_);
      }
  }
  prepared_ = false;
}

// ---- reference-style run loop with stdout blocks and .dat files --------------------------------
void Solver::write_logs(const StepLog& L, bool verbose) {
  if (plan_.rank != 0) return;
  const int N = plan_.NY, NX = plan_.NX, NZ = plan_.NZ, Nzp = plan_.Nzp;
  const double nu = 1.0 / cfg_.Re, LY = 2.0, Um = cfg_.Q / LY;
  const double N2 = static_cast<double>(NX) * Nzp;
  std::vector<double> U = mean_profile();
  std::vector<double> Nm(N, 0.0);
  HIP_CHECK(hipMemcpy(Nm.data(), d_mean_ + N, N * sizeof(double), hipMemcpyDeviceToHost));
  const double Uc = U[N / 2], ut = L.utau;
  const auto& y = grid_.y;
  const double dyc = y[N / 2 + 1] - y[N / 2], dyw = y[1] - y[0];
  if (verbose) {
    std::printf("*****RK_STATISTICS****\nmax_V=(%e,%e,%e)\n(dt_c,dt_v)=(%f,%f)\n", L.umax, L.vmax, L.wmax, L.dt_c,
                L.dt_v);
    std::printf("(time,counter)=(%f,%ld)\n", L.time, L.step);
    std::printf("(tau_1,tau_2)=(%e,%e)\n****MEAN_PROFILE_STATISTICS****\n", L.utau_lo, L.utau_hi);
    std::printf("(RE_t,RE_c,RE_m)=(%e,%e,%e)\n", ut * LY * 0.5 / nu, Uc * 0.5 * LY / nu, 1.0 / nu);
    std::printf("(Dx+,Dz+)=(%e,%e)\n", 1.5 * ut * cfg_.LX / (nu * NX), 1.5 * ut * cfg_.LZ / (nu * Nzp));
    std::printf("Dy+(max,min)=(%f,%f)\n", ut * dyc / nu, ut * dyw / nu);
    std::printf("C_f=%e\n", ut > 0 ? 2.0 * ut * ut / (Um * Um) : 0.0);
    std::printf("(Um+,Ux+,Um/Uc)=(%f,%f,%f)\n", ut > 0 ? Um / ut : 0.0, ut > 0 ? Uc / ut : 0.0, Uc != 0 ? Um / Uc : 0.0);
    std::fflush(stdout);
  }
  const std::string& pth = cfg_.path;
  auto app = [&](const char* name) { return std::ofstream(pth + name, std::ios::app); };
  {
    auto f = app("MEANPROFILE.dat");
    for (int j = 0; j < N; ++j) f << " " << std::fixed << U[j] * N2;
    f << " \n";
  }
  {
    auto f = app("MEANREAYNOLDS.dat");
    for (int j = 0; j < N; ++j) f << " " << std::fixed << Nm[j] * N2;
    f << " \n";
  }
  {
    auto f = app("UTAU.dat");
    f << " " << std::fixed << ut << "\n";
  }
  {
    auto f = app("STATISTICS.dat");
    f << std::scientific << ut * LY * 0.5 / nu << " " << Uc * 0.5 * LY / nu << " " << 1.0 / nu << " "
      << (ut > 0 ? Um / ut : 0.0) << " " << (ut > 0 ? Uc / ut : 0.0) << " " << (Uc != 0 ? Um / Uc : 0.0) << " "
      << 2.0 * ut * ut / (Um * Um) << " " << (Uc != 0 ? 2.0 * ut * ut / (Uc * Uc) : 0.0) << " \n";
  }
  {
    auto f = app("RESOLUTION.dat");
    f << std::fixed << 1.5 * ut * cfg_.LX / (nu * NX) << " " << 1.5 * ut * cfg_.LZ / (nu * Nzp) << " "
      << ut * dyc / nu << " " << ut * dyw / nu << "\n";
  }
  (void)NZ;
}

void Solver::write_stats_files(const std::vector<double>& st) {
  if (plan_.rank != 0) return;
  const int N = plan_.NY;
  auto app = [&](const char* name) { return std::ofstream(cfg_.path + name, std::ios::app); };
  auto sgn_sqrt = [](double x) { return x >= 0 ? std::sqrt(x) : -std::sqrt(-x); };
  {
    auto f = app("RSTRSS.dat");
    for (int j = 0; j < N; ++j) f << " " << std::fixed << sgn_sqrt(-st[3 * N + j]);
    f << " \n";
  }
  const char* names[3] = {"URMS.dat", "VRMS.dat", "WRMS.dat"};
  for (int s = 0; s < 3; ++s) {
    auto f = app(names[s]);
    for (int j = 0; j < N; ++j) f << " " << std::fixed << std::sqrt(std::max(0.0, st[s * N + j]));
    f << " \n";
  }
}

void Solver::run(long nsteps, bool verbose) {
  if (!prepared_) prepare();
  const int se = cfg_.stats_every, le = cfg_.log_every, ce = cfg_.checkpoint_every, ye = cfg_.symmetry_every;
  const int he = cfg_.health_every, pe = cfg_.spectra_every;
  const bool rb = cfg_.on_nan == "rollback";
  const int sn = cfg_.snapshot_every > 0 ? cfg_.snapshot_every : he;
  if (stats_pending_ && se > 0 && nstep_ % se == 0) write_stats_files(stats());
  stats_pending_ = false;
  if (rb && snap_step_ < 0) take_snapshot();
  tdt_valid_ = false;  // the state may have been reset or restored since the last run()
  auto t_log = std::chrono::steady_clock::now();
  long s_log = nstep_;
  for (long s = 0; s < nsteps; ++s) {
    const bool want_stats = se > 0 && (nstep_ + 1) % se == 0;
    step(want_stats);
    if (want_stats) {
      write_stats_files(stats());
      stats_pending_ = false;
    }
    const bool do_log = le > 0 && nstep_ % le == 0;
    if (do_log || (cfg_.health_check && nstep_ % he == 0)) {
      StepLog L = log();
      if (L.health) {
        if (rb && rollbacks_ < cfg_.max_rollbacks && snap_step_ >= 0) {
          const long lost = nstep_ - snap_step_;
          if (plan_.rank == 0)
            std::fprintf(stderr, "[channel] non-finite state at step %ld; rolling back to step %ld, cfl %g -> %g\n",
                         L.step, snap_step_, cfg_.cfl, cfg_.cfl * cfg_.rollback_cfl_factor);
          rollback();
          s = std::max(-1L, s - lost);  // the lost steps are redone
          continue;
        }
        std::fprintf(stderr, "[channel] non-finite state detected at step %ld (t=%g, dt=%g); aborting\n", L.step,
                     L.time, L.dt);
        if (comm_) abort_comms();
        CH_CHECK(false, "health check failed at step " << L.step);
      }
      if (rb && nstep_ - snap_step_ >= sn) take_snapshot();
      if (do_log) {
        const auto t = std::chrono::steady_clock::now();
        const double ms = 1e3 * std::chrono::duration<double>(t - t_log).count() / std::max(1L, nstep_ - s_log);
        t_log = t;
        s_log = nstep_;
        write_logs(L, verbose);
        write_json(L, ms);
      }
    }
    if (pe > 0 && nstep_ % pe == 0) write_spectra_files(spectra());
    if (ye > 0 && nstep_ % ye == 0) {
      symmetrize();
      prepare();
    }
    if (ce > 0 && nstep_ % ce == 0 && cfg_.out_G != "-") {
      const std::string sfx = "." + std::to_string(nstep_);
      const std::string um = cfg_.out_UMEAN != "-" ? cfg_.out_UMEAN + sfx : "-";
      if (cfg_.checkpoint_async) checkpoint_async(cfg_.out_G + sfx, cfg_.out_DDV + sfx, um);
      else write_restart(cfg_.out_G + sfx, cfg_.out_DDV + sfx, um);
    }
    if (cfg_.t_end > 0 && t_end_reached()) break;
  }
  synchronize();
  wait_checkpoint();
}

// t_end without a host sync per step (which would drain the CPU's run-ahead of the GPU): (dt, time)
// of every step is copied to pinned memory behind the step, and the decision after step s reads the
// copy of step s-1, which has finished while step s runs.  When that time is within one step's
// largest advance of t_end (dt_max, or dt_fixed when set) it reads the device time synchronously,
// so the run still stops at the first step whose end time reaches t_end.
bool Solver::t_end_reached() {
  if (!h_tdt_) {
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_tdt_), 4 * sizeof(double), hipHostMallocDefault));
    for (auto& e : ev_tdt_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    tdt_valid_ = false;
  }
  const int cur = static_cast<int>(nstep_ & 1);
  HIP_CHECK(hipMemcpyAsync(h_tdt_ + 2 * cur, d_dt_, 2 * sizeof(double), hipMemcpyDeviceToHost, s_comp_));
  HIP_CHECK(hipEventRecord(ev_tdt_[cur], s_comp_));
  const bool have_prev = tdt_valid_;
  tdt_valid_ = true;
  if (have_prev) {
    wait_event(ev_tdt_[cur ^ 1]);
    const double dt = h_tdt_[2 * (cur ^ 1)], t = h_tdt_[2 * (cur ^ 1) + 1];  // d_dt_, d_time_ adjacent
    // the step just queued advances the time by at most dt_max (dt_fixed when set): only within
    // that margin of t_end is the device time read synchronously (dt can jump to dt_max at once,
    // e.g. from a zero-velocity state, so a multiple of the previous dt is no bound)
    const double margin = cfg_.dt_fixed > 0.0 ? cfg_.dt_fixed : cfg_.dt_max;
    if (margin > 0.0 && t + (1.0 + 1e-12) * margin < cfg_.t_end) return false;
    (void)dt;
  }
  return time() >= cfg_.t_end;
}

// ---- failure handling ------------------------------------------------------------------------------
void Solver::invalidate_graphs() {
  HIP_CHECK(hipStreamSynchronize(s_comp_));
  for (int i = 0; i < 2; ++i) {
    if (gexec_[i]) (void)hipGraphExecDestroy(gexec_[i]);
    gexec_[i] = nullptr;
    graph_ok_[i] = false;
  }
}

void Solver::take_snapshot() {
  const size_t fb = spec_ * esz_;
  if (!snap_) HIP_CHECK(hipMalloc(&snap_, 2 * fb + 2 * sizeof(double)));
  char* d = static_cast<char*>(snap_);
  HIP_CHECK(hipMemcpyAsync(d, field_ptr(PHI), fb, hipMemcpyDeviceToDevice, s_comp_));
  HIP_CHECK(hipMemcpyAsync(d + fb, field_ptr(OMEGA), fb, hipMemcpyDeviceToDevice, s_comp_));
  HIP_CHECK(hipMemcpyAsync(d + 2 * fb, d_dt_, 2 * sizeof(double), hipMemcpyDeviceToDevice, s_comp_));
  snap_step_ = nstep_;
}

void Solver::rollback() {
  CH_CHECK(snap_ && snap_step_ >= 0, "rollback: no snapshot");
  synchronize();
  const size_t fb = spec_ * esz_;
  char* d = static_cast<char*>(snap_);
  HIP_CHECK(hipMemcpyAsync(field_ptr(PHI), d, fb, hipMemcpyDeviceToDevice, s_comp_));
  HIP_CHECK(hipMemcpyAsync(field_ptr(OMEGA), d + fb, fb, hipMemcpyDeviceToDevice, s_comp_));
  HIP_CHECK(hipMemcpyAsync(d_dt_, d + 2 * fb, 2 * sizeof(double), hipMemcpyDeviceToDevice, s_comp_));
  HIP_CHECK(hipMemsetAsync(field_ptr(RPHI), 0, 2 * fb, s_comp_));  // zeta_0 = 0: R is not needed at substep 0
  HIP_CHECK(hipMemsetAsync(d_max_, 0, 4 * sizeof(float), s_comp_));
  HIP_CHECK(hipMemsetAsync(d_health_, 0, sizeof(unsigned), s_comp_));
  HIP_CHECK(hipStreamSynchronize(s_comp_));
  nstep_ = snap_step_;
  tdt_valid_ = false;  // the lagged (dt, time) copy belongs to the discarded steps
  ++rollbacks_;
  cfg_.cfl *= cfg_.rollback_cfl_factor;  // captured as a kernel argument: re-capture the graphs
  invalidate_graphs();
  prepared_ = false;
  prepare();
}

void Solver::inject_nan(int f) {
  presend_done_ = false;
  // an interior point of line 1 of the field (line 0 on the owner rank holds U)
  const size_t elem = plan_.nkz_loc > 1 ? dev_index(plan_.NY / 2, 0, 1) : dev_index(plan_.NY / 2, std::min(1, plan_.nkx_loc - 1), 0);
  ::channel::inject_nan(field_ptr(f), elem, fp64_, s_comp_);
  HIP_CHECK(hipStreamSynchronize(s_comp_));
}

// ---- spectra --------------------------------------------------------------------------------------
Solver::Spectra Solver::spectra() {
  const Plan& p = plan_;
  Spectra out;
  out.planes = cfg_.spectra_plane_list();
  const int np = static_cast<int>(out.planes.size());
  const size_t nx = 3 * np * (p.Kx + 1), nz = 3 * np * p.nkz, nm = 3 * static_cast<size_t>(p.nkx) * p.nkz;
  const size_t need = (nx + nz + nm) * sizeof(double) + np * sizeof(int);
  if (spec_n_ < need) {
    if (d_spec_) HIP_CHECK(hipFree(d_spec_));
    HIP_CHECK(hipMalloc(&d_spec_, need));
    spec_n_ = need;
  }
  double* ekx = static_cast<double*>(d_spec_);
  double* ekz = ekx + nx;
  double* map = ekz + nz;
  int* planes = reinterpret_cast<int*>(map + nm);
  HIP_CHECK(hipMemsetAsync(d_spec_, 0, (nx + nz + nm) * sizeof(double), s_comp_));
  HIP_CHECK(hipMemcpyAsync(planes, out.planes.data(), np * sizeof(int), hipMemcpyHostToDevice, s_comp_));
  SpectraArgs a;
  a.dv = field_ptr(OUT0);
  a.v = field_ptr(OUT1);
  a.om = field_ptr(OMEGA);
  a.ax = p.ax;
  a.az = p.az;
  a.combine = combine_ ? 1 : 0;
  a.u = field_ptr(OUT0);
  a.w = field_ptr(OUT2);
  a.lines = p.nkx_loc * nkzs_;
  a.nkx_loc = p.nkx_loc;
  a.kx0 = p.kx0;
  a.nkz_loc = p.nkz_loc;
  a.nkzs = nkzs_;
  a.kzb = kzb_;
  a.kz0 = p.kz0;
  a.nkx = p.nkx;
  a.Kx = p.Kx;
  a.nkz = p.nkz;
  a.planes = planes;
  a.nplanes = np;
  a.ekx = ekx;
  a.ekz = ekz;
  a.map = map;
  for (int b = 0; b < nkb_; ++b) {  // per kx sub-block (accumulating; map rows are disjoint)
    SpectraArgs ab = a;
    const size_t off = kb_off_[b] * esz_;
    ab.dv = static_cast<const char*>(a.dv) + off;
    ab.v = static_cast<const char*>(a.v) + off;
    ab.om = static_cast<const char*>(a.om) + off;
    ab.u = static_cast<const char*>(a.u) + off;
    ab.w = static_cast<const char*>(a.w) + off;
    ab.lines = kb_cnt_[b] * nkzs_;
    ab.nkx_loc = kb_cnt_[b];
    ab.kx0 = p.kx0 + kb_start_[b];
    spectra_accumulate(ab, fp64_, s_comp_);
  }
  if (comm_) {
    HIP_CHECK(hipEventRecord(ev_stats_, s_comp_));
    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_stats_, 0));
    comm_->allreduce_sum_f64(ekx, nx + nz + nm, s_comm_);
    wait(s_comm_);
  }
  synchronize();
  out.ekx.resize(nx);
  out.ekz.resize(nz);
  out.map.resize(nm);
  HIP_CHECK(hipMemcpy(out.ekx.data(), ekx, nx * sizeof(double), hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(out.ekz.data(), ekz, nz * sizeof(double), hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemcpy(out.map.data(), map, nm * sizeof(double), hipMemcpyDeviceToHost));
  return out;
}

void Solver::write_spectra_files(const Spectra& sp) {
  if (plan_.rank != 0) return;
  const Plan& p = plan_;
  const int np = static_cast<int>(sp.planes.size());
  const double N2 = static_cast<double>(p.NX) * p.Nzp;
  // reference layout (statistics.cu:272-320): NX rows (FFT-order kx) x NZ columns of |q|^2 in the
  // file units (N2 * coefficient), plane planes[0]; overwritten each time like the reference's "w"
  const char* maps[3] = {"Uspec.dat", "Vspec.dat", "Wspec.dat"};
  for (int q = 0; q < 3; ++q) {
    std::ofstream f(cfg_.path + maps[q]);
    std::vector<int> ig_of_pos(p.NX, -1);
    for (int i = 0; i < p.nkx; ++i) ig_of_pos[p.kx_fft_pos(i)] = i;
    for (int x = 0; x < p.NX; ++x) {
      for (int kz = 0; kz < p.NZ; ++kz) {
        double v = 0.0;
        if (ig_of_pos[x] >= 0 && kz < p.nkz) v = sp.map[(static_cast<size_t>(q) * p.nkx + ig_of_pos[x]) * p.nkz + kz];
        f << " " << std::fixed << v * N2 * N2;
      }
      f << " \n";
    }
  }
  // time series of 1-D spectra (true-coefficient units): one line per (plane, component)
  auto app = [&](const char* name) { return std::ofstream(cfg_.path + name, std::ios::app); };
  auto fx = app("SPECTRA_KX.dat");
  auto fz = app("SPECTRA_KZ.dat");
  double hv[2];
  HIP_CHECK(hipMemcpy(hv, d_dt_, sizeof(hv), hipMemcpyDeviceToHost));
  for (int pl = 0; pl < np; ++pl)
    for (int q = 0; q < 3; ++q) {
      fx << nstep_ << " " << std::scientific << hv[1] << " " << sp.planes[pl] << " " << "uvw"[q];
      for (int k = 0; k <= p.Kx; ++k) fx << " " << sp.ekx[(static_cast<size_t>(q) * np + pl) * (p.Kx + 1) + k];
      fx << "\n";
      fz << nstep_ << " " << std::scientific << hv[1] << " " << sp.planes[pl] << " " << "uvw"[q];
      for (int k = 0; k < p.nkz; ++k) fz << " " << sp.ekz[(static_cast<size_t>(q) * np + pl) * p.nkz + k];
      fz << "\n";
    }
}

void Solver::write_json(const StepLog& L, double ms_per_step) {
  if (plan_.rank != 0 || cfg_.log_json.empty()) return;
  std::ofstream f(cfg_.log_json, std::ios::app);
  const double nu = 1.0 / cfg_.Re;
  std::ostringstream o;
  o.precision(9);
  o << "{\"step\": " << L.step << ", \"time\": " << L.time << ", \"dt\": " << L.dt << ", \"cfl\": " << L.cflsum * L.dt
    << ", \"umax\": " << L.umax << ", \"vmax\": " << L.vmax << ", \"wmax\": " << L.wmax << ", \"utau\": " << L.utau
    << ", \"Re_tau\": " << L.utau / nu << ", \"flux\": " << L.flux << ", \"dpdx\": " << L.dpdx
    << ", \"health\": " << L.health << ", \"rollbacks\": " << rollbacks_ << ", \"ms_per_step\": " << ms_per_step
    << ", \"ranks\": " << plan_.P << ", \"grid\": [" << plan_.NX << ", " << plan_.NY << ", " << plan_.Nzp << "]";
  if (phase_timing_) {
    o << ", \"phase_ms\": [";
    for (size_t i = 0; i < 4; ++i) o << (i ? ", " : "") << ph_ms_[i];
    o << "]";
  }
  o << "}\n";
  f << o.str();
}

// ---- restart I/O (Appendix B) --------------------------------------------------------------------
// A restart is taken in two parts: capture (synchronous: device state -> host copy, at a step
// boundary) and write (HDF5 planes of this rank into the one shared file, the ranks taking turns).
// write_restart does both now; checkpoint_async hands the write to a background thread (the time
// stepping continues) and the ranks pass the file between them through marker files, so the
// background writers never touch the communicator.  The reference wrote only at the end, gathering
// every plane on rank 0 with an MPI_Barrier per plane (hit_mpi.c:257-339, main.c:139-144).
Solver::RestartJob Solver::capture_restart(const std::string& g, const std::string& ddv, const std::string& umean) {
  RestartJob j;
  j.g = g;
  j.ddv = ddv;
  j.umean = umean;
  j.phi.resize(canon_);
  j.om.resize(canon_);
  j.U.resize(plan_.NY);
  get_state(j.phi.data(), j.om.data(), j.U.data());
  double hv[2];
  HIP_CHECK(hipMemcpy(hv, d_dt_, sizeof(hv), hipMemcpyDeviceToHost));
  j.dt = hv[0];
  j.time = hv[1];
  j.step = nstep_;
  j.serial = ++ckpt_serial_;
  return j;
}

void Solver::write_restart_job(const RestartJob& j, const std::function<void(int)>& turn) {
  const Plan& p = plan_;
  const int N = p.NY, NZ = p.NZ, lines = p.lines_loc();
  const double N2 = static_cast<double>(p.NX) * p.Nzp;
  std::vector<int> planes(p.nkx_loc);
  for (int i = 0; i < p.nkx_loc; ++i) planes[i] = p.kx_fft_pos(p.kx0 + i);
  // pencil ranks own a kz range of each plane: read-modify-write (ranks take turns)
  auto pack = [&](const std::vector<std::complex<double>>& f, std::vector<double>& d) {
    for (int i = 0; i < p.nkx_loc; ++i)
      for (int kzl = 0; kzl < p.nkz_loc; ++kzl)
        for (int jy = 0; jy < N; ++jy) {
          const auto v = f[static_cast<size_t>(jy) * lines + i * p.nkz_loc + kzl] * N2;
          const size_t o = ((static_cast<size_t>(i) * NZ + p.kz0 + kzl) * N + jy) * 2;
          d[o] = v.real();
          d[o + 1] = v.imag();
        }
  };
  std::map<std::string, double> attrs = {{"time", j.time}, {"dt", j.dt}, {"step", static_cast<double>(j.step)},
                                         {"Re", cfg_.Re},  {"Q", cfg_.Q},   {"LX", cfg_.LX},
                                         {"LZ", cfg_.LZ},  {"NX", double(p.NX)}, {"NY", double(N)},
                                         {"NZ", double(NZ)}, {"format_version", 2.0},
                                         {"fp64", fp64_ ? 1.0 : 0.0}};
  int stage = 0;
  for (int which = 0; which < 2; ++which) {
    const std::string& path = which == 0 ? j.g : j.ddv;
    if (path.empty() || path == "-") continue;
    for (int r = 0; r < p.P; ++r) {
      turn(stage * p.P + r);
      if (r != p.rank) continue;
      if (r == 0) {
        // fp64 storage writes H5T_NATIVE_DOUBLE (the reference's unused double writers,
        // hit_mpi.c:92-255); fp32 keeps the reference's float dataset
        h5_create_field(path, p.NX, N, NZ, fp64_, p.Kx);
        h5_write_attrs(path, attrs);
        // U(y) in full precision next to "u" (the UMEAN file keeps the reference's float32 records)
        if (which == 0 && p.owns_mean()) {
          std::vector<double> u(N);
          for (int jy = 0; jy < N; ++jy) u[jy] = j.U[jy] * N2;
          h5_write_vector(path, "umean", u);
        }
      }
      std::vector<double> data(static_cast<size_t>(p.nkx_loc) * NZ * N * 2, 0.0);
      if (p.pencil()) {
        int dims[3];
        h5_read_planes(path, planes, data, dims);
      }
      pack(which == 0 ? j.om : j.phi, data);
      h5_write_planes(path, planes, data);
    }
    ++stage;
  }
  turn(stage * p.P);  // everybody done
  if (p.owns_mean() && !j.umean.empty() && j.umean != "-") {
    std::vector<double> u(N);
    for (int jy = 0; jy < N; ++jy) u[jy] = j.U[jy] * N2;
    umean_write(j.umean, u);
  }
}

void Solver::write_restart(const std::string& g, const std::string& ddv, const std::string& umean) {
  wait_checkpoint();
  const RestartJob j = capture_restart(g, ddv, umean);
  // synchronous: the ranks take turns at device barriers
  write_restart_job(j, [this](int) { barrier(); });
  barrier();
}

void Solver::checkpoint_async(const std::string& g, const std::string& ddv, const std::string& umean) {
  wait_checkpoint();
  RestartJob j = capture_restart(g, ddv, umean);
  const int P = plan_.P, rank = plan_.rank;
  const double timeout = comm_timeout_s_ > 0 ? comm_timeout_s_ : 3600.0;
  ckpt_thread_ = std::thread([this, j = std::move(j), P, rank, timeout]() {
    try {
      // turn t belongs to rank t % P: rank r waits for the marker "<g>.turn" holding
      // "<run nonce> <serial> <t>" written by the previous writer (atomic rename), then passes it
      // on.  The nonce (from the communicator id) keeps a marker left behind by a crashed earlier
      // run of the same path from ever matching; rank 0 also removes any marker before its first
      // turn (it writes first, so nobody can be waiting on a current one yet).
      const std::string marker = (j.g != "-" ? j.g : j.ddv) + ".turn";
      const std::string tag = std::to_string(run_nonce_) + " " + std::to_string(j.serial) + " ";
      if (P > 1 && rank == 0) std::remove(marker.c_str());
      auto wait_turn = [&](int t) {
        if (P == 1 || t == 0) return;
        const std::string want = tag + std::to_string(t);
        const auto t0 = std::chrono::steady_clock::now();
        while (true) {
          std::ifstream f(marker);
          std::string line;
          if (f.good() && std::getline(f, line) && line == want) return;
          CH_CHECK(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < timeout,
                   "checkpoint: rank " << rank << " timed out waiting for its turn (" << want << ")");
          std::this_thread::sleep_for(std::chrono::milliseconds(2));
        }
      };
      auto pass_turn = [&](int t) {
        if (P == 1) return;
        const std::string tmp = marker + "." + std::to_string(rank);
        {
          std::ofstream f(tmp, std::ios::trunc);
          f << tag << t << "\n";
        }
        CH_CHECK(std::rename(tmp.c_str(), marker.c_str()) == 0, "checkpoint: cannot update " << marker);
      };
      // write step t belongs to rank t % P; turn(t) is called by every rank for every t in order,
      // so a rank's write at turn `last` is complete when it sees the next turn index
      int last = -1;
      write_restart_job(j, [&](int t) {
        if (last >= 0 && last % P == rank) pass_turn(last + 1);
        if (t % P == rank) wait_turn(t);  // rank 0's final turn waits until every rank has written
        last = t;
      });
      if (P > 1 && rank == 0) std::remove(marker.c_str());
    } catch (...) {
      ckpt_error_ = std::current_exception();
    }
  });
}

void Solver::wait_checkpoint() {
  if (ckpt_thread_.joinable()) ckpt_thread_.join();
  if (ckpt_error_) {
    std::exception_ptr e = ckpt_error_;
    ckpt_error_ = nullptr;
    std::rethrow_exception(e);
  }
}

void Solver::read_restart(const std::string& g, const std::string& ddv, const std::string& umean) {
  const Plan& p = plan_;
  const int N = p.NY, NZ = p.NZ, lines = p.lines_loc();
  const double N2 = static_cast<double>(p.NX) * p.Nzp;
  std::vector<int> planes(p.nkx_loc);
  for (int i = 0; i < p.nkx_loc; ++i) planes[i] = p.kx_fft_pos(p.kx0 + i);
  std::vector<std::complex<double>> phi(canon_, 0.0), om(canon_, 0.0);
  auto unpack = [&](const std::string& path, std::vector<std::complex<double>>& f) {
    std::vector<double> d;
    int dims[3];
    h5_read_planes(path, planes, d, dims);
    CH_CHECK(dims[0] == p.NX && dims[1] == N && dims[2] == 2 * NZ,
             "restart file " << path << " has dims " << dims[0] << "x" << dims[1] << "x" << dims[2]);
    for (int i = 0; i < p.nkx_loc; ++i)
      for (int kzl = 0; kzl < p.nkz_loc; ++kzl)
        for (int j = 0; j < N; ++j) {
          const size_t o = ((static_cast<size_t>(i) * NZ + p.kz0 + kzl) * N + j) * 2;
          f[static_cast<size_t>(j) * lines + i * p.nkz_loc + kzl] = std::complex<double>(d[o], d[o + 1]) / N2;
        }
  };
  unpack(g, om);
  unpack(ddv, phi);
  std::vector<double> U(N, 0.0);
  std::vector<double> u64;
  const bool umean_given = !umean.empty() && umean != "-";
  if (umean_given) {
    // an explicitly named UMEAN file wins (the reference's float32 records, meanUevol.c:153-176);
    // when it is the companion of G (the same profile rounded to float32), the full-precision copy
    // inside G is used instead
    U = umean_read(umean, N);
    bool companion = h5_read_vector(g, "umean", u64) && static_cast<int>(u64.size()) == N;
    for (int jy = 0; companion && jy < N; ++jy)
      companion = static_cast<float>(u64[jy]) == static_cast<float>(U[jy]);
    if (companion) {
      U = u64;
    } else if (plan_.rank == 0 && !u64.empty()) {
      std::cerr << "[channel] read_restart: U(y) from " << umean << " (differs from the 'umean' stored in " << g
                << ", which is ignored)\n";
    }
    for (auto& u : U) u /= N2;
  } else if (h5_read_vector(g, "umean", u64) && static_cast<int>(u64.size()) == N) {
    // no UMEAN file named: U at full precision from the G file written by this framework
    for (int jy = 0; jy < N; ++jy) U[jy] = u64[jy] / N2;
  } else {
    const auto& y = grid_.y;
    for (int j = 0; j < N; ++j) U[j] = 0.75 * cfg_.Q * (1.0 - y[j] * y[j]);
  }
  set_state(phi.data(), om.data(), U.data());
  auto attrs = h5_read_attrs(g);
  double t = attrs.count("time") ? attrs["time"] : 0.0, dt = attrs.count("dt") ? attrs["dt"] : 0.0;
  set_time(t, dt);
  nstep_ = attrs.count("step") ? static_cast<long>(attrs["step"]) : 0;
}

}  // namespace channel
