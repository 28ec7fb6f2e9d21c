// The channel-flow DNS solver: one instance per rank (one process per GPU).
//
// Formulation (reference README.md:4-6): Kim-Moin-Moser phi = lap(v) / omega_y,
// Fourier x,z with 2/3 dealiasing, compact FD in y, SMR low-storage RK3 with implicit viscous
// terms, constant flow rate, mean profile U(y) evolved on the rank that owns kx=0.
//
// Per RK3 substep (all device-resident, captured into one hipGraph per RK3 step):
//   K-SPEC (y-lines) -> [all-to-all per field, comm stream] -> x C2C inverse (per field)
//   -> z physical stage (C2R, u x omega, R2C, CFL maxima) -> x C2C forward (per field)
//   -> [all-to-all per field] -> next K-SPEC.
// The reference's equivalent is RKstep (RK3.c:111-193) with host-staged transposes.
#pragma once

#include <hip/hip_runtime.h>

#include <complex>
#include <exception>
#include <functional>
#include <memory>
#include <thread>
#include <chrono>
#include <string>
#include <vector>

#include "channel/comm.hpp"
#include "channel/config.hpp"
#include "channel/grid.hpp"
#include "channel/kernels.hpp"
#include "channel/plan.hpp"

namespace channel {

// SMR low-storage RK3 coefficients (RK3_kernels.cu:24-25, 113; RK3.c:14; meanUevol.c:35-38)
struct RK3Coef {
  static constexpr double gamma[3] = {8.0 / 15.0, 5.0 / 12.0, 3.0 / 4.0};
  static constexpr double zeta[3] = {0.0, -17.0 / 60.0, -5.0 / 12.0};
  static constexpr double alpha[3] = {29.0 / 96.0, -3.0 / 40.0, 1.0 / 6.0};
  static constexpr double beta[3] = {37.0 / 160.0, 5.0 / 24.0, 1.0 / 6.0};
};

struct StepLog {
  long step = 0;
  double time = 0, dt = 0, dt_c = 0, dt_v = 0;
  double umax = 0, vmax = 0, wmax = 0, cflsum = 0;
  double dUdy_lo = 0, dUdy_hi = 0, flux = 0, dpdx = 0;
  double utau_lo = 0, utau_hi = 0, utau = 0;
  unsigned health = 0;
};

class Solver {
 public:
  // nccl_uid: empty for P == 1
  Solver(const Config& cfg, int rank, int nranks, int device, const std::string& nccl_uid = std::string());
  ~Solver();
  Solver(const Solver&) = delete;
  Solver& operator=(const Solver&) = delete;

  const Config& config() const { return cfg_; }
  const Plan& plan() const { return plan_; }
  const YGrid& grid() const { return grid_; }
  hipStream_t stream() const { return s_comp_; }
  bool fp64() const { return fp64_; }

  // ---- state --------------------------------------------------------------------------
  // local spectral state, [y][kx_local][kz] true Fourier coefficients; U: NY (used on the owner)
  void set_state(const std::complex<double>* phi, const std::complex<double>* omega, const double* U);
  void get_state(std::complex<double>* phi, std::complex<double>* omega, double* U) const;
  void init_ic();      // config ic: random | laminar | zero (deterministic, independent of P)
  void prepare();      // fill the transform inputs from the state (K-SPEC mode 0)

  // ---- time stepping ---------------------------------------------------------------------
  void step(bool stats_for_next = false);  // one RK3 step
  void run(long nsteps, bool verbose = true);  // reference-style driver loop with logging/stats
  void synchronize();
  StepLog log();                     // reads device diagnostics (host sync)
  std::vector<double> stats();       // [4][NY] plane sums of the last stats step (global)
  std::vector<double> mean_profile();  // U(y) (owner rank; zeros elsewhere)
  unsigned health();                  // global OR of health flags
  double time() const;
  long steps_done() const { return nstep_; }
  void set_time(double t, double dt);
  void set_use_graph(bool on) { use_graph_ = on; }
  // true when the RK3 step is replayed from a captured hipGraph (after the first captured step)
  bool graph_active() const;
  // the communicator's kind ("rccl" | "shm") or "none" for the single-rank fast path
  std::string comm_kind() const;
  // per-phase timing: hipEvents around every stage on its own stream (no host sync inside the
  // step; the pairs are resolved once per step).  Runs eagerly and, at P = 1, on one stream so the
  // stages are serialised and the phase times add up to the step time.
  void set_phase_timing(bool on);
  // accumulated per-phase times [kspec, x_backward, z_physical, x_forward, a2a, reduce, io, other]
  std::vector<double> phase_times_ms();
  void reset_phase_times();
  // per-step device times: hipEvents recorded on the compute stream around every step() (graph
  // launches included); step_times_ms() synchronises and returns (and clears) them
  void set_step_timing(bool on) { step_timing_ = on; }
  std::vector<double> step_times_ms();
  // K-SPEC per-phase shader-clock sums over all waves (only with CHANNEL_KSPEC_PROF set)
  std::vector<double> kspec_profile();
  void symmetrize();                  // kz=0 Hermitian symmetry (any P; one column exchange)

  // ---- failure handling -------------------------------------------------------
  void take_snapshot();               // device copy of (phi, omega+U, dt, time, step)
  void rollback();                    // restore it; cfl *= rollback_cfl_factor; re-capture graphs
  long snapshot_step() const { return snap_step_; }
  int rollbacks() const { return rollbacks_; }
  double cfl() const { return cfg_.cfl; }
  void inject_nan(int field = PHI);   // fault injection (tests)

  // ---- diagnostics ---------------------------------------------------------------------------
  // energy spectra of u,v,w of the current state at cfg.spectra_planes (global sums):
  // ekx [3][np][Kx+1], ekz [3][np][nkz], map [3][nkx][nkz] at the first plane
  struct Spectra {
    std::vector<int> planes;
    std::vector<double> ekx, ekz, map;
  };
  Spectra spectra();

  // ---- restart files (reference-compatible, Appendix B) --------------------------------
  void write_restart(const std::string& g, const std::string& ddv, const std::string& umean);
  void read_restart(const std::string& g, const std::string& ddv, const std::string& umean);
  // capture the state now (host copy) and write the files from a background thread; the next
  // checkpoint / wait_checkpoint() / run() end / destructor joins it (and rethrows its error)
  void checkpoint_async(const std::string& g, const std::string& ddv, const std::string& umean);
  void wait_checkpoint();

  // ---- raw device access (tests / bindings) ----------------------------------------------
  enum Field { PHI = 0, OMEGA, RPHI, ROMEGA, OUT0, OUT1, OUT2, OUT3, OUT4, OUT5 };
  void* field_ptr(int f) const;
  // backward-exchanged field j: the combine mode's inputs (0 D1 v, 1 v, 2 D1 omega, 3 omega, 4 phi)
  // or the six physical-stage fields (choose_layout)
  static constexpr int kCmbIn = 5;
  int bwd_fields() const { return combine_ ? kCmbIn : 6; }
  bool combine() const { return combine_; }
  void* in_field(int j) const;
  void* phys_ptr() const { return phys_; }
  const YTablesDev& ytables() const { return ytab_; }
  // kx sub-blocks of the local spectral layout (1 = plain [y][kx_local][kz]; see nkb_)
  int kblocks() const { return nkb_; }
  // backward-exchange kx sub-block groups issued so far (host count: the pipeline bookkeeping of
  // the pre-send, checked by the capture-failure test)
  long long bwd_blocks_issued() const { return bwd_blocks_issued_; }
  // compute streams of the last P > 1 transform stage recorded inside a stream capture (0: none yet)
  int captured_compute_streams() const { return captured_streams_; }
  int spec_kzb() const { return kzb_; }  // spectral layout (spec_index)
  // abort every communicator (the per-axis split ones first: aborting the parent does not abort
  // communicators split from it), so no stream stays blocked in an exchange with a dead peer
  void abort_comms();
  void substep_debug(int n);            // one substep, eager (tests)
  void transforms_debug(bool dt_update);  // backward + phys + forward only (tests)
  Comm* comm() { return comm_.get(); }
  void barrier();
  // host value reduced (max) over all ranks through the solver's communicator (timing, control)
  double max_over_ranks(double v);

 private:
  void choose_layout();
  void alloc();
  void free_all();
  void transforms(int substep, bool stats);
  void kspec(int mode, int substep, bool stats);
  void a2a_spec(const void* spec, void* xb, bool to_phys);
  void a2a_rows(void* xexp, void* zrows, bool to_z);
  void step_body(bool stats);
  void ev(int phase, bool end, hipStream_t s = nullptr);
  void flush_phase_events();
  hipEvent_t timing_event();
  // P > 1 slab: y-chunked backward exchange -> x -> z -> x -> forward exchange pipeline
  void transforms_slab(int n, const XArgs& xa, const ZArgs& za, const DtArgs& da);
  // exchange of y chunk k (rows [k*ch, (k+1)*ch) of every rank's y range) for nf fields over the
  // column group (the world for the slab)
  void a2a_slab_chunk(int k, int ch, bool to_phys, int nf);
  // the same for rows [r0, r0 + nr) of every rank's y range and kx sub-blocks [blo, bhi) only
  void a2a_slab_rows(int r0, int nr, bool to_phys, int nf, int blo, int bhi);
  // pencil: the same y-chunked pipeline with the B exchange (row group, x <-> kz) between the x
  // transforms and the z stage
  void transforms_pencil(int n, const XArgs& xa, const ZArgs& za, const DtArgs& da);
  void b2b_pencil_chunk(int k, int ch, bool to_z, int nf);
  Comm* col_comm() const { return comm_col_ ? comm_col_.get() : comm_.get(); }
  bool comm_failed();
  void write_logs(const StepLog& L, bool verbose);
  void write_stats_files(const std::vector<double>& st);
  void write_spectra_files(const Spectra& sp);
  void write_json(const StepLog& L, double ms_per_step);
  void wait(hipStream_t s);           // stream sync with the communicator watchdog (P > 1)
  void invalidate_graphs();
  struct RestartJob {
    std::string g, ddv, umean;
    std::vector<std::complex<double>> phi, om;
    std::vector<double> U;
    double time = 0, dt = 0;
    long step = 0;
    long serial = 0;
  };
  RestartJob capture_restart(const std::string& g, const std::string& ddv, const std::string& umean);
  // turn(t) is called before every rank-ordered write step t (t % P = the writing rank)
  void write_restart_job(const RestartJob& j, const std::function<void(int)>& turn);

  Config cfg_;
  Plan plan_;
  YGrid grid_;
  bool fp64_ = false;
  int device_ = 0;
  size_t esz_ = 8;  // bytes per complex element
  hipStream_t s_comp_ = nullptr, s_comm_ = nullptr;
  std::unique_ptr<Comm> comm_;
  // pencil exchange groups (one communicator per decomposition axis): column group
  // (same process row, Pc ranks: A exchange kx <-> y) and row group (same column, Pr ranks: B)
  std::unique_ptr<Comm> comm_col_, comm_row_;
  YTablesDev ytab_;
  Twiddles tw_x_, tw_z_;

  void* state_ = nullptr;  // phi, omega, Rphi, Romega (4 * spec)
  void* out_ = nullptr;    // 6 * spec
  void* phys_ = nullptr;   // 6 * phys
  void* xbuf_ = nullptr;   // P>1: 6 * ny_loc*nkx*nkz_loc (A-exchange blocks)
  hipEvent_t ev_dtf_[2] = {nullptr, nullptr};  // P = 1 one-chunk path: dt update forked beside the x-forward
  unsigned* d_rowtab_ = nullptr;  // slab P > 1: per retained kx row, its exchange segment's offset / stride (XSrc::rowtab)
  void build_rowtab();
  void* zbuf_ = nullptr;   // pencil: 6 * ny_loc*nx_loc*nkz (B-exchange blocks, z stage in place)
  size_t spec_ = 0, physn_ = 0, xstride_ = 0, zstride_ = 0;
  // spectral layout (spec_index): kzb_ = 8 (one rank) blocks the lines by 8 kz, with the kz line
  // stride nkzs_ padded to a multiple of 8; canon_ = NY * nkx_loc * nkz_loc, the element count of
  // the canonical host layout [y][kx_loc][kz_loc] (set_state / get_state / restart files)
  int kzb_ = 0, nkzs_ = 0;
  bool combine_ = false;  // K-SPEC's combine-mode outputs + the combining x-backward (choose_layout)
  size_t canon_ = 0;

  // device scalars / diagnostics (one allocation)
  void* dscal_ = nullptr;
  double* d_dt_ = nullptr;
  double* d_time_ = nullptr;
  double* d_dtlog_ = nullptr;
  float* d_max_ = nullptr;
  double* d_stats_ = nullptr;
  double* d_mean_ = nullptr;
  unsigned* d_health_ = nullptr;
  unsigned long long* d_kprof_ = nullptr;
  bool kprof_on_ = false;
  int ystreams_ = 1;               // streams the y chunks alternate over (P = 1)
  std::vector<hipStream_t> s_extra_;   // streams beyond compute + comm for the chunk pipeline
  // P > 1 slab, CHANNEL_PSTREAMS=2: a second compute stream; the y chunks' transforms alternate
  // between s_comp_ and it (the comm stream carries the exchanges), as the P = 1 chunks do
  hipStream_t s_comp2_ = nullptr;
  hipEvent_t ev_comp2_ = nullptr;
  int pstreams_ = 1;  // compute streams of the P > 1 chunk pipeline (CHANNEL_PSTREAMS)
  std::vector<hipEvent_t> ev_join_;
  int ychunk_ = 0;                 // y planes per x->z->x pipeline chunk (P = 1), 0 = whole slab
  double* d_invdy_ = nullptr;
  double* d_red_ = nullptr;  // one double for max_over_ranks
  double* d_y_ = nullptr;    // y grid (analytic influence functions)

  std::vector<hipEvent_t> ev_a2a_, ev_xf_, ev_b_, ev_bb_;
  hipEvent_t ev_spec_ = nullptr, ev_phys_ = nullptr, ev_fwd_done_ = nullptr, ev_red_ = nullptr, ev_stats_ = nullptr;
  std::vector<hipEvent_t> ev_cb_, ev_cc_, ev_cc2_;  // per y-chunk: backward exchange done, compute done (part 0 / part 1)
  // pencil pipeline, per y chunk: A in, x-backward, B in, z stage, B out, x-forward done
  std::vector<hipEvent_t> ev_pen_[6];
  int ychunk_p_ = 0;                       // y planes per chunk of the P > 1 slab pipeline
  bool self_direct_ = true;                // slab: own kx block read/written in place (no self copy)
  // K-SPEC / exchange overlap (P > 1 slab, and a 1-rank communicator): the local spectral fields
  // are stored as nkb_ kx sub-blocks, each [y][kx in block][kz] (block b at element kb_off_[b] of
  // every field).  K-SPEC runs block by block and the backward exchange of block b goes out on the
  // comm stream while block b+1 is solved.  Every rank splits its
  // kx range the same way (balanced), so block (c, b) of rank c is one exchange segment of the x
  // transforms (Pc * nkb_ <= 8 segments).
  int nkb_ = 1;
  std::vector<int> kb_start_, kb_cnt_;     // local ikx start / count of block b (this rank)
  std::vector<size_t> kb_off_;             // element offset of block b in a spectral field
  std::vector<hipEvent_t> ev_kb_;          // K-SPEC block b done (compute stream)
  // Substep 0 of a step consumes a pre-send: the backward exchange of blocks 0 .. nkb_-2 of the
  // state's outputs goes out at the end of the previous step (behind the last K-SPEC's blocks,
  // inside its graph) or, after anything that recomputed the outputs (prepare()), eagerly before
  // the step.  presend_done_: that exchange has been issued for the next substep 0.
  bool presend_done_ = false;
  bool presend_saved_ = false;  // presend_done_ before a step capture (restored if the graph is dropped)
  long long bwd_blocks_issued_ = 0;
  int captured_streams_ = 0;
  int xnt_ = 0;  // non-temporal spectral accesses in the x transforms (XArgs::nt)
  bool kb_overlap() const { return nkb_ > 1 && comm_ != nullptr; }
  // Forward-path overlap (slab, kx sub-blocks): the last y chunk's forward exchange goes out block
  // by block (ev_fb_[b] on the comm stream) and K-SPEC block b waits only for block b's rows.
  // fwd_pending_: the next kspec() (or join_forward()) must consume those events.
  std::vector<hipEvent_t> ev_fb_;
  hipEvent_t ev_cfl_ = nullptr;
  bool fwd_split_ = true, fwd_pending_ = false;
  void join_forward();
  void presend_backward(bool wait_blocks);
  int kb_gstart(int c, int b) const;       // global retained-kx start of block b of column rank c
  int kb_gcount(int c, int b) const;
  size_t kb_index(int y, int ikx, int kz) const;  // blocked element index of (y, local kx, kz)
  size_t dev_index(int y, int ikx, int kz) const;  // device element index of (y, local kx, local kz)
  // phase timing: event pool and the (phase, start, end) pairs of the current step
  struct TPair {
    int phase;
    hipEvent_t a, b;
  };
  std::vector<hipEvent_t> tev_pool_;
  size_t tev_used_ = 0;
  std::vector<TPair> tpairs_;
  hipEvent_t topen_[8] = {};
  std::vector<double> ph_ms_;
  bool phase_timing_ = false;
  bool step_timing_ = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> step_ev_;
  size_t step_ev_used_ = 0;
  bool comm_warm_ = false;
  std::thread ckpt_thread_;
  std::exception_ptr ckpt_error_;
  long ckpt_serial_ = 0;
  unsigned long long run_nonce_ = 0;  // same on every rank of one run (from the communicator id): checkpoint markers
  // t_end checks without a per-step host sync: (dt, time) of the last two steps in pinned memory
  double* h_tdt_ = nullptr;
  hipEvent_t ev_tdt_[2] = {nullptr, nullptr};
  bool tdt_valid_ = false;
  bool t_end_reached();
  void wait_event(hipEvent_t e);      // event sync with the communicator watchdog (P > 1)

  // rollback snapshot
  void* snap_ = nullptr;
  long snap_step_ = -1;
  int rollbacks_ = 0;
  // spectra accumulators [ekx | ekz | map] and plane list (device)
  void* d_spec_ = nullptr;
  void* d_sym_ = nullptr;    // kz = 0 columns (local + gathered) for the distributed symmetrisation
  size_t spec_n_ = 0;
  double comm_timeout_s_ = 900.0;     // CHANNEL_COMM_TIMEOUT_S (0 = wait forever)

  bool use_graph_ = true;
  bool graph_ok_[2] = {false, false};
  // CHANNEL_MARKERS=1 (bench.py sets it at P > 1): one stderr line per rank after the eager warm-up
  // step, the capture and the first replay of each step graph, each after a (watchdog-polled)
  // synchronisation, so a first multi-GPU run that hangs shows which stage and rank stopped
  bool markers_ = false;
  bool capture_fail_test_ = false;
  bool replayed_[2] = {false, false};
  std::chrono::steady_clock::time_point t_created_ = std::chrono::steady_clock::now();
  void marker(const char* what);
  void end_failed_capture();
  hipGraphExec_t gexec_[2] = {nullptr, nullptr};
  bool prepared_ = false;
  long nstep_ = 0;
  bool stats_pending_ = false;
};

}  // namespace channel
