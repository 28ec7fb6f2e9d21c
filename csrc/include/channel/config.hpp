// Run configuration: parser for the libconfig subset used by the reference's run.conf
// (run.conf:1-23, read by config.c:4-42) plus the optional keys of SURVEY §5.6.
//
// Differences from the reference, by design:
//  * Grid sizes are runtime values (the reference baked NX/NY/NZ in as -D macros via
//    stripsizes.py, Makefile:8-11).
//  * Physical constants that were compile-time macros (channel.h:50-62) are optional keys with the
//    reference value as default.
#pragma once

#include <map>
#include <string>
#include <vector>

namespace channel {

// Generic parsed libconfig tree, flattened to dotted paths ("application.input.G").
class ConfigTree {
 public:
  static ConfigTree parse_string(const std::string& text);
  static ConfigTree parse_file(const std::string& path);

  bool has(const std::string& key) const;
  std::string get_string(const std::string& key, const std::string& dflt) const;
  long get_int(const std::string& key, long dflt) const;
  double get_double(const std::string& key, double dflt) const;
  bool get_bool(const std::string& key, bool dflt) const;
  // "key=value" override (CLI --set); value syntax as in the file.
  void set(const std::string& key, const std::string& raw_value);
  const std::map<std::string, std::string>& items() const { return kv_; }

 private:
  // Raw values; strings are stored unquoted with a leading '\x01' marker.
  std::map<std::string, std::string> kv_;
  friend struct ConfigParser;
};

struct Config {
  // Grid (run.conf application.NX/NY/NZ).  NZ = number of kz modes; physical z points = 2NZ-2
  // (fft.c:17; the run.conf:5 comment "2*NZ+2" is wrong).
  int NX = 128, NY = 129, NZ = 65;
  // I/O paths (run.conf:8-10, 18-20, 22).  "-" = none / generate.
  std::string in_G = "-", in_DDV = "-", in_UMEAN = "-";
  std::string out_G = "-", out_DDV = "-", out_UMEAN = "-";
  std::string path = "./";
  // Physics (channel.h:50-62, made runtime).
  double Re = 3250.0;           // 1/nu
  double Q = 1.8;               // flow rate over LY=2 -> bulk velocity Q/2
  double LX = 6.283185307179586;
  double LZ = 3.141592653589793;
  double stretch = 2.0;         // tanh mesh stretching (channel.h:21)
  // Run control (RK3.c:124 hard-coded 30000; A13).
  long nsteps = 30000;
  double t_end = 0.0;           // >0: stop when time >= t_end
  double cfl = 0.5;             // RK3.c:68
  double dt_fixed = 0.0;        // >0: fixed dt instead of CFL control
  double dt_max = 0.05;
  std::string cfl_mode = "corrected";   // corrected | parity (RK3.c:86-89)
  int stats_every = 10;         // FREC_STATS (channel.h:82)
  int symmetry_every = 1000;    // RK3.c:174
  int checkpoint_every = 0;     // 0 = only at the end (reference behaviour)
  bool checkpoint_async = true; // periodic checkpoints written by a background thread from a host copy
  int log_every = 1;            // stdout blocks / mean .dat files cadence (reference: every step)
  std::string precision = "fp32";      // storage: fp32 | fp64; y-solves are always fp64
  std::string decomposition = "slab";  // slab | pencil
  int pr = 0, pc = 0;                  // pencil grid (0 = automatic)
  unsigned long long seed = 12345;
  std::string ic = "random";    // random | laminar | file | os_mode
  double ic_amplitude = 0.1;
  std::string forcing = "implicit";    // implicit (exact flux) | parity (meanUevol.c:201-221)
  // Reference-parity switches: wall-BC influence functions discrete (default: v'(+-1)
  // = 0 to round-off) | analytic (the reference's cosh/sinh Green's functions, bilplacSolver_double
  // .cu:56-250, l1/l2 typo fixed); explicit viscous D2: compact (default) | dd (D1 o D1 as in
  // RK3_kernels.cu:160-164 / derivatives_nu_double.cu:440-446)
  std::string influence = "discrete";
  std::string explicit_d2 = "compact";
  bool health_check = true;
  // Failure handling (the reference only exit(1)'d the failing rank, check.cu).
  int health_every = 100;              // steps between global NaN/Inf checks
  std::string on_nan = "abort";        // abort | rollback (restore the last in-memory snapshot)
  int snapshot_every = 0;              // rollback snapshots (0 = health_every)
  int max_rollbacks = 3;
  double rollback_cfl_factor = 0.5;    // cfl *= factor after each rollback
  // Observability.
  int spectra_every = 0;               // 0 = off; 1-D kx/kz energy spectra + 2-D map (statistics.cu:245-326)
  std::string spectra_planes = "";     // comma-separated y indices ("" = NY/2)
  std::string log_json = "";           // JSON-lines run log path ("" = off)

  static Config from_tree(const ConfigTree& t);
  static Config from_file(const std::string& path, const std::vector<std::string>& overrides = {});
  std::string to_string() const;       // effective config echo (libconfig syntax)
  void validate() const;               // throws channel::Error on invalid settings

  int nzp() const { return 2 * NZ - 2; }
  bool fp64() const { return precision == "fp64"; }
  std::vector<int> spectra_plane_list() const;   // parsed spectra_planes (default {NY/2})
};

// FFT lengths the transform kernels are instantiated for: 2^k (16..2048) and 3, 5, 7, 9, 11, 13, 15 x 2^k
// (2^k >= 16, at most 2048 points)
bool fft_length_supported(int n);

}  // namespace channel
