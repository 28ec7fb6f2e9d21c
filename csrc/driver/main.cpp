// channel_mi355x — C++ driver binary, the counterpart of the reference's channelMPI.bin (main.c).
//
//   channel_mi355x [run.conf] [--set key=value ...] [--steps N] [--quiet]
//   torchrun --nproc-per-node 8 --no-python bin/channel_mi355x run.conf      (one rank per GPU)
//   mpirun -np 8 bin/channel_mi355x run.conf                                 (MPICH/Open MPI env)
//
// Flow (main.c:10-150): read run.conf on rank 0 and broadcast it (all keys, not only the input path
// as in main.c:106) -> device = local rank (not rank%2, main.c:87) -> RCCL communicator -> IC from
// the input files or generated (random/laminar) -> RK3 loop with the reference's stdout blocks and
// .dat statistics -> restart files (G, DDV, UMEAN) written in the reference format.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "channel/bootstrap.hpp"
#include "channel/comm.hpp"
#include "channel/common.hpp"
#include "channel/config.hpp"
#include "channel/solver.hpp"

using namespace channel;

int main(int argc, char** argv) {
  ProcInfo pi;
  try {
    pi = ProcInfo::from_env();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 2;
  }
  if (const char* ct = std::getenv("CHANNEL_CRASH_TRACE"); ct && std::atoi(ct) == 1) install_crash_handler();
  std::string conf = "run.conf";
  std::vector<std::string> overrides;
  long steps = -1;
  bool verbose = true;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--set" && i + 1 < argc) overrides.push_back(argv[++i]);
    else if (a == "--steps" && i + 1 < argc) steps = std::atol(argv[++i]);
    else if (a == "--quiet") verbose = false;
    else if (a == "-h" || a == "--help") {
      std::printf("usage: %s [run.conf] [--set key=value]... [--steps N] [--quiet]\n", argv[0]);
      return 0;
    } else conf = a;
  }
  std::unique_ptr<Solver> solver;
  try {
    int ndev = 0;
    HIP_CHECK(hipGetDeviceCount(&ndev));
    CH_CHECK(ndev > 0, "no GPU visible");
    const int device = pi.local_rank % ndev;
    HIP_CHECK(hipSetDevice(device));
    // rank 0 reads the config and creates the RCCL id; both travel in one payload
    std::string payload;
    if (pi.rank == 0) {
      std::ifstream f(conf);
      CH_CHECK(f.good(), "cannot open " << conf);
      std::stringstream ss;
      ss << f.rdbuf();
      std::string uid;
      // CHANNEL_FORCE_COMM=1: a communicator (and the exchange-based pipeline) even for one rank
      const char* fc = std::getenv("CHANNEL_FORCE_COMM");
      if (pi.size > 1 || (fc && std::atoi(fc) == 1)) {
        // CHANNEL_COMM=shm: host shared-memory loopback (ranks sharing one GPU, testing only)
        const char* cm = std::getenv("CHANNEL_COMM");
        const char* mp = std::getenv("MASTER_PORT");
        if (cm && std::string(cm) == "shm") uid = std::string("shm:chdrv_") + (mp ? mp : "0");
        else uid = Comm::new_unique_id();
      }
      payload = std::to_string(uid.size()) + "\n" + uid + ss.str();
    }
    payload = tcp_broadcast(pi, payload);
    const size_t nl = payload.find('\n');
    const size_t ulen = std::stoul(payload.substr(0, nl));
    const std::string uid = payload.substr(nl + 1, ulen);
    ConfigTree tree = ConfigTree::parse_string(payload.substr(nl + 1 + ulen));
    for (const auto& o : overrides) {
      const auto eq = o.find('=');
      CH_CHECK(eq != std::string::npos, "--set expects key=value");
      std::string k = o.substr(0, eq);
      if (tree.has("application." + k)) k = "application." + k;
      tree.set(k, o.substr(eq + 1));
    }
    Config cfg = Config::from_tree(tree);
    if (pi.rank == 0 && verbose) {
      std::printf("channel_mi355x: %d rank(s), grid %d x %d x %d (NZ=%d modes), Re=%g, %s\n", pi.size, cfg.NX, cfg.NY,
                  cfg.nzp(), cfg.NZ, cfg.Re, cfg.precision.c_str());
      std::printf("%s", cfg.to_string().c_str());
    }
    solver = std::make_unique<Solver>(cfg, pi.rank, pi.size, device, uid);
    if (cfg.ic == "file") solver->read_restart(cfg.in_G, cfg.in_DDV, cfg.in_UMEAN);
    else solver->init_ic();
    solver->prepare();
    const long n = steps >= 0 ? steps : cfg.nsteps;
    const auto t0 = std::chrono::steady_clock::now();
    solver->run(n, verbose);
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (pi.rank == 0)
      std::printf("\nchannel_mi355x: %ld RK3 steps in %.3f s (%.3f ms/step, %.3e grid-pts/s)\n", n, sec,
                  n ? 1e3 * sec / n : 0.0, n ? double(cfg.NX) * cfg.NY * cfg.nzp() * n / sec : 0.0);
    if (cfg.out_G != "-" && cfg.out_DDV != "-") solver->write_restart(cfg.out_G, cfg.out_DDV, cfg.out_UMEAN);
    solver.reset();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "[rank %d] fatal: %s\n", pi.rank, e.what());
    if (solver) solver->abort_comms();  // do not leave peers hanging
    std::fflush(stderr);
    std::_Exit(1);
  }
  return 0;
}
