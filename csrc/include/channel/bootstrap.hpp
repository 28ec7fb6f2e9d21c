// Process bootstrap for the C++ driver: rank/size from the launcher environment and a TCP
// rendezvous that broadcasts a payload (RCCL unique id + config text) from rank 0.
//
// The reference used MPI_Init + MPI_Bcast of nx/ny/nz and one path string (main.c:25-43, 106;
// other paths were never broadcast) and bound rank%2 to a device (main.c:87).
// Environment understood: RANK/WORLD_SIZE/LOCAL_RANK (torchrun), PMI_RANK/PMI_SIZE (MPICH
// hydra), OMPI_COMM_WORLD_RANK/SIZE/LOCAL_RANK (Open MPI); MASTER_ADDR/MASTER_PORT for the
// rendezvous (default 127.0.0.1:29511).
#pragma once

#include <string>

namespace channel {

struct ProcInfo {
  int rank = 0, size = 1, local_rank = 0;
  static ProcInfo from_env();
};

// Rank 0 sends `payload` to every other rank; returns the payload on every rank.
std::string tcp_broadcast(const ProcInfo& pi, const std::string& payload, int timeout_s = 300);

}  // namespace channel
