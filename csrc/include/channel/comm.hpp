// RCCL communicator wrapper (one process per GPU, device-direct collectives over xGMI).
//
// Replaces the reference's host-staged MPI_Alltoall transposes (channel_cuda_mpi.c:64-128: D2H copy,
// MPI_Alltoall of pageable buffers, H2D copy, per-item cublasCgeam) and its scalar MPI_Allreduce
// reductions (hit_mpi.c:427-455).  Bootstrap: the 128-byte ncclUniqueId is exchanged by the caller
// (torch.distributed broadcast in Python, MPI_Bcast in the C++ driver).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <string>
#include <vector>

namespace channel {

class Comm {
 public:
  static std::string new_unique_id();  // 128 raw bytes
  Comm(int rank, int nranks, const std::string& uid, int device);
  ~Comm();
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;

  int rank() const { return rank_; }
  int size() const { return size_; }

  // variable all-to-all; counts/offsets in bytes (multiples of 4)
  void alltoallv(const void* send, const std::vector<size_t>& scount, const std::vector<size_t>& soff, void* recv,
                 const std::vector<size_t>& rcount, const std::vector<size_t>& roff, hipStream_t s);
  void allreduce_max_f32(float* buf, size_t n, hipStream_t s);
  void allreduce_sum_f64(double* buf, size_t n, hipStream_t s);
  void allreduce_max_u32(unsigned* buf, size_t n, hipStream_t s);
  void broadcast(void* buf, size_t bytes, int root, hipStream_t s);
  void abort();

 private:
  int rank_ = 0, size_ = 1;
  void* comm_ = nullptr;  // ncclComm_t
};

}  // namespace channel
