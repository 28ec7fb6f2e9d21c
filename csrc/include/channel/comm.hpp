// Communicators for the slab decomposition (one process per GPU).
//
//  * RcclComm: device-direct RCCL collectives over xGMI (the production path).  Replaces the
//    reference's host-staged MPI_Alltoall transposes (channel_cuda_mpi.c:64-128: D2H copy,
//    MPI_Alltoall of pageable buffers, H2D copy, per-item cublasCgeam) and its scalar
//    MPI_Allreduce reductions (hit_mpi.c:427-455).  Bootstrap: the 128-byte ncclUniqueId is
//    exchanged by the caller (torch.distributed broadcast in Python, MPI_Bcast in the C++ driver).
//  * ShmComm: host shared-memory loopback for testing P ranks that share one GPU (RCCL refuses
//    two ranks on one device).  Synchronous and host-staged, so it is never captured in a graph;
//    it exercises exactly the same send/recv block addressing as RcclComm.  Selected by a
//    "shm:<name>" unique id.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstddef>
#include <memory>
#include <string>
#include <vector>

namespace channel {

// one variable all-to-all of a batch (counts/offsets in bytes, per peer)
struct A2ABlock {
  const void* send = nullptr;
  void* recv = nullptr;
  std::vector<size_t> scount, soff, rcount, roff;
};

class Comm {
 public:
  virtual ~Comm() = default;
  int rank() const { return rank_; }
  int size() const { return size_; }
  virtual bool graph_capturable() const = 0;
  virtual const char* kind() const = 0;  // "rccl" | "shm"

  // variable all-to-all; counts/offsets in bytes (multiples of 4)
  virtual void alltoallv(const void* send, const std::vector<size_t>& scount, const std::vector<size_t>& soff,
                         void* recv, const std::vector<size_t>& rcount, const std::vector<size_t>& roff,
                         hipStream_t s) = 0;
  // several all-to-alls issued as one exchange (RCCL: one group); default: one after the other
  virtual void alltoallv_batch(const std::vector<A2ABlock>& ops, hipStream_t s) {
    for (const auto& o : ops) alltoallv(o.send, o.scount, o.soff, o.recv, o.rcount, o.roff, s);
  }
  virtual void allreduce_max_f32(float* buf, size_t n, hipStream_t s) = 0;
  virtual void allreduce_sum_f64(double* buf, size_t n, hipStream_t s) = 0;
  virtual void allreduce_max_f64(double* buf, size_t n, hipStream_t s) = 0;
  virtual void allreduce_max_u32(unsigned* buf, size_t n, hipStream_t s) = 0;
  virtual void abort() = 0;
  // asynchronous communicator failure (peer died, network error); polled by the solver's watchdog
  virtual bool async_error() { return false; }

  // Sub-communicator of one exchange group (collective over this communicator: every rank calls it
  // with the member list of its own group; groups partition the ranks).  members[i] is the rank in
  // this communicator of group rank i.  RCCL: ncclCommSplit (color = members[0], key = position);
  // the host-staged loopback: a view that widens group counts to the world (every rank of the world
  // still enters each exchange, as the solver's schedule is identical on all ranks).
  virtual std::unique_ptr<Comm> group(const std::vector<int>& members) = 0;

  static std::string new_unique_id();  // 128 raw bytes (RCCL)
  // "shm:<name>" -> ShmComm, otherwise an RCCL unique id
  static std::unique_ptr<Comm> create(int rank, int nranks, const std::string& uid, int device);

 protected:
  int rank_ = 0, size_ = 1;
};

class RcclComm final : public Comm {
 public:
  RcclComm(int rank, int nranks, const std::string& uid, int device);
  ~RcclComm() override;
  bool graph_capturable() const override { return true; }
  const char* kind() const override { return "rccl"; }
  void alltoallv(const void* send, const std::vector<size_t>& scount, const std::vector<size_t>& soff, void* recv,
                 const std::vector<size_t>& rcount, const std::vector<size_t>& roff, hipStream_t s) override;
  void alltoallv_batch(const std::vector<A2ABlock>& ops, hipStream_t s) override;
  void allreduce_max_f32(float* buf, size_t n, hipStream_t s) override;
  void allreduce_sum_f64(double* buf, size_t n, hipStream_t s) override;
  void allreduce_max_f64(double* buf, size_t n, hipStream_t s) override;
  void allreduce_max_u32(unsigned* buf, size_t n, hipStream_t s) override;
  void abort() override;
  bool async_error() override;
  std::unique_ptr<Comm> group(const std::vector<int>& members) override;

 private:
  RcclComm() = default;
  void* comm_ = nullptr;  // ncclComm_t
  // the block a rank sends to itself is a D2D copy on the stream; CHANNEL_A2A_SELF=rccl routes it
  // through ncclSend/ncclRecv instead (lets a 1-rank communicator exercise RCCL's point-to-point path)
  bool self_via_rccl_ = false;
};

class ShmComm final : public Comm {
 public:
  ShmComm(int rank, int nranks, const std::string& name);
  ~ShmComm() override;
  bool graph_capturable() const override { return false; }
  const char* kind() const override { return "shm"; }
  void alltoallv(const void* send, const std::vector<size_t>& scount, const std::vector<size_t>& soff, void* recv,
                 const std::vector<size_t>& rcount, const std::vector<size_t>& roff, hipStream_t s) override;
  void allreduce_max_f32(float* buf, size_t n, hipStream_t s) override;
  void allreduce_sum_f64(double* buf, size_t n, hipStream_t s) override;
  void allreduce_max_f64(double* buf, size_t n, hipStream_t s) override;
  void allreduce_max_u32(unsigned* buf, size_t n, hipStream_t s) override;
  void abort() override { failed_ = true; }
  bool async_error() override { return failed_; }
  std::unique_ptr<Comm> group(const std::vector<int>& members) override;

 private:
  void barrier();
  std::atomic<bool> failed_{false};  // set by abort() (any thread): the barrier then raises at once
  double timeout_s_ = 300.0;  // CHANNEL_COMM_TIMEOUT_S
  char* slot(int src, int dst);
  template <typename T, typename Op>
  void allreduce(T* buf, size_t n, hipStream_t s, Op op);
  std::string name_;
  void* base_ = nullptr;
  size_t bytes_ = 0, slot_bytes_ = 0;
};

// Group view on a world communicator (exchange counts widened with zeros outside the group).
class GroupComm final : public Comm {
 public:
  GroupComm(Comm* world, std::vector<int> members);
  bool graph_capturable() const override { return world_->graph_capturable(); }
  const char* kind() const override { return world_->kind(); }
  void alltoallv(const void* send, const std::vector<size_t>& scount, const std::vector<size_t>& soff, void* recv,
                 const std::vector<size_t>& rcount, const std::vector<size_t>& roff, hipStream_t s) override;
  void alltoallv_batch(const std::vector<A2ABlock>& ops, hipStream_t s) override;
  // reductions stay on the world communicator (the solver never reduces over a group)
  void allreduce_max_f32(float*, size_t, hipStream_t) override { unsupported(); }
  void allreduce_sum_f64(double*, size_t, hipStream_t) override { unsupported(); }
  void allreduce_max_f64(double*, size_t, hipStream_t) override { unsupported(); }
  void allreduce_max_u32(unsigned*, size_t, hipStream_t) override { unsupported(); }
  void abort() override { world_->abort(); }
  bool async_error() override { return world_->async_error(); }
  std::unique_ptr<Comm> group(const std::vector<int>&) override;

 private:
  [[noreturn]] static void unsupported();
  A2ABlock widen(const A2ABlock& o) const;
  Comm* world_;
  std::vector<int> members_;
};

}  // namespace channel
