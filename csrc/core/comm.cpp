#include "channel/comm.hpp"

#include <rccl/rccl.h>

#include <cstring>

#include "channel/common.hpp"

namespace channel {

#define NCCL_CHECK(expr)                                                                             \
  do {                                                                                               \
    ncclResult_t _r = (expr);                                                                        \
    if (_r != ncclSuccess) ::channel::fail(std::string(#expr) + " -> " + ncclGetErrorString(_r), __FILE__, __LINE__); \
  } while (0)

std::string Comm::new_unique_id() {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(id.internal, id.internal + sizeof(id.internal));
}

Comm::Comm(int rank, int nranks, const std::string& uid, int device) : rank_(rank), size_(nranks) {
  CH_CHECK(uid.size() == sizeof(ncclUniqueId::internal), "bad ncclUniqueId size " << uid.size());
  HIP_CHECK(hipSetDevice(device));
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), uid.size());
  ncclComm_t c;
  NCCL_CHECK(ncclCommInitRank(&c, nranks, id, rank));
  comm_ = c;
}

Comm::~Comm() {
  if (comm_) ncclCommDestroy(static_cast<ncclComm_t>(comm_));
}

void Comm::abort() {
  if (comm_) ncclCommAbort(static_cast<ncclComm_t>(comm_));
  comm_ = nullptr;
}

void Comm::alltoallv(const void* send, const std::vector<size_t>& scount, const std::vector<size_t>& soff, void* recv,
                     const std::vector<size_t>& rcount, const std::vector<size_t>& roff, hipStream_t s) {
  auto c = static_cast<ncclComm_t>(comm_);
  const char* sb = static_cast<const char*>(send);
  char* rb = static_cast<char*>(recv);
  NCCL_CHECK(ncclGroupStart());
  for (int p = 0; p < size_; ++p) {
    if (scount[p]) NCCL_CHECK(ncclSend(sb + soff[p], scount[p] / 4, ncclFloat, p, c, s));
    if (rcount[p]) NCCL_CHECK(ncclRecv(rb + roff[p], rcount[p] / 4, ncclFloat, p, c, s));
  }
  NCCL_CHECK(ncclGroupEnd());
}

void Comm::allreduce_max_f32(float* buf, size_t n, hipStream_t s) {
  NCCL_CHECK(ncclAllReduce(buf, buf, n, ncclFloat, ncclMax, static_cast<ncclComm_t>(comm_), s));
}
void Comm::allreduce_sum_f64(double* buf, size_t n, hipStream_t s) {
  NCCL_CHECK(ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, static_cast<ncclComm_t>(comm_), s));
}
void Comm::allreduce_max_u32(unsigned* buf, size_t n, hipStream_t s) {
  NCCL_CHECK(ncclAllReduce(buf, buf, n, ncclUint32, ncclMax, static_cast<ncclComm_t>(comm_), s));
}
void Comm::broadcast(void* buf, size_t bytes, int root, hipStream_t s) {
  NCCL_CHECK(ncclBroadcast(buf, buf, bytes, ncclChar, root, static_cast<ncclComm_t>(comm_), s));
}

}  // namespace channel
