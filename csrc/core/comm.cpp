#include "channel/comm.hpp"

#include <fcntl.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

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

std::unique_ptr<Comm> Comm::create(int rank, int nranks, const std::string& uid, int device) {
  if (uid.rfind("shm:", 0) == 0) return std::make_unique<ShmComm>(rank, nranks, uid.substr(4));
  return std::make_unique<RcclComm>(rank, nranks, uid, device);
}

// ---- RCCL --------------------------------------------------------------------------------------
RcclComm::RcclComm(int rank, int nranks, const std::string& uid, int device) {
  rank_ = rank;
  size_ = nranks;
  CH_CHECK(uid.size() == sizeof(ncclUniqueId::internal), "bad ncclUniqueId size " << uid.size());
  HIP_CHECK(hipSetDevice(device));
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), uid.size());
  ncclComm_t c;
  NCCL_CHECK(ncclCommInitRank(&c, nranks, id, rank));
  comm_ = c;
  // (the solver normally never hands the self block to the exchange; see CHANNEL_A2A_SELF there)
  if (const char* e = std::getenv("CHANNEL_A2A_SELF")) self_via_rccl_ = std::string(e) == "rccl";
}

RcclComm::~RcclComm() {
  if (comm_) ncclCommDestroy(static_cast<ncclComm_t>(comm_));
}

void RcclComm::abort() {
  if (comm_) ncclCommAbort(static_cast<ncclComm_t>(comm_));
  comm_ = nullptr;
}

bool RcclComm::async_error() {
  if (!comm_) return true;
  ncclResult_t r = ncclSuccess;
  if (ncclCommGetAsyncError(static_cast<ncclComm_t>(comm_), &r) != ncclSuccess) return true;
  return r != ncclSuccess && r != ncclInProgress;
}

void RcclComm::alltoallv(const void* send, const std::vector<size_t>& scount, const std::vector<size_t>& soff,
                         void* recv, const std::vector<size_t>& rcount, const std::vector<size_t>& roff,
                         hipStream_t s) {
  A2ABlock b;
  b.send = send;
  b.recv = recv;
  b.scount = scount;
  b.soff = soff;
  b.rcount = rcount;
  b.roff = roff;
  alltoallv_batch({b}, s);
}

// All blocks of the batch go out in ONE ncclGroupStart/End, so RCCL schedules the sends and
// receives of every field to a peer over that peer's xGMI link together (one launch, every link
// busy at once).  The self block never leaves the device: a stream-ordered D2D copy
// (graph-capturable) unless CHANNEL_A2A_SELF=rccl.
void RcclComm::alltoallv_batch(const std::vector<A2ABlock>& ops, hipStream_t s) {
  auto c = static_cast<ncclComm_t>(comm_);
  CH_CHECK(c, "RcclComm: communicator was aborted");
  const bool self_copy = !self_via_rccl_;
  bool any_remote = false;
  for (const auto& o : ops) {
    CH_CHECK(o.scount.size() == static_cast<size_t>(size_) && o.rcount.size() == static_cast<size_t>(size_),
             "alltoallv: count vectors must have one entry per rank");
    if (self_copy && o.scount[rank_]) {
      CH_CHECK(o.scount[rank_] == o.rcount[rank_], "alltoallv: self block send/recv sizes differ");
      HIP_CHECK(hipMemcpyAsync(static_cast<char*>(o.recv) + o.roff[rank_],
                               static_cast<const char*>(o.send) + o.soff[rank_], o.scount[rank_],
                               hipMemcpyDeviceToDevice, s));
    }
    for (int p = 0; p < size_; ++p)
      if (!(self_copy && p == rank_) && (o.scount[p] || o.rcount[p])) any_remote = true;
  }
  if (!any_remote) return;
  NCCL_CHECK(ncclGroupStart());
  for (const auto& o : ops) {
    const char* sb = static_cast<const char*>(o.send);
    char* rb = static_cast<char*>(o.recv);
    for (int p = 0; p < size_; ++p) {
      if (self_copy && p == rank_) continue;
      if (o.scount[p]) NCCL_CHECK(ncclSend(sb + o.soff[p], o.scount[p] / 4, ncclFloat, p, c, s));
      if (o.rcount[p]) NCCL_CHECK(ncclRecv(rb + o.roff[p], o.rcount[p] / 4, ncclFloat, p, c, s));
    }
  }
  NCCL_CHECK(ncclGroupEnd());
}

std::unique_ptr<Comm> RcclComm::group(const std::vector<int>& members) {
  auto c = static_cast<ncclComm_t>(comm_);
  CH_CHECK(c, "RcclComm: communicator was aborted");
  int key = -1;
  for (size_t i = 0; i < members.size(); ++i)
    if (members[i] == rank_) key = static_cast<int>(i);
  CH_CHECK(key >= 0 && !members.empty(), "RcclComm::group: rank " << rank_ << " is not in its own group");
  ncclComm_t sub = nullptr;
  NCCL_CHECK(ncclCommSplit(c, members[0], key, &sub, nullptr));
  std::unique_ptr<RcclComm> g(new RcclComm());
  g->comm_ = sub;
  NCCL_CHECK(ncclCommUserRank(sub, &g->rank_));
  NCCL_CHECK(ncclCommCount(sub, &g->size_));
  CH_CHECK(g->rank_ == key && g->size_ == static_cast<int>(members.size()), "ncclCommSplit: unexpected group layout");
  g->self_via_rccl_ = self_via_rccl_;
  return g;
}

void RcclComm::allreduce_max_f32(float* buf, size_t n, hipStream_t s) {
  NCCL_CHECK(ncclAllReduce(buf, buf, n, ncclFloat, ncclMax, static_cast<ncclComm_t>(comm_), s));
}
void RcclComm::allreduce_sum_f64(double* buf, size_t n, hipStream_t s) {
  NCCL_CHECK(ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, static_cast<ncclComm_t>(comm_), s));
}
void RcclComm::allreduce_max_f64(double* buf, size_t n, hipStream_t s) {
  NCCL_CHECK(ncclAllReduce(buf, buf, n, ncclDouble, ncclMax, static_cast<ncclComm_t>(comm_), s));
}
void RcclComm::allreduce_max_u32(unsigned* buf, size_t n, hipStream_t s) {
  NCCL_CHECK(ncclAllReduce(buf, buf, n, ncclUint32, ncclMax, static_cast<ncclComm_t>(comm_), s));
}

// ---- group view -------------------------------------------------------------------------------
GroupComm::GroupComm(Comm* world, std::vector<int> members) : world_(world), members_(std::move(members)) {
  size_ = static_cast<int>(members_.size());
  rank_ = -1;
  for (int i = 0; i < size_; ++i)
    if (members_[i] == world_->rank()) rank_ = i;
  CH_CHECK(rank_ >= 0, "GroupComm: rank " << world_->rank() << " is not in its own group");
}

void GroupComm::unsupported() { CH_CHECK(false, "reductions over an exchange group are not supported"); }

A2ABlock GroupComm::widen(const A2ABlock& o) const {
  CH_CHECK(o.scount.size() == static_cast<size_t>(size_) && o.rcount.size() == static_cast<size_t>(size_),
           "alltoallv: count vectors must have one entry per group rank");
  const size_t W = static_cast<size_t>(world_->size());
  A2ABlock w;
  w.send = o.send;
  w.recv = o.recv;
  w.scount.assign(W, 0);
  w.soff.assign(W, 0);
  w.rcount.assign(W, 0);
  w.roff.assign(W, 0);
  for (int i = 0; i < size_; ++i) {
    const int g = members_[i];
    w.scount[g] = o.scount[i];
    w.soff[g] = o.soff[i];
    w.rcount[g] = o.rcount[i];
    w.roff[g] = o.roff[i];
  }
  return w;
}

void GroupComm::alltoallv(const void* send, const std::vector<size_t>& scount, const std::vector<size_t>& soff,
                          void* recv, const std::vector<size_t>& rcount, const std::vector<size_t>& roff,
                          hipStream_t s) {
  A2ABlock b;
  b.send = send;
  b.recv = recv;
  b.scount = scount;
  b.soff = soff;
  b.rcount = rcount;
  b.roff = roff;
  alltoallv_batch({b}, s);
}

void GroupComm::alltoallv_batch(const std::vector<A2ABlock>& ops, hipStream_t s) {
  std::vector<A2ABlock> w;
  w.reserve(ops.size());
  for (const auto& o : ops) w.push_back(widen(o));
  world_->alltoallv_batch(w, s);
}

std::unique_ptr<Comm> GroupComm::group(const std::vector<int>& members) {
  std::vector<int> m;
  for (int i : members) m.push_back(members_.at(i));
  return std::make_unique<GroupComm>(world_, m);
}

std::unique_ptr<Comm> ShmComm::group(const std::vector<int>& members) {
  return std::make_unique<GroupComm>(this, members);
}

// ---- shared-memory loopback (tests) -----------------------------------------------------------
namespace {
struct ShmHeader {
  std::atomic<int> ready;
  std::atomic<int> count;
  std::atomic<int> sense;
  int nranks;
  size_t slot_bytes;
};
constexpr size_t kHdr = 4096;
}  // namespace

ShmComm::ShmComm(int rank, int nranks, const std::string& name) : name_("/" + name) {
  rank_ = rank;
  size_ = nranks;
  const char* mb = std::getenv("CHANNEL_SHM_SLOT_MB");
  slot_bytes_ = static_cast<size_t>(mb ? std::atoi(mb) : 16) << 20;
  if (const char* t = std::getenv("CHANNEL_COMM_TIMEOUT_S")) timeout_s_ = std::atof(t);
  bytes_ = kHdr + static_cast<size_t>(nranks) * nranks * slot_bytes_;
  int fd = -1;
  if (rank == 0) {
    shm_unlink(name_.c_str());
    fd = shm_open(name_.c_str(), O_CREAT | O_RDWR, 0600);
    CH_CHECK(fd >= 0, "shm_open(" << name_ << ") failed");
    CH_CHECK(ftruncate(fd, static_cast<off_t>(bytes_)) == 0, "ftruncate shm failed");
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    while ((fd = shm_open(name_.c_str(), O_RDWR, 0600)) < 0) {
      CH_CHECK(std::chrono::steady_clock::now() - t0 < std::chrono::seconds(120), "timeout waiting for shm " << name_);
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
    struct stat st;
    do {
      fstat(fd, &st);
    } while (static_cast<size_t>(st.st_size) < bytes_);
  }
  base_ = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  CH_CHECK(base_ != MAP_FAILED, "mmap shm failed");
  auto* h = static_cast<ShmHeader*>(base_);
  if (rank == 0) {
    h->count.store(0);
    h->sense.store(0);
    h->nranks = nranks;
    h->slot_bytes = slot_bytes_;
    h->ready.store(0x5eed);
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    while (h->ready.load() != 0x5eed) {
      CH_CHECK(std::chrono::steady_clock::now() - t0 < std::chrono::seconds(120), "timeout waiting for shm init");
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  }
  barrier();
}

ShmComm::~ShmComm() {
  try {
    if (!failed_) barrier();
  } catch (...) {
  }
  if (base_) munmap(base_, bytes_);
  if (rank_ == 0) shm_unlink(name_.c_str());
}

void ShmComm::barrier() {
  auto* h = static_cast<ShmHeader*>(base_);
  const int my_sense = 1 - h->sense.load();
  if (h->count.fetch_add(1) == size_ - 1) {
    h->count.store(0);
    h->sense.store(my_sense);
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    while (h->sense.load() != my_sense) {
      CH_CHECK(!failed_, "ShmComm: communicator was aborted");
      if (timeout_s_ > 0 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s_) {
        failed_ = true;
        CH_CHECK(false, "ShmComm barrier timeout after " << timeout_s_ << " s (a peer rank died or hung)");
      }
      std::this_thread::yield();
    }
  }
}

char* ShmComm::slot(int src, int dst) {
  return static_cast<char*>(base_) + kHdr + (static_cast<size_t>(src) * size_ + dst) * slot_bytes_;
}

void ShmComm::alltoallv(const void* send, const std::vector<size_t>& scount, const std::vector<size_t>& soff,
                        void* recv, const std::vector<size_t>& rcount, const std::vector<size_t>& roff,
                        hipStream_t s) {
  HIP_CHECK(hipStreamSynchronize(s));
  if (scount[rank_]) {  // self block: device-to-device, never through host memory
    CH_CHECK(scount[rank_] == rcount[rank_], "alltoallv: self block send/recv sizes differ");
    HIP_CHECK(hipMemcpy(static_cast<char*>(recv) + roff[rank_], static_cast<const char*>(send) + soff[rank_],
                        scount[rank_], hipMemcpyDeviceToDevice));
  }
  for (int p = 0; p < size_; ++p) {
    if (p == rank_) continue;
    CH_CHECK(scount[p] <= slot_bytes_ && rcount[p] <= slot_bytes_,
             "ShmComm slot too small (" << scount[p] << " bytes); set CHANNEL_SHM_SLOT_MB");
    if (scount[p])
      HIP_CHECK(hipMemcpy(slot(rank_, p), static_cast<const char*>(send) + soff[p], scount[p], hipMemcpyDeviceToHost));
  }
  barrier();
  for (int p = 0; p < size_; ++p)
    if (p != rank_ && rcount[p])
      HIP_CHECK(hipMemcpy(static_cast<char*>(recv) + roff[p], slot(p, rank_), rcount[p], hipMemcpyHostToDevice));
  barrier();
}

template <typename T, typename Op>
void ShmComm::allreduce(T* buf, size_t n, hipStream_t s, Op op) {
  HIP_CHECK(hipStreamSynchronize(s));
  CH_CHECK(n * sizeof(T) <= slot_bytes_, "ShmComm allreduce too large");
  HIP_CHECK(hipMemcpy(slot(rank_, 0), buf, n * sizeof(T), hipMemcpyDeviceToHost));
  barrier();
  std::vector<T> acc(n);
  std::memcpy(acc.data(), slot(0, 0), n * sizeof(T));
  for (int p = 1; p < size_; ++p) {
    const T* v = reinterpret_cast<const T*>(slot(p, 0));
    for (size_t i = 0; i < n; ++i) acc[i] = op(acc[i], v[i]);
  }
  barrier();
  HIP_CHECK(hipMemcpy(buf, acc.data(), n * sizeof(T), hipMemcpyHostToDevice));
}

void ShmComm::allreduce_max_f32(float* buf, size_t n, hipStream_t s) {
  allreduce(buf, n, s, [](float a, float b) { return a > b ? a : b; });
}
void ShmComm::allreduce_sum_f64(double* buf, size_t n, hipStream_t s) {
  allreduce(buf, n, s, [](double a, double b) { return a + b; });
}
void ShmComm::allreduce_max_f64(double* buf, size_t n, hipStream_t s) {
  allreduce(buf, n, s, [](double a, double b) { return a > b ? a : b; });
}
void ShmComm::allreduce_max_u32(unsigned* buf, size_t n, hipStream_t s) {
  allreduce(buf, n, s, [](unsigned a, unsigned b) { return a > b ? a : b; });
}

}  // namespace channel
