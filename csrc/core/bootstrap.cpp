#include "channel/bootstrap.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "channel/common.hpp"

namespace channel {

namespace {
int env_int(std::initializer_list<const char*> names, int dflt) {
  for (const char* n : names) {
    const char* v = std::getenv(n);
    if (v && *v) return std::atoi(v);
  }
  return dflt;
}

void send_all(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n) {
    ssize_t k = ::send(fd, p, n, 0);
    CH_CHECK(k > 0, "bootstrap send failed");
    p += k;
    n -= static_cast<size_t>(k);
  }
}

void recv_all(int fd, void* buf, size_t n) {
  char* p = static_cast<char*>(buf);
  while (n) {
    ssize_t k = ::recv(fd, p, n, 0);
    CH_CHECK(k > 0, "bootstrap recv failed");
    p += k;
    n -= static_cast<size_t>(k);
  }
}
}  // namespace

ProcInfo ProcInfo::from_env() {
  ProcInfo p;
  p.rank = env_int({"RANK", "PMI_RANK", "OMPI_COMM_WORLD_RANK", "SLURM_PROCID"}, 0);
  p.size = env_int({"WORLD_SIZE", "PMI_SIZE", "OMPI_COMM_WORLD_SIZE", "SLURM_NTASKS"}, 1);
  p.local_rank = env_int({"LOCAL_RANK", "MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK", "SLURM_LOCALID"}, p.rank);
  CH_CHECK(p.size >= 1 && p.rank >= 0 && p.rank < p.size, "bad rank/size " << p.rank << "/" << p.size);
  return p;
}

std::string tcp_broadcast(const ProcInfo& pi, const std::string& payload, int timeout_s) {
  if (pi.size == 1) return payload;
  const char* addr_s = std::getenv("MASTER_ADDR");
  const char* port_s = std::getenv("MASTER_PORT");
  const std::string addr = addr_s && *addr_s ? addr_s : "127.0.0.1";
  // use a port distinct from torchrun's store port
  const int port = (port_s && *port_s ? std::atoi(port_s) : 29500) + 11;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s);
  if (pi.rank == 0) {
    int ls = ::socket(AF_INET, SOCK_STREAM, 0);
    CH_CHECK(ls >= 0, "socket failed");
    int one = 1;
    setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons(static_cast<uint16_t>(port));
    // Bind to MASTER_ADDR (only the interface the peers were told to use accepts connections; for
    // 127.0.0.1 that is the local host only).  Fallback to every interface when the address is not
    // local (NAT) so the bind fails, or when CHANNEL_BOOTSTRAP_BIND_ANY=1 (multi-node runs whose
    // MASTER_ADDR hostname resolves to a loopback alias on the master only).  Peers identify
    // themselves by rank; a duplicate or out-of-range rank is rejected below.
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    bool bound = false;
    const char* ba = std::getenv("CHANNEL_BOOTSTRAP_BIND_ANY");
    // a multi-node job (WORLD_SIZE > LOCAL_WORLD_SIZE) listens on every interface: its peers reach
    // the master from other hosts, whatever MASTER_ADDR resolves to locally
    const char* ws = std::getenv("WORLD_SIZE");
    const char* lws = std::getenv("LOCAL_WORLD_SIZE");
    const bool multinode = ws && lws && std::atoi(ws) > std::atoi(lws);
    if (!(ba && std::atoi(ba) == 1) && !multinode) {
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      if (getaddrinfo(addr.c_str(), nullptr, &hints, &res) == 0 && res) {
        sockaddr_in m = sa;
        m.sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
        freeaddrinfo(res);
        // a hostname that resolves to a loopback alias on the master only (127.0.1.1 through
        // /etc/hosts) would accept local peers and refuse remote ones: listen on every interface --
        // but only when the launcher does not say the job is single-node (no LOCAL_WORLD_SIZE);
        // a single-node job keeps the loopback bind (the bootstrap has no authentication)
        const bool single_node = ws && lws && std::atoi(ws) <= std::atoi(lws);
        const bool loop_alias = !single_node && (ntohl(m.sin_addr.s_addr) >> 24) == 127 && addr != "127.0.0.1" &&
                                addr != "localhost";
        if (loop_alias) {
          std::fprintf(stderr, "[channel] bootstrap: MASTER_ADDR %s resolves to a loopback address; listening on every interface\n",
                       addr.c_str());
        } else {
          bound = ::bind(ls, reinterpret_cast<sockaddr*>(&m), sizeof(m)) == 0;
          if (!bound)
            std::fprintf(stderr, "[channel] bootstrap: cannot bind MASTER_ADDR %s; listening on every interface\n",
                         addr.c_str());
        }
      }
    }
    CH_CHECK(bound || ::bind(ls, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) == 0,
             "bootstrap: bind to port " << port << " failed");
    CH_CHECK(::listen(ls, pi.size) == 0, "listen failed");
    std::vector<bool> seen(pi.size, false);
    seen[0] = true;
    for (int i = 1; i < pi.size; ++i) {
      // bounded wait: a peer that died before connecting is an error, not a hang
      pollfd pf{ls, POLLIN, 0};
      int left_ms = 0;
      while (true) {
        left_ms = static_cast<int>(std::chrono::duration_cast<std::chrono::milliseconds>(
                                       deadline - std::chrono::steady_clock::now()).count());
        CH_CHECK(left_ms > 0, "bootstrap: only " << i - 1 << " of " << pi.size - 1 << " peers connected within "
                                                 << timeout_s << " s");
        const int pr = ::poll(&pf, 1, std::min(left_ms, 1000));
        if (pr > 0) break;
      }
      int fd = ::accept(ls, nullptr, nullptr);
      CH_CHECK(fd >= 0, "accept failed");
      timeval tv{};
      tv.tv_sec = std::max(1, left_ms / 1000);
      setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
      int32_t peer = -1;
      recv_all(fd, &peer, sizeof(peer));
      CH_CHECK(peer > 0 && peer < pi.size && !seen[peer],
               "bootstrap: unexpected peer rank " << peer << " (world size " << pi.size << ")");
      seen[peer] = true;
      const uint64_t n = payload.size();
      send_all(fd, &n, sizeof(n));
      send_all(fd, payload.data(), payload.size());
      ::close(fd);
    }
    ::close(ls);
    return payload;
  }
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  CH_CHECK(getaddrinfo(addr.c_str(), std::to_string(port).c_str(), &hints, &res) == 0 && res,
           "cannot resolve MASTER_ADDR " << addr);
  int fd = -1;
  while (true) {
    fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0) break;
    ::close(fd);
    CH_CHECK(std::chrono::steady_clock::now() < deadline, "bootstrap connect timeout to " << addr << ":" << port);
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  freeaddrinfo(res);
  const int32_t me = pi.rank;
  send_all(fd, &me, sizeof(me));
  uint64_t n = 0;
  recv_all(fd, &n, sizeof(n));
  std::string out(n, '\0');
  recv_all(fd, out.data(), n);
  ::close(fd);
  return out;
}

}  // namespace channel
