// heat3d-mi355x — minimal TCP utilities and an out-of-band bootstrap.
//
// Replaces MPI_Init / MPI_Comm_rank (heat3D.cu:203-205) for the native CLI:
// processes find each other through MASTER_ADDR / MASTER_PORT-style env vars
// (torchrun compatible) and use the bootstrap to all-gather small blobs — the
// RCCL unique id, or the listening addresses of the socket transport.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace heat3d {
namespace net {

int listen_on(const std::string& host, int port, int* bound_port);  // port 0 = ephemeral
int accept_one(int lfd, double timeout_s);
int connect_to(const std::string& host, int port, double timeout_s);
void send_all(int fd, const void* p, std::size_t n);
void recv_all(int fd, void* p, std::size_t n);
void close_fd(int fd);
std::string local_ip_for(const std::string& peer_host);

// Star-topology bootstrap: rank 0 listens on `port`; every other rank
// connects.  allgather() returns every rank's blob in rank order.
class Bootstrap {
 public:
  Bootstrap(int rank, int size, const std::string& master_addr, int port, double timeout_s = 120.0);
  ~Bootstrap();
  std::vector<std::string> allgather(const std::string& blob);
  void barrier();
  int rank() const { return rank_; }
  int size() const { return size_; }

 private:
  int rank_, size_;
  int lfd_ = -1;
  std::vector<int> fds_;  // rank 0: fd per peer; others: fds_[0] = link to rank 0
};

}  // namespace net
}  // namespace heat3d
