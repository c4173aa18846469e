// heat3d-mi355x — SocketComm: TCP transport between CPU-backend processes.
//
// The host-buffer analogue of the reference's MPI usage (Isend/Recv/Waitall
// halos, heat3D.cu:610-755; Iallreduce scalars, heat3D.cu:1037-1104) for runs
// and tests without a GPU.  A full mesh of TCP connections is built once;
// an exchange drives all of this rank's sends and receives concurrently with
// poll(), so no ordering between neighbours can deadlock.
#include <fcntl.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <sstream>

#include "comm.hpp"
#include "net.hpp"

namespace heat3d {

namespace {

class SocketComm final : public Comm {
 public:
  // addrs[r] = "host:port" of rank r's listening socket.
  SocketComm(int rank, int size, int listen_fd, const std::vector<std::string>& addrs)
      : rank_(rank), size_(size), fds_(size, -1) {
    // rank i accepts connections from every j > i and connects to every j < i
    for (int j = 0; j < rank_; ++j) {
      auto pos = addrs[j].rfind(':');
      std::string host = addrs[j].substr(0, pos);
      int port = std::atoi(addrs[j].c_str() + pos + 1);
      int fd = net::connect_to(host, port, 120.0);
      int32_t me = rank_;
      net::send_all(fd, &me, sizeof(me));
      fds_[j] = fd;
    }
    for (int n = rank_ + 1; n < size_; ++n) {
      int fd = net::accept_one(listen_fd, 120.0);
      int32_t peer = -1;
      net::recv_all(fd, &peer, sizeof(peer));
      HEAT3D_CHECK(peer > rank_ && peer < size_ && fds_[peer] < 0, "socket comm: bad peer " << peer);
      fds_[peer] = fd;
    }
    net::close_fd(listen_fd);
  }
  ~SocketComm() override {
    for (int fd : fds_) net::close_fd(fd);
  }
  const char* name() const override { return "socket"; }
  int size() const override { return size_; }
  std::vector<int> local_ranks() const override { return {rank_}; }
  bool device_buffers() const override { return false; }

  void exchange(const std::vector<Transfer>& xs, Backend&, StreamId) override {
    struct Op {
      int fd;
      char* p;
      std::size_t left;
      bool send;
    };
    std::vector<Op> ops;
    for (const auto& x : xs) {
      if (x.src_rank == rank_ && x.dst_rank == rank_) {
        std::memmove(x.dst, x.src, x.bytes);
      } else if (x.src_rank == rank_) {
        ops.push_back({fds_.at(x.dst_rank), (char*)x.src, x.bytes, true});
      } else if (x.dst_rank == rank_) {
        ops.push_back({fds_.at(x.src_rank), (char*)x.dst, x.bytes, false});
      }
    }
    run(ops.data(), ops.size());
  }

  void allreduce(void* buf, std::size_t count, RedType t, RedOp op, Backend&, StreamId) override {
    const std::size_t es = t == RedType::I32 ? 4 : 8;
    const std::size_t bytes = es * count;
    std::vector<std::vector<char>> all(size_, std::vector<char>(bytes));
    std::memcpy(all[rank_].data(), buf, bytes);
    struct Op {
      int fd;
      char* p;
      std::size_t left;
      bool send;
    };
    std::vector<Op> ops;
    for (int r = 0; r < size_; ++r) {
      if (r == rank_) continue;
      ops.push_back({fds_[r], all[rank_].data(), bytes, true});
      ops.push_back({fds_[r], all[r].data(), bytes, false});
    }
    run(ops.data(), ops.size());
    // combine in rank order: identical result on every rank
    for (std::size_t i = 0; i < count; ++i) {
      if (t == RedType::F64) {
        double acc = 0;
        for (int r = 0; r < size_; ++r) {
          double v;
          std::memcpy(&v, all[r].data() + i * 8, 8);
          acc = r == 0 ? v : (op == RedOp::Sum ? acc + v : (v > acc ? v : acc));
        }
        std::memcpy(static_cast<char*>(buf) + i * 8, &acc, 8);
      } else if (t == RedType::U64) {
        unsigned long long acc = 0;
        for (int r = 0; r < size_; ++r) {
          unsigned long long v;
          std::memcpy(&v, all[r].data() + i * 8, 8);
          acc = r == 0 ? v : (op == RedOp::Sum ? acc + v : (v > acc ? v : acc));
        }
        std::memcpy(static_cast<char*>(buf) + i * 8, &acc, 8);
      } else {
        int32_t acc = 0;
        for (int r = 0; r < size_; ++r) {
          int32_t v;
          std::memcpy(&v, all[r].data() + i * 4, 4);
          acc = r == 0 ? v : (op == RedOp::Sum ? acc + v : (v > acc ? v : acc));
        }
        std::memcpy(static_cast<char*>(buf) + i * 4, &acc, 4);
      }
    }
  }

  void send(const void* buf, std::size_t bytes, int peer, Backend&, StreamId) override {
    net::send_all(fds_.at(peer), buf, bytes);
  }
  void recv(void* buf, std::size_t bytes, int peer, Backend&, StreamId) override {
    net::recv_all(fds_.at(peer), buf, bytes);
  }
  void barrier(Backend& be) override {
    int32_t z = 0;
    allreduce(&z, 1, RedType::I32, RedOp::Max, be, kCompute);
  }

 private:
  template <typename OpT>
  void run(OpT* ops, std::size_t n) {
    // all sockets non-blocking while the exchange is in flight
    for (std::size_t i = 0; i < n; ++i) {
      int fl = fcntl(ops[i].fd, F_GETFL, 0);
      fcntl(ops[i].fd, F_SETFL, fl | O_NONBLOCK);
    }
    // per fd, ops of one direction are serviced in list order
    std::size_t pending = 0;
    for (std::size_t i = 0; i < n; ++i) pending += ops[i].left ? 1 : 0;
    while (pending) {
      std::vector<pollfd> pf;
      std::vector<std::size_t> idx;
      for (std::size_t i = 0; i < n; ++i) {
        if (!ops[i].left) continue;
        // only the first unfinished op per (fd, direction)
        bool first = true;
        for (std::size_t j = 0; j < i; ++j)
          if (ops[j].left && ops[j].fd == ops[i].fd && ops[j].send == ops[i].send) first = false;
        if (!first) continue;
        pf.push_back({ops[i].fd, static_cast<short>(ops[i].send ? POLLOUT : POLLIN), 0});
        idx.push_back(i);
      }
      int r = poll(pf.data(), pf.size(), 120000);
      if (r <= 0) HEAT3D_THROW("socket comm: exchange timed out (peer dead?)");
      for (std::size_t q = 0; q < pf.size(); ++q) {
        if (!pf[q].revents) continue;
        auto& o = ops[idx[q]];
        if (pf[q].revents & (POLLERR | POLLNVAL)) HEAT3D_THROW("socket comm: connection error");
        ssize_t k = o.send ? ::send(o.fd, o.p, o.left, MSG_NOSIGNAL) : ::recv(o.fd, o.p, o.left, 0);
        if (k < 0) {
          if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) continue;
          HEAT3D_THROW("socket comm: " << std::strerror(errno));
        }
        if (k == 0 && !o.send) HEAT3D_THROW("socket comm: peer closed the connection");
        o.p += k;
        o.left -= static_cast<std::size_t>(k);
        if (!o.left) --pending;
      }
    }
    for (std::size_t i = 0; i < n; ++i) {
      int fl = fcntl(ops[i].fd, F_GETFL, 0);
      fcntl(ops[i].fd, F_SETFL, fl & ~O_NONBLOCK);
    }
  }

  int rank_, size_;
  std::vector<int> fds_;
};

}  // namespace

std::unique_ptr<Comm> make_socket_comm_from_table(int rank, int size, int listen_fd,
                                                  const std::vector<std::string>& addrs) {
  HEAT3D_CHECK((int)addrs.size() == size, "address table size mismatch");
  return std::unique_ptr<Comm>(new SocketComm(rank, size, listen_fd, addrs));
}

std::unique_ptr<Comm> make_socket_comm(int rank, int size, net::Bootstrap& boot) {
  int port = 0;
  int lfd = net::listen_on("0.0.0.0", 0, &port);
  std::ostringstream os;
  os << net::local_ip_for("127.0.0.1") << ":" << port;
  auto addrs = boot.allgather(os.str());
  return make_socket_comm_from_table(rank, size, lfd, addrs);
}

}  // namespace heat3d
