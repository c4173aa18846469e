#include "net.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <thread>

#include "../core/common.hpp"

namespace heat3d {
namespace net {

static sockaddr_in resolve(const std::string& host, int port) {
  sockaddr_in a;
  std::memset(&a, 0, sizeof(a));
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (host.empty() || host == "0.0.0.0") {
    a.sin_addr.s_addr = htonl(INADDR_ANY);
    return a;
  }
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) == 1) return a;
  addrinfo hints, *res = nullptr;
  std::memset(&hints, 0, sizeof(hints));
  hints.ai_family = AF_INET;
  if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res)
    HEAT3D_THROW("cannot resolve host '" << host << "'");
  a.sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
  freeaddrinfo(res);
  return a;
}

static void tune(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int buf = 4 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

int listen_on(const std::string& host, int port, int* bound_port) {
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) HEAT3D_THROW("socket() failed: " << std::strerror(errno));
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a = resolve(host, port);
  if (bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
    int e = errno;
    ::close(fd);
    HEAT3D_THROW("bind(" << host << ":" << port << ") failed: " << std::strerror(e));
  }
  if (listen(fd, 128) != 0) HEAT3D_THROW("listen failed: " << std::strerror(errno));
  if (bound_port) {
    socklen_t len = sizeof(a);
    getsockname(fd, reinterpret_cast<sockaddr*>(&a), &len);
    *bound_port = ntohs(a.sin_port);
  }
  return fd;
}

int accept_one(int lfd, double timeout_s) {
  pollfd p{lfd, POLLIN, 0};
  int r = poll(&p, 1, static_cast<int>(timeout_s * 1000));
  if (r <= 0) HEAT3D_THROW("accept timed out after " << timeout_s << " s");
  int fd = accept(lfd, nullptr, nullptr);
  if (fd < 0) HEAT3D_THROW("accept failed: " << std::strerror(errno));
  tune(fd);
  return fd;
}

int connect_to(const std::string& host, int port, double timeout_s) {
  auto t0 = std::chrono::steady_clock::now();
  sockaddr_in a = resolve(host, port);
  while (true) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) HEAT3D_THROW("socket() failed: " << std::strerror(errno));
    if (connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0) {
      tune(fd);
      return fd;
    }
    ::close(fd);
    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > timeout_s) HEAT3D_THROW("connect to " << host << ":" << port << " timed out");
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

void send_all(int fd, const void* p, std::size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      HEAT3D_THROW("send failed: " << std::strerror(errno));
    }
    c += w;
    n -= static_cast<std::size_t>(w);
  }
}

void recv_all(int fd, void* p, std::size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    ssize_t r = ::recv(fd, c, n, 0);
    if (r < 0) {
      if (errno == EINTR) continue;
      HEAT3D_THROW("recv failed: " << std::strerror(errno));
    }
    if (r == 0) HEAT3D_THROW("peer closed the connection");
    c += r;
    n -= static_cast<std::size_t>(r);
  }
}

void close_fd(int fd) {
  if (fd >= 0) ::close(fd);
}

std::string local_ip_for(const std::string& peer_host) {
  // the address of the interface that routes to the peer (UDP connect trick)
  int fd = socket(AF_INET, SOCK_DGRAM, 0);
  sockaddr_in a = resolve(peer_host, 9);
  std::string ip = "127.0.0.1";
  if (connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0) {
    sockaddr_in me;
    socklen_t len = sizeof(me);
    if (getsockname(fd, reinterpret_cast<sockaddr*>(&me), &len) == 0) {
      char buf[64];
      inet_ntop(AF_INET, &me.sin_addr, buf, sizeof(buf));
      ip = buf;
    }
  }
  ::close(fd);
  return ip;
}

Bootstrap::Bootstrap(int rank, int size, const std::string& master_addr, int port, double timeout_s)
    : rank_(rank), size_(size) {
  if (size_ <= 1) return;
  if (rank_ == 0) {
    lfd_ = listen_on("0.0.0.0", port, nullptr);
    fds_.assign(size_, -1);
    for (int i = 1; i < size_; ++i) {
      int fd = accept_one(lfd_, timeout_s);
      int32_t peer = -1;
      recv_all(fd, &peer, sizeof(peer));
      if (peer <= 0 || peer >= size_ || fds_[peer] >= 0) HEAT3D_THROW("bootstrap: bad peer rank " << peer);
      fds_[peer] = fd;
    }
  } else {
    int fd = connect_to(master_addr, port, timeout_s);
    int32_t me = rank_;
    send_all(fd, &me, sizeof(me));
    fds_.assign(1, fd);
  }
}

Bootstrap::~Bootstrap() {
  for (int fd : fds_) close_fd(fd);
  close_fd(lfd_);
}

std::vector<std::string> Bootstrap::allgather(const std::string& blob) {
  std::vector<std::string> all(size_);
  if (size_ <= 1) {
    all[0] = blob;
    return all;
  }
  auto put = [](int fd, const std::string& s) {
    uint64_t n = s.size();
    send_all(fd, &n, sizeof(n));
    if (n) send_all(fd, s.data(), n);
  };
  auto get = [](int fd) {
    uint64_t n = 0;
    recv_all(fd, &n, sizeof(n));
    std::string s(n, '\0');
    if (n) recv_all(fd, &s[0], n);
    return s;
  };
  if (rank_ == 0) {
    all[0] = blob;
    for (int i = 1; i < size_; ++i) all[i] = get(fds_[i]);
    for (int i = 1; i < size_; ++i)
      for (int r = 0; r < size_; ++r) put(fds_[i], all[r]);
  } else {
    put(fds_[0], blob);
    for (int r = 0; r < size_; ++r) all[r] = get(fds_[0]);
  }
  return all;
}

void Bootstrap::barrier() { allgather(std::string()); }

}  // namespace net
}  // namespace heat3d
