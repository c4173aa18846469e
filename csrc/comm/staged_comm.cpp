// heat3d-mi355x — StagedComm: a host transport (sockets) driven with device buffers.
//
// The reference's actual data path: GPU results are copied to host buffers and
// moved by a host-only transport (MPI Isend/Recv on host arrays,
// heat3D.cu:610-755; its "CUDA-aware" name notwithstanding).  Here it is the
// fallback for GPU ranks without RCCL (e.g. several processes sharing one
// device, which RCCL refuses: "Duplicate GPU detected") and the way the
// multi-process GPU schedule — overlapped streams, deep halos, lagged
// all-reduce — is exercised on a one-GPU box.
//
// Every operation copies device -> host on the caller's stream (so it is
// ordered exactly like an RCCL call enqueued there), synchronises that stream,
// runs the host transport, then copies host -> device on the same stream and
// synchronises again.  Correct and simple; not a production path (the host
// blocks per exchange and nothing is graph-capturable).
#include <cstring>
#include <vector>

#include "comm.hpp"

namespace heat3d {

namespace {

class StagedComm final : public Comm {
 public:
  explicit StagedComm(std::unique_ptr<Comm> inner) : inner_(std::move(inner)) {
    HEAT3D_CHECK(inner_ && !inner_->device_buffers() && inner_->local_ranks().size() == 1,
                 "staged comm wraps a single-rank host transport");
    rank_ = inner_->local_ranks()[0];
    name_ = std::string("staged-") + inner_->name();
  }
  const char* name() const override { return name_.c_str(); }
  int size() const override { return inner_->size(); }
  std::vector<int> local_ranks() const override { return inner_->local_ranks(); }
  bool device_buffers() const override { return true; }
  bool capturable() const override { return false; }

  void exchange(const std::vector<Transfer>& xs, Backend& be, StreamId s) override {
    std::vector<std::vector<char>> host(xs.size());
    std::vector<Transfer> hx;
    hx.reserve(xs.size());
    bool any_send = false;
    for (std::size_t i = 0; i < xs.size(); ++i) {
      const Transfer& x = xs[i];
      if (x.src_rank == rank_ && x.dst_rank == rank_) {
        be.copy(x.dst, x.src, x.bytes, CopyKind::D2D, s);
        continue;
      }
      if (x.src_rank != rank_ && x.dst_rank != rank_) continue;
      host[i].resize(x.bytes);
      Transfer h = x;
      if (x.src_rank == rank_) {
        be.copy(host[i].data(), x.src, x.bytes, CopyKind::D2H, s);
        h.src = host[i].data();
        any_send = true;
      } else {
        h.dst = host[i].data();
      }
      hx.push_back(h);
    }
    if (any_send) be.sync(s);
    if (hx.empty()) return;
    inner_->exchange(hx, be, s);
    bool any_recv = false;
    for (std::size_t i = 0; i < xs.size(); ++i)
      if (xs[i].dst_rank == rank_ && xs[i].src_rank != rank_) {
        be.copy(xs[i].dst, host[i].data(), xs[i].bytes, CopyKind::H2D, s);
        any_recv = true;
      }
    if (any_recv) be.sync(s);  // host buffers die with this frame
  }
  void allreduce(void* buf, std::size_t count, RedType t, RedOp op, Backend& be,
                 StreamId s) override {
    const std::size_t bytes = (t == RedType::I32 ? 4 : 8) * count;
    std::vector<char> h(bytes);
    be.copy(h.data(), buf, bytes, CopyKind::D2H, s);
    be.sync(s);
    inner_->allreduce(h.data(), count, t, op, be, s);
    be.copy(buf, h.data(), bytes, CopyKind::H2D, s);
    be.sync(s);
  }
  void send(const void* buf, std::size_t bytes, int peer, Backend& be, StreamId s) override {
    std::vector<char> h(bytes);
    be.copy(h.data(), buf, bytes, CopyKind::D2H, s);
    be.sync(s);
    inner_->send(h.data(), bytes, peer, be, s);
  }
  void recv(void* buf, std::size_t bytes, int peer, Backend& be, StreamId s) override {
    std::vector<char> h(bytes);
    inner_->recv(h.data(), bytes, peer, be, s);
    be.copy(buf, h.data(), bytes, CopyKind::H2D, s);
    be.sync(s);
  }
  void barrier(Backend& be) override { inner_->barrier(be); }
  void check_async_error() override { inner_->check_async_error(); }
  void abort() override { inner_->abort(); }

 private:
  std::unique_ptr<Comm> inner_;
  int rank_ = 0;
  std::string name_;
};

}  // namespace

std::unique_ptr<Comm> make_staged_comm(std::unique_ptr<Comm> inner) {
  return std::unique_ptr<Comm>(new StagedComm(std::move(inner)));
}

}  // namespace heat3d
