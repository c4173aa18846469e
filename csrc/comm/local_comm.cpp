// heat3d-mi355x — LocalComm: P virtual ranks hosted by one process.
//
// All subdomains share one device and one DeviceState, so halos are direct
// device-to-device box copies issued by the solver and reductions are
// implicit (every subdomain's kernel max-reduces into the same word).  This is
// how multi-rank behaviour is tested on the single-GPU gpurun box
// (SURVEY.md §4 item 3, §7.4 item 7).
#include <numeric>

#include "comm.hpp"

namespace heat3d {

namespace {

class LocalComm final : public Comm {
 public:
  explicit LocalComm(int n) : n_(n) {}
  const char* name() const override { return "local"; }
  int size() const override { return n_; }
  std::vector<int> local_ranks() const override {
    std::vector<int> r(n_);
    std::iota(r.begin(), r.end(), 0);
    return r;
  }
  bool device_buffers() const override { return false; }
  bool capturable() const override { return true; }
  bool all_local() const override { return true; }
  void exchange(const std::vector<Transfer>& xs, Backend& be, StreamId s) override {
    for (const auto& x : xs) {
      HEAT3D_CHECK(x.src && x.dst, "local transfer needs both ends");
      be.copy(x.dst, x.src, x.bytes, be.is_gpu() ? CopyKind::D2D : CopyKind::H2H, s);
    }
  }
  void allreduce(void*, std::size_t, RedType, RedOp, Backend&, StreamId) override {}
  void send(const void*, std::size_t, int, Backend&, StreamId) override {
    HEAT3D_THROW("LocalComm has no remote peers");
  }
  void recv(void*, std::size_t, int, Backend&, StreamId) override {
    HEAT3D_THROW("LocalComm has no remote peers");
  }
  void barrier(Backend&) override {}

 private:
  int n_;
};

}  // namespace

std::unique_ptr<Comm> make_local_comm(int nranks) {
  return std::unique_ptr<Comm>(new LocalComm(nranks));
}

}  // namespace heat3d
