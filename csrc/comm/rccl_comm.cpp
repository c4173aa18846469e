// heat3d-mi355x — RcclComm: halo exchange and reductions with RCCL over xGMI.
//
// Replaces the reference's host-staged MPI traffic (heat3D.cu:610-755,
// 1037-1063) with device-pointer RCCL calls enqueued on HIP streams:
//   * halo: ncclGroupStart; ncclSend/ncclRecv per neighbour face; ncclGroupEnd
//     (x faces are contiguous planes sent in place — no pack);
//   * convergence: ncclAllReduce(max) on the 8-byte residual words, on a second
//     communicator (ncclCommSplit) so that it does not queue behind halo traffic
//     inside RCCL's per-communicator stream ordering;
//   * failure detection: ncclCommGetAsyncError polling, ncclCommAbort on fault.
// On a fully connected 8x MI355X node every face neighbour is one direct xGMI
// link, so a slab drives 2 links per GPU and a 2x2x2 block 3.
//
// Ordering contract (why two communicators on two streams cannot deadlock or
// mismatch).  NCCL requires that every rank issue a communicator's operations
// in one order, and gives no order between operations of different
// communicators running on different streams.  The solver therefore never
// relies on the GPU's choice: it chains every collective it enqueues (halo
// group or all-reduce) behind the previous one with an event
// (Solver::comm_token_wait / comm_token_signal), and issues them in the same
// host order on every rank.  Each rank's GPU executes the collectives in one
// total order, identical across ranks, with at most one in flight.  The
// overlapped sweeps issue all-reduce(q) after halo(q+1) (Solver::enqueue_multi),
// so the chain costs the next halo nothing.  If ncclCommSplit is unavailable
// both kinds share one communicator: RCCL then serialises them in host issue
// order, which is the same total order.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <climits>
#include <cstdlib>
#include <cstring>
#include <sstream>

#include "comm.hpp"

namespace heat3d {

#define NCCL_CHECK(expr)                                                                \
  do {                                                                                  \
    ncclResult_t _r = (expr);                                                           \
    if (_r != ncclSuccess) HEAT3D_THROW("RCCL error '" << ncclGetErrorString(_r) << "' at " #expr); \
  } while (0)

bool rccl_available() { return true; }

std::string rccl_unique_id() {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

std::string rccl_version() {
  int v = 0;
  if (ncclGetVersion(&v) != ncclSuccess) return "unknown";
  std::ostringstream os;
  os << v / 10000 << "." << (v / 100) % 100 << "." << v % 100;
  return os.str();
}

// The file the dynamic linker bound librccl.so.1 to in this process (torch
// bundles a copy under the same soname; which one a process runs on depends
// on what it loaded first, so the bench records it).
std::string rccl_library_path() {
  Dl_info di;
  if (dladdr(reinterpret_cast<void*>(&ncclGetVersion), &di) && di.dli_fname) {
    char buf[4096];
    return realpath(di.dli_fname, buf) ? std::string(buf) : std::string(di.dli_fname);
  }
  return "unknown";
}

namespace {

ncclDataType_t to_nccl(RedType t) {
  switch (t) {
    case RedType::U64: return ncclUint64;
    case RedType::F64: return ncclFloat64;
    case RedType::I32: return ncclInt32;
  }
  return ncclUint64;
}

// Element type and count of a byte message: 8-byte words when the size allows
// (fewer, wider elements for RCCL's copy loops), else bytes.  Both sides of a
// transfer compute the same pair from the same byte count.
void message_shape(std::size_t bytes, ncclDataType_t* dt, std::size_t* count) {
  if (bytes % 8 == 0) {
    *dt = ncclUint64;
    *count = bytes / 8;
  } else {
    *dt = ncclUint8;
    *count = bytes;
  }
}

class RcclComm final : public Comm {
 public:
  RcclComm(int rank, int size, const std::string& uid, int device, const RcclOptions& o)
      : rank_(rank), size_(size), graph_(o.graph) {
    HEAT3D_CHECK(uid.size() == sizeof(ncclUniqueId), "bad ncclUniqueId size " << uid.size());
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    if (hipSetDevice(device) != hipSuccess) HEAT3D_THROW("hipSetDevice(" << device << ") failed");
    // P2P channel pool sized to the CUs the overlapped schedule keeps free
    // of the interior sweep (RCCL reads it at communicator initialisation;
    // an explicit NCCL_MAX_P2P_NCHANNELS in the environment wins)
    if (o.p2p_channels > 0 && !std::getenv("NCCL_MAX_P2P_NCHANNELS"))
      setenv("NCCL_MAX_P2P_NCHANNELS", std::to_string(o.p2p_channels).c_str(), 0);
    NCCL_CHECK(ncclCommInitRank(&halo_, size_, id, rank_));
    int n = 0;
    NCCL_CHECK(ncclCommCount(halo_, &n));
    HEAT3D_CHECK(n == size_, "RCCL communicator has " << n << " ranks, expected " << size_);
    // A second communicator for the scalar all-reduce (--rccl-shared forces
    // the single-communicator form, which tests exercise).
    if (o.shared || ncclCommSplit(halo_, 0, rank_, &red_, nullptr) != ncclSuccess || red_ == nullptr) {
      red_ = halo_;
      shared_ = true;
    }
  }
  ~RcclComm() override {
    if (bar_) (void)hipFree(bar_);
    if (red_ && !shared_) ncclCommDestroy(red_);
    if (halo_) ncclCommDestroy(halo_);
  }
  const char* name() const override { return shared_ ? "rccl(shared)" : "rccl"; }
  int size() const override { return size_; }
  std::vector<int> local_ranks() const override { return {rank_}; }
  bool device_buffers() const override { return true; }
  // RCCL calls are recorded into hipGraphs unless --no-rccl-graph (Config::rccl_graph, default on)
  bool capturable() const override { return graph_; }
  int transport_ranks() const override {
    int n = 0;
    if (!halo_ || ncclCommCount(halo_, &n) != ncclSuccess) return -1;
    return n;
  }
  bool ordered_collectives() const override { return true; }

  void exchange(const std::vector<Transfer>& xs, Backend& be, StreamId s) override {
    hipStream_t st = static_cast<hipStream_t>(be.op_begin(s));
    NCCL_CHECK(ncclGroupStart());
    for (const auto& x : xs) {
      ncclDataType_t dt;
      std::size_t cnt;
      message_shape(x.bytes, &dt, &cnt);
      // a transfer between two faces of this rank (periodic self-neighbour or
      // the 1-rank test) is a send and a receive to itself inside the group
      if (x.src_rank == rank_) NCCL_CHECK(ncclSend(x.src, cnt, dt, x.dst_rank, halo_, st));
      if (x.dst_rank == rank_) NCCL_CHECK(ncclRecv(x.dst, cnt, dt, x.src_rank, halo_, st));
    }
    NCCL_CHECK(ncclGroupEnd());
    be.op_end(s);
  }
  void allreduce(void* buf, std::size_t count, RedType t, RedOp op, Backend& be,
                 StreamId s) override {
    hipStream_t st = static_cast<hipStream_t>(be.op_begin(s));
    NCCL_CHECK(ncclAllReduce(buf, buf, count, to_nccl(t), op == RedOp::Max ? ncclMax : ncclSum,
                             red_, st));
    be.op_end(s);
  }
  void send(const void* buf, std::size_t bytes, int peer, Backend& be, StreamId s) override {
    hipStream_t st = static_cast<hipStream_t>(be.op_begin(s));
    ncclDataType_t dt;
    std::size_t cnt;
    message_shape(bytes, &dt, &cnt);
    NCCL_CHECK(ncclSend(buf, cnt, dt, peer, halo_, st));
    be.op_end(s);
  }
  void recv(void* buf, std::size_t bytes, int peer, Backend& be, StreamId s) override {
    hipStream_t st = static_cast<hipStream_t>(be.op_begin(s));
    ncclDataType_t dt;
    std::size_t cnt;
    message_shape(bytes, &dt, &cnt);
    NCCL_CHECK(ncclRecv(buf, cnt, dt, peer, halo_, st));
    be.op_end(s);
  }
  void barrier(Backend& be) override {
    if (!bar_ && hipMalloc(&bar_, 8) != hipSuccess) HEAT3D_THROW("hipMalloc failed");
    allreduce(bar_, 1, RedType::U64, RedOp::Max, be, kReduce);
    be.sync(kReduce);
  }
  void check_async_error() override {
    for (ncclComm_t c : {halo_, red_}) {
      ncclResult_t e = ncclSuccess;
      if (c && ncclCommGetAsyncError(c, &e) == ncclSuccess && e != ncclSuccess && e != ncclInProgress)
        HEAT3D_THROW("RCCL asynchronous error: " << ncclGetErrorString(e));
    }
  }
  void abort() override {
    if (red_ && !shared_) ncclCommAbort(red_);
    if (halo_) ncclCommAbort(halo_);
    red_ = halo_ = nullptr;
  }

 private:
  int rank_, size_;
  ncclComm_t halo_ = nullptr, red_ = nullptr;
  bool shared_ = false, graph_ = false;
  void* bar_ = nullptr;
};

}  // namespace

std::string rccl_p2p_channels_env() {
  const char* e = std::getenv("NCCL_MAX_P2P_NCHANNELS");
  return e ? std::string(e) : std::string();
}

std::unique_ptr<Comm> make_rccl_comm(int rank, int size, const std::string& unique_id, int device,
                                     const RcclOptions& o) {
  return std::unique_ptr<Comm>(new RcclComm(rank, size, unique_id, device, o));
}

}  // namespace heat3d
