// heat3d-mi355x — PhantomComm: one rank of a P-rank job, alone on one device.
//
// A performance proxy, not a transport: the process builds rank r's subdomain
// of a P-way decomposition and runs that rank's exact schedule (interior and
// boundary kernels, deep halos, streams, lagged all-reduce), while the peers
// are phantoms.  Received halos are filled with a same-sized face this rank
// sends (numerically meaningless, finite), every exchange occupies the stream
// for bytes-per-peer / --phantom-gbps, and every all-reduce for
// --phantom-allreduce-us.  Like RCCL, which moves p2p data with several
// channels (one workgroup each) per peer, the emulated transfer holds
// --phantom-channels workgroups per peer (default 4) for its duration, and
// the all-reduce one per ring channel (default 2): those workgroups must find
// free CUs next to the interior sweep, exactly the contention a real run has.
// Collectives are ordered like RCCL's (ordered_collectives).  This is how the
// per-GPU time of the multi-GPU bench is measured on the one-GPU box
// (tools/rank_proxy.py).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <map>

#include "comm.hpp"

namespace heat3d {

namespace {

class PhantomComm final : public Comm {
 public:
  PhantomComm(int rank, int size, const PhantomOptions& o)
      : rank_(rank), size_(size), gbps_(o.gbps), ar_us_(o.allreduce_us), channels_(o.channels),
        ar_channels_(o.allreduce_channels), overlap_(o.overlap_copies), paced_(o.paced),
        fat_(o.rccl_footprint) {
    HEAT3D_CHECK(rank >= 0 && rank < size, "phantom rank " << rank << " of " << size);
  }
  ~PhantomComm() override {
    if (slot_ && be_) be_->release(slot_);
  }
  const char* name() const override { return "phantom"; }
  int size() const override { return size_; }
  std::vector<int> local_ranks() const override { return {rank_}; }
  bool device_buffers() const override { return true; }
  bool capturable() const override { return true; }
  bool ordered_collectives() const override { return true; }

  void exchange(const std::vector<Transfer>& xs, Backend& be, StreamId s) override {
    be.set_comm_footprint(fat_);
    std::map<int, std::size_t> per_peer;
    for (const auto& x : xs)
      if (x.dst_rank == rank_ && x.src_rank != rank_) per_peer[x.src_rank] += x.bytes;
    std::size_t worst = 0;
    for (const auto& kv : per_peer) worst = std::max(worst, kv.second);
    // bytes / (GB/s) in us, every peer's channels in flight at once
    const double wire = worst && gbps_ > 0 ? worst / (gbps_ * 1e3) : 0.0;
    const int blocks = channels_ * (int)per_peer.size();
    // the paced copy moves 16-byte words: other transfers take the serial wire
    bool aligned16 = true;
    for (const auto& x : xs)
      aligned16 &= x.bytes % 16 == 0 && reinterpret_cast<std::uintptr_t>(x.src) % 16 == 0 &&
                   reinterpret_cast<std::uintptr_t>(x.dst) % 16 == 0;
    if (paced_ && wire > 0 && aligned16) {
      // every transfer from peer p ends bytes(p) / gbps after it starts
      // workgroups per transfer: the channels, and enough that none must
      // stream more than ~2 GB/s: a 256-lane group moves ~4 GB/s beside the
      // interior sweep whether it keeps four or eight 16-byte loads in flight
      // per lane (8 groups per 64 GB/s transfer ran the wire 2x long,
      // gpurun_out/r7x; 16 ran it 9-17 % long, r7m)
      // (at most 64, the copy kernel's limit: faster emulated links keep 64
      // groups, each then streaming more than ~2 GB/s)
      const int per = std::min(64, std::max(channels_, (int)std::ceil(gbps_ / 2.0)));
      std::vector<hip::PacedCopy> pc;
      for (const auto& x : xs) {
        if (x.dst_rank != rank_ || x.src_rank == rank_) continue;
        const void* src = nullptr;
        for (const auto& y : xs)
          if (y.src_rank == rank_ && y.bytes == x.bytes) src = y.src;
        if (!src) continue;
        const double peer_ticks = per_peer[x.src_rank] / (gbps_ * 1e3) * 100.0;  // 100 MHz clock
        const double share16 = std::max(1.0, std::ceil((double)(x.bytes / 16) / per));
        pc.push_back({src, x.dst, (int64_t)x.bytes, peer_ticks / share16});
      }
      be.paced_copy(pc, per, s);
      return;
    }
    // one clock stamp per stream: exchanges queued on different streams
    // (single-step halos, overlapped sweeps) must not share the stamp an
    // earlier delay_since still reads
    void* stamp = nullptr;
    if (overlap_ && wire > 0) {
      if (!slot_) {
        be_ = &be;
        slot_ = be.alloc(8 * kNumStreams);
      }
      stamp = static_cast<char*>(slot_) + 8 * (int)s;
      be.stamp(stamp, s);
    } else if (wire > 0) {
      be.delay(wire, s, blocks);
    }
    for (const auto& x : xs) {
      if (x.dst_rank != rank_ || x.src_rank == rank_) continue;
      const void* src = nullptr;
      for (const auto& y : xs)
        if (y.src_rank == rank_ && y.bytes == x.bytes) src = y.src;
      if (src) be.copy(x.dst, src, x.bytes, CopyKind::D2D, s);
    }
    if (overlap_ && wire > 0) be.delay_since(stamp, wire, s, blocks);
  }
  void allreduce(void*, std::size_t, RedType, RedOp, Backend& be, StreamId s) override {
    be.set_comm_footprint(fat_);
    if (ar_us_ > 0) be.delay(ar_us_, s, ar_channels_);
  }
  void send(const void*, std::size_t, int, Backend&, StreamId) override {}
  void recv(void*, std::size_t, int, Backend&, StreamId) override {}
  void barrier(Backend&) override {}

 private:
  int rank_, size_;
  double gbps_, ar_us_;
  int channels_, ar_channels_;
  bool overlap_, paced_, fat_;
  Backend* be_ = nullptr;  // owner of slot_ (outlives the communicator, ~Solver)
  void* slot_ = nullptr;   // device clock stamps of the exchanges in flight, one per stream
};

}  // namespace

std::unique_ptr<Comm> make_phantom_comm(int rank, int size, const PhantomOptions& o) {
  return std::unique_ptr<Comm>(new PhantomComm(rank, size, o));
}

}  // namespace heat3d
