// heat3d-mi355x — communication layer.
//
// The reference moves every halo through host std::vector buffers with
// MPI_Isend/MPI_Recv/MPI_Waitall (heat3D.cu:610-755) and reduces scalars with
// blocking MPI_Iallreduce+Wait (heat3D.cu:1037-1063, 1103-1104) — despite the
// repository name nothing is CUDA-aware.  Here a Comm moves
// device (or host, for the CPU backend) buffers stream-ordered:
//   * RcclComm   — ncclSend/ncclRecv in one group + ncclAllReduce on device
//                  pointers over xGMI, two communicators (halo, reduction) so
//                  the scalar all-reduce never queues behind halo traffic;
//   * SocketComm — TCP transport between CPU-backend processes (the host-MPI
//                  analogue, used for multi-process CPU runs and tests);
//   * LocalComm  — P virtual ranks inside one process (single-GPU tests of
//                  the multi-rank code path; RCCL refuses two ranks per GPU).
#pragma once

#include <cstddef>
#include <memory>
#include <string>
#include <vector>

#include "../runtime/backend.hpp"

namespace heat3d {

namespace net {
class Bootstrap;
}

enum class RedOp { Max, Sum };
enum class RedType { U64, F64, I32 };

// One directed halo message.  `src` is valid when src_rank is hosted by this
// process, `dst` when dst_rank is.
struct Transfer {
  int src_rank = -1, dst_rank = -1;
  const void* src = nullptr;
  void* dst = nullptr;
  std::size_t bytes = 0;
};

class Comm {
 public:
  virtual ~Comm() = default;
  virtual const char* name() const = 0;
  virtual int size() const = 0;
  virtual std::vector<int> local_ranks() const = 0;
  // Buffers passed to exchange/allreduce/send/recv must be device memory.
  virtual bool device_buffers() const = 0;
  // Safe to record inside a hipGraph stream capture.
  virtual bool capturable() const { return false; }
  // True when all ranks live in this process and share one DeviceState
  // (no reduction needed, halos are direct copies).
  virtual bool all_local() const { return false; }
  // Ranks as counted by the transport itself (RCCL: ncclCommCount), so a run
  // report can prove the communicator really spans the job.
  virtual int transport_ranks() const { return size(); }
  // True when exchange() and allreduce() are device-side collectives of one
  // job-wide ordering domain (RCCL): the solver then chains every such call
  // behind the previous one with events, so all ranks' GPUs execute them in
  // one identical total order (see Solver::comm_token_*).
  virtual bool ordered_collectives() const { return false; }

  virtual void exchange(const std::vector<Transfer>& xs, Backend& be, StreamId s) = 0;
  virtual void allreduce(void* buf, std::size_t count, RedType t, RedOp op, Backend& be,
                         StreamId s) = 0;
  virtual void send(const void* buf, std::size_t bytes, int peer, Backend& be, StreamId s) = 0;
  virtual void recv(void* buf, std::size_t bytes, int peer, Backend& be, StreamId s) = 0;
  virtual void barrier(Backend& be) = 0;
  // Failure detection: throws if the transport reported an asynchronous error.
  virtual void check_async_error() {}
  virtual void abort() {}
};

std::unique_ptr<Comm> make_local_comm(int nranks);
// TCP transport: peers found through the bootstrap (one process per rank).
std::unique_ptr<Comm> make_socket_comm(int rank, int size, net::Bootstrap& boot);
// Same, with the peer listening addresses supplied by the caller (Python
// passes them through torch.distributed); `listen_fd` is this rank's socket.
std::unique_ptr<Comm> make_socket_comm_from_table(int rank, int size, int listen_fd,
                                                  const std::vector<std::string>& addrs);

// A host transport (socket) used by a GPU backend: device buffers are staged
// through host memory on the caller's stream (the reference's MPI data path).
std::unique_ptr<Comm> make_staged_comm(std::unique_ptr<Comm> inner);

// Performance proxy: rank `rank` of a `size`-rank job alone on one device,
// peers emulated (phantom_comm.cpp): every exchange holds `channels`
// workgroups per peer for bytes / gbps, every all-reduce
// `allreduce_channels` workgroups for allreduce_us.
struct PhantomOptions {
  double gbps = 50.0, allreduce_us = 20.0;
  int channels = 4, allreduce_channels = 2;
  // false: an exchange is its wire time (bytes / gbps) followed by the D2D
  // copies that stand in for the data; true: the copies run inside the wire
  // time (an exchange lasts max(wire, copies)), as a transport that moves the
  // data while it is on the wire
  bool overlap_copies = false;
  // paced: the copies themselves move the data at the wire rate, `channels`
  // workgroups per transfer for the wire time (RCCL-like: a few channels
  // stream the face across the link; no burst copy after the wire time)
  bool paced = false;
  // the delay / copy kernels in RCCL's device-kernel footprint (256 threads,
  // 140 VGPRs, 20 KB LDS), so that they wait for CUs as RCCL's kernel does
  // (opt-in: the proxy numbers of rounds 2-5 use the small kernels)
  bool rccl_footprint = false;
};
std::unique_ptr<Comm> make_phantom_comm(int rank, int size, const PhantomOptions& o = {});

// RCCL: `unique_id` is the 128-byte ncclUniqueId from rank 0.
bool rccl_available();
std::string rccl_unique_id();
std::string rccl_version();
std::string rccl_library_path();  // the librccl.so.1 this process is bound to
// shared: one communicator for halos and all-reduces (else a second one from
// ncclCommSplit); graph: its calls may be recorded into hipGraphs.
struct RcclOptions {
  bool shared = false, graph = false;
  // RCCL's P2P channel pool (NCCL_MAX_P2P_NCHANNELS, exported before the
  // first communicator of the process unless the environment sets it):
  // > 0 that many, 0 = leave RCCL's default
  int p2p_channels = 0;
};
// The NCCL_MAX_P2P_NCHANNELS this process's communicators were created
// with ("" = RCCL's default)
std::string rccl_p2p_channels_env();
std::unique_ptr<Comm> make_rccl_comm(int rank, int size, const std::string& unique_id, int device,
                                     const RcclOptions& o = {});

}  // namespace heat3d
