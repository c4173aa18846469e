// heat3d-mi355x — execution backend (HIP device or CPU host).
//
// The reference allocated, copied and freed device buffers and re-selected the
// device inside every iteration (heat3D.cu:644-716).  A Backend is
// created once: it owns the device binding, three streams (compute, comm,
// reduce — SURVEY.md §7.2 step 6), an event pool and all allocations; the
// solver only enqueues work.  The CPU backend runs everything synchronously
// with OpenMP and turns stream/event calls into no-ops.
#pragma once

#include <cstddef>
#include <memory>
#include <string>

#include "../core/common.hpp"
#include "../kernels/kernels.hpp"

namespace heat3d {

enum StreamId : int { kCompute = 0, kComm = 1, kReduce = 2, kNumStreams = 3 };

enum class CopyKind { H2D, D2H, D2D, H2H };

typedef void* Event;

class Backend {
 public:
  virtual ~Backend() = default;
  virtual const char* name() const = 0;
  virtual bool is_gpu() const = 0;
  virtual int device() const { return -1; }

  virtual void* alloc(std::size_t bytes) = 0;        // device memory (host for CPU)
  virtual void release(void* p) = 0;
  virtual void* alloc_host(std::size_t bytes) = 0;   // pinned host memory
  virtual void release_host(void* p) = 0;
  // Free / total bytes of the memory alloc() draws from (device HBM; host
  // RAM on the CPU backend).  false: unknown.
  virtual bool mem_info(std::size_t* /*free*/, std::size_t* /*total*/) { return false; }
  virtual void copy(void* dst, const void* src, std::size_t bytes, CopyKind k, StreamId s) = 0;
  virtual void memset(void* dst, int v, std::size_t bytes, StreamId s) = 0;

  virtual void* stream(StreamId s) = 0;  // native handle (hipStream_t) or nullptr
  // Keep n CUs free of compute-stream work (HIP: the compute stream is
  // re-created with a CU mask; mask bit i is a CU of XCD i mod 8, so n = 8
  // reserves one CU per XCD) so that comm / boundary / check kernels of the
  // overlapped schedule start at once instead of waiting for a retiring
  // workgroup of the interior sweep.  Call before any work is enqueued.
  virtual void reserve_cus(int /*n*/) {}
  virtual int reserved_cus() const { return 0; }
  // Bracket work that a caller enqueues itself on stream s (RCCL calls):
  // op_begin returns the native stream to enqueue on — the real stream, or,
  // while a graph is being recorded, a private stream capturing this one
  // operation — and op_end closes it.
  virtual void* op_begin(StreamId s) { return stream(s); }
  virtual void op_end(StreamId /*s*/) {}
  virtual Event event_create() = 0;
  virtual void event_destroy(Event e) = 0;
  virtual void record(Event e, StreamId s) = 0;
  virtual void wait(StreamId s, Event e) = 0;
  virtual bool query(Event e) = 0;
  virtual void event_sync(Event e) = 0;
  virtual float elapsed_ms(Event a, Event b) = 0;
  virtual void sync(StreamId s) = 0;
  virtual void sync_all() = 0;
  // sync_all bounded by a host-side deadline: false if some stream is still
  // busy after `seconds` (its work keeps running)
  virtual bool sync_all_for(double /*seconds*/) {
    sync_all();
    return true;
  }

  // Graph recording: between begin_capture and end_capture nothing runs.
  //   * one graph (per_stream = false): every operation on any stream becomes
  //     a node of one graph, and event record / wait pairs become its
  //     dependency edges (HipBackend builds the graph explicitly, see
  //     hip_backend.cpp).  The executable graph is launched on the compute
  //     stream (a DAG with parallel branches: the HIP runtime replays them
  //     on streams of its own, without the CU mask and priorities).
  //   * one linear graph per stream (per_stream = true): each stream's
  //     operations in issue order, launched on that stream (CU mask and
  //     priority kept); a wait on an event another stream recorded inside
  //     the recording becomes a device-side wait on a signal slot, set by
  //     the recording stream (kernels graph_signal / graph_wait).  A wait
  //     that outlasts fault_state->wait_ticks (read when it runs) marks
  //     `fault_state` (fault = 2, done = 1).
  // launch_graph joins every stream into the compute stream afterwards.
  virtual bool supports_graphs() const { return false; }
  virtual void begin_capture(bool /*per_stream*/ = false, DeviceState* /*fault_state*/ = nullptr,
                             int /*max_signals*/ = 0) {}
  virtual void* end_capture() { return nullptr; }  // returns executable graph
  virtual void launch_graph(void* /*exec*/) {}
  virtual void destroy_graph(void* /*exec*/) {}

  // kernels (see kernels.hpp)
  virtual void init_field(DType t, const InitParams& p, StreamId s) = 0;
  virtual void stencil(DType t, const StencilParams& p, const KernelSpec& k, StreamId s) = 0;
  // K = k.K steps T^n -> T^{n+K} in one temporally blocked sweep (residual
  // slots p.slot .. p.slot + K - 1)
  virtual void sweep(DType t, const StencilParams& p, const KernelSpec& k, StreamId s) = 0;
  virtual void pack_box(DType t, const void* f, const Layout& L, const Box& b, void* buf,
                        StreamId s) = 0;
  virtual void unpack_box(DType t, void* f, const Layout& L, const Box& b, const void* buf,
                          StreamId s) = 0;
  virtual void copy_box(DType t, const void* src, const Layout& Ls, const Box& bs, void* dst,
                        const Layout& Ld, const Box& bd, StreamId s) = 0;
  // convergence checks of `count` consecutive iterations, residual slots
  // slot .. slot + count - 1, in order (one launch on the GPU)
  // last_only: every slot but the last only advances the count (Solver::residual_last_ok)
  virtual void check_convergence(DeviceState* st, int slot, StreamId s, int count = 1, bool last_only = false) = 0;
  virtual void error_accumulate(DType t, const void* f, const Layout& L, const Box& box,
                                const int64_t gstart[3], double hy, DeviceState* st,
                                StreamId s) = 0;
  virtual void poke(DType t, void* f, const Layout& L, int64_t i, int64_t j, int64_t k,
                    double value, StreamId s) = 0;
  // order-independent checksum of a box into *out (device memory on HIP)
  virtual void box_bitsum(DType t, const void* f, const Layout& L, const Box& b,
                          unsigned long long* out, StreamId s) = 0;
  // diagnostic: occupy stream s for `us` microseconds with `blocks` spinning
  // workgroups (emulated collective latency / transfer time); no-op on the CPU
  virtual void delay(double /*us*/, StreamId /*s*/, int /*blocks*/ = 1) {}
  // the phantom transport's delay / copy kernels in RCCL's device-kernel
  // footprint (GPU backends)
  virtual void set_comm_footprint(bool /*rccl_like*/) {}
  // device clock stamp into *slot (8 bytes of device memory), and a delay
  // that ends `us` after the stamp (emulated transfers overlapping copies)
  virtual void stamp(void* /*slot*/, StreamId /*s*/) {}
  virtual void delay_since(const void* /*slot*/, double us, StreamId s, int blocks = 1) { delay(us, s, blocks); }
  // transfers paced at a wire rate (phantom transport): plain copies by default
  virtual void paced_copy(const std::vector<hip::PacedCopy>& xs, int /*per*/, StreamId s) {
    for (const auto& x : xs) copy(x.dst, x.src, (std::size_t)x.bytes, CopyKind::D2D, s);
  }
  // tracing ranges (roctx on HIP)
  virtual void range_push(const char* /*name*/) {}
  virtual void range_pop() {}
};

// Factory helpers.  make_hip_backend throws if no GPU is visible.
std::unique_ptr<Backend> make_cpu_backend(int threads);
std::unique_ptr<Backend> make_hip_backend(int device);
int hip_device_count();  // 0 when no GPU / no driver
// The HIP runtime this process is bound to: hipRuntimeGetVersion (e.g.
// 70226015 = 7.2.26015) and the file libamdhip64.so.7 resolved to.  PyTorch
// bundles a HIP 7.0 runtime under the same soname: a process that imports
// torch before the solver runs on torch's copy (bench.py and smoke() do not).
struct HipRuntimeInfo {
  int runtime_version = 0, driver_version = 0;
  std::string library;
  std::string sync_wait;  // the device's host-wait scheduling (spin / yield / blocking / auto)
};
HipRuntimeInfo hip_runtime_info();
// block until every stream of `device` is idle (hipDeviceSynchronize)
void hip_device_synchronize(int device);

}  // namespace heat3d
