// heat3d-mi355x — HIP backend: one device, three prioritised streams,
// event pool, pinned host staging and explicitly built hipGraphs.
//
// Graphs.  Stream capture of the solver's three-stream schedule (compute,
// comm, reduce, forking and joining through events) overflows the host stack
// inside hipStreamEndCapture of the HIP runtime PyTorch ships (a recursion
// through the streams' parallel-capture lists; backtrace in
// docs/ARCHITECTURE.md, minimal single-op patterns in
// tools/graph_capture_repro.hip do not trigger it).  So the graph is built
// explicitly: while recording, each operation is captured alone on a private
// per-stream capture stream straight into the graph being built
// (hipStreamBeginCaptureToGraph) behind that stream's dependency frontier; an
// event record remembers the recording stream's frontier and a wait merges it
// into the waiting stream's.  The resulting DAG has exactly the dependencies
// of the eager schedule.  (Round 2's alternatives — every operation a
// child-graph node, or one-kernel captures re-added as kernel nodes — replayed
// without overlap or broke ordering on HIP 7.2 and were removed.)
//
// That DAG suits single-stream schedules.  A DAG with parallel branches is
// replayed by the HIP runtime on streams of its own, without the compute
// stream's CU mask and the comm stream's priority: the overlapped multi-rank
// schedule ran 1.7x slower as one (profiles/rank_proxy_r04.md).  So those
// schedules record one LINEAR graph per stream, each launched on its own
// stream — a linear graph launched on the CU-masked stream stays on its 248
// CUs (tools/probes/graph_streams_probe.hip) — and their cross-stream
// dependencies become device-side signal / wait kernels on slots reset
// before every launch.  (Captured hipStreamWaitValue64 nodes did not hold
// their wait on HIP 7.2: the same probe.)  An event wait resolves on the
// device when the work runs, not when it is enqueued, so each stream's graph
// can be launched whole although the streams depend on each other within it.
//
// The device is bound once (the reference called cudaSetDevice(rank % n) in
// every iteration, heat3D.cu:650-654).  The comm and reduce streams get the
// highest priority so that halo pack / boundary / convergence kernels are
// dispatched ahead of the long-running interior sweep they overlap with.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <thread>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "backend.hpp"

namespace heat3d {

#define HIP_CHECK(expr)                                                                 \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) HEAT3D_THROW("HIP error '" << hipGetErrorString(_e) << "' at " #expr); \
  } while (0)

int hip_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

HipRuntimeInfo hip_runtime_info() {
  HipRuntimeInfo r;
  if (hipRuntimeGetVersion(&r.runtime_version) != hipSuccess) (void)hipGetLastError();
  if (hipDriverGetVersion(&r.driver_version) != hipSuccess) (void)hipGetLastError();
  unsigned flags = 0;
  if (hip_device_count() > 0 && hipGetDeviceFlags(&flags) == hipSuccess) {
    const unsigned s = flags & hipDeviceScheduleMask;
    r.sync_wait = s == hipDeviceScheduleSpin ? "spin" : s == hipDeviceScheduleYield ? "yield"
                  : s == hipDeviceScheduleBlockingSync ? "blocking" : "auto";
  } else {
    (void)hipGetLastError();
  }
  Dl_info di;
  if (dladdr(reinterpret_cast<void*>(&hipRuntimeGetVersion), &di) && di.dli_fname) {
    char buf[4096];
    r.library = realpath(di.dli_fname, buf) ? std::string(buf) : std::string(di.dli_fname);
  }
  return r;
}

void hip_device_synchronize(int device) {
  HIP_CHECK(hipSetDevice(device));
  HIP_CHECK(hipDeviceSynchronize());
}

namespace {

struct Roctx {
  typedef int (*push_t)(const char*);
  typedef int (*pop_t)();
  push_t push = nullptr;
  pop_t pop = nullptr;
  Roctx() {
    const char* e = std::getenv("HEAT3D_ROCTX");
    if (!e || !*e || e[0] == '0') return;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    push = reinterpret_cast<push_t>(dlsym(h, "roctxRangePushA"));
    pop = reinterpret_cast<pop_t>(dlsym(h, "roctxRangePop"));
  }
};

class HipBackend final : public Backend {
 public:
  explicit HipBackend(int device) : dev_(device) {
    int n = hip_device_count();
    HEAT3D_CHECK(n > 0, "no HIP device visible");
    HEAT3D_CHECK(device >= 0 && device < n, "device " << device << " out of range (" << n << " visible)");
    HIP_CHECK(hipSetDevice(dev_));
    // How the host waits for the device (synchronize, event sync): spin, the
    // lowest wake-up latency, whatever HIP's auto heuristic would pick for
    // the host's core count (on the 1-GPU boxes it picks spin too:
    // tools/probes/sync_wake_probe.hip).  HEAT3D_SYNC_WAIT=auto|yield|spin.
    {
      const char* e = std::getenv("HEAT3D_SYNC_WAIT");
      const std::string m = e && *e ? e : "spin";
      const unsigned f = m == "auto" ? hipDeviceScheduleAuto : m == "yield" ? hipDeviceScheduleYield : hipDeviceScheduleSpin;
      if (hipSetDeviceFlags(f) != hipSuccess) (void)hipGetLastError();  // already active: keep the process's
    }
    int least = 0, greatest = 0;
    HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_CHECK(hipStreamCreateWithPriority(&streams_[kCompute], hipStreamNonBlocking, least));
    HIP_CHECK(hipStreamCreateWithPriority(&streams_[kComm], hipStreamNonBlocking, greatest));
    HIP_CHECK(hipStreamCreateWithPriority(&streams_[kReduce], hipStreamNonBlocking, greatest));
    prio_[kCompute] = least;
    prio_[kComm] = prio_[kReduce] = greatest;
    // capture streams are created while a graph is recorded and destroyed
    // after it: a process holds GPU_MAX_HW_QUEUES (4) hardware queues, and
    // idle extra streams would make the comm stream share one with the
    // interior sweep (2-rank RCCL on one GPU: 4.5 s -> 113 s)
  }
  hipStream_t capture_stream(StreamId s) {
    if (!caps_[s]) HIP_CHECK(hipStreamCreateWithPriority(&caps_[s], hipStreamNonBlocking, prio_[s]));
    return caps_[s];
  }
  void drop_capture_streams() {
    for (auto& c : caps_)
      if (c) {
        (void)hipStreamDestroy(c);
        c = nullptr;
      }
  }
  ~HipBackend() override {
    (void)hipSetDevice(dev_);
    if (rec_) (void)hipGraphDestroy(rec_);
    for (auto& g : recs_)
      if (g) (void)hipGraphDestroy(g);
    if (sig_) (void)hipFree(sig_);
    if (fork_ev_) (void)hipEventDestroy(fork_ev_);
    for (auto& e : join_ev_)
      if (e) (void)hipEventDestroy(e);
    for (auto& s : caps_)
      if (s) (void)hipStreamDestroy(s);
    if (err_scratch_) (void)hipFree(err_scratch_);
    for (auto& s : streams_)
      if (s) (void)hipStreamDestroy(s);
  }
  const char* name() const override { return "hip"; }
  bool is_gpu() const override { return true; }
  int device() const override { return dev_; }

  bool mem_info(std::size_t* free, std::size_t* total) override {
    HIP_CHECK(hipSetDevice(dev_));
    return hipMemGetInfo(free, total) == hipSuccess;
  }
  void* alloc(std::size_t bytes) override {
    void* p = nullptr;
    HIP_CHECK(hipMalloc(&p, bytes ? bytes : 256));
    return p;
  }
  void release(void* p) override {
    if (p) (void)hipFree(p);
  }
  void* alloc_host(std::size_t bytes) override {
    void* p = nullptr;
    HIP_CHECK(hipHostMalloc(&p, bytes ? bytes : 256, hipHostMallocDefault));
    return p;
  }
  void release_host(void* p) override {
    if (p) (void)hipHostFree(p);
  }
  void copy(void* dst, const void* src, std::size_t bytes, CopyKind k, StreamId s) override {
    if (!bytes) return;
    hipMemcpyKind kind = hipMemcpyDefault;
    switch (k) {
      case CopyKind::H2D: kind = hipMemcpyHostToDevice; break;
      case CopyKind::D2H: kind = hipMemcpyDeviceToHost; break;
      case CopyKind::D2D: kind = hipMemcpyDeviceToDevice; break;
      case CopyKind::H2H: kind = hipMemcpyHostToHost; break;
    }
    op(s, [&](hipStream_t st) { HIP_CHECK(hipMemcpyAsync(dst, src, bytes, kind, st)); });
  }
  void memset(void* dst, int v, std::size_t bytes, StreamId s) override {
    op(s, [&](hipStream_t st) { HIP_CHECK(hipMemsetAsync(dst, v, bytes, st)); });
  }

  void* stream(StreamId s) override { return streams_[s]; }
  void reserve_cus(int n) override {
    if (n <= 0 || n == reserved_) return;
    int cus = 0;
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_));
    HEAT3D_CHECK(n < cus, "cannot reserve " << n << " of " << cus << " CUs");
    const int words = (cus + 31) / 32;
    std::vector<uint32_t> mask(words, 0u);
    for (int i = 0; i < cus - n; ++i) mask[i / 32] |= 1u << (i % 32);  // clear the top n bits
    // Mask bit i is a CU of XCD i mod 8 (measured: tests/test_gpu_placement.py),
    // so the top n = 8 bits keep one CU per XCD free.  HIP offers no flags
    // or priority for a CU-masked stream: it is a blocking stream of normal
    // priority (the stream it replaces was non-blocking, lowest priority).
    // The comm / reduce streams keep their higher priority, and no solver
    // work is issued to the legacy null stream, so neither difference
    // orders anything the solver issues.
    hipStream_t s = nullptr;
    HIP_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask.data()));
    HIP_CHECK(hipStreamSynchronize(streams_[kCompute]));
    HIP_CHECK(hipStreamDestroy(streams_[kCompute]));
    streams_[kCompute] = s;
    reserved_ = n;
  }
  int reserved_cus() const override { return reserved_; }
  void* op_begin(StreamId s) override {
    if (!recording_) return streams_[s];
    if (split_) flush_sync(s);
    return cap_begin(s);
  }
  // open a capture of one operation on stream s straight into the graph
  // being recorded (s's own graph in per-stream mode), behind s's frontier
  void* cap_begin(StreamId s) {
    HEAT3D_CHECK(!in_op_, "graph recording: nested operation");
    in_op_ = true;
    op_s_ = s;
    // capture straight into the recorded graph, behind the stream's frontier
    auto& t = tail_[s];
    HIP_CHECK(hipStreamBeginCaptureToGraph(capture_stream(s), split_ ? recs_[s] : rec_, t.empty() ? nullptr : t.data(),
                                           nullptr, t.size(), hipStreamCaptureModeThreadLocal));
    return caps_[s];
  }
  void op_end(StreamId s) override {
    if (!recording_) return;
    HEAT3D_CHECK(in_op_ && op_s_ == s, "graph recording: unbalanced operation");
    in_op_ = false;
    hipGraph_t g = nullptr;
    // the new frontier: the capture's dependency set after the operation
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const hipGraphNode_t* deps = nullptr;
    std::size_t nd = 0;
    hipError_t e = hipStreamGetCaptureInfo_v2(caps_[s], &cs, nullptr, nullptr, &deps, &nd);
    std::vector<hipGraphNode_t> front(deps, deps + (e == hipSuccess ? nd : 0));
    hipError_t e2 = hipStreamEndCapture(caps_[s], &g);
    HIP_CHECK(e);
    HIP_CHECK(e2);
    if (!front.empty()) tail_[s] = std::move(front);
  }
  Event event_create() override {
    hipEvent_t e;
    HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDefault));
    return e;
  }
  void event_destroy(Event e) override { (void)hipEventDestroy(static_cast<hipEvent_t>(e)); }
  void record(Event e, StreamId s) override {
    if (recording_ && split_) {
      // a signal behind everything issued on s so far: records with no
      // operation between them share one slot (one signal kernel)
      auto& q = pend_[s];
      int slot;
      if (!q.empty() && q.back().signal) {
        slot = q.back().slots[0];
      } else {
        HEAT3D_CHECK(sig_n_ < sig_cap_, "per-stream graph: signal slots exhausted (" << sig_cap_ << ")");
        slot = sig_n_++;
        q.push_back({true, {slot}});
        ++sig_ord_[s];
      }
      evsig_[e] = {slot, s, sig_ord_[s]};
      return;
    }
    if (recording_) {
      evn_[e] = tail_[s];  // the recording stream's frontier
      return;
    }
    HIP_CHECK(hipEventRecord(static_cast<hipEvent_t>(e), streams_[s]));
  }
  void wait(StreamId s, Event e) override {
    if (recording_ && split_) {
      // recorded before the recording started: complete when the graphs run
      // (launched behind a join of every stream); same stream: stream order;
      // an earlier wait on a later signal of the same stream covers it
      auto it = evsig_.find(e);
      if (it == evsig_.end() || it->second.s == s) return;
      const Sig g = it->second;
      int& w = waited_[s][g.s];
      if (w >= g.ord) return;
      w = g.ord;
      auto& q = pend_[s];
      if (!q.empty() && !q.back().signal && q.back().slots.size() < 4) q.back().slots.push_back(g.slot);
      else q.push_back({false, {g.slot}});
      return;
    }
    if (recording_) {
      // an event recorded before the recording started is already complete
      // when the graph (launched behind a join of every stream) runs
      auto it = evn_.find(e);
      if (it == evn_.end()) return;
      auto& t = tail_[s];
      for (hipGraphNode_t n : it->second)
        if (std::find(t.begin(), t.end(), n) == t.end()) t.push_back(n);
      return;
    }
    HIP_CHECK(hipStreamWaitEvent(streams_[s], static_cast<hipEvent_t>(e), 0));
  }
  bool query(Event e) override {
    hipError_t r = hipEventQuery(static_cast<hipEvent_t>(e));
    if (r == hipSuccess) return true;
    if (r == hipErrorNotReady) return false;
    HIP_CHECK(r);
    return false;
  }
  void event_sync(Event e) override { HIP_CHECK(hipEventSynchronize(static_cast<hipEvent_t>(e))); }
  float elapsed_ms(Event a, Event b) override {
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, static_cast<hipEvent_t>(a), static_cast<hipEvent_t>(b)));
    return ms;
  }
  void sync(StreamId s) override { HIP_CHECK(hipStreamSynchronize(streams_[s])); }
  void sync_all() override {
    for (auto& s : streams_) HIP_CHECK(hipStreamSynchronize(s));
  }
  bool sync_all_for(double seconds) override {
    const auto t0 = std::chrono::steady_clock::now();
    for (auto& s : streams_) {
      for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) HIP_CHECK(e);
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > seconds) return false;
        std::this_thread::sleep_for(std::chrono::microseconds(100));
      }
    }
    return true;
  }

  bool supports_graphs() const override { return true; }
  void begin_capture(bool per_stream, DeviceState* fault_state, int max_signals) override {
    HEAT3D_CHECK(!recording_, "graph recording already active");
    split_ = per_stream;
    if (split_) {
      HEAT3D_CHECK(fault_state, "per-stream graphs need a device state for wait timeouts");
      for (auto& g : recs_) HIP_CHECK(hipGraphCreate(&g, 0));
      sig_cap_ = std::max(16, max_signals);
      HIP_CHECK(hipMalloc(&sig_, sizeof(unsigned) * sig_cap_));
      sig_n_ = 0;
      fault_ = fault_state;
      evsig_.clear();
      for (auto& q : pend_) q.clear();
      for (auto& w : waited_)
        for (int& v : w) v = 0;
      for (int& o : sig_ord_) o = 0;
    } else {
      HIP_CHECK(hipGraphCreate(&rec_, 0));
    }
    for (auto& t : tail_) t.clear();
    evn_.clear();
    in_op_ = false;
    recording_ = true;
  }
  void* end_capture() override {
    HEAT3D_CHECK(recording_, "no graph recording active");
    if (in_op_) abort_op();  // an operation threw while being captured
    std::unique_ptr<GraphSet> gs(new GraphSet);
    gs->per_stream = split_;
    hipError_t err = hipSuccess;
    if (split_) {
      // the signals / waits still pending at the end of each stream
      for (int s = 0; s < kNumStreams; ++s) {
        try {
          flush_sync(static_cast<StreamId>(s));
        } catch (...) {
          if (err == hipSuccess) err = hipErrorUnknown;
        }
      }
    }
    recording_ = false;
    evn_.clear();
    drop_capture_streams();
    if (split_) {
      split_ = false;
      gs->slots = sig_;
      gs->nslots = sig_n_;
      sig_ = nullptr;
      for (int s = 0; s < kNumStreams; ++s) {
        std::size_t n = 0;
        if (err == hipSuccess) err = hipGraphGetNodes(recs_[s], nullptr, &n);
        if (err == hipSuccess && n > 0) err = hipGraphInstantiateWithFlags(&gs->ex[s], recs_[s], 0);
        (void)hipGraphDestroy(recs_[s]);
        recs_[s] = nullptr;
      }
    } else {
      hipGraph_t g = rec_;
      rec_ = nullptr;
      err = hipGraphInstantiateWithFlags(&gs->ex[0], g, hipGraphInstantiateFlagUseNodePriority);
      (void)hipGraphDestroy(g);
    }
    if (err != hipSuccess) {
      destroy_graph(gs.release());
      HIP_CHECK(err);
    }
    // upload now so that the first launch does not pay for it (each on the
    // stream it will be launched on)
    for (int s = 0; s < kNumStreams; ++s)
      if (gs->ex[s]) HIP_CHECK(hipGraphUpload(gs->ex[s], streams_[gs->per_stream ? s : kCompute]));
    return gs.release();
  }
  void launch_graph(void* h) override {
    auto* g = static_cast<GraphSet*>(h);
    if (!g->per_stream) {
      HIP_CHECK(hipGraphLaunch(g->ex[0], streams_[kCompute]));
      return;
    }
    // The solver launches behind a join of every stream into the compute
    // stream: reset the signal slots there, fork, launch each stream's graph
    // on its stream, join back into the compute stream.
    if (!fork_ev_) {
      HIP_CHECK(hipEventCreateWithFlags(&fork_ev_, hipEventDisableTiming));
      for (auto& e : join_ev_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    if (g->nslots) HIP_CHECK(hipMemsetAsync(g->slots, 0, sizeof(unsigned) * g->nslots, streams_[kCompute]));
    HIP_CHECK(hipEventRecord(fork_ev_, streams_[kCompute]));
    for (int s = kComm; s < kNumStreams; ++s)
      if (g->ex[s]) HIP_CHECK(hipStreamWaitEvent(streams_[s], fork_ev_, 0));
    for (int s = 0; s < kNumStreams; ++s)
      if (g->ex[s]) HIP_CHECK(hipGraphLaunch(g->ex[s], streams_[s]));
    for (int s = kComm; s < kNumStreams; ++s)
      if (g->ex[s]) {
        HIP_CHECK(hipEventRecord(join_ev_[s], streams_[s]));
        HIP_CHECK(hipStreamWaitEvent(streams_[kCompute], join_ev_[s], 0));
      }
  }
  void destroy_graph(void* h) override {
    auto* g = static_cast<GraphSet*>(h);
    if (!g) return;
    for (auto& e : g->ex)
      if (e) (void)hipGraphExecDestroy(e);
    if (g->slots) (void)hipFree(g->slots);
    delete g;
  }

  void init_field(DType t, const InitParams& p, StreamId s) override {
    op(s, [&](hipStream_t st) { hip::init_field(t, p, st); });
  }
  void stencil(DType t, const StencilParams& p, const KernelSpec& k, StreamId s) override {
    op(s, [&](hipStream_t st) { hip::stencil(t, p, k, st); });
  }
  void sweep(DType t, const StencilParams& p, const KernelSpec& k, StreamId s) override {
    op(s, [&](hipStream_t st) { hip::sweep(t, p, k, st); });
  }
  void pack_box(DType t, const void* f, const Layout& L, const Box& b, void* buf, StreamId s) override {
    op(s, [&](hipStream_t st) { hip::pack_box(t, f, L, b, buf, st); });
  }
  void unpack_box(DType t, void* f, const Layout& L, const Box& b, const void* buf, StreamId s) override {
    op(s, [&](hipStream_t st) { hip::unpack_box(t, f, L, b, buf, st); });
  }
  void copy_box(DType t, const void* src, const Layout& Ls, const Box& bs, void* dst,
                const Layout& Ld, const Box& bd, StreamId s) override {
    op(s, [&](hipStream_t st) { hip::copy_box(t, src, Ls, bs, dst, Ld, bd, st); });
  }
  void delay(double us, StreamId s, int blocks) override {
    op(s, [&](hipStream_t st) { hip::delay(us, st, blocks, fat_comm_); });
  }
  void set_comm_footprint(bool rccl_like) override { fat_comm_ = rccl_like; }
  void stamp(void* slot, StreamId s) override { op(s, [&](hipStream_t st) { hip::stamp(slot, st); }); }
  void paced_copy(const std::vector<hip::PacedCopy>& xs, int per, StreamId s) override {
    if (xs.empty()) return;
    op(s, [&](hipStream_t st) { hip::paced_copy(xs.data(), (int)xs.size(), per, st, fat_comm_); });
  }
  void delay_since(const void* slot, double us, StreamId s, int blocks) override {
    op(s, [&](hipStream_t st) { hip::delay_since(slot, us, st, blocks, fat_comm_); });
  }
  void check_convergence(DeviceState* st, int slot, StreamId s, int count, bool last_only) override {
    op(s, [&](hipStream_t q) { hip::check_convergence(st, slot, q, count, last_only); });
  }
  void error_accumulate(DType t, const void* f, const Layout& L, const Box& box,
                        const int64_t gstart[3], double hy, DeviceState* st, StreamId s) override {
    if (!err_scratch_) err_scratch_ = static_cast<double*>(alloc(sizeof(double) * hip::error_scratch_elems()));
    op(s, [&](hipStream_t q) { hip::error_accumulate(t, f, L, box, gstart, hy, err_scratch_, st, q); });
  }
  void poke(DType t, void* f, const Layout& L, int64_t i, int64_t j, int64_t k, double value,
            StreamId s) override {
    op(s, [&](hipStream_t st) { hip::poke(t, f, L, i, j, k, value, st); });
  }
  void box_bitsum(DType t, const void* f, const Layout& L, const Box& b, unsigned long long* out,
                  StreamId s) override {
    op(s, [&](hipStream_t st) { hip::box_bitsum(t, f, L, b, out, st); });
  }
  void range_push(const char* n) override {
    if (roctx_.push) roctx_.push(n);
  }
  void range_pop() override {
    if (roctx_.pop) roctx_.pop();
  }

 private:
  // per-stream recording: the signal / wait kernels pending on each stream,
  // emitted in order before its next operation (consecutive waits merged)
  struct SyncItem {
    bool signal;
    std::vector<int> slots;
  };
  struct Sig {
    int slot;
    StreamId s;
    int ord;  // the how-manieth signal of stream s
  };
  void flush_sync(StreamId s) {
    auto& q = pend_[s];
    if (q.empty()) return;
    std::vector<SyncItem> items;
    items.swap(q);
    for (const SyncItem& it : items) {
      hipStream_t st = static_cast<hipStream_t>(cap_begin(s));
      try {
        if (it.signal) {
          hip::graph_signal(sig_ + it.slots[0], st);
        } else {
          const unsigned* p[4];
          for (std::size_t i = 0; i < it.slots.size(); ++i) p[i] = sig_ + it.slots[i];
          hip::graph_wait(p, (int)it.slots.size(), fault_, st);
        }
      } catch (...) {
        abort_op();
        throw;
      }
      op_end(s);
    }
  }
  struct GraphSet {
    bool per_stream = false;
    hipGraphExec_t ex[kNumStreams] = {nullptr, nullptr, nullptr};
    unsigned* slots = nullptr;  // per-stream graphs: signal slots
    int nslots = 0;
  };

  // run one operation: directly on the stream, or recorded as a graph node
  template <typename F>
  void op(StreamId s, F&& f) {
    hipStream_t st = static_cast<hipStream_t>(op_begin(s));
    if (!recording_) {
      f(st);
      return;
    }
    try {
      f(st);
    } catch (...) {
      abort_op();
      throw;
    }
    op_end(s);
  }

  void abort_op() {
    in_op_ = false;
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(caps_[op_s_], &g);  // g is rec_, owned by the recorder
    (void)hipGetLastError();
  }

  int dev_;
  int prio_[kNumStreams] = {0, 0, 0};
  int reserved_ = 0;
  bool fat_comm_ = false;  // phantom delay / copy kernels in RCCL's footprint
  hipStream_t streams_[kNumStreams] = {nullptr, nullptr, nullptr};
  // graph recording state
  bool recording_ = false, in_op_ = false;
  StreamId op_s_ = kCompute;
  hipGraph_t rec_ = nullptr;
  std::vector<hipGraphNode_t> tail_[kNumStreams];    // dependency frontier per stream
  hipStream_t caps_[kNumStreams] = {nullptr, nullptr, nullptr};
  std::unordered_map<Event, std::vector<hipGraphNode_t>> evn_;  // event -> frontier at record
  // per-stream recording
  bool split_ = false;
  hipGraph_t recs_[kNumStreams] = {nullptr, nullptr, nullptr};
  unsigned* sig_ = nullptr;
  int sig_cap_ = 0, sig_n_ = 0;
  DeviceState* fault_ = nullptr;
  std::unordered_map<Event, Sig> evsig_;
  std::vector<SyncItem> pend_[kNumStreams];
  int waited_[kNumStreams][kNumStreams] = {};  // [waiter][signaller]: highest signal waited for
  int sig_ord_[kNumStreams] = {};
  hipEvent_t fork_ev_ = nullptr, join_ev_[kNumStreams] = {nullptr, nullptr, nullptr};
  double* err_scratch_ = nullptr;
  Roctx roctx_;
};

}  // namespace

std::unique_ptr<Backend> make_hip_backend(int device) {
  return std::unique_ptr<Backend>(new HipBackend(device));
}

}  // namespace heat3d
