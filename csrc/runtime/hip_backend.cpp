// heat3d-mi355x — HIP backend: one device, three prioritised streams,
// event pool, pinned host staging and hipGraph capture.
//
// The device is bound once (the reference called cudaSetDevice(rank % n) in
// every iteration, heat3D.cu:650-654).  The comm and reduce streams get the
// highest priority so that halo pack / boundary / convergence kernels are
// dispatched ahead of the long-running interior sweep they overlap with.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

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
    int least = 0, greatest = 0;
    HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_CHECK(hipStreamCreateWithPriority(&streams_[kCompute], hipStreamNonBlocking, least));
    HIP_CHECK(hipStreamCreateWithPriority(&streams_[kComm], hipStreamNonBlocking, greatest));
    HIP_CHECK(hipStreamCreateWithPriority(&streams_[kReduce], hipStreamNonBlocking, greatest));
  }
  ~HipBackend() override {
    (void)hipSetDevice(dev_);
    if (err_scratch_) (void)hipFree(err_scratch_);
    for (auto& s : streams_)
      if (s) (void)hipStreamDestroy(s);
  }
  const char* name() const override { return "hip"; }
  bool is_gpu() const override { return true; }
  int device() const override { return dev_; }

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
    HIP_CHECK(hipMemcpyAsync(dst, src, bytes, kind, streams_[s]));
  }
  void memset(void* dst, int v, std::size_t bytes, StreamId s) override {
    HIP_CHECK(hipMemsetAsync(dst, v, bytes, streams_[s]));
  }

  void* stream(StreamId s) override { return streams_[s]; }
  Event event_create() override {
    hipEvent_t e;
    HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDefault));
    return e;
  }
  void event_destroy(Event e) override { (void)hipEventDestroy(static_cast<hipEvent_t>(e)); }
  void record(Event e, StreamId s) override {
    HIP_CHECK(hipEventRecord(static_cast<hipEvent_t>(e), streams_[s]));
  }
  void wait(StreamId s, Event e) override {
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

  bool supports_graphs() const override { return true; }
  void begin_capture() override {
    HIP_CHECK(hipStreamBeginCapture(streams_[kCompute], hipStreamCaptureModeRelaxed));
  }
  void* end_capture() override {
    hipGraph_t g = nullptr;
    HIP_CHECK(hipStreamEndCapture(streams_[kCompute], &g));
    hipGraphExec_t ex = nullptr;
    HIP_CHECK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    HIP_CHECK(hipGraphDestroy(g));
    return ex;
  }
  void launch_graph(void* ex) override {
    HIP_CHECK(hipGraphLaunch(static_cast<hipGraphExec_t>(ex), streams_[kCompute]));
  }
  void destroy_graph(void* ex) override {
    if (ex) (void)hipGraphExecDestroy(static_cast<hipGraphExec_t>(ex));
  }

  void init_field(DType t, const InitParams& p, StreamId s) override {
    hip::init_field(t, p, streams_[s]);
  }
  void stencil(DType t, const StencilParams& p, const KernelSpec& k, StreamId s) override {
    hip::stencil(t, p, k, streams_[s]);
  }
  void stencil2(DType t, const StencilParams& p, const KernelSpec& k, StreamId s) override {
    hip::sweep(t, p, k, streams_[s]);
  }
  void pack_box(DType t, const void* f, const Layout& L, const Box& b, void* buf, StreamId s) override {
    hip::pack_box(t, f, L, b, buf, streams_[s]);
  }
  void unpack_box(DType t, void* f, const Layout& L, const Box& b, const void* buf, StreamId s) override {
    hip::unpack_box(t, f, L, b, buf, streams_[s]);
  }
  void copy_box(DType t, const void* src, const Layout& Ls, const Box& bs, void* dst,
                const Layout& Ld, const Box& bd, StreamId s) override {
    hip::copy_box(t, src, Ls, bs, dst, Ld, bd, streams_[s]);
  }
  void delay(double us, StreamId s, int blocks) override { hip::delay(us, streams_[s], blocks); }
  void check_convergence(DeviceState* st, int slot, StreamId s, int count) override {
    hip::check_convergence(st, slot, streams_[s], count);
  }
  void error_accumulate(DType t, const void* f, const Layout& L, const Box& box,
                        const int64_t gstart[3], double hy, DeviceState* st, StreamId s) override {
    if (!err_scratch_) err_scratch_ = static_cast<double*>(alloc(sizeof(double) * hip::error_scratch_elems()));
    hip::error_accumulate(t, f, L, box, gstart, hy, err_scratch_, st, streams_[s]);
  }
  void poke(DType t, void* f, const Layout& L, int64_t i, int64_t j, int64_t k, double value,
            StreamId s) override {
    hip::poke(t, f, L, i, j, k, value, streams_[s]);
  }
  void box_bitsum(DType t, const void* f, const Layout& L, const Box& b, unsigned long long* out,
                  StreamId s) override {
    hip::box_bitsum(t, f, L, b, out, streams_[s]);
  }
  void range_push(const char* n) override {
    if (roctx_.push) roctx_.push(n);
  }
  void range_pop() override {
    if (roctx_.pop) roctx_.pop();
  }

 private:
  int dev_;
  hipStream_t streams_[kNumStreams] = {nullptr, nullptr, nullptr};
  double* err_scratch_ = nullptr;
  Roctx roctx_;
};

}  // namespace

std::unique_ptr<Backend> make_hip_backend(int device) {
  return std::unique_ptr<Backend>(new HipBackend(device));
}

}  // namespace heat3d
