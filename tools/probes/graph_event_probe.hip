// Probe: can CP-level event nodes replace the device-side spin waits of the
// per-stream graphs (hip_backend.cpp)?  Event record / wait nodes are
// captured with hipEventRecordWithFlags(..., hipEventRecordExternal) and
// hipStreamWaitEvent(..., hipEventWaitExternal) into two linear graphs, each
// launched whole on its own stream, as the solver launches its per-stream
// graphs.  Ticket kernels take numbers from one counter to witness the order.
//
//   hipcc --offload-arch=gfx950 -O2 tools/probes/graph_event_probe.hip -o /tmp/gep && /tmp/gep
//
// 1. one direction, producer graph launched first: A = [spin, ticket a,
//    record e]; B = [wait e, ticket b].  Expected a < b.
// 2. one direction, consumer graph launched first (B, then A).
// 3. both directions, as the overlapped schedule needs (the interior waits
//    for the last boundary slabs, the halo for the interior's buffer):
//    A = [ticket a0, record e1, wait e2, ticket a1];
//    B = [wait e1, spin, ticket b0, record e2].  Expected a0 < b0 < a1.
// Observed on HIP 7.2.26015 (profiles/r06/graph_event_probe.log): case 1
// ordered 5 of 5, case 2 unordered 5 of 5 (the wait node binds the event's
// state when its graph is launched), case 3 aborts inside the runtime
// (std::bad_alloc while capturing the second graph; an earlier build without
// the pre-recorded events died with SIGSEGV there).  So event nodes cannot
// replace the per-stream graphs' device-side waits.
// Every kernel ends on its own (bounded spins); nothing waits on the device
// for another kernel, so a dependency that does not hold shows as a wrong
// order, never as a hang.  Host-side waits give up after 5 s.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::printf("FAIL %s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);             \
      return 1;                                                                                \
    }                                                                                          \
  } while (0)

__global__ void spin_kernel(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

__global__ void ticket_kernel(unsigned* counter, unsigned* slot) {
  if (threadIdx.x == 0) *slot = atomicAdd(counter, 1u);
}

static bool wait_stream(hipStream_t s, double sec) {
  const auto t0 = std::chrono::steady_clock::now();
  while (hipStreamQuery(s) == hipErrorNotReady) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > sec) return false;
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  return true;
}

struct Ctx {
  hipStream_t cap, s1, s2;
  unsigned *tick, *slots;
};

// record / wait helpers inside a capture; report the API result once
static hipError_t rec(hipEvent_t e, hipStream_t s) { return hipEventRecordWithFlags(e, s, hipEventRecordExternal); }
static hipError_t wt(hipStream_t s, hipEvent_t e) { return hipStreamWaitEvent(s, e, hipEventWaitExternal); }

static int run_case(Ctx& c, int which, bool consumer_first) {
  hipEvent_t e1, e2;
  CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
  // both events recorded (complete) before the captures: the first probe
  // build, whose case 3 captured a wait on a never-recorded event, crashed
  // the HIP 7.2 runtime (SIGSEGV) in that capture
  CK(hipEventRecord(e1, c.s1));
  CK(hipEventRecord(e2, c.s1));
  CK(hipStreamSynchronize(c.s1));
  hipGraph_t ga, gb, tmp;
  CK(hipGraphCreate(&ga, 0));
  CK(hipGraphCreate(&gb, 0));
  const unsigned long long spin = 100000;  // 1 ms at 100 MHz
  hipError_t r1 = hipSuccess, r2 = hipSuccess, w1 = hipSuccess, w2 = hipSuccess;
  // graph A
  CK(hipStreamBeginCaptureToGraph(c.cap, ga, nullptr, nullptr, 0, hipStreamCaptureModeThreadLocal));
  if (which == 1) {
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, c.cap, spin);
    hipLaunchKernelGGL(ticket_kernel, dim3(1), dim3(64), 0, c.cap, c.tick, c.slots + 0);
    r1 = rec(e1, c.cap);
  } else {
    hipLaunchKernelGGL(ticket_kernel, dim3(1), dim3(64), 0, c.cap, c.tick, c.slots + 0);
    r1 = rec(e1, c.cap);
    w2 = wt(c.cap, e2);
    hipLaunchKernelGGL(ticket_kernel, dim3(1), dim3(64), 0, c.cap, c.tick, c.slots + 1);
  }
  hipError_t ea = hipStreamEndCapture(c.cap, &tmp);
  // graph B
  CK(hipStreamBeginCaptureToGraph(c.cap, gb, nullptr, nullptr, 0, hipStreamCaptureModeThreadLocal));
  w1 = wt(c.cap, e1);
  if (which == 1) {
    hipLaunchKernelGGL(ticket_kernel, dim3(1), dim3(64), 0, c.cap, c.tick, c.slots + 2);
  } else {
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, c.cap, spin);
    hipLaunchKernelGGL(ticket_kernel, dim3(1), dim3(64), 0, c.cap, c.tick, c.slots + 2);
    r2 = rec(e2, c.cap);
  }
  hipError_t eb = hipStreamEndCapture(c.cap, &tmp);
  std::printf("case %d%s: capture A %s (record %s, wait %s), B %s (wait %s, record %s)\n", which,
              consumer_first ? " consumer-first" : "", hipGetErrorString(ea), hipGetErrorString(r1),
              hipGetErrorString(w2), hipGetErrorString(eb), hipGetErrorString(w1), hipGetErrorString(r2));
  if (ea || eb || r1 || r2 || w1 || w2) {
    (void)hipGetLastError();
    return 0;
  }
  size_t na = 0, nb = 0;
  CK(hipGraphGetNodes(ga, nullptr, &na));
  CK(hipGraphGetNodes(gb, nullptr, &nb));
  hipGraphExec_t xa, xb;
  CK(hipGraphInstantiateWithFlags(&xa, ga, 0));
  CK(hipGraphInstantiateWithFlags(&xb, gb, 0));
  int good = 0;
  const int reps = 5;
  for (int rep = 0; rep < reps; ++rep) {
    CK(hipMemsetAsync(c.tick, 0, 4, c.s1));
    CK(hipMemsetAsync(c.slots, 0xff, 16, c.s1));
    CK(hipStreamSynchronize(c.s1));
    if (consumer_first) {
      CK(hipGraphLaunch(xb, c.s2));
      CK(hipGraphLaunch(xa, c.s1));
    } else {
      CK(hipGraphLaunch(xa, c.s1));
      CK(hipGraphLaunch(xb, c.s2));
    }
    if (!wait_stream(c.s1, 5.0) || !wait_stream(c.s2, 5.0)) {
      std::printf("  rep %d: host wait timed out\n", rep);
      return 2;
    }
    unsigned h[3];
    CK(hipMemcpy(h, c.slots, sizeof(h), hipMemcpyDeviceToHost));
    bool ok;
    if (which == 1) ok = h[0] < h[2];
    else ok = h[0] < h[2] && h[2] < h[1];
    good += ok;
    std::printf("  rep %d: tickets a0=%u a1=%d b=%u -> %s\n", rep, h[0], which == 1 ? -1 : (int)h[1], h[2],
                ok ? "ordered" : "WRONG ORDER");
  }
  std::printf("case %d%s: nodes A %zu B %zu, %d of %d ordered\n", which, consumer_first ? " consumer-first" : "",
              na, nb, good, reps);
  CK(hipGraphExecDestroy(xa));
  CK(hipGraphExecDestroy(xb));
  CK(hipGraphDestroy(ga));
  CK(hipGraphDestroy(gb));
  CK(hipEventDestroy(e1));
  CK(hipEventDestroy(e2));
  return 0;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  CK(hipSetDevice(0));
  int rv = 0;
  CK(hipRuntimeGetVersion(&rv));
  std::printf("HIP runtime %d\n", rv);
  Ctx c;
  CK(hipStreamCreateWithFlags(&c.cap, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c.s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c.s2, hipStreamNonBlocking));
  CK(hipMalloc(&c.tick, 4));
  CK(hipMalloc(&c.slots, 16));
  std::printf("(%s)\n", "tickets: a0 / a1 = graph A, b = graph B; -1 = not in this case");
  int rc = run_case(c, 1, false);
  if (!rc) rc = run_case(c, 1, true);
  if (!rc) rc = run_case(c, 2, false);
  std::printf("probe done rc=%d\n", rc);
  return rc;
}
