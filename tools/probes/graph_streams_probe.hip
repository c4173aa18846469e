// Probe: can the overlapped multi-stream schedule be replayed as one linear
// hipGraph per stream (launched on its own stream, keeping the stream's CU
// mask and priority), with the cross-stream dependencies as device-side
// value waits instead of events?
//
//   hipcc --offload-arch=gfx950 -O2 tools/probes/graph_streams_probe.hip -o /tmp/gsp && /tmp/gsp
//
// 1. a placement kernel captured into a graph, launched on a CU-masked
//    stream (top 8 mask bits cleared): how many CUs does it reach?
// 2. hipStreamWaitValue64 / hipStreamWriteValue64 captured into graphs
//    (hipStreamBeginCaptureToGraph, as hip_backend.cpp records): graph A on
//    stream 1 waits for a value graph B on stream 2 writes, B launched AFTER
//    A (the wait is resolved on the device at run time, not at launch).
// Every wait has a host-side escape: the signal slots live in pinned host
// memory and the host writes them itself if the device has not after 2 s.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <set>
#include <thread>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::printf("FAIL %s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);             \
      return 1;                                                                                \
    }                                                                                          \
  } while (0)

__global__ void probe_kernel(unsigned* out, unsigned long long ticks) {
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    out[blockIdx.x] = ((xcc & 0xf) << 8) | ((hw >> 8) & 0xff);
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

// order witness: stores a ticket taken from a shared counter
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

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  CK(hipSetDevice(0));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int words = (cus + 31) / 32;
  std::vector<uint32_t> mask(words, 0u);
  for (int i = 0; i < cus - 8; ++i) mask[i / 32] |= 1u << (i % 32);
  hipStream_t masked, plain, cap;
  CK(hipExtStreamCreateWithCUMask(&masked, (uint32_t)words, mask.data()));
  CK(hipStreamCreateWithFlags(&plain, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  const int blocks = 4096;
  unsigned* d_out;
  CK(hipMalloc(&d_out, blocks * sizeof(unsigned)));
  std::vector<unsigned> h(blocks);
  auto count = [&](const char* what) {
    CK(hipMemcpy(h.data(), d_out, blocks * sizeof(unsigned), hipMemcpyDeviceToHost));
    std::set<unsigned> s(h.begin(), h.end());
    std::printf("%-44s distinct CUs %zu of %d\n", what, s.size(), cus);
    return 0;
  };
  // eager, masked stream
  hipLaunchKernelGGL(probe_kernel, dim3(blocks), dim3(64), 0, masked, d_out, 2000ull);
  CK(hipStreamSynchronize(masked));
  if (count("eager on masked stream")) return 1;
  // graph captured to a graph (BeginCaptureToGraph on a helper stream), launched on the masked stream
  {
    hipGraph_t g;
    CK(hipGraphCreate(&g, 0));
    CK(hipStreamBeginCaptureToGraph(cap, g, nullptr, nullptr, 0, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(probe_kernel, dim3(blocks), dim3(64), 0, cap, d_out, 2000ull);
    hipLaunchKernelGGL(probe_kernel, dim3(blocks), dim3(64), 0, cap, d_out, 2000ull);
    hipGraph_t g2;
    CK(hipStreamEndCapture(cap, &g2));
    hipGraphExec_t ex;
    CK(hipGraphInstantiateWithFlags(&ex, g, 0));
    CK(hipMemset(d_out, 0, blocks * sizeof(unsigned)));
    CK(hipGraphLaunch(ex, masked));
    CK(hipStreamSynchronize(masked));
    if (count("linear 2-kernel graph launched on masked")) return 1;
    CK(hipGraphLaunch(ex, plain));
    CK(hipStreamSynchronize(plain));
    if (count("same graph launched on plain stream")) return 1;
    CK(hipGraphExecDestroy(ex));
    CK(hipGraphDestroy(g));
  }
  // value waits / writes inside graphs
  unsigned long long* sig = nullptr;  // pinned host: the host can always release a wait
  CK(hipHostMalloc(&sig, 4096, hipHostMallocDefault));
  unsigned long long* dsig = nullptr;
  CK(hipMalloc(&dsig, 4096));
  unsigned *tick, *slots;
  CK(hipMalloc(&tick, 4));
  CK(hipMalloc(&slots, 64));
  bool host_ok = false;
  for (int mem = 0; mem < 2; ++mem) {
    if (mem == 1 && !host_ok) break;  // device slots only after the host-releasable case worked
    unsigned long long* sp = mem == 0 ? sig : dsig;
    const char* where = mem == 0 ? "pinned host" : "device";
    CK(hipMemset(tick, 0, 4));
    CK(hipMemset(slots, 0xff, 64));
    if (mem == 0) sig[0] = sig[1] = 0;
    else CK(hipMemset(dsig, 0, 4096));
    hipGraph_t ga, gb;
    CK(hipGraphCreate(&ga, 0));
    CK(hipGraphCreate(&gb, 0));
    // A (masked stream): wait sig[0] >= 1, ticket -> slots[0], write sig[1] = 1
    hipError_t e1 = hipStreamBeginCaptureToGraph(cap, ga, nullptr, nullptr, 0, hipStreamCaptureModeThreadLocal);
    hipError_t ew = hipStreamWaitValue64(cap, sp + 0, 1, hipStreamWaitValueGte, ~0ull);
    hipLaunchKernelGGL(ticket_kernel, dim3(1), dim3(64), 0, cap, tick, slots + 0);
    hipError_t ewr = hipStreamWriteValue64(cap, sp + 1, 1, 0);
    hipGraph_t tmp;
    hipError_t e2 = hipStreamEndCapture(cap, &tmp);
    std::printf("[%s] capture A: begin %s, waitValue %s, writeValue %s, end %s\n", where, hipGetErrorString(e1),
                hipGetErrorString(ew), hipGetErrorString(ewr), hipGetErrorString(e2));
    if (e1 || ew || ewr || e2) {
      (void)hipGetLastError();
      if (mem == 0) sig[0] = sig[1] = 1;  // a wait that ran instead of being captured
      std::printf("capture of value ops failed: cap stream %s\n", wait_stream(cap, 2.0) ? "idle" : "STUCK");
      break;
    }
    std::printf("[%s] graph A nodes captured\n", where);
    // B (plain stream): ticket -> slots[1] after a 200 us spin, write sig[0] = 1, wait sig[1] >= 1, ticket -> slots[2]
    CK(hipStreamBeginCaptureToGraph(cap, gb, nullptr, nullptr, 0, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(64), 0, cap, d_out, 20000ull);
    hipLaunchKernelGGL(ticket_kernel, dim3(1), dim3(64), 0, cap, tick, slots + 1);
    CK(hipStreamWriteValue64(cap, sp + 0, 1, 0));
    CK(hipStreamWaitValue64(cap, sp + 1, 1, hipStreamWaitValueGte, ~0ull));
    hipLaunchKernelGGL(ticket_kernel, dim3(1), dim3(64), 0, cap, tick, slots + 2);
    CK(hipStreamEndCapture(cap, &tmp));
    hipGraphExec_t xa, xb;
    CK(hipGraphInstantiateWithFlags(&xa, ga, 0));
    CK(hipGraphInstantiateWithFlags(&xb, gb, 0));
    for (int rep = 0; rep < 3; ++rep) {
      if (mem == 0) {
        sig[0] = sig[1] = 0;
      } else {
        CK(hipMemsetAsync(dsig, 0, 16, plain));
      }
      CK(hipMemsetAsync(tick, 0, 4, plain));
      CK(hipStreamSynchronize(plain));
      CK(hipStreamSynchronize(masked));
      const auto t0 = std::chrono::steady_clock::now();
      CK(hipGraphLaunch(xa, masked));  // A first: its wait must hold until B writes
      CK(hipGraphLaunch(xb, plain));
      bool ok = wait_stream(masked, 2.0) && wait_stream(plain, 2.0);
      if (!ok) {
        std::printf("[%s] rep %d: TIMEOUT, releasing from the host\n", where, rep);
        if (mem == 0) {
          sig[0] = sig[1] = 1;
        } else {
          std::printf("device slots cannot be released from the host; giving up\n");
          return 2;
        }
        if (!wait_stream(masked, 2.0) || !wait_stream(plain, 2.0)) return 3;
      }
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      unsigned hs[3];
      CK(hipMemcpy(hs, slots, sizeof(hs), hipMemcpyDeviceToHost));
      // expected tickets: B's first (0), then A (1), then B's second (2)
      const bool ord = ok && hs[1] == 0 && hs[0] == 1 && hs[2] == 2;
      if (mem == 0) host_ok = (rep == 0 || host_ok) && ord;
      std::printf("[%s] rep %d: tickets B1=%u A=%u B2=%u (%s) %.0f us\n", where, rep, hs[1], hs[0], hs[2],
                  ord ? "ordered" : "WRONG ORDER", us);
    }
    CK(hipGraphExecDestroy(xa));
    CK(hipGraphExecDestroy(xb));
  }
  std::printf("probe done\n");
  return 0;
}
