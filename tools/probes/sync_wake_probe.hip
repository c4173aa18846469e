// Probe: how late does the host wake from a wait on in-flight work?
//
// bench.py's barrier before the timed window (stream syncs + a device-wide
// synchronize after the preheat sweeps) took ~1.3-1.5 s under HIP 7.2 while
// the GPU finished in ~18 ms (torch's HIP 7.0: 18 ms), idling the GPU before
// the timed window (gpurun_out/r6h trace, r6i-r6k phases).  This reproduces the
// preheat's shape — ~18 ms of kernels on stream A, then an event recorded on A
// that streams B and C wait for — and times each way of waiting for it.
//
//   hipcc --offload-arch=gfx950 -O2 tools/probes/sync_wake_probe.hip -o /tmp/swp && /tmp/swp
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::printf("FAIL %s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

__global__ void spin_kernel(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  CK(hipSetDevice(0));
  if (argc > 1) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  unsigned flags = 0;
  CK(hipGetDeviceFlags(&flags));
  int rv = 0;
  CK(hipRuntimeGetVersion(&rv));
  std::printf("HIP runtime %d, device flags 0x%x\n", rv, flags);
  hipStream_t a, b, c;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const unsigned long long per = 360000;  // 3.6 ms at 100 MHz
  auto issue = [&](bool fork) {
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(spin_kernel, dim3(256), dim3(64), 0, a, per);
    if (fork) {
      (void)hipEventRecord(ev, a);
      (void)hipStreamWaitEvent(b, ev, 0);
      (void)hipStreamWaitEvent(c, ev, 0);
    }
  };
  struct Way {
    const char* name;
    bool fork;
    int how;
  };
  const Way ways[] = {
      {"kernels only, hipStreamSynchronize(A)", false, 0},
      {"fork, hipStreamSynchronize(A)", true, 0},
      {"fork, hipStreamSynchronize(A, B, C)", true, 1},
      {"fork, hipDeviceSynchronize", true, 2},
      {"fork, hipEventSynchronize(ev) then B, C", true, 3},
      {"fork, poll hipStreamQuery(A, B, C)", true, 4},
      {"fork, hipStreamSynchronize(C) first", true, 5},
      {"kernels only, hipDeviceSynchronize", false, 2},
  };
  CK(hipDeviceSynchronize());
  for (const Way& w : ways) {
    for (int rep = 0; rep < 3; ++rep) {
      const double t0 = now_ms();
      issue(w.fork);
      switch (w.how) {
        case 0: CK(hipStreamSynchronize(a)); break;
        case 1:
          CK(hipStreamSynchronize(a));
          CK(hipStreamSynchronize(b));
          CK(hipStreamSynchronize(c));
          break;
        case 2: CK(hipDeviceSynchronize()); break;
        case 3:
          CK(hipEventSynchronize(ev));
          CK(hipStreamSynchronize(b));
          CK(hipStreamSynchronize(c));
          break;
        case 4:
          for (hipStream_t s : {a, b, c}) {
            hipError_t e;
            while ((e = hipStreamQuery(s)) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(20));
            CK(e);
          }
          break;
        case 5:
          CK(hipStreamSynchronize(c));
          CK(hipStreamSynchronize(a));
          CK(hipStreamSynchronize(b));
          break;
      }
      const double t1 = now_ms();
      std::printf("%-44s rep %d: %8.2f ms (GPU work ~18 ms)\n", w.name, rep, t1 - t0);
      CK(hipDeviceSynchronize());
    }
  }
  std::printf("probe done\n");
  return 0;
}
