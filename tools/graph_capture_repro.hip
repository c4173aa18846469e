// Minimal reproducer: hipStreamEndCapture overflows the host stack when two
// side streams of one capture wait on each other's events.
//
// Capture origin O forks side streams A and B (O records F; A, B wait F).
//   case 1: A and B only wait on O's events and O joins both   -> fine
//   case 2: additionally B waits on an event recorded on A      -> fine
//   case 3: additionally A waits on an event recorded on B      -> stack
//           overflow inside hipStreamEndCapture (libamdhip64 recurses
//           through the streams' parallel-capture lists, A -> B -> A -> ...)
// The solver's overlapped schedule has exactly case 3: the reduce stream waits
// for the comm stream's boundary slabs, the comm stream waits for the reduce
// stream's convergence check.  The solver therefore builds multi-stream graphs
// explicitly (HipBackend graph recording: one child graph per operation,
// dependencies from the recorded event edges) instead of capturing them.
//
//   hipcc --offload-arch=gfx950 -O2 tools/graph_capture_repro.hip -o /tmp/repro
//   /tmp/repro 2      # runs cases 1..2 (what tests/test_gpu_graph.py runs)
//   /tmp/repro 3      # also case 3: expect a SIGSEGV (documented, not in tests)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_)); \
      std::exit(2);                                                        \
    }                                                                      \
  } while (0)

__global__ void inc(int* p, int v) {
  if (threadIdx.x == 0) atomicAdd(p, v);
}

static int run_case(int c, hipStream_t O, hipStream_t A, hipStream_t B, int* d) {
  hipEvent_t ev[16];
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  CK(hipMemsetAsync(d, 0, sizeof(int), O));
  CK(hipStreamSynchronize(O));
  CK(hipStreamBeginCapture(O, hipStreamCaptureModeRelaxed));
  CK(hipEventRecord(ev[0], O));
  CK(hipStreamWaitEvent(A, ev[0], 0));
  CK(hipStreamWaitEvent(B, ev[0], 0));
  int expect = 0;
  for (int it = 0; it < 2; ++it) {
    hipLaunchKernelGGL(inc, dim3(1), dim3(64), 0, O, d, 1);
    hipLaunchKernelGGL(inc, dim3(1), dim3(64), 0, A, d, 10);
    CK(hipEventRecord(ev[1 + 4 * it], A));
    if (c >= 2) CK(hipStreamWaitEvent(B, ev[1 + 4 * it], 0));  // A -> B
    hipLaunchKernelGGL(inc, dim3(1), dim3(64), 0, B, d, 100);
    CK(hipEventRecord(ev[2 + 4 * it], B));
    if (c >= 3) CK(hipStreamWaitEvent(A, ev[2 + 4 * it], 0));  // B -> A: a cycle of side streams
    if (c >= 4) CK(hipStreamWaitEvent(O, ev[2 + 4 * it], 0));  // origin waits on B mid-capture
    expect += 111;
  }
  CK(hipEventRecord(ev[13], A));
  CK(hipEventRecord(ev[14], B));
  CK(hipStreamWaitEvent(O, ev[13], 0));
  CK(hipStreamWaitEvent(O, ev[14], 0));
  std::printf("case %d: end capture\n", c);
  std::fflush(stdout);
  hipGraph_t g;
  CK(hipStreamEndCapture(O, &g));
  hipGraphExec_t x;
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(x, O));
  CK(hipStreamSynchronize(O));
  int h = 0;
  CK(hipMemcpy(&h, d, sizeof(int), hipMemcpyDeviceToHost));
  std::printf("case %d: replay sum %d (expect %d) %s\n", c, h, expect, h == expect ? "ok" : "WRONG");
  std::fflush(stdout);
  CK(hipGraphExecDestroy(x));
  CK(hipGraphDestroy(g));
  for (auto& e : ev) CK(hipEventDestroy(e));
  return h == expect ? 0 : 1;
}

int main(int argc, char** argv) {
  const int upto = argc > 1 ? std::atoi(argv[1]) : 2;
  hipStream_t O, A, B;
  CK(hipStreamCreateWithFlags(&O, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  int* d = nullptr;
  CK(hipMalloc(&d, sizeof(int)));
  int bad = 0;
  for (int c = 1; c <= upto; ++c) bad += run_case(c, O, A, B, d);
  CK(hipFree(d));
  std::printf("done, %d wrong\n", bad);
  return bad ? 1 : 0;
}
