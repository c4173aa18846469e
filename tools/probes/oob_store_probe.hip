// Probe: raw-buffer stores whose voffset lies past num_records are dropped
// (gfx950 MUBUF range check), also with a non-zero soffset.  Safe by
// construction: the buffer is 2.5 GiB, so a store that were NOT dropped would
// land inside it (base + 2 GiB + soffset), where the host looks for it.
//   hipcc --offload-arch=gfx950 -O2 tools/probes/oob_store_probe.hip -o /tmp/oob && /tmp/oob
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void probe(double* base, int soff_bytes) {
  const int lane = threadIdx.x;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
  const unsigned voff = lane < 32 ? (unsigned)lane * 8u : 0x80000000u + (unsigned)lane * 8u;
  const double v = 1000.0 + lane;
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(unsigned __attribute__((ext_vector_type(2))), v), r, voff,
                                        soff_bytes, 0);
  // an out-of-range load returns 0
  const unsigned long long got = __builtin_amdgcn_raw_buffer_load_b64(r, 0x80000000u, 0, 0)[0];
  if (lane == 40 && got != 0) base[1] = -1.0;
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 2;                                                       \
    }                                                                 \
  } while (0)

int main() {
  const size_t bytes = (size_t)5 << 29;  // 2.5 GiB
  double* d = nullptr;
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(d, 0, bytes));
  int bad = 0;
  for (int soff : {0, 4096, 1 << 20}) {
    CK(hipMemset(d, 0, bytes));
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, soff);
    CK(hipDeviceSynchronize());
    std::vector<double> lo(1024), hi(1024);
    CK(hipMemcpy(lo.data(), (char*)d + soff, lo.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hi.data(), (char*)d + 0x80000000ull + soff, hi.size() * 8, hipMemcpyDeviceToHost));
    int inr = 0, leaked = 0;
    for (int l = 0; l < 32; ++l) inr += lo[l] == 1000.0 + l;
    for (int l = 0; l < 1024; ++l) leaked += hi[l] != 0.0;
    double flag = 0;
    CK(hipMemcpy(&flag, d + 1, 8, hipMemcpyDeviceToHost));
    std::printf("soffset %d: in-range stores %d/32, leaked past num_records %d, oob load nonzero %d\n", soff, inr,
                leaked, flag == -1.0);
    bad += inr != 32 || leaked != 0;
  }
  CK(hipFree(d));
  std::printf(bad ? "FAIL\n" : "OK: out-of-range raw-buffer stores are dropped\n");
  return bad ? 1 : 0;
}
