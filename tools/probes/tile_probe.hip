// Access-pattern ceiling of the tiled x-march (stencil_tbl's memory pattern
// without its arithmetic): a workgroup of 16 waves owns a TZ-column x 48-row
// tile of a 1024^3 fp64 field and marches it along x, reading each plane's
// tile rows and writing them to the output (optionally one barrier per plane,
// D planes of prefetch).  Compared with a flat copy of the same bytes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

constexpr int N = 1024;           // points per axis
constexpr long SY = N, SX = (long)N * N;

// V doubles per lane along z (a wave covers 64 V columns), R rows per wave,
// 16 waves: tile 64V x 16R; D planes loaded ahead; BAR: barrier per plane
template <int V, int R, int D, bool BAR>
__global__ __launch_bounds__(1024) void march(const double* __restrict__ in, double* __restrict__ out, int nzb) {
  // 96 KiB of LDS, as the K = 3 kernel: one workgroup per CU
  __shared__ double pad[12288];
  if (nzb < 0) pad[threadIdx.x] = 1.0;
  if (nzb < 0) out[0] = pad[threadIdx.x ^ 1];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int zb = blockIdx.x % nzb, yb = blockIdx.x / nzb;
  const int c0 = zb * 64 * V, r0 = yb * 16 * R + wave * R;
  double q[D + 1][R][V];
  auto ld = [&](int x, double (&d)[R][V]) {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int col = c0 + v * 64 + lane, row = r0 + r;
        d[r][v] = (col < N && row < N) ? in[(long)x * SX + (long)row * SY + col] : 0.0;
      }
  };
#pragma unroll
  for (int i = 0; i < D; ++i) ld(i, q[i]);
  for (int xb = 0; xb < N; xb += D + 1) {
#pragma unroll
    for (int ph = 0; ph <= D; ++ph) {
      const int x = xb + ph;
      if (x >= N) break;
      if (x + D < N) ld(x + D, q[(ph + D) % (D + 1)]);
      if (BAR) __syncthreads();
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const int col = c0 + v * 64 + lane, row = r0 + r;
          if (col < N && row < N) out[(long)x * SX + (long)row * SY + col] = q[ph][r][v] * 1.0000001;
        }
    }
  }
}

template <typename F>
static double time_ms(F&& f, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  f();
  CK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0, 0));
    f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main() {
  const size_t bytes = (size_t)N * N * N * sizeof(double);
  double *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
#define RUN(V, R, D, BAR)                                                                                  \
  {                                                                                                        \
    const int nzb = (N + 64 * V - 1) / (64 * V), nyb = (N + 16 * R - 1) / (16 * R);                       \
    const double ms = time_ms([&] { march<V, R, D, BAR><<<nzb * nyb, 1024>>>(a, b, nzb); }, 3);            \
    std::printf("{\"probe\": \"march\", \"V\": %d, \"R\": %d, \"D\": %d, \"barrier\": %d, \"blocks\": %d, " \
                "\"tbps\": %.3f}\n",                                                                       \
                V, R, D, (int)BAR, nzb * nyb, 2.0 * bytes / (ms * 1e-3) / 1e12);                           \
    std::fflush(stdout);                                                                                   \
  }
  RUN(1, 3, 1, true) RUN(1, 3, 2, true) RUN(1, 3, 3, true) RUN(1, 3, 1, false) RUN(1, 3, 3, false)
  RUN(2, 3, 1, true) RUN(2, 3, 2, true) RUN(4, 3, 1, true) RUN(1, 1, 1, true) RUN(1, 1, 4, true)
  RUN(2, 1, 2, true) RUN(4, 1, 2, true)
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
