// HBM bandwidth probe on one MI355X: copy / read / write streams in several
// shapes (bytes per lane per instruction, instructions in flight per lane,
// workgroups per CU), to find the copy rate the stencil sweeps should be
// compared with.  ./hbm_probe [GiB per buffer]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
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

typedef float f4 __attribute__((ext_vector_type(4)));

// grid-stride copy, U independent 16-B loads per lane in flight before the stores
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(const f4* __restrict__ a, f4* __restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * 256 * U;
  for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n; base += stride) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * 256;
      v[u] = i < n ? (NT ? __builtin_nontemporal_load(a + i) : a[i]) : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * 256;
      if (i < n) {
        if (NT) __builtin_nontemporal_store(v[u], b + i);
        else b[i] = v[u];
      }
    }
  }
}

// contiguous chunk per workgroup (each block streams its own slice)
template <int U>
__global__ __launch_bounds__(256) void copy_chunk_k(const f4* __restrict__ a, f4* __restrict__ b, size_t n) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  for (size_t base = lo + threadIdx.x; base < hi; base += 256 * U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * 256;
      v[u] = i < hi ? a[i] : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * 256;
      if (i < hi) b[i] = v[u];
    }
  }
}

template <int U>
__global__ __launch_bounds__(256) void read_k(const f4* __restrict__ a, size_t n, float* out) {
  const size_t stride = (size_t)gridDim.x * 256 * U;
  f4 acc{0, 0, 0, 0};
  for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n; base += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * 256;
      if (i < n) acc += a[i];
    }
  }
  if (acc.x == 12345.f) out[0] = acc.y;  // keeps the loads
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

int main(int argc, char** argv) {
  const double gib = argc > 1 ? std::atof(argv[1]) : 4.0;
  const size_t bytes = (size_t)(gib * (1ull << 30));
  const size_t n = bytes / 16;
  f4 *a, *b;
  float* o;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&o, 64));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  auto rep = [&](const char* name, int blocks, double moved, double ms) {
    std::printf("{\"probe\": \"%s\", \"blocks\": %d, \"GB\": %.2f, \"tbps\": %.3f}\n", name, blocks, moved / 1e9,
                moved / (ms * 1e-3) / 1e12);
    std::fflush(stdout);
  };
  for (int wpc : {2, 4, 8, 16}) {
    const int blocks = cus * wpc;
    rep("copy_u1", blocks, 2.0 * bytes, time_ms([&] { copy_k<1, false><<<blocks, 256>>>(a, b, n); }, 5));
    rep("copy_u4", blocks, 2.0 * bytes, time_ms([&] { copy_k<4, false><<<blocks, 256>>>(a, b, n); }, 5));
    rep("copy_u8", blocks, 2.0 * bytes, time_ms([&] { copy_k<8, false><<<blocks, 256>>>(a, b, n); }, 5));
    rep("copy_u4_nt", blocks, 2.0 * bytes, time_ms([&] { copy_k<4, true><<<blocks, 256>>>(a, b, n); }, 5));
    rep("copy_chunk_u4", blocks, 2.0 * bytes, time_ms([&] { copy_chunk_k<4><<<blocks, 256>>>(a, b, n); }, 5));
    rep("read_u4", blocks, 1.0 * bytes, time_ms([&] { read_k<4><<<blocks, 256>>>(a, n, o); }, 5));
    rep("read_u8", blocks, 1.0 * bytes, time_ms([&] { read_k<8><<<blocks, 256>>>(a, n, o); }, 5));
  }
  rep("hipMemcpyDtoD", 0, 2.0 * bytes, time_ms([&] { CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0)); }, 5));
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(o));
  return 0;
}
