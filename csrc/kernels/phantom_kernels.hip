// heat3d-mi355x — device kernels of the phantom-rank performance proxy
// (PhantomComm, tools/rank_proxy.py): emulated wire time, clock stamps and
// transfers paced at a link rate.  No production schedule launches them; they
// build only with HEAT3D_PHANTOM (CMake option, default ON: tests and the
// proxy tools use them), kept out of the solver's kernel unit (kernels_hip.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "hip_helpers.hpp"

namespace heat3d {
namespace hip {

// Phantom comm kernels in RCCL's footprint (fat): RCCL's device kernel on
// this image (rcclGenericKernel, gpurun_out/r7t) is 256 threads with 140
// VGPRs and 20 KB of LDS, too big to sit beside an interior workgroup (16
// waves x 112 VGPRs); the clobber makes the allocator reserve v0..v139 (no
// instruction is emitted) and the launch asks for the LDS.
constexpr int kFatThreads = 256, kFatLds = 20480;
template <bool FAT>
__device__ __forceinline__ void fat_footprint() {
  if constexpr (FAT) asm volatile("" ::: "v139");
}

template <bool FAT>
__global__ __launch_bounds__(256) void delay_kernel(unsigned long long ticks) {
  fat_footprint<FAT>();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

void delay(double us, void* stream, int blocks, bool fat) {
  if (us <= 0) return;
  if (fat)
    hipLaunchKernelGGL(delay_kernel<true>, dim3((unsigned)std::max(1, blocks)), dim3(kFatThreads), kFatLds,
                       S(stream), (unsigned long long)(us * 100.0));
  else
    hipLaunchKernelGGL(delay_kernel<false>, dim3((unsigned)std::max(1, blocks)), dim3(64), 0, S(stream),
                       (unsigned long long)(us * 100.0));
  HIPK_CHECK(hipGetLastError());
}

// phantom transfers whose copies overlap the wire time: one lane stores the
// 100 MHz clock (a vector store), the delay spins until `ticks` after it
__global__ void stamp_kernel(unsigned long long* slot) {
  if (threadIdx.x == 0) *slot = __builtin_amdgcn_s_memrealtime();
}
template <bool FAT>
__global__ __launch_bounds__(256) void delay_since_kernel(const unsigned long long* slot, unsigned long long ticks) {
  fat_footprint<FAT>();
  const unsigned long long t0 = *static_cast<const volatile unsigned long long*>(slot);
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

void stamp(void* slot, void* stream) {
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, S(stream), static_cast<unsigned long long*>(slot));
  HIPK_CHECK(hipGetLastError());
}

void delay_since(const void* slot, double us, void* stream, int blocks, bool fat) {
  if (us <= 0) return;
  if (fat)
    hipLaunchKernelGGL(delay_since_kernel<true>, dim3((unsigned)std::max(1, blocks)), dim3(kFatThreads), kFatLds,
                       S(stream), static_cast<const unsigned long long*>(slot), (unsigned long long)(us * 100.0));
  else
    hipLaunchKernelGGL(delay_since_kernel<false>, dim3((unsigned)std::max(1, blocks)), dim3(64), 0, S(stream),
                       static_cast<const unsigned long long*>(slot), (unsigned long long)(us * 100.0));
  HIPK_CHECK(hipGetLastError());
}

// phantom transfers paced at the wire rate (--phantom-wire paced): `per`
// workgroups per transfer copy contiguous shares of it in 16 KiB chunks, chunk
// c of a share not before c * ticks_per16 after the workgroup's first clock
// read, and end no earlier than the share's wire time — a transport moving the
// data across the link at its rate with a few channels, not a burst copy.
// Every loop is bounded by the share length and one clock deadline.
struct PacedArgs {
  PacedCopy x[kPacedMax];
  int nx, per;
};
template <bool FAT>
__global__ __launch_bounds__(256) void paced_copy_kernel(PacedArgs a) {
  fat_footprint<FAT>();
  const int xi = blockIdx.x / a.per, b = blockIdx.x % a.per;
  if (xi >= a.nx) return;
  const uint4* __restrict__ src = static_cast<const uint4*>(a.x[xi].src);
  uint4* __restrict__ dst = static_cast<uint4*>(a.x[xi].dst);
  const int64_t n = a.x[xi].bytes / 16;
  const int64_t share = (n + a.per - 1) / a.per;
  const int64_t lo = min(n, (int64_t)b * share), hi = min(n, lo + share);
  const double tp = a.x[xi].ticks_per16;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  constexpr int kU = 8;                // 16-byte loads in flight per lane
  constexpr int64_t CH = 256 * kU;     // 16-byte words per chunk (32 KiB)
  for (int64_t c = lo; c < hi; c += CH) {
    const unsigned long long due = t0 + (unsigned long long)((double)(c - lo) * tp);
    while (__builtin_amdgcn_s_memrealtime() < due) __builtin_amdgcn_s_sleep(2);
    const int64_t e = min(hi, c + CH);
    uint4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (c + threadIdx.x + u * 256 < e) v[u] = src[c + threadIdx.x + u * 256];
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (c + threadIdx.x + u * 256 < e) dst[c + threadIdx.x + u * 256] = v[u];
  }
  const unsigned long long end = t0 + (unsigned long long)((double)(hi - lo) * tp);
  while (__builtin_amdgcn_s_memrealtime() < end) __builtin_amdgcn_s_sleep(8);
}

void paced_copy(const PacedCopy* xs, int n, int per, void* stream, bool fat) {
  HEAT3D_CHECK(per >= 1 && per <= 64, "paced_copy: 1..64 workgroups per transfer");
  for (int i0 = 0; i0 < n; i0 += kPacedMax) {
    PacedArgs a{};
    a.nx = std::min(kPacedMax, n - i0);
    a.per = per;
    for (int i = 0; i < a.nx; ++i) {
      a.x[i] = xs[i0 + i];
      HEAT3D_CHECK(a.x[i].bytes % 16 == 0 && reinterpret_cast<uintptr_t>(a.x[i].src) % 16 == 0 &&
                       reinterpret_cast<uintptr_t>(a.x[i].dst) % 16 == 0 && a.x[i].ticks_per16 >= 0,
                   "paced_copy: 16-byte aligned transfers");
    }
    if (fat)
      hipLaunchKernelGGL(paced_copy_kernel<true>, dim3((unsigned)(a.nx * per)), dim3(256), kFatLds, S(stream), a);
    else
      hipLaunchKernelGGL(paced_copy_kernel<false>, dim3((unsigned)(a.nx * per)), dim3(256), 0, S(stream), a);
    HIPK_CHECK(hipGetLastError());
  }
}

}  // namespace hip
}  // namespace heat3d
