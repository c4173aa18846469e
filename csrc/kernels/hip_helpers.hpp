// heat3d-mi355x — device helpers shared by the gfx950 kernel translation units.
// Included only from .hip files.
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.hpp"

#pragma clang fp contract(off)

namespace heat3d {
namespace hip {

#define HIPK_CHECK(expr)                                                             \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess) HEAT3D_THROW("HIP error " << hipGetErrorString(_e) << " at " #expr); \
  } while (0)

static inline hipStream_t S(void* s) { return static_cast<hipStream_t>(s); }

template <typename Real, int V>
struct VecOf;
template <> struct VecOf<double, 1> { typedef double type; };
template <> struct VecOf<double, 2> { typedef double type __attribute__((ext_vector_type(2))); };
template <> struct VecOf<float, 1> { typedef float type; };
template <> struct VecOf<float, 2> { typedef float type __attribute__((ext_vector_type(2))); };
template <> struct VecOf<float, 4> { typedef float type __attribute__((ext_vector_type(4))); };

// FTCS 7-point update (heat3D.cu:128-131) with the reference GPU kernel's
// FMA contraction; the single definition lives in kernels.hpp (ftcs_update)
// and is shared with the CPU backend, so fields stay bitwise identical.
template <typename Real>
__device__ __forceinline__ Real ftcs(Real c, Real xm, Real xp, Real ym, Real yp, Real zm, Real zp,
                                     Real Dx, Real Dy, Real Dz) {
  return ftcs_update<Real>(c, xm, xp, ym, yp, zm, zp, Dx, Dy, Dz);
}

// ---- cross-lane helpers ----------------------------------------------------
// DPP wave_shr:1 (0x138): lane i <- lane i-1 ; lane 0 keeps `old`.
// DPP wave_shl:1 (0x130): lane i <- lane i+1 ; lane 63 keeps `old`.
__device__ __forceinline__ double dpp_shr1(double old, double v) {
  long long ov = __builtin_bit_cast(long long, old), vv = __builtin_bit_cast(long long, v);
  int lo = __builtin_amdgcn_update_dpp((int)ov, (int)vv, 0x138, 0xf, 0xf, false);
  int hi = __builtin_amdgcn_update_dpp((int)(ov >> 32), (int)(vv >> 32), 0x138, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double dpp_shl1(double old, double v) {
  long long ov = __builtin_bit_cast(long long, old), vv = __builtin_bit_cast(long long, v);
  int lo = __builtin_amdgcn_update_dpp((int)ov, (int)vv, 0x130, 0xf, 0xf, false);
  int hi = __builtin_amdgcn_update_dpp((int)(ov >> 32), (int)(vv >> 32), 0x130, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ float dpp_shr1(float old, float v) {
  int r = __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v),
                                      0x138, 0xf, 0xf, false);
  return __builtin_bit_cast(float, r);
}
__device__ __forceinline__ float dpp_shl1(float old, float v) {
  int r = __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v),
                                      0x130, 0xf, 0xf, false);
  return __builtin_bit_cast(float, r);
}
// Same shifts with the vacated lane (0 resp. 63) zero-filled (bound_ctrl):
// no "old" operand, so no register copy in front of the DPP move.  For
// neighbours whose edge lane is invalid anyway.
__device__ __forceinline__ double dpp_shr1z(double v) {
  long long vv = __builtin_bit_cast(long long, v);
  int lo = __builtin_amdgcn_mov_dpp((int)vv, 0x138, 0xf, 0xf, true);
  int hi = __builtin_amdgcn_mov_dpp((int)(vv >> 32), 0x138, 0xf, 0xf, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double dpp_shl1z(double v) {
  long long vv = __builtin_bit_cast(long long, v);
  int lo = __builtin_amdgcn_mov_dpp((int)vv, 0x130, 0xf, 0xf, true);
  int hi = __builtin_amdgcn_mov_dpp((int)(vv >> 32), 0x130, 0xf, 0xf, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ float dpp_shr1z(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float dpp_shl1z(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x130, 0xf, 0xf, true));
}
__device__ __forceinline__ double readlane(double v, int lane) {
  long long b = __builtin_bit_cast(long long, v);
  int lo = __builtin_amdgcn_readlane((int)b, lane);
  int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ float readlane(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

// Residual max over non-negative doubles, done on their IEEE bit patterns:
// integer order == double order, and a NaN (bits above +Inf) wins, so a
// blown-up field reaches the convergence check as a fault.
__device__ __forceinline__ double res_max(double m, double d) { return (d != d || d > m) ? d : m; }

__device__ __forceinline__ unsigned long long wave_max_bits(double m) {
  unsigned long long b = (unsigned long long)__builtin_bit_cast(long long, m);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long q = __shfl_xor(b, o, 64);
    b = q > b ? q : b;
  }
  return b;
}

// Device-scope max into a residual slot.  The slot only grows during a
// sweep, so a (possibly stale, hence never larger) relaxed read that is
// already >= b makes the atomic redundant: most workgroups skip it.  All
// workgroups of a grid finish at nearly the same time and agent-scope atomics
// on one address serialise at the memory side, so unfiltered per-wave
// atomics (1728 workgroups x 16 waves x K slots) cost ~0.5 ms per sweep.
__device__ __forceinline__ void slot_max(unsigned long long* slot, unsigned long long b) {
  if (b > __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(slot, b);
}

__device__ __forceinline__ void residual_commit(unsigned long long* slot, double m) {
  const unsigned long long b = wave_max_bits(m);
  if ((threadIdx.x & 63) == 0) slot_max(slot, b);
}

// Fused convergence check of a K-step sweep (StencilParams::fuse_check), run
// by every workgroup after its residual commit (or instead of it, when the
// sweep is a no-op because the run has converged): each workgroup takes a
// ticket once its residual atomics are acknowledged; the one that draws the
// last ticket swaps the K slots back to their initial value (an atomic
// exchange returns the value at the atomics' coherence point, whatever this
// XCD's L2 holds), runs check_convergence over them in order and resets the
// ticket counter —
// what check_kernel did after the sweep.  No agent-scope fences: a release
// fence is an L2 write-back (buffer_wbl2), which every one of the sweep's
// ~2000 workgroups issuing it cost 6-7 % of the 1022^3 sweep (round 6,
// gpurun_out/r6e); only the residual atomics must be ordered before the
// ticket (s_waitcnt), the state fields the last workgroup writes are read by
// later kernels and the host, after this kernel's end-of-kernel release.
// Every thread of the workgroup must reach it (barrier).
// RL (kResidualLastOnly): the sweep computed only its last step's residual.
// The residual max-norm of FTCS is non-increasing (Solver::residual_last_ok),
// so a last residual at or above the threshold means none of the sweep's
// steps converged: steps 0..K-2 only advance the iteration; a last residual
// below it sets done with conv_iter at the sweep's last iteration and
// `coarse` = K, and Solver::resolve_coarse finds the first converged one.
template <int K, bool RL = false>
__device__ __forceinline__ void fused_check_tail(DeviceState* st, int slot, int nblocks) {
  __syncthreads();
  if (threadIdx.x != 0) return;
  __builtin_amdgcn_s_waitcnt(0);  // this wave's residual atomics (wave 0 issued them) acknowledged
  const unsigned t = __hip_atomic_fetch_add(&st->sweep_tickets, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t != (unsigned)nblocks - 1u) return;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    // read and reset in one exchange (an idempotent read-modify-write would
    // be lowered to a plain load, which may hit this XCD's L2)
    const unsigned long long bits =
        __hip_atomic_exchange(&st->residual[slot + i], kResidualInitBits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (RL && i < K - 1) {
      st->iter = st->iter + 1;
      continue;
    }
    const int was = st->done;
    check_convergence_scalar(st, __builtin_bit_cast(double, (long long)bits));
    if (RL && !was && st->done) st->coarse = K;
  }
  (void)__hip_atomic_exchange(&st->sweep_tickets, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup-level commit of K residual slots: one wave max per slot into LDS,
// then lanes s < K of wave 0 reduce over the NW waves and commit once.  Must
// be reached by every thread of the workgroup (contains a barrier).
template <int NW, int K>
__device__ __forceinline__ void residual_commit_block(unsigned long long* slots, const double (&m)[K],
                                                      bool nan_any, unsigned long long (&red)[NW][K]) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool nan_w = __any(nan_any);
#pragma unroll
  for (int s = 0; s < K; ++s) {
    const unsigned long long b = wave_max_bits(m[s]);
    if (lane == 0) red[wave][s] = nan_w ? 0x7ff8000000000000ULL : b;
  }
  __syncthreads();
  if (wave == 0 && lane < K) {
    unsigned long long b = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) b = red[w][lane] > b ? red[w][lane] : b;
    slot_max(slots + lane, b);
  }
}

__device__ __forceinline__ bool flag_set(const int* done) {
  return done != nullptr && __builtin_nontemporal_load(done) != 0;
}

// Resident workgroups of `kernel` on the whole device (occupancy x CUs).
int device_slots(const void* kernel, int block);
// x-segment length for an x-marching kernel with `halo` extra planes per segment.
int choose_segment(int64_t nx, int64_t tiles, int slots, int halo = 2);

// x schedule of the register-ring kernel (TBRArgs): segments of `seg`
// planes; n1 pieces in whole rounds, then r leftover pieces cut at `split`
// into A parts and nb2 (0 or r) B parts.
struct XPlan {
  int seg = 1, n1 = 0, r = 0, split = 0, nb2 = 0;
};
// Chosen by simulating greedy in-order dispatch onto `slots` resident
// workgroups (cost of a piece: its planes + `fill` pipeline planes, rounded up
// to chunks of U); cached per shape.  equal_only: no split (previous policy).
// HEAT3D_TRACE launch diagnostics (read once per process)
bool trace_enabled();
XPlan plan_x(int64_t nx, int64_t tiles, int slots, int fill, int U, bool equal_only = false);
XPlan fixed_xplan(int64_t nx, int64_t tiles, int seg);
// Makespan of a plan in the same greedy-dispatch model (plane steps per slot).
double xplan_makespan(const XPlan& p, int64_t nx, int64_t tiles, int slots, int fill, int U);
// A tiling's sweep cost for the z-stride choice: max(makespan, work / HBM-saturating slots)
double tiling_cost(const XPlan& p, int64_t nx, int64_t tiles, int slots, int fill, int U);
// Compute units of the current device (cached per device).
int device_cus();

// Sweep-schedule autotuning (round 3).  The dispatch model above picks the
// best measured x segment on the 1022^3 boxes but not on every box, and the
// z-stride rule was set by proxies (the 8-GPU slab share's interior,
// 122 x 1022^2, runs 774 GLUPS with 56-column tiles against 723 with 58;
// profiles/xplan_calibration_r03.md).  tune_schedule times, twice each, every
// (z stride, spec field L) candidate on `s` — per stride in zs_opts the
// model's x plan (L = -3), fixed segments of nx/k planes and (round 6, with
// nyb > 0: the y tile count, so that the tiles of each stride are known) the
// model's best fixed segment lengths of any size, whose last piece per tile
// is short — keeps the
// fastest (the model's choice, candidate 0, unless another is >= 1.5% faster
// in a confirming interleaved rerun) per (device, kernel, box, slots,
// reserved CUs) and returns it; tuned_lookup returns a kept choice.
struct SchedChoice {
  int zs = 0, L = 0;
};
bool tuned_lookup(const void* kfn, const int64_t box[3], int slots, int reserved, SchedChoice* out);
SchedChoice tune_schedule(const char* name, const void* kfn, const int64_t box[3], int slots, int reserved, int U,
                          const std::vector<int>& zs_opts, hipStream_t s,
                          const std::function<void(int, int)>& launch, int64_t nyb = 0, int fill = 0);


}  // namespace hip
}  // namespace heat3d
