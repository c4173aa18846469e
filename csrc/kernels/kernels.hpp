// heat3d-mi355x — kernel launch API, implemented twice:
//   heat3d::hip::*  hand-written gfx950 kernels (kernels_hip.hip)
//   heat3d::cpu::*  OpenMP host kernels used by the CPU backend / oracle (kernels_cpu.cpp)
//
// Both evaluate the FTCS update through ftcs_update() below: the reference's
// per-cell expression (heat3D.cu:128-131) with the fused
// multiply-adds nvcc puts into the reference's GPU kernel, explicit, and no
// other contraction, so the GPU and CPU backends agree bit for bit.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../core/common.hpp"
#include "layout.hpp"

namespace heat3d {

struct KernelSpec {
  // Tile: the single-step kernel (kernels_hip.hip; single steps, rollback
  // recomputation, runs without temporal blocking).  Naive: one thread per
  // point, the simplest gfx950 form (a test oracle).  TBL: the K-step
  // temporally blocked lean kernel (stencil_tbl.hip; fp32 packed pairs in
  // stencil_tbp.hip), K time steps per HBM sweep.  The round-1/2 queue and
  // register-ring sweep kernels (tb2 / tbK / trK) were retired in round 3:
  // no default path used them (docs/PERFORMANCE.md keeps their numbers).
  enum Kind { Naive = 0, Tile = 2, TBL = 6 } kind = Tile;
  int K = 0;  // multi-step kinds: time steps per sweep
  int WZ = 0, WY = 0;  // waves per workgroup along z and y
  int V = 0;  // elements per lane along z (0 = default for dtype)
  int R = 0;  // rows per wave along y (0 = default)
  int L = 0;  // x-segment length per wave (0 = auto)
  int O = -1; // TBL: output-store cache-policy bits (2 = nt)
  int NT = 0; // TBL: T^n ring size
  int ZS = 0; // TBL: tile stride along z (stored columns per tile; 0 = chosen per box)
  bool multi_step() const { return kind == TBL; }
  static KernelSpec parse(const std::string& s);
  std::string str() const;
  // zero (default) fields replaced by the tuned defaults for dtype t
  // (profiles/kernel_sweep.md); the kernel dispatchers and kernel names use it
  KernelSpec resolved(DType t) const;
};

struct StencilParams {
  const void* in = nullptr;
  void* out = nullptr;
  Layout L;
  Box box;                  // local owned coordinates to update
  double D[3] = {0, 0, 0};  // Dx, Dy, Dz
  DeviceState* state = nullptr;
  int slot = 0;             // residual slot (multi-step kernels: first of K slots)
  // multi-step kernels only: x range [ux0, ux1) in which the intermediate
  // fields T^{n+s} are computed (beyond the box on faces with a deep
  // neighbour halo); outside it they stay T^n (Dirichlet ghosts).
  // ux1 < ux0 means "the box's x range".
  int64_t ux[2] = {0, -1};
  // same for y and z (block decompositions with deep y / z halos)
  int64_t uy[2] = {0, -1}, uz[2] = {0, -1};
  // CUs the launch stream's CU mask keeps free (persistent sweeps launch as
  // many workgroups as the remaining CUs hold)
  int cu_reserved = 0;
  // sweeps only: time the x-schedule candidates on this launch (a sweep is
  // idempotent: every candidate writes the same T^{n+K} to out) and keep the
  // fastest for this kernel and box shape (autotune_x_schedule)
  bool tune = false;
  // false: the kernel honours state->done (a no-op once converged) but
  // records no residual (Solver::preheat's idempotent warm-up sweeps)
  bool residual = true;
  // K-step sweeps of a single-subdomain run: the last workgroup to finish runs
  // the convergence check of the sweep's K residual slots (check_convergence
  // semantics, bitwise the same state) instead of a separate check kernel
  // after it, which cost ~10 us per sweep on the critical path (a one-lane
  // kernel and its dispatch; profiles/r06)
  bool fuse_check = false;
};

struct InitParams {
  void* field = nullptr;
  Layout L;
  int64_t gstart[3] = {0, 0, 0};  // global index of owned (0,0,0)
  int64_t N[3] = {0, 0, 0};
  double h[3] = {0, 0, 0};
};

// Apply the Dirichlet boundary value at a global vertex (heat3D.cu:414-453
// order: TOP (y = 1) <- 1.0, then LEFT/RIGHT/BACK/FRONT <- y overwrite,
// BOTTOM stays 0; interior 0).
H3D_HD inline double boundary_value(int64_t gi, int64_t gj, int64_t gk, const int64_t N[3],
                             const double h[3]) {
  if (gi == 0 || gi == N[0] - 1 || gk == 0 || gk == N[2] - 1)
    return static_cast<double>(gj) * h[1];
  if (gj == N[1] - 1) return 1.0;
  return 0.0;
}

namespace hip {
void init_field(DType t, const InitParams& p, void* stream);
void stencil(DType t, const StencilParams& p, const KernelSpec& k, void* stream);
// K-step temporally blocked sweep, lean kernel (stencil_tbl.hip), K = k.K
void stencil_lean(DType t, const StencilParams& p, const KernelSpec& k, void* stream);
// z tile stride of the lean kernel for a box (host-side choice, stencil_tbl.hip)
int lean_z_stride(int64_t nx, int64_t ny, int64_t nz, int K, int esize, int TY, int slots, int U, int L);
// The x plan the sweep kernels would take for a box of nx planes and `tiles`
// tiles on `slots` resident workgroups (seg > 0: fixed segments, -1: equal
// segments, 0: auto), with its greedy-dispatch makespan in plane steps
struct XPlanInfo {
  int seg = 1, n1 = 0, r = 0, split = 0, nb2 = 0;
  double makespan = 0;
};
XPlanInfo describe_xplan(int64_t nx, int64_t tiles, int slots, int fill, int U, int seg);
// The `count` fixed x-segment lengths (>= U planes, any length: a tile's last
// piece may be short) with the smallest modelled makespan for `tiles` tiles of
// nx planes on `slots` workgroups, best first.  Equal segments (nx / k) leave
// slots idle or add a round when tiles x k is just above a multiple of the
// slots; e.g. 1022^3 fp32 pairs (225 tiles): 918-plane segments model 932
// plane-steps per slot against the x plan's 1024 (ideal 902).
std::vector<int> best_fixed_segments(int64_t nx, int64_t tiles, int slots, int fill, int U, int count);

// sweep schedules chosen by timing (StencilParams::tune): kernel, box, the
// winning z tile stride and spec-field-L value (-3 = the model's x plan, > 0
// fixed segments) and the measured ms of the winner and of the model's choice
struct TunedSchedule {
  std::string kernel;
  int64_t nx = 0, ny = 0, nz = 0;
  int zs = 0;  // z tile stride
  int L = 0;
  double ms = 0, ms_model = 0;
  int candidates = 0;
};
std::vector<TunedSchedule> tuned_schedules();
// fp32 lean kernel on packed pairs of z columns (stencil_tbp.hip; spec tlK:2:…)
void stencil_lean_pair(DType t, const StencilParams& p, const KernelSpec& k, void* stream);
bool lean_pair_supported(DType t, const KernelSpec& k);
// z tile stride of the pair kernel for a box (host-side choice, stencil_tbp.hip)
int pair_z_stride(int64_t nx, int64_t ny, int64_t nz, int K, int TY, int slots, int U, int L, int esize);
// Is the lean kernel variant that k resolves to for dtype t instantiated?
bool lean_supported(DType t, const KernelSpec& k);
// Any multi-step kind -> its kernel
void sweep(DType t, const StencilParams& p, const KernelSpec& k, void* stream);
void pack_box(DType t, const void* f, const Layout& L, const Box& b, void* buf, void* stream);
void unpack_box(DType t, void* f, const Layout& L, const Box& b, const void* buf, void* stream);
void copy_box(DType t, const void* src, const Layout& Ls, const Box& bs, void* dst,
              const Layout& Ld, const Box& bd, void* stream);
void check_convergence(DeviceState* s, int slot, void* stream, int count = 1, bool last_only = false);
// kernel of `blocks` one-wave workgroups spinning for `us` microseconds on the
// 100 MHz real-time clock (each holds a wave slot of one CU while it spins)
// fat: in RCCL's device-kernel footprint (256 threads, 140 VGPRs, 20 KB LDS)
void delay(double us, void* stream, int blocks = 1, bool fat = false);
void stamp(void* slot, void* stream);
void delay_since(const void* slot, double us, void* stream, int blocks = 1, bool fat = false);
// a phantom transfer paced at the wire rate (phantom_comm.cpp, --phantom-wire
// paced): 16-byte aligned, ticks of the 100 MHz clock per 16 bytes of one
// workgroup's share
struct PacedCopy {
  const void* src = nullptr;
  void* dst = nullptr;
  int64_t bytes = 0;
  double ticks_per16 = 0.0;
};
constexpr int kPacedMax = 8;  // transfers per launch
void paced_copy(const PacedCopy* xs, int n, int per, void* stream, bool fat = false);
// placement probe: out[b] = XCC << 8 | SE/SH/CU id of workgroup b (blocks x 64 threads)
void cu_probe(unsigned* out, int blocks, double us, void* stream);
// Device-side stream dependencies of per-stream hipGraphs (hip_backend.cpp):
// signal stores 1 into *slot (release, agent scope) once the work before it on
// its stream is complete; wait spins (acquire) until its slots are != 0.  A wait that
// outlasts `timeout_s` sets st->fault = 2 and st->done (every later sweep is
// then a no-op) and returns, so a broken dependency cannot hang the GPU.
void graph_signal(unsigned* slot, void* stream);
// (wait: on every one of `n` <= 4 slots)
void graph_wait(const unsigned* const* slots, int n, DeviceState* st, void* stream);
// Adds Σ|T - y| and the point count over `box` into s->error_sum/error_count.
// `scratch` must hold at least error_scratch_elems() doubles.
void error_accumulate(DType t, const void* f, const Layout& L, const Box& box,
                      const int64_t gstart[3], double hy, double* scratch, DeviceState* s,
                      void* stream);
int64_t error_scratch_elems();
// Fault injection (tests): write `value` at local owned point (i,j,k).
void poke(DType t, void* f, const Layout& L, int64_t i, int64_t j, int64_t k, double value,
          void* stream);
// Order-independent checksum (sum of bit patterns mod 2^64) of a box -> *out (device).
void box_bitsum(DType t, const void* f, const Layout& L, const Box& b, unsigned long long* out,
                void* stream);
// HBM calibration: kind 0 = 16 B/lane copy src->dst, 1 = 16 B/lane read of src.
void bandwidth_probe(int kind, const void* src, void* dst, int64_t bytes, int blocks, void* stream);
}  // namespace hip

namespace cpu {
void set_threads(int n);
void init_field(DType t, const InitParams& p);
void stencil(DType t, const StencilParams& p);
// Definition of the K-step sweep kernels: K single steps through two scratch
// fields (allocated by the caller, L.bytes() each).  Step s updates the box
// widened by K-1-s planes into [ux0, ux1) and accumulates into residual slot
// slot + s.
void stencil_multi(DType t, const StencilParams& p, int K, void* scratch0, void* scratch1);
void pack_box(DType t, const void* f, const Layout& L, const Box& b, void* buf);
void unpack_box(DType t, void* f, const Layout& L, const Box& b, const void* buf);
void copy_box(DType t, const void* src, const Layout& Ls, const Box& bs, void* dst,
              const Layout& Ld, const Box& bd);
void check_convergence(DeviceState* s, int slot);
void error_accumulate(DType t, const void* f, const Layout& L, const Box& box,
                      const int64_t gstart[3], double hy, DeviceState* s);
void poke(DType t, void* f, const Layout& L, int64_t i, int64_t j, int64_t k, double value);
unsigned long long box_bitsum(DType t, const void* f, const Layout& L, const Box& b);
}  // namespace cpu

// Shared scalar logic of the convergence check (heat3D.cu:1026-1073 with the
// survey's fixes: global norm, global max residual).  Used verbatim by the
// CPU backend and mirrored by the single-thread HIP kernel.
// FTCS 7-point update of heat3D.cu:128-131,
//   T + Dx*(T[i+1] - 2T + T[i-1]) + Dy*(...) + Dz*(...),
// evaluated the way nvcc compiles it for the reference's GPU kernel (default
// -fmad=true): left to right, every "acc + D*a" contracted to one fused
// multiply-add, and "T[i+1] - 2T" to fma(-2, T, T[i+1]) (2T is exact, so that
// one is the same value either way).  Written with explicit fused operations
// so that the CPU backend (libm fma, correctly rounded) and every gfx950
// kernel (v_fma_f64 / v_fma_f32) produce bitwise identical fields.
H3D_HD inline double h3d_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
H3D_HD inline float h3d_fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
template <typename Real>
H3D_HD inline Real ftcs_update(Real c, Real xm, Real xp, Real ym, Real yp, Real zm, Real zp, Real Dx,
                               Real Dy, Real Dz) {
  const Real ax = h3d_fma(Real(-2), c, xp) + xm;
  const Real ay = h3d_fma(Real(-2), c, yp) + ym;
  const Real az = h3d_fma(Real(-2), c, zp) + zm;
  return h3d_fma(Dz, az, h3d_fma(Dy, ay, h3d_fma(Dx, ax, c)));
}

// Residual term of one point, |T^{n+1} - T^n|, taken in the field's
// precision as the reference takes fabs(T - T0) in its field type
// (heat3D.cu:1030-1033), then widened (exactly) to double for the max.  In
// fp32 that is one subtraction instead of two conversions and a double
// subtraction; in fp64 it is the same value as before.
H3D_HD inline double resid_abs(double nv, double c) { return __builtin_fabs(nv - c); }
H3D_HD inline double resid_abs(float nv, float c) { return (double)__builtin_fabsf(nv - c); }
H3D_HD inline float resid_abs_r(float nv, float c) { return __builtin_fabsf(nv - c); }
H3D_HD inline double resid_abs_r(double nv, double c) { return __builtin_fabs(nv - c); }

H3D_HD inline void check_convergence_scalar(DeviceState* s, double r) {
  const int64_t t = s->iter;
  if (s->hist_cap > 0) s->hist[t % s->hist_cap] = r;
  if (!s->done) {
    s->last_residual = r;
    if (!(r == r) || r > 1.7976931348623157e308) {  // NaN or Inf
      s->fault = 1;
      s->done = 1;
      s->conv_iter = t;
    } else {
      if (t == 0 && r != 0.0) s->norm = r;
      if (r / s->norm < s->eps) {
        s->done = 1;
        s->conv_iter = t;
      }
    }
  }
  s->iter = t + 1;
}

}  // namespace heat3d
