// heat3d-mi355x — local array geometry and device-resident solver state.
//
// One subdomain's field is a single contiguous allocation (no double*** pointer
// tables: reference heat3D.cu:60-111 / SURVEY.md C5, C15) holding the owned
// block plus a one-cell ghost shell (two planes deep in x when the 2-step
// temporally blocked schedule exchanges deep x halos), z fastest (the reference's T[i][j][k]
// order, heat3D.cu:394-406).  Rows are padded so that the first owned z point
// of every row is 128-byte aligned; that lets the stencil kernels issue
// 16-byte vector loads/stores on gfx950 without realignment.  All indices are
// 64-bit (4096^3 > 2^32 points).
#pragma once

#include <cstddef>
#include <cstdint>

#include "../core/common.hpp"

namespace heat3d {

struct Layout {
  int64_t n[3] = {0, 0, 0};  // owned extents
  int64_t sx = 0, sy = 0;    // element strides of x planes and y rows (z stride 1)
  int64_t zoff = 0;          // offset of owned k = 0 inside a row
  int64_t origin = 0;        // element index of owned (0,0,0)
  int64_t elems = 0;         // allocation length in elements (includes tail pad)
  int64_t esize = 8;
  int64_t gx = 1;            // ghost planes on each x side (K with deep halos)
  int64_t gy = 1, gz = 1;    // ghost rows / columns on each y / z side

  // i in [-gx, n0 + gx - 1], j in [-gy, n1 + gy - 1], k in [-gz, n2 + gz - 1]
  H3D_HD inline int64_t index(int64_t i, int64_t j, int64_t k) const {
    return origin + i * sx + j * sy + k;
  }
  // Alignment in elements used for the row offset / pitch.
  static int64_t align_elems(int64_t esize) { return 128 / esize; }
  static Layout make(const int64_t n[3], int64_t esize, int64_t gx = 1, int64_t gy = 1, int64_t gz = 1) {
    Layout L;
    L.gx = gx;
    L.gy = gy;
    L.gz = gz;
    for (int a = 0; a < 3; ++a) L.n[a] = n[a];
    L.esize = esize;
    const int64_t A = align_elems(esize);
    L.zoff = A;                                  // ghost k = -1 lives at A - 1
    if (gz > A) L.zoff = (gz + A - 1) / A * A;   // deep z ghosts (never with K <= 6)
    const int64_t need = L.zoff + n[2] + gz;     // through ghost k = nz + gz - 1
    L.sy = ((need + A - 1) / A) * A;
    // break power-of-two row pitches (HBM channel / cache-set aliasing)
    if ((L.sy & (L.sy - 1)) == 0) L.sy += A;
    L.sx = (n[1] + 2 * gy) * L.sy;
    L.origin = gx * L.sx + gy * L.sy + L.zoff;
    // tail pad: kernels may over-read up to one 256-wide z tile past a row end
    L.elems = (n[0] + 2 * gx) * L.sx + 2 * L.sy + 1024;
    return L;
  }
  // element offset of the start of x plane i (its ghost row j = -gy)
  H3D_HD inline int64_t plane_offset(int64_t i) const { return (gx + i) * sx; }
  std::size_t bytes() const { return static_cast<std::size_t>(elems * esize); }
};

// Device-resident convergence state.  One per process, shared by every local
// subdomain.  The residual accumulators hold the IEEE bit pattern of a
// non-negative double so that an unsigned 64-bit atomic max (and an RCCL
// uint64 max all-reduce) is an exact max of the doubles.
constexpr int kResidualSlots = 8;
// K-step sweep kernels: bit of the store-policy template argument (spec
// field 7) that computes only the last step's residual (fused_check_tail)
constexpr int kResidualLastOnly = 64;

struct DeviceState {
  // max |T^{n+1}-T^n| accumulators: single steps use slot t & 1, a K-step
  // temporally blocked sweep uses slots 0..K-1
  unsigned long long residual[kResidualSlots];
  double norm;                     // residual of iteration 0 (heat3D.cu:1026-1032)
  double eps;
  double last_residual;
  double error_sum;                // Σ|T - y| over owned points (error report)
  double error_count;
  int64_t iter;                    // iterations checked so far (next index)
  int64_t conv_iter;               // 0-based converged iteration, -1 until then
  int32_t done;                    // convergence reached (or fault): stencils early-exit
  int32_t fault;                   // 1 = NaN/Inf residual detected, 2 = a graph wait timed out
  // device-side cross-stream waits of per-stream hipGraphs give up after this
  // many 100 MHz ticks (read at every wait: the start-up canary shortens it)
  uint64_t wait_ticks;
  // sweeps with a fused convergence check (StencilParams::fuse_check): the
  // workgroups that finished the current sweep; the last one runs the check
  // and resets it to 0
  uint32_t sweep_tickets;
  // a sweep that computed only its last step's residual (kResidualLastOnly)
  // set done: the first converged (or faulted) iteration is one of its last
  // `coarse` iterations, conv_iter <= that; Solver::resolve_coarse finds it
  uint32_t coarse;
  int64_t hist_cap;                // residual history ring capacity
  double hist[1024];               // residual history ring (index = iter % cap)
};

// Residual accumulator initial value: the reference starts the max at
// numeric_limits<double>::min() (heat3D.cu:1019).
constexpr unsigned long long kResidualInitBits = 0x0010000000000000ULL;  // DBL_MIN

}  // namespace heat3d
