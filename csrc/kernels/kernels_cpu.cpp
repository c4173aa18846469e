// heat3d-mi355x — OpenMP host kernels (CPU backend and test oracle).
//
// This is the "64^3 fp64 CPU Jacobi reference" of BASELINE.json config 1 and
// the bitwise oracle for the gfx950 kernels.  Unlike the reference CPU twin
// (heat3D.cpp:606-612, whose interior update block is empty — SURVEY A9) it
// updates every owned point.  Compile with -ffp-contract=off (the update's
// fused multiply-adds are explicit, kernels.hpp ftcs_update).
#include <omp.h>

#include <cmath>
#include <cstring>

#include "cpu_rows.hpp"
#include "kernels.hpp"

namespace heat3d {
namespace cpu {

void set_threads(int n) {
  if (n > 0) omp_set_num_threads(n);
}

// Boxes below this many points run on the calling thread: the boundary pieces
// and deep-halo slabs of small decomposed grids are a few hundred points, and a
// parallel region per piece costs more than the piece (badly so when the host
// is oversubscribed, e.g. several ranks or test workers per core).
static inline bool omp_worth(int64_t points) { return points >= (int64_t(1) << 15); }

template <typename Real>
static void init_t(const InitParams& p) {
  Real* f = static_cast<Real*>(p.field);
  const Layout& L = p.L;
  // every ghost plane (deep x halos included) gets its Dirichlet ghost rows
#pragma omp parallel for collapse(2) schedule(static) if (omp_worth(static_cast<int64_t>(L.elems)))
  for (int64_t i = -L.gx; i < L.n[0] + L.gx; ++i)
    for (int64_t j = -L.gy; j < L.n[1] + L.gy; ++j) {
      const int64_t gi = p.gstart[0] + i, gj = p.gstart[1] + j;
      // deep ghosts beyond the domain stay 0 (never read by an update)
      if (gi < 0 || gi >= p.N[0] || gj < 0 || gj >= p.N[1]) continue;
      for (int64_t k = -L.gz; k < L.n[2] + L.gz; ++k) {
        const int64_t gk = p.gstart[2] + k;
        if (gk < 0 || gk >= p.N[2]) continue;
        const bool phys = gi == 0 || gi == p.N[0] - 1 || gj == 0 || gj == p.N[1] - 1 ||
                          gk == 0 || gk == p.N[2] - 1;
        f[L.index(i, j, k)] =
            phys ? static_cast<Real>(boundary_value(gi, gj, gk, p.N, p.h)) : Real(0);
      }
    }
}

void init_field(DType t, const InitParams& p) {
  // zero the whole allocation first (padding included) so that over-reads of
  // padding by vector kernels never see uninitialised bytes
  std::memset(p.field, 0, p.L.bytes());
  if (t == DType::F64) init_t<double>(p);
  else init_t<float>(p);
}

template <typename Real>
static void stencil_t(const StencilParams& p) {
  if (p.state && p.state->done) return;
  const Real* __restrict in = static_cast<const Real*>(p.in);
  Real* __restrict out = static_cast<Real*>(p.out);
  const Layout& L = p.L;
  const Box& b = p.box;
  if (b.empty()) return;
  const Real Dx = static_cast<Real>(p.D[0]), Dy = static_cast<Real>(p.D[1]),
             Dz = static_cast<Real>(p.D[2]);
  const int64_t sx = L.sx, sy = L.sy;
  // max |dT| reduced on the IEEE bit patterns of the non-negative doubles so
  // that a NaN (bits above +Inf) propagates to the convergence check
  unsigned long long resbits = 0;
  const auto rowfn = [] {
    if constexpr (sizeof(Real) == 8) return cpu_row_kernels().f64;
    else return cpu_row_kernels().f32;
  }();
  const int64_t nk = b.extent(2);
#pragma omp parallel for collapse(2) schedule(static) reduction(max : resbits) if (omp_worth(b.volume()))
  for (int64_t i = b.lo[0]; i < b.hi[0]; ++i)
    for (int64_t j = b.lo[1]; j < b.hi[1]; ++j) {
      const int64_t c = L.index(i, j, b.lo[2]);
      // heat3D.cu:128-131 with nvcc's FMA contraction (kernels.hpp ftcs_update)
      const double lres = nk > 0 ? rowfn(in + c, out + c, nk, sx, sy, Dx, Dy, Dz) : 0.0;
      unsigned long long bits;
      std::memcpy(&bits, &lres, sizeof(bits));
      resbits = bits > resbits ? bits : resbits;
    }
  if (p.state && p.residual) {
    unsigned long long* slot = &p.state->residual[p.slot];
    if (resbits > *slot) *slot = resbits;
  }
}

void stencil_multi(DType t, const StencilParams& p, int K, void* scratch0, void* scratch1) {
  if (p.state && p.state->done) return;
  void* scratch[2] = {scratch0, scratch1};
  std::memcpy(scratch[0], p.in, p.L.bytes());
  std::memcpy(scratch[1], p.in, p.L.bytes());
  const int64_t* u[3] = {p.ux, p.uy, p.uz};
  for (int s = 0; s < K; ++s) {
    StencilParams a = p;
    a.in = s == 0 ? p.in : scratch[(s - 1) & 1];
    a.out = s == K - 1 ? p.out : scratch[s & 1];
    a.slot = p.slot + s;
    // stage s computes the box widened by K-1-s into the deep halos (the
    // update range u of each axis), so that stage K-1 covers the box
    for (int ax = 0; ax < 3; ++ax)
      if (u[ax][1] >= u[ax][0]) {
        const int64_t w = K - 1 - s;
        a.box.lo[ax] = std::max(p.box.lo[ax] - w, u[ax][0]);
        a.box.hi[ax] = std::min(p.box.hi[ax] + w, u[ax][1]);
      }
    stencil(t, a);
  }
}

void stencil(DType t, const StencilParams& p) {
  if (t == DType::F64) stencil_t<double>(p);
  else stencil_t<float>(p);
}

template <typename Real>
static void pack_t(const Real* f, const Layout& L, const Box& b, Real* buf) {
  const int64_t ey = b.extent(1), ez = b.extent(2);
#pragma omp parallel for collapse(2) schedule(static) if (omp_worth(b.volume()))
  for (int64_t i = b.lo[0]; i < b.hi[0]; ++i)
    for (int64_t j = b.lo[1]; j < b.hi[1]; ++j) {
      const int64_t o = ((i - b.lo[0]) * ey + (j - b.lo[1])) * ez;
      std::memcpy(buf + o, f + L.index(i, j, b.lo[2]), sizeof(Real) * ez);
    }
}

template <typename Real>
static void unpack_t(Real* f, const Layout& L, const Box& b, const Real* buf) {
  const int64_t ey = b.extent(1), ez = b.extent(2);
#pragma omp parallel for collapse(2) schedule(static) if (omp_worth(b.volume()))
  for (int64_t i = b.lo[0]; i < b.hi[0]; ++i)
    for (int64_t j = b.lo[1]; j < b.hi[1]; ++j) {
      const int64_t o = ((i - b.lo[0]) * ey + (j - b.lo[1])) * ez;
      std::memcpy(f + L.index(i, j, b.lo[2]), buf + o, sizeof(Real) * ez);
    }
}

void pack_box(DType t, const void* f, const Layout& L, const Box& b, void* buf) {
  if (b.empty()) return;
  if (t == DType::F64) pack_t(static_cast<const double*>(f), L, b, static_cast<double*>(buf));
  else pack_t(static_cast<const float*>(f), L, b, static_cast<float*>(buf));
}

void unpack_box(DType t, void* f, const Layout& L, const Box& b, const void* buf) {
  if (b.empty()) return;
  if (t == DType::F64) unpack_t(static_cast<double*>(f), L, b, static_cast<const double*>(buf));
  else unpack_t(static_cast<float*>(f), L, b, static_cast<const float*>(buf));
}

template <typename Real>
static void copy_t(const Real* src, const Layout& Ls, const Box& bs, Real* dst, const Layout& Ld,
                   const Box& bd) {
  const int64_t ex = bs.extent(0), ey = bs.extent(1), ez = bs.extent(2);
#pragma omp parallel for collapse(2) schedule(static) if (omp_worth(bs.volume()))
  for (int64_t i = 0; i < ex; ++i)
    for (int64_t j = 0; j < ey; ++j)
      std::memcpy(dst + Ld.index(bd.lo[0] + i, bd.lo[1] + j, bd.lo[2]),
                  src + Ls.index(bs.lo[0] + i, bs.lo[1] + j, bs.lo[2]), sizeof(Real) * ez);
}

void copy_box(DType t, const void* src, const Layout& Ls, const Box& bs, void* dst,
              const Layout& Ld, const Box& bd) {
  HEAT3D_CHECK(bs.extent(0) == bd.extent(0) && bs.extent(1) == bd.extent(1) &&
                   bs.extent(2) == bd.extent(2),
               "copy_box extent mismatch " << bs.str() << " vs " << bd.str());
  if (bs.empty()) return;
  if (t == DType::F64)
    copy_t(static_cast<const double*>(src), Ls, bs, static_cast<double*>(dst), Ld, bd);
  else
    copy_t(static_cast<const float*>(src), Ls, bs, static_cast<float*>(dst), Ld, bd);
}

void check_convergence(DeviceState* s, int slot) {
  double r;
  std::memcpy(&r, &s->residual[slot], sizeof(r));
  check_convergence_scalar(s, r);
  s->residual[slot] = kResidualInitBits;
}

template <typename Real>
static void error_t(const Real* f, const Layout& L, const Box& b, const int64_t gstart[3],
                    double hy, DeviceState* s) {
  double sum = 0.0;
  // fixed-order reduction over x planes -> deterministic for a given thread count
#pragma omp parallel for schedule(static) reduction(+ : sum)
  for (int64_t i = b.lo[0]; i < b.hi[0]; ++i) {
    double ps = 0.0;
    for (int64_t j = b.lo[1]; j < b.hi[1]; ++j) {
      const double y = static_cast<double>(gstart[1] + j) * hy;
      const Real* row = f + L.index(i, j, 0);
      for (int64_t k = b.lo[2]; k < b.hi[2]; ++k) ps += std::fabs(static_cast<double>(row[k]) - y);
    }
    sum += ps;
  }
  s->error_sum += sum;
  s->error_count += static_cast<double>(b.volume());
}

void error_accumulate(DType t, const void* f, const Layout& L, const Box& box,
                      const int64_t gstart[3], double hy, DeviceState* s) {
  if (box.empty()) return;
  if (t == DType::F64) error_t(static_cast<const double*>(f), L, box, gstart, hy, s);
  else error_t(static_cast<const float*>(f), L, box, gstart, hy, s);
}

unsigned long long box_bitsum(DType t, const void* f, const Layout& L, const Box& b) {
  unsigned long long acc = 0;
  for (int64_t i = b.lo[0]; i < b.hi[0]; ++i)
    for (int64_t j = b.lo[1]; j < b.hi[1]; ++j)
      for (int64_t k = b.lo[2]; k < b.hi[2]; ++k) {
        const int64_t q = L.index(i, j, k);
        if (t == DType::F64) {
          unsigned long long u;
          std::memcpy(&u, static_cast<const double*>(f) + q, 8);
          acc += u;
        } else {
          unsigned u;
          std::memcpy(&u, static_cast<const float*>(f) + q, 4);
          acc += u;
        }
      }
  return acc;
}

void poke(DType t, void* f, const Layout& L, int64_t i, int64_t j, int64_t k, double value) {
  if (t == DType::F64) static_cast<double*>(f)[L.index(i, j, k)] = value;
  else static_cast<float*>(f)[L.index(i, j, k)] = static_cast<float>(value);
}

}  // namespace cpu
}  // namespace heat3d
