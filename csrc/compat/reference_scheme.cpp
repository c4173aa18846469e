// heat3d-mi355x — the reference's shared-plane decomposition scheme (see
// reference_scheme.hpp for what is emulated and why).
#include "reference_scheme.hpp"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <limits>

#include "../core/decomp.hpp"
#include "../io/io.hpp"
#include "../kernels/kernels.hpp"

#pragma STDC FP_CONTRACT OFF

namespace heat3d {

namespace {
constexpr int L = 0, Rt = 1, B = 2, Tp = 3, Bk = 4, Fr = 5;  // Face order LEFT..FRONT
}

ReferenceScheme::ReferenceScheme(const int64_t N[3], const std::array<int, 3>& dims) : dims_(dims) {
  for (int a = 0; a < 3; ++a) {
    N_[a] = N[a];
    // heat3D.cu:375-380: the reference asserts an exact split of N-1 cells
    HEAT3D_CHECK(dims[a] >= 1 && (N[a] - 1) % dims[a] == 0,
                 "reference scheme needs (N-1) % dims == 0 on every axis (N" << a << "=" << N[a] << ", dims="
                                                                            << dims[a] << ")");
    c_[a] = (N[a] - 1) / dims[a] + 1;
    HEAT3D_CHECK(c_[a] >= 3, "reference scheme: chunk of " << c_[a] << " points on axis " << a);
  }
  phys_ = Physics::make(N[0], N[1], N[2]);
  Topology topo;
  topo.dims = dims;
  const int P = topo.size();
  ranks_.resize(P);
  const int64_t vol = c_[0] * c_[1] * c_[2];
  for (int r = 0; r < P; ++r) {
    Rank& rk = ranks_[r];
    rk.coords = topo.coords(r);
    for (int f = 0; f < kNumFaces; ++f) rk.nb[f] = topo.neighbor(r, static_cast<Face>(f));
    rk.T.assign(vol, 0.0);
    // initial / boundary condition on the physical faces (heat3D.cu:414-453):
    // the analytic Dirichlet values of the global vertex
    for (int64_t i = 0; i < c_[0]; ++i)
      for (int64_t j = 0; j < c_[1]; ++j)
        for (int64_t k = 0; k < c_[2]; ++k) {
          const int64_t g[3] = {rk.coords[0] * (c_[0] - 1) + i, rk.coords[1] * (c_[1] - 1) + j,
                                rk.coords[2] * (c_[2] - 1) + k};
          const bool phys = (i == 0 && rk.nb[L] < 0) || (i == c_[0] - 1 && rk.nb[Rt] < 0) ||
                            (j == 0 && rk.nb[B] < 0) || (j == c_[1] - 1 && rk.nb[Tp] < 0) ||
                            (k == 0 && rk.nb[Bk] < 0) || (k == c_[2] - 1 && rk.nb[Fr] < 0);
          if (phys) rk.T[idx(i, j, k)] = boundary_value(g[0], g[1], g[2], N_.data(), phys_.h);
        }
    rk.T0 = rk.T;
  }
}

// One time step of every rank (heat3D.cu:543-1011, GPU build with a working
// interior update).  Expression order per cell as heat3D.cu:128-131 / 767-770.
void ReferenceScheme::step(int64_t) {
  const double Dx = phys_.D[0], Dy = phys_.D[1], Dz = phys_.D[2];
  const int64_t cx = c_[0], cy = c_[1], cz = c_[2];
  const int64_t sx = cy * cz, sy = cz;
  auto upd = [&](double c, double xm, double xp, double ym, double yp, double zm, double zp) {
    return ftcs_update<double>(c, xm, xp, ym, yp, zm, zp, Dx, Dy, Dz);
  };
  for (auto& rk : ranks_) rk.T0 = rk.T;  // heat3D.cu:543-548
  const int P = (int)ranks_.size();
#pragma omp parallel for schedule(static)
  for (int r = 0; r < P; ++r) {
    Rank& rk = ranks_[r];
    const double* t0 = rk.T0.data();
    double* t = rk.T.data();
    // chunk interior
    for (int64_t i = 1; i < cx - 1; ++i)
      for (int64_t j = 1; j < cy - 1; ++j)
        for (int64_t k = 1; k < cz - 1; ++k) {
          const int64_t p = idx(i, j, k);
          t[p] = upd(t0[p], t0[p - sx], t0[p + sx], t0[p - sy], t0[p + sy], t0[p - 1], t0[p + 1]);
        }
    // shared faces: the neighbour's second plane is the halo (heat3D.cu:757-853)
    auto nbT0 = [&](int f) { return ranks_[rk.nb[f]].T0.data(); };
    if (rk.nb[L] >= 0) {
      const double* h = nbT0(L);
      for (int64_t j = 1; j < cy - 1; ++j)
        for (int64_t k = 1; k < cz - 1; ++k) {
          const int64_t p = idx(0, j, k);
          t[p] = upd(t0[p], h[idx(cx - 2, j, k)], t0[p + sx], t0[p - sy], t0[p + sy], t0[p - 1], t0[p + 1]);
        }
    }
    if (rk.nb[Rt] >= 0) {
      const double* h = nbT0(Rt);
      for (int64_t j = 1; j < cy - 1; ++j)
        for (int64_t k = 1; k < cz - 1; ++k) {
          const int64_t p = idx(cx - 1, j, k);
          t[p] = upd(t0[p], t0[p - sx], h[idx(1, j, k)], t0[p - sy], t0[p + sy], t0[p - 1], t0[p + 1]);
        }
    }
    if (rk.nb[B] >= 0) {
      const double* h = nbT0(B);
      for (int64_t i = 1; i < cx - 1; ++i)
        for (int64_t k = 1; k < cz - 1; ++k) {
          const int64_t p = idx(i, 0, k);
          t[p] = upd(t0[p], t0[p - sx], t0[p + sx], h[idx(i, cy - 2, k)], t0[p + sy], t0[p - 1], t0[p + 1]);
        }
    }
    if (rk.nb[Tp] >= 0) {
      const double* h = nbT0(Tp);
      for (int64_t i = 1; i < cx - 1; ++i)
        for (int64_t k = 1; k < cz - 1; ++k) {
          const int64_t p = idx(i, cy - 1, k);
          t[p] = upd(t0[p], t0[p - sx], t0[p + sx], t0[p - sy], h[idx(i, 1, k)], t0[p - 1], t0[p + 1]);
        }
    }
    if (rk.nb[Bk] >= 0) {
      const double* h = nbT0(Bk);
      for (int64_t i = 1; i < cx - 1; ++i)
        for (int64_t j = 1; j < cy - 1; ++j) {
          const int64_t p = idx(i, j, 0);
          t[p] = upd(t0[p], t0[p - sx], t0[p + sx], t0[p - sy], t0[p + sy], h[idx(i, j, cz - 2)], t0[p + 1]);
        }
    }
    if (rk.nb[Fr] >= 0) {
      const double* h = nbT0(Fr);
      for (int64_t i = 1; i < cx - 1; ++i)
        for (int64_t j = 1; j < cy - 1; ++j) {
          const int64_t p = idx(i, j, cz - 1);
          t[p] = upd(t0[p], t0[p - sx], t0[p + sx], t0[p - sy], t0[p + sy], t0[p - 1], h[idx(i, j, 1)]);
        }
    }
    // shared edges: linear extrapolation from the new values (heat3D.cu:859-943)
    const bool n[6] = {rk.nb[L] >= 0, rk.nb[Rt] >= 0, rk.nb[B] >= 0, rk.nb[Tp] >= 0, rk.nb[Bk] >= 0, rk.nb[Fr] >= 0};
    for (int xs = 0; xs < 2; ++xs) {  // LEFT / RIGHT edges, extrapolated along x
      if (!n[xs]) continue;
      const int64_t i = xs ? cx - 1 : 0, d = xs ? -sx : sx;
      for (int ys = 0; ys < 2; ++ys) {  // with BOTTOM / TOP
        if (!n[2 + ys]) continue;
        const int64_t j = ys ? cy - 1 : 0;
        for (int64_t k = 1; k < cz - 1; ++k) {
          const int64_t p = idx(i, j, k);
          t[p] = 2.0 * t[p + d] - t[p + 2 * d];
        }
      }
      for (int zs = 0; zs < 2; ++zs) {  // with BACK / FRONT
        if (!n[4 + zs]) continue;
        const int64_t k = zs ? cz - 1 : 0;
        for (int64_t j = 1; j < cy - 1; ++j) {
          const int64_t p = idx(i, j, k);
          t[p] = 2.0 * t[p + d] - t[p + 2 * d];
        }
      }
    }
    for (int zs = 0; zs < 2; ++zs) {  // BACK / FRONT with BOTTOM / TOP, extrapolated along z
      if (!n[4 + zs]) continue;
      const int64_t k = zs ? cz - 1 : 0, d = zs ? -1 : 1;
      for (int ys = 0; ys < 2; ++ys) {
        if (!n[2 + ys]) continue;
        const int64_t j = ys ? cy - 1 : 0;
        for (int64_t i = 1; i < cx - 1; ++i) {
          const int64_t p = idx(i, j, k);
          t[p] = 2.0 * t[p + d] - t[p + 2 * d];
        }
      }
    }
    // shared corners: average of the three inward neighbours (heat3D.cu:947-1011)
    for (int xs = 0; xs < 2; ++xs)
      for (int ys = 0; ys < 2; ++ys)
        for (int zs = 0; zs < 2; ++zs) {
          if (!(n[xs] && n[2 + ys] && n[4 + zs])) continue;
          const int64_t p = idx(xs ? cx - 1 : 0, ys ? cy - 1 : 0, zs ? cz - 1 : 0);
          t[p] = 1.0 / 3.0 * ((t[p + (xs ? -sx : sx)] + t[p + (ys ? -sy : sy)]) + t[p + (zs ? -1 : 1)]);
        }
  }
}

// max |T - T0| over the chunk interior, starting from DBL_MIN (heat3D.cu:1016-1024)
double ReferenceScheme::residual(const Rank& rk) const {
  double res = std::numeric_limits<double>::min();
  for (int64_t i = 1; i < c_[0] - 1; ++i)
    for (int64_t j = 1; j < c_[1] - 1; ++j)
      for (int64_t k = 1; k < c_[2] - 1; ++k) {
        const int64_t p = idx(i, j, k);
        const double d = std::fabs(rk.T[p] - rk.T0[p]);
        if (d > res) res = d;
      }
  return res;
}

ReferenceSchemeResult ReferenceScheme::run(int64_t iter_max, double eps, int verbose) {
  ReferenceSchemeResult out;
  const int P = (int)ranks_.size();
  std::vector<double> norm(P, 1.0);  // heat3D.cu:323-324
  const auto t0 = std::chrono::steady_clock::now();
  for (int64_t time = 0; time < iter_max; ++time) {
    step(time);
    bool any = false;  // MPI_Iallreduce(MAX) of the break flags (heat3D.cu:1062)
    for (int r = 0; r < P; ++r) {
      const double res = residual(ranks_[r]);
      if (time == 0 && res != 0.0) norm[r] = res;  // local norm (heat3D.cu:1030-1032)
      if (r == 0) out.last_residual_rank0 = res;
      if (res / norm[r] < eps) any = true;
    }
    if (verbose > 0 && time % verbose == 0)
      std::printf("iteration %lld residual %.6e\n", (long long)time, out.last_residual_rank0 / norm[0]);
    out.iterations = time + 1;
    if (any) {
      out.converged = true;
      out.conv_iter = time;
      break;
    }
  }
  out.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  out.norm_rank0 = norm[0];
  // error vs the analytic steady state T = y (heat3D.cu:1093-1101)
  for (int r = 0; r < P; ++r) {
    const Rank& rk = ranks_[r];
    double error = 0.0;
    for (int64_t k = 1; k < c_[2] - 1; ++k)
      for (int64_t j = 1; j < c_[1] - 1; ++j)
        for (int64_t i = 1; i < c_[0] - 1; ++i) {
          const double y = (double)(rk.coords[1] * (c_[1] - 1) + j) * phys_.h[1];
          error += std::sqrt(std::pow(rk.T[idx(i, j, k)] - y, 2.0));
        }
    error /= (double)((c_[0] - 2) * (c_[1] - 2) * (c_[2] - 2));
    if (r == 0) out.error_rank0 = error;
  }
  // what the reference meant to report: the global mean
  const std::vector<double> g = gather();
  double sum = 0.0;
  for (int64_t i = 1; i < N_[0] - 1; ++i)
    for (int64_t j = 1; j < N_[1] - 1; ++j) {
      const double y = (double)j * phys_.h[1];
      for (int64_t k = 1; k < N_[2] - 1; ++k) sum += std::fabs(g[(std::size_t)((i * N_[1] + j) * N_[2] + k)] - y);
    }
  out.error_global = sum / (double)((N_[0] - 2) * (N_[1] - 2) * (N_[2] - 2));
  return out;
}

std::vector<double> ReferenceScheme::gather() const {
  std::vector<double> g((std::size_t)(N_[0] * N_[1] * N_[2]), 0.0);
  for (const auto& rk : ranks_)
    for (int64_t i = 0; i < c_[0]; ++i)
      for (int64_t j = 0; j < c_[1]; ++j)
        for (int64_t k = 0; k < c_[2]; ++k) {
          const int64_t gi = rk.coords[0] * (c_[0] - 1) + i, gj = rk.coords[1] * (c_[1] - 1) + j,
                        gk = rk.coords[2] * (c_[2] - 1) + k;
          g[(std::size_t)((gi * N_[1] + gj) * N_[2] + gk)] = rk.T[idx(i, j, k)];
        }
  return g;
}

void ReferenceScheme::write_tecplot(const std::string& path) const {
  std::vector<io::Zone> zones;
  for (int r = 0; r < (int)ranks_.size(); ++r) {
    io::Zone z;
    z.rank = r;
    z.title = 0;  // heat3D.cu:1148 printed `rank` (0) for every zone
    for (int a = 0; a < 3; ++a) {
      z.lo[a] = ranks_[r].coords[a] * (c_[a] - 1);
      z.hi[a] = z.lo[a] + c_[a];
    }
    zones.push_back(z);
  }
  io::write_tecplot(path, gather(), N_.data(), phys_.h, zones, ranks_.size() > 1);
}

}  // namespace heat3d
