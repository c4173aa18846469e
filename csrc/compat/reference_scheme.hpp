// heat3d-mi355x — emulation of the reference's own domain-decomposition scheme.
//
// The production solver (runtime/solver.hpp) uses non-overlapping ownership
// with a ghost shell, a global norm and a global max residual, which makes
// every result bitwise independent of the process grid.  The
// reference instead:
//
//   * splits the N vertices into equal chunks c = (N-1)/dims + 1 that SHARE
//     one plane with each neighbour (heat3D.cu:373-389), legal only when
//     (N-1) % dims == 0;
//   * updates the chunk interior [1, c-2]^3 from the T0 snapshot, then every
//     shared face with the neighbour's plane c-2 / 1 as halo
//     (heat3D.cu:757-853);
//   * extrapolates the 12 shared edges linearly from the new values
//     (heat3D.cu:859-943) and averages the 8 shared corners
//     (heat3D.cu:947-1011);
//   * takes each rank's residual over its chunk interior, normalises it by the
//     rank's OWN iteration-0 residual and stops when ANY rank's ratio < eps
//     (MAX of break flags, heat3D.cu:1016-1073);
//   * prints rank 0's local mean |T - y| as the "L2-norm error"
//     (heat3D.cu:1093-1106).
//
// ReferenceScheme runs all ranks of that scheme in one process (host, OpenMP),
// with the reference's per-cell expression (kernels.hpp ftcs_update),
// so its iteration counts can be checked against SURVEY.md App. B.3b
// (27^3, eps 1e-5: 2513 / 2511 / 2543 / 2615 iterations for 1x1x1 / 2x1x1 /
// 2x2x1 / 2x2x2).  It is the `--scheme reference` mode of the CLI; it exists
// for parity studies, not for speed.
#pragma once

#include <array>
#include <cstdint>
#include <string>
#include <vector>

#include "../core/config.hpp"

namespace heat3d {

struct ReferenceSchemeResult {
  bool converged = false;
  int64_t conv_iter = -1;     // 0-based break iteration (finalNumIterations)
  int64_t iterations = 0;     // time steps performed
  double seconds = 0.0;
  double norm_rank0 = 1.0;    // rank 0's normalisation (its iteration-0 residual)
  double error_rank0 = 0.0;   // what the reference prints (rank 0 local mean |T - y|)
  double error_global = 0.0;  // true mean |T - y| over the global interior (shared planes once)
  double last_residual_rank0 = 0.0;
};

class ReferenceScheme {
 public:
  ReferenceScheme(const int64_t N[3], const std::array<int, 3>& dims);
  const std::array<int64_t, 3>& chunk() const { return c_; }
  int ranks() const { return (int)ranks_.size(); }
  ReferenceSchemeResult run(int64_t iter_max, double eps, int verbose = 0);
  // Global N0*N1*N2 field (z fastest); on shared planes the highest rank wins
  // (the reference's Tecplot zones duplicate them).
  std::vector<double> gather() const;
  // Tecplot output with one zone per rank over its whole chunk (shared planes
  // duplicated), zone titles "0" as the reference printed.
  void write_tecplot(const std::string& path) const;

 private:
  struct Rank {
    std::array<int, 3> coords;
    std::array<int, 6> nb;  // neighbour rank per Face, -1 = physical boundary
    std::vector<double> T, T0;
  };
  int64_t idx(int64_t i, int64_t j, int64_t k) const { return (i * c_[1] + j) * c_[2] + k; }
  void step(int64_t t);
  double residual(const Rank& r) const;

  std::array<int64_t, 3> N_;
  std::array<int64_t, 3> c_;
  std::array<int, 3> dims_;
  Physics phys_;
  std::vector<Rank> ranks_;
};

}  // namespace heat3d
