// heat3d-mi355x — C++ unit tests (ctest; CPU only).
// Topology clone vs MPI_Dims_create results, decomposition tiling, layout
// alignment, CPU-backend goldens and LocalComm
// decomposition invariance.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "comm/comm.hpp"
#include "core/config.hpp"
#include "core/decomp.hpp"
#include "runtime/solver.hpp"

using namespace heat3d;

static int failures = 0;
#define EXPECT(c)                                                        \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                        \
    }                                                                    \
  } while (0)

static void test_dims() {
  auto eq = [](std::array<int, 3> a, int x, int y, int z) { return a[0] == x && a[1] == y && a[2] == z; };
  EXPECT(eq(dims_create(1), 1, 1, 1));
  EXPECT(eq(dims_create(2), 2, 1, 1));
  EXPECT(eq(dims_create(4), 2, 2, 1));
  EXPECT(eq(dims_create(6), 3, 2, 1));
  EXPECT(eq(dims_create(8), 2, 2, 2));
  EXPECT(eq(dims_create(12), 3, 2, 2));
  EXPECT(eq(dims_create(16), 4, 2, 2));
  EXPECT(eq(dims_create(64), 4, 4, 4));
  EXPECT(eq(dims_create(8, {8, 1, 1}), 8, 1, 1));
  EXPECT(eq(dims_create(8, {0, 1, 1}), 8, 1, 1));
}

static void test_decomp_tiles() {
  const int64_t N[3] = {27, 19, 33};
  for (auto dims : {std::array<int, 3>{1, 1, 1}, {2, 1, 1}, {2, 2, 2}, {3, 2, 1}, {1, 4, 2}}) {
    Decomposition d = Decomposition::make(N, dims);
    std::vector<int> cover(N[0] * N[1] * N[2], 0);
    for (auto& s : d.subs) {
      Box e = s.extended_global();
      for (int64_t i = e.lo[0]; i < e.hi[0]; ++i)
        for (int64_t j = e.lo[1]; j < e.hi[1]; ++j)
          for (int64_t k = e.lo[2]; k < e.hi[2]; ++k) cover[(i * N[1] + j) * N[2] + k]++;
      Box in;
      std::vector<Box> shell;
      Decomposition::split_interior(s, &in, &shell);
      int64_t vol = in.volume();
      for (auto& b : shell) vol += b.volume();
      EXPECT(vol == s.owned_points());
    }
    for (int c : cover) EXPECT(c == 1);
  }
}

static void test_layout() {
  const int64_t n[3] = {5, 7, 1022};
  Layout L = Layout::make(n, 8);
  EXPECT(L.index(0, 0, 0) % 16 == 0);
  EXPECT(L.index(3, 5, 0) % 16 == 0);
  EXPECT(L.index(-1, -1, -1) >= 0);
  EXPECT(L.sy >= L.zoff + n[2] + 1);
  Layout F = Layout::make(n, 4);
  EXPECT(F.index(2, 3, 0) % 32 == 0);
}

static RunResult solve(const char* nx, const char* eps, const char* iters, int vranks, std::vector<double>* field) {
  std::string vr = std::to_string(vranks);
  const char* argv[] = {"heat3d", nx, nx, nx, iters, eps, "--backend", "cpu", "--virtual-ranks", vr.c_str(), "--quiet"};
  Config c = Config::parse(11, argv);
  auto s = make_solver_from_env(c);
  s->initialize();
  RunResult r = s->run();
  s->compute_error(&r.error_mean, &r.error_local);
  if (field) s->gather_global(field);
  return r;
}

static void test_goldens() {
  // SURVEY.md App. B.3 (27^3): 938 / 1725 / 2513 iterations, 1.9155 / 0.1923 / 0.0192 %
  struct G { const char* eps; int64_t it; double err; } gs[] = {{"1e-3", 938, 1.9155}, {"1e-4", 1725, 0.1923}, {"1e-5", 2513, 0.0192}};
  for (auto& g : gs) {
    RunResult r = solve("27", g.eps, "100000", 1, nullptr);
    std::printf("27^3 eps=%s: iterations %lld, error %.4f %%\n", g.eps, (long long)r.conv_iter, 100 * r.error_mean);
    EXPECT(r.converged);
    EXPECT(r.conv_iter == g.it);
    EXPECT(std::fabs(100 * r.error_mean - g.err) < 6e-5);
  }
  RunResult r = solve("27", "1e-5", "100", 1, nullptr);
  EXPECT(!r.converged);
  EXPECT(std::fabs(100 * r.error_mean - 26.0129) < 6e-5);
  EXPECT(std::fabs(r.norm - 0.194872) < 1e-6);
}

static void test_invariance() {
  std::vector<double> f1, f8;
  RunResult a = solve("21", "1e-4", "100000", 1, &f1);
  RunResult b = solve("21", "1e-4", "100000", 8, &f8);
  EXPECT(a.conv_iter == b.conv_iter);
  EXPECT(f1.size() == f8.size());
  EXPECT(std::memcmp(f1.data(), f8.data(), f1.size() * sizeof(double)) == 0);
}

int main() {
  test_dims();
  test_decomp_tiles();
  test_layout();
  test_goldens();
  test_invariance();
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("all unit tests passed\n");
  return 0;
}
