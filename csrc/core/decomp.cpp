#include "decomp.hpp"

#include <algorithm>
#include <climits>
#include <sstream>

namespace heat3d {

std::array<int, 3> dims_create(int nprocs, std::array<int, 3> fixed) {
  HEAT3D_CHECK(nprocs >= 1, "nprocs must be >= 1");
  int fixed_prod = 1, nfree = 0;
  for (int a = 0; a < 3; ++a) {
    if (fixed[a] > 0) fixed_prod *= fixed[a];
    else ++nfree;
  }
  HEAT3D_CHECK(nprocs % fixed_prod == 0,
               "fixed dims product " << fixed_prod << " does not divide " << nprocs);
  const int rem = nprocs / fixed_prod;
  if (nfree == 0) {
    HEAT3D_CHECK(rem == 1, "fixed dims product " << fixed_prod << " != nprocs " << nprocs);
    return fixed;
  }
  // Exhaustive search over non-increasing factorizations of `rem` into `nfree`
  // factors; pick the most balanced (smallest max-min spread, then smallest
  // max).  Matches MPI_Dims_create on 2,4,6,8,12,16,24,32,48,64 (tests).
  std::vector<int> best;
  int best_spread = INT_MAX, best_max = INT_MAX;
  std::vector<int> cur;
  auto rec = [&](auto&& self, int left, int slots, int cap) -> void {
    if (slots == 1) {
      if (left > cap) return;
      cur.push_back(left);
      int mx = *std::max_element(cur.begin(), cur.end());
      int mn = *std::min_element(cur.begin(), cur.end());
      if (mx - mn < best_spread || (mx - mn == best_spread && mx < best_max)) {
        best_spread = mx - mn;
        best_max = mx;
        best = cur;
      }
      cur.pop_back();
      return;
    }
    for (int d = std::min(left, cap); d >= 1; --d) {
      if (left % d) continue;
      cur.push_back(d);
      self(self, left / d, slots - 1, d);
      cur.pop_back();
    }
  };
  rec(rec, rem, nfree, rem);
  std::array<int, 3> out = fixed;
  int bi = 0;
  for (int a = 0; a < 3; ++a)
    if (out[a] <= 0) out[a] = best[bi++];
  return out;
}

std::array<int, 3> Topology::coords(int rank) const {
  // MPI_Cart_coords, row-major with the last dimension fastest.
  std::array<int, 3> c;
  c[2] = rank % dims[2];
  c[1] = (rank / dims[2]) % dims[1];
  c[0] = rank / (dims[2] * dims[1]);
  return c;
}

int Topology::rank_of(std::array<int, 3> c) const {
  for (int a = 0; a < 3; ++a)
    if (c[a] < 0 || c[a] >= dims[a]) return -1;
  return (c[0] * dims[1] + c[1]) * dims[2] + c[2];
}

int Topology::neighbor(int rank, Face f) const {
  auto c = coords(rank);
  c[face_axis(f)] += face_side(f) ? 1 : -1;
  return rank_of(c);
}

void split_even(int64_t n, int parts, int p, int64_t* start, int64_t* count) {
  const int64_t base = n / parts, rem = n % parts;
  *count = base + (p < rem ? 1 : 0);
  *start = p * base + std::min<int64_t>(p, rem);
}

Box Subdomain::owned_global() const {
  Box b;
  for (int a = 0; a < 3; ++a) {
    b.lo[a] = gstart[a];
    b.hi[a] = gstart[a] + n[a];
  }
  return b;
}

Box Subdomain::extended_global() const {
  Box b = owned_global();
  for (int a = 0; a < 3; ++a) {
    if (!has_neighbor(face_of(a, 0))) b.lo[a] -= 1;
    if (!has_neighbor(face_of(a, 1))) b.hi[a] += 1;
  }
  return b;
}

Decomposition Decomposition::make(const int64_t N[3], std::array<int, 3> dims) {
  Decomposition d;
  for (int a = 0; a < 3; ++a) {
    d.N[a] = N[a];
    HEAT3D_CHECK(N[a] >= 3, "grid extent must be >= 3");
    HEAT3D_CHECK(dims[a] >= 1, "process grid extent must be >= 1");
    HEAT3D_CHECK(N[a] - 2 >= dims[a], "axis " << a << ": " << (N[a] - 2)
                 << " interior points cannot be split over " << dims[a] << " ranks");
  }
  d.topo.dims = dims;
  const int P = d.topo.size();
  d.subs.resize(P);
  for (int r = 0; r < P; ++r) {
    Subdomain& s = d.subs[r];
    s.rank = r;
    s.coords = d.topo.coords(r);
    for (int a = 0; a < 3; ++a) {
      int64_t st, cnt;
      split_even(N[a] - 2, dims[a], s.coords[a], &st, &cnt);
      s.n[a] = cnt;
      s.gstart[a] = 1 + st;  // global vertex 0 is the Dirichlet boundary
    }
    for (int f = 0; f < kNumFaces; ++f) s.neighbors[f] = d.topo.neighbor(r, static_cast<Face>(f));
  }
  return d;
}

void Decomposition::split_interior(const Subdomain& s, Box* interior, std::vector<Box>* shell) {
  Box in;
  for (int a = 0; a < 3; ++a) {
    in.lo[a] = s.has_neighbor(face_of(a, 0)) ? 1 : 0;
    in.hi[a] = s.n[a] - (s.has_neighbor(face_of(a, 1)) ? 1 : 0);
    if (in.hi[a] < in.lo[a]) in.hi[a] = in.lo[a];
  }
  // If the interior is degenerate along some axis, everything is shell.
  bool degenerate = in.empty();
  if (degenerate) {
    for (int a = 0; a < 3; ++a) in.lo[a] = in.hi[a] = 0;
  }
  *interior = in;
  shell->clear();
  // Peel slabs axis by axis: x-slabs span full y,z; y-slabs span the remaining
  // x range and full z; z-slabs span the remaining x,y ranges.
  Box rest;
  for (int a = 0; a < 3; ++a) {
    rest.lo[a] = 0;
    rest.hi[a] = s.n[a];
  }
  if (degenerate) {
    shell->push_back(rest);
    return;
  }
  for (int a = 0; a < 3; ++a) {
    if (in.lo[a] > rest.lo[a]) {
      Box b = rest;
      b.hi[a] = in.lo[a];
      shell->push_back(b);
      rest.lo[a] = in.lo[a];
    }
    if (in.hi[a] < rest.hi[a]) {
      Box b = rest;
      b.lo[a] = in.hi[a];
      shell->push_back(b);
      rest.hi[a] = in.hi[a];
    }
  }
}

std::string Decomposition::describe() const {
  std::ostringstream os;
  os << "grid " << N[0] << "x" << N[1] << "x" << N[2] << ", process grid " << topo.dims[0] << "x"
     << topo.dims[1] << "x" << topo.dims[2];
  return os.str();
}

}  // namespace heat3d
