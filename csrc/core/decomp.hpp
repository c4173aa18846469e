// heat3d-mi355x — process topology and domain decomposition.
//
// Topology: a clone of MPI_Dims_create (balanced, non-increasing factors) and
// the MPI Cartesian rank<->coords mapping with z fastest, non-periodic, -1 for
// "no neighbour" (reference heat3D.cu:224-263; survey §2.4 M2-M5).
//
// Decomposition differs from the reference on purpose:
// the reference splits the N vertices into equal chunks that *share* a node
// plane and requires (N-1) % dims == 0 (heat3D.cu:373-389).  Here only the
// N-2 interior (updated) vertices are owned, split as evenly as possible, and
// every subdomain carries a one-cell ghost shell that holds either a
// neighbour's halo or the Dirichlet boundary value.  Any N works with any
// process grid and the result is bitwise independent of the decomposition.
#pragma once

#include <array>
#include <cstdint>
#include <string>
#include <vector>

#include "common.hpp"

namespace heat3d {

// MPI_Dims_create clone for 3 dimensions.  Entries of `fixed` that are > 0 are
// kept (like MPI's non-zero input dims).
std::array<int, 3> dims_create(int nprocs, std::array<int, 3> fixed = {0, 0, 0});

struct Topology {
  std::array<int, 3> dims = {1, 1, 1};
  int size() const { return dims[0] * dims[1] * dims[2]; }
  std::array<int, 3> coords(int rank) const;
  int rank_of(std::array<int, 3> c) const;  // -1 if outside (non-periodic)
  int neighbor(int rank, Face f) const;      // MPI_Cart_shift equivalent; -1 = PROC_NULL
};

// Split `n` items into `parts` contiguous pieces, first (n % parts) pieces one
// larger.  Returns the start offset and count of piece `p`.
void split_even(int64_t n, int parts, int p, int64_t* start, int64_t* count);

// One rank's piece of the global grid.
struct Subdomain {
  int rank = 0;
  std::array<int, 3> coords = {0, 0, 0};
  int64_t n[3] = {0, 0, 0};        // owned interior points per axis
  int64_t gstart[3] = {0, 0, 0};   // global vertex index of owned local index 0
  int neighbors[kNumFaces] = {-1, -1, -1, -1, -1, -1};
  bool has_neighbor(Face f) const { return neighbors[static_cast<int>(f)] >= 0; }
  // Owned box extended into the ghost shell on every face that lies on the
  // physical boundary.  These boxes tile the whole N^3 grid exactly (global
  // indices) and define gather / checkpoint / Tecplot "owned" zones.
  Box extended_global() const;
  Box owned_global() const;
  int64_t owned_points() const { return n[0] * n[1] * n[2]; }
};

struct Decomposition {
  int64_t N[3] = {0, 0, 0};
  Topology topo;
  std::vector<Subdomain> subs;  // indexed by rank

  static Decomposition make(const int64_t N[3], std::array<int, 3> dims);
  // Boxes (local owned coordinates) for the overlap schedule: `interior` keeps
  // one cell away from every face that has a neighbour; `shell` lists
  // disjoint boxes covering owned \ interior.
  static void split_interior(const Subdomain& s, Box* interior, std::vector<Box>* shell);
  std::string describe() const;
};

}  // namespace heat3d
