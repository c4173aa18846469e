// heat3d-mi355x — hand-written gfx950 (CDNA4) kernels.
//
// Replaces the reference's single CUDA kernel `computeT` (heat3D.cu:118-142:
// one thread per x plane, 2-thread blocks, triple pointer chasing, never
// terminating k loop — SURVEY.md §2.2) and the host loop nests around it
// (T0 = T copy, face pack, residual scan, error scan: heat3D.cu:541-1106).
//
// Single-step kernels (the K-step sweeps that run by default are in
// stencil_tbl.hip / stencil_tbp.hip):
//   * stencil_tile: a workgroup of WZ x WY waves marches a (rows x z) tile
//     along x with the x-1 / x / x+1 planes in a register queue, z neighbours
//     through DPP, y halo rows exchanged through LDS once per plane, 16-byte
//     loads / stores, fused residual (NaN-propagating bit-pattern max, one
//     commit per workgroup), XCD-aware block order.  Single steps, the
//     rollback recomputation after convergence inside a sweep, and runs
//     without temporal blocking;
//   * stencil_naive: one lane per (y, z) column, seven loads per point — the
//     simplest gfx950 form of the update, kept as an oracle;
//   * a device flag set by the convergence check turns every kernel into a
//     no-op, so over-issued / graph-replayed iterations are harmless.
// Also here: IC/BC init, halo pack / unpack / copy, the convergence check,
// the error reduction, checksums, the x-plan model of the sweep kernels.
// Implicit contraction is disabled and the update's FMAs are explicit
// (ftcs_update), so results are bitwise identical to the CPU backend
// (kernels_cpu.cpp) and independent of the decomposition.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <tuple>
#include <mutex>
#include <map>
#include <functional>

#include "hip_helpers.hpp"

namespace heat3d {
namespace hip {

// ---- naive kernel: one lane per (y,z) column, 7 global loads per point -----
// Baseline and thin-box (boundary shell) kernel.  Block = 64 (z) x 4 (y).
template <typename Real>
__global__ __launch_bounds__(256) void stencil_naive(const Real* __restrict__ in,
                                                     Real* __restrict__ out, Layout L, Box b,
                                                     Real Dx, Real Dy, Real Dz,
                                                     unsigned long long* res, const int* done) {
  if (flag_set(done)) return;
  const int64_t k = b.lo[2] + (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int64_t j = b.lo[1] + (int64_t)blockIdx.y * 4 + (threadIdx.x >> 6);
  const int64_t x0 = b.lo[0] + (int64_t)blockIdx.z * 64;
  const int64_t x1 = min(x0 + 64, b.hi[0]);
  double m = 0.0;
  if (k < b.hi[2] && j < b.hi[1]) {
    const int64_t sx = L.sx, sy = L.sy;
    for (int64_t i = x0; i < x1; ++i) {
      const int64_t c = L.index(i, j, k);
      const Real T = in[c];
      const Real nv = ftcs<Real>(T, in[c - sx], in[c + sx], in[c - sy], in[c + sy], in[c - 1],
                                 in[c + 1], Dx, Dy, Dz);
      out[c] = nv;
      m = res_max(m, resid_abs(nv, T));
    }
  }
  if (res) residual_commit(res, m);
}

// ---- tile kernel: block-cooperative 2.5D blocking ---------------------------------
// A workgroup of WZ x WY waves owns a (WY*R rows) x (WZ*64*V points) tile and
// marches along x.  Each wave keeps its R x V column queue in registers, and
// the rows / edge points its neighbours need are
// exchanged through LDS once per plane (double-buffered by plane parity, one
// s_barrier per plane).  Only the tile's outer halo (2 rows, 2 edge columns)
// is fetched from memory, so HBM over-fetch drops from ~40 % (independent
// waves, profiles/) to 2/(WY*R) + edges.
struct TileGeom {
  int64_t z0a;        // first z of tile column 0 (box z0 rounded down to V)
  int nzb, nyb, nxs;  // tiles along z, y; x segments
  int seg;
  int64_t nblocks;
  int xq, xr;         // XCD remap
  int nt;
};

template <typename Real, int V, int R, int WZ, int WY>
__global__ __launch_bounds__(64 * WZ * WY) void stencil_tile(const Real* __restrict__ in,
                                                             Real* __restrict__ out, Layout L,
                                                             Box b, TileGeom g, Real Dx, Real Dy,
                                                             Real Dz, unsigned long long* res,
                                                             const int* done) {
  typedef typename VecOf<Real, V>::type Vec;
  constexpr int TZ = 64 * V;
  constexpr int NW = WZ * WY;
  // [parity][wave][bottom/top row][lane]
  __shared__ Vec s_rows[2][NW][2][64];
  // [parity][wave][row][left/right]
  __shared__ Real s_edge[2][NW][R][2];
  if (flag_set(done)) return;  // uniform across the block

  const int blk = blockIdx.x;
  const int xcd = blk & 7;
  int64_t t = xcd * g.xq + min(xcd, g.xr) + (blk >> 3);
  const int zb = (int)(t % g.nzb);
  t /= g.nzb;
  const int ybk = (int)(t % g.nyb);
  const int xs = (int)(t / g.nyb);

  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wz = wave % WZ, wy = wave / WZ;
  const int64_t kb = g.z0a + ((int64_t)zb * WZ + wz) * TZ;
  const int64_t k = kb + (int64_t)lane * V;
  const int64_t yb = b.lo[1] + ((int64_t)ybk * WY + wy) * R;
  const int ract = (int)max((int64_t)0, min((int64_t)R, b.hi[1] - yb));
  // neighbours in the tile: below (wy-1) always has R rows; above only if I am full
  const bool nb_lo = wy > 0;
  const bool nb_hi = (wy + 1 < WY) && (ract == R) && (yb + R < b.hi[1]);
  const bool nb_left = wz > 0, nb_right = wz + 1 < WZ;
  const int64_t xa = b.lo[0] + (int64_t)xs * g.seg;
  const int64_t xe = min(xa + (int64_t)g.seg, b.hi[0]);
  const int64_t sx = L.sx, sy = L.sy;

  bool valid[V];
  bool allvalid = true;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    valid[v] = (k + v >= b.lo[2]) && (k + v < b.hi[2]);
    allvalid &= valid[v];
  }
  const int64_t base0 = L.index(0, yb, k);
  // outer-edge gather: lanes [0,R) left edges (only the wz == 0 wave), lanes
  // [32,32+R) right edges (only the wz == WZ-1 wave)
  const int er = lane < 32 ? lane : lane - 32;
  const bool eload = er < ract && (lane < 32 ? !nb_left : !nb_right);
  const int64_t ebase = L.index(0, yb + er, lane < 32 ? kb - 1 : kb + TZ);

  auto ld = [&](int64_t plane, int r) -> Vec {
    return *reinterpret_cast<const Vec*>(in + base0 + plane * sx + (int64_t)r * sy);
  };

  Vec qm[R], qc[R], qp[R];
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (r < ract) {
      qm[r] = ld(xa - 1, r);
      qc[r] = ld(xa, r);
      qp[r] = ld(xa + 1, r);
    }
  Vec hb = {}, ht = {};
  if (ract > 0 && !nb_lo) hb = ld(xa, -1);
  if (ract > 0 && !nb_hi) ht = ld(xa, ract);
  Real ed = eload ? in[ebase + xa * sx] : Real(0);

  double m = 0.0;
  int par = 0;
  for (int64_t x = xa; x < xe; ++x) {
    // publish this wave's boundary rows / edge points of plane x
    if (ract > 0) {
      s_rows[par][wave][0][lane] = qc[0];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r == ract - 1) s_rows[par][wave][1][lane] = qc[r];  // static register index
        if (r < ract) {
          if (lane == 0) s_edge[par][wave][r][0] = qc[r][0];
          if (lane == 63) s_edge[par][wave][r][1] = qc[r][V - 1];
        }
      }
    }
    // prefetch plane x+2 centres and plane x+1 outer halo
    Vec qn[R];
    Vec hbn = {}, htn = {};
    Real edn = Real(0);
    const bool more = x + 1 < xe;
    if (more && ract > 0) {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (r < ract) qn[r] = ld(x + 2, r);
      if (!nb_lo) hbn = ld(x + 1, -1);
      if (!nb_hi) htn = ld(x + 1, ract);
      if (eload) edn = in[ebase + (x + 1) * sx];
    }
    __syncthreads();
    if (ract > 0) {
      const Vec ylo = nb_lo ? s_rows[par][wave - WZ][1][lane] : hb;
      const Vec yhi = nb_hi ? s_rows[par][wave + WZ][0][lane] : ht;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r < ract) {
          const Vec c = qc[r];
          const Vec ym = r == 0 ? ylo : qc[r > 0 ? r - 1 : 0];
          const Vec yp = (r == ract - 1) ? yhi : qc[r + 1 < R ? r + 1 : R - 1];
          const Real left = nb_left ? s_edge[par][wave - 1][r][1] : readlane(ed, r);
          const Real right = nb_right ? s_edge[par][wave + 1][r][0] : readlane(ed, 32 + r);
          Vec zm, zp, nv;
#pragma unroll
          for (int v = 0; v < V; ++v) {
            zm[v] = v == 0 ? dpp_shr1(left, c[V - 1]) : c[v > 0 ? v - 1 : 0];
            zp[v] = v == V - 1 ? dpp_shl1(right, c[0]) : c[v + 1 < V ? v + 1 : 0];
          }
#pragma unroll
          for (int v = 0; v < V; ++v) {
            nv[v] = ftcs<Real>(c[v], qm[r][v], qp[r][v], ym[v], yp[v], zm[v], zp[v], Dx, Dy, Dz);
            if (valid[v]) m = res_max(m, resid_abs(nv[v], c[v]));
          }
          Real* dst = out + base0 + x * sx + (int64_t)r * sy;
          if (allvalid) {
            if (g.nt) __builtin_nontemporal_store(nv, reinterpret_cast<Vec*>(dst));
            else *reinterpret_cast<Vec*>(dst) = nv;
          } else {
#pragma unroll
            for (int v = 0; v < V; ++v)
              if (valid[v]) dst[v] = nv[v];
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      qm[r] = qc[r];
      qc[r] = qp[r];
      qp[r] = qn[r];
    }
    hb = hbn;
    ht = htn;
    ed = edn;
    par ^= 1;
  }
  if (res) residual_commit(res, m);
}

// Resident workgroups of `kernel` on the whole device (occupancy x CUs).
// hipOccupancyMaxActiveBlocksPerMultiprocessor over-reports for kernels with
// large static LDS (it returned 8 x 1024-thread groups per CU for the 98 KiB
// tr3 kernel, which fits once in the 160 KiB of a CU), so the result is capped
// by our own LDS / wave-slot / VGPR bound.  HEAT3D_TRACE=1 prints both.
bool trace_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("HEAT3D_TRACE");
    return e && *e && e[0] != '0';
  }();
  return on;
}

int device_cus() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return std::max(1, cus);
}

int device_slots(const void* kernel, int block) {
  int dev = 0, cus = 256, per = 1, lds_cu = 160 * 1024;
  if (hipGetDevice(&dev) == hipSuccess) {
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) == hipSuccess && v > 0)
      lds_cu = v;
  }
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, 0) != hipSuccess || per < 1) per = 1;
  int own = 64;
  hipFuncAttributes a{};
  if (hipFuncGetAttributes(&a, kernel) == hipSuccess) {
    const int waves = (block + 63) / 64;
    if (a.sharedSizeBytes > 0) own = std::min<int>(own, lds_cu / (int)a.sharedSizeBytes);
    // 4 SIMDs x 512 VGPRs per lane (granule 8), at most 8 waves per SIMD
    const int vg = std::max(8, (a.numRegs + 7) / 8 * 8);
    const int per_simd = std::min(8, 512 / vg);
    own = std::min(own, (4 * per_simd) / std::max(1, waves));
  }
  const int pick = std::max(1, std::min(per, own));
  if (trace_enabled())
    std::fprintf(stderr, "[heat3d trace] device_slots: cus=%d api=%d own=%d lds=%zu vgpr=%d -> %d/CU\n", cus, per,
                 own, (size_t)a.sharedSizeBytes, a.numRegs, pick);
  return std::max(1, cus * pick);
}

// x-segment length for an x-marching kernel.  Each segment re-reads two
// planes, and the grid runs in ceil(blocks / slots) rounds, so the sweep costs
// ~ rounds * (seg + 2) plane-steps per slot.  Take the cheapest segment (ties:
// the longer one).  Measured on MI355X, 1024^3 fp64: 1 round of 511-plane
// segments 321 GLUPS vs 8 rounds of 64 planes 313 (profiles/kernel_sweep.md).
int choose_segment(int64_t nx, int64_t tiles, int slots, int halo) {
  if (nx <= 1) return 1;
  double best = 1e300;
  int pick = (int)nx;
  for (int64_t parts = 1; parts <= std::min<int64_t>(nx, 512); ++parts) {
    const int64_t seg = (nx + parts - 1) / parts;
    const int64_t nxs = (nx + seg - 1) / seg;
    const int64_t rounds = (tiles * nxs + slots - 1) / slots;
    const double cost = (double)rounds * (double)(seg + halo);
    if (cost < best - 1e-9) {
      best = cost;
      pick = (int)seg;
    }
  }
  return std::max(1, pick);
}

XPlan fixed_xplan(int64_t nx, int64_t tiles, int seg) {
  XPlan p;
  p.seg = (int)std::max<int64_t>(1, std::min<int64_t>(seg, std::max<int64_t>(1, nx)));
  const int64_t nxs = (nx + p.seg - 1) / p.seg;
  p.n1 = (int)(tiles * nxs);
  p.split = p.seg;
  return p;
}

// Greedy list scheduling of the pieces, in dispatch order, on `slots`
// workers; returns the makespan in plane-steps.
static double simulate_xplan(const XPlan& p, int64_t nx, int64_t tiles, int slots, int fill, int U,
                             std::vector<double>& heap) {
  const int64_t nxs = (nx + p.seg - 1) / p.seg;
  auto cost = [&](int64_t len) {
    const int64_t steps = len + fill;
    // + workgroup start-up and pipeline ramp
    return (double)((steps + U - 1) / U * U) + 8.0;
  };
  heap.assign((std::size_t)slots, 0.0);  // min-heap of worker free times
  auto run = [&](double c) {
    std::pop_heap(heap.begin(), heap.end(), std::greater<double>());
    heap.back() += c;
    std::push_heap(heap.begin(), heap.end(), std::greater<double>());
  };
  auto seg_len = [&](int64_t piece) {
    const int64_t xs = piece / tiles;  // segment index slowest
    const int64_t a = xs * p.seg;
    return std::min<int64_t>(p.seg, nx - a);
  };
  for (int64_t i = 0; i < p.n1; ++i) run(cost(seg_len(i)));
  for (int64_t i = 0; i < p.r; ++i) {
    const int64_t len = seg_len(p.n1 + i);
    run(cost(p.nb2 > 0 ? std::min<int64_t>(len, p.split) : len));
  }
  for (int64_t i = 0; i < p.nb2; ++i) {
    const int64_t len = seg_len(p.n1 + i);
    run(cost(std::max<int64_t>(0, len - p.split)));
  }
  double m = 0;
  for (double t : heap) m = std::max(m, t);
  (void)nxs;
  return m;
}

double xplan_makespan(const XPlan& p, int64_t nx, int64_t tiles, int slots, int fill, int U) {
  std::vector<double> heap;
  return simulate_xplan(p, nx, tiles, slots, fill, U, heap);
}

// Sweep time of a tiling in plane-steps per slot: the greedy-dispatch
// makespan, but never less than the total work spread over the workgroups
// that saturate HBM (~80% of the slots: tools/probes/tile_probe.hip, 176 of
// 256 workgroups already moved 5.45 TB/s).  The makespan alone sees no cost
// in a tile column that is almost empty as long as every tile still fits one
// round of workgroups — but the sweep is bandwidth-bound, so that column's
// loads are paid for: fp32 1022^3 with 112-column pair tiles (10 columns,
// the last 14 wide) ran 1294 GLUPS against 1397 with 120 (9 columns).
double tiling_cost(const XPlan& p, int64_t nx, int64_t tiles, int slots, int fill, int U) {
  const double work = (double)tiles * (double)(nx + fill) / (0.8 * std::max(1, slots));
  return std::max(xplan_makespan(p, nx, tiles, slots, fill, U), work);
}

std::vector<int> best_fixed_segments(int64_t nx, int64_t tiles, int slots, int fill, int U, int count) {
  std::vector<std::pair<double, int>> ms;
  std::vector<double> heap;
  if (nx < 2 * U || tiles < 1 || count < 1) return {};
  // a coarse grid of lengths (<= ~256 of them), then every length around the
  // best few: the makespan is piecewise smooth in the segment length
  const int lo = std::max<int>(U, (int)(nx / 32));
  const int step = std::max<int>(1, (int)((nx - lo) / 256));
  auto eval = [&](int seg) {
    for (const auto& m : ms)
      if (m.second == seg) return;
    ms.push_back({simulate_xplan(fixed_xplan(nx, tiles, seg), nx, tiles, slots, fill, U, heap), seg});
  };
  for (int seg = lo; seg <= (int)nx; seg += step) eval(seg);
  std::sort(ms.begin(), ms.end());
  std::vector<int> coarse;
  for (std::size_t i = 0; i < ms.size() && i < 3; ++i) coarse.push_back(ms[i].second);
  for (int c : coarse)
    for (int seg = std::max(lo, c - step); seg <= std::min<int>((int)nx, c + step); ++seg) eval(seg);
  std::sort(ms.begin(), ms.end());
  std::vector<int> out;
  for (const auto& m : ms) {
    if ((int)out.size() >= count) break;
    // distinct pieces: lengths giving the same segment count and makespan
    // within a chunk of each other add nothing to time
    bool near = false;
    for (int o : out) near |= std::abs(o - m.second) < U;
    if (!near) out.push_back(m.second);
  }
  return out;
}

XPlan plan_x(int64_t nx, int64_t tiles, int slots, int fill, int U, bool equal_only) {
  struct Key {
    int64_t nx, tiles;
    int slots, fill, U;
    bool eq;
    bool operator<(const Key& o) const {
      return std::tie(nx, tiles, slots, fill, U, eq) < std::tie(o.nx, o.tiles, o.slots, o.fill, o.U, o.eq);
    }
  };
  static std::mutex mu;
  static std::map<Key, XPlan> cache;
  const Key key{nx, tiles, slots, fill, U, equal_only};
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  // 1) equal segments from the round-count model (choose_segment), the
  // policy the kernel sweeps were tuned with (profiles/kernel_sweep.md)
  int seg0 = choose_segment(nx, tiles, slots, fill + 2);
  seg0 += (U - (seg0 + fill) % U) % U;  // segment steps in whole chunks of U
  XPlan best = fixed_xplan(nx, tiles, seg0);
  if (equal_only || !(tiles > slots && tiles <= 2 * (int64_t)slots && tiles % slots != 0)) {
    std::lock_guard<std::mutex> lk(mu);
    cache[key] = best;
    return best;
  }
  // 2) thin x boxes (an x slab of a 1024^2 face: 432 tiles on 256 CUs): one
  // whole-x piece per tile, the first `slots` of them a full round, the rest
  // cut in two and dispatched longest first so that the second round is
  // filled.  Taken only if the greedy-dispatch model predicts >= 10% — on
  // MI355X splitting long multi-round schedules (1024^3 fp64, 2049^3 fp32)
  // lost 5-15% to equal segments although the model favoured it slightly
  // (tools/probe_xplan.sh); the 128-plane slab gains 8%.
  std::vector<double> heap;
  const double base = simulate_xplan(best, nx, tiles, slots, fill, U, heap);
  XPlan c = fixed_xplan(nx, tiles, (int)nx);
  c.n1 = slots;
  c.r = (int)(tiles - slots);
  double best_t = base;
  for (int f = 1; f < 8; ++f) {
    XPlan t = c;
    t.split = std::max(1, c.seg * f / 8);
    t.nb2 = t.r;
    const double m = simulate_xplan(t, nx, tiles, slots, fill, U, heap);
    if (m < best_t - 1e-9 && m < 0.9 * base) {
      best_t = m;
      best = t;
    }
  }
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = best;
  return best;
}

namespace {
struct TuneKey {
  int dev;
  const void* kfn;
  int64_t n0, n1, n2;
  int slots, reserved;
  bool operator<(const TuneKey& o) const {
    return std::tie(dev, kfn, n0, n1, n2, slots, reserved) <
           std::tie(o.dev, o.kfn, o.n0, o.n1, o.n2, o.slots, o.reserved);
  }
};
std::mutex tune_mu;
std::map<TuneKey, TunedSchedule> tune_cache;
}  // namespace

bool tuned_lookup(const void* kfn, const int64_t box[3], int slots, int reserved, SchedChoice* out) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  std::lock_guard<std::mutex> lk(tune_mu);
  auto it = tune_cache.find(TuneKey{dev, kfn, box[0], box[1], box[2], slots, reserved});
  if (it == tune_cache.end()) return false;
  *out = SchedChoice{it->second.zs, it->second.L};
  return true;
}

SchedChoice tune_schedule(const char* name, const void* kfn, const int64_t box[3], int slots, int reserved, int U,
                          const std::vector<int>& zs_opts, hipStream_t s,
                          const std::function<void(int, int)>& launch, int64_t nyb, int fill) {
  int dev = 0;
  HIPK_CHECK(hipGetDevice(&dev));
  const TuneKey key{dev, kfn, box[0], box[1], box[2], slots, reserved};
  {
    std::unique_lock<std::mutex> lk(tune_mu);
    auto it = tune_cache.find(key);
    if (it != tune_cache.end()) {
      const SchedChoice c{it->second.zs, it->second.L};
      lk.unlock();
      launch(c.zs, c.L);
      return c;
    }
  }
  HEAT3D_CHECK(!zs_opts.empty(), "tune_schedule: no z stride");
  const int64_t nx = box[0];
  // candidates: per z stride, the model's x plan and segments of nx / k
  // planes (distinct, >= one unrolled chunk); candidate 0 = the model's
  // stride and plan, the reference every other must beat by 1.5 %
  std::vector<SchedChoice> cand;
  for (int zs : zs_opts) {
    cand.push_back({zs, -3});
    std::vector<int> segs;
    for (int k : {1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16}) {
      const int seg = (int)((nx + k - 1) / k);
      if (seg < U || seg >= (1 << 15) || std::find(segs.begin(), segs.end(), seg) != segs.end()) continue;
      segs.push_back(seg);
      cand.push_back({zs, seg});
    }
    if (nyb > 0) {
      const int64_t tiles = std::max<int64_t>(1, (box[2] + zs - 1) / zs) * nyb;
      for (int seg : best_fixed_segments(nx, tiles, slots, fill, U, 2)) {
        if (seg >= (1 << 15) || std::find(segs.begin(), segs.end(), seg) != segs.end()) continue;
        segs.push_back(seg);
        cand.push_back({zs, seg});
      }
    }
  }
  struct Ev {  // released on every exit, a throwing launch included
    hipEvent_t e = nullptr;
    Ev() { HIPK_CHECK(hipEventCreate(&e)); }
    ~Ev() { (void)hipEventDestroy(e); }
  } ev0, ev1;
  hipEvent_t e0 = ev0.e, e1 = ev1.e;
  // a candidate's time: `reps` back-to-back sweeps between two events, per
  // sweep, >= 4 ms in all (short sweeps timed one at a time are dominated by
  // launch gaps and timer noise)
  int reps = 1;
  auto timed = [&](const SchedChoice& c) {
    HIPK_CHECK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i) launch(c.zs, c.L);
    HIPK_CHECK(hipEventRecord(e1, s));
    HIPK_CHECK(hipEventSynchronize(e1));
    float ms = 0;
    HIPK_CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
  };
  std::vector<float> best(cand.size(), 1e30f);
  // warm (code object, caches, clocks), then size the repetitions to >= 4 ms
  launch(cand[0].zs, cand[0].L);
  reps = 3;
  const float t1 = timed(cand[0]);
  reps = std::max(1, std::min(16, (int)std::ceil(4.0f / std::max(1e-3f, t1))));
  for (int rep = 0; rep < 2; ++rep)
    for (std::size_t i = 0; i < cand.size(); ++i) best[i] = std::min(best[i], timed(cand[i]));
  std::size_t w = 0;
  for (std::size_t i = 1; i < cand.size(); ++i)
    if (best[i] < best[w]) w = i;
  if (best[w] > best[0] / 1.015f) w = 0;  // ties go to the model's choice
  if (w != 0) {
    // confirm against the model's choice, interleaved: a rival process on the
    // same GPU (or a clock step) during one candidate's runs must not decide
    float bw = 1e30f, b0 = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      b0 = std::min(b0, timed(cand[0]));
      bw = std::min(bw, timed(cand[w]));
    }
    best[w] = std::min(best[w], bw);
    best[0] = std::min(best[0], b0);
    if (bw > b0 / 1.015f) w = 0;
  }
  TunedSchedule t;
  t.kernel = name;
  t.nx = box[0];
  t.ny = box[1];
  t.nz = box[2];
  t.zs = cand[w].zs;
  t.L = cand[w].L;
  t.ms = best[w];
  t.ms_model = best[0];
  t.candidates = (int)cand.size();
  if (trace_enabled()) {
    std::fprintf(stderr, "[heat3d trace] schedule %s box %lldx%lldx%lld (%d reps):", name, (long long)box[0],
                 (long long)box[1], (long long)box[2], reps);
    for (std::size_t i = 0; i < cand.size(); ++i) std::fprintf(stderr, " %d/%d:%.3f", cand[i].zs, cand[i].L, best[i]);
    std::fprintf(stderr, " -> %d/%d\n", t.zs, t.L);
  }
  std::lock_guard<std::mutex> lk(tune_mu);
  tune_cache[key] = t;
  return cand[w];
}

std::vector<TunedSchedule> tuned_schedules() {
  std::lock_guard<std::mutex> lk(tune_mu);
  std::vector<TunedSchedule> v;
  for (auto& kv : tune_cache) v.push_back(kv.second);
  return v;
}

XPlanInfo describe_xplan(int64_t nx, int64_t tiles, int slots, int fill, int U, int seg) {
  const XPlan p = seg > 0 ? fixed_xplan(nx, tiles, seg) : plan_x(nx, tiles, slots, fill, U, seg == -1);
  XPlanInfo d;
  d.seg = p.seg;
  d.n1 = p.n1;
  d.r = p.r;
  d.split = p.split;
  d.nb2 = p.nb2;
  d.makespan = xplan_makespan(p, nx, tiles, slots, fill, U);
  return d;
}

template <typename Real, int V, int R, int WZ, int WY>
static void launch_tile(const StencilParams& p, const KernelSpec& k, hipStream_t s) {
  const Box& b = p.box;
  constexpr int TZ = 64 * V;
  TileGeom g;
  g.nt = k.NT;
  g.z0a = (b.lo[2] / V) * V;
  const int64_t nzt = (b.hi[2] - g.z0a + TZ - 1) / TZ;
  g.nzb = (int)((nzt + WZ - 1) / WZ);
  g.nyb = (int)((b.extent(1) + (int64_t)R * WY - 1) / ((int64_t)R * WY));
  int seg = k.L;
  if (seg <= 0) {
    // resident workgroups on the whole device, once per instantiation (a
    // magic static: thread-safe under --gpus N's host thread per GPU)
    static const int slots = device_slots(reinterpret_cast<const void*>(&stencil_tile<Real, V, R, WZ, WY>),
                                          64 * WZ * WY);
    seg = choose_segment(b.extent(0), (int64_t)g.nzb * g.nyb, slots);
  }
  g.seg = (int)std::min<int64_t>(seg, std::max<int64_t>(1, b.extent(0)));
  g.nxs = (int)((b.extent(0) + g.seg - 1) / g.seg);
  g.nblocks = (int64_t)g.nzb * g.nyb * g.nxs;
  HEAT3D_CHECK(g.nblocks < (1LL << 31), "too many blocks");
  g.xq = (int)(g.nblocks / 8);
  g.xr = (int)(g.nblocks % 8);
  unsigned long long* res = p.state && p.residual ? &p.state->residual[p.slot] : nullptr;
  const int* done = p.state ? &p.state->done : nullptr;
  hipLaunchKernelGGL((stencil_tile<Real, V, R, WZ, WY>), dim3((unsigned)g.nblocks),
                     dim3(64 * WZ * WY), 0, s, static_cast<const Real*>(p.in),
                     static_cast<Real*>(p.out), p.L, b, g, (Real)p.D[0], (Real)p.D[1],
                     (Real)p.D[2], res, done);
  HIPK_CHECK(hipGetLastError());
}

template <typename Real>
static void dispatch_tile(const StencilParams& p, const KernelSpec& k, hipStream_t s);

// ---- launch helpers -----------------------------------------------------------
template <typename Real>
static void launch_naive(const StencilParams& p, hipStream_t s) {
  const Box& b = p.box;
  dim3 grid((unsigned)((b.extent(2) + 63) / 64), (unsigned)((b.extent(1) + 3) / 4),
            (unsigned)((b.extent(0) + 63) / 64));
  unsigned long long* res = p.state && p.residual ? &p.state->residual[p.slot] : nullptr;
  const int* done = p.state ? &p.state->done : nullptr;
  hipLaunchKernelGGL(stencil_naive<Real>, grid, dim3(256), 0, s, static_cast<const Real*>(p.in),
                     static_cast<Real*>(p.out), p.L, b, (Real)p.D[0], (Real)p.D[1], (Real)p.D[2],
                     res, done);
  HIPK_CHECK(hipGetLastError());
}

template <typename Real>
static void dispatch_tile(const StencilParams& p, const KernelSpec& ks, hipStream_t s) {
  // defaults from the gfx950 sweep (KernelSpec::resolved, profiles/kernel_sweep.md)
  const KernelSpec k = ks.resolved(sizeof(Real) == 8 ? DType::F64 : DType::F32);
  const int V = k.V, R = k.R, WZ = k.WZ, WY = k.WY;
  if (p.box.extent(2) < 32 || p.box.extent(1) < 2) {
    launch_naive<Real>(p, s);
    return;
  }
#define H3D_TILE(VV, RR, ZZ, YY)                       \
  if (V == VV && R == RR && WZ == ZZ && WY == YY) {    \
    launch_tile<Real, VV, RR, ZZ, YY>(p, k, s);        \
    return;                                            \
  }
  H3D_TILE(2, 4, 1, 4) H3D_TILE(2, 4, 2, 2) H3D_TILE(2, 4, 2, 4) H3D_TILE(2, 4, 4, 2)
  H3D_TILE(2, 8, 1, 4) H3D_TILE(2, 8, 2, 2) H3D_TILE(2, 8, 4, 1) H3D_TILE(2, 8, 2, 4)
  H3D_TILE(2, 8, 4, 2) H3D_TILE(2, 6, 2, 2) H3D_TILE(2, 6, 2, 4) H3D_TILE(2, 8, 8, 1)
  if constexpr (sizeof(Real) == 4) {
    H3D_TILE(4, 4, 2, 2) H3D_TILE(4, 8, 2, 2) H3D_TILE(4, 8, 1, 4) H3D_TILE(4, 4, 2, 4)
  }
#undef H3D_TILE
  HEAT3D_THROW("unsupported tile kernel variant V=" << V << " R=" << R << " WZ=" << WZ
               << " WY=" << WY);
}

void stencil(DType t, const StencilParams& p, const KernelSpec& k, void* stream) {
  if (p.box.empty()) return;
  if (k.kind == KernelSpec::Naive) {
    if (t == DType::F64) launch_naive<double>(p, S(stream));
    else launch_naive<float>(p, S(stream));
  } else {
    HEAT3D_CHECK(k.kind == KernelSpec::Tile, "single-step kernels: naive | tile");
    if (t == DType::F64) dispatch_tile<double>(p, k, S(stream));
    else dispatch_tile<float>(p, k, S(stream));
  }
}

// ---- init ---------------------------------------------------------------------
template <typename Real>
__global__ __launch_bounds__(256) void init_kernel(Real* f, Layout L, InitParams p) {
  const int64_t ez = L.n[2] + 2 * L.gz;
  const int64_t kk = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (kk >= ez) return;
  const int64_t k = kk - L.gz, j = (int64_t)blockIdx.y - L.gy, i = (int64_t)blockIdx.z - L.gx;
  const int64_t gi = p.gstart[0] + i, gj = p.gstart[1] + j, gk = p.gstart[2] + k;
  // deep ghosts beyond the domain stay 0 (never read by an update)
  if (gi < 0 || gi >= p.N[0] || gj < 0 || gj >= p.N[1] || gk < 0 || gk >= p.N[2]) return;
  const bool phys = gi == 0 || gi == p.N[0] - 1 || gj == 0 || gj == p.N[1] - 1 || gk == 0 ||
                    gk == p.N[2] - 1;
  f[L.index(i, j, k)] = phys ? (Real)boundary_value(gi, gj, gk, p.N, p.h) : Real(0);
}

void init_field(DType t, const InitParams& p, void* stream) {
  HIPK_CHECK(hipMemsetAsync(p.field, 0, p.L.bytes(), S(stream)));
  // every ghost plane (deep x halos included) gets its Dirichlet ghost rows
  dim3 grid((unsigned)((p.L.n[2] + 2 * p.L.gz + 255) / 256), (unsigned)(p.L.n[1] + 2 * p.L.gy),
            (unsigned)(p.L.n[0] + 2 * p.L.gx));
  if (t == DType::F64)
    hipLaunchKernelGGL(init_kernel<double>, grid, dim3(256), 0, S(stream),
                       static_cast<double*>(p.field), p.L, p);
  else
    hipLaunchKernelGGL(init_kernel<float>, grid, dim3(256), 0, S(stream),
                       static_cast<float*>(p.field), p.L, p);
  HIPK_CHECK(hipGetLastError());
}

// ---- box <-> buffer copies (halo pack/unpack, local exchange) ------------------
// A workgroup of 256 threads covers tz consecutive z points (a power of two,
// min(256, ez rounded up)) of 256 / tz consecutive rows: grid x = z chunks of
// tz, y = row groups, z = planes (ex).  Thin boxes (the K-column z faces of
// block decompositions) thus fill their workgroups: one row per workgroup
// left 253 of 256 threads idle and made a 3 x 1030 x 1030 fp32 z face take
// ~0.9 ms to pack (phantom 2x2x2 trace, round 4).
template <typename Real, int DIR>
__global__ __launch_bounds__(256) void box_copy_kernel(const Real* __restrict__ src,
                                                       Real* __restrict__ dst, Layout Ls, Box bs,
                                                       Layout Ld, Box bd, int tz_log2) {
  const int64_t ez = bs.extent(2);
  const int tz = 1 << tz_log2;
  const int64_t kz = (int64_t)blockIdx.x * tz + (threadIdx.x & (tz - 1));
  const int64_t j = (int64_t)blockIdx.y * (256 >> tz_log2) + (threadIdx.x >> tz_log2), i = blockIdx.z;
  const int64_t ey = bs.extent(1);
  if (kz >= ez || j >= ey) return;
  int64_t si, di;
  if (DIR == 0) {  // field -> contiguous buffer
    si = Ls.index(bs.lo[0] + i, bs.lo[1] + j, bs.lo[2] + kz);
    di = (i * ey + j) * ez + kz;
  } else if (DIR == 1) {  // buffer -> field
    si = (i * ey + j) * ez + kz;
    di = Ld.index(bd.lo[0] + i, bd.lo[1] + j, bd.lo[2] + kz);
  } else {  // field -> field
    si = Ls.index(bs.lo[0] + i, bs.lo[1] + j, bs.lo[2] + kz);
    di = Ld.index(bd.lo[0] + i, bd.lo[1] + j, bd.lo[2] + kz);
  }
  dst[di] = src[si];
}

template <int DIR>
static void box_copy(DType t, const void* src, const Layout& Ls, const Box& bs, void* dst,
                     const Layout& Ld, const Box& bd, hipStream_t s) {
  if (bs.empty()) return;
  int lg = 0;
  while (lg < 8 && (int64_t(1) << lg) < bs.extent(2)) ++lg;
  const int64_t rows = 256 >> lg;
  HEAT3D_CHECK((bs.extent(1) + rows - 1) / rows < 65536 && bs.extent(0) < 65536, "box too large for copy grid");
  dim3 grid((unsigned)((bs.extent(2) + (1 << lg) - 1) >> lg), (unsigned)((bs.extent(1) + rows - 1) / rows),
            (unsigned)bs.extent(0));
  if (t == DType::F64)
    hipLaunchKernelGGL((box_copy_kernel<double, DIR>), grid, dim3(256), 0, s,
                       static_cast<const double*>(src), static_cast<double*>(dst), Ls, bs, Ld, bd, lg);
  else
    hipLaunchKernelGGL((box_copy_kernel<float, DIR>), grid, dim3(256), 0, s,
                       static_cast<const float*>(src), static_cast<float*>(dst), Ls, bs, Ld, bd, lg);
  HIPK_CHECK(hipGetLastError());
}

void pack_box(DType t, const void* f, const Layout& L, const Box& b, void* buf, void* stream) {
  box_copy<0>(t, f, L, b, buf, L, b, S(stream));
}
void unpack_box(DType t, void* f, const Layout& L, const Box& b, const void* buf, void* stream) {
  box_copy<1>(t, buf, L, b, f, L, b, S(stream));
}
void copy_box(DType t, const void* src, const Layout& Ls, const Box& bs, void* dst,
              const Layout& Ld, const Box& bd, void* stream) {
  HEAT3D_CHECK(bs.extent(0) == bd.extent(0) && bs.extent(1) == bd.extent(1) &&
                   bs.extent(2) == bd.extent(2),
               "copy_box extent mismatch " << bs.str() << " vs " << bd.str());
  box_copy<2>(t, src, Ls, bs, dst, Ld, bd, S(stream));
}

// ---- convergence check (single lane) ------------------------------------------
// last_only: the sweep's interior computed only its last residual (the
// monotone check, fused_check_tail): the other slots only advance the count
__global__ void check_kernel(DeviceState* s, int slot, int count, int last_only) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int i = slot; i < slot + count; ++i) {
    const double r = __builtin_bit_cast(double, (long long)s->residual[i]);
    s->residual[i] = kResidualInitBits;
    if (last_only && i < slot + count - 1) {
      s->iter = s->iter + 1;
      continue;
    }
    const int was = s->done;
    check_convergence_scalar(s, r);
    if (last_only && !was && s->done) s->coarse = (uint32_t)count;
  }
}

void check_convergence(DeviceState* s, int slot, void* stream, int count, bool last_only) {
  HEAT3D_CHECK(slot >= 0 && count >= 1 && slot + count <= kResidualSlots, "residual slots " << slot << "+" << count);
  hipLaunchKernelGGL(check_kernel, dim3(1), dim3(64), 0, S(stream), s, slot, count, last_only ? 1 : 0);
  HIPK_CHECK(hipGetLastError());
}

// Placement probe: every workgroup records (XCC id, SE / SH / CU id) of the
// CU it ran on (s_getreg of HW_REG_XCC_ID and HW_REG_HW_ID bits [15:8]), after
// spinning `ticks` so that the grid spreads over every CU it may use.
__global__ void cu_probe_kernel(unsigned* out, unsigned long long ticks) {
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20); // HW_REG_XCC_ID
    out[blockIdx.x] = ((xcc & 0xf) << 8) | ((hw >> 8) & 0xff);
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

void cu_probe(unsigned* out, int blocks, double us, void* stream) {
  hipLaunchKernelGGL(cu_probe_kernel, dim3((unsigned)blocks), dim3(64), 0, S(stream), out,
                     (unsigned long long)(us * 100.0));
  HIPK_CHECK(hipGetLastError());
}

__global__ void graph_signal_kernel(unsigned* slot) {
  if (threadIdx.x == 0) __hip_atomic_store(slot, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

struct WaitSlots {
  const unsigned* p[4];
};

// Waits for 1..4 signal slots of other streams' graphs.  Polls with relaxed
// agent-scope loads (an acquire load invalidates the L2 lines of the XCD at
// every poll, under an interior sweep that lives on L2 hits) and sleeps
// between polls; one acquire fence once every slot has flipped.  Gives up
// after st->wait_ticks (100 MHz) and flags fault 2 + done, and a wait that
// finds the fault already flagged returns at once, so one broken dependency
// drains the rest of the graph in one timeout.
__global__ void graph_wait_kernel(WaitSlots w, int n, DeviceState* st) {
  if (threadIdx.x != 0) return;
  if (__hip_atomic_load(&st->fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 2) return;
  const unsigned long long ticks = __hip_atomic_load(&st->wait_ticks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; ++i) {
    while (__hip_atomic_load(w.p[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
        __hip_atomic_store(&st->fault, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&st->done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

void graph_signal(unsigned* slot, void* stream) {
  hipLaunchKernelGGL(graph_signal_kernel, dim3(1), dim3(64), 0, S(stream), slot);
  HIPK_CHECK(hipGetLastError());
}

void graph_wait(const unsigned* const* slots, int n, DeviceState* st, void* stream) {
  HEAT3D_CHECK(n >= 1 && n <= 4 && st, "graph_wait: 1..4 slots and a state");
  WaitSlots w{};
  for (int i = 0; i < n; ++i) w.p[i] = slots[i];
  hipLaunchKernelGGL(graph_wait_kernel, dim3(1), dim3(64), 0, S(stream), w, n, st);
  HIPK_CHECK(hipGetLastError());
}

// ---- error vs analytic steady state T = y -------------------------------------
constexpr int kErrBlocks = 1024;
int64_t error_scratch_elems() { return kErrBlocks; }

template <typename Real>
__global__ __launch_bounds__(256) void error_partial_kernel(const Real* f, Layout L, Box b,
                                                            int64_t gj0, double hy,
                                                            double* partial) {
  __shared__ double red[4];
  const int64_t ey = b.extent(1), ez = b.extent(2);
  const int64_t rows = b.extent(0) * ey;
  double s = 0.0;
  for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
    const int64_t i = b.lo[0] + row / ey, j = b.lo[1] + row % ey;
    const double y = (double)(gj0 + j) * hy;
    const Real* p = f + L.index(i, j, b.lo[2]);
    for (int64_t k = threadIdx.x; k < ez; k += 256) s += fabs((double)p[k] - y);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ void error_final_kernel(const double* partial, int n, double count, DeviceState* s) {
  if (threadIdx.x != 0) return;
  double acc = 0.0;
  for (int i = 0; i < n; ++i) acc += partial[i];  // fixed order: deterministic
  s->error_sum += acc;
  s->error_count += count;
}

void error_accumulate(DType t, const void* f, const Layout& L, const Box& box,
                      const int64_t gstart[3], double hy, double* scratch, DeviceState* s,
                      void* stream) {
  if (box.empty()) return;
  if (t == DType::F64)
    hipLaunchKernelGGL(error_partial_kernel<double>, dim3(kErrBlocks), dim3(256), 0, S(stream),
                       static_cast<const double*>(f), L, box, gstart[1], hy, scratch);
  else
    hipLaunchKernelGGL(error_partial_kernel<float>, dim3(kErrBlocks), dim3(256), 0, S(stream),
                       static_cast<const float*>(f), L, box, gstart[1], hy, scratch);
  HIPK_CHECK(hipGetLastError());
  hipLaunchKernelGGL(error_final_kernel, dim3(1), dim3(64), 0, S(stream), scratch, kErrBlocks,
                     (double)box.volume(), s);
  HIPK_CHECK(hipGetLastError());
}

// ---- halo verification: order-independent checksum of a box -------------------
// Sum (mod 2^64) of the values' bit patterns: exact and independent of the
// summation order, so sender and receiver of a halo can compare checksums.
template <typename Real>
__global__ __launch_bounds__(256) void bitsum_kernel(const Real* f, Layout L, Box b,
                                                     unsigned long long* out) {
  const int64_t ey = b.extent(1), ez = b.extent(2);
  const int64_t n = b.extent(0) * ey * ez;
  unsigned long long acc = 0;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < n; q += (int64_t)gridDim.x * 256) {
    const int64_t k = q % ez, j = (q / ez) % ey, i = q / (ez * ey);
    const Real v = f[L.index(b.lo[0] + i, b.lo[1] + j, b.lo[2] + k)];
    if constexpr (sizeof(Real) == 8) acc += (unsigned long long)__builtin_bit_cast(long long, v);
    else acc += (unsigned long long)(unsigned)__builtin_bit_cast(int, v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}

void box_bitsum(DType t, const void* f, const Layout& L, const Box& b, unsigned long long* out,
                void* stream) {
  HIPK_CHECK(hipMemsetAsync(out, 0, 8, S(stream)));
  if (b.empty()) return;
  const int blocks = (int)std::min<int64_t>(1024, (b.volume() + 255) / 256);
  if (t == DType::F64)
    hipLaunchKernelGGL(bitsum_kernel<double>, dim3(blocks), dim3(256), 0, S(stream),
                       static_cast<const double*>(f), L, b, out);
  else
    hipLaunchKernelGGL(bitsum_kernel<float>, dim3(blocks), dim3(256), 0, S(stream),
                       static_cast<const float*>(f), L, b, out);
  HIPK_CHECK(hipGetLastError());
}

// ---- bandwidth probes (roofline calibration on the box) ------------------------
__global__ __launch_bounds__(256) void copy16_kernel(const uint4* __restrict__ src,
                                                     uint4* __restrict__ dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    dst[i] = src[i];
}

__global__ __launch_bounds__(256) void read16_kernel(const uint4* __restrict__ src, int64_t n,
                                                     unsigned* sink) {
  unsigned acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;  // practically never: keeps the loads live
}

// 4 independent 16-B loads in flight per lane; NT = non-temporal loads/stores
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ __launch_bounds__(256) void copy16x4_kernel(const u32x4* __restrict__ src,
                                                       u32x4* __restrict__ dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], dst + i + u * stride);
      else dst[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

// each block copies one contiguous chunk (DRAM-page friendly)
__global__ __launch_bounds__(256) void copy16_chunk_kernel(const uint4* __restrict__ src,
                                                           uint4* __restrict__ dst, int64_t n) {
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t b0 = (int64_t)blockIdx.x * per, b1 = min(n, b0 + per);
  for (int64_t i = b0 + threadIdx.x; i < b1; i += 1024) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * 256 < b1) v[u] = src[i + u * 256];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * 256 < b1) dst[i + u * 256] = v[u];
  }
}

void bandwidth_probe(int kind, const void* src, void* dst, int64_t bytes, int blocks, void* stream) {
  const int64_t n = bytes / 16;
  if (kind >= 2) {
    const uint4* s = static_cast<const uint4*>(src);
    uint4* d = static_cast<uint4*>(dst);
    const u32x4* vs = static_cast<const u32x4*>(src);
    u32x4* vd = static_cast<u32x4*>(dst);
    if (kind == 2) hipLaunchKernelGGL(copy16x4_kernel<false>, dim3(blocks), dim3(256), 0, S(stream), vs, vd, n);
    else if (kind == 3) hipLaunchKernelGGL(copy16x4_kernel<true>, dim3(blocks), dim3(256), 0, S(stream), vs, vd, n);
    else hipLaunchKernelGGL(copy16_chunk_kernel, dim3(blocks), dim3(256), 0, S(stream), s, d, n);
    HIPK_CHECK(hipGetLastError());
    return;
  }
  if (kind == 0)
    hipLaunchKernelGGL(copy16_kernel, dim3(blocks), dim3(256), 0, S(stream),
                       static_cast<const uint4*>(src), static_cast<uint4*>(dst), n);
  else
    hipLaunchKernelGGL(read16_kernel, dim3(blocks), dim3(256), 0, S(stream),
                       static_cast<const uint4*>(src), n, static_cast<unsigned*>(dst));
  HIPK_CHECK(hipGetLastError());
}

template <typename Real>
__global__ void poke_kernel(Real* f, int64_t idx, double v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) f[idx] = (Real)v;
}

void poke(DType t, void* f, const Layout& L, int64_t i, int64_t j, int64_t k, double value,
          void* stream) {
  const int64_t idx = L.index(i, j, k);
  if (t == DType::F64)
    hipLaunchKernelGGL(poke_kernel<double>, dim3(1), dim3(64), 0, S(stream),
                       static_cast<double*>(f), idx, value);
  else
    hipLaunchKernelGGL(poke_kernel<float>, dim3(1), dim3(64), 0, S(stream),
                       static_cast<float*>(f), idx, value);
  HIPK_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace heat3d
