// heat3d-mi355x — 2-step temporally blocked FTCS kernel for gfx950.
//
// The single-step kernels are HBM-bound at 16 B/point/iteration (fp64).  This
// kernel advances T^n -> T^{n+2} in ONE sweep: each workgroup keeps the
// intermediate u = T^{n+1} of its tile in registers (a second x-queue next to
// the T^n queue) and writes only T^{n+2}, i.e. 8 B read + 8 B written per point
// per TWO iterations.  Every point still goes through the reference update
// twice, with the same arithmetic (kernels.hpp ftcs_update), so T^{n+2}
// and both residuals are bitwise identical to two single-step sweeps
// (tests/test_gpu_kernels.py).
//
// Tiling: overlapped tiles.  A workgroup of WZ x WY waves computes u on its
// whole (WY*R rows) x (WZ*64*V points) tile (from T^n plus the usual 1-deep
// halo) and T^{n+2} on the tile minus a 1-row / V-column ring; neighbouring
// tiles overlap by that ring (2 rows, 2V columns), so each stored point is
// produced by exactly one tile.  Boundary rows / edge points of u and T^n
// are exchanged between the waves of a tile through LDS once per plane.
// Outside the u range (StencilParams::ux, default the box) u = T^n: the
// Dirichlet ghosts.  Single GPU: box = the whole subdomain.  Multi-GPU slabs:
// the x faces with a neighbour carry a 2-plane halo of T^n, the u range is
// extended one plane into it, and the solver launches the kernel on the
// interior planes [2, n0-2) (no halo needed) while the halo is exchanged, then
// on the two 2-plane boundary slabs.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "hip_helpers.hpp"

namespace heat3d {
namespace hip {

// Compact kernel arguments: 32-bit coordinates (extents < 2^31), 64-bit
// strides.  Passing Layout/Box wholesale cost ~8 extra spilled SGPRs.
struct TB2Args {
  int64_t sx, sy, origin;  // plane / row strides, element index of owned (0,0,0)
  int blo[3], bhi[3];      // store box
  int ulo, uhi;            // x range where u = FTCS(T^n)
  int xlo_live, xhi_live;  // x planes present in memory
  int kb0, yb0;            // first u column / row of tile (0, 0)
  int nzb, nyb, seg;
  int xq, xr;              // XCD remap: blocks per XCD (quotient / remainder)
};

template <typename Real, int V, int R, int WZ, int WY>
__global__ __launch_bounds__(64 * WZ * WY) void stencil_tb2(const Real* __restrict__ in,
                                                            Real* __restrict__ out, TB2Args g,
                                                            Real Dx, Real Dy, Real Dz,
                                                            unsigned long long* res1,
                                                            unsigned long long* res2,
                                                            const int* done) {
  typedef typename VecOf<Real, V>::type Vec;
  constexpr int TZ = 64 * V;
  constexpr int NW = WZ * WY;
  constexpr int TZB = WZ * TZ;
  constexpr int TYB = WY * R;
  __shared__ Vec s_tr[2][NW][2][64];   // T^n bottom/top rows per wave
  __shared__ Vec s_ur[2][NW][2][64];   // u bottom/top rows per wave
  __shared__ Real s_te[2][NW][R][2];   // T^n left/right edge points per wave row
  __shared__ Real s_ue[2][NW][R][2];   // u left/right edge points per wave row
  if (flag_set(done)) return;

  const int blk = blockIdx.x;
  const int xcd = blk & 7;
  int t = xcd * g.xq + min(xcd, g.xr) + (blk >> 3);
  const int zb = t % g.nzb;
  t /= g.nzb;
  const int ybk = t % g.nyb;
  const int xs = t / g.nyb;

  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wz = wave % WZ, wy = wave / WZ;
  const int tkb = g.kb0 + zb * (TZB - 2 * V);  // tile's first column
  const int tyb = g.yb0 + ybk * (TYB - 2);     // tile's first row
  const int kb = tkb + wz * TZ;
  const int k = kb + lane * V;
  const int yb = tyb + wy * R;
  const int ylo = g.blo[1], yhi = g.bhi[1];
  // rows with index <= yhi (the ghost row above the box) are loaded ("live")
  const int rlive = max(0, min(R, yhi + 1 - yb));
  const int xa = g.blo[0] + xs * g.seg;
  const int xe = min(xa + g.seg, g.bhi[0]);
  const int64_t sx = g.sx, sy = g.sy;
  const int xlo_live = g.xlo_live, xhi_live = g.xhi_live;  // planes present in memory

  // per-lane column predicates
  bool zin[V];     // inside the box
  bool zst[V];     // stored (inside box and not in the tile's V-column ring)
  bool allst = true;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int kk = k + v;
    zin[v] = kk >= g.blo[2] && kk < g.bhi[2];
    zst[v] = zin[v] && kk >= tkb + V && kk < tkb + TZB - V;
    allst &= zst[v];
  }
  const int64_t base0 = g.origin + (int64_t)yb * sy + k;
  // outer T^n edge gather (wz == 0 left / wz == WZ-1 right)
  const int er = lane < 32 ? lane : lane - 32;
  const bool eload = er < rlive && yb + er >= -1 && (lane < 32 ? wz == 0 : wz == WZ - 1);
  const int64_t ebase = g.origin + (int64_t)(yb + er) * sy + (lane < 32 ? kb - 1 : kb + TZ);
  const bool has_lo = wy > 0, has_hi = wy + 1 < WY;
  const bool hb_live = !has_lo && yb - 1 >= -1 && rlive > 0;
  const bool ht_live = !has_hi && yb + R <= yhi && rlive == R;

  auto plane_live = [&](int x) { return x >= xlo_live && x <= xhi_live; };
  auto ld = [&](int plane, int r) -> Vec {
    return *reinterpret_cast<const Vec*>(in + base0 + (int64_t)plane * sx + (int64_t)r * sy);
  };
  auto load_plane = [&](int x, Vec* q) {
    const bool pl = plane_live(x);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (pl && r < rlive && yb + r >= -1) q[r] = ld(x, r);
      else q[r] = Vec{};
    }
  };

  Vec qm[R], qc[R], qp[R], um[R], uc[R];
  load_plane(xa - 2, qm);
  load_plane(xa - 1, qc);
  load_plane(xa, qp);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    um[r] = Vec{};
    uc[r] = Vec{};
  }
  Vec hb = {}, ht = {};
  Real ed = Real(0);
  if (plane_live(xa - 1)) {
    if (hb_live) hb = ld(xa - 1, -1);
    if (ht_live) ht = ld(xa - 1, R);
    if (eload) ed = in[ebase + (int64_t)(xa - 1) * sx];
  }

  double m1 = 0.0, m2 = 0.0;
  int par = 0;
  for (int x = xa - 1; x <= xe; ++x) {
    // publish T^n(x) and u(x-1) boundary rows / edge points
    s_tr[par][wave][0][lane] = qc[0];
    s_tr[par][wave][1][lane] = qc[R - 1];
    s_ur[par][wave][0][lane] = uc[0];
    s_ur[par][wave][1][lane] = uc[R - 1];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (lane == 0) {
        s_te[par][wave][r][0] = qc[r][0];
        s_ue[par][wave][r][0] = uc[r][0];
      }
      if (lane == 63) {
        s_te[par][wave][r][1] = qc[r][V - 1];
        s_ue[par][wave][r][1] = uc[r][V - 1];
      }
    }
    // prefetch T^n(x+2) and the outer halo of plane x+1
    Vec qn[R];
    load_plane(x + 2, qn);
    Vec hbn = {}, htn = {};
    Real edn = Real(0);
    if (plane_live(x + 1)) {
      if (hb_live) hbn = ld(x + 1, -1);
      if (ht_live) htn = ld(x + 1, R);
      if (eload) edn = in[ebase + (int64_t)(x + 1) * sx];
    }
    __syncthreads();

    // ---- u(x) = FTCS(T^n) inside the box, T^n outside (Dirichlet ghosts)
    const bool xin = x >= g.ulo && x < g.uhi;
    Vec un[R];
    {
      const Vec tlo = has_lo ? s_tr[par][wave - WZ][1][lane] : hb;
      const Vec thi = has_hi ? s_tr[par][wave + WZ][0][lane] : ht;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const Vec c = qc[r];
        const Vec ym = r == 0 ? tlo : qc[r > 0 ? r - 1 : 0];
        const Vec yp = r == R - 1 ? thi : qc[r + 1 < R ? r + 1 : 0];
        const Real left = wz > 0 ? s_te[par][wave - 1][r][1] : readlane(ed, r);
        const Real right = wz + 1 < WZ ? s_te[par][wave + 1][r][0] : readlane(ed, 32 + r);
        const bool yin = xin && (yb + r >= ylo) && (yb + r < yhi);
        Vec u;
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const Real zm = v == 0 ? dpp_shr1(left, c[V - 1]) : c[v > 0 ? v - 1 : 0];
          const Real zp = v == V - 1 ? dpp_shl1(right, c[0]) : c[v + 1 < V ? v + 1 : 0];
          const Real nv = ftcs<Real>(c[v], qm[r][v], qp[r][v], ym[v], yp[v], zm, zp, Dx, Dy, Dz);
          const bool in_box = yin && zin[v];
          u[v] = in_box ? nv : c[v];
          if (in_box) m1 = res_max(m1, resid_abs(nv, c[v]));
        }
        un[r] = u;
      }
    }

    // ---- T^{n+2}(x-1) = FTCS(u) on the stored region
    const int xo = x - 1;
    if (xo >= xa && xo < xe) {
      const Vec ulo = has_lo ? s_ur[par][wave - WZ][1][lane] : uc[0];
      const Vec uhi = has_hi ? s_ur[par][wave + WZ][0][lane] : uc[R - 1];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int row = yb + r;
        // stored rows: inside the box and not in the tile's 1-row ring
        const bool rst = row >= ylo && row < yhi && row >= tyb + 1 && row < tyb + TYB - 1;
        const Vec c = uc[r];
        const Vec ym = r == 0 ? ulo : uc[r > 0 ? r - 1 : 0];
        const Vec yp = r == R - 1 ? uhi : uc[r + 1 < R ? r + 1 : 0];
        const Real left = wz > 0 ? s_ue[par][wave - 1][r][1] : c[0];
        const Real right = wz + 1 < WZ ? s_ue[par][wave + 1][r][0] : c[V - 1];
        Vec nv;
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const Real zm = v == 0 ? dpp_shr1(left, c[V - 1]) : c[v > 0 ? v - 1 : 0];
          const Real zp = v == V - 1 ? dpp_shl1(right, c[0]) : c[v + 1 < V ? v + 1 : 0];
          nv[v] = ftcs<Real>(c[v], um[r][v], un[r][v], ym[v], yp[v], zm, zp, Dx, Dy, Dz);
          if (rst && zst[v]) m2 = res_max(m2, resid_abs(nv[v], c[v]));
        }
        if (rst) {
          Real* dst = out + base0 + (int64_t)xo * sx + (int64_t)r * sy;
          if (allst) {
            *reinterpret_cast<Vec*>(dst) = nv;
          } else {
#pragma unroll
            for (int v = 0; v < V; ++v)
              if (zst[v]) dst[v] = nv[v];
          }
        }
      }
    }
    // ---- rotate queues
#pragma unroll
    for (int r = 0; r < R; ++r) {
      qm[r] = qc[r];
      qc[r] = qp[r];
      qp[r] = qn[r];
      um[r] = uc[r];
      uc[r] = un[r];
    }
    hb = hbn;
    ht = htn;
    ed = edn;
    par ^= 1;
  }
  if (res1) residual_commit(res1, m1);
  if (res2) residual_commit(res2, m2);
}

template <typename Real, int V, int R, int WZ, int WY>
static void launch_tb2(const StencilParams& p, const KernelSpec& k, hipStream_t s) {
  const Box& b = p.box;
  constexpr int TZ = 64 * V;
  constexpr int TZB = WZ * TZ, TYB = WY * R;
  static_assert(TYB > 2 && TZB > 2 * V, "tile too small");
  const Layout& L = p.L;
  HEAT3D_CHECK(L.n[0] + 2 * L.gx < (1LL << 30) && L.n[1] + 2 < (1LL << 30) && L.sy < (1LL << 30),
               "tb2: extents exceed 32-bit tile coordinates");
  TB2Args g;
  g.sx = L.sx;
  g.sy = L.sy;
  g.origin = L.origin;
  for (int a = 0; a < 3; ++a) {
    g.blo[a] = (int)b.lo[a];
    g.bhi[a] = (int)b.hi[a];
  }
  g.ulo = (int)(p.ux[1] >= p.ux[0] ? p.ux[0] : b.lo[0]);
  g.uhi = (int)(p.ux[1] >= p.ux[0] ? p.ux[1] : b.hi[0]);
  g.xlo_live = (int)-L.gx;
  g.xhi_live = (int)(L.n[0] + L.gx - 1);
  HEAT3D_CHECK(g.ulo > g.xlo_live && g.uhi <= g.xhi_live && g.ulo <= b.lo[0] && g.uhi >= b.hi[0],
               "tb2: u range [" << g.ulo << "," << g.uhi << ") outside the ghosted layout");
  int64_t kb0 = ((b.lo[2] - V) / V) * V;
  if (kb0 > b.lo[2] - V) kb0 -= V;  // floor for negative values
  g.kb0 = (int)kb0;
  g.yb0 = (int)(b.lo[1] - 1);
  // tiles step by (TZB - 2V) columns and (TYB - 2) rows; stored columns of
  // tile zb: [kb0 + zb*(TZB-2V) + V, ... + TZB - V)
  const int64_t zspan = b.hi[2] - (kb0 + V);
  g.nzb = (int)std::max<int64_t>(1, (zspan + (TZB - 2 * V) - 1) / (TZB - 2 * V));
  const int64_t yspan = b.hi[1] - (g.yb0 + 1);
  g.nyb = (int)std::max<int64_t>(1, (yspan + (TYB - 2) - 1) / (TYB - 2));
  int seg = k.L;
  if (seg <= 0) {
    static const int slots = device_slots(reinterpret_cast<const void*>(&stencil_tb2<Real, V, R, WZ, WY>),
                                          64 * WZ * WY);  // magic static: thread-safe
    seg = choose_segment(b.extent(0), (int64_t)g.nzb * g.nyb, slots, 4);
  }
  g.seg = (int)std::min<int64_t>(seg, std::max<int64_t>(1, b.extent(0)));
  const int64_t nxs = (b.extent(0) + g.seg - 1) / g.seg;
  const int64_t nblocks = (int64_t)g.nzb * g.nyb * nxs;
  HEAT3D_CHECK(nblocks < (1LL << 31), "too many blocks");
  g.xq = (int)(nblocks / 8);
  g.xr = (int)(nblocks % 8);
  unsigned long long* r1 = p.state ? &p.state->residual[p.slot] : nullptr;
  unsigned long long* r2 = p.state ? &p.state->residual[p.slot ^ 1] : nullptr;
  const int* done = p.state ? &p.state->done : nullptr;
  hipLaunchKernelGGL((stencil_tb2<Real, V, R, WZ, WY>), dim3((unsigned)nblocks),
                     dim3(64 * WZ * WY), 0, s, static_cast<const Real*>(p.in),
                     static_cast<Real*>(p.out), g, (Real)p.D[0], (Real)p.D[1], (Real)p.D[2], r1,
                     r2, done);
  HIPK_CHECK(hipGetLastError());
}

template <typename Real>
static void dispatch_tb2(const StencilParams& p, const KernelSpec& k, hipStream_t s) {
  // defaults (KernelSpec::resolved) from the MI355X sweep: one wave per tile
  // column, 8 waves of 2 rows stacked in y (~100 VGPRs: 2 blocks/CU)
  const KernelSpec r = k.resolved(sizeof(Real) == 8 ? DType::F64 : DType::F32);
  const int V = r.V, R = r.R, WZ = r.WZ, WY = r.WY;
#define H3D_TB2(VV, RR, ZZ, YY)                      \
  if (V == VV && R == RR && WZ == ZZ && WY == YY) {  \
    launch_tb2<Real, VV, RR, ZZ, YY>(p, k, s);       \
    return;                                          \
  }
  H3D_TB2(2, 4, 2, 4) H3D_TB2(2, 4, 4, 2) H3D_TB2(2, 4, 1, 4) H3D_TB2(2, 4, 2, 2)
  H3D_TB2(2, 8, 2, 2) H3D_TB2(2, 6, 2, 2) H3D_TB2(2, 2, 2, 8)
  H3D_TB2(2, 4, 1, 2) H3D_TB2(2, 4, 1, 8) H3D_TB2(2, 6, 1, 4) H3D_TB2(2, 8, 1, 4)
  H3D_TB2(2, 2, 1, 8) H3D_TB2(2, 3, 1, 4) H3D_TB2(2, 5, 1, 4) H3D_TB2(2, 6, 1, 2)
  H3D_TB2(2, 2, 1, 16) H3D_TB2(2, 3, 1, 8) H3D_TB2(2, 2, 1, 4) H3D_TB2(2, 2, 2, 4)
  if constexpr (sizeof(Real) == 4) {
    H3D_TB2(4, 4, 2, 4) H3D_TB2(4, 4, 2, 2) H3D_TB2(4, 4, 1, 4) H3D_TB2(4, 4, 1, 8)
    H3D_TB2(4, 2, 1, 8) H3D_TB2(4, 6, 1, 4) H3D_TB2(4, 4, 1, 2) H3D_TB2(4, 3, 1, 4)
    H3D_TB2(4, 2, 1, 16) H3D_TB2(4, 2, 1, 4) H3D_TB2(4, 3, 1, 8) H3D_TB2(4, 1, 1, 16)
  }
#undef H3D_TB2
  HEAT3D_THROW("unsupported tb2 kernel variant V=" << V << " R=" << R << " WZ=" << WZ
               << " WY=" << WY);
}

void stencil2(DType t, const StencilParams& p, const KernelSpec& k, void* stream) {
  if (p.box.empty()) return;
  if (t == DType::F64) dispatch_tb2<double>(p, k, S(stream));
  else dispatch_tb2<float>(p, k, S(stream));
}

}  // namespace hip
}  // namespace heat3d
