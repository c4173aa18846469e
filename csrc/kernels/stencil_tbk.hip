// heat3d-mi355x — K-step temporally blocked FTCS kernel for gfx950 (K >= 2).
//
// Generalises stencil_tb2.hip: one HBM sweep advances T^n -> T^{n+K}.  A
// workgroup marches its tile along x and keeps K register pipelines: stage s
// turns F_s = T^{n+s} into F_{s+1}, lagging stage s-1 by one plane, so that
// at plane step x
//     F_1(x), F_2(x-1), ..., F_K(x-K+1)
// are produced and only F_K is written.  Per point and per K iterations the
// kernel reads T^n once and writes T^{n+K} once: 16 B / K per iteration in
// fp64 instead of 16 B.  Every F_s value goes through the reference update
// (heat3D.cu:128-131) with the same arithmetic (kernels.hpp ftcs_update), so
// T^{n+K} and all K residuals are bitwise identical to K single steps.
//
// Tiles overlap: F_1 is valid on the whole (WY*R rows) x (WZ*64*V columns)
// tile (the T^n halo around it is loaded), F_{s+1} loses one row / column per
// side per stage, T^{n+K} is stored on the tile minus a (K-1)-row ring and a
// zring-column ring (K-1 rounded up to V).  Rows of the "centre" plane of
// every stage are exchanged between the waves of a tile through LDS once per
// plane step (double-buffered: one barrier per step).  Residuals count only
// the valid, in-box points of each stage.
//
// Dirichlet ghosts: outside the u range [ulo, uhi) in x and outside the box
// in y / z, F_s = T^n.  Deep neighbour halos (K planes of T^n exchanged every
// K iterations, x slabs) widen [ulo, uhi) by K-1 planes into the halo.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "hip_helpers.hpp"

namespace heat3d {
namespace hip {

struct TBKArgs {
  int64_t sx, sy, origin;  // plane / row strides, element index of owned (0,0,0)
  int blo[3], bhi[3];      // store box
  int ulo, uhi;            // x range where F_{s+1} = FTCS(F_s)
  int xlo_live, xhi_live;  // x planes present in memory
  int kb0, yb0;            // first column / row of tile (0, 0)
  int zstep, zring;        // tile stride along z, stored column ring
  int nzb, nyb, seg;
  int xq, xr;              // XCD remap: blocks per XCD (quotient / remainder)
};

template <typename Real, int V>
__device__ __forceinline__ void ldv(const Real* p, Real (&d)[V]) {
  if constexpr (V == 1) {
    d[0] = *p;
  } else {
    typedef typename VecOf<Real, V>::type Vec;
    const Vec t = *reinterpret_cast<const Vec*>(p);
#pragma unroll
    for (int v = 0; v < V; ++v) d[v] = t[v];
  }
}

template <typename Real, int V>
__device__ __forceinline__ void stv(Real* p, const Real (&s)[V]) {
  if constexpr (V == 1) {
    *p = s[0];
  } else {
    typedef typename VecOf<Real, V>::type Vec;
    Vec t;
#pragma unroll
    for (int v = 0; v < V; ++v) t[v] = s[v];
    *reinterpret_cast<Vec*>(p) = t;
  }
}

template <typename Real, int V>
__device__ __forceinline__ void cpv(Real (&d)[V], const Real (&s)[V]) {
#pragma unroll
  for (int v = 0; v < V; ++v) d[v] = s[v];
}

template <typename Real, int V, int R, int WZ, int WY, int K, int PD>
__global__ __launch_bounds__(64 * WZ * WY) void stencil_tbk(const Real* __restrict__ in,
                                                            Real* __restrict__ out, TBKArgs g,
                                                            Real Dx, Real Dy, Real Dz,
                                                            unsigned long long* res,
                                                            const int* done) {
  static_assert(K >= 2 && K <= 6, "temporal depth");
  static_assert(PD >= 1 && PD <= 4, "prefetch depth");
  constexpr int TZ = 64 * V;
  constexpr int NW = WZ * WY;
  constexpr int NE = WZ > 1 ? NW : 1;
  constexpr int TZB = WZ * TZ;
  constexpr int TYB = WY * R;
  static_assert(TYB > 2 * (K - 1) && R <= 32, "tile too small");
  // centre-plane bottom/top rows and left/right edge points of every stage
  __shared__ __attribute__((aligned(16))) Real s_row[2][K][NW][2][TZ];
  __shared__ Real s_edge[2][K][NE][R][2];
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
  const int tkb = g.kb0 + zb * g.zstep;         // tile's first column
  const int tyb = g.yb0 + ybk * (TYB - 2 * (K - 1));  // tile's first row
  const int kb = tkb + wz * TZ;
  const int k = kb + lane * V;
  const int yb = tyb + wy * R;
  const int ylo = g.blo[1], yhi = g.bhi[1];
  const int rlive = max(0, min(R, yhi + 1 - yb));  // rows <= yhi are loaded
  const int xa = g.blo[0] + xs * g.seg;
  const int xe = min(xa + g.seg, g.bhi[0]);
  const int64_t sx = g.sx, sy = g.sy;

  int cp[V];     // column position inside the tile
  bool zin[V];   // inside the box (z)
  bool zst[V];   // stored column
  bool allst = true;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int kk = k + v;
    cp[v] = kk - tkb;
    zin[v] = kk >= g.blo[2] && kk < g.bhi[2];
    zst[v] = zin[v] && cp[v] >= g.zring && cp[v] < TZB - g.zring;
    allst &= zst[v];
  }
  const int64_t base0 = g.origin + (int64_t)yb * sy + k;
  const int er = lane & 31;
  const bool eload = er < rlive && yb + er >= -1 && (lane < 32 ? wz == 0 : wz == WZ - 1);
  const int64_t ebase = g.origin + (int64_t)(yb + er) * sy + (lane < 32 ? kb - 1 : kb + TZ);
  const bool has_lo = wy > 0, has_hi = wy + 1 < WY;
  const bool hb_live = !has_lo && yb - 1 >= -1 && rlive > 0;
  const bool ht_live = !has_hi && yb + R <= yhi && rlive == R;

  auto plane_live = [&](int x) { return x >= g.xlo_live && x <= g.xhi_live; };
  auto load_plane = [&](int x, Real (&q)[R][V]) {
    const bool pl = plane_live(x);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (pl && r < rlive && yb + r >= -1) {
        ldv<Real, V>(in + base0 + (int64_t)x * sx + (int64_t)r * sy, q[r]);
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) q[r][v] = Real(0);
      }
    }
  };
  auto load_halo = [&](int x, Real (&hb)[V], Real (&ht)[V], Real& ed) {
#pragma unroll
    for (int v = 0; v < V; ++v) hb[v] = ht[v] = Real(0);
    ed = Real(0);
    if (plane_live(x)) {
      if (hb_live) ldv<Real, V>(in + base0 + (int64_t)x * sx - sy, hb);
      if (ht_live) ldv<Real, V>(in + base0 + (int64_t)x * sx + (int64_t)R * sy, ht);
      if (eload) ed = in[ebase + (int64_t)x * sx];
    }
  };

  // F_0 = T^n queue (planes x-1, x, x+1) and stages F_1..F_{K-1} (m, c, n)
  Real qm[R][V], qc[R][V], qp[R][V];
  Real f[K - 1][3][R][V];
  const int x0 = xa - (K - 1);
  load_plane(x0 - 1, qm);
  load_plane(x0, qc);
  load_plane(x0 + 1, qp);
#pragma unroll
  for (int s = 0; s < K - 1; ++s)
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int v = 0; v < V; ++v) f[s][i][r][v] = Real(0);
  Real hb[V], ht[V], ed;
  load_halo(x0, hb, ht, ed);
  // loads in flight: T^n planes x+2 .. x+PD and halos of planes x+1 .. x+PD-1
  // (PD planes ahead keeps enough bytes in flight per wave to cover HBM latency)
  Real pre[PD][R][V], hpb[PD][V], hpt[PD][V], hpe[PD];
#pragma unroll
  for (int i = 0; i < PD - 1; ++i) {
    load_plane(x0 + 2 + i, pre[i]);
    load_halo(x0 + 1 + i, hpb[i], hpt[i], hpe[i]);
  }

  double m[K];
#pragma unroll
  for (int s = 0; s < K; ++s) m[s] = 0.0;
  int par = 0;
  for (int x = x0; x <= xe + K - 2; ++x) {
    // ---- publish the centre rows / edge points of every stage
#pragma unroll
    for (int s = 0; s < K; ++s) {
      Real (&C)[R][V] = s == 0 ? qc : f[s > 0 ? s - 1 : 0][1];
      stv<Real, V>(&s_row[par][s][wave][0][lane * V], C[0]);
      stv<Real, V>(&s_row[par][s][wave][1][lane * V], C[R - 1]);
      if constexpr (WZ > 1) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (lane == 0) s_edge[par][s][wave][r][0] = C[r][0];
          if (lane == 63) s_edge[par][s][wave][r][1] = C[r][V - 1];
        }
      }
    }
    // ---- prefetch T^n(x+2) and the outer halo of plane x+1
    load_plane(x + 1 + PD, pre[PD - 1]);
    load_halo(x + PD, hpb[PD - 1], hpt[PD - 1], hpe[PD - 1]);
    __syncthreads();

#pragma unroll
    for (int s = 0; s < K; ++s) {
      Real (&C)[R][V] = s == 0 ? qc : f[s > 0 ? s - 1 : 0][1];
      Real (&M)[R][V] = s == 0 ? qm : f[s > 0 ? s - 1 : 0][0];
      Real (&P)[R][V] = s == 0 ? qp : f[s > 0 ? s - 1 : 0][2];
      const int p = x - s;  // plane produced by this stage
      const bool xin = p >= g.ulo && p < g.uhi;
      const bool xval = x >= xa - K + 2 * s + 1;  // inputs of this plane were valid
      Real lo[V], hi[V];
      if (has_lo) {
        ldv<Real, V>(&s_row[par][s][wave - WZ][1][lane * V], lo);
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) lo[v] = s == 0 ? hb[v] : C[0][v];
      }
      if (has_hi) {
        ldv<Real, V>(&s_row[par][s][wave + WZ][0][lane * V], hi);
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) hi[v] = s == 0 ? ht[v] : C[R - 1][v];
      }
      if (s < K - 1) {
        Real (&N)[R][V] = f[s < K - 1 ? s : 0][2];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int row = yb + r, rp = wy * R + r;
          const bool yin = xin && row >= ylo && row < yhi;
          const bool rval = xval && rp >= s && rp < TYB - s;
          Real left, right;
          if constexpr (WZ > 1) {
            left = wz > 0 ? s_edge[par][s][wave - 1][r][1] : (s == 0 ? readlane(ed, r) : C[r][0]);
            right = wz + 1 < WZ ? s_edge[par][s][wave + 1][r][0] : (s == 0 ? readlane(ed, 32 + r) : C[r][V - 1]);
          } else {
            left = s == 0 ? readlane(ed, r) : C[r][0];
            right = s == 0 ? readlane(ed, 32 + r) : C[r][V - 1];
          }
          const Real* ym = r == 0 ? lo : C[r > 0 ? r - 1 : 0];
          const Real* yp = r == R - 1 ? hi : C[r + 1 < R ? r + 1 : 0];
          Real nr[V];
#pragma unroll
          for (int v = 0; v < V; ++v) {
            const Real zm = v == 0 ? dpp_shr1(left, C[r][V - 1]) : C[r][v > 0 ? v - 1 : 0];
            const Real zp = v == V - 1 ? dpp_shl1(right, C[r][0]) : C[r][v + 1 < V ? v + 1 : 0];
            const Real nv = ftcs<Real>(C[r][v], M[r][v], P[r][v], ym[v], yp[v], zm, zp, Dx, Dy, Dz);
            const bool in_box = yin && zin[v];
            nr[v] = in_box ? nv : C[r][v];
            if (in_box && rval && cp[v] >= s && cp[v] < TZB - s)
              m[s] = res_max(m[s], resid_abs(nv, C[r][v]));
          }
          cpv<Real, V>(N[r], nr);
        }
      } else {
        // final stage: T^{n+K}(p) on the stored region
        if (p >= xa && p < xe) {
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int row = yb + r, rp = wy * R + r;
            const bool rst = row >= ylo && row < yhi && rp >= K - 1 && rp < TYB - (K - 1);
            Real left, right;
            if constexpr (WZ > 1) {
              left = wz > 0 ? s_edge[par][s][wave - 1][r][1] : C[r][0];
              right = wz + 1 < WZ ? s_edge[par][s][wave + 1][r][0] : C[r][V - 1];
            } else {
              left = C[r][0];
              right = C[r][V - 1];
            }
            const Real* ym = r == 0 ? lo : C[r > 0 ? r - 1 : 0];
            const Real* yp = r == R - 1 ? hi : C[r + 1 < R ? r + 1 : 0];
            Real nv[V];
#pragma unroll
            for (int v = 0; v < V; ++v) {
              const Real zm = v == 0 ? dpp_shr1(left, C[r][V - 1]) : C[r][v > 0 ? v - 1 : 0];
              const Real zp = v == V - 1 ? dpp_shl1(right, C[r][0]) : C[r][v + 1 < V ? v + 1 : 0];
              nv[v] = ftcs<Real>(C[r][v], M[r][v], P[r][v], ym[v], yp[v], zm, zp, Dx, Dy, Dz);
              if (rst && zst[v]) m[s] = res_max(m[s], resid_abs(nv[v], C[r][v]));
            }
            if (rst) {
              Real* dst = out + base0 + (int64_t)p * sx + (int64_t)r * sy;
              if (allst) {
                stv<Real, V>(dst, nv);
              } else {
#pragma unroll
                for (int v = 0; v < V; ++v)
                  if (zst[v]) dst[v] = nv[v];
              }
            }
          }
        }
      }
    }
    // ---- rotate queues
#pragma unroll
    for (int r = 0; r < R; ++r) {
      cpv<Real, V>(qm[r], qc[r]);
      cpv<Real, V>(qc[r], qp[r]);
      cpv<Real, V>(qp[r], pre[0][r]);
#pragma unroll
      for (int i = 0; i + 1 < PD; ++i) cpv<Real, V>(pre[i][r], pre[i + 1][r]);
#pragma unroll
      for (int s = 0; s < K - 1; ++s) {
        cpv<Real, V>(f[s][0][r], f[s][1][r]);
        cpv<Real, V>(f[s][1][r], f[s][2][r]);
      }
    }
    cpv<Real, V>(hb, hpb[0]);
    cpv<Real, V>(ht, hpt[0]);
    ed = hpe[0];
#pragma unroll
    for (int i = 0; i + 1 < PD; ++i) {
      cpv<Real, V>(hpb[i], hpb[i + 1]);
      cpv<Real, V>(hpt[i], hpt[i + 1]);
      hpe[i] = hpe[i + 1];
    }
    par ^= 1;
  }
  if (res) {
#pragma unroll
    for (int s = 0; s < K; ++s) residual_commit(res + s, m[s]);
  }
}

template <typename Real, int V, int R, int WZ, int WY, int K, int PD>
static void launch_tbk(const StencilParams& p, const KernelSpec& ks, hipStream_t s) {
  const Box& b = p.box;
  constexpr int TZ = 64 * V;
  constexpr int TZB = WZ * TZ, TYB = WY * R;
  const Layout& L = p.L;
  HEAT3D_CHECK(L.gx >= 1 && L.n[0] + 2 * L.gx < (1LL << 30) && L.n[1] + 2 < (1LL << 30) &&
                   L.sy < (1LL << 30),
               "tbk: extents exceed 32-bit tile coordinates");
  TBKArgs g;
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
  // F_1 on plane ulo needs T^n on ulo - 1; the widest u range is K-1 planes
  // into a K-deep halo
  HEAT3D_CHECK(g.ulo - 1 >= g.xlo_live && g.uhi <= g.xhi_live && g.ulo <= b.lo[0] &&
                   g.uhi >= b.hi[0],
               "tbk: u range [" << g.ulo << "," << g.uhi << ") outside the ghosted layout");
  g.zring = ((K - 1 + V - 1) / V) * V;
  g.zstep = TZB - 2 * g.zring;
  HEAT3D_CHECK(g.zstep > 0, "tbk: tile too narrow for depth " << K);
  int64_t kb0 = b.lo[2] - g.zring;
  kb0 = (kb0 >= 0 ? kb0 / V : -((-kb0 + V - 1) / V)) * V;  // floor to a multiple of V
  g.kb0 = (int)kb0;
  g.yb0 = (int)(b.lo[1] - (K - 1));
  const int64_t zspan = b.hi[2] - (kb0 + g.zring);
  g.nzb = (int)std::max<int64_t>(1, (zspan + g.zstep - 1) / g.zstep);
  const int ystep = TYB - 2 * (K - 1);
  g.nyb = (int)std::max<int64_t>(1, (b.extent(1) + ystep - 1) / ystep);
  int seg = ks.L;
  if (seg <= 0) {
    static const int slots =  // magic static: thread-safe
        device_slots(reinterpret_cast<const void*>(&stencil_tbk<Real, V, R, WZ, WY, K, PD>), 64 * WZ * WY);
    seg = choose_segment(b.extent(0), (int64_t)g.nzb * g.nyb, slots, 2 * K);
  }
  g.seg = (int)std::min<int64_t>(seg, std::max<int64_t>(1, b.extent(0)));
  const int64_t nxs = (b.extent(0) + g.seg - 1) / g.seg;
  const int64_t nblocks = (int64_t)g.nzb * g.nyb * nxs;
  HEAT3D_CHECK(nblocks < (1LL << 31), "too many blocks");
  g.xq = (int)(nblocks / 8);
  g.xr = (int)(nblocks % 8);
  HEAT3D_CHECK(!p.state || p.slot + K <= kResidualSlots, "tbk: residual slots " << p.slot << "+" << K);
  unsigned long long* r = p.state ? &p.state->residual[p.slot] : nullptr;
  const int* done = p.state ? &p.state->done : nullptr;
  hipLaunchKernelGGL((stencil_tbk<Real, V, R, WZ, WY, K, PD>), dim3((unsigned)nblocks), dim3(64 * WZ * WY), 0, s,
                     static_cast<const Real*>(p.in), static_cast<Real*>(p.out), g, (Real)p.D[0],
                     (Real)p.D[1], (Real)p.D[2], r, done);
  HIPK_CHECK(hipGetLastError());
}

template <typename Real>
static void dispatch_tbk(const StencilParams& p, const KernelSpec& k, hipStream_t s) {
  const int K = k.K;
  // defaults (KernelSpec::resolved) from the MI355X sweep (profiles/kernel_sweep.md)
  const KernelSpec r = k.resolved(sizeof(Real) == 8 ? DType::F64 : DType::F32);
  const int V = r.V, R = r.R, WZ = r.WZ, WY = r.WY;
  const int PD = r.NT;  // 7th spec field: prefetch depth in planes
#define H3D_TBK(VV, RR, ZZ, YY, KK, PP)                                     \
  if (V == VV && R == RR && WZ == ZZ && WY == YY && K == KK && PD == PP) {  \
    launch_tbk<Real, VV, RR, ZZ, YY, KK, PP>(p, k, s);                      \
    return;                                                                 \
  }
#define H3D_TBK_PD(VV, RR, ZZ, YY, KK) \
  H3D_TBK(VV, RR, ZZ, YY, KK, 1) H3D_TBK(VV, RR, ZZ, YY, KK, 2) H3D_TBK(VV, RR, ZZ, YY, KK, 3)
  H3D_TBK_PD(1, 4, 1, 8, 2) H3D_TBK_PD(1, 4, 1, 16, 2) H3D_TBK_PD(1, 4, 1, 8, 3)
  H3D_TBK_PD(1, 4, 1, 16, 3) H3D_TBK_PD(1, 6, 1, 8, 3) H3D_TBK_PD(1, 4, 1, 8, 4)
  H3D_TBK_PD(1, 6, 1, 8, 4) H3D_TBK_PD(1, 4, 1, 16, 4) H3D_TBK_PD(1, 3, 1, 16, 3)
  H3D_TBK(2, 2, 1, 8, 2, 1) H3D_TBK(2, 2, 1, 8, 2, 2) H3D_TBK(2, 2, 1, 8, 3, 2) H3D_TBK(2, 2, 1, 8, 3, 1)
  H3D_TBK(1, 4, 2, 8, 3, 2) H3D_TBK(1, 4, 2, 8, 3, 1) H3D_TBK(1, 2, 1, 16, 2, 2) H3D_TBK(1, 2, 1, 16, 3, 2)
  if constexpr (sizeof(Real) == 4) {
    H3D_TBK_PD(2, 4, 1, 8, 2) H3D_TBK_PD(2, 4, 1, 8, 3) H3D_TBK_PD(2, 4, 1, 8, 4)
    H3D_TBK_PD(2, 4, 1, 16, 3) H3D_TBK(2, 6, 1, 8, 4, 2) H3D_TBK(4, 2, 1, 8, 3, 2) H3D_TBK(4, 2, 1, 8, 3, 1)
  }
#undef H3D_TBK_PD
#undef H3D_TBK
  HEAT3D_THROW("unsupported tbk kernel variant V=" << V << " R=" << R << " WZ=" << WZ << " WY=" << WY
                                                   << " K=" << K << " PD=" << PD);
}

void stencil_multi(DType t, const StencilParams& p, const KernelSpec& k, void* stream) {
  if (p.box.empty()) return;
  if (t == DType::F64) dispatch_tbk<double>(p, k, S(stream));
  else dispatch_tbk<float>(p, k, S(stream));
}

}  // namespace hip
}  // namespace heat3d
