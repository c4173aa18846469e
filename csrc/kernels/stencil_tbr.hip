// heat3d-mi355x — K-step temporally blocked FTCS kernel, register-ring form.
//
// Same algorithm and bitwise results as stencil_tbk.hip (one HBM sweep turns
// T^n into T^{n+K}; stage s turns F_s = T^{n+s} into F_{s+1}, lagging stage
// s-1 by one plane; every point goes through the reference update,
// heat3D.cu:128-131, with the same arithmetic (kernels.hpp ftcs_update)), but
// restructured after the rocprofv3 counters of stencil_tbk on MI355X
// (profiles/pmc_tbk.md, profiles/kernel_sweep.md): there, 28% of the wave cycles issued, 45%
// waited, and of the VALU stream ~10% were plain register moves rotating
// the x-queues, ~10% the NaN-propagating residual compares, and SALU work was
// 40% of the VALU count.  Here
//
//   * queues are rings indexed by (step mod Q): the x-loop is unrolled by
//     U = lcm(Q, 3) so every ring index is a compile-time constant and no
//     value is ever moved between registers;
//   * with Q = 4 the T^n plane x+2 is loaded at the start of step x (one full
//     step of latency cover); with Q = 3 it is loaded into the slot stage 0
//     has just freed (the remaining K-1 stages cover it) — fewer VGPRs;
//   * the per-stage residual is a plain v_max_f64 (IEEE max, drops NaN) over
//     the valid region; NaN detection moves to the stored T^{n+K}: a NaN
//     produced at any stage at point p stays at p in every later stage (the
//     centre term) and p is stored by exactly one tile, so if any stored
//     value is NaN all K residual slots are set to NaN and the convergence
//     check faults.  For NaN-free fields the residuals are bit-identical to
//     the single-step kernels' (max of non-negative doubles is exact);
//   * only WZ = 1 tiles (one wave spans the tile's z extent; the MI355X sweep
//     showed z-split tiles lose), so z edges need no LDS.
//
// Tiles, Dirichlet ghosts, deep x halos and the u range are exactly as in
// stencil_tbk.hip (shared TBKArgs geometry, launch_tbr mirrors launch_tbk).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "hip_helpers.hpp"

namespace heat3d {
namespace hip {

struct TBRArgs {
  int64_t sx, sy, origin;  // plane / row strides, element index of owned (0,0,0)
  int blo[3], bhi[3];      // store box
  int ulo, uhi;            // x range where F_{s+1} = FTCS(F_s)
  int uylo, uyhi;          // same in y (box range unless deep y halos)
  int uzlo, uzhi;          // same in z
  int xlo_live, xhi_live;  // x planes present in memory
  int ylo_live, yhi_live;  // y rows present in memory
  int kb0, yb0;            // first column / row of tile (0, 0)
  int zstep, zring;        // tile stride along z, stored column ring
  int nzb, nyb;
  // x schedule (XPlan, kernels_hip.hip): pieces = (tile, x segment of seg
  // planes), segment index slowest.  The first n1 pieces fill whole rounds of
  // resident workgroups; each of the r remaining pieces is cut at `split`
  // into an A part and, if the B flag is set, a B part, dispatched after them,
  // so the last round is filled longest-first instead of leaving CUs idle.
  // Packed (seg | split << 16, r | B << 30): this struct must not grow — at
  // 144 bytes the default fp64 variant starts spilling VGPRs.
  int segsplit;
  int n1, rb;
};

namespace {

constexpr int gcd_c(int a, int b) { return b == 0 ? a : gcd_c(b, a % b); }
constexpr int lcm_c(int a, int b) { return a / gcd_c(a, b) * b; }

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

template <typename Real, int V, bool NTS = false>
__device__ __forceinline__ void stv(Real* p, const Real (&s)[V]) {
  if constexpr (V == 1) {
    if constexpr (NTS) __builtin_nontemporal_store(s[0], p);
    else *p = s[0];
  } else {
    typedef typename VecOf<Real, V>::type Vec;
    Vec t;
#pragma unroll
    for (int v = 0; v < V; ++v) t[v] = s[v];
    if constexpr (NTS) __builtin_nontemporal_store(t, reinterpret_cast<Vec*>(p));
    else *reinterpret_cast<Vec*>(p) = t;
  }
}

}  // namespace

template <typename Real, int V, int R, int WY, int K, int Q, bool NTS>
__global__ __launch_bounds__(64 * WY) void stencil_tbr(const Real* __restrict__ in,
                                                       Real* __restrict__ out, TBRArgs g,
                                                       Real Dx, Real Dy, Real Dz,
                                                       unsigned long long* res,
                                                       const int* done) {
  static_assert(K >= 2 && K <= 6, "temporal depth");
  static_assert(Q == 3 || Q == 4, "T^n ring size");
  constexpr int TZ = 64 * V;
  constexpr int TYB = WY * R;
  constexpr int QS = 3;                 // stage ring: planes x-s-1, x-s, x-s+1
  constexpr int U = lcm_c(Q, QS);       // x-loop unroll making ring indices static
  static_assert(TYB > 2 * (K - 1) && R <= 32, "tile too small");
  // centre-plane bottom/top rows of every stage, double-buffered by step parity
  __shared__ __attribute__((aligned(16))) Real s_row[2][K][WY][2][TZ];
  __shared__ unsigned long long s_red[WY][K];  // per-wave residual maxima
  if (flag_set(done)) return;

  // Blocks are dispatched in index order, round-robin over the 8 XCDs; within
  // each class the index is permuted so that consecutive pieces (neighbouring
  // tiles) land on one XCD and share its L2.
  auto remap = [](int i, int n) {
    const int c = i & 7;
    return c * (n >> 3) + min(c, n & 7) + (i >> 3);
  };
  const int blk = blockIdx.x;
  int pc, part;
  if (blk < g.n1) {
    pc = remap(blk, g.n1);
    part = 0;
  } else if (blk < g.n1 + (g.rb & 0x3fffffff)) {
    const int r = g.rb & 0x3fffffff;
    pc = g.n1 + remap(blk - g.n1, r);
    part = 1;
  } else {
    const int r = g.rb & 0x3fffffff;
    pc = g.n1 + remap(blk - g.n1 - r, r);
    part = 2;
  }
  const int zb = pc % g.nzb;
  const int tq = pc / g.nzb;
  const int ybk = tq % g.nyb;
  const int xs = tq / g.nyb;
  const int nxb = g.bhi[0] - g.blo[0];
  const int seg = g.segsplit & 0xffff, split = g.segsplit >> 16;
  int xlo_p = xs * seg, xhi_p = min(xlo_p + seg, nxb);
  if (part == 1 && (g.rb >> 30)) xhi_p = min(xhi_p, xlo_p + split);
  if (part == 2) xlo_p = min(xlo_p + split, xhi_p);

  // the wave index is uniform: keep it (and every row / plane offset derived
  // from it) in SGPRs, so that a load is an SGPR base + one shared VGPR lane
  // offset instead of a 64-bit VGPR address per row and step
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int tkb = g.kb0 + zb * g.zstep;                 // tile's first column
  const int tyb = g.yb0 + ybk * (TYB - 2 * (K - 1));    // tile's first row
  const int k = tkb + lane * V;
  const int yb = tyb + wave * R;
  const int uylo = g.uylo, uyhi = g.uyhi;
  const int xa = g.blo[0] + xlo_p;
  const int xe = g.blo[0] + xhi_p;
  const int64_t sx = g.sx, sy = g.sy;

  // per-lane column masks: in the box, stored.  The residual's column
  // validity (stage s: columns [s, TZ - s) of the tile) is applied once, to
  // per-column accumulators at the end (kColAcc), instead of per point — except
  // for V > 1 in 16-wave groups, where K x V accumulators overflow the
  // 128-VGPR budget: those keep per-point masks.
  constexpr bool kColAcc = V == 1 || WY * 64 <= 512;
  constexpr int VA = kColAcc ? V : 1;  // residual accumulators per stage
  // zin: column in the update range (the box, or wider into deep z halos);
  // zst: column stored by this tile (in the box)
  bool zin[V], zst[V];
  bool allst = true;
  bool lres[kColAcc ? 1 : K][V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int kk = k + v, cp = lane * V + v;
    zin[v] = kk >= g.uzlo && kk < g.uzhi;
    zst[v] = kk >= g.blo[2] && kk < g.bhi[2] && cp >= g.zring && cp < TZ - g.zring;
    allst &= zst[v];
    if constexpr (!kColAcc)
#pragma unroll
      for (int s = 0; s < K; ++s)
        lres[s][v] = zin[v] && cp >= s && cp < TZ - s && kk >= g.blo[2] - (K - 1 - s) && kk < g.bhi[2] + (K - 1 - s);
  }
  const int64_t wbase = g.origin + (int64_t)yb * sy + tkb;
  const Real* __restrict__ inw = in + wbase;
  Real* __restrict__ outw = out + wbase;
  const int lo_off = lane * V;
  // Loads are unconditional, with rows clamped to the ghosted layout
  // [ylo_live, yhi_live] and planes to [xlo_live, xhi_live]: a clamped value is a real (finite)
  // field value standing in for a point outside the layout, and such points
  // only ever feed copies outside the update box, never a stored value or a
  // residual (no zero-fill moves, no per-row branches in the step).
  // (32-bit: |row offset| <= (R + 1) * sy < 2^31, checked in launch_tbr)
  auto crow = [&](int row) { return (min(max(row, g.ylo_live), g.yhi_live) - yb) * (int)sy; };
  int roff[R];
#pragma unroll
  for (int r = 0; r < R; ++r) roff[r] = crow(yb + r);
  const int roff_lo = crow(yb - 1), roff_hi = crow(yb + R);
  const int er = lane & 31;
  const bool eload = er < R;
  const int eoff = (min(max(yb + er, g.ylo_live), g.yhi_live) - yb) * (int)sy + (lane < 32 ? -1 : TZ);  // halo column of row er
  const bool has_lo = wave > 0, has_hi = wave + 1 < WY;

  // rings: T^n plane p and its y/z halo live in slot (p - x0 + 1) mod Q;
  // F_{s+1} produced at step x lives in f[s][(x - x0) mod 3]
  Real q[Q][R][V];
  Real hb[Q][V], ht[Q][V], ed[Q];
  Real f[K - 1][QS][R][V];

  auto load_plane = [&](int x, Real (&d)[R][V], Real (&b)[V], Real (&tp)[V], Real& e) {
    const Real* pl0 = inw + (int64_t)min(max(x, g.xlo_live), g.xhi_live) * sx;
#pragma unroll
    for (int r = 0; r < R; ++r) ldv<Real, V>(pl0 + roff[r] + lo_off, d[r]);
    if (!has_lo) ldv<Real, V>(pl0 + roff_lo + lo_off, b);
    if (!has_hi) ldv<Real, V>(pl0 + roff_hi + lo_off, tp);
    // halo columns: lanes r and 32 + r (r < R) only — all 64 lanes would touch
    // 64 different rows' cache lines per plane
    if (eload) e = pl0[eoff];
  };

  const int x0 = xa - (K - 1);
  const int xlast = xe + K - 2;
#pragma unroll
  for (int i = 0; i < 3; ++i) load_plane(x0 - 1 + i, q[i], hb[i], ht[i], ed[i]);
#pragma unroll
  for (int s = 0; s < K - 1; ++s)
#pragma unroll
    for (int i = 0; i < QS; ++i)
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int v = 0; v < V; ++v) f[s][i][r][v] = Real(0);

  Real m[K][VA];  // residual maxima in the field's precision (widened at the end)
  bool nan_seen[VA];
#pragma unroll
  for (int v = 0; v < VA; ++v) {
    nan_seen[v] = false;
#pragma unroll
    for (int s = 0; s < K; ++s) m[s][v] = Real(0);
  }
  int par = 0;

  // whole chunks of U steps (no early exit: the unrolled body needs a constant
  // trip count).  Steps past xlast only compute planes beyond the segment's
  // widened box: nothing of them is stored or counted in a residual;
  // launch_tbr sizes segments so that only a box's last segment pads.
  for (int xb = x0; xb <= xlast; xb += U) {
#pragma unroll
    for (int ph = 0; ph < U; ++ph) {
      const int x = xb + ph;
      const int sM = ph % Q, sC = (ph + 1) % Q, sP = (ph + 2) % Q;
      const int fw = ph % QS, fc = (ph + QS - 1) % QS, fm = (ph + QS - 2) % QS;
      // T^n plane x+2 (Q = 4: its slot is free at the start of the step)
      if constexpr (Q == 4) {
        constexpr int sN = 3;
        load_plane(x + 2, q[(ph + sN) % Q], hb[(ph + sN) % Q], ht[(ph + sN) % Q], ed[(ph + sN) % Q]);
      }
      // ---- publish the centre rows of every stage
#pragma unroll
      for (int s = 0; s < K; ++s) {
        Real (&C)[R][V] = s == 0 ? q[sC] : f[s > 0 ? s - 1 : 0][fc];
        stv<Real, V>(&s_row[par][s][wave][0][lane * V], C[0]);
        stv<Real, V>(&s_row[par][s][wave][1][lane * V], C[R - 1]);
      }
      __syncthreads();

#pragma unroll
      for (int s = 0; s < K; ++s) {
        Real (&M)[R][V] = s == 0 ? q[sM] : f[s > 0 ? s - 1 : 0][fm];
        Real (&C)[R][V] = s == 0 ? q[sC] : f[s > 0 ? s - 1 : 0][fc];
        Real (&P)[R][V] = s == 0 ? q[sP] : f[s > 0 ? s - 1 : 0][fw];
        const int p = x - s;  // plane produced by this stage
        const bool xin = p >= g.ulo && p < g.uhi;
        const bool xval = x >= xa - K + 2 * s + 1;  // its inputs were valid
        Real lo[V], hi[V];
        if (has_lo) {
          ldv<Real, V>(&s_row[par][s][wave - 1][1][lane * V], lo);
        } else {
#pragma unroll
          for (int v = 0; v < V; ++v) lo[v] = s == 0 ? hb[sC][v] : C[0][v];
        }
        if (has_hi) {
          ldv<Real, V>(&s_row[par][s][wave + 1][0][lane * V], hi);
        } else {
#pragma unroll
          for (int v = 0; v < V; ++v) hi[v] = s == 0 ? ht[sC][v] : C[R - 1][v];
        }
        if (s < K - 1) {
          Real (&N)[R][V] = f[s < K - 1 ? s : 0][fw];
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int row = yb + r, rp = wave * R + r;
            const bool yin = xin && row >= uylo && row < uyhi;
            // padded steps past xlast compute planes beyond the sweep's box
            // widened by K-1-s (possibly from halo planes still being
            // exchanged): never counted
            // counted: valid inputs (tile-relative), and within the box
            // widened by K-1-s — beyond it a stage-s value may come from
            // held or still-arriving halo data (deep y halos)
            const bool rres = yin && xval && x <= xlast && rp >= s && rp < TYB - s &&
                              row >= g.blo[1] - (K - 1 - s) && row < g.bhi[1] + (K - 1 - s);
            const Real left = s == 0 ? readlane(ed[sC], r) : Real(0);
            const Real right = s == 0 ? readlane(ed[sC], 32 + r) : Real(0);
            const Real* ym = r == 0 ? lo : C[r > 0 ? r - 1 : 0];
            const Real* yp = r == R - 1 ? hi : C[r + 1 < R ? r + 1 : 0];
#pragma unroll
            for (int v = 0; v < V; ++v) {
              // stage 0: the tile's halo columns enter lanes 0 / 63; later
              // stages: those lanes are outside the valid region anyway
              const Real zm = v > 0 ? C[r][v > 0 ? v - 1 : 0]
                              : s == 0 ? dpp_shr1(left, C[r][V - 1]) : dpp_shr1z(C[r][V - 1]);
              const Real zp = v < V - 1 ? C[r][v + 1 < V ? v + 1 : 0]
                              : s == 0 ? dpp_shl1(right, C[r][0]) : dpp_shl1z(C[r][0]);
              const Real nv = ftcs<Real>(C[r][v], M[r][v], P[r][v], ym[v], yp[v], zm, zp, Dx, Dy, Dz);
              N[r][v] = (yin && zin[v]) ? nv : C[r][v];
              if (rres) {
                const Real d = resid_abs_r(nv, C[r][v]);
                if constexpr (kColAcc) m[s][v < VA ? v : 0] = fmax(m[s][v < VA ? v : 0], d);
                else m[s][0] = fmax(m[s][0], lres[kColAcc ? 0 : s][v] ? d : Real(0));
              }
            }
          }
        } else {
          // final stage: T^{n+K}(p) on the stored region
          if (p >= xa && p < xe) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
              const int row = yb + r, rp = wave * R + r;
              const bool rst = row >= g.blo[1] && row < g.bhi[1] && rp >= K - 1 && rp < TYB - (K - 1);
              if (!rst) continue;
              const Real* ym = r == 0 ? lo : C[r > 0 ? r - 1 : 0];
              const Real* yp = r == R - 1 ? hi : C[r + 1 < R ? r + 1 : 0];
              Real nv[V];
#pragma unroll
              for (int v = 0; v < V; ++v) {
                const Real zm = v > 0 ? C[r][v > 0 ? v - 1 : 0] : dpp_shr1z(C[r][V - 1]);
                const Real zp = v < V - 1 ? C[r][v + 1 < V ? v + 1 : 0] : dpp_shl1z(C[r][0]);
                nv[v] = ftcs<Real>(C[r][v], M[r][v], P[r][v], ym[v], yp[v], zm, zp, Dx, Dy, Dz);
                const Real d = resid_abs_r(nv[v], C[r][v]);
                if constexpr (kColAcc) {
                  m[s][v < VA ? v : 0] = fmax(m[s][v < VA ? v : 0], d);
                  nan_seen[v < VA ? v : 0] |= nv[v] != nv[v];
                } else {
                  m[s][0] = fmax(m[s][0], zst[v] ? d : Real(0));
                  nan_seen[0] |= zst[v] && nv[v] != nv[v];
                }
              }
              Real* dst = outw + ((int64_t)p * sx + (int64_t)r * sy) + lo_off;
              if (allst) {
                stv<Real, V, NTS>(dst, nv);
              } else {
#pragma unroll
                for (int v = 0; v < V; ++v)
                  if (zst[v]) dst[v] = nv[v];
              }
            }
          }
        }
        // T^n plane x+2 into the slot stage 0 has just freed (Q = 3)
        if constexpr (Q == 3) {
          if (s == 0) load_plane(x + 2, q[sM], hb[sM], ht[sM], ed[sM]);
        }
      }
      par ^= 1;
    }
  }
  if (res) {
    bool nan_any = false;
    double mm[K];
#pragma unroll
    for (int s = 0; s < K; ++s) mm[s] = 0.0;
#pragma unroll
    for (int v = 0; v < VA; ++v) {
      const int cp = lane * V + v;
      nan_any |= (!kColAcc || zst[v]) && nan_seen[v];
#pragma unroll
      for (int s = 0; s < K; ++s) {
        const int kk = k + v;
        const bool ok = !kColAcc || (s == K - 1 ? zst[v]
                                                : (zin[v] && cp >= s && cp < TZ - s && kk >= g.blo[2] - (K - 1 - s) &&
                                                   kk < g.bhi[2] + (K - 1 - s)));
        mm[s] = fmax(mm[s], ok ? (double)m[s][v] : 0.0);
      }
    }
    residual_commit_block<WY, K>(res, mm, nan_any, s_red);
  }
}

template <typename Real, int V, int R, int WY, int K, int Q, bool NTS>
static void launch_tbr(const StencilParams& p, const KernelSpec& ks, hipStream_t s) {
  const Box& b = p.box;
  constexpr int TZ = 64 * V;
  constexpr int TYB = WY * R;
  const Layout& L = p.L;
  HEAT3D_CHECK(L.gx >= 1 && L.n[0] + 2 * L.gx < (1LL << 30) && L.n[1] + 2 * L.gy < (1LL << 30) &&
                   L.sy * (TYB + 2 * L.gy) < (1LL << 31),
               "tbr: extents exceed 32-bit tile coordinates");
  TBRArgs g;
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
  g.ylo_live = (int)-L.gy;
  g.yhi_live = (int)(L.n[1] + L.gy - 1);
  const bool wy = p.uy[1] >= p.uy[0], wz = p.uz[1] >= p.uz[0];
  g.uylo = (int)(wy ? p.uy[0] : b.lo[1]);
  g.uyhi = (int)(wy ? p.uy[1] : b.hi[1]);
  g.uzlo = (int)(wz ? p.uz[0] : b.lo[2]);
  g.uzhi = (int)(wz ? p.uz[1] : b.hi[2]);
  // stage 0 reads one row / column beyond the update range
  HEAT3D_CHECK(g.uylo - 1 >= -L.gy && g.uyhi <= L.n[1] + L.gy && g.uylo <= b.lo[1] && g.uyhi >= b.hi[1] &&
                   g.uzlo - 1 >= -L.gz && g.uzhi <= L.n[2] + L.gz && g.uzlo <= b.lo[2] && g.uzhi >= b.hi[2],
               "tbr: y/z update range outside the ghosted layout");
  HEAT3D_CHECK(g.ulo - 1 >= g.xlo_live && g.uhi <= g.xhi_live && g.ulo <= b.lo[0] &&
                   g.uhi >= b.hi[0],
               "tbr: u range [" << g.ulo << "," << g.uhi << ") outside the ghosted layout");
  g.zring = ((K - 1 + V - 1) / V) * V;
  g.zstep = TZ - 2 * g.zring;
  HEAT3D_CHECK(g.zstep > 0, "tbr: tile too narrow for depth " << K);
  int64_t kb0 = b.lo[2] - g.zring;
  kb0 = (kb0 >= 0 ? kb0 / V : -((-kb0 + V - 1) / V)) * V;  // floor to a multiple of V
  g.kb0 = (int)kb0;
  g.yb0 = (int)(b.lo[1] - (K - 1));
  const int64_t zspan = b.hi[2] - (kb0 + g.zring);
  g.nzb = (int)std::max<int64_t>(1, (zspan + g.zstep - 1) / g.zstep);
  const int ystep = TYB - 2 * (K - 1);
  g.nyb = (int)std::max<int64_t>(1, (b.extent(1) + ystep - 1) / ystep);
  static const int slots =  // magic static: thread-safe under --gpus N
      device_slots(reinterpret_cast<const void*>(&stencil_tbr<Real, V, R, WY, K, Q, NTS>), 64 * WY);
  const int64_t ntiles = (int64_t)g.nzb * g.nyb;
  const int64_t nxb = b.extent(0);
  constexpr int U = Q == 3 ? 3 : 12;  // a piece runs its steps in chunks of U = lcm(Q, 3)
  XPlan xp;
  if (ks.L > 0) {
    xp = fixed_xplan(nxb, ntiles, ks.L);  // explicit segment length, no split
  } else {
    xp = plan_x(nxb, ntiles, slots, 2 * (K - 1), U, ks.L < 0);
  }
  HEAT3D_CHECK(xp.seg < (1 << 15) && xp.split < (1 << 15) && xp.r < (1 << 30), "tbr: x plan out of range");
  g.segsplit = xp.seg | (xp.split << 16);
  g.n1 = xp.n1;
  g.rb = xp.r | (xp.nb2 > 0 ? (1 << 30) : 0);
  const int64_t nblocks = (int64_t)xp.n1 + xp.r + xp.nb2;
  HEAT3D_CHECK(nblocks < (1LL << 31) && nblocks >= 1, "tbr: bad block count " << nblocks);
  if (std::getenv("HEAT3D_TRACE"))
    std::fprintf(stderr, "[heat3d trace] tbr K=%d box x %lld: seg=%d tiles=%dx%d blocks=%lld (n1=%d r=%d split=%d nb2=%d)\n",
                 K, (long long)nxb, xp.seg, g.nzb, g.nyb, (long long)nblocks, xp.n1, xp.r, xp.split, xp.nb2);
  HEAT3D_CHECK(!p.state || p.slot + K <= kResidualSlots, "tbr: residual slots " << p.slot << "+" << K);
  // Variants whose registers spill are slow and, with the ring fully unrolled,
  // have been miscompiled on ROCm 7.2 (tr4:1:4:1:16:0:4 produced wrong row-0
  // values); refuse them unless explicitly allowed.
  static const int spill = [] {
    hipFuncAttributes a{};
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&stencil_tbr<Real, V, R, WY, K, Q, NTS>)) == hipSuccess
               ? (int)a.localSizeBytes
               : 0;
  }();
  static const bool allow = std::getenv("HEAT3D_ALLOW_SPILL") && std::getenv("HEAT3D_ALLOW_SPILL")[0] == '1';
  HEAT3D_CHECK(spill == 0 || allow, "tbr variant " << ks.str() << " spills " << spill
                                                   << " B of registers per lane; pick a smaller tile / ring "
                                                      "(HEAT3D_ALLOW_SPILL=1 overrides)");
  unsigned long long* r = p.state ? &p.state->residual[p.slot] : nullptr;
  const int* done = p.state ? &p.state->done : nullptr;
  hipLaunchKernelGGL((stencil_tbr<Real, V, R, WY, K, Q, NTS>), dim3((unsigned)nblocks), dim3(64 * WY), 0, s,
                     static_cast<const Real*>(p.in), static_cast<Real*>(p.out), g, (Real)p.D[0],
                     (Real)p.D[1], (Real)p.D[2], r, done);
  HIPK_CHECK(hipGetLastError());
}

template <typename Real>
static void dispatch_tbr(const StencilParams& p, const KernelSpec& k, hipStream_t s) {
  const int K = k.K;
  const KernelSpec r = k.resolved(sizeof(Real) == 8 ? DType::F64 : DType::F32);
  const int V = r.V, R = r.R, WY = r.WY, Q = r.NT;
  const bool nts = r.O == 1;  // 8th spec field: 1 = non-temporal T^{n+K} stores
  HEAT3D_CHECK(r.WZ == 1, "tbr kernels span the tile's z extent with one wave (WZ = 1)");
#define H3D_TBR(VV, RR, YY, KK, QQ)                                 \
  if (V == VV && R == RR && WY == YY && K == KK && Q == QQ && !nts) { \
    launch_tbr<Real, VV, RR, YY, KK, QQ, false>(p, k, s);             \
    return;                                                         \
  }
  // variants also built with non-temporal output stores
#define H3D_TBRN(VV, RR, YY, KK, QQ)                                \
  H3D_TBR(VV, RR, YY, KK, QQ)                                       \
  if (V == VV && R == RR && WY == YY && K == KK && Q == QQ && nts) {  \
    launch_tbr<Real, VV, RR, YY, KK, QQ, true>(p, k, s);              \
    return;                                                         \
  }
#define H3D_TBR_Q(VV, RR, YY, KK) H3D_TBR(VV, RR, YY, KK, 3) H3D_TBR(VV, RR, YY, KK, 4)
  H3D_TBRN(1, 3, 16, 3, 3) H3D_TBRN(1, 6, 8, 3, 3) H3D_TBRN(2, 2, 16, 2, 3)
  H3D_TBR_Q(1, 4, 16, 2) H3D_TBR_Q(1, 4, 16, 3) H3D_TBR_Q(1, 4, 16, 4)
  H3D_TBR_Q(1, 4, 8, 3) H3D_TBR_Q(1, 4, 8, 4) H3D_TBR(1, 6, 8, 4, 3) H3D_TBR(1, 3, 16, 4, 3)
  H3D_TBR(1, 3, 16, 3, 4) H3D_TBR_Q(1, 2, 16, 3) H3D_TBR_Q(1, 3, 16, 2)
  H3D_TBR_Q(1, 2, 16, 2) H3D_TBR_Q(2, 2, 8, 2) H3D_TBR(2, 2, 16, 2, 4)
  H3D_TBR(1, 2, 16, 4, 3) H3D_TBR(2, 2, 8, 3, 3) H3D_TBR(1, 5, 8, 3, 3)
  if constexpr (sizeof(Real) == 4) {
    H3D_TBRN(2, 4, 8, 3, 3) H3D_TBRN(1, 4, 8, 4, 3) H3D_TBR(2, 4, 8, 3, 4)
    H3D_TBR_Q(2, 4, 8, 4) H3D_TBR_Q(2, 4, 16, 3) H3D_TBR_Q(2, 4, 8, 2)
  }
#undef H3D_TBR_Q
#undef H3D_TBRN
#undef H3D_TBR
  HEAT3D_THROW("unsupported tbr kernel variant V=" << V << " R=" << R << " WY=" << WY << " K=" << K
                                                   << " Q=" << Q);
}

void stencil_ring(DType t, const StencilParams& p, const KernelSpec& k, void* stream) {
  if (p.box.empty()) return;
  if (t == DType::F64) dispatch_tbr<double>(p, k, S(stream));
  else dispatch_tbr<float>(p, k, S(stream));
}

void sweep(DType t, const StencilParams& p, const KernelSpec& k, void* stream) {
  if (p.xpair > 0 && k.kind != KernelSpec::TBL) {
    // two x slabs, one launch each (only the lean kernel pairs them)
    StencilParams a = p;
    a.xpair = 0;
    sweep(t, a, k, stream);
    a.box.lo[0] += p.xpair;
    a.box.hi[0] += p.xpair;
    sweep(t, a, k, stream);
    return;
  }
  switch (k.kind) {
    case KernelSpec::TBR: stencil_ring(t, p, k, stream); break;
    case KernelSpec::TBL: stencil_lean(t, p, k, stream); break;
    case KernelSpec::TBK: stencil_multi(t, p, k, stream); break;
    case KernelSpec::TB2: stencil2(t, p, k, stream); break;
    default: HEAT3D_THROW("sweep needs a multi-step kernel (tb2 | tbk2 | tb3..tb6 | tr2..tr6 | tl2..tl6)");
  }
}

}  // namespace hip
}  // namespace heat3d
