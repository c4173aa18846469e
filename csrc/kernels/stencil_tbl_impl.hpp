// heat3d-mi355x — the lean K-step sweep kernel and its launcher (shared by
// stencil_tbl.hip, which dispatches, and the stencil_tbl_part*.hip units, which
// instantiate the variants listed in stencil_tbl_variants.inc in parallel).
#pragma once

// heat3d-mi355x — K-step temporally blocked FTCS kernel, lean form ("tl").
//
// Same contract as stencil_tbr.hip (one HBM sweep turns T^n into T^{n+K};
// every point goes through the reference update heat3D.cu:128-131 with the
// arithmetic of kernels.hpp ftcs_update, so fields and all K residuals are
// bitwise identical to K single steps), re-planned after the ISA and
// counters of the ring kernel on MI355X: ~40% of its VALU stream per point
// update was overhead (SGPR spill reloads through v_readlane, read-lanes of
// separately loaded halo columns, per-point validity selects), which is what
// kept a 4-step variant from fitting 16 waves x 128 VGPRs.  Here
//
//   * halos are ordinary lanes and rows: a tile loads 64 consecutive columns
//     (one wave wide) and WY*R rows; stage s output is valid on lanes
//     [s+1, 63-s) and tile rows [s+1, TY-s-1); T^{n+K} is stored on
//     lanes [K, 64-K) x rows [K, TY-K).  z neighbours are zero-filling DPP
//     shifts (no "old" operand, no read-lanes, no halo registers); the tile's
//     outer rows take a wave's own edge row from LDS as a stand-in (finite,
//     outside every stored / counted point);
//   * residuals accumulate per lane without masks; the per-lane validity of
//     stage s (cone, update range, box widened by K-1-s) is applied once, at
//     the end;
//   * a wave whose rows are inside the box, the update range and the tile's
//     cone runs a mask-free step ("fast"): 9 fp64 ops for the update, 2 for
//     the residual, 4 DPP moves.  Steps of the pipeline fill / drain, tiles on
//     a Dirichlet face and waves on the tile's edge run the masked step (the
//     same code with uniform x / y conditions and a per-lane z mask); the
//     choice is a uniform branch per step, both forms hold one barrier;
//   * loads are an SGPR row base plus one lane offset (global_load saddr
//     form), clamped rows / planes fold into the SGPR base.
//
// Tiles advance along z by 64 - 2K columns and along y by WY*R - 2K rows;
// workgroups march along x segments (XPlan, as the ring kernel), dispatched
// XCD-aware.  y rows of each stage's centre plane go through LDS once per
// step (double-buffered by step parity: one barrier per step).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <map>
#include <mutex>
#include <cstdlib>
#include <type_traits>

#include "hip_helpers.hpp"

namespace heat3d {
namespace hip {

struct TBLArgs {
  int64_t sx, sy, origin;      // plane / row strides, element index of owned (0,0,0)
  int blo[3], bhi[3];          // store box
  int ulo, uhi, uylo, uyhi;    // update ranges (x, y)
  int uzlo, uzhi;              // update range (z)
  int xlo_live, xhi_live;      // x planes present in memory
  int ylo_live, yhi_live;      // y rows present in memory
  int c00, r00;                // first loaded column / row of tile (0, 0)
  int nzb, nyb;
  int segsplit, n1, rb;        // x plan: seg | split << 16, whole pieces, r | split-tail << 30
  int zs;                      // tile stride along z = stored columns per tile (<= 64 - 2K)
  DeviceState* fst;            // fused convergence check (fused_check_tail): state, nullptr = off
  int fslot, fblocks;          // its first residual slot and the grid's workgroup count
};

namespace {

constexpr int gcd_l(int a, int b) { return b == 0 ? a : gcd_l(b, a % b); }
constexpr int lcm_l(int a, int b) { return a / gcd_l(a, b) * b; }

__device__ __forceinline__ int sgpr(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Raw buffer resource over one x plane (SGPRs: 48-bit base, no range limit;
// dword 3 = the gfx9 untyped-buffer word).  A row load / store is then
// buffer_{load,store}_dwordx2 v, v_lane_bytes, s[rsrc], s_row_bytes offen:
// no per-lane 64-bit address registers, no address VALU.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)0xffffffff, 0x00020000);
}
template <typename Real>
__device__ __forceinline__ Real buf_load(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  if constexpr (sizeof(Real) == 8)
    return __builtin_bit_cast(Real, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
  else
    return __builtin_bit_cast(Real, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
// AUX = cache policy bits of the store (2 = nt: streaming, not kept in L2)
template <typename Real, int AUX = 0>
__device__ __forceinline__ void buf_store(Real v, __amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  if constexpr (sizeof(Real) == 8)
    __builtin_amdgcn_raw_buffer_store_b64(
        __builtin_bit_cast(unsigned __attribute__((ext_vector_type(2))), v), r, voff, soff, AUX);
  else
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, voff, soff, AUX);
}

// f(integral_constant<int, I>) for I = B .. E-1, unrolled at compile time
template <int B, int E, typename Fn>
__device__ __forceinline__ void static_for(Fn&& fn) {
  if constexpr (B < E) {
    fn(std::integral_constant<int, B>{});
    static_for<B + 1, E>(fn);
  }
}

}  // namespace

// NTS: store cache policy; SW: swapped axes (x planes are the tile rows, the
// kernel marches y): the row neighbours are the x terms of the update.
template <typename Real, int R, int WY, int K, int Q, int NTS = 0, bool SW = false>
__global__ __launch_bounds__(64 * WY) void stencil_tbl(const Real* __restrict__ in, Real* __restrict__ out,
                                                       TBLArgs g, Real Dx, Real Dy, Real Dz,
                                                       unsigned long long* res, const int* done) {
  static_assert(K >= 2 && K <= 6, "temporal depth");
  // T^n ring: Q = 3 loads plane x+2 into the slot stage 0 frees at step x
  // ((K-1)/K of a step of latency cover); Q >= 4 loads plane x+Q-2 at the
  // start of step x (Q-3 steps of cover)
  static_assert(Q == 3 || Q == 4 || Q == 6, "T^n ring size");
  constexpr int TY = WY * R;
  constexpr int YS = TY - 2 * K;   // tile stride along y (stored rows)
  // x-loop unroll making every ring index and the LDS parity static
  constexpr int U = lcm_l(lcm_l(Q, 3), 2);
  static_assert(YS > 0 && R <= 16, "tile too small for depth K");
  // NTS bit kResidualLastOnly: only the last step's residual (monotone check)
  constexpr bool RL = (NTS & kResidualLastOnly) != 0;
  constexpr int ST = NTS & ~kResidualLastOnly;  // the stores' cache-policy bits
  __shared__ __attribute__((aligned(16))) Real s_row[2][K][WY][2][64];
  static_assert(sizeof(s_row) >= WY * K * sizeof(unsigned long long), "residual scratch");
  if (flag_set(done)) {
    if (g.fst) fused_check_tail<K, RL>(g.fst, g.fslot, g.fblocks);
    return;
  }

  // piece decode: blocks dealt round-robin over the 8 XCDs; consecutive
  // pieces (neighbouring tiles) share an XCD's L2 (same encoding as tbr)
  auto remap = [](int i, int n) {
    const int c = i & 7;
    return c * (n >> 3) + min(c, n & 7) + (i >> 3);
  };
  const int blk = blockIdx.x;
  const int zs = g.zs;
  const int ntile = g.nzb * g.nyb;
  const int nxb = g.bhi[0] - g.blo[0];
  // This workgroup's piece: plane steps [w, wend) of the tile-major list
  // (tile t, plane x) -> t * nxb + x, one piece per block, x segments of
  // `seg` planes (plan_x: whole rounds of pieces, then a split tail); each
  // piece pays the 2(K-1)-plane pipeline fill.  (The persistent walk of round 3,
  // every block a contiguous 1/n of the list, measured 18-22% slower on
  // MI355X: the x plan's concurrent workgroups sweep neighbouring tiles over
  // the same x planes, so their overlapping halo rows are L2 hits.)
  int64_t w, wend;
  {
    int pc, part;
    const int rr = g.rb & 0x3fffffff;
    if (blk < g.n1) {
      pc = remap(blk, g.n1);
      part = 0;
    } else if (blk < g.n1 + rr) {
      pc = g.n1 + remap(blk - g.n1, rr);
      part = 1;
    } else {
      pc = g.n1 + remap(blk - g.n1 - rr, rr);
      part = 2;
    }
    const int xs = pc / ntile;
    const int tt = pc - xs * ntile;
    const int seg = g.segsplit & 0xffff, split = g.segsplit >> 16;
    int xlo_p = xs * seg, xhi_p = min(xlo_p + seg, nxb);
    if (part == 1 && (g.rb >> 30)) xhi_p = min(xhi_p, xlo_p + split);
    if (part == 2) xlo_p = min(xlo_p + split, xhi_p);
    w = (int64_t)tt * nxb + xlo_p;
    wend = (int64_t)tt * nxb + xhi_p;
  }

  // tile order: z fastest
  const int tt = (int)(w / nxb);
  const int xlo_p = (int)(w - (int64_t)tt * nxb);
  const int xhi_p = (int)min((int64_t)nxb, xlo_p + (wend - w));
  const int zb = tt % g.nzb, ybk = tt / g.nzb;

  const int wave = sgpr(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int c0 = g.c00 + zb * zs;         // tile's first loaded column
  const int r0 = g.r00 + ybk * YS;          // tile's first loaded row
  const int yb = r0 + wave * R;             // this wave's first row
  const int col = c0 + lane;
  const int xa = g.blo[0] + xlo_p, xe = g.blo[0] + xhi_p;
  const int x0 = xa - (K - 1), xlast = xe + K - 2;
  const int64_t sx = g.sx;

  // ---- uniform (per wave) classification
  const bool zfast = c0 >= g.uzlo && c0 + 64 <= g.uzhi;
  const bool wrows = wave * R >= K && wave * R + R <= TY - K && yb >= g.uylo && yb + R <= g.uyhi &&
                     yb >= g.blo[1] && yb + R <= g.bhi[1];
  const bool wfast = zfast && wrows;
  // steps whose every stage is valid, updated, counted and (last stage) stored
  const int xf_lo = max(max(x0 + 2 * (K - 1), g.ulo + K - 1), g.blo[0] + K - 1);
  const int xf_hi = min(min(xlast, g.uhi - 1), g.bhi[0] + K - 2);

  // masked form, per row r (uniform, one SGPR): bit r = row in the update
  // range, bit R + r = stored row, bit 2R + s*R + r = row counted at stage s
  // (64-bit when the rows x stages outgrow one SGPR: 8-wave tiles of 6 rows)
  using YMask = std::conditional_t<(2 * R + K * R <= 32), unsigned, unsigned long long>;
  static_assert(2 * R + K * R <= 64, "row mask bits");
  YMask ybits = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int row = yb + r, rp = wave * R + r;
    if (row >= g.uylo && row < g.uyhi) ybits |= YMask(1) << r;
    if (rp >= K && rp < TY - K && row >= g.blo[1] && row < g.bhi[1]) ybits |= YMask(1) << (R + r);
#pragma unroll
    for (int s = 0; s < K; ++s)
      if (row >= g.uylo && row < g.uyhi && rp >= s + 1 && rp < TY - s - 1 && row >= g.blo[1] - (K - 1 - s) &&
          row < g.bhi[1] + (K - 1 - s))
        ybits |= YMask(1) << (2 * R + s * R + r);
  }
  if constexpr (sizeof(YMask) == 4) {
    ybits = (unsigned)sgpr((int)ybits);
  } else {
    ybits = ((YMask)(unsigned)sgpr((int)(ybits >> 32)) << 32) | (unsigned)sgpr((int)(unsigned)ybits);
  }

  // per-lane masks (constant over the piece)
  const bool zin = col >= g.uzlo && col < g.uzhi;
  const bool zst = lane >= K && lane < K + zs && col >= g.blo[2] && col < g.bhi[2];

  // ---- addressing: uniform base of row yb, column c0; clamped row offsets
  // (uniform by construction: kernel arguments and the readfirstlane'd wave
  // index; pointers stay in the global address space)
  // Loads: base at the wave's first clamped row; a buffer soffset is an
  // unsigned 32-bit value, so every row offset must be >= 0 (clamping is
  // monotonic: clamp(yb + r) >= clamp(yb)).  Stores only touch stored rows,
  // which are real rows at or after yb.
  auto yclamp = [&](int row) { return min(max(row, g.ylo_live), g.yhi_live); };
  const int ybc = yclamp(yb);
  const Real* __restrict__ inw = in + (g.origin + (int64_t)ybc * g.sy + c0);
  Real* __restrict__ outw = out + (g.origin + (int64_t)yb * g.sy + c0);
  // row byte offsets (clamped rows fold in), 0 <= roff < 2^31: checked in launch_tbl
  int roff[R];
#pragma unroll
  for (int r = 0; r < R; ++r) roff[r] = sgpr((yclamp(yb + r) - ybc) * (int)g.sy * (int)sizeof(Real));
  const int sy_b = (int)g.sy * (int)sizeof(Real);
  const unsigned lane_b = (unsigned)lane * (unsigned)sizeof(Real);

  Real q[Q][R];              // T^n ring: plane p in slot (p - x0 + 1) mod Q
  Real f[K - 1][3][R];       // F_{s+1}(p) in f[s][(p + s) mod 3]
  Real m[K];                 // per-lane residual maxima (field precision, widened at the end)
  bool nan_seen = false;
#pragma unroll
  for (int s = 0; s < K; ++s) m[s] = Real(0);
#pragma unroll
  for (int s = 0; s < K - 1; ++s)
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int r = 0; r < R; ++r) f[s][i][r] = Real(0);

  auto load_plane = [&](int x, Real (&d)[R]) {
    const int xc = min(max(x, g.xlo_live), g.xhi_live);
    const __amdgpu_buffer_rsrc_t rs = plane_rsrc(inw + (int64_t)xc * sx);
#pragma unroll
    for (int r = 0; r < R; ++r) d[r] = buf_load<Real>(rs, lane_b, roff[r]);
  };
  constexpr int NPRE = Q == 3 ? 3 : Q - 1;  // planes resident / in flight before step x0
#pragma unroll
  for (int i = 0; i < NPRE; ++i) load_plane(x0 - 1 + i, q[i]);

  // One plane step.  FAST: every condition below is known true.
  auto step = [&](auto fast_tag, const int x, auto ph_tag) {
    constexpr bool FAST = decltype(fast_tag)::value;
    constexpr int ph = decltype(ph_tag)::value;
    constexpr int sM = ph % Q, sC = (ph + 1) % Q, sP = (ph + 2) % Q;
    constexpr int fw = ph % 3, fc = (ph + 2) % 3, fm = (ph + 1) % 3;
    constexpr int par = ph & 1;  // LDS buffer (U is even)
    if constexpr (Q >= 4) load_plane(x + Q - 2, q[(ph + Q - 1) % Q]);
    // publish the edge rows of every stage's centre plane
#pragma unroll
    for (int s = 0; s < K; ++s) {
      const Real(&C)[R] = s == 0 ? q[sC] : f[s > 0 ? s - 1 : 0][fc];
      s_row[par][s][wave][0][lane] = C[0];
      s_row[par][s][wave][1][lane] = C[R - 1];
    }
    __syncthreads();
    const int wl = max(wave - 1, 0), wh = min(wave + 1, WY - 1);
#pragma unroll
    for (int s = 0; s < K; ++s) {
      Real(&M)[R] = s == 0 ? q[sM] : f[s > 0 ? s - 1 : 0][fm];
      Real(&C)[R] = s == 0 ? q[sC] : f[s > 0 ? s - 1 : 0][fc];
      Real(&P)[R] = s == 0 ? q[sP] : f[s > 0 ? s - 1 : 0][fw];
      const Real lo = s_row[par][s][wl][1][lane];
      const Real hi = s_row[par][s][wh][0][lane];
      const int p = x - s;
      // masked form: uniform x conditions of this stage
      bool xin = true, xcnt = true, xst = true;
      if constexpr (!FAST) {
        xin = p >= g.ulo && p < g.uhi;
        xcnt = xin && x >= x0 + 2 * s && x <= xlast && p >= g.blo[0] - (K - 1 - s) && p < g.bhi[0] + (K - 1 - s);
        xst = p >= xa && p < xe;
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const Real ym = r == 0 ? lo : C[r > 0 ? r - 1 : 0];
        const Real yp = r == R - 1 ? hi : C[r + 1 < R ? r + 1 : 0];
        const Real zm = dpp_shr1z(C[r]);
        const Real zp = dpp_shl1z(C[r]);
        // same operation order as kernels.hpp ftcs_update in both frames
        const Real nv = SW ? ftcs<Real>(C[r], ym, yp, M[r], P[r], zm, zp, Dx, Dy, Dz)
                           : ftcs<Real>(C[r], M[r], P[r], ym, yp, zm, zp, Dx, Dy, Dz);
        const Real d = resid_abs_r(nv, C[r]);
        bool upd = true, cnt = true, st = true;
        if constexpr (!FAST) {
          upd = xin && ((ybits >> r) & 1);
          cnt = xcnt && ((ybits >> (2 * R + s * R + r)) & 1);
          st = xst && ((ybits >> (R + r)) & 1);
        }
        if (s < K - 1) {
          Real(&N)[R] = f[s < K - 1 ? s : 0][fw];
          if constexpr (FAST) N[r] = nv;
          else N[r] = (upd && zin) ? nv : C[r];
        }
        if (!RL || s == K - 1) {
          if constexpr (FAST) {
            m[s] = fmax(m[s], d);
          } else {
            if (cnt) m[s] = fmax(m[s], d);
          }
        }
        if (s == K - 1 && st) {
          // T^{n+K} on the stored region (inside the box, hence the update range)
          nan_seen |= zst && (nv != nv);
          if (zst) buf_store<Real, ST>(nv, plane_rsrc(outw + (int64_t)p * sx), lane_b, r * sy_b);
        }
      }
      if constexpr (Q == 3) {
        if (s == 0) load_plane(x + 2, q[sM]);  // the slot stage 0 has just freed
      }
    }
  };

  // whole chunks of U steps (the unrolled body needs a constant trip count);
  // padded steps past xlast take the masked form and count / store nothing
  for (int xb = x0; xb <= xlast; xb += U) {
    static_for<0, U>([&](auto ph_tag) {
      constexpr int ph = decltype(ph_tag)::value;
      const int x = xb + ph;
      if (wfast && x >= xf_lo && x <= xf_hi) step(std::true_type{}, x, ph_tag);
      else step(std::false_type{}, x, ph_tag);
    });
  }

  // this piece's residuals (the lane masks depend on its tile)
  if (res) {
    double mm[K];
#pragma unroll
    for (int s = 0; s < K; ++s) {
      // stage s counts lanes inside its cone, the update range and the box
      // widened by K-1-s (deep-halo points still in flight stay excluded)
      const bool ok = zin && lane >= s + 1 && lane < 63 - s && col >= g.blo[2] - (K - 1 - s) &&
                      col < g.bhi[2] + (K - 1 - s);
      mm[s] = ok ? (double)m[s] : 0.0;
    }
    // the row exchange buffer is dead: reuse it for the per-wave maxima
    __syncthreads();
    residual_commit_block<WY, K>(res, mm, nan_seen,
                                 *reinterpret_cast<unsigned long long(*)[WY][K]>(&s_row[0][0][0][0][0]));
  }
  if (g.fst) fused_check_tail<K, RL>(g.fst, g.fslot, g.fblocks);
}

template <typename Real, int R, int WY, int K, int Q, int NTS = 0, bool SW = false>
void launch_tbl(const StencilParams& p, const KernelSpec& ks, hipStream_t s) {
  constexpr bool swap_xy = SW;
  const void* kfn = reinterpret_cast<const void*>(&stencil_tbl<Real, R, WY, K, Q, NTS, SW>);
  Box b = p.box;
  constexpr int TY = WY * R;
  // swap_xy: march along y with x as the tile rows (thin x slabs: a tile of
  // WY*R x-rows covers the slab and its K-deep halos, workgroups march the
  // long y extent).  The kernel is axis-agnostic through its strides and
  // ranges, so the swap is a relabelling of the arguments.
  const Layout& L = p.L;
  const int64_t Lsx = swap_xy ? L.sy : L.sx, Lsy = swap_xy ? L.sx : L.sy;
  const int64_t Ln0 = swap_xy ? L.n[1] : L.n[0], Ln1 = swap_xy ? L.n[0] : L.n[1];
  const int64_t Lg0 = swap_xy ? L.gy : L.gx, Lg1 = swap_xy ? L.gx : L.gy;
  const int64_t(&pux)[2] = swap_xy ? p.uy : p.ux;
  const int64_t(&puy)[2] = swap_xy ? p.ux : p.uy;
  if (swap_xy) {
    std::swap(b.lo[0], b.lo[1]);
    std::swap(b.hi[0], b.hi[1]);
  }
  HEAT3D_CHECK(Ln0 + 2 * Lg0 < (1LL << 30) && Ln1 + 2 * Lg1 < (1LL << 30) &&
                   Lsy * (int64_t)sizeof(Real) * (R + 2 * Lg1 + TY + 2 * K) < (1LL << 31),
               "tl: extents exceed 32-bit tile coordinates");
  TBLArgs g{};
  g.sx = Lsx;
  g.sy = Lsy;
  g.origin = L.origin;
  for (int a = 0; a < 3; ++a) {
    g.blo[a] = (int)b.lo[a];
    g.bhi[a] = (int)b.hi[a];
  }
  g.ulo = (int)(pux[1] >= pux[0] ? pux[0] : b.lo[0]);
  g.uhi = (int)(pux[1] >= pux[0] ? pux[1] : b.hi[0]);
  const bool wy = puy[1] >= puy[0], wz = p.uz[1] >= p.uz[0];
  g.uylo = (int)(wy ? puy[0] : b.lo[1]);
  g.uyhi = (int)(wy ? puy[1] : b.hi[1]);
  g.uzlo = (int)(wz ? p.uz[0] : b.lo[2]);
  g.uzhi = (int)(wz ? p.uz[1] : b.hi[2]);
  g.xlo_live = (int)-Lg0;
  g.xhi_live = (int)(Ln0 + Lg0 - 1);
  g.ylo_live = (int)-Lg1;
  g.yhi_live = (int)(Ln1 + Lg1 - 1);
  // every loaded column of every tile lies inside the row's allocation: the
  // row starts zoff >= 16 elements before k = 0 (tiles start K <= 6 columns
  // before the box) and the tail pad covers the last tile's overhang
  HEAT3D_CHECK(b.lo[2] - K >= -L.zoff, "tl: tile columns before the row start");
  HEAT3D_CHECK(g.uylo - 1 >= -Lg1 && g.uyhi <= Ln1 + Lg1 && g.uylo <= b.lo[1] && g.uyhi >= b.hi[1] &&
                   g.uzlo - 1 >= -L.gz && g.uzhi <= L.n[2] + L.gz && g.uzlo <= b.lo[2] && g.uzhi >= b.hi[2],
               "tl: y/z update range outside the ghosted layout");
  HEAT3D_CHECK(g.ulo - 1 >= g.xlo_live && g.uhi <= g.xhi_live + 1 && g.ulo <= b.lo[0] && g.uhi >= b.hi[0],
               "tl: u range [" << g.ulo << "," << g.uhi << ") outside the ghosted layout");
  constexpr int YS = TY - 2 * K;
  static const int slots = device_slots(kfn, 64 * WY);  // magic static: thread-safe under --gpus N
  constexpr int U = Q == 4 ? 12 : 6;  // the kernel's unroll (lcm(Q, 3, 2))
  const int ZS = ks.ZS > 0 ? ks.ZS
                           : lean_z_stride(b.extent(0), b.extent(1), b.extent(2), K, (int)sizeof(Real), TY, slots, U, ks.L);
  HEAT3D_CHECK(ZS >= 1 && ZS <= 64 - 2 * K, "tl: z stride " << ZS << " outside [1, " << 64 - 2 * K << "]");
  g.c00 = (int)(b.lo[2] - K);
  g.r00 = (int)(b.lo[1] - K);
  g.nyb = (int)std::max<int64_t>(1, (b.extent(1) + YS - 1) / YS);
  auto set_zs = [&](TBLArgs& ga, int zs) {
    ga.zs = zs;
    ga.nzb = (int)std::max<int64_t>(1, (b.extent(2) + zs - 1) / zs);
    return (int64_t)ga.nzb * ga.nyb;
  };
  (void)set_zs(g, ZS);
  const int64_t nxb = b.extent(0);
  HEAT3D_CHECK(ks.L != -2, "tl: the persistent walk (L = -2) was retired in round 5 (18-22% slower than the x plan)");
  HEAT3D_CHECK(!p.state || p.slot + K <= kResidualSlots, "tl: residual slots " << p.slot << "+" << K);
  auto scratch = [](const void* f) {
    hipFuncAttributes a{};
    return hipFuncGetAttributes(&a, f) == hipSuccess ? (int)a.localSizeBytes : 0;
  };
  static const int spill = scratch(kfn);
  // a spilling variant is refused (one was miscompiled on ROCm 7.2)
  HEAT3D_CHECK(spill == 0, "tl variant " << ks.str() << " spills " << spill << " B of registers per lane");
  unsigned long long* r = p.state && p.residual ? &p.state->residual[p.slot] : nullptr;
  const int* done = p.state ? &p.state->done : nullptr;
  // spec field L: > 0 fixed segments, -1 equal segments, -3 the x plan;
  // 0: the schedule timed for this box (tune_schedule: z stride and x
  // schedule), else the x plan
  auto fire = [&](int zs, int Lx) {
    TBLArgs ga = g;
    const int64_t tiles = set_zs(ga, zs);
    const XPlan xp = Lx > 0 ? fixed_xplan(nxb, tiles, Lx) : plan_x(nxb, tiles, slots, 2 * (K - 1), U, Lx == -1);
    HEAT3D_CHECK(xp.seg < (1 << 15) && xp.split < (1 << 15) && xp.r < (1 << 30), "tl: x plan out of range");
    ga.segsplit = xp.seg | (xp.split << 16);
    ga.n1 = xp.n1;
    ga.rb = xp.r | (xp.nb2 > 0 ? (1 << 30) : 0);
    const int64_t nblocks = (int64_t)xp.n1 + xp.r + xp.nb2;
    HEAT3D_CHECK(nblocks < (1LL << 31) && nblocks >= 1, "tl: bad block count " << nblocks);
    ga.fst = p.fuse_check && r ? p.state : nullptr;
    ga.fslot = p.slot;
    ga.fblocks = (int)nblocks;
    if (trace_enabled())
      std::fprintf(stderr, "[heat3d trace] tl K=%d box x %lld: zs=%d L=%d seg=%d tiles=%dx%d blocks=%lld (model %.1f)\n",
                   K, (long long)nxb, zs, Lx, xp.seg, ga.nzb, ga.nyb, (long long)nblocks,
                   xplan_makespan(xp, nxb, tiles, slots, 2 * (K - 1), U));
    hipLaunchKernelGGL((stencil_tbl<Real, R, WY, K, Q, NTS, SW>), dim3((unsigned)nblocks), dim3(64 * WY), 0,
                       s, static_cast<const Real*>(p.in), static_cast<Real*>(p.out), ga, (Real)p.D[0], (Real)p.D[1],
                       (Real)p.D[2], r, done);
    HIPK_CHECK(hipGetLastError());
  };
  if (ks.L == 0 && ks.ZS == 0 && !SW) {
    const int64_t box[3] = {b.extent(0), b.extent(1), b.extent(2)};
    if (p.tune) {
      // z strides: the model's, and the other of 64 - 2K / its 64-byte-aligned form
      std::vector<int> zs_opts{ZS};
      const int wide = 64 - 2 * K, aligned = sizeof(Real) == 8 ? wide & ~7 : wide;
      for (int z : {wide, aligned})
        if (std::find(zs_opts.begin(), zs_opts.end(), z) == zs_opts.end()) zs_opts.push_back(z);
      tune_schedule(sizeof(Real) == 8 ? "tl-fp64" : "tl-fp32", kfn, box, slots, p.cu_reserved, U, zs_opts, s, fire,
                    g.nyb, 2 * (K - 1));
      return;  // every candidate computed this sweep
    }
    SchedChoice c;
    if (tuned_lookup(kfn, box, slots, p.cu_reserved, &c)) {
      fire(c.zs, c.L);
      return;
    }
    fire(ZS, 0);
    return;
  }
  fire(ZS, ks.L);
}

}  // namespace hip
}  // namespace heat3d
