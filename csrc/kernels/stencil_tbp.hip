// heat3d-mi355x — K-step temporally blocked FTCS kernel with two z columns
// per lane ("tlK:2:…"): fp32 in packed math, fp64 in 16-byte pairs.
//
// Same contract and structure as the lean kernel (stencil_tbl.hip: T^n ring,
// K stages one plane apart, edge rows through LDS once per step, mask-free
// interior steps, residual masks applied once at the end), but every lane
// holds a pair of consecutive z columns and every arithmetic step is one
// v_pk_fma_f32 / v_pk_add_f32 on the pair.  Counted on MI355X, the fp32 lean
// kernel issues ~22 VALU instructions per point update and keeps the VALU
// ~65-70% busy (profiles/hbm_probes_r02.md, pmc): it is instruction-bound,
// and the pair form halves the update's instructions.  z neighbours of a pair
// (a, b) at lane l: zm = (b of lane l-1, a), zp = (b, a of lane l+1) — one
// wave-shift DPP move per direction per pair.
//
// A wave covers 128 columns, so a tile is 128 x (WY R) points, 8-byte lane
// accesses (the fp64 kernel's access shape).  Tiles start on an even column
// (8-byte aligned pairs): the first tile loads from floor_even(lo - K), its
// stored columns start hl = lo - c00 (K or K + 1) columns in, and tiles
// advance by ZS = 128 - 2K - 2 columns, so every stored column lies in
// [K, 128 - K) of its tile, inside the last stage's cone.
//
// Fields, residuals and iteration counts are bitwise identical to the
// single-step kernels: each element goes through kernels.hpp ftcs_update's
// operation sequence (packed FMA is two correctly rounded fp32 FMAs), and the
// residual is |T^{n+1} - T^n| in the field's precision (resid_abs_r).
//
// fp64 pairs (round 5, opt-in: --kernel2 tl3:2).  The one-value-per-lane
// fp64 tile (64 x 48 points, 16 waves of 3 rows, 112 of 128 VGPRs) loads 64
// columns to store 58 — 5 of the 128-byte L2 lines per 58 columns — and its
// sweep reads 1.36x the field from HBM (profiles/l2_reuse_r04.md).  A pair
// lane doubles the tile's width to 128 columns (122 stored, 9 lines) with
// 16-byte loads and stores and one wave shift per direction per pair.  A
// pair of doubles is 4 VGPRs and K = 3 keeps 9 plane rows per tile row, so
// only 4 rows per wave fit 8 waves x 256 VGPRs (227; 5 and 6 rows spill):
// 128 x 32 tiles.  Measured (profiles/fp64_pairs_r05.md): bitwise equal to
// the lean kernel; half its VMEM, LDS and SALU instructions and 0.95x its
// VALU per point, but the same HBM reads (1.38x against 1.36x: the shorter
// tiles lose in y what the wider ones gain in z) and 825 against 838 GLUPS
// on 1022^3; faster alone on the 8-GPU slab share's 122-plane interior (744
// against 711: 360 tiles are 1.45 rounds of 248 CUs, 450 are 1.81) but not
// inside the overlapped schedule, so the lean kernel stays the default.
#include <hip/hip_runtime.h>

#include <array>
#include <map>
#include <mutex>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "hip_helpers.hpp"

namespace heat3d {
namespace hip {

struct TBPArgs {
  int64_t sx, sy, origin;      // plane / row strides, element index of owned (0,0,0)
  int blo[3], bhi[3];          // store box
  int ulo, uhi, uylo, uyhi;    // update ranges (x, y)
  int uzlo, uzhi;              // update range (z)
  int xlo_live, xhi_live;      // x planes present in memory
  int ylo_live, yhi_live;      // y rows present in memory
  int c00, r00;                // first loaded column (even) / row of tile (0, 0)
  int nzb, nyb;
  int segsplit, n1, rb;        // x plan (TBRArgs encoding)
  int hl;                      // first stored column of a tile, from its first loaded one
  int zs;                      // tile stride along z = stored columns per tile (even, <= 128 - 2K - 2)
  DeviceState* fst;            // fused convergence check (fused_check_tail): state, nullptr = off
  int fslot, fblocks;          // its first residual slot and the grid's workgroup count
};

namespace {

template <typename T>
using vec2 = T __attribute__((ext_vector_type(2)));

constexpr int gcd_p(int a, int b) { return b == 0 ? a : gcd_p(b, a % b); }
constexpr int lcm_p(int a, int b) { return a / gcd_p(a, b) * b; }

__device__ __forceinline__ int sgpr(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t prs(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)0xffffffff, 0x00020000);
}
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// a pair load: 8 bytes (fp32) or 16 bytes (fp64) per lane
template <typename T>
__device__ __forceinline__ vec2<T> ld2(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  if constexpr (sizeof(T) == 8)
    return __builtin_bit_cast(vec2<T>, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
  else
    return __builtin_bit_cast(vec2<T>, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
// AUX = cache-policy bits of the output stores (0 = default, 2 = nt)
template <int AUX, typename T>
__device__ __forceinline__ void st2(vec2<T> v, __amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  if constexpr (sizeof(T) == 8)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, voff, soff, AUX);
  else
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, voff, soff, AUX);
}
template <int AUX, typename T>
__device__ __forceinline__ void st1(T v, __amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  if constexpr (sizeof(T) == 8)
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, voff, soff, AUX);
  else
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, voff, soff, AUX);
}
template <typename T>
__device__ __forceinline__ vec2<T> fma2(vec2<T> a, vec2<T> b, vec2<T> c) {
  return __builtin_elementwise_fma(a, b, c);
}

// kernels.hpp ftcs_update on a pair, same operation order per element
template <typename T>
__device__ __forceinline__ vec2<T> ftcs2(vec2<T> c, vec2<T> xm, vec2<T> xp, vec2<T> ym, vec2<T> yp, vec2<T> zm,
                                         vec2<T> zp, vec2<T> Dx, vec2<T> Dy, vec2<T> Dz) {
  typedef vec2<T> f2;
  const f2 m2 = {T(-2), T(-2)};
  const f2 ax = fma2(m2, c, xp) + xm;
  const f2 ay = fma2(m2, c, yp) + ym;
  const f2 az = fma2(m2, c, zp) + zm;
  return fma2(Dz, az, fma2(Dy, ay, fma2(Dx, ax, c)));
}

template <int B, int E, typename Fn>
__device__ __forceinline__ void static_for_p(Fn&& fn) {
  if constexpr (B < E) {
    fn(std::integral_constant<int, B>{});
    static_for_p<B + 1, E>(fn);
  }
}

}  // namespace

template <typename T, int R, int WY, int K, int Q, int AUX = 0>
__global__ __launch_bounds__(64 * WY) void stencil_tbp(const T* __restrict__ in, T* __restrict__ out,
                                                       TBPArgs g, T Dxs, T Dys, T Dzs,
                                                       unsigned long long* res, const int* done) {
  typedef vec2<T> f2;
  static_assert(K >= 2 && K <= 6, "temporal depth");
  static_assert(Q == 3 || Q == 4, "T^n ring size");
  constexpr int TY = WY * R;
  constexpr int YS = TY - 2 * K;       // tile stride along y (stored rows)
  constexpr int U = lcm_p(lcm_p(Q, 3), 2);
  static_assert(YS > 0 && R <= 16, "tile too small for depth K");
  // AUX bit kResidualLastOnly: only the last step's residual (monotone check)
  constexpr bool RL = (AUX & kResidualLastOnly) != 0;
  constexpr int ST = AUX & ~kResidualLastOnly;  // the stores' cache-policy bits
  __shared__ __attribute__((aligned(16))) f2 s_row[2][K][WY][2][64];
  static_assert(sizeof(s_row) >= WY * K * sizeof(unsigned long long), "residual scratch");
  if (flag_set(done)) {
    if (g.fst) fused_check_tail<K, RL>(g.fst, g.fslot, g.fblocks);
    return;
  }

  auto remap = [](int i, int n) {
    const int c = i & 7;
    return c * (n >> 3) + min(c, n & 7) + (i >> 3);
  };
  const int blk = blockIdx.x;
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
  const int zb = pc % g.nzb;
  const int tq = pc / g.nzb;
  const int ybk = tq % g.nyb;
  const int xs = tq / g.nyb;
  const int nxb = g.bhi[0] - g.blo[0];
  const int seg = g.segsplit & 0xffff, split = g.segsplit >> 16;
  int xlo_p = xs * seg, xhi_p = min(xlo_p + seg, nxb);
  if (part == 1 && (g.rb >> 30)) xhi_p = min(xhi_p, xlo_p + split);
  if (part == 2) xlo_p = min(xlo_p + split, xhi_p);

  const int wave = sgpr(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int c0 = g.c00 + zb * g.zs;  // tile's first loaded column (even)
  const int r0 = g.r00 + ybk * YS;
  const int yb = r0 + wave * R;
  const int j0 = 2 * lane, j1 = j0 + 1;  // the pair's columns within the tile
  const int col0 = c0 + j0, col1 = col0 + 1;
  const int xa = g.blo[0] + xlo_p, xe = g.blo[0] + xhi_p;
  const int x0 = xa - (K - 1), xlast = xe + K - 2;
  const int64_t sx = g.sx;

  const bool zfast = c0 >= g.uzlo && c0 + 128 <= g.uzhi;
  const bool wrows = wave * R >= K && wave * R + R <= TY - K && yb >= g.uylo && yb + R <= g.uyhi &&
                     yb >= g.blo[1] && yb + R <= g.bhi[1];
  const bool wfast = zfast && wrows;
  const int xf_lo = max(max(x0 + 2 * (K - 1), g.ulo + K - 1), g.blo[0] + K - 1);
  const int xf_hi = min(min(xlast, g.uhi - 1), g.bhi[0] + K - 2);

  // row masks (uniform): bit r = row in the update range, R + r = stored
  // row, 2R + sR + r = row counted at stage s (64-bit for tall 8-wave tiles)
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

  const bool zin0 = col0 >= g.uzlo && col0 < g.uzhi, zin1 = col1 >= g.uzlo && col1 < g.uzhi;
  const bool zst0 = j0 >= g.hl && j0 < g.hl + g.zs && col0 >= g.blo[2] && col0 < g.bhi[2];
  const bool zst1 = j1 >= g.hl && j1 < g.hl + g.zs && col1 >= g.blo[2] && col1 < g.bhi[2];
  const bool zst2 = zst0 && zst1;

  auto yclamp = [&](int row) { return min(max(row, g.ylo_live), g.yhi_live); };
  const int ybc = yclamp(yb);
  const T* __restrict__ inw = in + (g.origin + (int64_t)ybc * g.sy + c0);
  T* __restrict__ outw = out + (g.origin + (int64_t)yb * g.sy + c0);
  int roff[R];
#pragma unroll
  for (int r = 0; r < R; ++r) roff[r] = sgpr((yclamp(yb + r) - ybc) * (int)g.sy * (int)sizeof(T));
  const int sy_b = (int)g.sy * (int)sizeof(T);
  const unsigned lane_b = (unsigned)lane * (unsigned)sizeof(f2);
  const f2 Dx = {Dxs, Dxs}, Dy = {Dys, Dys}, Dz = {Dzs, Dzs};

  f2 q[Q][R];         // T^n ring: plane p in slot (p - x0 + 1) mod Q
  f2 f[K - 1][3][R];  // F_{s+1}(p) in f[s][(p + s) mod 3]
  f2 m[K];            // per-element residual maxima (field precision, widened at the end)
  bool nan_seen = false;
#pragma unroll
  for (int s = 0; s < K; ++s) m[s] = f2{T(0), T(0)};
#pragma unroll
  for (int s = 0; s < K - 1; ++s)
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int r = 0; r < R; ++r) f[s][i][r] = f2{T(0), T(0)};

  auto load_plane = [&](int x, f2 (&d)[R]) {
    const int xc = min(max(x, g.xlo_live), g.xhi_live);
    const __amdgpu_buffer_rsrc_t rs = prs(inw + (int64_t)xc * sx);
#pragma unroll
    for (int r = 0; r < R; ++r) d[r] = ld2<T>(rs, lane_b, roff[r]);
  };
  constexpr int NPRE = Q == 3 ? 3 : Q - 1;
#pragma unroll
  for (int i = 0; i < NPRE; ++i) load_plane(x0 - 1 + i, q[i]);

  auto step = [&](auto fast_tag, const int x, auto ph_tag) {
    constexpr bool FAST = decltype(fast_tag)::value;
    constexpr int ph = decltype(ph_tag)::value;
    constexpr int sM = ph % Q, sC = (ph + 1) % Q, sP = (ph + 2) % Q;
    constexpr int fw = ph % 3, fc = (ph + 2) % 3, fm = (ph + 1) % 3;
    constexpr int par = ph & 1;
    if constexpr (Q >= 4) load_plane(x + Q - 2, q[(ph + Q - 1) % Q]);
#pragma unroll
    for (int s = 0; s < K; ++s) {
      const f2(&C)[R] = s == 0 ? q[sC] : f[s > 0 ? s - 1 : 0][fc];
      s_row[par][s][wave][0][lane] = C[0];
      s_row[par][s][wave][1][lane] = C[R - 1];
    }
    __syncthreads();
    const int wl = max(wave - 1, 0), wh = min(wave + 1, WY - 1);
#pragma unroll
    for (int s = 0; s < K; ++s) {
      f2(&M)[R] = s == 0 ? q[sM] : f[s > 0 ? s - 1 : 0][fm];
      f2(&C)[R] = s == 0 ? q[sC] : f[s > 0 ? s - 1 : 0][fc];
      f2(&P)[R] = s == 0 ? q[sP] : f[s > 0 ? s - 1 : 0][fw];
      const f2 lo = s_row[par][s][wl][1][lane];
      const f2 hi = s_row[par][s][wh][0][lane];
      const int p = x - s;
      bool xin = true, xcnt = true, xst = true;
      if constexpr (!FAST) {
        xin = p >= g.ulo && p < g.uhi;
        xcnt = xin && x >= x0 + 2 * s && x <= xlast && p >= g.blo[0] - (K - 1 - s) && p < g.bhi[0] + (K - 1 - s);
        xst = p >= xa && p < xe;
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const f2 c = C[r];
        const f2 ym = r == 0 ? lo : C[r > 0 ? r - 1 : 0];
        const f2 yp = r == R - 1 ? hi : C[r + 1 < R ? r + 1 : 0];
        const f2 zm = {dpp_shr1z(c.y), c.x};
        const f2 zp = {c.y, dpp_shl1z(c.x)};
        const f2 nv = ftcs2<T>(c, M[r], P[r], ym, yp, zm, zp, Dx, Dy, Dz);
        const f2 d = __builtin_elementwise_abs(nv - c);  // resid_abs_r per element
        bool upd = true, cnt = true, st = true;
        if constexpr (!FAST) {
          upd = xin && ((ybits >> r) & 1);
          cnt = xcnt && ((ybits >> (2 * R + s * R + r)) & 1);
          st = xst && ((ybits >> (R + r)) & 1);
        }
        if (s < K - 1) {
          f2(&N)[R] = f[s < K - 1 ? s : 0][fw];
          if constexpr (FAST) N[r] = nv;
          else N[r] = f2{(upd && zin0) ? nv.x : c.x, (upd && zin1) ? nv.y : c.y};
        }
        if (!RL || s == K - 1) {
          if constexpr (FAST) {
            m[s] = __builtin_elementwise_max(m[s], d);
          } else {
            if (cnt) m[s] = __builtin_elementwise_max(m[s], d);
          }
        }
        if (s == K - 1 && st) {
          nan_seen |= (zst0 && nv.x != nv.x) || (zst1 && nv.y != nv.y);
          const __amdgpu_buffer_rsrc_t ro = prs(outw + (int64_t)p * sx);
          if (zst2) {
            st2<ST, T>(nv, ro, lane_b, r * sy_b);
          } else {
            if (zst0) st1<ST, T>(nv.x, ro, lane_b, r * sy_b);
            if (zst1) st1<ST, T>(nv.y, ro, lane_b + (unsigned)sizeof(T), r * sy_b);
          }
        }
      }
      if constexpr (Q == 3) {
        if (s == 0) load_plane(x + 2, q[sM]);
      }
    }
  };

  for (int xb = x0; xb <= xlast; xb += U) {
    static_for_p<0, U>([&](auto ph_tag) {
      constexpr int ph = decltype(ph_tag)::value;
      const int x = xb + ph;
      if (wfast && x >= xf_lo && x <= xf_hi) step(std::true_type{}, x, ph_tag);
      else step(std::false_type{}, x, ph_tag);
    });
  }

  if (res) {
    double mm[K];
#pragma unroll
    for (int s = 0; s < K; ++s) {
      const bool ok0 = zin0 && j0 >= s + 1 && j0 < 127 - s && col0 >= g.blo[2] - (K - 1 - s) &&
                       col0 < g.bhi[2] + (K - 1 - s);
      const bool ok1 = zin1 && j1 >= s + 1 && j1 < 127 - s && col1 >= g.blo[2] - (K - 1 - s) &&
                       col1 < g.bhi[2] + (K - 1 - s);
      const double a = ok0 ? (double)m[s].x : 0.0, b = ok1 ? (double)m[s].y : 0.0;
      mm[s] = a > b ? a : b;
    }
    __syncthreads();
    residual_commit_block<WY, K>(res, mm, nan_seen,
                                 *reinterpret_cast<unsigned long long(*)[WY][K]>(&s_row[0][0][0][0][0]));
  }
  if (g.fst) fused_check_tail<K, RL>(g.fst, g.fslot, g.fblocks);
}

// Tile stride along z: 128 - 2K - 2 stored columns (tiles start on even
// columns), or the largest multiple of a 64-byte line (16 fp32, 8 fp64)
// below it, which starts every tile's stored strip on a 64-byte boundary
// (whole 64-B write segments at both seams; 2049^3 fp32 1456 -> 1531 GLUPS
// with 112 instead of 120, round 3).
// The narrower stride can add a tile column, so — as lean_z_stride does for
// fp64 — it is taken only where the tiling cost (tiling_cost), with that
// gain, predicts a shorter sweep, and only for boxes of >= 500 x planes
// (1022^3: 120 keeps 9 tile columns, 112 would add a 14-wide 10th: 1397 vs
// 1294 GLUPS).
static int pair_z_stride_plan(int64_t nx, int64_t ny, int64_t nz, int K, int TY, int slots, int U, int L, int esize);
static int pair_aligned_stride(int wide, int esize) { return wide & ~(64 / esize - 1); }
int pair_z_stride(int64_t nx, int64_t ny, int64_t nz, int K, int TY, int slots, int U, int L, int esize) {
  // memoised: every eager launch asks
  static std::mutex mu;
  static std::map<std::array<int64_t, 9>, int> memo;
  const std::array<int64_t, 9> key{nx, ny, nz, K, TY, slots, U, L, esize};
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = memo.find(key);
    if (it != memo.end()) return it->second;
  }
  const int zs = pair_z_stride_plan(nx, ny, nz, K, TY, slots, U, L, esize);
  std::lock_guard<std::mutex> lk(mu);
  memo[key] = zs;
  return zs;
}

static int pair_z_stride_plan(int64_t nx, int64_t ny, int64_t nz, int K, int TY, int slots, int U, int L, int esize) {
  const int wide = 128 - 2 * K - 2;
  const int aligned = pair_aligned_stride(wide, esize);
  if (aligned == wide || aligned <= 0 || nx < 500) return wide;
  const int64_t nyb = std::max<int64_t>(1, (ny + TY - 2 * K - 1) / (TY - 2 * K));
  auto cost = [&](int zs) {
    const int64_t tiles = std::max<int64_t>(1, (nz + zs - 1) / zs) * nyb;
    const XPlan p = L > 0 ? fixed_xplan(nx, tiles, L) : plan_x(nx, tiles, slots, 2 * (K - 1), U, L < 0);
    return tiling_cost(p, nx, tiles, slots, 2 * (K - 1), U);
  };
  constexpr double kAlignedGain = 0.92;
  return cost(aligned) * kAlignedGain < cost(wide) ? aligned : wide;
}

template <typename T, int R, int WY, int K, int Q, int AUX = 0>
static void launch_tbp(const StencilParams& p, const KernelSpec& ks, hipStream_t s) {
  const Box& b = p.box;
  constexpr int TY = WY * R;
  const Layout& L = p.L;
  HEAT3D_CHECK(L.esize == (int64_t)sizeof(T), "tl pair kernel: field element size " << L.esize);
  HEAT3D_CHECK(L.n[0] + 2 * L.gx < (1LL << 30) && L.n[1] + 2 * L.gy < (1LL << 30) &&
                   L.sy * (int64_t)sizeof(T) * (R + 2 * L.gy + TY + 2 * K) < (1LL << 31),
               "tl pair: extents exceed 32-bit tile coordinates");
  TBPArgs g{};
  g.sx = L.sx;
  g.sy = L.sy;
  g.origin = L.origin;
  for (int a = 0; a < 3; ++a) {
    g.blo[a] = (int)b.lo[a];
    g.bhi[a] = (int)b.hi[a];
  }
  g.ulo = (int)(p.ux[1] >= p.ux[0] ? p.ux[0] : b.lo[0]);
  g.uhi = (int)(p.ux[1] >= p.ux[0] ? p.ux[1] : b.hi[0]);
  const bool wy = p.uy[1] >= p.uy[0], wz = p.uz[1] >= p.uz[0];
  g.uylo = (int)(wy ? p.uy[0] : b.lo[1]);
  g.uyhi = (int)(wy ? p.uy[1] : b.hi[1]);
  g.uzlo = (int)(wz ? p.uz[0] : b.lo[2]);
  g.uzhi = (int)(wz ? p.uz[1] : b.hi[2]);
  g.xlo_live = (int)-L.gx;
  g.xhi_live = (int)(L.n[0] + L.gx - 1);
  g.ylo_live = (int)-L.gy;
  g.yhi_live = (int)(L.n[1] + L.gy - 1);
  // first loaded column: lo - K rounded down to even (aligned pairs; rows are
  // 128-B aligned), so a tile's stored columns start K or K + 1 in
  const int c = (int)b.lo[2] - K;
  g.c00 = c - (c & 1);
  g.hl = (int)b.lo[2] - g.c00;
  // the tail pad (layout.hpp: two rows + 1024 elements) covers the last
  // tile's overhang of at most 127 columns; the row starts zoff >= 32 before k = 0
  HEAT3D_CHECK(g.c00 >= -L.zoff, "tl pair: tile columns before the row start");
  HEAT3D_CHECK(L.zoff % 2 == 0 && L.sy % 2 == 0 && L.origin % 2 == 0, "tl pair: rows not pair-aligned");
  HEAT3D_CHECK(g.uylo - 1 >= -L.gy && g.uyhi <= L.n[1] + L.gy && g.uylo <= b.lo[1] && g.uyhi >= b.hi[1] &&
                   g.uzlo - 1 >= -L.gz && g.uzhi <= L.n[2] + L.gz && g.uzlo <= b.lo[2] && g.uzhi >= b.hi[2],
               "tl pair: y/z update range outside the ghosted layout");
  HEAT3D_CHECK(g.ulo - 1 >= g.xlo_live && g.uhi <= g.xhi_live + 1 && g.ulo <= b.lo[0] && g.uhi >= b.hi[0],
               "tl pair: u range [" << g.ulo << "," << g.uhi << ") outside the ghosted layout");
  static const int slots =  // magic static: thread-safe under --gpus N
      device_slots(reinterpret_cast<const void*>(&stencil_tbp<T, R, WY, K, Q, AUX>), 64 * WY);
  constexpr int U = Q == 4 ? 12 : 6;
  const int ZS =
      ks.ZS > 0 ? ks.ZS : pair_z_stride(b.extent(0), b.extent(1), b.extent(2), K, TY, slots, U, ks.L, (int)sizeof(T));
  HEAT3D_CHECK(ZS >= 2 && ZS % 2 == 0 && ZS <= 128 - 2 * K - 2,
               "tl pair: z stride " << ZS << " must be even and in [2, " << 128 - 2 * K - 2 << "]");
  constexpr int YS = TY - 2 * K;
  g.r00 = (int)(b.lo[1] - K);
  g.nyb = (int)std::max<int64_t>(1, (b.extent(1) + YS - 1) / YS);
  auto set_zs = [&](TBPArgs& ga, int zs) {
    ga.zs = zs;
    ga.nzb = (int)std::max<int64_t>(1, (b.extent(2) + zs - 1) / zs);
    return (int64_t)ga.nzb * ga.nyb;
  };
  set_zs(g, ZS);
  const int64_t nxb = b.extent(0);
  HEAT3D_CHECK(!p.state || p.slot + K <= kResidualSlots, "tl pair: residual slots " << p.slot << "+" << K);
  static const int spill = [] {
    hipFuncAttributes a{};
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&stencil_tbp<T, R, WY, K, Q, AUX>)) == hipSuccess
               ? (int)a.localSizeBytes
               : 0;
  }();
  HEAT3D_CHECK(spill == 0, "tl pair variant " << ks.str() << " spills " << spill << " B of registers per lane");
  unsigned long long* r = p.state && p.residual ? &p.state->residual[p.slot] : nullptr;
  const int* done = p.state ? &p.state->done : nullptr;
  // spec fields L and ZS as in launch_tbl (L = 0, ZS = 0: the timed schedule of this box)
  auto fire = [&](int zs, int Lx) {
    TBPArgs ga = g;
    const int64_t tiles = set_zs(ga, zs);
    const XPlan xp = Lx > 0 ? fixed_xplan(nxb, tiles, Lx) : plan_x(nxb, tiles, slots, 2 * (K - 1), U, Lx == -1);
    HEAT3D_CHECK(xp.seg < (1 << 15) && xp.split < (1 << 15) && xp.r < (1 << 30), "tl pair: x plan out of range");
    ga.segsplit = xp.seg | (xp.split << 16);
    ga.n1 = xp.n1;
    ga.rb = xp.r | (xp.nb2 > 0 ? (1 << 30) : 0);
    const int64_t nblocks = (int64_t)xp.n1 + xp.r + xp.nb2;
    HEAT3D_CHECK(nblocks < (1LL << 31) && nblocks >= 1, "tl pair: bad block count " << nblocks);
    ga.fst = p.fuse_check && r ? p.state : nullptr;
    ga.fslot = p.slot;
    ga.fblocks = (int)nblocks;
    if (trace_enabled())
      std::fprintf(stderr,
                   "[heat3d trace] tl pair K=%d box x %lld: zs=%d L=%d seg=%d tiles=%dx%d blocks=%lld slots=%d "
                   "(model %.1f)\n",
                   K, (long long)nxb, zs, Lx, xp.seg, ga.nzb, ga.nyb, (long long)nblocks, slots,
                   xplan_makespan(xp, nxb, tiles, slots, 2 * (K - 1), U));
    hipLaunchKernelGGL((stencil_tbp<T, R, WY, K, Q, AUX>), dim3((unsigned)nblocks), dim3(64 * WY), 0, s,
                       static_cast<const T*>(p.in), static_cast<T*>(p.out), ga, (T)p.D[0], (T)p.D[1], (T)p.D[2], r,
                       done);
    HIPK_CHECK(hipGetLastError());
  };
  const void* kfn = reinterpret_cast<const void*>(&stencil_tbp<T, R, WY, K, Q, AUX>);
  if (ks.L == 0 && ks.ZS == 0) {
    const int64_t box[3] = {b.extent(0), b.extent(1), b.extent(2)};
    if (p.tune) {
      std::vector<int> zs_opts{ZS};
      const int wide = 128 - 2 * K - 2, aligned = pair_aligned_stride(wide, (int)sizeof(T));
      for (int z : {wide, aligned})
        if (z > 0 && std::find(zs_opts.begin(), zs_opts.end(), z) == zs_opts.end()) zs_opts.push_back(z);
      tune_schedule(sizeof(T) == 8 ? "tl-fp64-pair" : "tl-fp32-pair", kfn, box, slots, p.cu_reserved, U, zs_opts, s,
                    fire, g.nyb, 2 * (K - 1));
      return;
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

// p == nullptr: only report whether the variant k resolves to exists
template <typename T>
static bool run_tbp(const StencilParams* p, const KernelSpec& k, hipStream_t s) {
  const KernelSpec r = k.resolved(sizeof(T) == 8 ? DType::F64 : DType::F32);
  const int K = k.K, R = r.R, WY = r.WY, Q = r.NT;
  if (r.V != 2 || r.WZ != 1) return false;
  // AA: the output stores' cache-policy bits (spec field 7; 0 = default,
  // which a spec without the field, O <= 0, selects)
#define H3D_TBP(RR, YY, KK, QQ, AA)                                                             \
  if (R == RR && WY == YY && K == KK && Q == QQ && (r.O == (AA) || ((AA) == 0 && r.O <= 0))) {  \
    if (p) launch_tbp<T, RR, YY, KK, QQ, (AA)>(*p, k, s);                                       \
    return true;                                                                                \
  }
  if constexpr (sizeof(T) == 4) {
    // output-store cache policy (spec field 7), default shape only
    H3D_TBP(3, 16, 3, 3, 2) H3D_TBP(3, 16, 3, 3, 3) H3D_TBP(3, 16, 3, 3, 17) H3D_TBP(3, 16, 3, 3, 19)
    H3D_TBP(3, 16, 3, 3, 2 | kResidualLastOnly)
    // the long (K = 4) and partial (K = 2) sweeps' default shapes, last residual only
    H3D_TBP(2, 16, 4, 3, kResidualLastOnly) H3D_TBP(2, 16, 2, 3, kResidualLastOnly)
    H3D_TBP(3, 16, 3, 3, 0) H3D_TBP(3, 16, 3, 4, 0) H3D_TBP(2, 16, 3, 3, 0) H3D_TBP(2, 16, 4, 3, 0)
    H3D_TBP(2, 16, 4, 4, 0) H3D_TBP(3, 16, 4, 3, 0) H3D_TBP(2, 16, 2, 3, 0) H3D_TBP(3, 16, 2, 3, 0)
  } else {
    // fp64 pairs: 8 waves (<= 256 VGPRs, 2 waves per SIMD) of 4 rows at
    // K = 3 (5 and 6 rows spill: a pair is 4 VGPRs and K = 3 holds 9 plane
    // rows per tile row; 16 waves of 2 rows take 145 VGPRs and 192 KiB of
    // LDS), K = 2 in 6 rows and K = 4 in 3 rows of 8 waves; nt stores (2) or
    // default (0)
    H3D_TBP(4, 8, 3, 3, 2) H3D_TBP(4, 8, 3, 3, 0) H3D_TBP(6, 8, 2, 3, 2)
    H3D_TBP(4, 8, 3, 3, 2 | kResidualLastOnly) H3D_TBP(6, 8, 2, 3, 2 | kResidualLastOnly)
    H3D_TBP(3, 8, 4, 3, 2 | kResidualLastOnly)
    H3D_TBP(3, 8, 4, 3, 2)
  }
#undef H3D_TBP
  return false;
}

bool lean_pair_supported(DType t, const KernelSpec& k) {
  return t == DType::F64 ? run_tbp<double>(nullptr, k, nullptr) : run_tbp<float>(nullptr, k, nullptr);
}

void stencil_lean_pair(DType t, const StencilParams& p, const KernelSpec& k, void* stream) {
  if (p.box.empty()) return;
  const bool ok = t == DType::F64 ? run_tbp<double>(&p, k, S(stream)) : run_tbp<float>(&p, k, S(stream));
  if (!ok) {
    const KernelSpec r = k.resolved(t);
    HEAT3D_THROW("unsupported tl pair variant V=" << r.V << " R=" << r.R << " WY=" << r.WY << " K=" << k.K
                                                  << " Q=" << r.NT << " O=" << r.O);
  }
}

}  // namespace hip
}  // namespace heat3d
