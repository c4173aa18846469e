// heat3d-mi355x — K-step temporally blocked FTCS sweeps, lean form ("tl"):
// variant dispatch, z-stride planner and the public entry points.  The kernel
// and its launcher live in stencil_tbl_impl.hpp; the variants (listed in
// stencil_tbl_variants.inc) are instantiated by the stencil_tbl_part*.hip
// units so that they compile in parallel.
#include "stencil_tbl_impl.hpp"

#include <array>
#include <map>
#include <mutex>

namespace heat3d {
namespace hip {

// every variant dispatch_tbl can launch, instantiated elsewhere
#define H3D_V(T, R, WY, K, Q, N, S, P) \
  extern template void launch_tbl<T, R, WY, K, Q, N, S>(const StencilParams&, const KernelSpec&, hipStream_t);
#include "stencil_tbl_variants.inc"
#undef H3D_V

// Tile stride along z.  64 - 2K stored columns per 64-lane tile, or — fp64
// only — the largest multiple of 8 below it, which starts every tile's stored
// strip on a 64-byte boundary: whole 64-B write segments instead of partial
// ones at both seams, worth 2-10% per sweep at equal tile counts (MI355X,
// fp64 K = 3: 768^3 +2%, 1000^3 +3.5%, 1280^3 +10%; tools/gpu_zs2.sh).  The
// narrower stride can add a tile column, so it is taken only where the
// x-plan model, with that gain, predicts a shorter sweep (1024^3: 56 of 58,
// +4.6%; 512^3 would cross a round of workgroups and keeps 58), and only for
// boxes of >= 500 x planes: the slab shares of the 4- and 8-GPU runs (250 and
// 122 interior planes) lost 13% and 8% with it in the phantom-rank proxy
// while the 2-GPU share (510 planes) gained 1.5%.
static int lean_z_stride_plan(int64_t nx, int64_t ny, int64_t nz, int K, int esize, int TY, int slots, int U, int L);
int lean_z_stride(int64_t nx, int64_t ny, int64_t nz, int K, int esize, int TY, int slots, int U, int L) {
  // memoised: every eager launch asks (the N > 1 schedule is eager)
  static std::mutex mu;
  static std::map<std::array<int64_t, 9>, int> memo;
  const std::array<int64_t, 9> key{nx, ny, nz, K, esize, TY, slots, U, L};
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = memo.find(key);
    if (it != memo.end()) return it->second;
  }
  const int zs = lean_z_stride_plan(nx, ny, nz, K, esize, TY, slots, U, L);
  std::lock_guard<std::mutex> lk(mu);
  memo[key] = zs;
  return zs;
}

static int lean_z_stride_plan(int64_t nx, int64_t ny, int64_t nz, int K, int esize, int TY, int slots, int U, int L) {
  const int wide = 64 - 2 * K;
  const int aligned = esize == 8 ? wide & ~7 : wide;
  if (aligned == wide || aligned <= 0 || nx < 500) return wide;
  const int64_t nyb = std::max<int64_t>(1, (ny + TY - 2 * K - 1) / (TY - 2 * K));
  auto cost = [&](int zs) {
    const int64_t tiles = std::max<int64_t>(1, (nz + zs - 1) / zs) * nyb;
    const XPlan p = L > 0 ? fixed_xplan(nx, tiles, L) : plan_x(nx, tiles, slots, 2 * (K - 1), U, L == -1);
    return tiling_cost(p, nx, tiles, slots, 2 * (K - 1), U);
  };
  constexpr double kAlignedGain = 0.92;
  return cost(aligned) * kAlignedGain < cost(wide) ? aligned : wide;
}

// p == nullptr: only report whether the variant k resolves to exists
template <typename Real>
static bool dispatch_tbl(const StencilParams* p, const KernelSpec& k, hipStream_t s) {
  const KernelSpec r = k.resolved(sizeof(Real) == 8 ? DType::F64 : DType::F32);
  const int K = k.K, R = r.R, WY = r.WY, Q = r.NT;
  // Thin x slabs (the K-plane boundary slabs of x-slab decompositions) with
  // the default tile: 3-wave tiles of 9 x-rows marching along y
  // (launch_tbl swap_xy) instead of 48-row tiles marching 3 planes plus a
  // 4-plane pipeline fill along x.  Phantom rank of the 1024^3 fp64 slab
  // bench (64 GB/s emulated links): 8 ranks 0.2135 -> 0.2084 ms per step, 4
  // ranks 0.379 -> 0.359, 2 ranks unchanged (profiles/boundary_slabs_r02.md).
  if (p) {
    const Box& bx = p->box;
    // 4-plane slabs of a K = 3 sweep before a long sweep (Solver::enqueue_multi
    // thick): 5-wave tiles of 10 x-rows store all 4 planes in one tile
    if (K == 3 && k.V == 0 && k.R == 0 && k.WY == 0 && k.NT == 0 && bx.extent(0) == 4 &&
        bx.extent(1) >= 16 * bx.extent(0)) {
      if constexpr (sizeof(Real) == 8) launch_tbl<Real, 2, 5, 3, 3, 2, true>(*p, k, s);
      else launch_tbl<Real, 2, 5, 3, 3, 0, true>(*p, k, s);
      return true;
    }
    if (K == 3 && k.V == 0 && k.R == 0 && k.WY == 0 && k.NT == 0 && bx.extent(0) > 0 && bx.extent(0) <= 2 * K &&
        bx.extent(1) >= 16 * bx.extent(0)) {
      if constexpr (sizeof(Real) == 8) launch_tbl<Real, 3, 3, 3, 3, 2, true>(*p, k, s);
      else launch_tbl<Real, 3, 3, 3, 3, 0, true>(*p, k, s);
      return true;
    }
    // the (K+1)-plane boundary slabs of long sweeps across x halos (K = 4):
    // 4-wave tiles of 12 x-rows store the 4 slab planes
    if (K == 4 && k.V == 0 && k.R == 0 && k.WY == 0 && k.NT == 0 && bx.extent(0) > 0 && bx.extent(0) <= K &&
        bx.extent(1) >= 16 * bx.extent(0)) {
      if constexpr (sizeof(Real) == 8) launch_tbl<Real, 3, 4, 4, 3, 2, true>(*p, k, s);
      else launch_tbl<Real, 3, 4, 4, 3, 0, true>(*p, k, s);
      return true;
    }
  }
  if (r.V == 2) {  // two columns per lane: packed fp32 / 16-byte fp64 pairs (stencil_tbp.hip)
    const DType t = sizeof(Real) == 8 ? DType::F64 : DType::F32;
    if (!p) return lean_pair_supported(t, k);
    stencil_lean_pair(t, *p, k, s);
    return true;
  }
  if (r.V != 1 || r.WZ != 1) return false;  // one value per lane, one wave across z
#define H3D_TBL(RR, YY, KK, QQ)                                    \
  if (R == RR && WY == YY && K == KK && Q == QQ && r.O <= 0) {     \
    if (p) launch_tbl<Real, RR, YY, KK, QQ>(*p, k, s);             \
    return true;                                                   \
  }
  // output-store cache-policy bits (spec field 7: 2 = nt, 1 / 16 = sc0 / sc1), default shapes only
#define H3D_TBLA(RR, YY, KK, AA)                                       \
  if (R == RR && WY == YY && K == KK && Q == 3 && r.O == (AA)) {       \
    if (p) launch_tbl<Real, RR, YY, KK, 3, (AA), false>(*p, k, s);      \
    return true;                                                       \
  }
  H3D_TBLA(3, 16, 3, 2) H3D_TBLA(3, 16, 3, 3) H3D_TBLA(3, 16, 3, 17)
  H3D_TBLA(3, 16, 3, 18) H3D_TBLA(3, 16, 3, 19)
  H3D_TBLA(3, 16, 3, 2 | kResidualLastOnly)  // fp64 / fp32 K = 3 default, last residual only
  // ... and the partial / long sweeps' shapes (K = 2 candidates, the K = 4 default)
  H3D_TBLA(3, 16, 2, 2 | kResidualLastOnly) H3D_TBLA(5, 16, 2, 2 | kResidualLastOnly)
  H3D_TBLA(3, 12, 4, 2 | kResidualLastOnly)
  if constexpr (sizeof(Real) == 8) {
    // fp64 48-row K = 4 and 36-row K = 5 tiles of 12 waves: 167 VGPRs without
    // the K - 1 residual maxima
    H3D_TBLA(4, 12, 4, 2 | kResidualLastOnly) H3D_TBLA(3, 12, 5, 2 | kResidualLastOnly)
  }
  H3D_TBLA(2, 16, 4, 2) H3D_TBLA(3, 16, 2, 2) H3D_TBLA(5, 16, 2, 2)
  H3D_TBLA(3, 12, 4, 2)  // the fp64 K = 4 default (long sweeps: 12 waves, 36 rows)
  H3D_TBLA(4, 12, 4, 2)
#undef H3D_TBLA
  // 16 waves (<= 128 VGPRs, LDS 2K x 16 KiB): K <= 4; 12 waves (<= 168 VGPRs): K = 5
  H3D_TBL(3, 16, 4, 3) H3D_TBL(3, 16, 4, 4) H3D_TBL(3, 16, 3, 3) H3D_TBL(3, 16, 3, 4)
  H3D_TBL(2, 16, 4, 3) H3D_TBL(2, 16, 4, 4) H3D_TBL(2, 16, 5, 3) H3D_TBL(2, 16, 3, 3)
  H3D_TBL(2, 16, 4, 6) H3D_TBL(2, 16, 3, 6) H3D_TBL(3, 16, 3, 6) H3D_TBL(2, 16, 2, 6)
  H3D_TBL(3, 16, 2, 3) H3D_TBL(2, 16, 2, 3)
  H3D_TBL(4, 12, 4, 3) H3D_TBL(4, 12, 4, 4) H3D_TBL(4, 12, 5, 3) H3D_TBL(3, 12, 5, 3) H3D_TBL(3, 12, 4, 3)
  // 8 waves (<= 256 VGPRs, 2 per SIMD): 48-row tiles at K = 4; the fp64 K = 5 / 6 defaults
  H3D_TBL(6, 8, 4, 3) H3D_TBL(6, 8, 3, 3) H3D_TBL(6, 8, 4, 4) H3D_TBL(5, 8, 4, 3)
  H3D_TBL(3, 8, 5, 3) H3D_TBL(3, 8, 6, 3)
  if constexpr (sizeof(Real) == 4) {
    // fp32: half the registers and LDS per row, so deeper sweeps fit 16 waves
    H3D_TBL(4, 16, 4, 3) H3D_TBL(3, 16, 5, 3) H3D_TBL(4, 16, 5, 3) H3D_TBL(3, 16, 6, 3)
    H3D_TBL(4, 16, 6, 3) H3D_TBL(4, 16, 4, 4) H3D_TBL(3, 16, 5, 6)
  }
#undef H3D_TBL
  return false;
}

bool lean_supported(DType t, const KernelSpec& k) {
  return t == DType::F64 ? dispatch_tbl<double>(nullptr, k, nullptr) : dispatch_tbl<float>(nullptr, k, nullptr);
}

void stencil_lean(DType t, const StencilParams& p, const KernelSpec& k, void* stream) {
  if (p.box.empty()) return;
  const bool ok = t == DType::F64 ? dispatch_tbl<double>(&p, k, S(stream)) : dispatch_tbl<float>(&p, k, S(stream));
  if (!ok) {
    const KernelSpec r = k.resolved(t);
    HEAT3D_THROW("unsupported tl kernel variant V=" << r.V << " R=" << r.R << " WY=" << r.WY << " K=" << k.K
                                                    << " Q=" << r.NT);
  }
}

void sweep(DType t, const StencilParams& p, const KernelSpec& k, void* stream) {
  HEAT3D_CHECK(k.multi_step(), "sweep needs a K-step kernel (tl2..tl6)");
  stencil_lean(t, p, k, stream);
}

}  // namespace hip
}  // namespace heat3d
