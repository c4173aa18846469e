// heat3d-mi355x — FTCS row kernels (see cpu_rows.hpp).  This file is compiled
// twice: as is (namespace rows_generic) and from cpu_rows_fma.cpp with
// H3D_ROWS_NS=rows_fma and -mfma -mavx2.
#include <cmath>

#include "cpu_rows.hpp"
#include "kernels.hpp"

#ifndef H3D_ROWS_NS
#define H3D_ROWS_NS rows_generic
#define H3D_ROWS_DISPATCH 1
#endif

namespace heat3d {
namespace cpu {
namespace H3D_ROWS_NS {

template <typename Real>
static inline double row(const Real* __restrict in, Real* __restrict out, int64_t n, int64_t sx, int64_t sy,
                         Real Dx, Real Dy, Real Dz) {
  double lres = 0.0;
  bool nan = false;
  for (int64_t k = 0; k < n; ++k) {
    const Real T = in[k];
    const Real nv = ftcs_update<Real>(T, in[k - sx], in[k + sx], in[k - sy], in[k + sy], in[k - 1], in[k + 1], Dx,
                                      Dy, Dz);
    out[k] = nv;
    const double d = resid_abs(nv, T);  // in the field's precision (kernels.hpp)
    nan |= d != d;
    lres = d > lres ? d : lres;
  }
  return nan ? std::nan("") : lres;
}

double ftcs_row_f64(const double* in, double* out, int64_t n, int64_t sx, int64_t sy, double Dx, double Dy,
                    double Dz) {
  return row<double>(in, out, n, sx, sy, Dx, Dy, Dz);
}
double ftcs_row_f32(const float* in, float* out, int64_t n, int64_t sx, int64_t sy, float Dx, float Dy, float Dz) {
  return row<float>(in, out, n, sx, sy, Dx, Dy, Dz);
}

}  // namespace H3D_ROWS_NS

#ifdef H3D_ROWS_DISPATCH
const RowKernels& cpu_row_kernels() {
  static const RowKernels k = [] {
    __builtin_cpu_init();
    if (__builtin_cpu_supports("fma") && __builtin_cpu_supports("avx2"))
      return RowKernels{rows_fma::ftcs_row_f64, rows_fma::ftcs_row_f32, "x86-64+fma+avx2"};
    return RowKernels{rows_generic::ftcs_row_f64, rows_generic::ftcs_row_f32, "x86-64 (libm fma)"};
  }();
  return k;
}
#endif

}  // namespace cpu
}  // namespace heat3d
