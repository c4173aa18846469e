// heat3d-mi355x — CPU inner row of the FTCS update, built twice.
//
// The update's fused multiply-adds (kernels.hpp ftcs_update) must be real,
// correctly rounded FMAs on the host too.  Compiled for baseline x86-64 they
// become libm fma() calls (exact, but ~15x slower and never vectorised), so
// the row loop lives in cpu_rows.cpp, which CMake builds once for baseline
// x86-64 and once with -mfma -mavx2 (cpu_rows_fma.cpp); cpu_row_kernels()
// picks the FMA build when the running CPU has FMA + AVX2.  Both builds give
// bitwise identical results.
#pragma once

#include <cstdint>

namespace heat3d {
namespace cpu {

// out[k] = ftcs_update(in[k], ...) for k in [0, n); returns max |out - in|
// (NaN-propagating, as a double).
template <typename Real>
using FtcsRowFn = double (*)(const Real* in, Real* out, int64_t n, int64_t sx, int64_t sy, Real Dx, Real Dy,
                             Real Dz);

struct RowKernels {
  FtcsRowFn<double> f64;
  FtcsRowFn<float> f32;
  const char* isa;
};

const RowKernels& cpu_row_kernels();

namespace rows_generic {
double ftcs_row_f64(const double*, double*, int64_t, int64_t, int64_t, double, double, double);
double ftcs_row_f32(const float*, float*, int64_t, int64_t, int64_t, float, float, float);
}  // namespace rows_generic
namespace rows_fma {
double ftcs_row_f64(const double*, double*, int64_t, int64_t, int64_t, double, double, double);
double ftcs_row_f32(const float*, float*, int64_t, int64_t, int64_t, float, float, float);
}  // namespace rows_fma

}  // namespace cpu
}  // namespace heat3d
