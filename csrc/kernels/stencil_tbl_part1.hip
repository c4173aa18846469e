// heat3d-mi355x — instantiation unit 1 of the lean sweep kernel variants
// (stencil_tbl_variants.inc entries with PART = 1); see stencil_tbl.hip.
#include "stencil_tbl_impl.hpp"

namespace heat3d {
namespace hip {

#define H3D_SEL0(...)
#define H3D_SEL1(...)
#define H3D_SEL2(...)
#define H3D_SEL3(...)
#undef H3D_SEL1
#define H3D_SEL1(...) __VA_ARGS__
#define H3D_V(T, R, WY, K, Q, N, S, P) \
  H3D_SEL##P(template void launch_tbl<T, R, WY, K, Q, N, S>(const StencilParams&, const KernelSpec&, hipStream_t);)
#include "stencil_tbl_variants.inc"
#undef H3D_V

}  // namespace hip
}  // namespace heat3d
