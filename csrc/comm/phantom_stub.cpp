// heat3d-mi355x — stand-ins for the phantom-rank proxy in a build without it
// (cmake -DHEAT3D_PHANTOM=OFF): the production solver never reaches them; a
// --phantom run or a proxy tool gets a clear error instead of a link failure.
#include "comm.hpp"

namespace heat3d {

std::unique_ptr<Comm> make_phantom_comm(int, int, const PhantomOptions&) {
  HEAT3D_THROW("phantom-rank proxy not built (cmake -DHEAT3D_PHANTOM=ON)");
}

namespace hip {
void delay(double, void*, int, bool) { HEAT3D_THROW("phantom-rank proxy not built (HEAT3D_PHANTOM=OFF)"); }
void stamp(void*, void*) { HEAT3D_THROW("phantom-rank proxy not built (HEAT3D_PHANTOM=OFF)"); }
void delay_since(const void*, double, void*, int, bool) {
  HEAT3D_THROW("phantom-rank proxy not built (HEAT3D_PHANTOM=OFF)");
}
void paced_copy(const PacedCopy*, int, int, void*, bool) {
  HEAT3D_THROW("phantom-rank proxy not built (HEAT3D_PHANTOM=OFF)");
}
}  // namespace hip

}  // namespace heat3d
