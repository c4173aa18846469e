// heat3d-mi355x — shared basic types.
//
// Face / axis enums mirror the reference's COORDINATE / DIRECTION enums
// (reference heat3D.cu:157-174): LEFT/RIGHT = -x/+x, BOTTOM/TOP = -y/+y,
// BACK/FRONT = -z/+z.  Everything here is plain C++17 and builds without HIP.
#pragma once

#include <cstdint>
#include <sstream>
#include <stdexcept>
#include <string>

// Functions shared by host code and gfx950 kernels (header-only helpers).
#if defined(__HIPCC__)
#define H3D_HD __host__ __device__
#else
#define H3D_HD
#endif

namespace heat3d {

enum Axis : int { AX_X = 0, AX_Y = 1, AX_Z = 2 };

enum class Face : int { Left = 0, Right = 1, Bottom = 2, Top = 3, Back = 4, Front = 5 };
constexpr int kNumFaces = 6;

inline int face_axis(Face f) { return static_cast<int>(f) / 2; }
inline int face_side(Face f) { return static_cast<int>(f) % 2; }  // 0 = low, 1 = high
inline Face face_of(int axis, int side) { return static_cast<Face>(axis * 2 + side); }
inline Face opposite(Face f) { return static_cast<Face>(static_cast<int>(f) ^ 1); }
const char* face_name(Face f);

enum class DType : int { F64 = 0, F32 = 1 };
inline std::size_t dtype_size(DType t) { return t == DType::F64 ? 8 : 4; }
const char* dtype_name(DType t);
DType parse_dtype(const std::string& s);

// Half-open 3D index box [x0,x1) x [y0,y1) x [z0,z1) in some index space.
struct Box {
  int64_t lo[3] = {0, 0, 0};
  int64_t hi[3] = {0, 0, 0};
  H3D_HD int64_t extent(int a) const { return hi[a] > lo[a] ? hi[a] - lo[a] : 0; }
  H3D_HD int64_t volume() const { return extent(0) * extent(1) * extent(2); }
  H3D_HD bool empty() const { return volume() == 0; }
  std::string str() const;
};

// Error type carrying file:line context; every fatal condition in the
// framework throws this (the reference aborted silently, heat3D.cu:291).
class Error : public std::runtime_error {
 public:
  explicit Error(const std::string& m) : std::runtime_error(m) {}
};

#define HEAT3D_THROW(msg)                                                    \
  do {                                                                       \
    std::ostringstream _h3d_os;                                              \
    _h3d_os << __FILE__ << ":" << __LINE__ << ": " << msg;                   \
    throw ::heat3d::Error(_h3d_os.str());                                    \
  } while (0)

#define HEAT3D_CHECK(cond, msg)                                              \
  do {                                                                       \
    if (!(cond)) HEAT3D_THROW("check failed: " #cond ": " << msg);          \
  } while (0)

}  // namespace heat3d
