// Minimal planning::Vector2D / Vector3D for compiling the drop-in HybridAStar.h in the
// test harness without the ROS package (whose own common.h provides the full types).
// Only the members the wrapper and the harness touch are defined.
#ifndef HASTAR_TEST_COMMON_H
#define HASTAR_TEST_COMMON_H
namespace planning {
template <typename T>
struct Vector2D {
  T _x, _y;
  Vector2D(T x, T y) : _x(x), _y(y) {}
};
template <typename T>
struct Vector3D {
  T _x, _y, _heading;
  Vector3D(T x, T y, T heading) : _x(x), _y(y), _heading(heading) {}
};
}  // namespace planning
#endif
