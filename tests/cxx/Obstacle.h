// Minimal planning::Obstacle for the test harness (see common.h in this directory).
#ifndef HASTAR_TEST_OBSTACLE_H
#define HASTAR_TEST_OBSTACLE_H
#include "common.h"
namespace planning {
template <typename T>
struct Obstacle {
  Vector3D<T> _pose2D;
  Vector2D<T> _velocity;
  Vector2D<T> _dimensions;
  Obstacle(T x, T y, T dx, T dy) : _pose2D(x, y, 0), _velocity(0, 0), _dimensions(dx, dy) {}
};
}  // namespace planning
#endif
