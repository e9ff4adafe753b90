// Obstacle.h — box obstacle record of the planning package (reference
// include/path_planning_pkg/Obstacle.h, lib/Obstacle.cpp:6-19): centre pose, velocity,
// dimensions along x and y.
#ifndef OBSTACLE
#define OBSTACLE

#include <cmath>

#include "common.h"

namespace planning {

template <typename T>
struct Obstacle {
  Vector3D<T> _pose2D;      // centre (heading unused by the planner)
  Vector2D<T> _velocity;
  Vector2D<T> _dimensions;  // extent along x and y
  Obstacle(T position_x, T position_y, T velocity_x, T velocity_y, T dimension_x, T dimension_y)
      : _pose2D(position_x, position_y, T(0)), _velocity(velocity_x, velocity_y), _dimensions(dimension_x, dimension_y) {
    _pose2D._heading = std::atan2(_velocity._y, _velocity._x);  // heading of motion (Obstacle.cpp:13)
  }
  Obstacle(T position_x, T position_y, T dimension_x, T dimension_y)
      : Obstacle(position_x, position_y, T(0), T(0), dimension_x, dimension_y) {}
};

}  // namespace planning

#endif  // OBSTACLE
