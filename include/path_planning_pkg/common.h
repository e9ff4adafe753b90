// common.h — the planning package's shared value types and angle helpers
// (reference include/path_planning_pkg/common.h:8-169), for code that includes the
// reference's headers and links libhastar_amd.so.  Host-side value types: the arithmetic is
// the reference's (same expression types; T = float angles go through glibc's cosf/sinf/
// fmod like the reference build), so values built here equal the reference's bit for bit.
#ifndef PLANNING_COMMON
#define PLANNING_COMMON

#include <cmath>

namespace planning {

// common.h:8-12: nearest multiple of `precision`
template <typename T>
T round_to_nearest(const T value, const T precision) {
  return std::round(value / precision) * precision;
}

// common.h:15-29: angle into [-pi, pi]; the fmod and the comparisons promote to double
template <typename T>
T wrap_pi(const T angle) {
  const T w = std::fmod(angle, 2 * M_PI);
  return (w > M_PI) ? static_cast<T>(w - 2 * M_PI) : (w < -M_PI) ? static_cast<T>(w + 2 * M_PI) : w;
}

// common.h:31-36: discrete heading bin (truncation after the double offset by pi)
template <typename T>
int get_heading_index(const T heading, const T precision) {
  return static_cast<int>((round_to_nearest(heading, precision) + M_PI) / precision);
}

// common.h:40-122: 2-D vector
template <typename T>
struct Vector2D {
  T _x, _y;
  Vector2D() : _x(T(0)), _y(T(0)) {}
  Vector2D(T x, T y) : _x(x), _y(y) {}
  Vector2D(const Vector2D&) = default;
  template <typename U>
  Vector2D(const Vector2D<U>& o) : _x(static_cast<T>(o._x)), _y(static_cast<T>(o._y)) {}
  Vector2D& operator=(const Vector2D&) = default;
  template <typename U>
  Vector2D& operator=(const Vector2D<U>& o) {
    _x = static_cast<T>(o._x);
    _y = static_cast<T>(o._y);
    return *this;
  }
  // the vector expressed in a frame rotated by `angle` (x' = x c + y s, y' = -x s + y c)
  Vector2D get_rotated_vector(const T angle) const {
    const T c = std::cos(angle), s = std::sin(angle);
    return Vector2D(_x * c + _y * s, -_x * s + _y * c);
  }
  void rotate_vector(const T angle) { *this = get_rotated_vector(angle); }
  Vector2D operator+(const Vector2D& o) const { return Vector2D(_x + o._x, _y + o._y); }
  Vector2D operator-(const Vector2D& o) const { return Vector2D(_x - o._x, _y - o._y); }
  Vector2D operator*(const Vector2D& o) const { return Vector2D(_x * o._x, _y * o._y); }
  Vector2D operator/(const Vector2D& o) const { return Vector2D(_x / o._x, _y / o._y); }
  Vector2D operator+(const T v) const { return Vector2D(_x + v, _y + v); }
  Vector2D operator-(const T v) const { return Vector2D(_x - v, _y - v); }
  Vector2D operator*(const T v) const { return Vector2D(_x * v, _y * v); }
  Vector2D operator/(const T v) const { return Vector2D(_x / v, _y / v); }
};

// common.h:124-169: 2-D pose (heading w.r.t. the x axis)
template <typename T>
struct Vector3D {
  T _x, _y, _heading;
  Vector3D() : _x(T(0)), _y(T(0)), _heading(T(0)) {}
  Vector3D(T x, T y, T heading) : _x(x), _y(y), _heading(heading) {}
  Vector3D(const Vector3D&) = default;
  template <typename U>
  Vector3D(const Vector3D<U>& o)
      : _x(static_cast<T>(o._x)), _y(static_cast<T>(o._y)), _heading(static_cast<T>(o._heading)) {}
  Vector3D& operator=(const Vector3D&) = default;
  template <typename U>
  Vector3D& operator=(const Vector3D<U>& o) {
    _x = static_cast<T>(o._x);
    _y = static_cast<T>(o._y);
    _heading = static_cast<T>(o._heading);
    return *this;
  }
  // the pose in a frame rotated by `angle`: position as Vector2D, heading wrapped
  Vector3D get_rotated_vector(const T angle) const {
    const T c = std::cos(angle), s = std::sin(angle);
    return Vector3D(_x * c + _y * s, -_x * s + _y * c, wrap_pi<T>(_heading - angle));
  }
  Vector3D operator+(const Vector3D& o) const { return Vector3D(_x + o._x, _y + o._y, _heading + o._heading); }
  Vector3D operator-(const Vector3D& o) const { return Vector3D(_x - o._x, _y - o._y, _heading - o._heading); }
  Vector3D operator*(const Vector3D& o) const { return Vector3D(_x * o._x, _y * o._y, _heading * o._heading); }
  Vector3D operator/(const Vector3D& o) const { return Vector3D(_x / o._x, _y / o._y, _heading / o._heading); }
};

}  // namespace planning

#endif  // PLANNING_COMMON
