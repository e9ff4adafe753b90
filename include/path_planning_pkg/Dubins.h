// Dubins.h — drop-in planning::Dubins<T> (reference include/path_planning_pkg/Dubins.h:
// 21-60, lib/Dubins.cpp), computed on the MI355X through include/hastar_units.h.
// T = float is bit-exact with the reference (the search kernel's glibc float ports);
// T = double runs ports of glibc 2.35's double libm for the CSC words: bit-exact as well
// (for |angles| < 2^27 * pi/2, where the ports' sin/cos need no __branred reduction).
// Like the reference object, the last call's word and parameters are kept (get_path_type).
#ifndef DUBINS
#define DUBINS

#include <array>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "common.h"
#include "hastar_dropin.h"

namespace planning {

enum class Path { RSR, RSL, LSR, LSL };

template <typename T>
class Dubins {
  static_assert(std::is_same<T, float>::value || std::is_same<T, double>::value, "Dubins<float> or Dubins<double>");

 public:
  Dubins(T r_min, T step_size)
      : _r_min(r_min), _step_size(step_size), _ang_step_size(step_size / r_min), _path_type(Path::RSR) {}

  // Dubins.cpp:19-69: length of the shortest CSC path
  T get_shortest_path_length(const Vector3D<T>& start, const Vector3D<T>& goal) {
    Vector2D<T> a, b, c, d;
    return get_shortest_path_length(start, goal, a, b, c, d);
  }
  T get_shortest_path_length(const Vector3D<T>& start, const Vector3D<T>& goal, Vector2D<T>& center_s_r,
                             Vector2D<T>& center_s_l, Vector2D<T>& center_g_r, Vector2D<T>& center_g_l) {
    const T s[3] = {start._x, start._y, start._heading}, g[3] = {goal._x, goal._y, goal._heading};
    T len = 0, ctr[8];
    int word = 0;
    if constexpr (std::is_same<T, float>::value)
      hastar_dropin::check(hastar_dubins_length_f32(hastar_dropin::device(), _r_min, 1, s, g, &len, &word, ctr), true);
    else
      hastar_dropin::check(hastar_dubins_length_f64(hastar_dropin::device(), _r_min, 1, s, g, &len, &word, ctr), true);
    center_s_r = Vector2D<T>(ctr[0], ctr[1]);
    center_s_l = Vector2D<T>(ctr[2], ctr[3]);
    center_g_r = Vector2D<T>(ctr[4], ctr[5]);
    center_g_l = Vector2D<T>(ctr[6], ctr[7]);
    _path_type = static_cast<Path>(word);
    return len;
  }
  // Dubins.cpp:125-153: the sampled shortest path (path / curvature are resized to the
  // samples) and {length, first arc longer than 90 degrees}
  std::pair<T, bool> get_shortest_path(const Vector3D<T>& start, const Vector3D<T>& goal, std::vector<Vector3D<T>>& path,
                                       std::vector<T>& path_curvature) {
    const T s[3] = {start._x, start._y, start._heading}, g[3] = {goal._x, goal._y, goal._heading};
    int cap = 4096, n = 0, flag = 0, word = 0;
    T len = 0;
    std::vector<T> xyh, cv;
    for (int attempt = 0; attempt < 2; ++attempt) {
      xyh.resize(3 * (size_t)cap);
      cv.resize(cap);
      int rc;
      if constexpr (std::is_same<T, float>::value)
        rc = hastar_dubins_path_f32(hastar_dropin::device(), _r_min, _step_size, s, g, xyh.data(), cv.data(), cap, &n,
                                    &len, &flag, &word);
      else
        rc = hastar_dubins_path_f64(hastar_dropin::device(), _r_min, _step_size, s, g, xyh.data(), cv.data(), cap, &n,
                                    &len, &flag, &word);
      if (rc == HASTAR_ENOSPC && n < 0 && attempt == 0) {
        cap = -n;
        continue;
      }
      hastar_dropin::check(rc, true);
      break;
    }
    path.resize(n);
    path_curvature.resize(n);
    for (int i = 0; i < n; ++i) {
      path[i] = Vector3D<T>(xyh[3 * i], xyh[3 * i + 1], xyh[3 * i + 2]);
      path_curvature[i] = cv[i];
    }
    _path_type = static_cast<Path>(word);
    return {len, flag != 0};
  }
  std::string get_path_type() const {
    static const char* names[4] = {"RSR", "RSL", "LSR", "LSL"};
    const int w = static_cast<int>(_path_type);
    return (w >= 0 && w < 4) ? std::string(names[w]) : std::string("undefined");
  }

 private:
  const T _r_min, _step_size, _ang_step_size;
  Path _path_type;
};

}  // namespace planning

#endif  // DUBINS
