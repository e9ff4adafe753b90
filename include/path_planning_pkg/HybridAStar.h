// HybridAStar.h — drop-in replacement of the reference's planner facade
// `planning::HybridAStar<T>` (reference include/path_planning_pkg/HybridAStar.h:27-75,
// lib/HybridAStar.cpp:7-286), implemented on the MI355X C ABI (include/hastar.h).
//
// The public member functions keep their reference signatures, so the unchanged caller
// (src/local_planner.cpp:158-316) compiles against this header and links
// libhastar_amd.so instead of lib/HybridAStar.cpp + Grid2D/Grid3D/AStar/Dubins/
// VehicleModel/Node*.cpp.  The vector types come from the package's own "common.h" and
// "Obstacle.h" (Vector2D/Vector3D/Obstacle), which this header does not redefine.
//
// Both instantiations of the reference exist (HybridAStar.cpp:285-286): T = float over
// include/hastar.h (bit-exact with the reference), T = double over include/hastar_f64.h (the
// GPU search in f64 on ports of glibc 2.35's double libm: bit-exact).  The ROS node runs
// float (local_planner.cpp:509) and compiles LocalPlanner<double> too (:378-500).
// Differences a caller can observe:
//   * a HIP/device failure throws std::runtime_error (the reference has no device to fail);
//   * a search ended by HASTAR_MAX_POPS_HARD or by exhausted device memory returns
//     {FLT_MAX, false} (the reference has no pop limit and would throw bad_alloc);
//   * find_path appends to `path`/`curvature` like the reference does for the empty
//     vectors its caller passes (HybridAStar.cpp:208-262 mixes push_back and resize, so
//     non-empty inputs are not a supported contract there either);
//   * the device is HIP ordinal $HASTAR_DEVICE (default 0);
//   * extension: set_relaxed(true) — or $HASTAR_RELAXED=1 at construction, so the unchanged
//     caller can opt in — routes find_path to the RELAXED search mode
//     (hastar_find_path_relaxed_batch).  That mode is NOT the reference's
//     algorithm: its paths are valid and comparable in cost but not identical.  It keeps its
//     heuristic field until reset() / update_goal(), as the reference keeps its A* memo.
#ifndef HYBRID_ASTAR
#define HYBRID_ASTAR

#include <cstdio>
#include <cstdlib>
#include <limits>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../hastar.h"
#include "../hastar_f64.h"
#include "Obstacle.h"
#include "common.h"

namespace planning {

template <typename T>
class HybridAStar;  // float and double specialisations below (the reference's two instantiations)

template <>
class HybridAStar<float> {
 public:
  // HybridAStar.h:33-38 — same 20 arguments, same order and meaning.
  HybridAStar(int dubins_shot_interval, int dubins_shot_interval_decay, float grid_resolution,
              float obstacle_threshold, float obstacle_prob_min, float obstacle_prob_max, float obstacle_prob_free,
              int grid_size, bool grid_2d_allow_diag_moves, float step_size, float max_lat_acc, float max_long_dec,
              float wheelbase, float rear_to_cg, float apf_rep_constant, float apf_active_angle, int num_angle_bins,
              int num_actions, const std::vector<float>& steering, const std::vector<float>& curvature_weights)
      : _n(grid_size) {
    if (steering.size() != curvature_weights.size())
      throw std::invalid_argument("HybridAStar: steering and curvature_weights differ in length");
    hastar_params p{};
    p.dubins_shot_interval = dubins_shot_interval;
    p.dubins_shot_interval_decay = dubins_shot_interval_decay;
    p.grid_resolution = grid_resolution;
    p.obstacle_threshold = obstacle_threshold;
    p.obstacle_prob_min = obstacle_prob_min;
    p.obstacle_prob_max = obstacle_prob_max;
    p.obstacle_prob_free = obstacle_prob_free;
    p.grid_size = grid_size;
    p.grid_2d_allow_diag_moves = grid_2d_allow_diag_moves ? 1 : 0;
    p.step_size = step_size;
    p.max_lat_acc = max_lat_acc;
    p.max_long_dec = max_long_dec;
    p.wheelbase = wheelbase;
    p.rear_to_cg = rear_to_cg;
    p.apf_rep_constant = apf_rep_constant;
    p.apf_active_angle = apf_active_angle;
    p.num_angle_bins = num_angle_bins;
    p.num_actions = num_actions;
    p.num_steering = (int)steering.size();
    p.steering = steering.data();
    p.curvature_weights = curvature_weights.data();
    const char* dev = std::getenv("HASTAR_DEVICE");
    check(hastar_create_f32(&p, dev ? std::atoi(dev) : 0, &_h));
    // The unchanged caller cannot call set_relaxed(), so it may opt in through the
    // environment; since that silently changes find_path's results (a different algorithm),
    // the switch is announced once on stderr.
    const char* rel = std::getenv("HASTAR_RELAXED");
    _relaxed = rel && std::atoi(rel) != 0;
    if (_relaxed) {
      static bool announced = false;
      if (!announced) {
        announced = true;
        std::fprintf(stderr, "HybridAStar: HASTAR_RELAXED=1 selects the relaxed (non-reference) search mode\n");
      }
    }
  }
  // extension (not in the reference): select the relaxed search mode for find_path
  void set_relaxed(bool on) { _relaxed = on; }
  bool relaxed() const { return _relaxed; }
  ~HybridAStar() {
    if (_h) hastar_destroy(_h);
  }
  HybridAStar(const HybridAStar&) = delete;
  HybridAStar& operator=(const HybridAStar&) = delete;

  // HybridAStar.cpp:29-33 (Grid3D.cpp:22-44 + Grid2D.cpp:99-139)
  void update_obstacles(const std::vector<Obstacle<float>>& obstacles, const std::vector<float>& confidence,
                        const float apf_added_radius) {
    std::vector<float> b(obstacles.size() * 4);
    for (size_t k = 0; k < obstacles.size(); ++k) {
      b[4 * k] = obstacles[k]._pose2D._x;
      b[4 * k + 1] = obstacles[k]._pose2D._y;
      b[4 * k + 2] = obstacles[k]._dimensions._x;
      b[4 * k + 3] = obstacles[k]._dimensions._y;
    }
    check(hastar_update_boxes(_h, b.data(), confidence.data(), (int)obstacles.size(), apf_added_radius));
  }
  // HybridAStar.cpp:36-40 (Grid2D.cpp:142-194)
  void update_obstacles(const std::vector<std::pair<Vector2D<float>, Vector2D<float>>>& lines,
                        const std::vector<float>& confidence, const float line_width) {
    std::vector<float> l(lines.size() * 4);
    for (size_t k = 0; k < lines.size(); ++k) {
      l[4 * k] = lines[k].first._x;
      l[4 * k + 1] = lines[k].first._y;
      l[4 * k + 2] = lines[k].second._x;
      l[4 * k + 3] = lines[k].second._y;
    }
    check(hastar_update_lines(_h, l.data(), confidence.data(), (int)lines.size(), line_width));
  }
  // HybridAStar.cpp:43-46 (Grid2D.cpp:197-208)
  void update_obstacles() { check(hastar_decay(_h)); }
  // HybridAStar.cpp:49-52
  void reset() { check(hastar_reset(_h)); }
  // HybridAStar.cpp:55-59
  void update_goal(const Vector3D<float>& goal, const Vector3D<float>& start) {
    const float g[3] = {goal._x, goal._y, goal._heading};
    const float s[3] = {start._x, start._y, start._heading};
    check(hastar_update_goal(_h, g, s));
  }
  // HybridAStar.h:48 — rows of the log-odds map, as the reference's Grid2D stores it
  const std::vector<std::vector<float>>& get_obstacles() const {
    std::vector<float> flat((size_t)_n * _n);
    check(hastar_get_obstacles(_h, flat.data()));
    _grid_cache.assign(_n, std::vector<float>(_n));
    for (int i = 0; i < _n; ++i)
      for (int j = 0; j < _n; ++j) _grid_cache[i][j] = flat[(size_t)i * _n + j];
    return _grid_cache;
  }
  // HybridAStar.cpp:68-88
  std::pair<float, bool> find_path(const float vel_init, const Vector3D<float>& start,
                                   std::vector<Vector3D<float>>& path, std::vector<float>& curvature) {
    const float s[3] = {start._x, start._y, start._heading};
    int len = 0, ok = 0;
    float cost = std::numeric_limits<float>::max();
    if (_xyh.size() < 3 * _cap) _xyh.resize(3 * _cap);
    if (_curv.size() < _cap) _curv.resize(_cap);
    int rc;
    if (_relaxed) {
      hastar_relaxed_opts o{};
      o.reuse_heuristic = 1;
      hastar_stats st{};
      rc = hastar_find_path_relaxed_batch(&_h, 1, &vel_init, s, _xyh.data(), _curv.data(), (int)_cap, &len, &cost,
                                          &ok, &st, &o);
    } else {
      rc = hastar_find_path(_h, vel_init, s, _xyh.data(), _curv.data(), (int)_cap, &len, &cost, &ok, nullptr);
    }
    if (rc == HASTAR_ENOSPC && len > (int)_cap) {  // grow and fetch the stored path
      _cap = (size_t)len;
      _xyh.resize(3 * _cap);
      _curv.resize(_cap);
      rc = hastar_copy_path(_h, _xyh.data(), _curv.data(), (int)_cap, &len);
    }
    // A search never stops at a fixed arena size (it is parked and resumed in a larger one),
    // so HASTAR_EOVERFLOW only means an explicit HASTAR_MAX_POPS_HARD budget or exhausted
    // device memory: reported as the reference's failure pair, like a search that found
    // no path, not as an exception the unchanged caller would not catch.
    if (rc == HASTAR_EOVERFLOW) return {std::numeric_limits<float>::max(), false};
    check(rc);
    for (int i = 0; i < len; ++i) {
      path.emplace_back(_xyh[3 * i], _xyh[3 * i + 1], _xyh[3 * i + 2]);
      curvature.push_back(_curv[i]);
    }
    return {cost, ok != 0};
  }

 private:
  static void check(int rc) {
    if (rc < 0) throw std::runtime_error(std::string("hastar: ") + hastar_last_error());
  }
  hastar_handle _h = nullptr;
  int _n;
  size_t _cap = 4096;
  bool _relaxed = false;
  std::vector<float> _xyh, _curv;
  mutable std::vector<std::vector<float>> _grid_cache;
};

// HybridAStar<double> (HybridAStar.cpp:285-286), used by LocalPlanner<double>
// (local_planner.cpp:158-166, 378-500): the same members over include/hastar_f64.h.
template <>
class HybridAStar<double> {
 public:
  HybridAStar(int dubins_shot_interval, int dubins_shot_interval_decay, double grid_resolution,
              double obstacle_threshold, double obstacle_prob_min, double obstacle_prob_max, double obstacle_prob_free,
              int grid_size, bool grid_2d_allow_diag_moves, double step_size, double max_lat_acc, double max_long_dec,
              double wheelbase, double rear_to_cg, double apf_rep_constant, double apf_active_angle,
              int num_angle_bins, int num_actions, const std::vector<double>& steering,
              const std::vector<double>& curvature_weights)
      : _n(grid_size) {
    if (steering.size() != curvature_weights.size())
      throw std::invalid_argument("HybridAStar: steering and curvature_weights differ in length");
    hastar_params_f64 p{};
    p.dubins_shot_interval = dubins_shot_interval;
    p.dubins_shot_interval_decay = dubins_shot_interval_decay;
    p.grid_resolution = grid_resolution;
    p.obstacle_threshold = obstacle_threshold;
    p.obstacle_prob_min = obstacle_prob_min;
    p.obstacle_prob_max = obstacle_prob_max;
    p.obstacle_prob_free = obstacle_prob_free;
    p.grid_size = grid_size;
    p.grid_2d_allow_diag_moves = grid_2d_allow_diag_moves ? 1 : 0;
    p.step_size = step_size;
    p.max_lat_acc = max_lat_acc;
    p.max_long_dec = max_long_dec;
    p.wheelbase = wheelbase;
    p.rear_to_cg = rear_to_cg;
    p.apf_rep_constant = apf_rep_constant;
    p.apf_active_angle = apf_active_angle;
    p.num_angle_bins = num_angle_bins;
    p.num_actions = num_actions;
    p.num_steering = (int)steering.size();
    p.steering = steering.data();
    p.curvature_weights = curvature_weights.data();
    const char* dev = std::getenv("HASTAR_DEVICE");
    check(hastar64_create(&p, dev ? std::atoi(dev) : 0, &_h));
  }
  ~HybridAStar() {
    if (_h) hastar64_destroy(_h);
  }
  HybridAStar(const HybridAStar&) = delete;
  HybridAStar& operator=(const HybridAStar&) = delete;

  void update_obstacles(const std::vector<Obstacle<double>>& obstacles, const std::vector<double>& confidence,
                        const double apf_added_radius) {
    std::vector<double> b(obstacles.size() * 4);
    for (size_t k = 0; k < obstacles.size(); ++k) {
      b[4 * k] = obstacles[k]._pose2D._x;
      b[4 * k + 1] = obstacles[k]._pose2D._y;
      b[4 * k + 2] = obstacles[k]._dimensions._x;
      b[4 * k + 3] = obstacles[k]._dimensions._y;
    }
    check(hastar64_update_boxes(_h, b.data(), confidence.data(), (int)obstacles.size(), apf_added_radius));
  }
  void update_obstacles(const std::vector<std::pair<Vector2D<double>, Vector2D<double>>>& lines,
                        const std::vector<double>& confidence, const double line_width) {
    std::vector<double> l(lines.size() * 4);
    for (size_t k = 0; k < lines.size(); ++k) {
      l[4 * k] = lines[k].first._x;
      l[4 * k + 1] = lines[k].first._y;
      l[4 * k + 2] = lines[k].second._x;
      l[4 * k + 3] = lines[k].second._y;
    }
    check(hastar64_update_lines(_h, l.data(), confidence.data(), (int)lines.size(), line_width));
  }
  void update_obstacles() { check(hastar64_decay(_h)); }
  void reset() { check(hastar64_reset(_h)); }
  void update_goal(const Vector3D<double>& goal, const Vector3D<double>& start) {
    const double g[3] = {goal._x, goal._y, goal._heading};
    const double s[3] = {start._x, start._y, start._heading};
    check(hastar64_update_goal(_h, g, s));
  }
  const std::vector<std::vector<double>>& get_obstacles() const {
    std::vector<double> flat((size_t)_n * _n);
    check(hastar64_get_obstacles(_h, flat.data()));
    _grid_cache.assign(_n, std::vector<double>(_n));
    for (int i = 0; i < _n; ++i)
      for (int j = 0; j < _n; ++j) _grid_cache[i][j] = flat[(size_t)i * _n + j];
    return _grid_cache;
  }
  std::pair<double, bool> find_path(const double vel_init, const Vector3D<double>& start,
                                    std::vector<Vector3D<double>>& path, std::vector<double>& curvature) {
    const double s[3] = {start._x, start._y, start._heading};
    int len = 0, ok = 0;
    double cost = std::numeric_limits<double>::max();
    if (_xyh.size() < 3 * _cap) _xyh.resize(3 * _cap);
    if (_curv.size() < _cap) _curv.resize(_cap);
    int rc = hastar64_find_path(_h, vel_init, s, _xyh.data(), _curv.data(), (int)_cap, &len, &cost, &ok, nullptr);
    if (rc == HASTAR_ENOSPC && len > (int)_cap) {
      _cap = (size_t)len;
      _xyh.resize(3 * _cap);
      _curv.resize(_cap);
      rc = hastar64_copy_path(_h, _xyh.data(), _curv.data(), (int)_cap, &len);
    }
    if (rc == HASTAR_EOVERFLOW) return {std::numeric_limits<double>::max(), false};  // no device memory left
    check(rc);
    for (int i = 0; i < len; ++i) {
      path.emplace_back(_xyh[3 * i], _xyh[3 * i + 1], _xyh[3 * i + 2]);
      curvature.push_back(_curv[i]);
    }
    return {cost, ok != 0};
  }

 private:
  static void check(int rc) {
    if (rc < 0) throw std::runtime_error(std::string("hastar: ") + hastar_last_error());
  }
  hastar64_handle _h = nullptr;
  int _n;
  size_t _cap = 4096;
  std::vector<double> _xyh, _curv;
  mutable std::vector<std::vector<double>> _grid_cache;
};

}  // namespace planning

#endif  // HYBRID_ASTAR
