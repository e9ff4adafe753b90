// AStar.h — drop-in planning::AStar<float> (reference include/path_planning_pkg/AStar.h:
// 27-73, lib/AStar.cpp), the holonomic-with-obstacles search on its own, as
// utils/astar/test_astar.cpp uses it.  It owns a planner handle used as a plain Grid2D
// (the reference's AStar without STORE_GRID_AS_REFERENCE owns its Grid2D, AStar.h:63-66):
// goal changes re-orient the frame without relocating the map, the map lives in HBM, and
// every search runs on the MI355X (the search kernel's holonomic A*: LDS open tree, exact
// std::set semantics, the node map's memoised and stale f values).  Only T = float.
#ifndef ASTAR
#define ASTAR

#include <limits>
#include <utility>
#include <vector>

#include "Node2D.h"
#include "Obstacle.h"
#include "common.h"
#include "hastar_dropin.h"

namespace planning {

template <typename T>
class AStar;  // only the float specialisation is provided

template <>
class AStar<float> {
 public:
  // AStar.cpp:7-13: the grid's constructor arguments (Grid2D.cpp:7-62)
  AStar(float grid_resolution, float obstacle_threshold, float obstacle_prob_min, float obstacle_prob_max,
        float obstacle_prob_free, int grid_size, bool grid_allow_diag_moves = true)
      : _n(grid_size) {
    const float steer = 0.0f, weight = 0.0f;
    hastar_params p{};
    p.dubins_shot_interval = 300;
    p.dubins_shot_interval_decay = 10;
    p.grid_resolution = grid_resolution;
    p.obstacle_threshold = obstacle_threshold;
    p.obstacle_prob_min = obstacle_prob_min;
    p.obstacle_prob_max = obstacle_prob_max;
    p.obstacle_prob_free = obstacle_prob_free;
    p.grid_size = grid_size;
    p.grid_2d_allow_diag_moves = grid_allow_diag_moves ? 1 : 0;
    p.step_size = 1.0f;
    p.max_lat_acc = 1.0f;
    p.max_long_dec = 1.0f;
    p.wheelbase = 1.0f;
    p.rear_to_cg = 0.5f;
    p.apf_rep_constant = 0.0f;
    p.apf_active_angle = 1.0f;
    p.num_angle_bins = 1;
    p.num_actions = 0;
    p.num_steering = 1;
    p.steering = &steer;
    p.curvature_weights = &weight;
    p.max_pops = 64;  // no Hybrid A* search runs on this handle
    hastar_dropin::check(hastar_create_f32(&p, hastar_dropin::device(), &_h));
    const float zero[2] = {0.0f, 0.0f};  // Grid2D's 7-argument constructor: goal = start = (0, 0)
    hastar_dropin::check(hastar_grid2d_update_goal_heading(_h, zero, zero));
  }
  ~AStar() {
    if (_h) hastar_destroy(_h);
  }
  AStar(const AStar&) = delete;
  AStar& operator=(const AStar&) = delete;

  void update_goal_node(const Node2D<float>& goal_node) {
    hastar_dropin::check(hastar_astar_set_goal_cell(_h, goal_node._posd._x, goal_node._posd._y));
  }
  // AStar.cpp:30-35: re-orient the grid on (goal, start), soft-reset the start cell
  void update_goal_start(const Vector2D<float>& goal, const Vector2D<float>& start, Node2D<float>& start_node) {
    const float g[2] = {goal._x, goal._y}, s[2] = {start._x, start._y};
    hastar_dropin::check(hastar_grid2d_update_goal_heading(_h, g, s));
    int cell[2];
    hastar_dropin::check(hastar_grid2d_set_start_node(_h, s, cell));
    float f = 0.0f;
    hastar_dropin::check(hastar_grid2d_node_cost(_h, cell[0], cell[1], &f));
    start_node = Node2D<float>(cell[0], cell[1], 0.0f, f, nullptr);  // soft reset: g = 0, f = h
  }
  // Grid2D::update_obstacles(obstacles, confidence) (Grid2D.cpp:99-139)
  void update_obstacles(const std::vector<Obstacle<float>>& obstacles, const std::vector<float>& confidence) {
    std::vector<float> b(obstacles.size() * 4);
    for (size_t k = 0; k < obstacles.size(); ++k) {
      b[4 * k] = obstacles[k]._pose2D._x;
      b[4 * k + 1] = obstacles[k]._pose2D._y;
      b[4 * k + 2] = obstacles[k]._dimensions._x;
      b[4 * k + 3] = obstacles[k]._dimensions._y;
    }
    hastar_dropin::check(hastar_update_boxes(_h, b.data(), confidence.data(), (int)obstacles.size(), 0.0f));
  }
  // Grid2D::update_obstacles(lines, confidence, line_width) (Grid2D.cpp:142-194)
  void update_obstacles(const std::vector<std::pair<Vector2D<float>, Vector2D<float>>>& lines,
                        const std::vector<float>& confidence, const float line_width) {
    std::vector<float> l(lines.size() * 4);
    for (size_t k = 0; k < lines.size(); ++k) {
      l[4 * k] = lines[k].first._x;
      l[4 * k + 1] = lines[k].first._y;
      l[4 * k + 2] = lines[k].second._x;
      l[4 * k + 3] = lines[k].second._y;
    }
    hastar_dropin::check(hastar_update_lines(_h, l.data(), confidence.data(), (int)lines.size(), line_width));
  }
  void update_obstacles() { hastar_dropin::check(hastar_decay(_h)); }  // Grid2D.cpp:197-208
  void reset() { hastar_dropin::check(hastar_reset(_h)); }              // AStar.cpp:56-60
  const std::vector<std::vector<float>>& get_obstacles() const {
    std::vector<float> flat((size_t)_n * _n);
    hastar_dropin::check(hastar_get_obstacles(_h, flat.data()));
    _grid.assign(_n, std::vector<float>(_n));
    for (int i = 0; i < _n; ++i)
      for (int j = 0; j < _n; ++j) _grid[i][j] = flat[(size_t)i * _n + j];
    return _grid;
  }
  // AStar.cpp:70-84: cost, and the path goal -> start (goal first) appended to `path`
  float find_path(const Vector2D<float>& goal, const Vector2D<float>& start, std::vector<Vector2D<float>>& path) {
    const float g[2] = {goal._x, goal._y}, s[2] = {start._x, start._y};
    float cost = std::numeric_limits<float>::max();
    int n = 0;
    std::vector<float> xy(2 * (size_t)_n * _n + 2);
    hastar_dropin::check(hastar_astar_find_path(_h, g, s, 0, &cost, xy.data(), (int)(xy.size() / 2), &n));
    if (cost < std::numeric_limits<float>::max()) {
      path.push_back(goal);
      for (int i = 0; i < n; ++i) path.emplace_back(xy[2 * i], xy[2 * i + 1]);
    }
    return cost;
  }
  // AStar.cpp:87-97
  float find_path(const Vector2D<float>& goal, const Vector2D<float>& start, bool get_cost_only = true) {
    const float g[2] = {goal._x, goal._y}, s[2] = {start._x, start._y};
    float cost = std::numeric_limits<float>::max();
    hastar_dropin::check(hastar_astar_find_path(_h, g, s, get_cost_only ? 1 : 0, &cost, nullptr, 0, nullptr));
    return cost;
  }
  // AStar.cpp:100-113: memoised cost-to-goal of a cell
  float find_path(const int start_i, const int start_j) {
    float cost = std::numeric_limits<float>::max();
    hastar_dropin::check(hastar_astar_cost(_h, start_i, start_j, &cost));
    return cost;
  }

 private:
  hastar_handle _h = nullptr;
  int _n;
  mutable std::vector<std::vector<float>> _grid;
};

}  // namespace planning

#endif  // ASTAR
