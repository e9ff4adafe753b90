// Grid2D.h — drop-in planning::Grid2D<float> (reference include/path_planning_pkg/Grid2D.h:
// 16-61, lib/Grid2D.cpp): the log-odds occupancy map and node map of one planner, held in
// HBM by a planner handle (include/hastar.h) and updated by the MI355X map kernels.
// Node access: the device keeps each node's f (memoised cost-to-goal or stale f) and its h;
// g and prev are search-internal there, so Node2D objects handed out (get_neighbors,
// update_goal_heading, set_start_node*) carry f and h with g = 0, prev = null, and are owned
// by this object (pointers stay valid for its lifetime).  update_costs (AStar's memo write)
// runs inside the device search and is not exposed.  Only T = float.
#ifndef GRID2D
#define GRID2D

#include <cmath>
#include <memory>
#include <unordered_map>
#include <utility>
#include <vector>

#include "Node2D.h"
#include "Obstacle.h"
#include "common.h"
#include "hastar_dropin.h"

namespace planning {

template <typename T>
class Grid2D;  // only the float specialisation is provided

template <>
class Grid2D<float> {
 public:
  Grid2D(float resolution, float obstacle_threshold, float obstacle_prob_min, float obstacle_prob_max,
         float obstacle_prob_free, int grid_size, Vector2D<float> goal, Vector2D<float> start, bool allow_diag_moves)
      : Grid2D(resolution, obstacle_threshold, obstacle_prob_min, obstacle_prob_max, obstacle_prob_free, grid_size,
               allow_diag_moves) {
    update_goal_heading(goal, start);
  }
  Grid2D(float resolution, float obstacle_threshold, float obstacle_prob_min, float obstacle_prob_max,
         float obstacle_prob_free, int grid_size, bool allow_diag_moves)
      : _res(resolution), _n(grid_size), _diag(allow_diag_moves), _thr(logodds(obstacle_threshold)) {
    hastar_params p = base_params(resolution, obstacle_threshold, obstacle_prob_min, obstacle_prob_max,
                                  obstacle_prob_free, grid_size, allow_diag_moves);
    const float steer = 0.0f, weight = 0.0f;
    p.num_steering = 1;
    p.steering = &steer;
    p.curvature_weights = &weight;
    hastar_dropin::check(hastar_create_f32(&p, hastar_dropin::device(), &_h));
    const float zero[2] = {0.0f, 0.0f};
    hastar_dropin::check(hastar_grid2d_update_goal_heading(_h, zero, zero));
  }
  virtual ~Grid2D() {
    if (_h) hastar_destroy(_h);
  }
  Grid2D(const Grid2D&) = delete;
  Grid2D& operator=(const Grid2D&) = delete;

  // Grid2D.cpp:72-96: traversable neighbour cells of (xd, yd) with their move costs
  void get_neighbors(const int xd, const int yd, std::vector<std::pair<Node2D<float>*, float>>& neighbors) {
    static const int d8[8][2] = {{0, -1}, {1, -1}, {1, 0}, {1, 1}, {0, 1}, {-1, 1}, {-1, 0}, {-1, -1}};
    static const int d4[4][2] = {{0, -1}, {1, 0}, {0, 1}, {-1, 0}};
    const auto& occ = get_obstacle_map();
    neighbors.clear();
    const int na = _diag ? 8 : 4;
    for (int k = 0; k < na; ++k) {
      const int dx = _diag ? d8[k][0] : d4[k][0], dy = _diag ? d8[k][1] : d4[k][1];
      const int i = xd + dx, j = yd + dy;
      if (i > -1 && i < _n && j > -1 && j < _n && occ[i][j] < _thr)
        neighbors.emplace_back(node(i, j), _res * std::sqrt(static_cast<float>(dx * dx + dy * dy)));
    }
  }
  // Grid2D.cpp:99-208: box raster (no APF list), lines, free-space decay
  void update_obstacles(const std::vector<Obstacle<float>>& obstacles, const std::vector<float>& confidence) {
    boxes(obstacles, confidence, 0.0f);
  }
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
  void update_obstacles() { hastar_dropin::check(hastar_decay(_h)); }
  void clear_obstacles() { hastar_dropin::check(hastar_grid2d_clear(_h)); }
  float get_node_total_cost(const int i, const int j) const {
    float f = 0.0f;
    hastar_dropin::check(hastar_grid2d_node_cost(_h, i, j, &f));
    return f;
  }
  float get_grid_heading() const { return _heading; }
  float get_grid_resolution() const { return _res; }
  int get_grid_size() const { return _n; }
  const std::vector<std::vector<float>>& get_obstacle_map() const {
    std::vector<float> flat((size_t)_n * _n);
    hastar_dropin::check(hastar_get_obstacles(_h, flat.data()));
    _map.assign(_n, std::vector<float>(_n));
    for (int i = 0; i < _n; ++i)
      for (int j = 0; j < _n; ++j) _map[i][j] = flat[(size_t)i * _n + j];
    return _map;
  }
  // Grid2D.cpp:260-266 (no relocation; Grid3D's version relocates)
  Node2D<float> update_goal_heading(const Vector2D<float>& goal, const Vector2D<float>& start) {
    const float g[2] = {goal._x, goal._y}, s[2] = {start._x, start._y};
    hastar_dropin::check(hastar_grid2d_update_goal_heading(_h, g, s));
    _heading = std::atan2(goal._y - start._y, goal._x - start._x);
    return *node(goal_i(), goal_j());
  }
  Node2D<float> set_start_node(const Vector2D<float>& start) {  // Grid2D.cpp:270-290
    const float s[2] = {start._x, start._y};
    int cell[2];
    hastar_dropin::check(hastar_grid2d_set_start_node(_h, s, cell));
    return *node(cell[0], cell[1]);
  }
  Node2D<float> set_start_node_grid(const int i, const int j) {  // Grid2D.cpp:294-299
    hastar_dropin::check(hastar_grid2d_set_start_node_grid(_h, i, j));
    return *node(i, j);
  }

 protected:
  struct Raw {};
  Grid2D(Raw, float resolution, float obstacle_threshold, int grid_size, bool allow_diag_moves, hastar_handle h)
      : _h(h), _res(resolution), _n(grid_size), _diag(allow_diag_moves), _thr(logodds(obstacle_threshold)) {}
  static float logodds(float p) { return std::log(p / (1.0 - p)); }  // Grid2D.cpp:10
  static hastar_params base_params(float res, float thr, float pmin, float pmax, float pfree, int n, bool diag) {
    hastar_params p{};
    p.dubins_shot_interval = 300;
    p.dubins_shot_interval_decay = 10;
    p.grid_resolution = res;
    p.obstacle_threshold = thr;
    p.obstacle_prob_min = pmin;
    p.obstacle_prob_max = pmax;
    p.obstacle_prob_free = pfree;
    p.grid_size = n;
    p.grid_2d_allow_diag_moves = diag ? 1 : 0;
    p.step_size = 1.0f;
    p.max_lat_acc = 1.0f;
    p.max_long_dec = 1.0f;
    p.wheelbase = 1.0f;
    p.rear_to_cg = 0.5f;
    p.apf_rep_constant = 0.0f;
    p.apf_active_angle = 1.0f;
    p.num_angle_bins = 1;
    p.num_actions = 0;
    p.max_pops = 64;
    return p;
  }
  void boxes(const std::vector<Obstacle<float>>& obstacles, const std::vector<float>& confidence, float apf_r) {
    std::vector<float> b(obstacles.size() * 4);
    for (size_t k = 0; k < obstacles.size(); ++k) {
      b[4 * k] = obstacles[k]._pose2D._x;
      b[4 * k + 1] = obstacles[k]._pose2D._y;
      b[4 * k + 2] = obstacles[k]._dimensions._x;
      b[4 * k + 3] = obstacles[k]._dimensions._y;
    }
    hastar_dropin::check(hastar_update_boxes(_h, b.data(), confidence.data(), (int)obstacles.size(), apf_r));
  }
  int goal_i() const { return (int)std::round(_n * 0.8); }
  int goal_j() const { return (int)std::round(_n * 0.5); }
  // the node object of cell (i, j): f from the device node map, h = Euclidean (Grid2D.cpp:303-316)
  Node2D<float>* node(int i, int j) const {
    auto& p = _nodes[i * _n + j];
    if (!p) p.reset(new Node2D<float>(i, j));
    const float dx = (float)(goal_i() - i) * _res, dy = (float)(goal_j() - j) * _res;
    const float h = std::sqrt(dx * dx + dy * dy);
    float f = 0.0f;
    hastar_dropin::check(hastar_grid2d_node_cost(_h, i, j, &f));
    p->_cost_g = 0.0f;
    p->_cost_h = h;
    p->_cost_f = f;
    p->_prev = nullptr;
    return p.get();
  }
  hastar_handle _h = nullptr;
  float _res;
  int _n;
  bool _diag;
  float _thr = 0.0f;
  float _heading = 0.0f;
  mutable std::vector<std::vector<float>> _map;
  mutable std::unordered_map<int, std::unique_ptr<Node2D<float>>> _nodes;
};

}  // namespace planning

#endif  // GRID2D
