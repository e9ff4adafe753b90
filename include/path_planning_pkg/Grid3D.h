// Grid3D.h — drop-in planning::Grid3D<float> (reference include/path_planning_pkg/Grid3D.h:
// 14-46, lib/Grid3D.cpp): the goal-centred 2-D grid with the vehicle model and the APF
// obstacle list, on a planner handle (the same state the search kernel reads).
// update_goal_heading relocates the map on the device; get_neighbors and check_path run on
// the device.  Successors' base nodes are this object's Node2D objects (see Grid2D.h).
#ifndef GRID3D
#define GRID3D

#include <utility>
#include <vector>

#include "Grid2D.h"
#include "Node3D.h"
#include "VehicleModel.h"
#include "common.h"

namespace planning {

template <typename T>
class Grid3D;  // only the float specialisation is provided

template <>
class Grid3D<float> : public Grid2D<float> {
 public:
  Grid3D(float resolution, float obstacle_threshold, float obstacle_prob_min, float obstacle_prob_max,
         float obstacle_prob_free, int grid_size, bool allow_diag_moves, float step_size, float max_lat_acc,
         float max_long_dec, float wheelbase, float rear_to_cg, float apf_rep_constant, float apf_active_angle,
         int num_angle_bins, int num_actions, const std::vector<float>& steering,
         const std::vector<float>& curvature_weights)
      : Grid2D<float>(Raw{}, resolution, obstacle_threshold, grid_size, allow_diag_moves,
                      create(resolution, obstacle_threshold, obstacle_prob_min, obstacle_prob_max, obstacle_prob_free,
                             grid_size, allow_diag_moves, step_size, max_lat_acc, max_long_dec, wheelbase, rear_to_cg,
                             apf_rep_constant, apf_active_angle, num_angle_bins, num_actions, steering,
                             curvature_weights)),
        _model(step_size, max_lat_acc, max_long_dec, wheelbase, rear_to_cg, num_angle_bins, num_actions, steering,
               curvature_weights) {}

  using Grid2D<float>::update_obstacles;
  // Grid3D.cpp:22-44: APF list in the grid frame + the box raster
  void update_obstacles(const std::vector<Obstacle<float>>& obstacles, const std::vector<float>& confidence,
                        const float apf_added_radius) {
    boxes(obstacles, confidence, apf_added_radius);
  }
  // Grid3D.cpp:47-74
  bool get_neighbors(const Node3D<float>& node, std::vector<Node3D<float>>& neighbors) const {
    hastar_node3_f32 in{node._pose2D._x, node._pose2D._y, node._pose2D._heading, node._cost_g, node._vmin_sqr,
                        node._curvature_index, node._angle_bin};
    const int cap = 64;
    hastar_node3_f32 out[cap];
    int cells[2 * cap], count = 0, neglect = 0;
    hastar_dropin::check(hastar_grid3d_neighbors(_h, &in, cap, out, cells, &count, &neglect));
    neighbors.clear();
    for (int k = 0; k < count && k < cap; ++k) {
      Vector3D<float> pose(out[k].x, out[k].y, out[k].heading);
      Node3D<float> n(pose, out[k].g, out[k].vmin_sqr, out[k].curvature_index, out[k].angle_bin,
                      node_ptr(cells[2 * k], cells[2 * k + 1]), &node);
      neighbors.push_back(n);  // _cost_f == _cost_g (field included), as the reference leaves it
    }
    return neglect != 0;
  }
  // Grid3D.cpp:78-93
  bool check_path(const std::vector<Vector3D<float>>& path) const {
    std::vector<float> xyh(path.size() * 3);
    for (size_t k = 0; k < path.size(); ++k) {
      xyh[3 * k] = path[k]._x;
      xyh[3 * k + 1] = path[k]._y;
      xyh[3 * k + 2] = path[k]._heading;
    }
    int is_free = 0;
    hastar_dropin::check(hastar_grid3d_check_path(_h, xyh.data(), (int)path.size(), &is_free));
    return is_free != 0;
  }
  Vector3D<float> get_goal_location() const { return _goal3; }
  // Grid3D.cpp:102-124: re-orient, relocate the map (device), return the goal node
  Node3D<float> update_goal_heading(const Vector3D<float>& goal, const Vector3D<float>& start) {
    const float g[3] = {goal._x, goal._y, goal._heading}, s[3] = {start._x, start._y, start._heading};
    hastar_dropin::check(hastar_update_goal(_h, g, s));
    _goal3 = goal;
    _heading = std::atan2(goal._y - start._y, goal._x - start._x);
    hastar_node3_f32 gn{};
    hastar_dropin::check(hastar_grid3d_goal_node(_h, &gn));
    Vector3D<float> pose(gn.x, gn.y, gn.heading);
    return Node3D<float>(pose, 0.0f, 0.0f, 0, gn.angle_bin, node_ptr(goal_i(), goal_j()), nullptr);
  }
  // Grid3D.cpp:127-160
  Node3D<float> set_start_node(const Vector3D<float>& start) {
    const float s[3] = {start._x, start._y, start._heading};
    hastar_node3_f32 sn{};
    int cell[2];
    hastar_dropin::check(hastar_grid3d_set_start_node(_h, s, &sn, cell));
    Vector3D<float> pose(sn.x, sn.y, sn.heading);
    return Node3D<float>(pose, 0.0f, 0.0f, sn.curvature_index, sn.angle_bin, node_ptr(cell[0], cell[1]), nullptr);
  }
  const std::vector<float>& get_abs_curvatures() const { return _model.get_abs_curvatures(); }

 private:
  static hastar_handle create(float res, float thr, float pmin, float pmax, float pfree, int n, bool diag, float step,
                              float a_lat, float a_dec, float wb, float lr, float rep, float ang, int bins, int na,
                              const std::vector<float>& steering, const std::vector<float>& weights) {
    if (steering.size() != weights.size())
      throw std::invalid_argument("Grid3D: steering and curvature_weights differ in length");
    hastar_params p = base_params(res, thr, pmin, pmax, pfree, n, diag);
    p.step_size = step;
    p.max_lat_acc = a_lat;
    p.max_long_dec = a_dec;
    p.wheelbase = wb;
    p.rear_to_cg = lr;
    p.apf_rep_constant = rep;
    p.apf_active_angle = ang;
    p.num_angle_bins = bins;
    p.num_actions = na;
    p.num_steering = (int)steering.size();
    p.steering = steering.data();
    p.curvature_weights = weights.data();
    hastar_handle h = nullptr;
    hastar_dropin::check(hastar_create_f32(&p, hastar_dropin::device(), &h));
    return h;
  }
  const Node2D<float>* node_ptr(int i, int j) const { return node(i, j); }
  VehicleModel<float> _model;  // the same tables as the handle's (get_abs_curvatures)
  Vector3D<float> _goal3;
};

}  // namespace planning

#endif  // GRID3D
