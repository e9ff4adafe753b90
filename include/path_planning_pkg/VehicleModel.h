// VehicleModel.h — drop-in planning::VehicleModel<T> (reference
// include/path_planning_pkg/VehicleModel.h:14-42, lib/VehicleModel.cpp), on the MI355X
// through include/hastar_units.h: the motion-primitive tables are integrated once at
// construction and kept on the device; get_neighbors / simulate_action run there.
// Results equal the reference's bit for bit for float and double (the tables are built
// with the reference's libm calls; the per-node arithmetic needs no transcendentals).
// Successor nodes carry no base node (the reference's VehicleModel sets none either).
#ifndef VEHICLE_MODEL
#define VEHICLE_MODEL

#include <type_traits>
#include <utility>
#include <vector>

#include "Node3D.h"
#include "common.h"
#include "hastar_dropin.h"

namespace planning {

template <typename T>
class VehicleModel {
  static_assert(std::is_same<T, float>::value || std::is_same<T, double>::value,
                "VehicleModel<float> or VehicleModel<double>");
  using NodeC = typename std::conditional<std::is_same<T, float>::value, hastar_node3_f32, hastar_node3_f64>::type;

 public:
  // VehicleModel.cpp:7-47
  VehicleModel(T ts, T max_lat_acc, T max_long_dec, T wheelbase, T rear_to_cg, int num_angle_bins, int num_actions,
               const std::vector<T>& steering, const std::vector<T>& curvature_weights) {
    if (steering.size() != curvature_weights.size())
      throw std::invalid_argument("VehicleModel: steering and curvature_weights differ in length");
    int rc;
    if constexpr (std::is_same<T, float>::value)
      rc = hastar_vehicle_create_f32(hastar_dropin::device(), ts, max_lat_acc, max_long_dec, wheelbase, rear_to_cg,
                                     num_angle_bins, num_actions, (int)steering.size(), steering.data(),
                                     curvature_weights.data(), &_v);
    else
      rc = hastar_vehicle_create_f64(hastar_dropin::device(), ts, max_lat_acc, max_long_dec, wheelbase, rear_to_cg,
                                     num_angle_bins, num_actions, (int)steering.size(), steering.data(),
                                     curvature_weights.data(), &_v);
    hastar_dropin::check(rc, true);
    double prec = 0;
    hastar_dropin::check(hastar_vehicle_info(_v, &prec, &_default_action, &_nsteer), true);
    _precision = static_cast<T>(prec);
    _abs_curvatures.resize(_nsteer);
    hastar_dropin::check(hastar_vehicle_abs_curvatures(_v, _abs_curvatures.data()), true);
    _max_neighbors = 2 * num_actions + 1;
  }
  // the earlier 8-argument form (utils/vehicle_dubins/test_vehicle_dubins.cpp:67): no
  // curvature weights, i.e. all zero
  VehicleModel(T ts, T max_lat_acc, T max_long_dec, T wheelbase, T rear_to_cg, int num_angle_bins, int num_actions,
               const std::vector<T>& steering)
      : VehicleModel(ts, max_lat_acc, max_long_dec, wheelbase, rear_to_cg, num_angle_bins, num_actions, steering,
                     std::vector<T>(steering.size(), T(0))) {}
  ~VehicleModel() {
    if (_v) hastar_vehicle_destroy(_v);
  }
  VehicleModel(const VehicleModel&) = delete;
  VehicleModel& operator=(const VehicleModel&) = delete;

  T get_precision() const { return _precision; }
  int get_default_action_index() const { return _default_action; }
  const std::vector<T>& get_abs_curvatures() const { return _abs_curvatures; }

  // VehicleModel.cpp:63-105: successors of `node` (their _prev is &node); returns whether
  // accelerations were neglected (squared speed below 1)
  bool get_neighbors(const Node3D<T>& node, std::vector<Node3D<T>>& neighbors) const {
    NodeC in = to_c(node);
    std::vector<NodeC> out((size_t)std::max(_max_neighbors, 1));
    int count = 0, neglect = 0;
    int rc;
    if constexpr (std::is_same<T, float>::value)
      rc = hastar_vehicle_neighbors_f32(_v, 1, &in, _max_neighbors, out.data(), &count, &neglect);
    else
      rc = hastar_vehicle_neighbors_f64(_v, 1, &in, _max_neighbors, out.data(), &count, &neglect);
    hastar_dropin::check(rc, true);
    neighbors.clear();
    for (int i = 0; i < count; ++i) neighbors.push_back(from_c(out[i], &node));
    return neglect != 0;
  }
  // VehicleModel.cpp:108-136
  std::pair<bool, Node3D<T>> simulate_action(const Node3D<T>& node, const int action_index) const {
    NodeC in = to_c(node), out{};
    int ok = 0;
    int rc;
    if constexpr (std::is_same<T, float>::value)
      rc = hastar_vehicle_simulate_f32(_v, 1, &in, &action_index, &out, &ok);
    else
      rc = hastar_vehicle_simulate_f64(_v, 1, &in, &action_index, &out, &ok);
    hastar_dropin::check(rc, true);
    if (!ok) return {false, node};
    return {true, from_c(out, &node)};
  }

 private:
  static NodeC to_c(const Node3D<T>& n) {
    NodeC c{};
    c.x = n._pose2D._x;
    c.y = n._pose2D._y;
    c.heading = n._pose2D._heading;
    c.g = n._cost_g;
    c.vmin_sqr = n._vmin_sqr;
    c.curvature_index = n._curvature_index;
    c.angle_bin = n._angle_bin;
    return c;
  }
  static Node3D<T> from_c(const NodeC& c, const Node3D<T>* prev) {
    Vector3D<T> pose(c.x, c.y, c.heading);
    return Node3D<T>(pose, c.g, c.vmin_sqr, c.curvature_index, c.angle_bin, prev);
  }
  hastar_vehicle _v = nullptr;
  T _precision = T(0);
  int _default_action = 0, _nsteer = 0, _max_neighbors = 1;
  std::vector<T> _abs_curvatures;
};

}  // namespace planning

#endif  // VEHICLE_MODEL
