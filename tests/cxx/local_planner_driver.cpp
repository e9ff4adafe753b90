// Test driver of the reference's ROS node, src/local_planner.cpp, compiled UNCHANGED against the
// drop-in planner headers (include/path_planning_pkg/) and the ROS stand-ins of tests/cxx/stubs/
// (tests/test_local_planner.py).  local_planner.cpp is built with -Dmain=reference_local_planner_main
// so that this file can construct LocalPlanner<float> or LocalPlanner<double> (local_planner.h:98-135)
// and run the node's own run() loop for a scripted scenario:
//
//   turn 1: odometry, a waypoint, objects (cars), lanes  -> callbacks, then update_trajectory()
//   turn 2: moved objects, lanes                          -> callbacks, then update_trajectory()
//
// After each turn it prints the published trajectory message (local_planner.cpp:346-372 /
// 474-500) as hex bit patterns: "T <turn> <n>" then n values.
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>

#include "local_planner.h"

template <class M>
static void print_traj(int turn, const char* topic) {
  const M* m = ros::stub::last<M>(topic);
  if (!m) {
    std::printf("T %d 0\n", turn);
    return;
  }
  std::printf("T %d %zu\n", turn, m->data.size());
  for (auto v : m->data) {
    if constexpr (sizeof(v) == 4) {
      uint32_t u;
      std::memcpy(&u, &v, 4);
      std::printf("%08x\n", u);
    } else {
      uint64_t u;
      std::memcpy(&u, &v, 8);
      std::printf("%016" PRIx64 "\n", u);
    }
  }
}

static void set_params() {
  auto& P = ros::stub::params();
  P.num = {{"/local_planner/grid_size", 60},
           {"/local_planner/grid_resolution", 0.5},
           {"/local_planner/obstacle_threshold", 0.75},
           {"/local_planner/obstacle_prob_min", 0.1},
           {"/local_planner/obstacle_prob_max", 0.95},
           {"/local_planner/obstacle_prob_free", 0.4},
           {"/local_planner/step_size", 0.75},
           {"/local_planner/max_lat_acc", 4.0},
           {"/local_planner/max_long_dec", 2.0},
           {"/local_planner/wheelbase", 2.269},
           {"/local_planner/rear_to_cg", 1.1},
           {"/local_planner/num_angle_bins", 72},
           {"/local_planner/num_actions", 1},
           {"/local_planner/dubins_shot_interval", 300},
           {"/local_planner/dubins_shot_interval_decay", 10}};
  P.vec = {{"/local_planner/steering", {-30.0, -15.0, 0.0, 15.0, 30.0}},
           {"/local_planner/curvature_weights", {0.0, 0.1, 0.0, 0.1, 0.0}}};
}

template <class T, class LaneMsg>
static void scenario(const char* traj_type) {
  (void)traj_type;
  ros::NodeHandle nh;
  LocalPlanner<T> node(nh);
  // odometry: the node stores {y, -x, yaw} (local_planner.cpp:180-184): the planner pose (18, 18, 0)
  nav_msgs::Odometry od;
  od.pose.pose.position.x = -18.0;
  od.pose.pose.position.y = 18.0;
  od.twist.twist.linear.x = 2.0;
  path_planning_pkg::Waypoint wp;
  wp.pose.position.x = 26.0;
  wp.pose.position.y = 36.0;
  auto objects = [](double dx) {
    perception_pkg::bounding_box_array a;
    const double c[3][3] = {{18.0, 22.8, 3.4}, {14.25, 28.5, 3.0}, {18.0, 34.8, 3.4}};
    for (auto& b : c) {
      perception_pkg::bounding_box bb;
      bb.class_name = "car";
      bb.centroid.x = b[0] + dx;
      bb.centroid.y = b[1];
      bb.length = (float)b[2];
      bb.width = (float)(b[2] - 0.5);
      bb.confidence = 0.8f;
      a.bbs_array.push_back(bb);
    }
    return a;
  };
  LaneMsg lanes;
  lanes.layout.dim.resize(2);
  lanes.layout.dim[0].size = 3;
  lanes.layout.dim[1].size = 4;
  lanes.data = {21.9, 4.5, 21.9, 31.5, 10.5, 4.5, 10.5, 40.5, 9.0, 42.0, 39.0, 42.0};
  ros::stub::deliver("/odometry", od);
  ros::stub::deliver("/waypoints", wp);
  ros::stub::deliver("/objects", objects(0.0));
  ros::stub::deliver("/lanes", lanes);
  ros::stub::ok_turns() = 1;
  node.run();
  print_traj<LaneMsg>(1, "/local_planner/trajectory");
  ros::stub::deliver("/objects", objects(0.5));
  ros::stub::deliver("/lanes", lanes);
  ros::stub::ok_turns() = 1;
  node.run();
  print_traj<LaneMsg>(2, "/local_planner/trajectory");
}

int main(int argc, char** argv) {
  set_params();
  const std::string mode = argc > 1 ? argv[1] : "float";
  if (mode == "double")
    scenario<double, std_msgs::Float64MultiArray>("double");
  else
    scenario<float, std_msgs::Float32MultiArray>("float");
  return 0;
}
