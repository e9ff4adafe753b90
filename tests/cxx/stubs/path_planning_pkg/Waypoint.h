// path_planning_pkg/Waypoint (msg/Waypoint.msg of the reference) stand-in (TEST HARNESS ONLY)
#pragma once
#include <memory>
#include "geometry_msgs/Pose.h"
namespace path_planning_pkg {
struct Waypoint {
  bool stop_at_waypoint = false;
  geometry_msgs::Pose pose;
  typedef std::shared_ptr<const Waypoint> ConstPtr;
};
}  // namespace path_planning_pkg
