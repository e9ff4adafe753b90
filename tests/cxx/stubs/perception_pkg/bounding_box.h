// perception_pkg/bounding_box stand-in (TEST HARNESS ONLY): the fields local_planner.cpp:224-237 reads
#pragma once
#include <string>
#include "geometry_msgs/Pose.h"
namespace perception_pkg {
struct bounding_box {
  std::string class_name;
  float confidence = 0, length = 0, width = 0;
  geometry_msgs::Point centroid;
};
}  // namespace perception_pkg
