// nav_msgs/Odometry stand-in (TEST HARNESS ONLY, see ros/ros.h)
#pragma once
#include <memory>
#include "geometry_msgs/Pose.h"
namespace nav_msgs {
struct Odometry {
  struct {
    geometry_msgs::Pose pose;
  } pose;
  struct {
    geometry_msgs::Twist twist;
  } twist;
  typedef std::shared_ptr<const Odometry> ConstPtr;
};
}  // namespace nav_msgs
