// std_msgs/Float64MultiArray stand-in (TEST HARNESS ONLY, see ros/ros.h)
#pragma once
#include <memory>
#include <vector>
#include "std_msgs/MultiArrayDimension.h"
namespace std_msgs {
struct Float64MultiArray {
  MultiArrayLayout layout;
  std::vector<double> data;
  typedef std::shared_ptr<const Float64MultiArray> ConstPtr;
};
}  // namespace std_msgs
