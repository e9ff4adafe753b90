// std_msgs/Float32MultiArray stand-in (TEST HARNESS ONLY, see ros/ros.h)
#pragma once
#include <memory>
#include <vector>
#include "std_msgs/MultiArrayDimension.h"
namespace std_msgs {
struct Float32MultiArray {
  MultiArrayLayout layout;
  std::vector<float> data;
  typedef std::shared_ptr<const Float32MultiArray> ConstPtr;
};
}  // namespace std_msgs
