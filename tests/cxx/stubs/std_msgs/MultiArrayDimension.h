// std_msgs/MultiArrayDimension + MultiArrayLayout stand-ins (TEST HARNESS ONLY, see ros/ros.h)
#pragma once
#include <cstdint>
#include <string>
#include <vector>
namespace std_msgs {
struct MultiArrayDimension {
  std::string label;
  uint32_t size = 0, stride = 0;
};
struct MultiArrayLayout {
  std::vector<MultiArrayDimension> dim;
  uint32_t data_offset = 0;
};
}  // namespace std_msgs
