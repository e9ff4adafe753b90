// perception_pkg/bounding_box_array stand-in (TEST HARNESS ONLY)
#pragma once
#include <memory>
#include <vector>
#include "perception_pkg/bounding_box.h"
namespace perception_pkg {
struct bounding_box_array {
  std::vector<bounding_box> bbs_array;
  typedef std::shared_ptr<const bounding_box_array> ConstPtr;
};
}  // namespace perception_pkg
