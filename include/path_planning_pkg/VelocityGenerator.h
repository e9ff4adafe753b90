// VelocityGenerator.h — drop-in replacement of the reference's velocity-profile facade
// `planning::VelocityGenerator<T>` (reference include/path_planning_pkg/VelocityGenerator.h:8-28,
// lib/VelocityGenerator.cpp:7-84), implemented on the MI355X C ABI (include/hastar.h,
// hastar_velocity_profile_batch).
//
// Same constructor and generate_velocity_profile signature, so local_planner.cpp:164-165,
// 323, 332, 451, 460 compile unchanged against this header.  Both instantiations of the
// reference exist (VelocityGenerator.cpp:88-89): float and double, both bit-exact (the double
// one on ports of glibc 2.35's hypot/atan2).  Differences a caller can observe:
//   * an empty path (undefined behaviour in the reference) or a device failure throws
//     std::runtime_error;
//   * generate_velocity_profiles (not in the reference) profiles many paths in one launch;
//   * the device is HIP ordinal $HASTAR_DEVICE (default 0).
#ifndef VELOCITY_GENERATOR
#define VELOCITY_GENERATOR

#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "../hastar.h"
#include "../hastar_f64.h"
#include "common.h"

namespace planning {

template <typename T>
class VelocityGenerator;  // float and double specialisations below

template <>
class VelocityGenerator<float> {
 public:
  // VelocityGenerator.h:16 — same arguments, same order and meaning.
  VelocityGenerator(float max_velocity, float coast_velocity, float max_lat_acc, float max_long_acc,
                    float max_long_dec)
      : _p{max_velocity, coast_velocity, max_lat_acc, max_long_acc, max_long_dec} {
    const char* d = std::getenv("HASTAR_DEVICE");
    _device = d ? std::atoi(d) : 0;
  }

  // VelocityGenerator.h:19-21 / VelocityGenerator.cpp:19-84.  `path` and `curvature` are
  // goal -> start, as find_path returns them; `velocity` is resized to the path's length.
  bool generate_velocity_profile(const float vel_init, const float max_velocity_curr,
                                 const std::vector<Vector3D<float>>& path, const std::vector<float>& curvature,
                                 std::vector<float>& velocity, bool coast_to_goal, bool stop_at_goal = false) const {
    if (path.empty() || curvature.size() < path.size())
      throw std::runtime_error("VelocityGenerator: empty path or short curvature vector");
    const long long off[2] = {0, (long long)path.size()};
    std::vector<float> xyh(3 * path.size());
    for (size_t i = 0; i < path.size(); ++i) {
      xyh[3 * i] = path[i]._x;
      xyh[3 * i + 1] = path[i]._y;
      xyh[3 * i + 2] = path[i]._heading;
    }
    velocity.resize(path.size());
    const unsigned char flags = (unsigned char)((coast_to_goal ? 1 : 0) | (stop_at_goal ? 2 : 0));
    unsigned char feasible = 0;
    const int rc = hastar_velocity_profile_batch(_device, &_p, 1, off, xyh.data(), curvature.data(), &vel_init,
                                                 &max_velocity_curr, &flags, velocity.data(), &feasible);
    if (rc != 0) throw std::runtime_error(std::string("hastar_velocity_profile_batch: ") + hastar_last_error());
    return feasible != 0;
  }

 private:
  hastar_velocity_params _p;
  int _device;
};

template <>
class VelocityGenerator<double> {
 public:
  VelocityGenerator(double max_velocity, double coast_velocity, double max_lat_acc, double max_long_acc,
                    double max_long_dec)
      : _p{max_velocity, coast_velocity, max_lat_acc, max_long_acc, max_long_dec} {
    const char* d = std::getenv("HASTAR_DEVICE");
    _device = d ? std::atoi(d) : 0;
  }
  bool generate_velocity_profile(const double vel_init, const double max_velocity_curr,
                                 const std::vector<Vector3D<double>>& path, const std::vector<double>& curvature,
                                 std::vector<double>& velocity, bool coast_to_goal, bool stop_at_goal = false) const {
    if (path.empty() || curvature.size() < path.size())
      throw std::runtime_error("VelocityGenerator: empty path or short curvature vector");
    const long long off[2] = {0, (long long)path.size()};
    std::vector<double> xyh(3 * path.size());
    for (size_t i = 0; i < path.size(); ++i) {
      xyh[3 * i] = path[i]._x;
      xyh[3 * i + 1] = path[i]._y;
      xyh[3 * i + 2] = path[i]._heading;
    }
    velocity.resize(path.size());
    const unsigned char flags = (unsigned char)((coast_to_goal ? 1 : 0) | (stop_at_goal ? 2 : 0));
    unsigned char feasible = 0;
    const int rc = hastar_velocity_profile_batch_f64(_device, &_p, 1, off, xyh.data(), curvature.data(), &vel_init,
                                                     &max_velocity_curr, &flags, velocity.data(), &feasible);
    if (rc != 0) throw std::runtime_error(std::string("hastar_velocity_profile_batch_f64: ") + hastar_last_error());
    return feasible != 0;
  }

 private:
  hastar_velocity_params_f64 _p;
  int _device;
};

}  // namespace planning

#endif
