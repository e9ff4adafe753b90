// tf::Quaternion / tf::Matrix3x3 stand-ins (TEST HARNESS ONLY): getRPY of a unit quaternion
#pragma once
#include <cmath>
namespace tf {
struct Quaternion {
  double x, y, z, w;
  Quaternion(double x_, double y_, double z_, double w_) : x(x_), y(y_), z(z_), w(w_) {}
};
struct Matrix3x3 {
  double m[3][3];
  explicit Matrix3x3(const Quaternion& q) {
    const double xx = q.x * q.x, yy = q.y * q.y, zz = q.z * q.z;
    const double xy = q.x * q.y, xz = q.x * q.z, yz = q.y * q.z, wx = q.w * q.x, wy = q.w * q.y, wz = q.w * q.z;
    m[0][0] = 1 - 2 * (yy + zz); m[0][1] = 2 * (xy - wz);     m[0][2] = 2 * (xz + wy);
    m[1][0] = 2 * (xy + wz);     m[1][1] = 1 - 2 * (xx + zz); m[1][2] = 2 * (yz - wx);
    m[2][0] = 2 * (xz - wy);     m[2][1] = 2 * (yz + wx);     m[2][2] = 1 - 2 * (xx + yy);
  }
  void getRPY(double& roll, double& pitch, double& yaw) const {
    yaw = std::atan2(m[1][0], m[0][0]);
    pitch = std::asin(-m[2][0]);
    roll = std::atan2(m[2][1], m[2][2]);
  }
};
}  // namespace tf
