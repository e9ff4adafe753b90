// hastar_dubins_f64.h — Dubins<double> on the device (Dubins.cpp:19-153, 180-563 with
// T = double): the shortest CSC word of one start pose and its sampled path, one thread.
// Used by the unit kernels (hastar_units.hip: Dubins<double> of include/hastar_units.h) and by
// the double planner's search (hastar_f64.hip: HybridAStar<double>'s heuristic and shots).
// Its sin/cos/atan2/acos are ports of glibc 2.35's (hastar_libm64.h), bit for bit the host's.
#pragma once
#include <hip/hip_runtime.h>
#include "hastar_device.h"
#include "hastar_libm64.h"

namespace hastar {

// The CSC words of Dubins.cpp:180-323 for T = double (the float path is hastar_device.h's).
struct DubD {
  double r, step, ang_step;
  double prm[4];
  int word;
  double cx[4], cy[4];  // centres: start right, start left, goal right, goal left (Dubins.cpp:76-87)
};
__device__ inline double dub_word_d(const DubD& D, int w, double csx, double csy, double cgx, double cgy, double sh, double gh,
                             double q[4]) {
  const double dx = cgx - csx, dy = cgy - csy;
  const double r = D.r;
  if (w == 0 || w == 3) {  // RSR / LSL
    const double th = gm64::atan2(dy, dx);
    const double sgn = (w == 0) ? 1.0 : -1.0;
    q[0] = sgn * M_PI_2 + sh;
    const double t1 = sgn * M_PI_2 + th;
    q[2] = t1;
    const double tg = sgn * M_PI_2 + gh;
    q[1] = t1 - q[0];
    q[3] = tg - q[2];
    if (w == 0) {
      if (q[1] > 0) q[1] -= 2 * M_PI;
      if (q[3] > 0) q[3] -= 2 * M_PI;
    } else {
      if (q[1] < 0) q[1] += 2 * M_PI;
      if (q[3] < 0) q[3] += 2 * M_PI;
    }
    const double dst = ::sqrt(dx * dx + dy * dy);
    return (w == 0) ? dst + r * -(q[1] + q[3]) : dst + r * (q[1] + q[3]);
  }
  const double dist = ::sqrt(dx * dx + dy * dy);
  const double th = gm64::atan2(dy, dx);
  double t1;
  if (w == 1) {  // RSL
    q[0] = M_PI_2 + sh;
    t1 = gm64::acos(2 * r / dist) + th;
    q[2] = t1 - M_PI;
    const double tg = -M_PI_2 + gh;
    q[1] = t1 - q[0];
    if (q[1] > 0) q[1] -= 2 * M_PI;
    q[3] = tg - q[2];
    if (q[3] < 0) q[3] += 2 * M_PI;
  } else {  // LSR
    q[0] = -M_PI_2 + sh;
    t1 = -gm64::acos(2 * r / dist) + th;
    q[2] = t1 + M_PI;
    const double tg = M_PI_2 + gh;
    q[1] = t1 - q[0];
    if (q[1] < 0) q[1] += 2 * M_PI;
    q[3] = tg - q[2];
    if (q[3] > 0) q[3] -= 2 * M_PI;
  }
  const double ax = csx + r * gm64::cos(t1), ay = csy + r * gm64::sin(t1);
  const double bx = cgx + r * gm64::cos(q[2]), by = cgy + r * gm64::sin(q[2]);
  const double ex = bx - ax, ey = by - ay;
  const double dst = ::sqrt(ex * ex + ey * ey);
  return (w == 1) ? dst + r * (-q[1] + q[3]) : dst + r * (q[1] - q[3]);
}
// Dubins.cpp:19-69: the four words in order, first strictly shorter one kept (a NaN
// length, acos of a ratio > 1, never compares shorter)
__device__ inline double dub_shortest_d(DubD& D, double sx, double sy, double sh, double gx, double gy, double gh) {
  const double r = D.r;
  D.cx[0] = sx + r * gm64::sin(sh);
  D.cy[0] = sy - r * gm64::cos(sh);
  D.cx[1] = sx - r * gm64::sin(sh);
  D.cy[1] = sy + r * gm64::cos(sh);
  D.cx[2] = gx + r * gm64::sin(gh);
  D.cy[2] = gy - r * gm64::cos(gh);
  D.cx[3] = gx - r * gm64::sin(gh);
  D.cy[3] = gy + r * gm64::cos(gh);
  const int si[4] = {0, 0, 1, 1}, gi[4] = {2, 3, 2, 3};
  double best = 0;
  D.word = 0;
  for (int w = 0; w < 4; ++w) {
    double q[4];
    const double len = dub_word_d(D, w, D.cx[si[w]], D.cy[si[w]], D.cx[gi[w]], D.cy[gi[w]], sh, gh, q);
    if (w == 0 || len < best) {
      best = len;
      D.word = w;
      for (int k = 0; k < 4; ++k) D.prm[k] = q[k];
    }
  }
  return best;
}
// Dubins.cpp:326-563 for T = double, one thread (the loops accumulate angle and distance)
__device__ inline int dub_sample_d(const DubD& D, double* xyh, double* curv, int cap) {
  const int w = D.word;
  const bool s_right = (w == 0 || w == 1), g_right = (w == 0 || w == 2);
  const int si[4] = {0, 0, 1, 1}, gi[4] = {2, 3, 2, 3};
  const double csx = D.cx[si[w]], csy = D.cy[si[w]], cgx = D.cx[gi[w]], cgy = D.cy[gi[w]];
  const double r = D.r;
  const double ax = csx + r * gm64::cos(D.prm[0] + D.prm[1]), ay = csy + r * gm64::sin(D.prm[0] + D.prm[1]);
  const double bx = cgx + r * gm64::cos(D.prm[2]), by = cgy + r * gm64::sin(D.prm[2]);
  const double ex = bx - ax, ey = by - ay;
  const double lst = ::sqrt(ex * ex + ey * ey);
  const int n1 = (int)::floor((s_right ? -D.prm[1] : D.prm[1]) / D.ang_step);
  const int n2 = n1 + (int)::floor(lst / D.step);
  const int n3 = n2 + (int)::floor((g_right ? -D.prm[3] : D.prm[3]) / D.ang_step);
  if (n1 < 0 || n2 < n1 || n3 < n2 || n3 + 1 > cap) return -(n3 + 1);
  const double k = 1 / r;
  double th = D.prm[0];
  for (int i = 0; i < n1; ++i) {
    xyh[3 * i] = csx + r * gm64::cos(th);
    xyh[3 * i + 1] = csy + r * gm64::sin(th);
    xyh[3 * i + 2] = s_right ? wrap_pi_d(th - M_PI_2) : wrap_pi_d(th + M_PI_2);
    curv[i] = k;
    th = s_right ? th - D.ang_step : th + D.ang_step;
  }
  const double ts = gm64::atan2(ey, ex), ct = gm64::cos(ts), st = gm64::sin(ts);
  double dd = 0;
  for (int i = n1; i < n2; ++i) {
    xyh[3 * i] = ax + dd * ct;
    xyh[3 * i + 1] = ay + dd * st;
    xyh[3 * i + 2] = ts;
    curv[i] = 0;
    dd += D.step;
  }
  th = D.prm[2];
  for (int i = n2; i < n3; ++i) {
    xyh[3 * i] = cgx + r * gm64::cos(th);
    xyh[3 * i + 1] = cgy + r * gm64::sin(th);
    xyh[3 * i + 2] = g_right ? wrap_pi_d(th - M_PI_2) : wrap_pi_d(th + M_PI_2);
    curv[i] = k;
    th = g_right ? th - D.ang_step : th + D.ang_step;
  }
  const double e = D.prm[2] + D.prm[3];
  xyh[3 * n3] = cgx + r * gm64::cos(e);
  xyh[3 * n3 + 1] = cgy + r * gm64::sin(e);
  xyh[3 * n3 + 2] = g_right ? wrap_pi_d(e - M_PI_2) : wrap_pi_d(e + M_PI_2);
  curv[n3] = 0;
  return n3 + 1;
}

}  // namespace hastar
