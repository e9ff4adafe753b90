// Exercises the unit-level drop-in classes (include/path_planning_pkg/{AStar,Dubins,
// VehicleModel}.h) with the scenarios of the reference's manual harnesses
// (utils/astar/test_astar.cpp:14-110, utils/vehicle_dubins/test_vehicle_dubins.cpp:17-67;
// inputs restated as data), printing every result for tests/test_cxx_units.py:
//   D <type> <len %.17g> <n>          then n lines "x y h" (%.17g)   Dubins<double>
//   F <type> <len bits> <n> <flag>    then n lines of float bits      Dubins<float>
//   VD <n> / VF <n>                    simulate_action chain positions (double %.17g / float bits)
//   NB <count> <neglect> then lines    get_neighbors of the chain's start node (float bits)
//   A <cost bits> x4, AP <n> + points, AM <N> + map rows as bits     AStar<float>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <utility>
#include <vector>

#include "AStar.h"
#include "Dubins.h"
#include "VehicleModel.h"

using namespace planning;

static uint32_t fb(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}

template <class T>
static T rmin_of() {  // test_vehicle_dubins.cpp:19-24
  const T wb = T(2.269), lr = T(1.1);
  const T ms = T(30.0 * M_PI / 180.0);
  const T beta = std::atan2(lr * std::tan(ms), wb);
  return wb / (std::tan(ms) * std::cos(beta));
}

static const int kActions[] = {6, 6, 6, 6, 6, 6, 5, 5, 5, 5, 4, 4, 4, 4, 4, 3,
                               3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 4, 4, 4, 4};

template <class T>
static std::vector<Node3D<T>> chain(VehicleModel<T>& model) {
  Vector3D<T> start(T(0), T(0), T(0));
  std::vector<Node3D<T>> out;
  out.reserve(64);
  out.emplace_back(start, T(0), T(16), 3, get_heading_index(T(0), T(5.0 * M_PI / 180.0)), nullptr);
  for (int a : kActions) {
    auto r = model.simulate_action(out.back(), a);
    if (!r.first) break;
    out.push_back(r.second);
  }
  return out;
}

int main() {
  // ---- Dubins<double> / <float>: start (0, 0, 0), goal (20, -20, pi/2), step 0.5
  {
    Dubins<double> d(rmin_of<double>(), 0.5);
    std::vector<Vector3D<double>> path;
    std::vector<double> curv;
    const double L0 = d.get_shortest_path_length(Vector3D<double>(0, 0, 0), Vector3D<double>(20, -20, M_PI_2));
    auto r = d.get_shortest_path(Vector3D<double>(0, 0, 0), Vector3D<double>(20, -20, M_PI_2), path, curv);
    std::printf("D %s %.17g %zu %.17g %d %.17g\n", d.get_path_type().c_str(), r.first, path.size(), L0, r.second ? 1 : 0,
                rmin_of<double>());
    for (const auto& p : path) std::printf("%.17g %.17g %.17g\n", p._x, p._y, p._heading);
  }
  {
    Dubins<float> d(rmin_of<float>(), 0.5f);
    std::vector<Vector3D<float>> path;
    std::vector<float> curv;
    auto r = d.get_shortest_path(Vector3D<float>(0, 0, 0), Vector3D<float>(20, -20, (float)M_PI_2), path, curv);
    std::printf("F %s %08x %zu %d %08x\n", d.get_path_type().c_str(), fb(r.first), path.size(), r.second ? 1 : 0,
                fb(rmin_of<float>()));
    for (size_t i = 0; i < path.size(); ++i)
      std::printf("%08x %08x %08x %08x\n", fb(path[i]._x), fb(path[i]._y), fb(path[i]._heading), fb(curv[i]));
  }
  // ---- VehicleModel: step 0.5, a_lat 4, a_dec 2, wheelbase 2.269, l_r 1.1, 72 bins, 1 action
  {
    std::vector<double> st{-30.0 * M_PI / 180.0, -20.0 * M_PI / 180.0, -10.0 * M_PI / 180.0, 0.0,
                           10.0 * M_PI / 180.0,  20.0 * M_PI / 180.0,  30.0 * M_PI / 180.0};
    VehicleModel<double> m(0.5, 4.0, 2.0, 2.269, 1.1, 72, 1, st);  // the harness's 8-argument form
    auto c = chain(m);
    std::printf("VD %zu\n", c.size());
    for (const auto& n : c) std::printf("%.17g %.17g\n", n._pose2D._x, n._pose2D._y);
  }
  {
    std::vector<float> st;
    for (double d : {-30.0, -20.0, -10.0, 0.0, 10.0, 20.0, 30.0}) st.push_back((float)(d * M_PI / 180.0));
    VehicleModel<float> m(0.5f, 4.0f, 2.0f, 2.269f, 1.1f, 72, 1, st, std::vector<float>(st.size(), 0.0f));
    auto c = chain(m);
    std::printf("VF %zu\n", c.size());
    for (const auto& n : c) std::printf("%08x %08x\n", fb(n._pose2D._x), fb(n._pose2D._y));
    std::vector<Node3D<float>> nb;
    const bool neglect = m.get_neighbors(c[5], nb);
    std::printf("NB %zu %d\n", nb.size(), neglect ? 1 : 0);
    for (const auto& n : nb)
      std::printf("%08x %08x %08x %08x %08x %d %d\n", fb(n._pose2D._x), fb(n._pose2D._y), fb(n._pose2D._heading),
                  fb(n._cost_g), fb(n._vmin_sqr), n._curvature_index, n._angle_bin);
    // the same window through simulate_action (VehicleModel.cpp:108-136), feasible ones only
    std::vector<Node3D<float>> sim;
    for (int a = c[5]._curvature_index - 1; a <= c[5]._curvature_index + 1; ++a) {
      if (a < 0 || a >= 7) continue;
      auto r = m.simulate_action(c[5], a);
      if (r.first) sim.push_back(r.second);
    }
    std::printf("SIM %zu\n", sim.size());
    for (const auto& n : sim)
      std::printf("%08x %08x %08x %08x %08x %d %d\n", fb(n._pose2D._x), fb(n._pose2D._y), fb(n._pose2D._heading),
                  fb(n._cost_g), fb(n._vmin_sqr), n._curvature_index, n._angle_bin);
  }
  // ---- AStar<float>: test_astar.cpp:14-110 (60 x 60 at 0.5 m, 4 lines, 3 boxes, 5 cycles)
  {
    AStar<float> astar(0.5f, 0.75f, 0.1f, 0.95f, 0.4f, 60);
    Vector2D<float> goal(25.5f, 36.0f), start(18.0f, 18.0f);
    std::vector<std::pair<Vector2D<float>, Vector2D<float>>> lines{{{21.9f, 4.5f}, {21.9f, 31.5f}},
                                                                   {{20.4f, 33.0f}, {38.4f, 33.0f}},
                                                                   {{10.5f, 4.5f}, {10.5f, 40.5f}},
                                                                   {{9.0f, 42.0f}, {39.0f, 42.0f}}};
    std::vector<Obstacle<float>> obs{Obstacle<float>(18.0f, 22.8f, 4.0f, 3.4f), Obstacle<float>(14.25f, 28.5f, 3.0f, 5.8f),
                                     Obstacle<float>(18.0f, 34.8f, 4.0f, 3.4f)};
    Node2D<float> s(0, 0);
    astar.update_goal_start(goal, start, s);
    for (int i = 0; i < 5; ++i) {
      astar.update_obstacles();
      astar.update_obstacles(lines, std::vector<float>(lines.size(), 0.6f), 1.0f);
      astar.update_obstacles(obs, std::vector<float>(obs.size(), 0.75f));
    }
    const float c1 = astar.find_path(s._posd._x, s._posd._y);
    const float c2 = astar.find_path(33, 36);
    const float c3 = astar.find_path(s._posd._x + 6, s._posd._y + 10);
    std::vector<Vector2D<float>> path;
    const float c4 = astar.find_path(goal, start, path);
    std::printf("A %08x %08x %08x %08x %d %d\n", fb(c1), fb(c2), fb(c3), fb(c4), s._posd._x, s._posd._y);
    std::printf("AP %zu\n", path.size());
    for (const auto& p : path) std::printf("%08x %08x\n", fb(p._x), fb(p._y));
    const auto& m = astar.get_obstacles();
    std::printf("AM %zu\n", m.size());
    for (const auto& row : m) {
      for (float v : row) std::printf("%08x ", fb(v));
      std::printf("\n");
    }
  }
  return 0;
}
