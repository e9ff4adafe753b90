// The reference's manual harness scenario (utils/hybrid_astar/test_hybrid_astar.cpp:13-129:
// 60x60x72 grid, 4 lines + 3 boxes, 5 decay/update cycles, reset, find_path at 2 m/s),
// written against the drop-in C++ class.  Prints "ok cost_bits len" and one line of
// float bit patterns (x y heading curvature) per pose, for tests/test_cxx_dropin.py.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <utility>
#include <vector>

#include "HybridAStar.h"

using namespace planning;

static uint32_t bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}

int main() {
  std::vector<float> steering = {-30.0f, -15.0f, 0.0f, 15.0f, 30.0f};
  for (float& a : steering) a = a * M_PI / 180.0f;
  std::vector<float> weights(steering.size(), 0.0f);
  HybridAStar<float> planner(300, 10, 0.5f, 0.75f, 0.1f, 0.95f, 0.4f, 60, true, 0.75f, 4.0f, 2.0f, 2.269f, 1.1f,
                             1.0f, static_cast<float>(M_PI / 4), 72, 1, steering, weights);
  std::vector<std::pair<Vector2D<float>, Vector2D<float>>> lines = {
      {Vector2D<float>(21.9f, 4.5f), Vector2D<float>(21.9f, 31.5f)},
      {Vector2D<float>(20.4f, 33.0f), Vector2D<float>(38.4f, 33.0f)},
      {Vector2D<float>(10.5f, 4.5f), Vector2D<float>(10.5f, 40.5f)},
      {Vector2D<float>(9.0f, 42.0f), Vector2D<float>(39.0f, 42.0f)}};
  std::vector<Obstacle<float>> boxes = {Obstacle<float>(18.0f, 22.8f, 3.5f, 2.9f),
                                        Obstacle<float>(14.25f, 28.5f, 2.0f, 5.3f),
                                        Obstacle<float>(18.0f, 34.8f, 3.5f, 2.9f)};
  const Vector3D<float> start(18.0f, 18.0f, M_PI_2), goal(26.0f, 36.0f, 0.0f);
  planner.update_goal(goal, start);
  for (int c = 0; c < 5; ++c) {
    planner.update_obstacles();
    planner.update_obstacles(lines, std::vector<float>(lines.size(), 0.6f), 1.25f);
    planner.update_obstacles(boxes, std::vector<float>(boxes.size(), 0.75f), 2.5f);
  }
  planner.reset();
  std::vector<Vector3D<float>> path;
  std::vector<float> curvature;
  const std::pair<float, bool> r = planner.find_path(2.0f, start, path, curvature);
  const auto& grid = planner.get_obstacles();
  std::printf("%d %08x %zu %zu\n", r.second ? 1 : 0, bits(r.first), path.size(), grid.size());
  for (size_t i = 0; i < path.size(); ++i)
    std::printf("%08x %08x %08x %08x\n", bits(path[i]._x), bits(path[i]._y), bits(path[i]._heading),
                bits(curvature[i]));
  return 0;
}
