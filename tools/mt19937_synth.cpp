// mt19937_synth.cpp — SURVEY.md §8d's synthetic box generator with std::mt19937(seed), in the
// draw-order / distribution variants the survey's one-line description admits, so that the
// pop counts the survey measured on the reference binary (§8d: cfg3 seed 1 = 3,297 pops, seed 3 =
// 7,107 pops / 21,170 successors / 20,234 inner A* pops) can be compared with the oracle's.
//   g++ -O2 -std=c++17 tools/mt19937_synth.cpp -o /tmp/mt19937_synth
//   /tmp/mt19937_synth <N> <K> <seed> <variant>   -> one JSON list of [cx, cy, sx, sy] boxes
// variant bits: 0 = float distributions (else double), 1 = centres drawn before sizes,
//               2-3 = clearance rule: 0 centre within 8 m, 1 within 8 m + hypot(sx, sy) / 2,
//                                     2 within 8 m + max(sx, sy) / 2
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

template <class T>
static std::vector<T> gen(int N, int K, unsigned seed, int variant) {
  const T res = 0.5, W = N * res, clear = 8;
  std::mt19937 rng(seed);
  std::uniform_real_distribution<T> size(1, 6), ux(-0.8 * W, 0.2 * W), uy(-0.5 * W, 0.5 * W);
  const T stx = -0.6 * W, sty = 0, gx = 0, gy = 0;
  std::vector<T> out;
  while ((int)out.size() < 4 * K) {
    T sx, sy, cx, cy;
    if (variant & 2) {
      cx = ux(rng);
      cy = uy(rng);
      sx = size(rng);
      sy = size(rng);
    } else {
      sx = size(rng);
      sy = size(rng);
      cx = ux(rng);
      cy = uy(rng);
    }
    const int rule = (variant >> 2) & 3;
    const T r = rule == 0 ? T(0) : rule == 1 ? std::hypot(sx, sy) / 2 : std::max(sx, sy) / 2;
    if (std::hypot(cx - stx, cy - sty) < clear + r || std::hypot(cx - gx, cy - gy) < clear + r) continue;
    out.insert(out.end(), {cx, cy, sx, sy});
  }
  return out;
}

int main(int argc, char** argv) {
  if (argc < 5) return 2;
  const int N = std::atoi(argv[1]), K = std::atoi(argv[2]), variant = std::atoi(argv[4]);
  const unsigned seed = (unsigned)std::strtoul(argv[3], nullptr, 10);
  std::printf("[");
  if (variant & 1) {
    const auto v = gen<float>(N, K, seed, variant);
    for (size_t i = 0; i < v.size(); ++i) std::printf("%s%.9g", i ? "," : "", (double)v[i]);
  } else {
    const auto v = gen<double>(N, K, seed, variant);
    for (size_t i = 0; i < v.size(); ++i) std::printf("%s%.17g", i ? "," : "", v[i]);
  }
  std::printf("]\n");
  return 0;
}
