// hastar_oracle.cpp — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's
// Hybrid A* hot path, used as the parity checker and as bench.py's cpu_baseline.
// Nothing in path_planning_pkg_amd/ links, loads or calls this file; only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg do.
//
// The reference (ShehabAshraf101/path_planning_pkg) is UNBUILDABLE in this image: every
// translation unit includes <boost/functional/hash.hpp> (Node2D.h:6, Node3D.h:7) and Boost
// is not installed; making it build would need a stand-in header, which we do not write.
// This restatement is pinned instead by the reference's own golden vectors
// (tests/golden/, see tests/test_oracle_golden.py):
//   * utils/hybrid_astar/plot.py:47-51  — 43-pose path of test_hybrid_astar.cpp (float)
//   * utils/dubins_paths.py:6           — 73-pose RSL Dubins path (double)
//   * utils/vehicle_mode.py:12          — 33 positions of VehicleModel::simulate_action (double)
//
// Semantics that decide the closed set are restated with the SAME library machinery
// the reference uses, so they are faithful by construction:
//   * open sets are std::set with the reference's non-strict-weak comparator
//     (Node3D.h:50-54, Node2D.h:41-45): equal-f inserts are dropped, find() may hit
//     an equal-f node of another cell, outcomes depend on the libstdc++ RB-tree shape;
//   * closed sets are node-based hash sets keyed exactly by (x, y[, bin]) (the
//     reference's hash caches codes, so Node3D::operator== comparing only the cell,
//     Node3D.h:42, still yields (x, y, bin) membership); duplicates return the OLD
//     element (HybridAStar.cpp:110-111);
//   * float/double promotions follow the reference expressions (M_PI literals,
//     std::fmod(float, double), std::pow(double, 2) -> x*x as GCC folds it);
//   * transcendental calls go to the host glibc libm, like the reference.
// Build: oracle/Makefile (g++ -O3 -ffp-contract=off, x86-64 baseline ISA; -O3 as the
// reference's CMakeLists.txt:128 build, so the CPU timing proxy uses the same optimisation).
// -DORC_LEAN (build/libhastar_oracle_lean.so): the TIMING build of bench.py's cpu_baseline — the
// same containers, comparator and arithmetic, with the checker's bookkeeping the reference does
// not do compiled out (pop and closed-set digests, successor / shot / inner-search counters; the
// pop count stays).  Its results (path, cost, success, pops) are the full build's.
#include <atomic>
#include <cmath>
#include <cfloat>
#include <cstdint>
#include <cstring>
#include <limits>
#include <queue>
#include <set>
#include <unordered_set>
#include <vector>
#include <algorithm>
#include <numeric>
#include <chrono>
#include <thread>

#include "../include/hastar.h"
#include "../include/hastar_f64.h"

namespace orc {
// Optional pop limit for census tools (0 = none, the reference's behaviour): a search that
// reaches it stops with stats.status = HASTAR_EOVERFLOW and is reported as failed.
long long g_max_pops = 0;
#ifdef ORC_BRANCH_STATS
// analysis build (tools/branch_stats.py): how often the inner A*'s per-neighbour branches go
// each way (valid neighbours, closed, find hits, replacements, inserts, closed re-pops)
long long g_br[8];
#endif
#ifdef ORC_OUTER_STATS
// analysis build (tools/outer_shape_stats.py): how often the OUTER open set's tree shape can
// decide a find / insert (a node of the same key on the "wrong" side of the probe f)
long long g_oshape[16];
#endif
#ifdef ORC_SHAPE_STATS
long long g_shape[16];
bool g_search_unsafe;       // the current inner search met a shape-dependent find/insert
int g_migrated;             // bit k: the current inner search's open set has exceeded kCaps[k]
long long g_search_pops;    // pops of the current inner search
long long g_pops_to_unsafe; // pops before its first shape-dependent event
#endif

template <class T> struct P2 { T x, y; };
template <class T> struct P3 { T x, y, h; };

// common.h:15-29
template <class T> T wrap_pi(T a) {
  T w = std::fmod(a, 2 * M_PI);
  if (w > M_PI) return w - 2 * M_PI;
  if (w < -M_PI) return w + 2 * M_PI;
  return w;
}
// common.h:8-12, 31-36
template <class T> int heading_bin(T h, T prec) {
  T r = std::round(h / prec) * prec;
  return static_cast<int>((r + M_PI) / prec);
}
// common.h:55-61 (Vector2D::get_rotated_vector / rotate_vector)
template <class T> P2<T> rot2(T x, T y, T ang) {
  T c = std::cos(ang), s = std::sin(ang);
  return {x * c + y * s, -x * s + y * c};
}
// common.h:162-169 (Vector3D::get_rotated_vector)
template <class T> P3<T> rot3(P3<T> p, T ang) {
  T c = std::cos(ang), s = std::sin(ang);
  return {p.x * c + p.y * s, -p.x * s + p.y * c, wrap_pi<T>(p.h - ang)};
}
template <class T> T stl_max(T a, T b) { return (a < b) ? b : a; }
template <class T> T stl_min(T a, T b) { return (b < a) ? b : a; }

static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
static inline uint32_t f32bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
// the pop digest's g term: the float bit pattern, or the double's 64 bits (HybridAStar<double>)
static inline uint64_t gbits(float g) { return f32bits(g); }
static inline uint64_t gbits(double g) { uint64_t u; std::memcpy(&u, &g, 8); return u; }

// ------------------------------------------------------------------ Dubins (Dubins.cpp)
enum Word { RSR = 0, RSL = 1, LSR = 2, LSL = 3 };

template <class T> struct DubinsCSC {
  T r, step, ang_step;
  T prm[4];
  int word = RSR;
  DubinsCSC(T r_min, T step_size) : r(r_min), step(step_size), ang_step(step_size / r_min) {
    prm[0] = prm[1] = prm[2] = prm[3] = 0;
  }
  // Dubins.cpp:180-323 — one CSC word: fills q[4] and returns its length
  T word_len(int w, P2<T> cs, P2<T> cg, const P3<T>& s, const P3<T>& g, T q[4]) const {
    P2<T> d{cg.x - cs.x, cg.y - cs.y};
    if (w == RSR || w == LSL) {
      T th = std::atan2(d.y, d.x);
      T sgn = (w == RSR) ? 1 : -1;
      q[0] = sgn * M_PI_2 + s.h;
      T t1 = sgn * M_PI_2 + th;
      q[2] = t1;
      T tg = sgn * M_PI_2 + g.h;
      q[1] = t1 - q[0];
      q[3] = tg - q[2];
      if (w == RSR) {
        if (q[1] > 0) q[1] -= 2 * M_PI;
        if (q[3] > 0) q[3] -= 2 * M_PI;
      } else {
        if (q[1] < 0) q[1] += 2 * M_PI;
        if (q[3] < 0) q[3] += 2 * M_PI;
      }
      T dst = std::sqrt(d.x * d.x + d.y * d.y);
      return (w == RSR) ? dst + r * -(q[1] + q[3]) : dst + r * (q[1] + q[3]);
    }
    T dist = std::sqrt(d.x * d.x + d.y * d.y);
    T th = std::atan2(d.y, d.x);
    T t1;
    if (w == RSL) {
      q[0] = M_PI_2 + s.h;
      t1 = std::acos(2 * r / dist) + th;
      q[2] = t1 - M_PI;
      T tg = -M_PI_2 + g.h;
      q[1] = t1 - q[0];
      if (q[1] > 0) q[1] -= 2 * M_PI;
      q[3] = tg - q[2];
      if (q[3] < 0) q[3] += 2 * M_PI;
    } else {
      q[0] = -M_PI_2 + s.h;
      t1 = -std::acos(2 * r / dist) + th;
      q[2] = t1 + M_PI;
      T tg = M_PI_2 + g.h;
      q[1] = t1 - q[0];
      if (q[1] < 0) q[1] += 2 * M_PI;
      q[3] = tg - q[2];
      if (q[3] > 0) q[3] -= 2 * M_PI;
    }
    P2<T> a{cs.x, cs.y}, b{cg.x, cg.y};
    a.x += r * std::cos(t1);
    a.y += r * std::sin(t1);
    b.x += r * std::cos(q[2]);
    b.y += r * std::sin(q[2]);
    P2<T> e{b.x - a.x, b.y - a.y};
    T dst = std::sqrt(e.x * e.x + e.y * e.y);
    return (w == RSL) ? dst + r * (-q[1] + q[3]) : dst + r * (q[1] - q[3]);
  }
  // Dubins.cpp:19-69 (+ centres, 76-87)
  T shortest(const P3<T>& s, const P3<T>& g, P2<T> c[4]) {
    c[0] = {s.x + r * std::sin(s.h), s.y - r * std::cos(s.h)};  // start right
    c[1] = {s.x - r * std::sin(s.h), s.y + r * std::cos(s.h)};  // start left
    c[2] = {g.x + r * std::sin(g.h), g.y - r * std::cos(g.h)};  // goal right
    c[3] = {g.x - r * std::sin(g.h), g.y + r * std::cos(g.h)};  // goal left
    static const int si[4] = {0, 0, 1, 1}, gi[4] = {2, 3, 2, 3};
    T best = 0;
    for (int w = 0; w < 4; ++w) {
      T q[4];
      T len = word_len(w, c[si[w]], c[gi[w]], s, g, q);
      if (w == 0 || len < best) {
        best = len;
        word = w;
        std::copy(q, q + 4, prm);
      }
    }
    return best;
  }
  T shortest(const P3<T>& s, const P3<T>& g) {
    P2<T> c[4];
    return shortest(s, g, c);
  }
  // Dubins.cpp:326-563: three segments + final pose; first/second arc direction by word
  void sample(P2<T> cs, P2<T> cg, std::vector<P3<T>>& out, std::vector<T>& curv) const {
    const bool s_right = (word == RSR || word == RSL);
    const bool g_right = (word == RSR || word == LSR);
    P2<T> a = cs, b = cg;
    a.x += r * std::cos(prm[0] + prm[1]);
    a.y += r * std::sin(prm[0] + prm[1]);
    b.x += r * std::cos(prm[2]);
    b.y += r * std::sin(prm[2]);
    P2<T> e{b.x - a.x, b.y - a.y};
    T lst = std::sqrt(e.x * e.x + e.y * e.y);
    int n1 = static_cast<int>(std::floor((s_right ? -prm[1] : prm[1]) / ang_step));
    int n2 = n1 + static_cast<int>(std::floor(lst / step));
    int n3 = n2 + static_cast<int>(std::floor((g_right ? -prm[3] : prm[3]) / ang_step));
    out.resize(n3 + 1);
    curv.resize(n3 + 1);
    T th = prm[0], k = 1 / r;
    for (int i = 0; i < n1; ++i) {
      out[i].x = cs.x + r * std::cos(th);
      out[i].y = cs.y + r * std::sin(th);
      // wrap_pi(theta -/+ M_PI_2) deduces T = double in Dubins.cpp:417,477,537,597
      out[i].h = static_cast<T>(s_right ? wrap_pi<double>(th - M_PI_2) : wrap_pi<double>(th + M_PI_2));
      curv[i] = k;
      if (s_right) th -= ang_step; else th += ang_step;
    }
    th = std::atan2(e.y, e.x);
    T ct = std::cos(th), st = std::sin(th), dd = 0;
    for (int i = n1; i < n2; ++i) {
      out[i].x = a.x + dd * ct;
      out[i].y = a.y + dd * st;
      out[i].h = th;
      curv[i] = 0;
      dd += step;
    }
    th = prm[2];
    for (int i = n2; i < n3; ++i) {
      out[i].x = cg.x + r * std::cos(th);
      out[i].y = cg.y + r * std::sin(th);
      out[i].h = static_cast<T>(g_right ? wrap_pi<double>(th - M_PI_2) : wrap_pi<double>(th + M_PI_2));
      curv[i] = k;
      if (g_right) th -= ang_step; else th += ang_step;
    }
    out[n3].x = cg.x + r * std::cos(prm[2] + prm[3]);
    out[n3].y = cg.y + r * std::sin(prm[2] + prm[3]);
    out[n3].h = static_cast<T>(g_right ? wrap_pi<double>(prm[2] + prm[3] - M_PI_2)
                                        : wrap_pi<double>(prm[2] + prm[3] + M_PI_2));
    curv[n3] = 0;
  }
  // Dubins.cpp:125-153: returns {length, first arc longer than 90 deg}
  std::pair<T, bool> path(const P3<T>& s, const P3<T>& g, std::vector<P3<T>>& out, std::vector<T>& curv) {
    P2<T> c[4];
    T len = shortest(s, g, c);
    static const int si[4] = {0, 0, 1, 1}, gi[4] = {2, 3, 2, 3};
    sample(c[si[word]], c[gi[word]], out, curv);
    return {len, std::abs(prm[1]) > static_cast<T>(M_PI_2)};
  }
};

// ------------------------------------------------------------ motion primitives
// VehicleModel.cpp:7-47 and 147-164.  The table row for heading bin == num_angle_bins
// (reached when a heading rounds to +pi, VehicleModel.cpp:145) reads past the end of
// the reference's vector (UB); glibc hands it the next chunk's unused prev_size word,
// i.e. (0, 0).  We store that (0, 0) row explicitly.
template <class T> struct Motion {
  T ts, a_lat, a_lat2, prec;
  int na, bins, nsteer;
  std::vector<T> curv_abs, curv_signed, cost, dth;
  std::vector<P2<T>> off;  // nsteer x (bins + 1)
  Motion(T ts_, T max_lat_acc, T wheelbase, T rear_to_cg, int bins_, int na_, const std::vector<T>& steer,
         const std::vector<T>& w)
      : ts(ts_), a_lat(max_lat_acc), a_lat2(max_lat_acc * max_lat_acc), prec(2 * M_PI / bins_), na(na_),
        bins(bins_), nsteer((int)steer.size()) {
    std::vector<T> beta(nsteer);
    curv_signed.resize(nsteer);
    for (int i = 0; i < nsteer; ++i) {
      beta[i] = std::atan2(rear_to_cg * std::tan(steer[i]), wheelbase);
      curv_signed[i] = std::cos(beta[i]) * std::tan(steer[i]) / wheelbase;
    }
    cost.resize(nsteer);
    dth.resize(nsteer);
    off.assign((size_t)nsteer * (bins + 1), P2<T>{0, 0});
    for (int i = 0; i < nsteer; ++i) {
      dth[i] = ts * curv_signed[i];
      cost[i] = ts + w[i] * std::abs(curv_signed[i]);
      for (int j = 0; j < bins; ++j) {
        T head = -M_PI + j * prec;
        // calculate_offset(): explicit Euler, dt = 1 ms
        const T dt = static_cast<T>(0.001);
        T ox = 0, oy = 0, hh = head;
        int n = static_cast<int>(ts / dt);
        for (int k = 0; k < n; ++k) {
          ox += dt * std::cos(beta[i] + hh);
          oy += dt * std::sin(beta[i] + hh);
          hh += dt * curv_signed[i];
        }
        off[(size_t)i * (bins + 1) + j] = {ox, oy};
      }
    }
    curv_abs.resize(nsteer);
    for (int i = 0; i < nsteer; ++i) curv_abs[i] = std::abs(curv_signed[i]);
  }
  const P2<T>& offset(int a, int bin) const { return off[(size_t)a * (bins + 1) + bin]; }
};

// ------------------------------------------------------------------ nodes + sets
template <class T> struct N3 {
  P3<T> pose;
  T g, f, vmin;
  int ci, bin, cx, cy;
  const N3* prev;
};
template <class T> struct N3Less {
  bool operator()(const N3<T>& a, const N3<T>& b) const {
    return (a.cx != b.cx || a.cy != b.cy || a.bin != b.bin) && a.f < b.f;
  }
};
template <class T> struct N3Hash {
  size_t operator()(const N3<T>& n) const {
    return mix64(((uint64_t)(uint32_t)n.cx << 40) ^ ((uint64_t)(uint32_t)n.cy << 16) ^ (uint32_t)n.bin);
  }
};
template <class T> struct N3Eq {
  bool operator()(const N3<T>& a, const N3<T>& b) const {
    return a.cx == b.cx && a.cy == b.cy && a.bin == b.bin;
  }
};
template <class T> struct N2 {
  int x, y;
  T g, f;
  const N2* prev;
};
template <class T> struct N2Less {
  bool operator()(const N2<T>& a, const N2<T>& b) const { return (a.x != b.x || a.y != b.y) && a.f < b.f; }
};
template <class T> struct N2Hash {
  size_t operator()(const N2<T>& n) const { return mix64(((uint64_t)(uint32_t)n.x << 32) | (uint32_t)n.y); }
};
template <class T> struct N2Eq {
  bool operator()(const N2<T>& a, const N2<T>& b) const { return a.x == b.x && a.y == b.y; }
};

// ------------------------------------------------------------------ the planner
template <class T> struct Planner {
  // parameters
  int shot_interval, shot_decay;
  T res, thr, lp_min, lp_max, lp_free;
  int N, n2, n45;
  bool diag;
  T apf_rep, apf_ang;
  Motion<T> mv;
  DubinsCSC<T> dub;
  // Grid2D state (Grid2D.h:47-60)
  T grid_heading = 0;
  P2<T> goal2{0, 0};
  std::vector<T> occ;      // log-odds, N*N, [i*N + j]
  std::vector<T> nm_h, nm_f;
  std::vector<int> act_dx, act_dy;
  std::vector<T> act_cost;
  // Grid3D state
  P3<T> goal3{0, 0, 0};
  struct Apf { T x, y, r; };
  std::vector<Apf> apf;
  // AStar state (AStar.h:63-72)
  std::vector<uint8_t> visited;
  N2<T> astar_goal{0, 0, 0, 0, nullptr};
  std::set<N2<T>, N2Less<T>> op2;
  std::unordered_set<N2<T>, N2Hash<T>, N2Eq<T>> cl2;
  // HybridAStar state
  N3<T> goal_node{};
  std::set<N3<T>, N3Less<T>> op3;
  std::unordered_set<N3<T>, N3Hash<T>, N3Eq<T>> cl3;
  bool shot_ok = false;
  std::vector<P3<T>> shot_path;
  std::vector<T> shot_curv;
  N3<T> terminal{};
  // statistics
  hastar_stats st{};

  template <class In> static std::vector<T> tovec(const In* p, int n) { return std::vector<T>(p, p + n); }

  // PR = hastar_params (float inputs) or hastar_params_f64 (HybridAStar<double>)
  template <class PR> explicit Planner(const PR& p)
      : shot_interval(p.dubins_shot_interval), shot_decay(p.dubins_shot_interval_decay),
        res(p.grid_resolution),
        thr(std::log(static_cast<T>(p.obstacle_threshold) / (1.0 - static_cast<T>(p.obstacle_threshold)))),
        lp_min(std::log(static_cast<T>(p.obstacle_prob_min) / (1.0 - static_cast<T>(p.obstacle_prob_min)))),
        lp_max(std::log(static_cast<T>(p.obstacle_prob_max) / (1.0 - static_cast<T>(p.obstacle_prob_max)))),
        lp_free(std::log(static_cast<T>(p.obstacle_prob_free) / (1.0 - static_cast<T>(p.obstacle_prob_free)))),
        N(p.grid_size), n2(static_cast<int>(std::round(p.grid_size * 0.5))),
        n45(static_cast<int>(std::round(p.grid_size * 0.8))), diag(p.grid_2d_allow_diag_moves != 0),
        apf_rep(p.apf_rep_constant), apf_ang(p.apf_active_angle),
        mv(p.step_size, p.max_lat_acc, p.wheelbase, p.rear_to_cg, p.num_angle_bins, p.num_actions,
           tovec(p.steering, p.num_steering), tovec(p.curvature_weights, p.num_steering)),
        dub(min_radius(p), p.step_size) {
    occ.assign((size_t)N * N, 0);
    nm_h.resize((size_t)N * N);
    for (int i = 0; i < N; ++i) {  // Grid2D::compute_heuristic (Grid2D.cpp:303-316)
      T dx = (n45 - i) * res;
      T dx2 = dx * dx;
      for (int j = 0; j < N; ++j) {
        T dy = (n2 - j) * res;
        T dy2 = dy * dy;
        nm_h[(size_t)i * N + j] = std::sqrt(dx2 + dy2);
      }
    }
    nm_f = nm_h;  // Node2D(i, j) then set_heuristic_cost: f = 0 + h
    static const int d8x[8] = {0, 1, 1, 1, 0, -1, -1, -1}, d8y[8] = {-1, -1, 0, 1, 1, 1, 0, -1};
    static const int d4x[4] = {0, 1, 0, -1}, d4y[4] = {-1, 0, 1, 0};
    int na = diag ? 8 : 4;
    for (int k = 0; k < na; ++k) {
      int ax = diag ? d8x[k] : d4x[k], ay = diag ? d8y[k] : d4y[k];
      act_dx.push_back(ax);
      act_dy.push_back(ay);
      act_cost.push_back(res * std::sqrt(static_cast<T>(ax * ax + ay * ay)));
    }
    visited.assign((size_t)N * N, 0);
  }
  // HybridAStar.cpp:22-24 (tan_max over steering, HybridAStar.h:20-25)
  template <class PR> static T min_radius(const PR& p) {
    T mx = *std::max_element(p.steering, p.steering + p.num_steering);
    T tm = std::tan(mx);
    return static_cast<T>(p.wheelbase) / (std::cos(std::atan2(static_cast<T>(p.rear_to_cg) * tm,
                                                             static_cast<T>(p.wheelbase))) * tm);
  }

  bool inside(int i, int j) const { return i > -1 && i < N && j > -1 && j < N; }
  T& cell(int i, int j) { return occ[(size_t)i * N + j]; }
  void bump(int i, int j, T delta) {  // Grid2D.cpp:131-132
    T& m = cell(i, j);
    m += delta;
    m = stl_max(stl_min(m, lp_max), lp_min);
  }

  // ---------------------------------------------------------------- map upkeep
  // Grid2D::update_obstacles() (Grid2D.cpp:197-208)
  void decay() {
    for (auto& m : occ) {
      m += lp_free;
      m = stl_max(stl_min(m, lp_max), lp_min);
    }
  }
  // Grid3D::update_obstacles(boxes) (Grid3D.cpp:22-44) + Grid2D boxes (Grid2D.cpp:99-139)
  template <class In> void boxes(const In* b, const In* conf, int n, T apf_r) {
    apf.clear();
    for (int k = 0; k < n; ++k) {
      T ox = b[4 * k], oy = b[4 * k + 1], dx = b[4 * k + 2], dy = b[4 * k + 3];
      P2<T> p = rot2<T>(ox - goal3.x, oy - goal3.y, grid_heading);
      p.x += n45 * res;
      p.y += n2 * res;
      apf.push_back({p.x, p.y, std::max(dx, dy) / 2 + apf_r});
    }
    for (int k = 0; k < n; ++k) {
      T ox = b[4 * k], oy = b[4 * k + 1], dx = b[4 * k + 2], dy = b[4 * k + 3];
      P2<T> bl = rot2<T>((ox - dx / 2) - goal2.x, (oy - dy / 2) - goal2.y, grid_heading);
      int si = static_cast<int>(std::round(bl.x / res) + n45);
      int sj = static_cast<int>(std::round(bl.y / res) + n2);
      int ei = static_cast<int>(std::ceil(dx / res)), ej = static_cast<int>(std::ceil(dy / res));
      T lc = std::log(static_cast<T>(conf[k]) / (1.0 - static_cast<T>(conf[k])));
      for (int i = 0; i < 2 * ei; ++i)
        for (int j = 0; j < 2 * ej; ++j) {
          P2<T> o = rot2<T>(i * 0.5, j * 0.5, grid_heading);
          int ip = si + static_cast<int>(std::round(o.x));
          int jp = sj + static_cast<int>(std::round(o.y));
          if (inside(ip, jp)) bump(ip, jp, lc - lp_free);
        }
    }
  }
  // Grid2D::update_obstacles(lines) (Grid2D.cpp:142-194)
  template <class In> void lines(const In* L, const In* conf, int n, T width) {
    for (int k = 0; k < n; ++k) {
      P2<T> a = rot2<T>(static_cast<T>(L[4 * k]) - goal2.x, static_cast<T>(L[4 * k + 1]) - goal2.y, grid_heading);
      P2<T> b = rot2<T>(static_cast<T>(L[4 * k + 2]) - goal2.x, static_cast<T>(L[4 * k + 3]) - goal2.y, grid_heading);
      P2<T> d{b.x - a.x, b.y - a.y};
      T len = std::hypot(d.x, d.y);
      P2<T> nrm{-d.y / len, d.x / len};
      d = {d.x / len, d.y / len};
      T lc = std::log(static_cast<T>(conf[k]) / (1.0 - static_cast<T>(conf[k])));
      T pl = 0;
      for (size_t it = 0; pl <= len && it < 100; ++it, pl += res) {
        P2<T> c{a.x + d.x * pl, a.y + d.y * pl};
        for (T pw = 0; pw <= width; pw += res) {
          P2<T> p1{c.x + nrm.x * pw, c.y + nrm.y * pw};
          P2<T> p2{c.x - nrm.x * pw, c.y - nrm.y * pw};
          int i1 = static_cast<int>(std::round(p1.x / res)) + n45, i2 = static_cast<int>(std::round(p2.x / res)) + n45;
          int j1 = static_cast<int>(std::round(p1.y / res)) + n2, j2 = static_cast<int>(std::round(p2.y / res)) + n2;
          if (inside(i1, j1)) bump(i1, j1, lc - lp_free);
          if (inside(i2, j2)) bump(i2, j2, lc - lp_free);
        }
      }
    }
  }
  // Grid3D::update_goal_heading + relocate_obstacles (Grid3D.cpp:102-124, 169-203)
  void update_goal(const P3<T>& g, const P3<T>& s) {
    T gh_prev = grid_heading;
    P3<T> g3_prev = goal3;
    goal2 = {g.x, g.y};
    grid_heading = std::atan2(g.y - s.y, g.x - s.x);
    goal3 = g;
    // relocate
    T dh = grid_heading - gh_prev;
    P2<T> gp = rot2<T>(static_cast<T>(n45), static_cast<T>(n2), dh);
    P2<T> gno = rot2<T>(g3_prev.x - goal3.x, g3_prev.y - goal3.y, grid_heading);
    P2<T> org{static_cast<T>(n45) + gno.x / res, static_cast<T>(n2) + gno.y / res};
    org = {org.x - gp.x, org.y - gp.y};
    std::vector<T> nm((size_t)N * N, static_cast<T>(0));
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < N; ++j) {
        P2<T> q = rot2<T>(static_cast<T>(i), static_cast<T>(j), dh);
        q = {q.x + org.x, q.y + org.y};
        int a = static_cast<int>(std::round(q.x)), b = static_cast<int>(std::round(q.y));
        if (inside(a, b)) nm[(size_t)a * N + b] = occ[(size_t)i * N + j];
      }
    occ.swap(nm);
    // goal node (Grid3D.cpp:115-123); AStar::update_goal_node takes the cell
    goal_node = N3<T>{};
    goal_node.pose = {n45 * res, n2 * res, wrap_pi<T>(g.h - grid_heading)};
    goal_node.bin = heading_bin<T>(goal_node.pose.h, mv.prec);
    goal_node.cx = n45;
    goal_node.cy = n2;
    astar_goal = {n45, n2, 0, nm_f[(size_t)n45 * N + n2], nullptr};
  }
  void reset() { std::fill(visited.begin(), visited.end(), 0); }
  // ---- the stand-alone AStar's plain Grid2D (AStar.h without STORE_GRID_AS_REFERENCE) ----
  // Grid2D::update_goal_heading (Grid2D.cpp:260-266): no relocation
  void goal_2d(const P2<T>& g, const P2<T>& s) {
    goal2 = g;
    grid_heading = std::atan2(g.y - s.y, g.x - s.x);
    astar_goal = {n45, n2, 0, nm_f[(size_t)n45 * N + n2], nullptr};
  }
  // Grid2D::set_start_node (Grid2D.cpp:270-290)
  std::pair<int, int> start_2d(const P2<T>& s) {
    P2<T> rel = rot2<T>(s.x - goal2.x, s.y - goal2.y, grid_heading);
    int i = static_cast<int>(rel.x / res) + n45, j = static_cast<int>(rel.y / res) + n2;
    if (!inside(i, j)) i = j = 0;
    nm_f[(size_t)i * N + j] = nm_h[(size_t)i * N + j];
    return {i, j};
  }
  // AStar::reconstruct_path (AStar.cpp:189-205): world points of the goal's predecessors
  void path_2d(const P2<T>& goal, std::vector<P2<T>>& out) const {
    for (const N2<T>* p = astar_goal.prev; p; p = p->prev) {
      P2<T> rel{(p->x - astar_goal.x) * res, (p->y - astar_goal.y) * res};
      P2<T> w = rot2<T>(rel.x, rel.y, -grid_heading);
      out.push_back({w.x + goal.x, w.y + goal.y});
    }
  }

#ifdef ORC_SHAPE_STATS
  // Analysis build only (tools/astar_shape_stats.py): how often the open tree's shape can
  // matter for find/insert (a node of the same cell on the "wrong" side of the probe f).
  template <class S> void shape_probe(const S& op, int i, int j, T fprobe, T fn) {
    bool same = false, unsafe_find = false, unsafe_ins = false;
    int nsame = 0;
    T prev = -std::numeric_limits<T>::infinity();
    for (const auto& n : op) {
      if (!(n.f > prev)) g_shape[7]++;  // strict f order violated
      prev = n.f;
      if (n.x == i && n.y == j) {
        same = true;
        ++nsame;
        if (n.f < fprobe) unsafe_find = true;
        if (n.f > fn) unsafe_ins = true;
      }
    }
    g_shape[0]++;
    g_shape[1] += same;
    g_shape[2] += unsafe_find;
    g_shape[3] += unsafe_ins;
    // the kernel's rank-only path is exact unless one of these holds (csrc: astar_loop_lds)
    if ((unsafe_find || unsafe_ins || nsame > 1) && !g_search_unsafe) {
      g_search_unsafe = true;
      g_pops_to_unsafe = g_search_pops;
    }
  }
  // per inner search: [8] searches, [9] searches with a shape-dependent event, [10] pops of all
  // searches, [11] pops of those searches, [12] their pops before the first event
  void shape_search_end() {
    g_shape[8]++;
    g_shape[10] += g_search_pops;
    if (g_search_unsafe) {
      g_shape[9]++;
      g_shape[11] += g_search_pops;
      g_shape[12] += g_pops_to_unsafe;
    }
    g_search_unsafe = false;
    g_search_pops = 0;
    g_migrated = 0;
  }
  void shape_size(size_t n) {
    if ((long long)n > g_shape[4]) g_shape[4] = (long long)n;
    g_shape[5] += n > 256;
    g_shape[6] += n > 1024;
    // [13..15]: pops of inner searches after their open set first exceeded 703 / 767 / 1023
    // nodes (the LDS pool sizes of the kernel, minus the header): the pops an LDS pool of that
    // size would run in HBM mode (migration is one-way)
    static const size_t kCaps[3] = {703, 767, 1023};
    for (int k = 0; k < 3; ++k) {
      if (n > kCaps[k]) g_migrated |= 1 << k;
      if (g_migrated & (1 << k)) g_shape[13 + k]++;
    }
  }
#endif
  // ----------------------------------------------------- holonomic heuristic (AStar)
  // AStar::update_visted + Grid2D::update_costs (AStar.cpp:209-218, Grid2D.cpp:219-227)
  void memoise(T total, const N2<T>* last) {
    for (const N2<T>* p = last; p; p = p->prev) visited[(size_t)p->x * N + p->y] = 1;
    for (const N2<T>* p = last; p; p = p->prev) nm_f[(size_t)p->x * N + p->y] = total - p->g;
  }
  // AStar::find_path(int, int) (AStar.cpp:100-113) + a_star_search (118-186)
  T holonomic(int si, int sj) {
    if (visited[(size_t)si * N + sj]) return nm_f[(size_t)si * N + sj];
    return a_star(si, sj, true);
  }
  // AStar::a_star_search(start, get_cost_only) (AStar.cpp:118-186) from the soft-reset start
  T a_star(int si, int sj, bool cost_only) {
    nm_f[(size_t)si * N + sj] = nm_h[(size_t)si * N + sj];  // Node2D::soft_reset
#ifndef ORC_LEAN
    st.astar_searches++;
#endif
    cl2.clear();
    op2.clear();
    op2.insert(N2<T>{si, sj, 0, nm_f[(size_t)si * N + sj], nullptr});
#ifdef ORC_SHAPE_STATS
    struct End {
      Planner* p;
      ~End() { p->shape_search_end(); }
    } end_{this};
#endif
    while (!op2.empty()) {
#ifdef ORC_SHAPE_STATS
      shape_size(op2.size());
      g_search_pops++;
#endif
      auto it = op2.begin();
#ifdef ORC_BRANCH_STATS
      const auto ins_r = cl2.insert(*it);
      const N2<T>* cur = &*ins_r.first;
      g_br[6]++;
      g_br[7] += !ins_r.second;  // the popped cell was closed already
#else
      const N2<T>* cur = &*cl2.insert(*it).first;
#endif
      op2.erase(it);
#ifndef ORC_LEAN
      st.astar_pops++;
#endif
      if (cur->x == astar_goal.x && cur->y == astar_goal.y) {
        astar_goal = *cur;
        if (cost_only) memoise(astar_goal.f, &astar_goal);
        return astar_goal.f;
      }
      const T g0 = cur->g;
      for (size_t k = 0; k < act_dx.size(); ++k) {
        int i = cur->x + act_dx[k], j = cur->y + act_dy[k];
        if (!inside(i, j) || !(occ[(size_t)i * N + j] < thr)) continue;  // Grid2D::get_neighbors
        const size_t c = (size_t)i * N + j;
        if (cost_only && visited[c]) {
          T tot = nm_f[c] + g0 + act_cost[k];
          memoise(tot, cur);
          return tot;
        }
        N2<T> probe{i, j, 0, nm_f[c], nullptr};
#ifdef ORC_BRANCH_STATS
        g_br[0]++;
        if (cl2.find(probe) != cl2.end()) { g_br[1]++; continue; }
#else
        if (cl2.find(probe) != cl2.end()) continue;
#endif
#ifdef ORC_SHAPE_STATS
        shape_probe(op2, i, j, nm_f[c], g0 + act_cost[k] + nm_h[c]);
#endif
        auto hit = op2.find(probe);
        const T gn = g0 + act_cost[k];
#ifdef ORC_BRANCH_STATS
        g_br[2] += hit != op2.end();
        g_br[3] += hit != op2.end() && gn < hit->g;
        g_br[4] += hit == op2.end();
        {  // an open node of this cell exists (the kernel's cell hint)
          bool any = false;
          for (const auto& n : op2) any |= (n.x == i && n.y == j);
          g_br[5] += any;
        }
#endif
        if (hit == op2.end()) {
          nm_f[c] = gn + nm_h[c];  // Node2D::set_accumulated_cost
          op2.insert(N2<T>{i, j, gn, nm_f[c], cur});
        } else if (gn < hit->g) {
          op2.erase(hit);
          nm_f[c] = gn + nm_h[c];
          op2.insert(N2<T>{i, j, gn, nm_f[c], cur});
        }
      }
    }
    return std::numeric_limits<T>::max();
  }

  // -------------------------------------------------------------- successors
  // Grid3D::get_field_intensity (Grid3D.cpp:206-227)
  T field(const P3<T>& p) const {
    T acc = static_cast<T>(0.0);
    for (const Apf& o : apf) {
      T d = std::hypot(o.x - p.x, o.y - p.y);
      T ang = std::abs(wrap_pi<T>(p.h - std::atan2(o.y - p.y, o.x - p.x)));
      ang = stl_max<T>(apf_ang - ang, static_cast<T>(0.0));
      T fp = 0;
      if (d < o.r) {
        double t = 1.0 / d - 1.0 / o.r;
        fp = apf_rep * (t * t);  // std::pow(t, 2) is folded to t*t by GCC
        fp = fp * ang / apf_ang;
      }
      acc = acc + fp;
    }
    return acc;
  }
  // VehicleModel::get_neighbors (VehicleModel.cpp:63-105) + Grid3D filter (Grid3D.cpp:47-74)
  bool expand(const N3<T>& nd, std::vector<N3<T>>& out) {
    out.clear();
    int size = mv.nsteer;
    int lo = nd.ci - mv.na;
    lo = lo < 0 ? 0 : lo;
    const bool slow = nd.vmin < static_cast<T>(1.0);
    for (int i = lo; i < lo + 2 * mv.na + 1 && i < size; ++i) {
      T vm = 0;
      if (!slow) {
        T lat = nd.vmin * mv.curv_abs[i];
        if (lat > mv.a_lat) continue;
        T al = std::sqrt(1.0 - ((lat * lat) / mv.a_lat2));
        vm = nd.vmin - 2 * al * mv.ts;
      }
      const P2<T>& o = mv.offset(i, nd.bin);
      N3<T> s;
      s.pose = {nd.pose.x + o.x, nd.pose.y + o.y, wrap_pi<T>(nd.pose.h + mv.dth[i])};
      s.g = nd.g + mv.cost[i];
      s.f = s.g;
      s.vmin = vm;
      s.ci = i;
      s.bin = heading_bin<T>(s.pose.h, mv.prec);
      s.prev = &nd;
      int ci = static_cast<int>(s.pose.x / res), cj = static_cast<int>(s.pose.y / res);
      if (!(inside(ci, cj) && occ[(size_t)ci * N + cj] < thr)) continue;
      T fc = field(s.pose);
      s.g += fc;
      s.f += fc;
      s.cx = ci;
      s.cy = cj;
      out.push_back(s);
    }
#ifndef ORC_LEAN
    st.successors += (long long)out.size();
#endif
    return slow;
  }
  // Grid3D::check_path (Grid3D.cpp:78-93)
  bool free_path(const std::vector<P3<T>>& path) const {
    for (const auto& q : path) {
      int i = static_cast<int>(std::round(q.x / res)), j = static_cast<int>(std::round(q.y / res));
      if (!inside(i, j) || occ[(size_t)i * N + j] >= thr) return false;
    }
    return true;
  }

#ifdef ORC_OUTER_STATS
  bool g_oevent = false;
  void outer_ins_stat(const N3<T>& s) {
    int nsame = 0;
    bool gt = false;
    for (const auto& n : op3)
      if (n.cx == s.cx && n.cy == s.cy && n.bin == s.bin) {
        ++nsame;
        gt |= n.f > s.f;
      }
    g_oshape[3]++;
    g_oshape[4] += gt;
    g_oshape[5] += nsame > 1;
    if ((gt || nsame > 1) && !g_oevent) { g_oevent = true; g_oshape[7] += st.pops; }
  }
#endif
  // ----------------------------------------------------------------- search
  // HybridAStar::hybrid_a_star_search (HybridAStar.cpp:93-199)
  std::pair<T, bool> search(const N3<T>& start) {
#ifdef ORC_OUTER_STATS
    g_oevent = false;
    struct OEnd {
      Planner* p;
      ~OEnd() {
        g_oshape[10]++;
        if (!p->g_oevent) g_oshape[7] += p->st.pops;  // a search without event: all its pops
        else g_oshape[11]++;
      }
    } oend_{this};
#endif
    int counter = 0, interval = shot_interval;
    bool shot_allowed = false;
    shot_ok = false;
    cl3.clear();
    op3.clear();
    op3.insert(start);
    std::vector<N3<T>> nb;
    uint64_t dig = 0x243f6a8885a308d3ull;
    std::pair<T, bool> out{std::numeric_limits<T>::max(), false};
    while (!op3.empty()) {
      if (g_max_pops > 0 && st.pops >= g_max_pops) {
        st.status = HASTAR_EOVERFLOW;
        break;
      }
      auto it = op3.begin();
      const N3<T>* cur = &*cl3.insert(*it).first;
      op3.erase(it);
      st.pops++;
#ifndef ORC_LEAN
      dig = mix64(dig ^ (((uint64_t)(uint32_t)cur->cx << 40) | ((uint64_t)(uint32_t)cur->cy << 16) |
                         (uint64_t)(uint32_t)cur->bin)) + gbits(cur->g);
#endif
      if (cur->cx == goal_node.cx && cur->cy == goal_node.cy) {
        terminal = *cur;
        out = {terminal.g, true};
        break;
      }
      if (shot_allowed) {
        if (++counter == interval) {
#ifndef ORC_LEAN
          st.shots++;
#endif
          auto pr = dub.path(cur->pose, goal_node.pose, shot_path, shot_curv);
          if (!pr.second && free_path(shot_path)) {
            terminal = *cur->prev;
            shot_ok = true;
            out = {cur->g + pr.first, true};
            break;
          }
          counter = 0;
          interval = std::max(interval - shot_decay, 50);
        }
      }
      shot_allowed = expand(*cur, nb);
#ifdef ORC_OUTER_STATS
      g_oshape[6]++;
      if ((long long)op3.size() > g_oshape[8]) g_oshape[8] = (long long)op3.size();
#endif
      for (auto& s : nb) {
        if (cl3.find(s) != cl3.end()) continue;
#ifdef ORC_OUTER_STATS
        {
          int nsame = 0;
          bool lt = false;
          for (const auto& n : op3)
            if (n.cx == s.cx && n.cy == s.cy && n.bin == s.bin) {
              ++nsame;
              lt |= n.f < s.g;
            }
          g_oshape[0]++;
          g_oshape[1] += nsame > 0;
          g_oshape[2] += lt;
          g_oshape[5] += nsame > 1;
          g_oshape[9] += !op3.empty() && s.g > op3.begin()->f;
          if ((lt || nsame > 1) && !g_oevent) { g_oevent = true; g_oshape[7] += st.pops; }
        }
#endif
        auto hit = op3.find(s);
        if (hit == op3.end()) {
          T h1 = holonomic(s.cx, s.cy);
          T h2 = dub.shortest(s.pose, goal_node.pose);
          s.f += stl_max(h1, h2);
          s.prev = cur;
#ifdef ORC_OUTER_STATS
          outer_ins_stat(s);
#endif
          op3.insert(s);
        } else if (s.g < hit->g) {
          op3.erase(hit);
          T h1 = holonomic(s.cx, s.cy);
          T h2 = dub.shortest(s.pose, goal_node.pose);
          s.f += stl_max(h1, h2);
          s.prev = cur;
#ifdef ORC_OUTER_STATS
          outer_ins_stat(s);
#endif
          op3.insert(s);
        }
      }
    }
    st.pop_digest = dig;
    st.closed_size = (long long)cl3.size();
    uint64_t cd = 0;
#ifndef ORC_LEAN
    for (const auto& n : cl3)
      cd += mix64(((uint64_t)(uint32_t)n.cx << 40) | ((uint64_t)(uint32_t)n.cy << 16) | (uint64_t)(uint32_t)n.bin);
#endif
    st.closed_digest = cd;
    st.via_shot = shot_ok ? 1 : 0;
    if (st.status != 0) out = {std::numeric_limits<T>::max(), false};
    return out;
  }
  // HybridAStar::find_path (HybridAStar.cpp:68-88) incl. Grid3D::set_start_node (127-160)
  // and reconstruct_path (208-262).  Appends to empty path/curv vectors.
  std::pair<T, bool> find_path(T vel, const P3<T>& start, std::vector<P3<T>>& path, std::vector<T>& curv) {
    st = hastar_stats{};
    P3<T> rel = rot3<T>(P3<T>{start.x - goal3.x, start.y - goal3.y, start.h}, grid_heading);
    P3<T> pose{rel.x + n45 * res, rel.y + n2 * res, rel.h};
    int i = static_cast<int>(pose.x / res), j = static_cast<int>(pose.y / res);
    N3<T> s{};
    if (inside(i, j)) {
      nm_f[(size_t)i * N + j] = nm_h[(size_t)i * N + j];
      s.pose = pose;
      s.cx = i;
      s.cy = j;
    } else {
      nm_f[0] = nm_h[0];
      s.pose = {0, 0, 0};
      s.cx = 0;
      s.cy = 0;
    }
    s.ci = mv.nsteer / 2;
    s.bin = heading_bin<T>(s.pose.h, mv.prec);
    s.vmin = vel * vel;
    s.f = std::numeric_limits<T>::max();
    s.prev = nullptr;
    auto res_pair = search(s);
    if (res_pair.second) {
      const P3<T> gg = goal_node.pose;
      curv.push_back(static_cast<T>(0));
      if (shot_ok) {
        size_t D = shot_path.size();
        path.resize(D);
        curv.resize(D + 1);
        for (size_t k = 0; k < D; ++k) {
          size_t q = D - k - 1;
          P3<T> p = rot3<T>(P3<T>{shot_path[q].x - gg.x, shot_path[q].y - gg.y, shot_path[q].h}, -grid_heading);
          p.x += goal3.x;
          p.y += goal3.y;
          path[k] = p;
          curv[k + 1] = shot_curv[q];
        }
      }
      for (const N3<T>* n = &terminal; n; n = n->prev) {
        P3<T> p = rot3<T>(P3<T>{n->pose.x - gg.x, n->pose.y - gg.y, n->pose.h}, -grid_heading);
        p.x += goal3.x;
        p.y += goal3.y;
        path.push_back(p);
        curv.push_back(mv.curv_abs[n->ci]);
      }
      curv.pop_back();
    }
    return res_pair;
  }
};

}  // namespace orc

// =================================================================== C interface
using OP = orc::Planner<float>;

extern "C" {

void* orc_create(const hastar_params* p) { return new OP(*p); }
void orc_destroy(void* h) { delete static_cast<OP*>(h); }
void orc_update_goal(void* h, const float g[3], const float s[3]) {
  static_cast<OP*>(h)->update_goal({g[0], g[1], g[2]}, {s[0], s[1], s[2]});
}
void orc_reset(void* h) { static_cast<OP*>(h)->reset(); }
void orc_update_boxes(void* h, const float* b, const float* c, int n, float r) {
  static_cast<OP*>(h)->boxes(b, c, n, r);
}
void orc_update_lines(void* h, const float* l, const float* c, int n, float w) {
  static_cast<OP*>(h)->lines(l, c, n, w);
}
void orc_decay(void* h) { static_cast<OP*>(h)->decay(); }
void orc_get_obstacles(void* h, float* out) {
  auto* P = static_cast<OP*>(h);
  std::memcpy(out, P->occ.data(), P->occ.size() * sizeof(float));
}
// The backward grid-distance field of csrc/hastar_field.hip (include/hastar.h:
// hastar_heuristic_field), restated as a float Dijkstra from the goal cell (n45, n2): field(v) =
// min over neighbours u that can be expanded (the goal, or log-odds < thr) of field(u) + the
// move's cost (act_cost of Grid2D.cpp:22-40's axis / diagonal moves), +inf where nothing reaches.
// A settled value never falls again (costs > 0, float addition monotone), so this is the least
// solution of those equations, which is their only one.
void orc_heuristic_field(void* h, float* out) {
  auto* P = static_cast<OP*>(h);
  const int N = P->N;
  const size_t NN = (size_t)N * N;
  const float inf = std::numeric_limits<float>::infinity();
  std::vector<float> d(NN, inf);
  std::vector<uint8_t> done(NN, 0);
  using E = std::pair<float, size_t>;
  std::priority_queue<E, std::vector<E>, std::greater<E>> q;
  const size_t g = (size_t)P->n45 * N + P->n2;
  d[g] = 0.0f;
  q.push({0.0f, g});
  while (!q.empty()) {
    const auto [du, u] = q.top();
    q.pop();
    if (done[u] || du != d[u]) continue;
    done[u] = 1;
    if (!(u == g || P->occ[u] < P->thr)) continue;  // reached, but cannot be expanded
    const int ui = (int)(u / N), uj = (int)(u % N);
    for (size_t k = 0; k < P->act_dx.size(); ++k) {
      const int vi = ui + P->act_dx[k], vj = uj + P->act_dy[k];
      if (vi < 0 || vi >= N || vj < 0 || vj >= N) continue;
      const size_t v = (size_t)vi * N + vj;
      const float c = du + P->act_cost[k];
      if (c < d[v]) {
        d[v] = c;
        q.push({c, v});
      }
    }
  }
  std::memcpy(out, d.data(), NN * sizeof(float));
}
// test hook: overwrite the log-odds map (arbitrary values exercise the relocation's winners)
void orc_set_obstacles(void* h, const float* in) {
  auto* P = static_cast<OP*>(h);
  std::memcpy(P->occ.data(), in, P->occ.size() * sizeof(float));
}
void orc_get_memo(void* h, float* f_out, unsigned char* visited_out) {
  auto* P = static_cast<OP*>(h);
  std::memcpy(f_out, P->nm_f.data(), P->nm_f.size() * sizeof(float));
  std::memcpy(visited_out, P->visited.data(), P->visited.size());
}
int orc_apf_count(void* h) { return (int)static_cast<OP*>(h)->apf.size(); }
void orc_get_apf(void* h, float* out) {
  auto* P = static_cast<OP*>(h);
  for (size_t k = 0; k < P->apf.size(); ++k) {
    out[3 * k] = P->apf[k].x;
    out[3 * k + 1] = P->apf[k].y;
    out[3 * k + 2] = P->apf[k].r;
  }
}
// Returns 0 or HASTAR_ENOSPC (then *len = required length).
int orc_find_path(void* h, float vel, const float start[3], float* xyh, float* curv, int cap, int* len,
                  float* cost, int* ok, hastar_stats* stats, double* wall_ms) {
  auto* P = static_cast<OP*>(h);
  std::vector<orc::P3<float>> path;
  std::vector<float> cv;
  auto t0 = std::chrono::steady_clock::now();
  auto r = P->find_path(vel, {start[0], start[1], start[2]}, path, cv);
  auto t1 = std::chrono::steady_clock::now();
  if (wall_ms) *wall_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  *cost = r.first;
  *ok = r.second ? 1 : 0;
  if (stats) *stats = P->st;
  *len = (int)path.size();
  if ((int)path.size() > cap) return HASTAR_ENOSPC;
  for (size_t k = 0; k < path.size(); ++k) {
    xyh[3 * k] = path[k].x;
    xyh[3 * k + 1] = path[k].y;
    xyh[3 * k + 2] = path[k].h;
    curv[k] = cv[k];
  }
  return 0;
}
// Closed-set keys (cx, cy, bin) of the last search, sorted; returns the count.
int orc_closed_keys(void* h, int* out, int cap) {
  auto* P = static_cast<OP*>(h);
  std::vector<long long> k;
  for (const auto& n : P->cl3) k.push_back(((long long)n.cx << 40) | ((long long)n.cy << 16) | n.bin);
  std::sort(k.begin(), k.end());
  int n = (int)k.size();
  for (int i = 0; i < n && i < cap; ++i) {
    out[3 * i] = (int)(k[i] >> 40);
    out[3 * i + 1] = (int)((k[i] >> 16) & 0xffffff);
    out[3 * i + 2] = (int)(k[i] & 0xffff);
  }
  return n;
}

// ---- unit-level hooks (the GPU library exposes the same operations as test kernels)
// Motion-primitive tables: off (nsteer x (bins+1) x 2), dth, cost, curv_abs; returns precision.
float orc_motion_tables(void* h, float* off, float* dth, float* cost, float* curv_abs) {
  auto* P = static_cast<OP*>(h);
  const auto& m = P->mv;
  for (size_t k = 0; k < m.off.size(); ++k) {
    off[2 * k] = m.off[k].x;
    off[2 * k + 1] = m.off[k].y;
  }
  for (int i = 0; i < m.nsteer; ++i) {
    dth[i] = m.dth[i];
    cost[i] = m.cost[i];
    curv_abs[i] = m.curv_abs[i];
  }
  return m.prec;
}
float orc_min_radius(void* h) { return static_cast<OP*>(h)->dub.r; }
// APF field of n poses (xyh) against the planner's current obstacle list.
void orc_field(void* h, const float* xyh, int n, float* out) {
  auto* P = static_cast<OP*>(h);
  for (int k = 0; k < n; ++k) out[k] = P->field({xyh[3 * k], xyh[3 * k + 1], xyh[3 * k + 2]});
}
// Dubins shortest length of n start poses to one goal pose (float).
void orc_dubins_len(float r_min, float step, const float* starts, int n, const float goal[3], float* out,
                    int* word) {
  orc::DubinsCSC<float> d(r_min, step);
  for (int k = 0; k < n; ++k) {
    out[k] = d.shortest({starts[3 * k], starts[3 * k + 1], starts[3 * k + 2]}, {goal[0], goal[1], goal[2]});
    if (word) word[k] = d.word;
  }
}
// Dubins sampled path (double, golden vector utils/dubins_paths.py:6).
int orc_dubins_path_d(double r_min, double step, const double s[3], const double g[3], double* xyh, int cap,
                      double* length, int* word) {
  orc::DubinsCSC<double> d(r_min, step);
  std::vector<orc::P3<double>> p;
  std::vector<double> c;
  auto r = d.path({s[0], s[1], s[2]}, {g[0], g[1], g[2]}, p, c);
  *length = r.first;
  *word = d.word;
  int n = (int)p.size();
  for (int k = 0; k < n && k < cap; ++k) {
    xyh[3 * k] = p[k].x;
    xyh[3 * k + 1] = p[k].y;
    xyh[3 * k + 2] = p[k].h;
  }
  return n;
}
// Dubins sampled path (float) for the shot kernel parity test.
int orc_dubins_path_f(float r_min, float step, const float s[3], const float g[3], float* xyh, float* curv,
                      int cap, float* length, int* first_arc_gt_90) {
  orc::DubinsCSC<float> d(r_min, step);
  std::vector<orc::P3<float>> p;
  std::vector<float> c;
  auto r = d.path({s[0], s[1], s[2]}, {g[0], g[1], g[2]}, p, c);
  *length = r.first;
  *first_arc_gt_90 = r.second ? 1 : 0;
  int n = (int)p.size();
  for (int k = 0; k < n && k < cap; ++k) {
    xyh[3 * k] = p[k].x;
    xyh[3 * k + 1] = p[k].y;
    xyh[3 * k + 2] = p[k].h;
    curv[k] = c[k];
  }
  return n;
}
// VehicleModel<double>::simulate_action chain (golden vector utils/vehicle_mode.py:12;
// VehicleModel.cpp:108-136; inputs of utils/vehicle_dubins/test_vehicle_dubins.cpp:61-67).
int orc_vehicle_chain_d(double ts, double a_lat, double wheelbase, double rear_to_cg, int bins, int na,
                        const double* steer, const double* w, int nsteer, double vmin0, int ci0,
                        const int* actions, int nact, double* xy_out) {
  std::vector<double> sv(steer, steer + nsteer), wv(w, w + nsteer);
  orc::Motion<double> m(ts, a_lat, wheelbase, rear_to_cg, bins, na, sv, wv);
  double x = 0, y = 0, h = 0, vmin = vmin0;
  int bin = orc::heading_bin<double>(0.0, 5.0 * M_PI / 180.0);
  (void)ci0;
  xy_out[0] = x;
  xy_out[1] = y;
  int n = 1;
  for (int k = 0; k < nact; ++k) {
    int a = actions[k];
    double vm = 0;
    if (vmin > 1.0) {
      double lat = vmin * m.curv_abs[a];
      if (lat > m.a_lat) break;
      double al = std::sqrt(1.0 - ((lat * lat) / m.a_lat2));
      vm = vmin - 2 * al * m.ts;
    }
    const auto& o = m.offset(a, bin);
    x = x + o.x;
    y = y + o.y;
    h = orc::wrap_pi<double>(h + m.dth[a]);
    bin = orc::heading_bin<double>(h, m.prec);
    vmin = vm;
    xy_out[2 * n] = x;
    xy_out[2 * n + 1] = y;
    ++n;
  }
  return n;
}

// VelocityGenerator<float>::generate_velocity_profile (VelocityGenerator.cpp:19-84), restated
// with the reference's own containers and expression types (T = float; `1.0 - x` promotes
// to double as in the reference).  prm = {max_velocity, coast_velocity, max_lat_acc,
// max_long_acc, max_long_dec}; xyh is goal -> start, 3 floats per point.  Returns feasible.
int orc_velocity_profile(const float prm[5], float vel_init, float max_velocity_curr, const float* xyh,
                         const float* curv, int n, int coast_to_goal, int stop_at_goal, float* out) {
  using T = float;
  const T vmax_param = prm[0], vcoast = prm[1], a_lat = prm[2], a_lat2 = prm[2] * prm[2], a_acc = prm[3],
          a_dec = prm[4];
  struct P3 { T _x, _y, _h; };
  std::vector<P3> path((size_t)n);
  for (int i = 0; i < n; ++i) path[i] = {xyh[3 * i], xyh[3 * i + 1], xyh[3 * i + 2]};
  std::vector<T> curvature(curv, curv + n);
  T max_velocity = coast_to_goal ? vcoast : vmax_param;
  max_velocity = std::min(max_velocity, max_velocity_curr);
  const T max_velocity_sqr = max_velocity * max_velocity;
  const std::size_t path_size = path.size();
  std::vector<T> velocity(path_size), velocity_sqr(path_size);
  velocity_sqr[0] = vel_init * vel_init;
  T max_velocity_sqr_curr = velocity_sqr[0];
  for (std::size_t i = 0; i + 1 < path_size; i++) {  // initial profile (VelocityGenerator.cpp:35-48)
    const std::size_t pi = path_size - i - 1;
    T step = std::hypot(path[pi - 1]._x - path[pi]._x, path[pi - 1]._y - path[pi]._y);
    T lat = velocity_sqr[i] * curvature[pi];
    T rem = a_dec * std::sqrt(1.0 - (lat * lat) / a_lat2);
    max_velocity_sqr_curr = std::max(max_velocity_sqr_curr - 2 * rem * step, max_velocity_sqr);
    velocity_sqr[i + 1] = (curvature[pi - 1] != 0) ? std::min(a_lat / curvature[pi - 1], max_velocity_sqr_curr)
                                                   : max_velocity_sqr_curr;
  }
  velocity_sqr[path_size - 1] = stop_at_goal ? 0 : velocity_sqr[path_size - 1];  // (51)
  for (std::size_t i = 0; i + 1 < path_size; i++) {  // forward pass (54-63)
    const std::size_t pi = path_size - i - 1;
    T step = std::hypot(path[pi - 1]._x - path[pi]._x, path[pi - 1]._y - path[pi]._y);
    T lat = velocity_sqr[i] * curvature[pi];
    T rem = a_acc * std::sqrt(1.0 - (lat * lat) / a_lat2);
    velocity_sqr[i + 1] = std::min(velocity_sqr[i] + 2 * rem * step, velocity_sqr[i + 1]);
  }
  for (std::size_t i = path_size - 1; i > 0; i--) {  // backward pass (66-76)
    const std::size_t pi = path_size - i - 1;
    T step = std::hypot(path[pi + 1]._x - path[pi]._x, path[pi + 1]._y - path[pi]._y);
    T lat = velocity_sqr[i] * curvature[pi];
    T rem = a_dec * std::sqrt(1.0 - (lat * lat) / a_lat2);
    velocity_sqr[i - 1] = std::min(velocity_sqr[i] + 2 * rem * step, velocity_sqr[i - 1]);
    velocity[i - 1] = std::sqrt(velocity_sqr[i - 1]);
  }
  velocity[path_size - 1] = std::sqrt(velocity_sqr[path_size - 1]);  // (79-82)
  for (int i = 0; i < n; ++i) out[i] = velocity[i];
  constexpr T tol = static_cast<T>(0.25);
  return vel_init < (velocity[0] + tol) ? 1 : 0;
}

}  // extern "C"

// glibc reference values for the GPU libm-port test (fn numbering of hastar_test_math).
extern "C" void orc_libm(int fn, const float* a, const float* b, float* out, int n) {
  for (int i = 0; i < n; ++i) {
    float v = 0.0f;
    switch (fn) {
      case 0: v = std::sin(a[i]); break;
      case 1: v = std::cos(a[i]); break;
      case 2: v = std::atan2(a[i], b[i]); break;
      case 3: v = std::acos(a[i]); break;
      case 4: v = std::hypot(a[i], b[i]); break;
      case 5: v = orc::wrap_pi<float>(a[i]); break;
      case 6: v = (float)orc::heading_bin<float>(a[i], b[i]); break;
      default: v = std::atan(a[i]); break;
    }
    out[i] = v;
  }
}

extern "C" void orc_set_max_pops(long long n) { orc::g_max_pops = n; }

// The stand-alone AStar<float> (utils/astar/test_astar.cpp) on a planner's plain Grid2D.
extern "C" void orc_grid2d_goal(void* h, const float g[2], const float s[2]) {
  static_cast<OP*>(h)->goal_2d({g[0], g[1]}, {s[0], s[1]});
}
extern "C" void orc_grid2d_start(void* h, const float s[2], int cell[2]) {
  auto c = static_cast<OP*>(h)->start_2d({s[0], s[1]});
  cell[0] = c.first;
  cell[1] = c.second;
}
extern "C" float orc_astar_cost(void* h, int i, int j) { return static_cast<OP*>(h)->holonomic(i, j); }
// AStar::find_path(goal, start, path / cost_only): returns the cost; *n path points after the goal
extern "C" float orc_astar_find_path(void* h, const float g[2], const float s[2], int cost_only, float* xy, int cap,
                                     int* n) {
  auto* P = static_cast<OP*>(h);
  P->goal_2d({g[0], g[1]}, {s[0], s[1]});
  auto c = P->start_2d({s[0], s[1]});
  const float cost = P->a_star(c.first, c.second, cost_only != 0);
  std::vector<orc::P2<float>> pts;
  if (!cost_only && cost < std::numeric_limits<float>::max()) P->path_2d({g[0], g[1]}, pts);
  *n = (int)pts.size();
  for (int k = 0; k < (int)pts.size() && k < cap; ++k) {
    xy[2 * k] = pts[k].x;
    xy[2 * k + 1] = pts[k].y;
  }
  return cost;
}
// Grid3D::get_neighbors (Grid3D.cpp:47-74) of one node: out n x {x, y, h, g, vmin, ci, bin}
// (ci / bin as float-encoded ints), cells n x 2; returns the count, *neglect the flag
extern "C" int orc_grid3d_neighbors(void* h, const float nd[5], int ci, int bin, float* out, int* cells, int cap,
                                    int* neglect) {
  auto* P = static_cast<OP*>(h);
  orc::N3<float> n{};
  n.pose = {nd[0], nd[1], nd[2]};
  n.g = nd[3];
  n.vmin = nd[4];
  n.ci = ci;
  n.bin = bin;
  std::vector<orc::N3<float>> nb;
  *neglect = P->expand(n, nb) ? 1 : 0;
  for (int k = 0; k < (int)nb.size() && k < cap; ++k) {
    float* o = out + 7 * k;
    o[0] = nb[k].pose.x;
    o[1] = nb[k].pose.y;
    o[2] = nb[k].pose.h;
    o[3] = nb[k].g;
    o[4] = nb[k].vmin;
    std::memcpy(&o[5], &nb[k].ci, 4);
    std::memcpy(&o[6], &nb[k].bin, 4);
    cells[2 * k] = nb[k].cx;
    cells[2 * k + 1] = nb[k].cy;
  }
  return (int)nb.size();
}
// Grid3D::check_path (Grid3D.cpp:78-93)
extern "C" int orc_check_path(void* h, const float* xyh, int n) {
  std::vector<orc::P3<float>> p(n);
  for (int k = 0; k < n; ++k) p[k] = {xyh[3 * k], xyh[3 * k + 1], xyh[3 * k + 2]};
  return static_cast<OP*>(h)->free_path(p) ? 1 : 0;
}

// VehicleModel<float>::simulate_action over an action list from the harness start node
extern "C" int orc_vehicle_chain_f(float ts, float a_lat, float wheelbase, float rear_to_cg, int bins, int na,
                                   const float* steer, const float* w, int nsteer, float vmin0, const int* actions,
                                   int nact, float* xy_out) {
  std::vector<float> sv(steer, steer + nsteer), wv(w, w + nsteer);
  orc::Motion<float> m(ts, a_lat, wheelbase, rear_to_cg, bins, na, sv, wv);
  float x = 0, y = 0, h = 0, vmin = vmin0;
  int bin = orc::heading_bin<float>(0.0f, (float)(5.0 * M_PI / 180.0));
  xy_out[0] = x;
  xy_out[1] = y;
  int n = 1;
  for (int k = 0; k < nact; ++k) {
    int a = actions[k];
    float vm = 0;
    if (vmin > 1.0) {
      float lat = vmin * m.curv_abs[a];
      if (lat > m.a_lat) break;
      float al = std::sqrt(1.0 - ((lat * lat) / m.a_lat2));
      vm = vmin - 2 * al * m.ts;
    }
    const auto& o = m.offset(a, bin);
    x = x + o.x;
    y = y + o.y;
    h = orc::wrap_pi<float>(h + m.dth[a]);
    bin = orc::heading_bin<float>(h, m.prec);
    vmin = vm;
    xy_out[2 * n] = x;
    xy_out[2 * n + 1] = y;
    ++n;
  }
  return n;
}

// CPU baseline (bench.py cpu_baseline): `threads` std::threads, each taking whole planners
// from a shared counter (one private planner per thread at a time, as BASELINE.md's plan
// says), and running `replans` x (reset + find_path) on it, timed around find_path only
// (test_hybrid_astar.cpp:123-126).  out[0] = total pops, out[1] = wall seconds of the
// parallel region, out[2] = sum of find_path seconds (for the mean plan latency), out[3] =
// plans; per_plan_ms (n x replans, may be null) receives each plan's latency; last_digest /
// last_cost / last_ok (n, may be null) the last replan's pop digest and result.
extern "C" void orc_run_batch_threads(void* const* hs, int n, const float* vel, const float* starts, int replans,
                                      int threads, double* out, double* per_plan_ms, unsigned long long* last_digest,
                                      float* last_cost, int* last_ok) {
  std::atomic<int> next{0};
  std::atomic<long long> pops{0};
  std::vector<double> tsum((size_t)std::max(threads, 1), 0.0);
  auto work = [&](int t) {
    for (int i = next++; i < n; i = next++) {
      auto* P = static_cast<OP*>(hs[i]);
      for (int r = 0; r < replans; ++r) {
        P->reset();
        std::vector<orc::P3<float>> path;
        std::vector<float> cv;
        const auto t0 = std::chrono::steady_clock::now();
        const auto res = P->find_path(vel[i], {starts[3 * i], starts[3 * i + 1], starts[3 * i + 2]}, path, cv);
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        tsum[t] += s;
        if (per_plan_ms) per_plan_ms[(size_t)i * replans + r] = s * 1e3;
        pops += P->st.pops;
        if (r == replans - 1) {
          if (last_digest) last_digest[i] = P->st.pop_digest;
          if (last_cost) last_cost[i] = res.first;
          if (last_ok) last_ok[i] = res.second ? 1 : 0;
        }
      }
    }
  };
  const auto w0 = std::chrono::steady_clock::now();
  std::vector<std::thread> pool;
  for (int t = 0; t < std::max(threads, 1); ++t) pool.emplace_back(work, t);
  for (auto& th : pool) th.join();
  out[1] = std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();
  out[0] = (double)pops.load();
  out[2] = std::accumulate(tsum.begin(), tsum.end(), 0.0);
  out[3] = (double)n * replans;
}

#ifdef ORC_BRANCH_STATS
extern "C" void orc_branch_stats(long long* out) {
  for (int q = 0; q < 8; ++q) out[q] = orc::g_br[q], orc::g_br[q] = 0;
}
#endif
#ifdef ORC_OUTER_STATS
extern "C" void orc_outer_stats(long long* out) {
  for (int q = 0; q < 16; ++q) out[q] = orc::g_oshape[q], orc::g_oshape[q] = 0;
}
#endif
#ifdef ORC_SHAPE_STATS
extern "C" void orc_shape_stats(long long* out) {
  for (int q = 0; q < 16; ++q) out[q] = orc::g_shape[q], orc::g_shape[q] = 0;
}
#endif

// =========================================== HybridAStar<double> / VelocityGenerator<double>
// The reference's second instantiation (HybridAStar.cpp:285-286, VelocityGenerator.cpp:88-89),
// the checker of the device double planner (include/hastar_f64.h): the same templated
// restatement as above with T = double, glibc double libm.
using OP64 = orc::Planner<double>;

extern "C" {

void* orc64_create(const hastar_params_f64* p) { return new OP64(*p); }
void orc64_destroy(void* h) { delete static_cast<OP64*>(h); }
void orc64_update_goal(void* h, const double g[3], const double s[3]) {
  static_cast<OP64*>(h)->update_goal({g[0], g[1], g[2]}, {s[0], s[1], s[2]});
}
void orc64_reset(void* h) { static_cast<OP64*>(h)->reset(); }
void orc64_update_boxes(void* h, const double* b, const double* c, int n, double r) { static_cast<OP64*>(h)->boxes(b, c, n, r); }
void orc64_update_lines(void* h, const double* l, const double* c, int n, double w) { static_cast<OP64*>(h)->lines(l, c, n, w); }
void orc64_decay(void* h) { static_cast<OP64*>(h)->decay(); }
void orc64_get_obstacles(void* h, double* out) {
  auto* P = static_cast<OP64*>(h);
  std::memcpy(out, P->occ.data(), P->occ.size() * sizeof(double));
}
void orc64_get_memo(void* h, double* f_out, unsigned char* visited_out) {
  auto* P = static_cast<OP64*>(h);
  std::memcpy(f_out, P->nm_f.data(), P->nm_f.size() * sizeof(double));
  std::memcpy(visited_out, P->visited.data(), P->visited.size());
}
int orc64_find_path(void* h, double vel, const double start[3], double* xyh, double* curv, int cap, int* len,
                    double* cost, int* ok, hastar_stats* stats, double* wall_ms) {
  auto* P = static_cast<OP64*>(h);
  std::vector<orc::P3<double>> path;
  std::vector<double> cv;
  auto t0 = std::chrono::steady_clock::now();
  auto r = P->find_path(vel, {start[0], start[1], start[2]}, path, cv);
  auto t1 = std::chrono::steady_clock::now();
  if (wall_ms) *wall_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  *cost = r.first;
  *ok = r.second ? 1 : 0;
  if (stats) *stats = P->st;
  *len = (int)path.size();
  if ((int)path.size() > cap) return HASTAR_ENOSPC;
  for (size_t k = 0; k < path.size(); ++k) {
    xyh[3 * k] = path[k].x;
    xyh[3 * k + 1] = path[k].y;
    xyh[3 * k + 2] = path[k].h;
    curv[k] = cv[k];
  }
  return 0;
}
int orc64_closed_keys(void* h, int* out, int cap) {
  auto* P = static_cast<OP64*>(h);
  std::vector<long long> k;
  for (const auto& n : P->cl3) k.push_back(((long long)n.cx << 40) | ((long long)n.cy << 16) | n.bin);
  std::sort(k.begin(), k.end());
  int n = (int)k.size();
  for (int i = 0; i < n && i < cap; ++i) {
    out[3 * i] = (int)(k[i] >> 40);
    out[3 * i + 1] = (int)((k[i] >> 16) & 0xffffff);
    out[3 * i + 2] = (int)(k[i] & 0xffff);
  }
  return n;
}

// VelocityGenerator<double>::generate_velocity_profile (VelocityGenerator.cpp:19-84), T = double
int orc64_velocity_profile(const double prm[5], double vel_init, double max_velocity_curr, const double* xyh,
                           const double* curv, int n, int coast_to_goal, int stop_at_goal, double* out) {
  using T = double;
  const T vmax_param = prm[0], vcoast = prm[1], a_lat = prm[2], a_lat2 = prm[2] * prm[2], a_acc = prm[3],
          a_dec = prm[4];
  struct P3 { T _x, _y, _h; };
  std::vector<P3> path((size_t)n);
  for (int i = 0; i < n; ++i) path[i] = {xyh[3 * i], xyh[3 * i + 1], xyh[3 * i + 2]};
  std::vector<T> curvature(curv, curv + n);
  T max_velocity = coast_to_goal ? vcoast : vmax_param;
  max_velocity = std::min(max_velocity, max_velocity_curr);
  const T max_velocity_sqr = max_velocity * max_velocity;
  const std::size_t path_size = path.size();
  std::vector<T> velocity(path_size), velocity_sqr(path_size);
  velocity_sqr[0] = vel_init * vel_init;
  T max_velocity_sqr_curr = velocity_sqr[0];
  for (std::size_t i = 0; i + 1 < path_size; i++) {
    const std::size_t pi = path_size - i - 1;
    T step = std::hypot(path[pi - 1]._x - path[pi]._x, path[pi - 1]._y - path[pi]._y);
    T lat = velocity_sqr[i] * curvature[pi];
    T rem = a_dec * std::sqrt(1.0 - (lat * lat) / a_lat2);
    max_velocity_sqr_curr = std::max(max_velocity_sqr_curr - 2 * rem * step, max_velocity_sqr);
    velocity_sqr[i + 1] = (curvature[pi - 1] != 0) ? std::min(a_lat / curvature[pi - 1], max_velocity_sqr_curr)
                                                   : max_velocity_sqr_curr;
  }
  velocity_sqr[path_size - 1] = stop_at_goal ? 0 : velocity_sqr[path_size - 1];
  for (std::size_t i = 0; i + 1 < path_size; i++) {
    const std::size_t pi = path_size - i - 1;
    T step = std::hypot(path[pi - 1]._x - path[pi]._x, path[pi - 1]._y - path[pi]._y);
    T lat = velocity_sqr[i] * curvature[pi];
    T rem = a_acc * std::sqrt(1.0 - (lat * lat) / a_lat2);
    velocity_sqr[i + 1] = std::min(velocity_sqr[i] + 2 * rem * step, velocity_sqr[i + 1]);
  }
  for (std::size_t i = path_size - 1; i > 0; i--) {
    const std::size_t pi = path_size - i - 1;
    T step = std::hypot(path[pi + 1]._x - path[pi]._x, path[pi + 1]._y - path[pi]._y);
    T lat = velocity_sqr[i] * curvature[pi];
    T rem = a_dec * std::sqrt(1.0 - (lat * lat) / a_lat2);
    velocity_sqr[i - 1] = std::min(velocity_sqr[i] + 2 * rem * step, velocity_sqr[i - 1]);
    velocity[i - 1] = std::sqrt(velocity_sqr[i - 1]);
  }
  velocity[path_size - 1] = std::sqrt(velocity_sqr[path_size - 1]);
  for (int i = 0; i < n; ++i) out[i] = velocity[i];
  constexpr T tol = static_cast<T>(0.25);
  return vel_init < (velocity[0] + tol) ? 1 : 0;
}

}  // extern "C"
