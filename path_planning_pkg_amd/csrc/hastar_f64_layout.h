// hastar_f64_layout.h — device-resident state of one HybridAStar<double> planner
// (include/hastar_f64.h), shared by hastar_f64.hip and hastar_f64.cpp.
//
// Same organisation as the float planner (hastar_layout.h): flat, index-linked records in
// HBM, the open sets as libstdc++ RB trees over pool indices (rbtree_dev.h), the closed sets
// as generation-stamped tables.  The double planner is the reference's second
// instantiation (HybridAStar.cpp:285-286), used by LocalPlanner<double>
// (local_planner.cpp:378-500); it is not the benchmarked path, so each planner owns its
// search arena and one wavefront runs one search.
#pragma once
#include <stdint.h>

namespace hastar {

// std::set<Node3D<double>> node (HybridAStar.h:72): {key, l, r, p} + f in the first 24 B
struct alignas(16) Node3d {
  uint32_t key;  // (x, y, bin) packed as key3()
  int l, r, p;
  double f;
  int color, ci;
  double g, vmin, x, y, h;
  int prev, pad;  // closed-record index of the predecessor
};
static_assert(sizeof(Node3d) == 80, "Node3d layout");

// unordered_set<Node3D<double>> element (HybridAStar.h:73-74): a copy of the popped node
struct alignas(16) Closed3d {
  uint32_t key;
  int prev, ci, pad;
  double g, vmin, x, y, h, pad2;
};
static_assert(sizeof(Closed3d) == 64, "Closed3d layout");

// std::set<Node2D<double>> node (AStar.h:70); key = x << 16 | y
struct alignas(16) Node2d {
  uint32_t key;
  int l, r, p;
  double f, g;
  int color, prev;  // prev = cell index of the predecessor's closed record
  int pad0, pad1;
};
static_assert(sizeof(Node2d) == 48, "Node2d layout");

// per-cell closed record of the inner A* (unordered_set<Node2D<double>>, AStar.h:71-72):
// closed in the current inner search iff gen == the search's generation
struct alignas(16) Cell2d {
  uint32_t gen;
  int prev;
  double g;
};

// closed-set hash slot of the outer search: live iff gen == the search's generation
struct alignas(16) Slot3d {
  uint32_t key, gen;
  int idx, pad;
};

// arena growth requests (Result64::need): the search stops, the host restores the memo
// (node-map f and visited flags as they were before the search), grows the named arena 4x
// and runs the search again, so no arena size changes a result
constexpr int NEED_OUTER = 1;  // open3 / closed3
constexpr int NEED_INNER = 2;  // open2
constexpr int NEED_SHOT = 4;   // Dubins shot samples

struct Result64 {
  long long pops, successors, astar_pops, astar_searches, shots, closed_size;
  unsigned long long pop_digest, closed_digest;
  int ok, via_shot, need, path_len;
  double cost;
  int terminal, dubins_len, chain_len, pad;
};

struct Planner64Dev {
  // --- constants (Grid2D.cpp:7-62, VehicleModel.cpp:7-47, HybridAStar.cpp:7-24)
  int N, n2, n45, diag;
  int bins, nsteer, na, shot_interval;
  int shot_decay, n_apf, pad0, pad1;
  double res, thr, apf_rep, apf_ang;
  double ts, a_lat, a_lat2, prec;
  double r_min, step, ang_step, act_cost_axis;
  double act_cost_diag;
  // --- goal node (grid frame) and the grid -> world transform of reconstruct_path
  double goal_x, goal_y, goal_h;
  int goal_cx, goal_cy, goal_bin, pad2;
  double world_goal_x, world_goal_y, rot_c, rot_s, neg_heading;
  // --- start node of this search (Grid3D::set_start_node, Grid3D.cpp:127-160)
  double start_x, start_y, start_h, start_vmin;
  int start_cx, start_cy, start_bin, start_ci;
  // --- persistent planner state
  double* occ;          // N*N log-odds
  double* nm_f;         // N*N node-map f (A* memo value + stale f)
  uint32_t* visited;    // memo flags, bitmap
  double* apf;          // n_apf x {x, y, r}
  double* off;          // nsteer x (bins + 1) x {dx, dy}
  double* dth;
  double* act_cost;
  double* curv_abs;
  // --- search arena (owned by the planner)
  Node3d* open3;        int open3_cap;   int pad3;
  Closed3d* closed3;    int closed3_cap; int pad4;
  Slot3d* slots3;       uint32_t slots3_mask; int pad5;
  Node2d* open2;        int open2_cap;   int pad6;
  Cell2d* cell2;        // N*N
  uint32_t* gens;       // [0] outer closed-set generation, [1] inner closed generation
  double* dub_xyh;      double* dub_curv; int dub_cap; int pad7;
  int* chain;           // closed3_cap: terminal -> start chain (reconstruct)
  // --- output
  double* out_xyh;      double* out_curv; int out_cap; int pad8;
  Result64* result;
};

}  // namespace hastar
