/* hastar_f64.h — C ABI of the double-precision planner: the reference's
 * `planning::HybridAStar<double>` and `planning::VelocityGenerator<double>`.
 *
 * The reference instantiates both classes for double (lib/HybridAStar.cpp:285-286,
 * lib/VelocityGenerator.cpp:88-89), and its ROS node compiles a `LocalPlanner<double>`
 * specialization that constructs and calls them (src/local_planner.h:119-135,
 * src/local_planner.cpp:158-166, 378-379, 444, 451, 460).  The drop-in headers
 * include/path_planning_pkg/HybridAStar.h and VelocityGenerator.h implement those
 * specializations on the entry points below, so local_planner.cpp compiles and links
 * unchanged against libhastar_amd.so.
 *
 * The search runs on the GPU in f64 (csrc/hastar_f64.hip): one wavefront per planner with
 * the reference's exact open/closed-set semantics.  Per-call scalar preparation (grid frame,
 * motion tables, raster parameters, start node) is done on the host with the reference's
 * double arithmetic and glibc libm; the kernels' APF field, Dubins lengths and shot sampling
 * use ports of glibc 2.35's own sin/cos/atan2/acos/hypot (csrc/hastar_libm64.h: bit for bit
 * the host libm on every sampled argument), so results equal the reference's bit for bit, as
 * the float planner's do: success, cost, statistics, closed set, path and memo
 * (tests/test_gpu_f64.py; the oracle is the reference's algorithm instantiated for double,
 * parity with the reference itself being pinned by its Dubins/VehicleModel double vectors
 * only).  There is no CPU fallback.
 *
 * Status codes, statistics and the path output format are those of include/hastar.h.
 */
#ifndef PATH_PLANNING_PKG_AMD_HASTAR_F64_H
#define PATH_PLANNING_PKG_AMD_HASTAR_F64_H

#include "hastar.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The 20 constructor arguments of HybridAStar<double>::HybridAStar (HybridAStar.h:33-38),
 * in the reference's order and meaning, as doubles; arena sizes as in hastar_params
 * (0 = default).  An arena that fills up is replaced by a 4x larger one and the search
 * re-run from the same memo state, so these are not limits. */
typedef struct hastar_params_f64 {
  int dubins_shot_interval;
  int dubins_shot_interval_decay;
  double grid_resolution;
  double obstacle_threshold;
  double obstacle_prob_min;
  double obstacle_prob_max;
  double obstacle_prob_free;
  int grid_size;
  int grid_2d_allow_diag_moves;
  double step_size;
  double max_lat_acc;
  double max_long_dec;
  double wheelbase;
  double rear_to_cg;
  double apf_rep_constant;
  double apf_active_angle;  /* radians */
  int num_angle_bins;
  int num_actions;
  int num_steering;
  const double* steering;   /* radians */
  const double* curvature_weights;
  int max_pops;             /* initial outer arena, in pops [65536] */
  int max_astar_nodes;      /* initial inner open-tree arena [min(N*N + 16, 65536)] */
  int max_dubins_samples;   /* initial shot sample arena [from N] */
} hastar_params_f64;

typedef struct hastar64_s* hastar64_handle;

/* HybridAStar<double>(...) (HybridAStar.cpp:7-24). */
int hastar64_create(const hastar_params_f64* params, int device, hastar64_handle* out);
int hastar64_destroy(hastar64_handle h);
/* update_goal(goal, start) (HybridAStar.cpp:55-59) */
int hastar64_update_goal(hastar64_handle h, const double goal[3], const double start[3]);
/* reset() (HybridAStar.cpp:49-52) */
int hastar64_reset(hastar64_handle h);
/* update_obstacles(obstacles, confidence, apf_added_radius) (HybridAStar.cpp:29-33):
 * boxes = n x {center_x, center_y, dimension_x, dimension_y} */
int hastar64_update_boxes(hastar64_handle h, const double* boxes, const double* confidence, int n,
                          double apf_added_radius);
/* update_obstacles(lines, confidence, line_width) (HybridAStar.cpp:36-40): n x {x1, y1, x2, y2} */
int hastar64_update_lines(hastar64_handle h, const double* lines, const double* confidence, int n,
                          double line_width);
/* update_obstacles() (HybridAStar.cpp:43-46) */
int hastar64_decay(hastar64_handle h);
/* get_obstacles() (HybridAStar.h:48): N x N log-odds map, row i = x cell */
int hastar64_get_obstacles(hastar64_handle h, double* out);
/* find_path(vel_init, start, path, curvature) (HybridAStar.cpp:68-88); same output
 * contract as hastar_find_path (goal first, start last; HASTAR_ENOSPC keeps the path for
 * hastar64_copy_path). */
int hastar64_find_path(hastar64_handle h, double vel_init, const double start[3], double* xyh, double* curv,
                       int cap, int* len, double* cost, int* ok, hastar_stats* stats);
int hastar64_copy_path(hastar64_handle h, double* xyh, double* curv, int cap, int* len);
int hastar64_grid_size(hastar64_handle h);

/* VelocityGenerator<double>::generate_velocity_profile (VelocityGenerator.cpp:19-84) of n
 * paths; arguments as hastar_velocity_profile_batch, in double. */
typedef struct hastar_velocity_params_f64 {
  double max_velocity;
  double coast_velocity;
  double max_lat_acc;
  double max_long_acc;
  double max_long_dec;
} hastar_velocity_params_f64;
int hastar_velocity_profile_batch_f64(int device, const hastar_velocity_params_f64* vp, int n,
                                      const long long* offsets, const double* xyh, const double* curv,
                                      const double* vel_init, const double* max_velocity_curr,
                                      const unsigned char* flags, double* velocity, unsigned char* feasible);

/* ---- test hooks ---- */
/* the A* memo after the last call: node-map f (N*N) and visited flags (N*N bytes) */
int hastar64_debug_memo(hastar64_handle h, double* f_out, unsigned char* visited_out);
/* closed-set keys (cx, cy, bin) of the last search, sorted; returns the count (or < 0) */
int hastar64_debug_closed_keys(hastar64_handle h, int* out, int cap);
/* arena state: {open3 capacity in nodes, inner open-tree capacity, shot samples, re-runs of the last find_path} */
int hastar64_debug_arena(hastar64_handle h, long long* out4);

#ifdef __cplusplus
}
#endif

#endif /* PATH_PLANNING_PKG_AMD_HASTAR_F64_H */
