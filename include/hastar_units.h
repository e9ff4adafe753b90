/* hastar_units.h — C ABI of the unit-level classes of the reference's public headers
 * (reference include/path_planning_pkg/{Dubins,VehicleModel,AStar,Grid2D,Grid3D}.h,
 * CMakeLists.txt:125 puts them on the include path; the utils harnesses use them directly).
 * The drop-in headers include/path_planning_pkg/ headers implement those classes on these calls.
 *
 * Every call runs on the HIP device `device` (gfx950); there is no CPU path: without a
 * device each call returns HASTAR_EDEVICE.  Host buffers in and out.  float is bit-exact
 * with the reference (glibc float libm ports); double too (ports of glibc 2.35's double
 * sin/cos/atan2/acos, csrc/hastar_libm64.h).
 */
#ifndef PATH_PLANNING_PKG_AMD_HASTAR_UNITS_H
#define PATH_PLANNING_PKG_AMD_HASTAR_UNITS_H

#include "hastar.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Last error message of the unit calls of this thread (static storage). */
const char* hastar_units_last_error(void);

/* Node3D<T> fields the vehicle model reads / writes (Node3D.h:17-24) */
typedef struct hastar_node3_f32 {
  float x, y, heading, g, vmin_sqr;
  int curvature_index, angle_bin;
} hastar_node3_f32;
typedef struct hastar_node3_f64 {
  double x, y, heading, g, vmin_sqr;
  int curvature_index, angle_bin;
} hastar_node3_f64;

/* ---- Dubins<T> (Dubins.h:21-60, Dubins.cpp) ----
 * get_shortest_path_length(start, goal[, centres]) for n start poses (n x 3) against one
 * goal pose: length[i], word[i] (0 RSR, 1 RSL, 2 LSR, 3 LSL = Dubins.h Path), and when
 * centres != NULL the 4 circle centres of pose i (start right, start left, goal right,
 * goal left; n x 8) as the 6-argument overload returns them (Dubins.cpp:76-87). */
int hastar_dubins_length_f32(int device, float r_min, int n, const float* starts, const float goal[3], float* length,
                             int* word, float* centres);
int hastar_dubins_length_f64(int device, double r_min, int n, const double* starts, const double goal[3],
                             double* length, int* word, double* centres);
/* get_shortest_path(start, goal, path, curvature) (Dubins.cpp:125-153): the sampled poses
 * (xyh: n x 3) and curvatures; *n = sample count (if it exceeds cap, -required and nothing
 * is written); *length = path length; *first_arc_gt_90 = the returned flag; *word. */
int hastar_dubins_path_f32(int device, float r_min, float step, const float start[3], const float goal[3], float* xyh,
                           float* curv, int cap, int* n, float* length, int* first_arc_gt_90, int* word);
int hastar_dubins_path_f64(int device, double r_min, double step, const double start[3], const double goal[3],
                           double* xyh, double* curv, int cap, int* n, double* length, int* first_arc_gt_90, int* word);

/* ---- VehicleModel<T> (VehicleModel.h:14-42, VehicleModel.cpp) ---- */
typedef struct hastar_vehicle_s* hastar_vehicle;
/* VehicleModel(ts, max_lat_acc, max_long_dec, wheelbase, rear_to_cg, num_angle_bins,
 * num_actions, steering, curvature_weights) (VehicleModel.cpp:7-47); the offset tables are
 * integrated at create time (calculate_offset, VehicleModel.cpp:147-164) and kept on the device. */
int hastar_vehicle_create_f32(int device, float ts, float max_lat_acc, float max_long_dec, float wheelbase,
                              float rear_to_cg, int num_angle_bins, int num_actions, int nsteer, const float* steering,
                              const float* curvature_weights, hastar_vehicle* out);
int hastar_vehicle_create_f64(int device, double ts, double max_lat_acc, double max_long_dec, double wheelbase,
                              double rear_to_cg, int num_angle_bins, int num_actions, int nsteer, const double* steering,
                              const double* curvature_weights, hastar_vehicle* out);
int hastar_vehicle_destroy(hastar_vehicle v);
/* get_precision(), get_default_action_index(), number of actions (steering angles) */
int hastar_vehicle_info(hastar_vehicle v, double* precision, int* default_action, int* nsteer);
/* get_abs_curvatures() (nsteer values of the handle's type: float* or double*) */
int hastar_vehicle_abs_curvatures(hastar_vehicle v, void* out);
/* get_neighbors(node, neighbors) of n nodes: node i's successors at out[i * max_per_node ...],
 * counts[i] of them; neglect[i] = the returned bool (VehicleModel.cpp:63-105). */
int hastar_vehicle_neighbors_f32(hastar_vehicle v, int n, const hastar_node3_f32* nodes, int max_per_node,
                                 hastar_node3_f32* out, int* counts, int* neglect);
int hastar_vehicle_neighbors_f64(hastar_vehicle v, int n, const hastar_node3_f64* nodes, int max_per_node,
                                 hastar_node3_f64* out, int* counts, int* neglect);
/* simulate_action(node, action_index) of n nodes (VehicleModel.cpp:108-136): ok[i] = the
 * returned bool, out[i] the new node (the input node when ok[i] = 0). */
int hastar_vehicle_simulate_f32(hastar_vehicle v, int n, const hastar_node3_f32* nodes, const int* actions,
                                hastar_node3_f32* out, int* ok);
int hastar_vehicle_simulate_f64(hastar_vehicle v, int n, const hastar_node3_f64* nodes, const int* actions,
                                hastar_node3_f64* out, int* ok);

/* ---- AStar<float> / Grid2D<float> (AStar.h:27-60, Grid2D.h:16-47) on a planner handle ----
 * The reference's stand-alone AStar owns a plain Grid2D (no STORE_GRID_AS_REFERENCE): a goal
 * change only re-orients the frame and the start cell rounds differently from Grid3D's.
 * Map updates, reset() and get_obstacles() are the handle's hastar_* calls. */
/* Grid2D::update_goal_heading(goal, start) (Grid2D.cpp:260-266): no relocation */
int hastar_grid2d_update_goal_heading(hastar_handle h, const float goal[2], const float start[2]);
/* Grid2D::set_start_node(start) (Grid2D.cpp:270-290): cell = the soft-reset start cell */
int hastar_grid2d_set_start_node(hastar_handle h, const float start[2], int cell[2]);
/* Grid2D::set_start_node_grid(i, j) (Grid2D.cpp:294-299) */
int hastar_grid2d_set_start_node_grid(hastar_handle h, int i, int j);
/* AStar::update_goal_node(goal_node) (AStar.cpp:24-28): the goal cell of later searches */
int hastar_astar_set_goal_cell(hastar_handle h, int i, int j);
/* Grid2D::get_node_total_cost(i, j) (Grid2D.cpp:229-233): the node map's f (memo / stale) */
int hastar_grid2d_node_cost(hastar_handle h, int i, int j, float* f);
/* AStar::find_path(i, j) (AStar.cpp:100-113): memoised cost-to-goal of cell (i, j) */
int hastar_astar_cost(hastar_handle h, int i, int j, float* cost);
/* AStar::find_path(goal, start, get_cost_only) / find_path(goal, start, path) (AStar.cpp:70-97).
 * With xy != NULL and cost_only == 0, *n points (x, y) of the path after the goal are written
 * (the reference's path vector is the goal followed by them). */
int hastar_astar_find_path(hastar_handle h, const float goal[2], const float start[2], int cost_only, float* cost,
                           float* xy, int cap, int* n);

/* Grid2D::clear_obstacles() (Grid2D.cpp:66-71) */
int hastar_grid2d_clear(hastar_handle h);

/* ---- Grid3D<float> (Grid3D.h:14-46) on a planner handle: the map, goal frame, APF list
 * and motion tables are the planner's (hastar_update_goal = update_goal_heading with the
 * relocation, hastar_update_boxes / _lines / hastar_decay = update_obstacles) ---- */
/* Grid3D::set_start_node(start) (Grid3D.cpp:127-160): the node and its cell (soft-reset) */
int hastar_grid3d_set_start_node(hastar_handle h, const float start[3], hastar_node3_f32* node, int cell[2]);
/* the goal node Grid3D::update_goal_heading returned at the last hastar_update_goal */
int hastar_grid3d_goal_node(hastar_handle h, hastar_node3_f32* node);
/* Grid3D::get_neighbors(node, neighbors) (Grid3D.cpp:47-74): successors inside the grid and
 * below the threshold, with the APF field added to g; cells = their (i, j). */
int hastar_grid3d_neighbors(hastar_handle h, const hastar_node3_f32* node, int cap, hastar_node3_f32* out, int* cells,
                            int* count, int* neglect);
/* Grid3D::check_path(path) (Grid3D.cpp:78-93) over n poses (n x 3) */
int hastar_grid3d_check_path(hastar_handle h, const float* xyh, int n, int* is_free);

#ifdef __cplusplus
}
#endif

#endif /* PATH_PLANNING_PKG_AMD_HASTAR_UNITS_H */
