/* hastar.h — C ABI of the MI355X-native Hybrid A* planner (path_planning_pkg_amd).
 *
 * This is the drop-in boundary for the reference's planner facade
 * `planning::HybridAStar<T>` (reference: include/path_planning_pkg/HybridAStar.h:27-75,
 * lib/HybridAStar.cpp:7-286).  Every entry point below replaces one public member
 * function of that class; the C++ header include/path_planning_pkg/HybridAStar.h
 * re-implements the class on top of these calls so src/local_planner.cpp links
 * unchanged.
 *
 * Plain C: opaque handles, plain pointers and sizes, no torch/HIP types.
 * All functions return 0 on success or a negative HASTAR_E* code.
 * A handle is single-threaded like the reference object; the batch call runs many
 * handles' searches concurrently on one GPU (one wavefront per planner).
 *
 * Arithmetic type: float (the reference's ROS node instantiates HybridAStar<float>,
 * src/local_planner.cpp:509).
 */
#ifndef PATH_PLANNING_PKG_AMD_HASTAR_H
#define PATH_PLANNING_PKG_AMD_HASTAR_H

#ifdef __cplusplus
extern "C" {
#endif

#define HASTAR_OK 0
#define HASTAR_EINVAL (-22)     /* bad argument / handle */
#define HASTAR_ENOSPC (-28)     /* output buffer too small: *len holds the length needed */
#define HASTAR_ENOMEM (-12)     /* device allocation failed */
#define HASTAR_EDEVICE (-5)     /* HIP runtime / kernel error (message via hastar_last_error) */
#define HASTAR_EOVERFLOW (-75)  /* search exceeded the handle's arena (max_pops etc.) */

/* Constructor arguments: the 20 parameters of HybridAStar<T>::HybridAStar
 * (HybridAStar.h:33-38, called by src/local_planner.cpp:158-161), in the same order
 * and meaning, plus arena limits for the device search. */
typedef struct hastar_params {
  int dubins_shot_interval;        /* pops between Dubins shots (HybridAStar.cpp:98) */
  int dubins_shot_interval_decay;  /* interval decrement after a failed shot */
  float grid_resolution;           /* metres per cell */
  float obstacle_threshold;        /* occupancy probability threshold */
  float obstacle_prob_min;         /* log-odds clamp, as probabilities */
  float obstacle_prob_max;
  float obstacle_prob_free;        /* decay step, as probability */
  int grid_size;                   /* N (square N x N grid) */
  int grid_2d_allow_diag_moves;    /* bool: 8- vs 4-connected holonomic A* */
  float step_size;                 /* motion primitive length (m) */
  float max_lat_acc;
  float max_long_dec;
  float wheelbase;
  float rear_to_cg;
  float apf_rep_constant;
  float apf_active_angle;          /* radians */
  int num_angle_bins;
  int num_actions;
  int num_steering;                /* length of steering[] and curvature_weights[] */
  const float* steering;           /* radians */
  const float* curvature_weights;
  /* ---- extensions (0 = default) ---- */
  int max_pops;                    /* initial arena of a search, in pops (default 262144); a search
                                      that outgrows it is parked and resumed in a 4x larger arena,
                                      so this is NOT a limit (the reference has none) */
  int max_astar_nodes;             /* arena: open-set nodes of one inner A* search (default min(N*N+16, 65536)) */
  int max_dubins_samples;          /* arena: samples of one Dubins shot (default from N) */
} hastar_params;

typedef struct hastar_handle_s* hastar_handle;

/* Per-search statistics (work units of the measurement in DESIGN.md). */
typedef struct hastar_stats {
  long long pops;              /* iterations of HybridAStar.cpp:107 (incl. re-expanded duplicates) */
  long long successors;        /* successors that passed the bounds/occupancy filter (Grid3D.cpp:54-59) */
  long long astar_pops;        /* pops of the lazy holonomic A* (AStar.cpp:127) */
  long long astar_searches;    /* a_star_search() calls (memo misses) */
  long long shots;             /* Dubins shots attempted */
  long long closed_size;       /* Hybrid A* closed-set size at termination */
  unsigned long long pop_digest;    /* ordered digest of (cell, bin, g bits) of every pop */
  unsigned long long closed_digest; /* order-independent digest of the closed-set keys */
  int via_shot;                /* success came from an analytic Dubins shot */
  int status;                  /* this planner's outcome: 0, HASTAR_EOVERFLOW (HASTAR_MAX_POPS_HARD
                                  budget, or no larger arena could be allocated nor lent by idle
                                  slot arenas of the pool), HASTAR_ENOSPC (path longer
                                  than the caller's cap: *len is the length needed) */
  int parks;                   /* times the search outgrew its arena and was resumed in a larger one */
  int pad;
} hastar_stats;

/* HybridAStar(...) (HybridAStar.cpp:7-24). device = HIP device ordinal. */
int hastar_create_f32(const hastar_params* params, int device, hastar_handle* out);
int hastar_destroy(hastar_handle h);

/* n planners with the same constructor arguments in one call (out: n handles, each behaving
 * like one from hastar_create_f32 and destroyed one by one): their maps share one
 * allocation and one shared copy of the motion tables (freed with the last of them), and
 * the node maps are initialised in one launch. */
int hastar_create_batch_f32(const hastar_params* params, int n, int device, hastar_handle* out);

/* update_goal(goal, start) (HybridAStar.cpp:55-59): goal/start = {x, y, heading}. */
int hastar_update_goal(hastar_handle h, const float goal[3], const float start[3]);

/* reset() (HybridAStar.cpp:49-52): clears the holonomic A* memo. */
int hastar_reset(hastar_handle h);

/* reset() of n planners in one call (batch drivers; same effect as n hastar_reset calls). */
int hastar_reset_batch(const hastar_handle* hs, int n);

/* Scheduling hint (no counterpart in the reference): the planner's expected search cost, the
 * key of the longest-first order of its next batched find_path (larger first; equal keys keep
 * the caller's order; units: 10-ns ticks of expected search time).  After every exact search the
 * library keys the planner by the longer of its last two search durations (a hint set here counts
 * alone until the next search); 0 (a fresh planner) = unknown: the planner is then keyed by its
 * last boxes' distances to the straight start-goal route.  Results never depend on it, only the order in
 * which a batch's searches start and, for a large batch, which of them run on the latency
 * CUs. */
int hastar_set_cost_hint(hastar_handle h, long long hint);

/* Device pool reservation (no counterpart in the reference): sizes the device context's search
 * arenas, batch tables and, when path_points > 0, the packed-path buffers for a batched
 * find_path of these n planners, so that the batch's first call allocates nothing.  Optional:
 * find_path grows the pool itself.  Same errors as hastar_find_path_batch (HASTAR_ENOMEM when
 * the pool cannot be had). */
int hastar_reserve(const hastar_handle* hs, int n, long long path_points);

/* update_obstacles(obstacles, confidence, apf_added_radius) (HybridAStar.cpp:29-33):
 * boxes = n x {center_x, center_y, dimension_x, dimension_y} (Obstacle.h:16-21). */
int hastar_update_boxes(hastar_handle h, const float* boxes, const float* confidence, int n,
                        float apf_added_radius);

/* update_obstacles(lines, confidence, line_width) (HybridAStar.cpp:36-40):
 * lines = n x {x1, y1, x2, y2}. */
int hastar_update_lines(hastar_handle h, const float* lines, const float* confidence, int n,
                        float line_width);

/* update_obstacles() (HybridAStar.cpp:43-46): free-space decay of every cell. */
int hastar_decay(hastar_handle h);

/* ---- batched map updates: the calls above for n planners of ONE device at once (the
 * reference updates one instance at a time, Grid2D.cpp:99-208, Grid3D.cpp:22-44, 102-203;
 * a batch equals n single calls in planner order, bit for bit).  One staged upload and a
 * few launches serve the whole batch, instead of ~12 C calls with their pageable copies and
 * launches per planner. ---- */
/* update_goal of planner i with goals[3i..3i+2], starts[3i..3i+2]. */
int hastar_update_goal_batch(const hastar_handle* hs, int n, const float* goals, const float* starts);
/* update_obstacles() of every planner. */
int hastar_decay_batch(const hastar_handle* hs, int n);
/* update_obstacles(boxes, confidence, apf_added_radius): planner i takes counts[i] boxes
 * (4 floats each) and confidences, packed after planner i-1's. */
int hastar_update_boxes_batch(const hastar_handle* hs, int n, const float* boxes, const float* confidence,
                              const int* counts, float apf_added_radius);

/* find_path(vel_init, start, path, curvature) (HybridAStar.cpp:68-88).
 * xyh receives len x {x, y, heading} in the order the reference appends them
 * (goal first, start last; HybridAStar.cpp:208-262), curv receives len curvatures.
 * cap = capacity in poses.  On HASTAR_ENOSPC *len is the required length and the
 * search state is kept (call hastar_copy_path with a bigger buffer).
 * *cost / *ok are the reference's returned pair (FLT_MAX, 0 on failure).
 * stats may be NULL. */
int hastar_find_path(hastar_handle h, float vel_init, const float start[3], float* xyh, float* curv,
                     int cap, int* len, float* cost, int* ok, hastar_stats* stats);

/* Copy the path of the last find_path again (for a retry after HASTAR_ENOSPC). */
int hastar_copy_path(hastar_handle h, float* xyh, float* curv, int cap, int* len);

/* Batched find_path over n independent planners: one kernel launch, one wavefront per
 * planner.  Arrays are indexed by planner; xyh is n x cap x 3, curv n x cap, len/cost/ok n.
 * Returns the first error; per-planner status is in stats[i].status when stats != NULL. */
int hastar_find_path_batch(const hastar_handle* hs, int n, const float* vel_init, const float* starts,
                           float* xyh, float* curv, int cap, int* len, float* cost, int* ok,
                           hastar_stats* stats);

/* ---- RELAXED search mode (no reference counterpart) ----
 * NOT bit-exact with the reference, by design: a frontier-parallel Hybrid A* (one workgroup
 * of 8 wavefronts per planner) whose heuristic is a backward Dijkstra over the grid (the
 * converged value of the reference's lazy holonomic A*, AStar.cpp:118-186) and whose rounds
 * expand every open node with f <= min f + delta at once, with a best-g table per node key
 * instead of the closed set.  Same successors, costs, APF field, Dubins shots and output
 * format as hastar_find_path_batch, so a caller can switch per call; paths are valid
 * (collision-free, start to goal) but may differ from, and cost more or less than, the
 * reference's.  The exact mode's memo (node-map f, visited flags) is neither read nor written.
 * opts may be NULL (defaults in brackets). */
typedef struct hastar_relaxed_opts {
  float delta;     /* frontier width in metres [0.25] */
  float h_stop;    /* the Dijkstra covers the ellipse d(c) + |c - start| <= h_stop x |goal - start| + 64 moves;
                      cells outside get bound - |c - start| [1.2] */
  int max_nodes;   /* node capacity per search; beyond it the search ends with HASTAR_EOVERFLOW [1 << 18] */
  int max_rounds;  /* [1 << 20] */
  float h_weight;  /* f = g + h_weight x max(h, Dubins length); > 1 trades cost for speed [1.35]
                      (defaults from profiles/r03t_relaxed_sweep.json: costs 0.92-1.01 x the exact
                      mode's, the cfg3 and cfg5 groups in 10.3 and 8.4 ms) */
  int reuse_heuristic; /* 1: the planner keeps its heuristic field (N*N floats of device memory)
                          and later relaxed calls reuse it until reset() or update_goal(), as the
                          reference's A* memo persists across replans; map updates in between
                          leave it stale (it only guides: every successor is checked against the
                          current map) [0: recompute per call] */
  int h_coarse;    /* the Dijkstra field runs over blocks of h_coarse x h_coarse map cells (1, 2 or 4):
                      a block is passable when any of its cells is, and a cell's heuristic is its
                      block's distance [2] */
  float reverse_cost; /* > 0: a REVERSING motion model, which the reference does not have
                         (VehicleModel.cpp:97-101 drives forward only; BASELINE.json configs[2] asks
                         for "Reeds-Shepp reversals"): every steering also gets its reverse arc, whose
                         action cost is multiplied by reverse_cost, and the Dubins heuristic and shots
                         become Reeds-Shepp ones (csrc/hastar_rs.h) whose reverse segments cost
                         reverse_cost x their length [0: forward only, the reference's model] */
  float gear_cost;    /* with reverse_cost > 0: metres added at each change of direction [0] */
} hastar_relaxed_opts;
int hastar_find_path_relaxed_batch(const hastar_handle* hs, int n, const float* vel_init, const float* starts,
                                   float* xyh, float* curv, int cap, int* len, float* cost, int* ok,
                                   hastar_stats* stats, const hastar_relaxed_opts* opts);
/* The same, plus each pose's direction of travel: dir[i * cap + k] = +1 when pose k of path i
   was reached driving forward, -1 in reverse (always +1 without reverse_cost; the path's first
   pose, at the goal end, carries the direction of the motion that reached the goal).  dir may
   be NULL. */
int hastar_find_path_relaxed_batch_dir(const hastar_handle* hs, int n, const float* vel_init, const float* starts,
                                       float* xyh, float* curv, signed char* dir, int cap, int* len, float* cost, int* ok,
                                       hastar_stats* stats, const hastar_relaxed_opts* opts);

/* get_obstacles() (HybridAStar.cpp:62-65): copies the N x N log-odds map (row i = x cell). */
int hastar_get_obstacles(hastar_handle h, float* out);

/* ---- row-block sharding of the map build (no reference
 * counterpart: the reference builds Grid2D::_grid (Grid2D.cpp:99-208) on one core) ----
 * hastar_set_row_window limits hastar_decay / hastar_update_boxes / hastar_update_lines to
 * rows [row0, row1) of the N x N log-odds map (row i = x cell); [0, N) is the default and
 * the reference's behaviour.  The union of disjoint windows equals the full build bit for
 * bit.  hastar_update_goal (relocate) ignores the window.  export/import copy rows between
 * the planner's map and a DEVICE buffer on the planner's device (N floats per row) and
 * return after the copy completed: a rank exports its block, the blocks are all-gathered
 * (RCCL), and every rank imports the gathered map with row0 = 0, row1 = N. */
int hastar_set_row_window(hastar_handle h, int row0, int row1);
int hastar_export_rows(hastar_handle h, int row0, int row1, float* dst_device);
int hastar_import_rows(hastar_handle h, int row0, int row1, const float* src_device);

/* ---- the backward grid-distance field to the goal, row-sharded (BASELINE.json north_star:
 * "Grid2D heuristic fill ... backward-Dijkstra heuristic precompute shards across GPUs"; no
 * reference counterpart: the reference computes the same distances lazily, cell by cell, in
 * AStar::find_path(int, int), AStar.cpp:100-186, over Grid2D.cpp:22-40's moves) ----
 * field(v) = min over neighbours u that can be expanded (the goal cell, or log-odds < the
 * occupancy threshold) of field(u) + move cost (act cost axis / diagonal, 4 or 8 moves), in
 * float; field(goal) = 0; +inf where nothing reaches.  The system has one solution, so the
 * result does not depend on how the rows are split (csrc/hastar_field.hip).
 * hastar_heuristic_field writes the whole N x N field (row i = x cell) to a DEVICE buffer.
 * hastar_field_rows relaxes rows [r0, r1) of a DEVICE buffer of (r1 - r0 + 2) x N floats
 * (halo row r0 - 1, the block, halo row r1) until it is stable for its halo rows: init = 1
 * fills it (+inf, the goal 0) first; otherwise halo_changed bit 0 / bit 1 say that the upper /
 * lower halo row was overwritten since the last call.  *changed: bit 0 any cell, bit 1 row
 * r0, bit 2 row r1 - 1 changed; *passes: relaxation passes queued, in batches of 8 (either
 * may be NULL).  Ranks exchange their first / last rows into their neighbours' halos and call
 * again until no rank's edge rows change (path_planning_pkg_amd/shard.py:heuristic_field_sharded).
 * hastar_relaxed_set_field installs a whole field (DEVICE, N x N) as the planner's relaxed-mode
 * heuristic: relaxed calls with reuse_heuristic = 1 and h_coarse = 1 use it until
 * hastar_reset or hastar_update_goal. */
int hastar_heuristic_field(hastar_handle h, float* dst_device, int* passes);
int hastar_field_rows(hastar_handle h, float* field_device, int r0, int r1, int init, int halo_changed, int* changed,
                      int* passes);
int hastar_relaxed_set_field(hastar_handle h, const float* src_device);

/* ---- VelocityGenerator<float> (post-search path products) ----
 * Replaces VelocityGenerator<T>::VelocityGenerator (VelocityGenerator.cpp:7-15) and
 * generate_velocity_profile (VelocityGenerator.cpp:19-84), called by local_planner.cpp:323,
 * 332, 451, 460 on find_path's output.  One call profiles n paths on `device`:
 * path p is points [offsets[p], offsets[p+1]) of xyh (3 floats per point, goal -> start
 * order as find_path returns it) and curv; flags[p] bit 0 = coast_to_goal, bit 1 =
 * stop_at_goal.  velocity gets one float per point, feasible[p] the reference's return
 * value.  Host buffers in and out.  A path with 0 points (undefined behaviour in the
 * reference) is -EINVAL. */
typedef struct hastar_velocity_params {
  float max_velocity;   /* _max_velocity (m/s) */
  float coast_velocity; /* _coast_velocity (m/s) */
  float max_lat_acc;    /* _max_lat_acc (m/s^2) */
  float max_long_acc;   /* _max_long_acc (m/s^2) */
  float max_long_dec;   /* _max_long_dec (m/s^2) */
} hastar_velocity_params;
int hastar_velocity_profile_batch(int device, const hastar_velocity_params* vp, int n,
                                  const long long* offsets, const float* xyh, const float* curv,
                                  const float* vel_init, const float* max_velocity_curr,
                                  const unsigned char* flags, float* velocity, unsigned char* feasible);

/* The same profile over the paths of this device's last hastar_find_path_batch, which
 * stay packed in HBM (local_planner.cpp:316-323 profiles the search's own output): no path
 * upload.  n must equal that batch's planner count; path i has the len[i] points the batch
 * returned (0 points: feasible[i] = 0, no velocities) and velocity receives sum(len)
 * floats in planner order. */
int hastar_velocity_profile_last_batch(int device, const hastar_velocity_params* vp, int n, const float* vel_init,
                                       const float* max_velocity_curr, const unsigned char* flags, float* velocity,
                                       unsigned char* feasible);

/* Grid size N of the handle. */
int hastar_grid_size(hastar_handle h);

/* Last error message of this thread (static storage). */
const char* hastar_last_error(void);

/* ---- timing hooks used by bench.py (device time of the last search launch) ---- */
/* Milliseconds of the last search kernel (HIP events on the launch stream). */
float hastar_last_search_ms(void);

#ifdef __cplusplus
}
#endif

#endif /* PATH_PLANNING_PKG_AMD_HASTAR_H */
