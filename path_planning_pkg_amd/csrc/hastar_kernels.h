// hastar_kernels.h — host-callable launch wrappers of hastar_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include "hastar_layout.h"

namespace hastar {
// the batch kernel: 8 search waves per CU (n_slots arenas; slot s runs in d_arenas[s])
hipError_t launch_search(const PlannerDev* d_descs, int n, const SlotArena* d_arenas, int n_slots, const int* d_order, int n_prio,
                         int* d_next, long long hard_pops, hipStream_t st, int arena_base = 0, int q0 = 0,
                         int head_wgs = 0);
hipError_t launch_resume(const PlannerDev* d_descs, int n, const SlotArena* d_arenas, const int* d_order,
                         long long hard_pops, hipStream_t st);
// the latency kernel: one search per CU (batches no larger than the CU count, resumes)
hipError_t launch_search_wide(const PlannerDev* d_descs, int n, const SlotArena* d_arenas, int n_slots,
                              const int* d_order, int* d_next, long long hard_pops, hipStream_t st, int head = 0,
                              int arena_base = 0);
int search_slots_per_cu();
hipError_t launch_relaxed(const PlannerDev* d_descs, int n, const RelaxArena* d_arenas, int n_arenas, int* d_next,
                          const RelaxParams& rp, RelaxField* d_fields, hipStream_t st);
int relaxed_waves();
// the backward grid-distance field over a block of rows (hastar_field.hip)
hipError_t launch_field_init(float* f, int N, int r0, int r1, int gi, int gj, hipStream_t st);
int field_tiles(int N, int r0, int r1, int* ntx, int* nty);
hipError_t launch_field_activate(int* act, int ntx, int nty, int mode, int* pending, hipStream_t st);
hipError_t launch_field_pass(const PlannerDev& P, float* f, int r0, int r1, const int* act, int* nxt, int* flags,
                             int* pending, hipStream_t st);
hipError_t launch_test_rs(float r, const float* starts, int n, float gx, float gy, float gh, float* len, int* word,
                          float* seg, float* len_groups, hipStream_t st);
hipError_t launch_grid3d_neighbors(const PlannerDev* d_desc, const float node[5], int nci, int nbin, float* out,
                                   int* cells, int cap, int* count, int* neglect, hipStream_t st);
hipError_t launch_grid3d_check_path(const PlannerDev* d_desc, const float* xyh, int n, int* is_free, hipStream_t st);
hipError_t launch_astar_query(const PlannerDev* d_desc, const SlotArena* d_arena, int si, int sj, int mode, float gwx,
                              float gwy, float rc, float rs, float* out_cost, float* xy, int cap, int* out_n,
                              hipStream_t st);
hipError_t launch_gather_paths(const PlannerDev* d_descs, const long long* d_off, const int* d_len, int n, float* xyh,
                               float* curv, hipStream_t st);
hipError_t launch_init_nodemap(const PlannerDev& P, hipStream_t st);
hipError_t launch_init_nodemap_batch(const PlannerDev& P, char* base, size_t stride, int n, hipStream_t st);
hipError_t launch_clear_bitmaps(uint32_t* const* ptrs, int n, size_t words, hipStream_t st);
hipError_t launch_decay(float* occ, size_t NN, float lp_free, float lp_min, float lp_max, hipStream_t st);
hipError_t launch_raster_boxes(float* occ, int* cnt, int N, const int* rp, const float* dl, const int* ids, int nid,
                               float c, float s, float lp_min, float lp_max, int row0, int row1, hipStream_t st);
hipError_t launch_raster_lines(float* occ, int* cnt, int N, int n45, int n2, float res, const float* lp,
                               const float* seq_len, const float* seq_wid, int seq_stride, int nline, float lp_min,
                               float lp_max, int row0, int row1, hipStream_t st);
hipError_t launch_decay_batch(const DecayItem* items, int n, size_t max_cells, hipStream_t st);
hipError_t launch_relocate_batch(const RelocItem* items, int n, size_t max_cells, hipStream_t st);
hipError_t launch_relocate_invert(const RelocItem* items, int n, size_t max_cells, hipStream_t st);
hipError_t launch_raster_boxes_batch(const RasterMap* maps, const RasterBox* boxes, int nbox, hipStream_t st);
hipError_t launch_copy_batch(const CopyItem* items, int n, const float* src, hipStream_t st);
struct VelParams { float max_velocity, coast_velocity, max_lat_acc, max_lat_acc_sqr, max_long_acc, max_long_dec; };
hipError_t launch_velocity_profile(const VelParams& vp, int n, const long long* off, const float* xyh, const float* curv,
                                   const float* vel_init, const float* vmax_curr, const unsigned char* flags, float* vel,
                                   unsigned char* feasible, hipStream_t st);
hipError_t launch_test_math(int fn, const float* a, const float* b, float* out, int n, hipStream_t st);
hipError_t launch_test_field(const PlannerDev& P, const float* poses, int n, float* out, hipStream_t st);
hipError_t launch_test_dubins_len(float r, const float* starts, int n, float gx, float gy, float gh, float* out,
                                  int* word, hipStream_t st);
hipError_t launch_test_dubins_path(const PlannerDev& P, float sx, float sy, float sh, float* xyh, float* curv,
                                   int cap, int* n_out, float* len_out, int* flag_out, hipStream_t st);
}  // namespace hastar
