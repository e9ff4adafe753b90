/* hastar_test.h — unit-level test and debug hooks of libhastar_amd.so.
 *
 * Not part of the reference's interface: these let the parity tests compare one
 * building block at a time (libm ports, APF field, Dubins length/sampling, motion
 * tables, memo and closed set) between the GPU and the CPU oracle.
 */
#ifndef PATH_PLANNING_PKG_AMD_HASTAR_TEST_H
#define PATH_PLANNING_PKG_AMD_HASTAR_TEST_H
#include "hastar.h"

#ifdef __cplusplus
extern "C" {
#endif

/* fn: 0 sinf, 1 cosf, 2 atan2f(a, b), 3 acosf, 4 hypotf(a, b), 5 wrap_pi, 6 heading index(a, prec b), 7 atanf */
int hastar_test_math(int fn, const float* a, const float* b, float* out, int n);
/* Grid3D::get_field_intensity of n poses (x, y, heading) against the handle's obstacle list. */
int hastar_test_field(hastar_handle h, const float* poses, int n, float* out);
/* Dubins::get_shortest_path_length of n start poses to one goal; word = 0 RSR, 1 RSL, 2 LSR, 3 LSL. */
int hastar_test_dubins_len(float r_min, const float* starts, int n, const float goal[3], float* out, int* word);
/* The relaxed mode's Reeds-Shepp code (csrc/hastar_rs.h; no reference counterpart): for n start
   poses and one goal, turning radius r_min: the shortest length (metres), its word (0..17,
   oracle/reeds_shepp.py WORDS) and 5 signed segment lengths (radius units, seg[5 i ..]), and the
   grouped-lane length the successor heuristic uses, with groups of 4 and 16 lanes
   (len_groups[2 i], [2 i + 1]). */
int hastar_test_reeds_shepp(float r_min, const float* starts, int n, const float goal[3], float* len, int* word,
                            float* seg, float* len_groups);
/* Dubins::get_shortest_path from start to the handle's goal pose (grid frame), sampled. */
int hastar_test_dubins_path(hastar_handle h, const float start[3], float* xyh, float* curv, int cap, int* n,
                            float* length, int* first_arc_gt_90);
/* Copies of the device state. */
int hastar_debug_memo(hastar_handle h, float* f_out, unsigned char* visited_out);
int hastar_debug_apf(hastar_handle h, float* out, int cap);
int hastar_debug_motion(hastar_handle h, float* off, float* dth, float* cost, float* curv_abs, float* prec,
                        float* r_min);
int hastar_debug_closed_keys(hastar_handle h, int* out, int cap);
/* Cycles per search phase of the last search (all zero unless built with -DHASTAR_STAMPS). */
int hastar_debug_cycles(hastar_handle h, unsigned long long* out40);
/* {inner A* searches migrated from LDS to HBM, inner A* pops done in HBM mode} of the last search. */
int hastar_debug_astar_modes(hastar_handle h, long long* out2);
/* Timing of the last search: {t_start, t_end} in s_memrealtime ticks (100 MHz, chip-wide
 * clock) and the slot (persistent wavefront) that ran it. */
int hastar_debug_timing(hastar_handle h, unsigned long long* out3);
/* Where the last search ran: XCC_ID << 16 | HW_ID[15:0] (wave, SIMD, pipe, CU, SH, SE fields) of
 * its wavefront at the end of the search. */
int hastar_debug_hw_id(hastar_handle h, int* out);
/* Search-slot pool of the handle's device: {resident wavefronts, search waves per CU, arenas, MiB per arena,
   latency CUs of a split launch (0: none)}. */
int hastar_debug_slots(hastar_handle h, long long* out5);
/* head arenas of the device's split launches: {count, pool arenas per head arena (0 = own
 * allocation), outer capacity in pops} (hastar_capi.cpp head_acquire) */
int hastar_debug_head_arenas(hastar_handle h, long long* out3);
/* the device's last split launch (hastar_find_path_batch of a large batch): ms from the timed
 * region's start to the head kernel's start and end, and to the bulk kernel's start and end */
int hastar_debug_split(hastar_handle h, float* out4);
/* searches the device's last split launch handed from batch-kernel slots to latency CUs */
int hastar_debug_handoffs(hastar_handle h, int* out);
/* resume arenas carved from idle slot arenas of the pool so far (process-wide count) */
int hastar_debug_pooled_resumes(long long* out);
/* The device's relaxed-mode arena pool: {arenas (= resident workgroups of a relaxed launch), MiB each}. */
int hastar_debug_relaxed_pool(hastar_handle h, long long* out2);
/* The cold-order score of a planner with no history (host only): sum over the boxes {x, y, dx, dy}
 * (world frame) of (1 + t) / (1 + d)^3, d = distance between the box and the start-goal segment,
 * t = the box centre's position along it (0 at the start, 1 at the goal). */
double hastar_test_route_score(const float* boxes, int n, const float start[2], const float goal[2]);
/* The relaxed kernel's per-wave progress words (4 per wave: phase, round, expansion-set size,
 * expansion index; workgroup b, wave w at [(b * 8 + w) * 4]) in pinned host memory, readable
 * while a launch runs; null unless HASTAR_RELAXED_PROGRESS was set before the first relaxed call. */
const unsigned* hastar_debug_relaxed_progress(void);

#ifdef __cplusplus
}
#endif
#endif
