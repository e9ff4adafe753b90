// hastar_layout.h — device-resident state of one planner, shared by the HIP kernels
// (hastar_kernels.hip) and the host runtime (hastar_capi.cpp).
//
// One planner == one reference HybridAStar<float> object (HybridAStar.h:61-74 and the
// Grid3D/Grid2D/AStar/VehicleModel/Dubins members it owns).  Everything the search
// touches lives in HBM in flat, index-linked arrays (no pointers inside records), so a
// batch of planners is just an array of PlannerDev descriptors, one wavefront each.
#pragma once
#include <stdint.h>

namespace hastar {

constexpr int NIL = -1;
constexpr int RB_RED = 0;
constexpr int RB_BLACK = 1;

// Open-set (std::set<Node3D<float>>, HybridAStar.h:72) tree node, 48 B = three 16-B
// quads.  Index 0 of the pool is the libstdc++ header: p = root, l = leftmost,
// r = rightmost, color = red.  key = cell x << 20 | cell y << 8 | angle bin
// (Node3D::operator!=, Node3D.h:44-47).  The RB color lives in byte 0 of `cc` (written
// with byte stores, so rebalancing never rewrites ci) and the curvature index in byte 1.
struct alignas(16) Node3 {
  uint32_t key;           // (x, y, bin)
  float f;                // _cost_f: the comparator's order key
  int l, r;               // tree links (pool indices, NIL = null): {key, f, l, r} = one 16-B load per walk step
  int p;                  // parent link
  uint32_t cc;            // color (byte 0) | _curvature_index << 8
  float g;                // _cost_g
  float vmin;             // _vmin_sqr
  float x, y, h;          // _pose2D (grid frame)
  int prev;               // closed-record index of the predecessor (NIL for the start)
};
static_assert(sizeof(Node3) == 48, "Node3 is three quads");

// Closed-set record (unordered_set<Node3D>, HybridAStar.h:73-74): a copy of the popped
// open node (its f is never read again).  Records never move, so prev links stay valid
// like the reference's pointers into the node-based hash set.
struct alignas(16) Closed3 {
  uint32_t key;
  float g, vmin;
  int prev;
  float x, y, h;
  int ci;
};
static_assert(sizeof(Closed3) == 32, "Closed3 is two quads");

// Holonomic A* open-set node (std::set<Node2D<float>>, AStar.h:70).
// key = x << 16 | y (Node2D::operator!=, Node2D.h:35-38).
struct alignas(16) Node2 {
  uint32_t key;
  float f;
  int l, r;               // {key, f, l, r}: one 16-B load per walk step
  int p, color;
  float g;
  int prev;               // index into the A* closed records of the current search
};

// Per-cell record of the inner A* (slot arena, N*N, generation-stamped so a new search
// needs no clearing).  It is also the search's closed record of the cell
// (unordered_set<Node2D>, AStar.h:71-72): a cell is closed at most once per search, so
// the record lives at the cell's index and `prev` links are cell indices.
//   cgen == search generation  -> closed, with the popped node's g and prev cell;
//   oinfo = (generation & 0x7fff) << 17 | hint: the cell's last inserted open node of the
//   LDS tree (bits 0-15) and bit 16, set once a second node of the cell was inserted while
//   another was still open.  A hint whose 15-bit generation matches a stale search is
//   harmless: it is only used after checking the node's key (and `dup` only forces the
//   exact scan).
struct alignas(16) Cell2 {
  uint32_t cgen;
  float g;
  int prev;
  uint32_t oinfo;
};
constexpr int CELL2_OGEN_SHIFT = 17;
constexpr uint32_t CELL2_OGEN_MASK = 0x7fffu;
constexpr uint32_t CELL2_HINT_MASK = 0x1ffffu;

// Closed-set hash slot (open addressing).  gi = generation (8 bits) << 24 | record
// index; a slot is live iff its generation is the search's, so clear() is O(1).  The
// generation cycles through 1..255; when it wraps the wave zeroes its table.  24 index
// bits allow 16 M closed records (a search that outgrows its arena is parked and resumed
// in a bigger one, see SearchResult).
struct Slot3 {
  uint32_t key;
  uint32_t gi;
};
constexpr int SLOT3_IDX_BITS = 24;
constexpr uint32_t SLOT3_IDX_MASK = (1u << SLOT3_IDX_BITS) - 1;
constexpr uint32_t SLOT3_GEN_MASK = 0xffu;

// diagnostic phase counters of the search kernel (-DHASTAR_STAMPS)
constexpr int NSTAMP = 40;

// Search status codes of SearchResult::status besides 0 / HASTAR_E* (host-side only).
constexpr int SEARCH_NOT_RUN = -1;  // the host's sentinel: no wave took this planner
constexpr int SEARCH_PARKED = 1;    // the arena filled up at a pop boundary: state kept for a resume
constexpr int SEARCH_HANDOFF = 2;   // (in flight only) a bulk wave handed the search to a latency CU

// Handoff board of a split launch ("Handoff"): a batch-kernel wave whose search
// has run `thr` pops offers it (POSTED, in the entry of its arena index); a latency-kernel wave
// that is free claims the oldest offer (CLAIMED); the batch wave parks the search at its next
// check (every 64 pops) exactly as a capacity park does, in its own arena, and publishes it
// (READY) and takes no more work; the latency wave copies the parked records into its own arena
// (COPIED) and continues the search there in resume mode, as a host resume would.  A search
// that ends before its wave sees the claim is withdrawn (CANCELLED; the latency wave empties the
// entry).  No side waits for the other except a claimer for its claimed entry, answered within
// 64 pops or at the search's end.
constexpr uint32_t HANDOFF_EMPTY = 0, HANDOFF_POSTED = 2, HANDOFF_CLAIMED = 3, HANDOFF_READY = 4,
                   HANDOFF_CANCELLED = 5, HANDOFF_COPIED = 6;
constexpr int HANDOFF_CAP = 4096;  // entries (arena indices 0 .. HANDOFF_CAP-1 can offer)
struct SlotArena;
struct alignas(16) HandoffEntry {
  unsigned long long t_start;      // when the search was offered (s_memrealtime): claims take the oldest
  int slot;                        // the batch wave's arena index (the search's state stays there)
  int pidx;                        // the planner (index into the launch's descriptors), set at READY
};
struct HandoffBoard {
  int enabled;      // 1 only while a split launch runs (the host sets it per launch)
  int thr;          // pops after which a batch-kernel search is offered
  int posted;       // entries in state POSTED (a claimer scans only when > 0)
  int bulk_active;  // batch-kernel waves still running (latency waves wait for offers until 0)
  int n;            // entries in use (the pool's arena count)
  int handoffs;     // searches handed over in this launch (diagnostic)
  const SlotArena* pool;  // the pool's arena descriptors (entry slot s = pool + s)
  int pad[8];
  uint32_t state[HANDOFF_CAP];
  HandoffEntry entry[HANDOFF_CAP];
};

// Per-search result block (written by the search kernel, read by the host).
// A search whose arena cannot take one more pop PARKS (status SEARCH_PARKED): the open tree
// and closed records stay in the arena it ran in (arena index park_arena of its launch),
// and the loop state needed to continue lives here (pop_digest holds the running digest).
// The host copies the records into a larger arena and relaunches the search in resume
// mode, so no search the reference would finish is cut short by a fixed capacity
// (the reference's sets grow without limit, HybridAStar.cpp:107).
struct SearchResult {
  long long pops, successors, astar_pops, astar_searches, shots, closed_size, astar_pops_hbm;
  unsigned long long pop_digest, closed_digest;
  int ok, via_shot, status, path_len;
  float cost;
  int terminal;           // closed record index the path is rebuilt from
  int dubins_len;         // samples of the successful shot
  int astar_migrations;   // inner A* searches that outgrew LDS
  unsigned long long cycles[NSTAMP]; // diagnostic build (-DHASTAR_STAMPS): s_memtime per phase
  unsigned long long t_start, t_end;  // s_memrealtime (100 MHz, chip-wide) around the search
  int slot;                           // slot (wavefront) that ran it
  int hw_id;                          // where: XCC_ID << 16 | HW_ID bits 15:0 (SE, SH, CU, SIMD, wave) at the end
  // park state (status == SEARCH_PARKED)
  int park_arena;                     // arena index (in the launch's arena array) holding the state
  int counter, interval, shot_allowed;  // Dubins-shot schedule (HybridAStar.cpp:96-154)
  int n_closed3, ps3_next, ps3_free;  // closed records and open-pool state in that arena
  int parks;                          // times this search was parked (diagnostic)
};

// Descriptor of one planner: constants + device pointers.  Lives in HBM; the kernel
// reads it once into scalar registers.
struct PlannerDev {
  // --- grid / vehicle constants (Grid2D.cpp:7-62, VehicleModel.cpp:7-47, HybridAStar.cpp:7-24)
  int N, n2, n45, diag;
  int bins, nsteer, na, shot_interval;
  int shot_decay, n_apf, arena_pops, span_alloc;  // arena_pops: initial outer capacity in pops (max_pops)
  float res, thr, apf_rep, apf_ang;
  float ts, a_lat, a_lat2, prec;
  float r_min, step, ang_step, act_cost_diag;   // Dubins radius/step; 2D diagonal move cost
  float act_cost_axis, apf_reach, pad_f1, pad_f2;  // apf_reach: max |successor offset| per axis (+ margin)
  // --- goal (grid frame) and world transform for path reconstruction
  float goal_x, goal_y, goal_h;                // _goal_node._pose2D
  int goal_cx, goal_cy, goal_bin;
  float world_goal_x, world_goal_y;            // _goal_location3D
  float rot_c, rot_s, grid_heading, pad_f3;    // cos/sin(-grid_heading)
  // --- start node of the next search (Grid3D::set_start_node, Grid3D.cpp:127-160)
  float start_x, start_y, start_h, start_vmin;
  int start_cx, start_cy, start_bin, start_ci;
  // --- state arrays
  float* occ;            // N*N log-odds (_obstacle_map), row i = x cell
  float* nm_f;           // N*N Node2D::_cost_f of _node_map (A* memo + stale f)
  uint32_t* visited;     // AStar::_visted as a bitmap: cell c is visited iff bit c & 31 of word c >> 5
  float* apf;            // n_apf x {x, y, r} (Grid3D::_apf_obstacles)
  float* off;            // nsteer x (bins + 1) x {dx, dy} (VehicleModel::_offset_xy + zero row)
  float* dth;            // nsteer  _offset_heading
  float* act_cost;       // nsteer  _actions_cost
  float* curv_abs;       // nsteer  _abs_curvatures
  float* out_xyh;        // reconstructed path (out_cap x 3) and curvature (out_cap)
  float* out_curv;
  int out_cap;
  int astar_cap;         // max_astar_nodes + 1: the inner open tree's pool, whatever arena runs the search
  SearchResult* result;
};

// ---- batched map updates (hastar_*_batch): one launch serves many planners' maps ----
// Grid2D::update_obstacles() of one map window (Grid2D.cpp:197-208)
struct DecayItem {
  float* occ;        // first cell of the window
  long long cells;   // cells in the window
  float lp_free, lp_min, lp_max, pad;
};
// Grid3D::relocate_obstacles of one map (Grid3D.cpp:169-203) with its scratch
struct RelocItem {
  float* occ;        // map (source, then destination of the copy-back)
  float* tmp;        // N*N scratch: the relocated map
  int* winner;       // N*N scratch, kept at -1 between uses
  int N;
  float c, s, ox, oy;
  int pad;
};
// one planner of a batched box raster
struct RasterMap {
  float* occ;
  int N, r0, r1;     // map size and row window
  float c, s, lp_min, lp_max;
  int pad;
};
// one box (Grid2D.cpp:99-139): sub-sample origin and counts, log-odds delta, and the cell
// window that holds every sub-sample (the layer footprint of hastar_update_boxes)
struct RasterBox {
  int map;           // index into the RasterMap array
  int si, sj, ni, nj;
  float d;
  int bi0, bj0;      // footprint origin (cells)
  int bw, bh;        // footprint size (cells), bw * bh <= RASTER_HIST
  int pad0, pad1;
};
constexpr int RASTER_HIST = 8192;  // LDS hit counters of one box footprint (32 KiB)
// a device-to-device copy of `count` floats (APF lists of a batch)
struct CopyItem {
  float* dst;
  long long src_off;
  int count, pad;
};

// Open-tree capacity of an inner A* search while it stays in LDS (kernel and host agree).
constexpr int ASTAR_LDS_CAP = 1024;

// Search arena of one resident wavefront ("slot").  Every search is transient state
// (HybridAStar's open/closed sets, AStar's open/closed sets, the Dubins scratch), so it
// belongs to the wave that runs the search, not to the planner: a persistent kernel with
// W slots serves any number of planners, and the planners keep only their maps.
struct SlotArena {
  Node3* open3;     int open3_cap;   int pops_grant;  // > 0: a head arena's own outer capacity in pops (else the planner's rule)
  Closed3* closed3; int closed3_cap; int pad1;
  Slot3* slots3;    uint32_t slots3_mask; int pad2;
  Node2* open2;     int open2_cap;   int pad3;
  Cell2* cell2;     // N*N per-cell records (closed state + open hint) of the current inner A* search
  size_t cells;     // capacity of cell2 (max N*N served)
  uint32_t* gens;   // [0] closed-set generation, [1] A* closed generation
  float* dub_xyh; float* dub_curv; int dub_cap; int pad5;
  int* out_chain;   int chain_cap;   int pad6;
  int* prevl;       // {prev link, g bits} of the LDS-resident A* tree nodes (2 x A_CAP)
  HandoffBoard* board;  // the device's handoff board (pool and head arenas; null elsewhere)
};

// Scratch of one planner in the RELAXED (non-parity) search mode (hastar_relaxed.hip,
// SURVEY.md §8(f) rank 4): one workgroup per planner, so one arena per resident workgroup.
//   dist    N*N backward 8-connected distance to the goal cell (the heuristic), float bits
//           updated with atomicMin (non-negative floats order like their bit patterns); used
//           when the planner keeps no field of its own (RelaxField)
//   bucket  8 x bcap {cell, distance bits} entries (a ring of Dial buckets of width act_cost_axis)
//   table   best {g, tie} per node key (open addressing; key 0xffffffff = empty; left empty by
//           every search)
//   nodes   every node ever generated (Node3 records; prev = parent node, l = its table slot,
//           r = its tie)
//   lists   3 x list_cap lists of {f bits, node} (8 B): the open list, the next open list
//           (the round's raw successors first) and the round's expansion set (node indices)
//   dub_*   one Dubins-shot scratch of dub_cap samples per shot of a round
//   chain   path reconstruction scratch
struct BucketEntry { uint32_t cell, d; };  // a Dial-bucket entry: cell (i << 16 | j) and its distance bits
// best-g table slot of the relaxed search: best = g bits << 32 | tie, where tie hashes the
// (parent key, action) that generated the node, so equal-g offers resolve by value, not by
// which wavefront got there first
struct alignas(16) RelaxSlot {
  uint32_t key;
  uint32_t pad;
  unsigned long long best;
};
struct RelaxArena {
  float* dist;
  BucketEntry* bucket;    int bcap;       int pad0;
  RelaxSlot* table; uint32_t tmask; int pad1;
  Node3* nodes;     int node_cap;   int pad2;
  int* lists;       int list_cap;   int pad3;
  float* dub_xyh;   float* dub_curv; int dub_cap; int pad4;
  int* chain;       int chain_cap;  int pad5;
  size_t cells;     // N*N served
};
// A planner's own heuristic field (hastar_relaxed_opts.reuse_heuristic): computed once, then
// reused by later relaxed searches until reset() or update_goal() (the reference's A* memo
// persists across find_path calls the same way, AStar.cpp:56-60, local_planner.cpp:316).
struct RelaxField {
  float* dist;      // N*N, or null: use the arena's scratch
  float hlim;       // the ellipse bound the field was built with (relaxed_h)
  int valid;        // 1: dist/hlim hold a finished field
  int start_ij;     // the start cell (i << 16 | j) the ellipse was built around
};
// options of a relaxed launch (kernel side of hastar_relaxed_opts)
struct RelaxParams {
  float delta;      // frontier width (m): every open node with f <= min f + delta is expanded in a round
  float h_stop;     // the Dijkstra covers the ellipse d(c) + |c - start| <= h_stop x |goal - start| + 64 moves
  int max_rounds;
  float h_weight;   // f = g + h_weight x max(h, Dubins length) (1: the reference's f)
  int h_coarse;     // the Dijkstra field's block side in map cells (1, 2 or 4)
  unsigned* progress;  // debug (HASTAR_RELAXED_PROGRESS): per-wave phase words in host memory, or null
  // reversing motion model (round 6; hastar_relaxed_opts::reverse_cost): rev_cost > 0 adds the
  // reverse arcs (action cost x rev_cost) and makes the heuristic and the shots Reeds-Shepp
  // (hastar_rs.h); 0 keeps the reference's forward model
  float rev_cost;
  float gear_cost;      // added to a motion or shot segment that changes the direction of travel (m)
  signed char* dir_out; // per-pose direction (+1 forward, -1 reverse) of planner i's path at dir_out + i * dir_stride, or null
  int dir_stride;
};

}  // namespace hastar
