// hastar_capi.cpp — host runtime behind include/hastar.h (the drop-in C ABI).
//
// Ownership model (HBM layout):
//   * a planner (hastar_handle) owns its persistent state: log-odds map, node-map f
//     (A* memo + stale values), memo flags, APF list, motion tables, output buffers;
//   * the transient search state (open/closed sets of both searches, Dubins scratch)
//     lives in per-slot arenas owned by the device context: one arena per resident
//     wavefront of the persistent search kernel, reused across planners and calls;
//   * all work of a device goes to one HIP stream, so map updates are asynchronous and
//     stream-ordered (the reference API is synchronous only where it returns data:
//     find_path, get_obstacles).
// Per-call scalar preparation (rotations of the call's inputs into the goal-centred grid
// frame, per-box/per-line raster parameters, the start node) is done here with the
// reference's float arithmetic and the bit-faithful libm ports; every per-cell and
// per-expansion operation runs in the HIP kernels.  There is no CPU fallback: without a
// usable gfx950 device every call returns HASTAR_EDEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <atomic>
#include <mutex>
#include <unordered_map>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hastar.h"
#include "../../include/hastar_test.h"
#include "../../include/hastar_units.h"
#include "glibc_mathf.h"
#include "hastar_kernels.h"
#include "hastar_layout.h"

using namespace hastar;
using gmath::g_atan2f;
using gmath::g_cosf;
using gmath::g_hypotf;
using gmath::g_sinf;

namespace {

thread_local std::string g_err;
thread_local float g_last_ms = 0.0f;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
}  // namespace

// the other host modules (hastar_f64.cpp) report through the same hastar_last_error()
namespace hastar {
int set_last_error(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace hastar

namespace {

#define HIPCHK(expr)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) return fail(HASTAR_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// ---- reference scalar helpers on the host (common.h) ----
float wrap_pi_h(float a) {
  const float w = (float)std::fmod((double)a, 2 * M_PI);
  if ((double)w > M_PI) return (float)((double)w - 2 * M_PI);
  if ((double)w < -M_PI) return (float)((double)w + 2 * M_PI);
  return w;
}
int heading_bin_h(float h, float prec) {
  const float r = std::round(h / prec) * prec;
  return gmath::x86_trunc_int(((double)r + M_PI) / (double)prec);
}
struct V2 { float x, y; };
// Vector2D::get_rotated_vector (common.h:55-61)
V2 rot2(float x, float y, float ang) {
  const float c = g_cosf(ang), s = g_sinf(ang);
  return {x * c + y * s, -x * s + y * c};
}

template <class T>
hipError_t dalloc(T** p, size_t n) {
  return hipMalloc(reinterpret_cast<void**>(p), std::max<size_t>(n, 1) * sizeof(T));
}
size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
struct DeviceCtx;
template <class T>
hipError_t side_alloc(DeviceCtx& D, T** p, size_t n);
template <class T>
void side_free(DeviceCtx& D, T* p, size_t n);
// 32-bit words of a visited bitmap of NN cells, rounded up to 16-byte stores
size_t bitmap_words(size_t NN) { return ((NN + 31) / 32 + 3) & ~(size_t)3; }

// Arena requirements of one planner (the pool is sized for the maximum over a batch).
struct ArenaReq {
  int open3 = 0, closed3 = 0, open2 = 0, dub = 0, chain = 0;
  uint32_t slots = 1;
  size_t cells = 0;
  bool covers(const ArenaReq& o) const {
    return open3 >= o.open3 && closed3 >= o.closed3 && open2 >= o.open2 && dub >= o.dub &&
           chain >= o.chain && slots >= o.slots && cells >= o.cells;
  }
  void merge(const ArenaReq& o) {
    open3 = std::max(open3, o.open3);
    closed3 = std::max(closed3, o.closed3);
    open2 = std::max(open2, o.open2);
    dub = std::max(dub, o.dub);
    chain = std::max(chain, o.chain);
    slots = std::max(slots, o.slots);
    cells = std::max(cells, o.cells);
  }
};

// Sub-allocator for the planners' small device buffers (visited bitmap, motion tables, path
// output, obstacle lists).  hipMalloc hands out 2-MiB granules, so a planner whose maps
// (2 x 4 MiB at N = 1024) shared one allocation with these few hundred KiB used 10 MiB;
// here the maps are one exact allocation and the rest is carved from 64-MiB chunks.
// Freed blocks are kept per size and reused (planners of one configuration all ask for
// the same sizes).
struct SidePool {
  std::mutex mu;
  std::vector<void*> chunks;
  char* cur = nullptr;
  size_t left = 0;
  std::unordered_map<size_t, std::vector<void*>> freed;
  static size_t round(size_t b) { return (std::max<size_t>(b, 1) + 255) & ~(size_t)255; }
  hipError_t alloc(void** p, size_t bytes) {
    std::lock_guard<std::mutex> lk(mu);
    bytes = round(bytes);
    auto it = freed.find(bytes);
    if (it != freed.end() && !it->second.empty()) {
      *p = it->second.back();
      it->second.pop_back();
      return hipSuccess;
    }
    if (left < bytes) {
      const size_t sz = std::max<size_t>(bytes, (size_t)64 << 20);
      void* c = nullptr;
      const hipError_t e = hipMalloc(&c, sz);
      if (e != hipSuccess) return e;
      chunks.push_back(c);
      cur = static_cast<char*>(c);
      left = sz;
    }
    *p = cur;
    cur += bytes;
    left -= bytes;
    return hipSuccess;
  }
  void release(void* p, size_t bytes) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(mu);
    freed[round(bytes)].push_back(p);
  }
};

// Everything a device shares among its planners.
struct DeviceCtx {
  std::mutex mu;
  SidePool side;
  bool init = false;
  int device = -1;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  int resident_slots = 0;       // W: resident wavefronts of the search kernel
  int n_cu = 0;                 // compute units: workgroups of the latency (one-search-per-CU) kernel
  // Split launch of a large batch: the head of the longest-first queue runs on the latency
  // kernel on `head_cus` CUs, the rest on the batch kernel on the others, concurrently (two
  // streams forked from and joined into `stream`).  Every workgroup of either kernel takes a
  // whole CU's LDS, and the batch kernel gets n_cu - head_cus workgroups, so the two kernels
  // land on disjoint CUs whichever is dispatched first.
  int head_cus = 0;
  hipStream_t head_st = nullptr, bulk_st = nullptr;
  hipEvent_t ev_fork = nullptr, ev_head = nullptr, ev_bulk = nullptr, ev_hs = nullptr, ev_bs = nullptr;
  float split_ms[4] = {0, 0, 0, 0};  // last split launch: head start / end, bulk start / end after ev0
  // handoff board of split launches (HandoffBoard, hastar_layout.h): every pool and head arena
  // descriptor points at it; enabled only while a split launch runs
  HandoffBoard* d_board = nullptr;
  int handoffs = 0;                  // searches the last split launch handed to latency CUs
  // map-update scratch (relocation target + claim table, raster hit counters)
  size_t scratch_cap = 0;
  float* tmp = nullptr;
  int* winner = nullptr;        // kept at -1 between uses
  int* cnt = nullptr;           // kept at 0 between uses
  // slot arenas (one HBM slab)
  ArenaReq areq;
  int n_arenas = 0;
  int fit_arenas = 1 << 30;     // pool size the memory budget allowed at the last build
  void* slab = nullptr;
  SlotArena* d_arenas = nullptr;
  size_t arena_bytes = 0;       // bytes per arena of the current pool
  // batch buffers
  PlannerDev* d_descs = nullptr;
  int* d_order = nullptr;
  int* d_next = nullptr;
  bool kernels_warm = false;  // the search kernels' code objects are loaded (hastar_reserve)
  SearchResult* d_results = nullptr;
  SearchResult* h_results = nullptr;   // pinned
  long long* d_off = nullptr;          // path point offsets of the packed hand-back
  int* d_len = nullptr;
  long long* h_offlen = nullptr;       // pinned: n + 1 offsets then n lengths (as int)
  int batch_cap = 0;
  // packed paths of a batch (device staging + pinned host copy)
  float* d_pxyh = nullptr;
  float* d_pcurv = nullptr;
  float* h_pxyh = nullptr;
  float* h_pcurv = nullptr;
  size_t pts_cap = 0;
  uint32_t** d_ptrs = nullptr;  // bitmap pointers of a batched reset
  size_t ptrs_cap = 0;
  char* stage = nullptr;          // batched map updates: staged items / lists (grown, reused)
  size_t stage_cap = 0;
  char* bscratch = nullptr;       // batched relocation: bs_maps tmp maps, then bs_maps winner maps (-1)
  size_t bs_maps = 0, bs_nn = 0;  // capacity: maps x cells per map
  int last_n = 0;                 // the last batch's packed paths (d_pxyh/d_pcurv, offsets d_off)
  long long last_total = 0;
  char* vel_slab = nullptr;       // velocity-profile staging (grown, reused)
  size_t vel_cap = 0;
  // Head arenas of a split launch: after a search parked in a split launch, the latency CUs of
  // the next ones get arenas sized for it (so the head's longest searches run through without
  // waiting for the launch's end to resume): an allocation of their own when the HBM has room,
  // else carved from the pool's first head_n * head_k arenas (the bulk keeps the rest).
  // head_n = 0: none (the head uses plain pool arenas).
  int head_k = 0, head_n = 0;     // head_k: pool arenas per carved head arena (0: own allocation)
  void* head_slab = nullptr;      // the own allocation
  long long head_grant = 0;       // their outer capacity in pops (SlotArena::pops_grant)
  long long head_want = 0;        // pops of the longest search that outgrew its plain arena (windowed max)
  int head_extra = 0;             // latency CUs added to the head: such searches (windowed max)
  // the last kHeadWindow split launches' {longest outgrowing search, number of them}: head_want
  // and head_extra are their maxima, so a workload change lets the head shrink back
  long long head_win_pops[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int head_win_cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int head_win_at = 0;
  ArenaReq head_req;              // the requirement the head arenas were carved for
  int head_span = 0;
  SlotArena* d_head = nullptr;    // their descriptors (head_n); the head kernel's slot ids start at n_arenas
  std::vector<SlotArena> h_head;
  SlotArena* d_resume = nullptr;  // arena descriptors of a resume launch
  int* d_resume_order = nullptr;
  size_t resume_cap = 0;
  // relaxed-mode arenas (hastar_find_path_relaxed_batch): one per resident planner workgroup
  void* rslab = nullptr;
  RelaxArena* d_rarenas = nullptr;
  int n_rarenas = 0;
  size_t r_cells = 0;
  int r_nodes = 0, r_N = 0;
  int r_asked = 0;  // workgroups the pool was sized for (fewer when HBM capped it)
  RelaxField* d_rfields = nullptr;   // per-planner heuristic fields of a relaxed batch
  size_t rfields_cap = 0;
  signed char* d_dir = nullptr;      // per-pose directions of a relaxed batch (hastar_find_path_relaxed_batch_dir)
  size_t dir_cap = 0;
};

// A larger arena that continues one parked search (hastar_find_path_batch).
struct ResumeArena {
  void* slab = nullptr;  // own allocation (nullptr: carved from idle slot arenas of the pool)
  SlotArena desc{};
  int planner = -1;
  int pool_first = -1, pool_count = 0;  // pool arenas [first, first + count) it occupies
};
std::atomic<long long> g_pooled_resumes{0};  // resume arenas carved from the slot pool (diagnostics)
constexpr size_t kHeadroom = (size_t)2 << 30;  // HBM the arena pool and resume arenas leave free
DeviceCtx g_dev[64];

template <class T>
hipError_t side_alloc(DeviceCtx& D, T** p, size_t n) {
  return D.side.alloc(reinterpret_cast<void**>(p), std::max<size_t>(n, 1) * sizeof(T));
}
template <class T>
void side_free(DeviceCtx& D, T* p, size_t n) {
  D.side.release(p, std::max<size_t>(n, 1) * sizeof(T));
}

int device_ctx(int dev, DeviceCtx** out) {
  DeviceCtx& D = g_dev[dev & 63];
  if (!D.init) {
    D.device = dev;
    HIPCHK(hipSetDevice(dev));
    HIPCHK(hipStreamCreateWithFlags(&D.stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreate(&D.ev0));
    HIPCHK(hipEventCreate(&D.ev1));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, dev));
    D.resident_slots = search_slots_per_cu() * prop.multiProcessorCount;
    D.n_cu = prop.multiProcessorCount;
    // head CUs (HASTAR_HEAD_CUS, default 16; 0 = no split).  16 rather than 8: with 8, one step
    // in 6-10 ran every latency-CU search 1.6-1.9x slower; 56 steps with 16 showed none, at the
    // same mean (profiles/r03s_bench_h*.all.jsonl)
    int hc = 16;
    if (const char* e = std::getenv("HASTAR_HEAD_CUS")) hc = std::atoi(e);
    if (hc > 0 && D.n_cu >= 8 * hc) {
      if (hipStreamCreateWithFlags(&D.head_st, hipStreamNonBlocking) == hipSuccess &&
          hipStreamCreateWithFlags(&D.bulk_st, hipStreamNonBlocking) == hipSuccess &&
          hipEventCreateWithFlags(&D.ev_fork, hipEventDisableTiming) == hipSuccess &&
          hipEventCreate(&D.ev_head) == hipSuccess && hipEventCreate(&D.ev_bulk) == hipSuccess &&
          hipEventCreate(&D.ev_hs) == hipSuccess && hipEventCreate(&D.ev_bs) == hipSuccess) {
        D.head_cus = hc;
      } else {
        // a partial set is released and the split launch stays off (visible as head_cus = 0 in
        // hastar_debug_slots); said once, since results are unaffected
        for (hipStream_t* s : {&D.head_st, &D.bulk_st})
          if (*s) hipStreamDestroy(*s), *s = nullptr;
        for (hipEvent_t* e : {&D.ev_fork, &D.ev_head, &D.ev_bulk, &D.ev_hs, &D.ev_bs})
          if (*e) hipEventDestroy(*e), *e = nullptr;
        std::fprintf(stderr, "hastar: split launch disabled (stream/event creation failed)\n");
      }
    }
    HIPCHK(dalloc(&D.d_next, 4));  // [0] work counter, [1] head placement, [2] head done
    D.init = true;
  }
  *out = &D;
  return 0;
}

// the velocity-profile staging slab: grown on demand, kept (hipFree would synchronise the
// device, stalling a search batch in flight on it)
int vel_slab_acquire(DeviceCtx& D, size_t bytes) {
  if (D.vel_cap >= bytes) return 0;
  HIPCHK(hipStreamSynchronize(D.stream));
  if (D.vel_slab) hipFree(D.vel_slab);
  D.vel_slab = nullptr;
  D.vel_cap = 0;
  const size_t want = bytes + bytes / 2;
  if (hipMalloc(reinterpret_cast<void**>(&D.vel_slab), want) != hipSuccess) {
    D.vel_slab = nullptr;
    return fail(HASTAR_ENOMEM, "velocity_profile: hipMalloc failed");
  }
  D.vel_cap = want;
  return 0;
}

// device staging for the batched map updates (stream-ordered reuse; growth waits for the
// stream so no queued kernel still reads the old buffer)
int stage_acquire(DeviceCtx& D, size_t bytes) {
  if (D.stage_cap >= bytes) return 0;
  HIPCHK(hipStreamSynchronize(D.stream));
  if (D.stage) hipFree(D.stage);
  D.stage = nullptr;
  D.stage_cap = 0;
  const size_t want = bytes + bytes / 2 + 4096;
  if (hipMalloc(reinterpret_cast<void**>(&D.stage), want) != hipSuccess) {
    D.stage = nullptr;
    return fail(HASTAR_ENOMEM, "batched map update: staging hipMalloc failed");
  }
  D.stage_cap = want;
  return 0;
}
// relocation scratch for `maps` maps of up to NN cells: bs_maps tmp maps (floats) followed
// by bs_maps winner maps (ints), each bs_nn cells; the winner maps start (and stay) at -1
int bscratch_acquire(DeviceCtx& D, size_t maps, size_t NN) {
  if (D.bs_maps >= maps && D.bs_nn >= NN) return 0;
  HIPCHK(hipStreamSynchronize(D.stream));
  if (D.bscratch) hipFree(D.bscratch);
  D.bscratch = nullptr;
  D.bs_maps = D.bs_nn = 0;
  const size_t bytes = maps * NN * 8;
  if (hipMalloc(reinterpret_cast<void**>(&D.bscratch), bytes) != hipSuccess) {
    D.bscratch = nullptr;
    return fail(HASTAR_ENOMEM, "batched relocation: scratch hipMalloc failed");
  }
  HIPCHK(hipMemsetAsync(D.bscratch + maps * NN * 4, 0xff, maps * NN * 4, D.stream));
  D.bs_maps = maps;
  D.bs_nn = NN;
  return 0;
}

int scratch_acquire(DeviceCtx& D, size_t NN) {
  if (D.scratch_cap >= NN) return 0;
  if (D.tmp) hipFree(D.tmp);
  if (D.winner) hipFree(D.winner);
  if (D.cnt) hipFree(D.cnt);
  D.tmp = nullptr;
  D.winner = D.cnt = nullptr;
  D.scratch_cap = 0;
  HIPCHK(dalloc(&D.tmp, NN));
  HIPCHK(dalloc(&D.winner, NN));
  HIPCHK(dalloc(&D.cnt, NN));
  HIPCHK(hipMemsetAsync(D.winner, 0xff, NN * sizeof(int), D.stream));
  HIPCHK(hipMemsetAsync(D.cnt, 0, NN * sizeof(int), D.stream));
  D.scratch_cap = NN;
  return 0;
}

// Byte layout of one arena covering `r` (a slot arena of the pool, or a resume arena).
struct ArenaLayout {
  size_t open3, closed3, slots, open2, cell, gens, dub, dubc, chain, prevl;
  size_t total() const { return open3 + closed3 + slots + open2 + cell + gens + dub + dubc + chain + prevl; }
};
ArenaLayout arena_layout(const ArenaReq& r) {
  ArenaLayout L;
  L.open3 = align256((size_t)r.open3 * sizeof(Node3));
  L.closed3 = align256((size_t)r.closed3 * sizeof(Closed3));
  L.slots = align256((size_t)r.slots * sizeof(Slot3));
  L.open2 = align256((size_t)r.open2 * sizeof(Node2));
  L.cell = align256(r.cells * sizeof(Cell2));
  L.gens = 256;
  L.dub = align256((size_t)r.dub * 3 * sizeof(float));
  L.dubc = align256((size_t)r.dub * sizeof(float));
  L.chain = align256((size_t)r.chain * sizeof(int));
  L.prevl = align256((size_t)2048 * 2 * sizeof(int));  // {prev, g} per LDS A* node (any LDS pool size)
  return L;
}
// Carve the arena at `q` and queue the clearing of its generation-stamped tables.
hipError_t carve_arena(char* q, const ArenaReq& r, const ArenaLayout& L, SlotArena* out, hipStream_t st) {
  SlotArena& A = *out;
  std::memset(&A, 0, sizeof(A));
  A.open3 = reinterpret_cast<Node3*>(q); q += L.open3;
  A.closed3 = reinterpret_cast<Closed3*>(q); q += L.closed3;
  A.slots3 = reinterpret_cast<Slot3*>(q); q += L.slots;
  A.open2 = reinterpret_cast<Node2*>(q); q += L.open2;
  A.cell2 = reinterpret_cast<Cell2*>(q); q += L.cell;
  A.gens = reinterpret_cast<uint32_t*>(q); q += L.gens;
  A.dub_xyh = reinterpret_cast<float*>(q); q += L.dub;
  A.dub_curv = reinterpret_cast<float*>(q); q += L.dubc;
  A.out_chain = reinterpret_cast<int*>(q); q += L.chain;
  A.prevl = reinterpret_cast<int*>(q); q += L.prevl;
  A.open3_cap = r.open3;
  A.closed3_cap = r.closed3;
  A.slots3_mask = r.slots - 1;
  A.open2_cap = r.open2;
  A.cells = r.cells;
  A.dub_cap = r.dub;
  A.chain_cap = r.chain;
  // generation-stamped tables start at generation 0 (all stale)
  hipError_t e = hipMemsetAsync(A.slots3, 0, L.slots, st);
  if (e == hipSuccess) e = hipMemsetAsync(A.cell2, 0, L.cell, st);
  if (e == hipSuccess) e = hipMemsetAsync(A.gens, 0, L.gens, st);
  return e;
}
// Outer-search capacities of an arena for `pops` pops (a pop frees one open node and adds
// at most `span` successors; a replacement erases before it inserts).
void size_outer(ArenaReq& R, long long pops, int span) {
  R.open3 = (int)std::min<long long>(2 + (long long)(span - 1) * pops + 64, (long long)INT32_MAX / 2);
  R.closed3 = (int)std::min<long long>(pops + 1, (long long)SLOT3_IDX_MASK);
  R.slots = 1;
  while (R.slots < 2u * (uint32_t)R.closed3 + 64) R.slots <<= 1;
  R.chain = R.closed3 + 2;
}

// (Re)build the arena pool so that n arenas each cover `need`.
// The pool may come out smaller than n when n arenas do not fit the memory budget.
int arenas_acquire(DeviceCtx& D, const ArenaReq& need, int n) {
  if (D.n_arenas >= n && D.areq.covers(need)) return 0;
  if (D.n_arenas > 0 && D.areq.covers(need) && D.n_arenas >= D.fit_arenas) return 0;
  ArenaReq r = D.areq;
  r.merge(need);
  n = std::max(n, D.n_arenas);
  HIPCHK(hipStreamSynchronize(D.stream));
  if (D.slab) hipFree(D.slab);
  if (D.d_arenas) hipFree(D.d_arenas);
  D.slab = nullptr;
  D.d_arenas = nullptr;
  D.n_arenas = 0;
  // head arenas (carved from the old slab, or an own allocation sized for the old requirement)
  // do not outlive the pool: the next split launch carves them again for the new one
  if (D.head_slab) hipFree(D.head_slab);
  D.head_slab = nullptr;
  D.head_k = D.head_n = 0;
  D.head_grant = 0;
  const ArenaLayout lay = arena_layout(r);
  const size_t per = lay.total();
  // memory budget of the pool: HASTAR_ARENA_MB, else HASTAR_ARENA_FRAC (default 0.8) of
  // the free HBM
  size_t budget = 0;
  if (const char* e = std::getenv("HASTAR_ARENA_MB")) budget = (size_t)std::strtoull(e, nullptr, 10) << 20;
  if (budget == 0) {
    size_t fr = 0, tot = 0;
    HIPCHK(hipMemGetInfo(&fr, &tot));
    double frac = 0.8;
    if (const char* e = std::getenv("HASTAR_ARENA_FRAC")) frac = std::min(0.97, std::max(0.05, std::atof(e)));
    budget = (size_t)((double)fr * frac);
    // leave kHeadroom free for the runtime (code objects loaded at a kernel's first launch,
    // staging) and for the batch buffers
    budget = std::min(budget, fr > kHeadroom ? fr - kHeadroom : (size_t)0);
  }
  const int n_want = n;
  n = (int)std::max<size_t>(1, std::min<size_t>((size_t)n, budget / per));
  hipError_t e = hipMalloc(&D.slab, per * (size_t)n);
  if (e != hipSuccess) {
    D.slab = nullptr;
    return fail(HASTAR_ENOMEM, "search arenas: hipMalloc of " + std::to_string(per * (size_t)n >> 20) + " MiB failed");
  }
  if (!D.d_board) {
    HIPCHK(dalloc(&D.d_board, 1));
    HIPCHK(hipMemsetAsync(D.d_board, 0, sizeof(HandoffBoard), D.stream));
  }
  std::vector<SlotArena> host(n);
  char* base = static_cast<char*>(D.slab);
  for (int i = 0; i < n; ++i) {
    HIPCHK(carve_arena(base + per * (size_t)i, r, lay, &host[i], D.stream));
    host[i].board = D.d_board;
  }
  HIPCHK(dalloc(&D.d_arenas, (size_t)n));
  HIPCHK(hipMemcpyAsync(D.d_arenas, host.data(), (size_t)n * sizeof(SlotArena), hipMemcpyHostToDevice, D.stream));
  HIPCHK(hipStreamSynchronize(D.stream));
  D.areq = r;
  D.n_arenas = n;
  D.arena_bytes = per;
  D.fit_arenas = n < n_want ? n : (1 << 30);
  return 0;
}

// Head arenas released: the pool arenas a head carve took get their plain layout back (fresh
// generation-stamped tables; the descriptors in d_arenas never changed), an own allocation is
// freed.
int head_release(DeviceCtx& D) {
  if (D.head_n == 0) return 0;
  if (D.head_k > 0) {
    const ArenaLayout lay = arena_layout(D.areq);
    for (int q = 0; q < D.head_n * D.head_k; ++q) {
      SlotArena tmp;
      HIPCHK(carve_arena(static_cast<char*>(D.slab) + D.arena_bytes * (size_t)q, D.areq, lay, &tmp, D.stream));
    }
  }
  HIPCHK(hipStreamSynchronize(D.stream));
  if (D.head_slab) hipFree(D.head_slab);
  D.head_slab = nullptr;
  D.head_k = D.head_n = 0;
  D.head_grant = 0;
  return 0;
}

// Head arenas for a split launch with `head` latency CUs, each holding a search of head_want
// pops (+25 %): an own allocation when the HBM keeps kHeadroom beside it, else k consecutive
// pool arenas each, while at most a third of the launch's `slots` arenas go to them.  None
// when no search needs them or neither way has the room.
int head_acquire(DeviceCtx& D, int head, int span, int slots) {
  // (a parked search outgrew its planner's capacity rule, P.arena_pops << 2 parks, whatever
  // the pool arena's size: the grant lifts that rule in the head arenas, hastar_kernels.hip)
  if (D.head_want <= 0 || D.arena_bytes == 0) return head_release(D);
  const long long grant = std::min(D.head_want + D.head_want / 4, (long long)SLOT3_IDX_MASK - 1);
  // reuse the current head arenas only when they were carved for this pool's requirement (a
  // larger grid or inner capacity that joined the device since rebuilt the pool, and a wider
  // span needs more open nodes per pop)
  if (D.head_n == head && D.head_grant == grant && D.head_req.covers(D.areq) && D.head_span >= span) return 0;
  if (int rc = head_release(D)) return rc;
  ArenaReq r = D.areq;
  size_outer(r, grant, span);
  r.merge(D.areq);
  const ArenaLayout lay = arena_layout(r);
  const size_t each = lay.total();
  size_t fr = 0, tot = 0;
  int k = 0;
  if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr > each * (size_t)head + kHeadroom &&
      hipMalloc(&D.head_slab, each * (size_t)head) == hipSuccess) {
    k = 0;
  } else {
    D.head_slab = nullptr;
    k = (int)((each + D.arena_bytes - 1) / D.arena_bytes);
    if ((long long)head * k > slots / 3) return 0;  // the bulk would lose too many arenas
  }
  D.h_head.assign((size_t)head, SlotArena{});
  for (int b = 0; b < head; ++b) {
    char* at = D.head_slab ? static_cast<char*>(D.head_slab) + each * (size_t)b
                           : static_cast<char*>(D.slab) + D.arena_bytes * (size_t)b * k;
    HIPCHK(carve_arena(at, r, lay, &D.h_head[(size_t)b], D.stream));
    D.h_head[(size_t)b].pops_grant = (int)grant;
    D.h_head[(size_t)b].board = D.d_board;
  }
  if (D.d_head) hipFree(D.d_head);
  D.d_head = nullptr;
  HIPCHK(dalloc(&D.d_head, (size_t)head));
  HIPCHK(hipMemcpyAsync(D.d_head, D.h_head.data(), (size_t)head * sizeof(SlotArena), hipMemcpyHostToDevice, D.stream));
  HIPCHK(hipStreamSynchronize(D.stream));
  D.head_k = k;
  D.head_n = head;
  D.head_grant = grant;
  D.head_req = r;
  D.head_span = span;
  return 0;
}

}  // namespace

struct hastar_handle_s {
  int device = 0;
  DeviceCtx* dc = nullptr;
  PlannerDev desc{};            // host copy of the descriptor (device copies are batch-local)
  float lp_min = 0, lp_max = 0, lp_free = 0;
  int max_pops = 0;              // initial outer-search arena capacity in pops
  int span = 2;
  ArenaReq areq;
  std::vector<float> curv_abs;
  // grid-frame state (Grid2D::_grid_heading/_goal_location, Grid3D::_goal_location3D)
  float grid_heading = 0, goal2x = 0, goal2y = 0, goal3x = 0, goal3y = 0, goal3h = 0;
  bool goal_set = false;
  // per-call upload buffers
  int apf_cap = 0;
  int* d_rp = nullptr;
  float* d_dl = nullptr;
  int rp_cap = 0;
  int* d_ids = nullptr;          // box indices grouped by raster layer
  int ids_cap = 0;
  float* d_lp = nullptr;
  float* d_seq = nullptr;
  float* d_wid = nullptr;
  int lp_cap = 0, wid_cap = 0;
  void* slab = nullptr;         // the planner's maps (log-odds + node-map f), one exact allocation
  void* side = nullptr;         // bitmap, motion tables, path output: from the device's SidePool
  size_t side_bytes = 0;
  SearchResult last{};
  bool have_last = false;
  long long last_pops = 0;      // work estimate for longest-first scheduling (last search's duration)
  long long prev_pops = 0;      // the one before (the key is the longer of the two: a replan loop
                                // whose long searches alternate with short ones stays at the head)
  std::vector<float> boxes_w;   // the last update_obstacles(boxes) call's boxes (world frame): cold-order key
  int row0 = 0, row1 = 0;       // map-build row window [row0, row1) (hastar_set_row_window); [0, N) by default
  std::shared_ptr<struct BatchSlab> batch;  // planners of one hastar_create_batch_f32 share it
  // relaxed mode's own heuristic field (hastar_relaxed_opts.reuse_heuristic): kept until
  // reset() / update_goal(), like the exact mode's memo
  float* rfield = nullptr;
  bool rvalid = false;
  float rhlim = 0.0f;
  int rstart = 0;
  int rcoarse = 0;              // the kept field's block side (a call with another one rebuilds it)
};

// One allocation for the persistent state of a batch of identical planners
// (hastar_create_batch_f32): per planner the log-odds map, node-map f plane, memo bitmap and
// path output, plus one shared copy of the read-only motion tables.  Freed with the last
// planner of the batch.
struct BatchSlab {
  void* slab = nullptr;
  void* tables = nullptr;
  int device = 0;
  ~BatchSlab() {
    hipSetDevice(device);
    if (slab) hipFree(slab);
    if (tables) hipFree(tables);
  }
};

static void free_handle(hastar_handle h) {
  if (!h) return;
  hipSetDevice(h->device);
  if (h->dc) hipStreamSynchronize(h->dc->stream);
  if (h->slab) hipFree(h->slab);
  if (h->rfield) hipFree(h->rfield);
  if (h->dc) {
    DeviceCtx& DC = *h->dc;
    if (h->side) DC.side.release(h->side, h->side_bytes);
    side_free(DC, h->d_rp, (size_t)h->rp_cap * 4);
    side_free(DC, h->d_dl, (size_t)h->rp_cap);
    side_free(DC, h->d_ids, (size_t)h->ids_cap);
    side_free(DC, h->d_lp, (size_t)h->lp_cap * 9);
    side_free(DC, h->d_seq, (size_t)h->lp_cap * 100);
    side_free(DC, h->d_wid, (size_t)h->wid_cap);
    side_free(DC, h->desc.apf, (size_t)h->apf_cap * 3);
  }
  delete h;
}

// work(a, b) over [0, n), spread over up to 16 host threads for large n
template <class F>
static void host_parallel(int n, F&& work) {
  const int nt = n >= 256 ? (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency())) : 1;
  if (nt <= 1) {
    work(0, n);
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; ++t) pool.emplace_back(work, (int)((long long)n * t / nt), (int)((long long)n * (t + 1) / nt));
  for (auto& th : pool) th.join();
}

extern "C" {

const char* hastar_last_error(void) { return g_err.c_str(); }
float hastar_last_search_ms(void) { return g_last_ms; }
int hastar_grid_size(hastar_handle h) { return h ? h->desc.N : HASTAR_EINVAL; }

// Host half of the constructor (HybridAStar.cpp:7-24 and the member constructors it runs):
// every scalar of the planner descriptor, its arena requirements, and the motion tables
// (VehicleModel.cpp:7-47), which the caller uploads (one copy per planner, or one shared
// copy for a batch of identical planners).
struct HostTables {
  std::vector<float> off, dth, cost;
};
static hastar_handle new_planner(const hastar_params* p, int device, DeviceCtx* dc, HostTables& T) {
  hastar_handle h = new hastar_handle_s();
  h->device = device;
  h->dc = dc;
  PlannerDev& D = h->desc;
  const int N = p->grid_size;
  D.N = N;
  h->row0 = 0;
  h->row1 = N;
  D.n2 = (int)std::round(N * 0.5);
  D.n45 = (int)std::round(N * 0.8);
  D.diag = p->grid_2d_allow_diag_moves ? 1 : 0;
  D.bins = p->num_angle_bins;
  D.nsteer = p->num_steering;
  D.na = p->num_actions;
  D.shot_interval = p->dubins_shot_interval;
  D.shot_decay = p->dubins_shot_interval_decay;
  D.res = p->grid_resolution;
  // Grid2D.cpp:9-12: log-odds of the probability parameters (double log, stored as T)
  auto logodds = [](float pr) { return (float)std::log((double)pr / (1.0 - (double)pr)); };
  D.thr = logodds(p->obstacle_threshold);
  h->lp_min = logodds(p->obstacle_prob_min);
  h->lp_max = logodds(p->obstacle_prob_max);
  h->lp_free = logodds(p->obstacle_prob_free);
  D.apf_rep = p->apf_rep_constant;
  D.apf_ang = p->apf_active_angle;
  D.act_cost_axis = D.res * std::sqrt(1.0f);   // Grid2D.cpp:54-58
  D.act_cost_diag = D.res * std::sqrt(2.0f);
  // VehicleModel (VehicleModel.cpp:7-47)
  D.ts = p->step_size;
  D.a_lat = p->max_lat_acc;
  D.a_lat2 = p->max_lat_acc * p->max_lat_acc;
  D.prec = (float)(2 * M_PI / D.bins);
  const int ns = D.nsteer, bins = D.bins;
  std::vector<float> beta(ns), curv(ns);
  std::vector<float>& dth = T.dth;
  std::vector<float>& cost = T.cost;
  std::vector<float>& off = T.off;
  dth.assign(ns, 0.0f);
  cost.assign(ns, 0.0f);
  off.assign((size_t)ns * (bins + 1) * 2, 0.0f);
  for (int i = 0; i < ns; ++i) {
    beta[i] = g_atan2f(p->rear_to_cg * std::tan(p->steering[i]), p->wheelbase);
    curv[i] = g_cosf(beta[i]) * std::tan(p->steering[i]) / p->wheelbase;
  }
  for (int i = 0; i < ns; ++i) {
    dth[i] = D.ts * curv[i];
    cost[i] = D.ts + p->curvature_weights[i] * std::fabs(curv[i]);
    for (int j = 0; j < bins; ++j) {
      const float head = (float)(-M_PI + (double)((float)j * D.prec));
      const float dt = 0.001f;  // VehicleModel::calculate_offset (VehicleModel.cpp:147-164)
      float ox = 0.0f, oy = 0.0f, hh = head;
      const int nup = (int)(D.ts / dt);
      for (int k = 0; k < nup; ++k) {
        ox += dt * g_cosf(beta[i] + hh);
        oy += dt * g_sinf(beta[i] + hh);
        hh += dt * curv[i];
      }
      off[2 * ((size_t)i * (bins + 1) + j)] = ox;
      off[2 * ((size_t)i * (bins + 1) + j) + 1] = oy;
    }
    // row `bins` stays (0, 0): the reference's one-past-the-end read (VehicleModel.cpp:145)
  }
  h->curv_abs.resize(ns);
  for (int i = 0; i < ns; ++i) h->curv_abs[i] = std::fabs(curv[i]);
  // APF culling radius: a successor lies within max |offset| per axis of its parent (plus
  // the rounding of parent + offset; the margin covers it many times over)
  float max_off = 0.0f;
  for (float v : off) max_off = std::max(max_off, std::fabs(v));
  D.apf_reach = max_off * 1.001f + 0.01f;
  // Dubins radius (HybridAStar.cpp:22-24, tan_max HybridAStar.h:20-25)
  const float tmax = std::tan(*std::max_element(p->steering, p->steering + ns));
  D.r_min = p->wheelbase / (g_cosf(g_atan2f(p->rear_to_cg * tmax, p->wheelbase)) * tmax);
  D.step = p->step_size;
  D.ang_step = p->step_size / D.r_min;

  // arena requirements of this planner
  const size_t NN = (size_t)N * N;
  h->max_pops = p->max_pops > 0 ? p->max_pops : 262144;
  ArenaReq& R = h->areq;
  // live open nodes: each pop removes one and adds at most `span` successors (a
  // replacement erases before it inserts), so after max_pops pops at most
  // 1 + max_pops * (span - 1) are live; freed nodes are reused before the pool grows
  const int span = std::max(2, std::min(2 * D.na + 1, D.nsteer));
  h->span = span;
  D.arena_pops = h->max_pops;
  D.span_alloc = span;
  size_outer(R, h->max_pops, span);
  // inner A*: the closed records are bounded by the cells (N^2); the open tree by its
  // frontier, which stays far below N^2 (max_astar_nodes, default min(N^2 + 16, 65536))
  const int astar_cap =
      p->max_astar_nodes > 0 ? p->max_astar_nodes : (int)std::min<size_t>(NN + 16, (size_t)65536);
  R.open2 = astar_cap + 1;
  D.astar_cap = astar_cap + 1;  // the planner's own bound: an arena of the pool may hold more
  R.cells = NN;
  int dub_cap = p->max_dubins_samples;
  if (dub_cap <= 0) {
    const double span = 2.0 * N * D.res;
    dub_cap = (int)(span / D.step) + 2 * (int)(2 * M_PI / D.ang_step + 2) + 64;
  }
  R.dub = dub_cap;
  // path buffer of the planner: Dubins samples + the prev chain of the terminal node.  A
  // chain visits distinct (cell, bin) keys one step apart, so 8 N poses cover any
  // realistic path; a longer one ends the search with HASTAR_ENOSPC (reported, never
  // truncated).
  D.out_cap = dub_cap + std::min(h->max_pops + 2, 8 * N + 64);

  return h;
}

static int check_params(const hastar_params* p) {
  if (p->grid_size < 2 || p->grid_size > 4095) return fail(HASTAR_EINVAL, "grid_size must be in [2, 4095]");
  if (p->num_angle_bins < 1 || p->num_angle_bins > 254) return fail(HASTAR_EINVAL, "num_angle_bins must be in [1, 254]");
  if (p->num_steering < 1 || p->num_steering > 16 || !p->steering || !p->curvature_weights)
    return fail(HASTAR_EINVAL, "num_steering must be in [1, 16] with steering/curvature_weights arrays");
  if (p->num_actions < 0) return fail(HASTAR_EINVAL, "num_actions must be >= 0");
  if (p->max_pops > (int)SLOT3_IDX_MASK - 1) return fail(HASTAR_EINVAL, "max_pops must be below 2^24 - 1");
  if (p->max_pops < 0) return fail(HASTAR_EINVAL, "max_pops must be >= 0");
  if (!(p->grid_resolution > 0) || !(p->step_size > 0)) return fail(HASTAR_EINVAL, "resolution/step must be > 0");
  return 0;
}

// HybridAStar::HybridAStar (HybridAStar.cpp:7-24) and the member constructors it runs:
// Grid2D (Grid2D.cpp:7-62), VehicleModel (VehicleModel.cpp:7-47), Dubins (Dubins.cpp:7-16).
int hastar_create_f32(const hastar_params* p, int device, hastar_handle* out) {
  if (!p || !out) return fail(HASTAR_EINVAL, "null argument");
  *out = nullptr;
  if (int rc = check_params(p)) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(HASTAR_EDEVICE, "no HIP device available (this library has no CPU path)");
  if (device < 0 || device >= ndev || device >= 64) return fail(HASTAR_EINVAL, "device ordinal out of range");
  DeviceCtx* dc = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_dev[device].mu);
    if (int rc = device_ctx(device, &dc)) return rc;
  }
  HIPCHK(hipSetDevice(device));

  HostTables T;
  hastar_handle h = new_planner(p, device, dc, T);
  PlannerDev& D = h->desc;
  const int N = D.N;
  const int ns = D.nsteer;
  const size_t NN = (size_t)N * N;
  std::vector<float>& off = T.off;
  std::vector<float>& dth = T.dth;
  std::vector<float>& cost = T.cost;
  // the planner's persistent state: the two N x N maps in one exact allocation (8 MiB at
  // N = 1024, a whole number of 2-MiB granules), everything else from the device's pool
  const size_t b_occ = align256(NN * sizeof(float)), b_nm = align256(NN * sizeof(float));
  const size_t b_vis = align256(bitmap_words(NN) * sizeof(uint32_t));
  const size_t b_off = align256(off.size() * sizeof(float)), b_s = align256((size_t)ns * sizeof(float));
  const size_t b_ox = align256((size_t)D.out_cap * 3 * sizeof(float)), b_oc = align256((size_t)D.out_cap * sizeof(float));
  h->side_bytes = b_vis + b_off + 3 * b_s + b_ox + b_oc;
  if (hipMalloc(&h->slab, b_occ + b_nm) != hipSuccess) {
    h->slab = nullptr;
    free_handle(h);
    return fail(HASTAR_ENOMEM, "planner state allocation failed");
  }
  if (dc->side.alloc(&h->side, h->side_bytes) != hipSuccess) {
    h->side = nullptr;
    free_handle(h);
    return fail(HASTAR_ENOMEM, "planner side-buffer allocation failed");
  }
  char* q = static_cast<char*>(h->slab);
  D.occ = reinterpret_cast<float*>(q); q += b_occ;
  D.nm_f = reinterpret_cast<float*>(q); q += b_nm;
  q = static_cast<char*>(h->side);
  D.visited = reinterpret_cast<uint32_t*>(q); q += b_vis;
  D.off = reinterpret_cast<float*>(q); q += b_off;
  D.dth = reinterpret_cast<float*>(q); q += b_s;
  D.act_cost = reinterpret_cast<float*>(q); q += b_s;
  D.curv_abs = reinterpret_cast<float*>(q); q += b_s;
  D.out_xyh = reinterpret_cast<float*>(q); q += b_ox;
  D.out_curv = reinterpret_cast<float*>(q); q += b_oc;
  D.result = nullptr;  // set per batch to the device context's result array
  D.apf = nullptr;
  D.n_apf = 0;
  hipStream_t st = dc->stream;
  hipError_t he = hipMemsetAsync(D.occ, 0, NN * sizeof(float), st);
  if (he == hipSuccess) he = hipMemsetAsync(D.visited, 0, bitmap_words(NN) * sizeof(uint32_t), st);
  if (he == hipSuccess) he = hipMemcpyAsync(D.off, off.data(), off.size() * sizeof(float), hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = hipMemcpyAsync(D.dth, dth.data(), ns * sizeof(float), hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = hipMemcpyAsync(D.act_cost, cost.data(), ns * sizeof(float), hipMemcpyHostToDevice, st);
  if (he == hipSuccess)
    he = hipMemcpyAsync(D.curv_abs, h->curv_abs.data(), ns * sizeof(float), hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = launch_init_nodemap(D, st);
  if (he == hipSuccess) he = hipStreamSynchronize(st);  // the host vectors above go out of scope
  if (he != hipSuccess) {
    free_handle(h);
    return fail(HASTAR_EDEVICE, std::string("init: ") + hipGetErrorString(he));
  }
  *out = h;
  return HASTAR_OK;
}

// n planners with the same constructor arguments (a batch of independent queries): one
// allocation for all their maps, one shared copy of the motion tables, one initialisation
// launch and one synchronisation, instead of n of each.  out[i] are independent handles
// (each behaves exactly like one from hastar_create_f32); the shared memory is released
// with the last of them.
int hastar_create_batch_f32(const hastar_params* p, int n, int device, hastar_handle* out) {
  if (!p || !out || n < 0) return fail(HASTAR_EINVAL, "bad argument");
  if (n == 0) return HASTAR_OK;
  for (int i = 0; i < n; ++i) out[i] = nullptr;
  if (int rc = check_params(p)) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(HASTAR_EDEVICE, "no HIP device available (this library has no CPU path)");
  if (device < 0 || device >= ndev || device >= 64) return fail(HASTAR_EINVAL, "device ordinal out of range");
  DeviceCtx* dc = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_dev[device].mu);
    if (int rc = device_ctx(device, &dc)) return rc;
  }
  HIPCHK(hipSetDevice(device));
  HostTables T;
  hastar_handle h0 = new_planner(p, device, dc, T);
  const PlannerDev D0 = h0->desc;
  const size_t NN = (size_t)D0.N * D0.N;
  const int ns = D0.nsteer;
  const size_t b_map = align256(NN * sizeof(float)), b_vis = align256(bitmap_words(NN) * sizeof(uint32_t));
  const size_t b_ox = align256((size_t)D0.out_cap * 3 * sizeof(float)), b_oc = align256((size_t)D0.out_cap * sizeof(float));
  const size_t stride = 2 * b_map + b_vis + b_ox + b_oc;
  const size_t b_off = align256(T.off.size() * sizeof(float)), b_s = align256((size_t)ns * sizeof(float));
  auto bs = std::make_shared<BatchSlab>();
  bs->device = device;
  if (hipMalloc(&bs->slab, stride * (size_t)n) != hipSuccess || hipMalloc(&bs->tables, b_off + 3 * b_s) != hipSuccess) {
    delete h0;
    return fail(HASTAR_ENOMEM, "batch planner state allocation failed (" + std::to_string(stride * (size_t)n >> 20) + " MiB)");
  }
  char* t = static_cast<char*>(bs->tables);
  float* d_off = reinterpret_cast<float*>(t);
  float* d_dth = reinterpret_cast<float*>(t + b_off);
  float* d_cost = reinterpret_cast<float*>(t + b_off + b_s);
  float* d_ca = reinterpret_cast<float*>(t + b_off + 2 * b_s);
  hipStream_t st = dc->stream;
  hipError_t he = hipMemsetAsync(bs->slab, 0, stride * (size_t)n, st);
  if (he == hipSuccess) he = hipMemcpyAsync(d_off, T.off.data(), T.off.size() * sizeof(float), hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = hipMemcpyAsync(d_dth, T.dth.data(), ns * sizeof(float), hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = hipMemcpyAsync(d_cost, T.cost.data(), ns * sizeof(float), hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = hipMemcpyAsync(d_ca, h0->curv_abs.data(), ns * sizeof(float), hipMemcpyHostToDevice, st);
  for (int i = 0; i < n && he == hipSuccess; ++i) {
    hastar_handle h = i == 0 ? h0 : new hastar_handle_s(*h0);
    char* q = static_cast<char*>(bs->slab) + stride * (size_t)i;
    PlannerDev& D = h->desc;
    D.occ = reinterpret_cast<float*>(q);
    D.nm_f = reinterpret_cast<float*>(q + b_map);
    D.visited = reinterpret_cast<uint32_t*>(q + 2 * b_map);
    D.out_xyh = reinterpret_cast<float*>(q + 2 * b_map + b_vis);
    D.out_curv = reinterpret_cast<float*>(q + 2 * b_map + b_vis + b_ox);
    D.off = d_off;
    D.dth = d_dth;
    D.act_cost = d_cost;
    D.curv_abs = d_ca;
    D.result = nullptr;
    D.apf = nullptr;
    D.n_apf = 0;
    h->slab = nullptr;
    h->side = nullptr;
    h->side_bytes = 0;
    h->batch = bs;
    out[i] = h;
  }
  // the node-map f planes (Grid2D ctor + compute_heuristic) of every planner in one launch
  if (he == hipSuccess) he = launch_init_nodemap_batch(out[0]->desc, static_cast<char*>(bs->slab) + b_map, stride, n, st);
  if (he == hipSuccess) he = hipStreamSynchronize(st);
  if (he != hipSuccess) {
    // h0 is out[0] unless an async call failed before the handle loop stored it
    if (out[0] != h0) delete h0;
    for (int i = 0; i < n; ++i) {
      if (out[i]) delete out[i];
      out[i] = nullptr;
    }
    return fail(HASTAR_EDEVICE, std::string("batch init: ") + hipGetErrorString(he));
  }
  return HASTAR_OK;
}

int hastar_destroy(hastar_handle h) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  free_handle(h);
  return HASTAR_OK;
}

// HybridAStar::update_goal -> Grid3D::update_goal_heading + relocate_obstacles
// (Grid3D.cpp:102-124, 169-203); AStar::update_goal_node takes the goal cell.
struct RelocPrep {
  float c, s, ox, oy;
};
// Host half of update_goal: the new grid frame, the goal node, and the rotation + origin of
// the map relocation (Grid3D.cpp:102-124, 169-203), with the reference's float arithmetic.
static RelocPrep goal_prep(hastar_handle h, const float goal[3], const float start[3]);
static int update_boxes_legacy(hastar_handle h, const float* boxes, const float* conf, int n, float apf_added_radius);
static int update_boxes_impl(const hastar_handle* hs, int n, const float* boxes, const float* conf, const int* counts,
                             float apf_added_radius);

// Relocate the maps of `items` (distinct maps; DC.mu held) in chunks that share one scratch
// allocation: every destination finds its winning source by inverting the rotation
// (k_relocate_invert_batch, no claim table), then the chunk is copied back.  A chunk's scratch
// maps total <= HASTAR_RELOC_CHUNK_MB (default 256 MB; 16 MB-1 GB measured within 2 % of each
// other from 32 MB up, profiles/r06g_reloc_chunk_sweep.txt).  HASTAR_RELOC=claim selects the
// round-5 passes (atomic claim, gather, copy; <= 1 GiB of claim tables) for A/B measurements.
static int relocate_maps(DeviceCtx& DC, std::vector<RelocItem>& items, size_t NNmax) {
  const int n = (int)items.size();
  if (n == 0) return HASTAR_OK;
  static const bool claim = [] {
    const char* e = std::getenv("HASTAR_RELOC");
    return e && std::string(e) == "claim";
  }();
  static const size_t chunk_bytes = [] {
    const char* e = std::getenv("HASTAR_RELOC_CHUNK_MB");
    return (size_t)(e ? std::max(1, std::atoi(e)) : 256) << 20;
  }();
  const int chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)n, chunk_bytes / (claim ? 8 * NNmax : 4 * NNmax)));
  if (int rc = bscratch_acquire(DC, (size_t)chunk, NNmax)) return rc;
  if (int rc = stage_acquire(DC, (size_t)n * sizeof(RelocItem))) return rc;
  float* tmp0 = reinterpret_cast<float*>(DC.bscratch);
  int* win0 = reinterpret_cast<int*>(DC.bscratch + DC.bs_maps * DC.bs_nn * 4);
  for (int i = 0; i < n; ++i) {
    items[i].tmp = tmp0 + (size_t)(i % chunk) * DC.bs_nn;
    items[i].winner = win0 + (size_t)(i % chunk) * DC.bs_nn;
  }
  HIPCHK(hipMemcpyAsync(DC.stage, items.data(), (size_t)n * sizeof(RelocItem), hipMemcpyHostToDevice, DC.stream));
  const RelocItem* d_items = reinterpret_cast<const RelocItem*>(DC.stage);
  for (int c0 = 0; c0 < n; c0 += chunk) {
    if (claim) HIPCHK(launch_relocate_batch(d_items + c0, std::min(chunk, n - c0), NNmax, DC.stream));
    else HIPCHK(launch_relocate_invert(d_items + c0, std::min(chunk, n - c0), NNmax, DC.stream));
  }
  return HASTAR_OK;
}

int hastar_update_goal(hastar_handle h, const float goal[3], const float start[3]) {
  if (!h || !goal || !start) return fail(HASTAR_EINVAL, "null argument");
  HIPCHK(hipSetDevice(h->device));
  DeviceCtx& DC = *h->dc;
  PlannerDev& D = h->desc;
  const RelocPrep rp = goal_prep(h, goal, start);
  std::lock_guard<std::mutex> lk(DC.mu);
  std::vector<RelocItem> items{RelocItem{D.occ, nullptr, nullptr, D.N, rp.c, rp.s, rp.ox, rp.oy, 0}};
  return relocate_maps(DC, items, (size_t)D.N * D.N);
}

static RelocPrep goal_prep(hastar_handle h, const float goal[3], const float start[3]) {
  PlannerDev& D = h->desc;
  const float gh_prev = h->grid_heading;
  const float g3px = h->goal3x, g3py = h->goal3y;
  h->goal2x = goal[0];
  h->goal2y = goal[1];
  h->grid_heading = g_atan2f(goal[1] - start[1], goal[0] - start[0]);
  h->goal3x = goal[0];
  h->goal3y = goal[1];
  h->goal3h = goal[2];
  const float gh = h->grid_heading;
  const float dh = gh - gh_prev;
  const V2 gp = rot2((float)D.n45, (float)D.n2, dh);
  const V2 gno = rot2(g3px - h->goal3x, g3py - h->goal3y, gh);
  V2 org{(float)D.n45 + gno.x / D.res, (float)D.n2 + gno.y / D.res};
  org = {org.x - gp.x, org.y - gp.y};
  const RelocPrep out{g_cosf(dh), g_sinf(dh), org.x, org.y};
  // the goal node (Grid3D.cpp:115-123)
  D.goal_x = D.n45 * D.res;
  D.goal_y = D.n2 * D.res;
  D.goal_h = wrap_pi_h(goal[2] - gh);
  D.goal_bin = heading_bin_h(D.goal_h, D.prec);
  D.goal_cx = D.n45;
  D.goal_cy = D.n2;
  D.world_goal_x = goal[0];
  D.world_goal_y = goal[1];
  D.grid_heading = gh;
  D.rot_c = g_cosf(-gh);
  D.rot_s = g_sinf(-gh);
  h->goal_set = true;
  h->rvalid = false;
  return out;
}

// HybridAStar::reset -> AStar::reset (AStar.cpp:56-60)
int hastar_reset(hastar_handle h) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  HIPCHK(hipSetDevice(h->device));
  h->rvalid = false;
  // the memo flags are a bitmap (N*N / 8 bytes): reset clears it
  const PlannerDev& D = h->desc;
  HIPCHK(hipMemsetAsync(D.visited, 0, bitmap_words((size_t)D.N * D.N) * sizeof(uint32_t), h->dc->stream));
  return HASTAR_OK;
}

// the caller's longest-first key of the planner's next batched search (include/hastar.h)
int hastar_set_cost_hint(hastar_handle h, long long hint) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  h->last_pops = hint;
  h->prev_pops = 0;
  return HASTAR_OK;
}

// reset() of n planners: one kernel clears every bitmap of a device (planners grouped by
// device and grid size)
int hastar_reset_batch(const hastar_handle* hs, int n) {
  if (!hs || n < 0) return fail(HASTAR_EINVAL, "bad argument");
  for (int i = 0; i < n; ++i)
    if (!hs[i]) return fail(HASTAR_EINVAL, "null handle");
  for (int i = 0; i < n; ++i) hs[i]->rvalid = false;
  std::vector<char> done(n, 0);
  for (int i = 0; i < n; ++i) {
    if (done[i]) continue;
    const int dev = hs[i]->device, N = hs[i]->desc.N;
    std::vector<uint32_t*> ptrs;
    for (int j = i; j < n; ++j)
      if (!done[j] && hs[j]->device == dev && hs[j]->desc.N == N) {
        ptrs.push_back(hs[j]->desc.visited);
        done[j] = 1;
      }
    HIPCHK(hipSetDevice(dev));
    DeviceCtx& DC = *hs[i]->dc;
    std::lock_guard<std::mutex> lk(DC.mu);
    if (ptrs.size() > DC.ptrs_cap) {
      HIPCHK(hipStreamSynchronize(DC.stream));
      if (DC.d_ptrs) hipFree(DC.d_ptrs);
      DC.d_ptrs = nullptr;
      DC.ptrs_cap = 0;
      HIPCHK(hipMalloc(reinterpret_cast<void**>(&DC.d_ptrs), ptrs.size() * sizeof(uint32_t*)));
      DC.ptrs_cap = ptrs.size();
    }
    // pageable source: the copy is staged before hipMemcpyAsync returns
    HIPCHK(hipMemcpyAsync(DC.d_ptrs, ptrs.data(), ptrs.size() * sizeof(uint32_t*), hipMemcpyHostToDevice, DC.stream));
    HIPCHK(launch_clear_bitmaps(DC.d_ptrs, (int)ptrs.size(), bitmap_words((size_t)N * N), DC.stream));
  }
  return HASTAR_OK;
}

// Host half of Grid3D::update_obstacles(boxes) for one planner: the APF list in the grid
// frame (Grid3D.cpp:22-44), each box's sub-sample origin and counts and log-odds delta
// (Grid2D.cpp:99-139), and its raster footprint and layer.  Layers: box k goes one layer
// above every earlier box whose footprint it may share, so boxes within a layer touch
// disjoint cells (applied concurrently) and overlapping boxes are applied in the
// reference's order.  Footprint: the rotated sub-sample rectangle's bounds plus a 2-cell
// margin for rounding.
struct BoxPrep {
  std::vector<float> apf, dl;
  std::vector<int> rp, bb, layer;
  int n_layers = 0;
  bool big = false;  // some footprint exceeds RASTER_HIST cells
};
static void boxes_prep(hastar_handle h, const float* boxes, const float* conf, int n, float apf_added_radius,
                       BoxPrep& P) {
  const PlannerDev& D = h->desc;
  const float gh = h->grid_heading;
  P.apf.resize((size_t)n * 3);
  P.rp.resize((size_t)n * 4);
  P.dl.resize((size_t)n);
  P.bb.resize((size_t)n * 4);
  P.layer.assign((size_t)n, 0);
  P.n_layers = 0;
  P.big = false;
  const float cg = g_cosf(gh), sg = g_sinf(gh);
  for (int k = 0; k < n; ++k) {
    const float ox = boxes[4 * k], oy = boxes[4 * k + 1], dx = boxes[4 * k + 2], dy = boxes[4 * k + 3];
    V2 pp = rot2(ox - h->goal3x, oy - h->goal3y, gh);
    pp.x += D.n45 * D.res;
    pp.y += D.n2 * D.res;
    P.apf[3 * k] = pp.x;
    P.apf[3 * k + 1] = pp.y;
    P.apf[3 * k + 2] = std::max(dx, dy) / 2 + apf_added_radius;
    const V2 bl = rot2((ox - dx / 2) - h->goal2x, (oy - dy / 2) - h->goal2y, gh);
    int* rp = &P.rp[4 * k];
    rp[0] = gmath::x86_trunc_int(std::round(bl.x / D.res) + (float)D.n45);
    rp[1] = gmath::x86_trunc_int(std::round(bl.y / D.res) + (float)D.n2);
    rp[2] = std::max(0, 2 * gmath::x86_trunc_int(std::ceil(dx / D.res)));
    rp[3] = std::max(0, 2 * gmath::x86_trunc_int(std::ceil(dy / D.res)));
    const float lc = (float)std::log((double)conf[k] / (1.0 - (double)conf[k]));
    P.dl[k] = lc - h->lp_free;
    const float X = (rp[2] - 1) * 0.5f, Y = (rp[3] - 1) * 0.5f;
    const float xs[4] = {0.0f, X * cg, Y * sg, X * cg + Y * sg};
    const float ys[4] = {0.0f, -X * sg, Y * cg, -X * sg + Y * cg};
    int* bb = &P.bb[4 * k];
    bb[0] = rp[0] + (int)std::floor(*std::min_element(xs, xs + 4)) - 2;
    bb[1] = rp[0] + (int)std::ceil(*std::max_element(xs, xs + 4)) + 2;
    bb[2] = rp[1] + (int)std::floor(*std::min_element(ys, ys + 4)) - 2;
    bb[3] = rp[1] + (int)std::ceil(*std::max_element(ys, ys + 4)) + 2;
    if ((long long)(bb[1] - bb[0] + 1) * (bb[3] - bb[2] + 1) > RASTER_HIST) P.big = true;
    int l = 0;
    for (int j = 0; j < k; ++j) {
      const int* b2 = &P.bb[4 * j];
      if (P.layer[j] >= l && b2[0] <= bb[1] && bb[0] <= b2[1] && b2[2] <= bb[3] && bb[2] <= b2[3]) l = P.layer[j] + 1;
    }
    P.layer[k] = l;
    P.n_layers = std::max(P.n_layers, l + 1);
  }
}

// update_obstacles(boxes) of n planners of one device (planner i's counts[i] boxes follow
// planner i-1's in `boxes` / `conf`): one staged upload, one copy launch for the APF lists,
// and one raster launch per layer index over every planner's boxes of that layer.
static int update_boxes_run(const hastar_handle* hs, int n, const float* boxes, const float* conf, const int* counts,
                            float apf_added_radius, const std::vector<long long>& first);
static int update_boxes_impl(const hastar_handle* hs, int n, const float* boxes, const float* conf, const int* counts,
                             float apf_added_radius) {
  if (n <= 0) return HASTAR_OK;
  std::vector<long long> first(n + 1, 0);
  for (int i = 0; i < n; ++i) first[i + 1] = first[i] + (counts[i] > 0 ? counts[i] : 0);
  const int rc = update_boxes_run(hs, n, boxes, conf, counts, apf_added_radius, first);
  // the cold-order key's input (route_score): the boxes of the last update that went through.
  // Line obstacles do not enter the key (it only orders a batch's searches, never their results).
  if (rc == HASTAR_OK)
    for (int i = 0; i < n; ++i) hs[i]->boxes_w.assign(boxes + 4 * first[i], boxes + 4 * first[i + 1]);
  return rc;
}
static int update_boxes_run(const hastar_handle* hs, int n, const float* boxes, const float* conf, const int* counts,
                            float apf_added_radius, const std::vector<long long>& first) {
  const int dev = hs[0]->device;
  for (int i = 0; i < n; ++i) {
    if (!hs[i] || hs[i]->device != dev) return fail(HASTAR_EINVAL, "null handle or handles on different devices");
    if (counts[i] < 0) return fail(HASTAR_EINVAL, "negative box count");
  }
  HIPCHK(hipSetDevice(dev));
  DeviceCtx& DC = *hs[0]->dc;
  std::vector<BoxPrep> prep(n);
  // host preparation of every planner (rotations, raster origins, layers: O(boxes^2) each),
  // spread over host threads for large batches
  {
    auto work = [&](int a, int b) {
      for (int i = a; i < b; ++i) {
        const long long o = first[i];
        boxes_prep(hs[i], boxes + 4 * o, conf + o, counts[i], apf_added_radius, prep[i]);
      }
    };
    host_parallel(n, work);
  }
  int max_layers = 0;
  for (int i = 0; i < n; ++i)
    if (!prep[i].big) max_layers = std::max(max_layers, prep[i].n_layers);
  // planners with an oversized box footprint take the per-planner kernel
  for (int i = 0; i < n; ++i)
    if (prep[i].big)
      if (int rc = update_boxes_legacy(hs[i], boxes + 4 * first[i], conf + first[i], counts[i], apf_added_radius)) return rc;
  std::lock_guard<std::mutex> lk(DC.mu);
  // APF buffers of the planners (grown on demand; growth waits for queued readers)
  bool grow = false;
  for (int i = 0; i < n; ++i) grow |= !prep[i].big && counts[i] > hs[i]->apf_cap;
  if (grow) {
    HIPCHK(hipStreamSynchronize(DC.stream));
    for (int i = 0; i < n; ++i) {
      hastar_handle h = hs[i];
      if (prep[i].big || counts[i] <= h->apf_cap) continue;
      side_free(DC, h->desc.apf, (size_t)h->apf_cap * 3);
      h->desc.apf = nullptr;
      h->apf_cap = 0;
      HIPCHK(side_alloc(DC, &h->desc.apf, (size_t)counts[i] * 3));
      h->apf_cap = counts[i];
    }
  }
  // staged arrays: maps, boxes by layer, APF copy items, APF floats
  std::vector<RasterMap> maps;
  std::vector<CopyItem> copies;
  std::vector<float> apf;
  std::vector<std::vector<RasterBox>> by_layer(max_layers);
  for (int i = 0; i < n; ++i) {
    if (prep[i].big) continue;
    hastar_handle h = hs[i];
    const BoxPrep& P = prep[i];
    h->desc.n_apf = counts[i];
    if (counts[i] == 0) continue;
    CopyItem ci{h->desc.apf, (long long)apf.size(), counts[i] * 3, 0};
    copies.push_back(ci);
    apf.insert(apf.end(), P.apf.begin(), P.apf.end());
    const int mi = (int)maps.size();
    RasterMap m;
    m.occ = h->desc.occ;
    m.N = h->desc.N;
    m.r0 = h->row0;
    m.r1 = h->row1;
    m.c = g_cosf(h->grid_heading);
    m.s = g_sinf(h->grid_heading);
    m.lp_min = h->lp_min;
    m.lp_max = h->lp_max;
    m.pad = 0;
    maps.push_back(m);
    for (int k = 0; k < counts[i]; ++k) {
      const int* rp = &P.rp[4 * k];
      const int* bb = &P.bb[4 * k];
      if (rp[2] == 0 || rp[3] == 0) continue;  // no sub-samples
      RasterBox b;
      b.map = mi;
      b.si = rp[0];
      b.sj = rp[1];
      b.ni = rp[2];
      b.nj = rp[3];
      b.d = P.dl[k];
      b.bi0 = bb[0];
      b.bj0 = bb[2];
      b.bw = bb[1] - bb[0] + 1;
      b.bh = bb[3] - bb[2] + 1;
      b.pad0 = b.pad1 = 0;
      by_layer[P.layer[k]].push_back(b);
    }
  }
  size_t nbox = 0;
  for (auto& v : by_layer) nbox += v.size();
  const size_t b_maps = align256(maps.size() * sizeof(RasterMap)), b_boxes = align256(nbox * sizeof(RasterBox));
  const size_t b_copy = align256(copies.size() * sizeof(CopyItem)), b_apf = align256(apf.size() * sizeof(float));
  const size_t total = b_maps + b_boxes + b_copy + b_apf;
  if (total == 0) return HASTAR_OK;
  if (int rc = stage_acquire(DC, total)) return rc;
  std::vector<char> host(total);
  char* q = host.data();
  std::memcpy(q, maps.data(), maps.size() * sizeof(RasterMap));
  std::vector<size_t> layer_off(max_layers + 1, 0);
  {
    char* bq = q + b_maps;
    size_t o = 0;
    for (int l = 0; l < max_layers; ++l) {
      layer_off[l] = o;
      std::memcpy(bq + o * sizeof(RasterBox), by_layer[l].data(), by_layer[l].size() * sizeof(RasterBox));
      o += by_layer[l].size();
    }
    layer_off[max_layers] = o;
  }
  std::memcpy(q + b_maps + b_boxes, copies.data(), copies.size() * sizeof(CopyItem));
  std::memcpy(q + b_maps + b_boxes + b_copy, apf.data(), apf.size() * sizeof(float));
  hipStream_t st = DC.stream;
  HIPCHK(hipMemcpyAsync(DC.stage, host.data(), total, hipMemcpyHostToDevice, st));
  const RasterMap* d_maps = reinterpret_cast<const RasterMap*>(DC.stage);
  const RasterBox* d_boxes = reinterpret_cast<const RasterBox*>(DC.stage + b_maps);
  HIPCHK(launch_copy_batch(reinterpret_cast<const CopyItem*>(DC.stage + b_maps + b_boxes), (int)copies.size(),
                           reinterpret_cast<const float*>(DC.stage + b_maps + b_boxes + b_copy), st));
  for (int l = 0; l < max_layers; ++l)
    HIPCHK(launch_raster_boxes_batch(d_maps, d_boxes + layer_off[l], (int)(layer_off[l + 1] - layer_off[l]), st));
  return HASTAR_OK;
}

extern "C" {

// update_obstacles(boxes, confidence, apf_added_radius) of n planners of one device.
int hastar_update_boxes_batch(const hastar_handle* hs, int n, const float* boxes, const float* conf, const int* counts,
                              float apf_added_radius) {
  if (!hs || n < 0 || (n > 0 && !counts)) return fail(HASTAR_EINVAL, "bad argument");
  long long tot = 0;
  for (int i = 0; i < n; ++i) tot += counts[i] > 0 ? counts[i] : 0;
  if (tot > 0 && (!boxes || !conf)) return fail(HASTAR_EINVAL, "bad argument");
  return update_boxes_impl(hs, n, boxes, conf, counts, apf_added_radius);
}

// update_obstacles() (Grid2D.cpp:197-208) of n planners of one device: one launch.
int hastar_decay_batch(const hastar_handle* hs, int n) {
  if (!hs || n < 0) return fail(HASTAR_EINVAL, "bad argument");
  if (n == 0) return HASTAR_OK;
  const int dev = hs[0] ? hs[0]->device : -1;
  std::vector<DecayItem> items(n);
  size_t max_cells = 0;
  for (int i = 0; i < n; ++i) {
    hastar_handle h = hs[i];
    if (!h || h->device != dev) return fail(HASTAR_EINVAL, "null handle or handles on different devices");
    const size_t N = (size_t)h->desc.N;
    items[i] = DecayItem{h->desc.occ + (size_t)h->row0 * N, (long long)((size_t)(h->row1 - h->row0) * N), h->lp_free,
                         h->lp_min, h->lp_max, 0.0f};
    max_cells = std::max(max_cells, (size_t)items[i].cells);
  }
  HIPCHK(hipSetDevice(dev));
  DeviceCtx& DC = *hs[0]->dc;
  std::lock_guard<std::mutex> lk(DC.mu);
  if (int rc = stage_acquire(DC, (size_t)n * sizeof(DecayItem))) return rc;
  HIPCHK(hipMemcpyAsync(DC.stage, items.data(), (size_t)n * sizeof(DecayItem), hipMemcpyHostToDevice, DC.stream));
  HIPCHK(launch_decay_batch(reinterpret_cast<const DecayItem*>(DC.stage), n, max_cells, DC.stream));
  return HASTAR_OK;
}

// update_goal(goal, start) of n planners of one device (goals / starts: n x 3): the map
// relocations run in chunks of maps that share one scratch allocation (<= 1 GiB).
int hastar_update_goal_batch(const hastar_handle* hs, int n, const float* goals, const float* starts) {
  if (!hs || n < 0 || (n > 0 && (!goals || !starts))) return fail(HASTAR_EINVAL, "bad argument");
  if (n == 0) return HASTAR_OK;
  const int dev = hs[0] ? hs[0]->device : -1;
  size_t NNmax = 0;
  for (int i = 0; i < n; ++i) {
    if (!hs[i] || hs[i]->device != dev) return fail(HASTAR_EINVAL, "null handle or handles on different devices");
    NNmax = std::max(NNmax, (size_t)hs[i]->desc.N * hs[i]->desc.N);
  }
  HIPCHK(hipSetDevice(dev));
  DeviceCtx& DC = *hs[0]->dc;
  // a planner named k times is relocated k times, in order (as k single calls): round r takes
  // each planner's r-th occurrence, so the maps of one launch are distinct
  std::vector<std::vector<RelocItem>> rounds;
  std::unordered_map<const float*, int> seen;
  for (int i = 0; i < n; ++i) {
    const RelocPrep rp = goal_prep(hs[i], goals + 3 * i, starts + 3 * i);
    const int r = seen[hs[i]->desc.occ]++;
    if ((int)rounds.size() <= r) rounds.emplace_back();
    rounds[(size_t)r].push_back(RelocItem{hs[i]->desc.occ, nullptr, nullptr, hs[i]->desc.N, rp.c, rp.s, rp.ox, rp.oy, 0});
  }
  std::lock_guard<std::mutex> lk(DC.mu);
  for (auto& items : rounds)
    if (int rc = relocate_maps(DC, items, NNmax)) return rc;
  return HASTAR_OK;
}

}  // extern "C"

// Grid2D::update_obstacles() (Grid2D.cpp:197-208)
int hastar_decay(hastar_handle h) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  HIPCHK(hipSetDevice(h->device));
  const size_t N = (size_t)h->desc.N;
  HIPCHK(launch_decay(h->desc.occ + (size_t)h->row0 * N, (size_t)(h->row1 - h->row0) * N, h->lp_free, h->lp_min,
                      h->lp_max, h->dc->stream));
  return HASTAR_OK;
}

// Grid3D::update_obstacles(boxes) (Grid3D.cpp:22-44) + Grid2D boxes (Grid2D.cpp:99-139):
// one planner is a batch of one (see update_boxes_impl below)
int hastar_update_boxes(hastar_handle h, const float* boxes, const float* conf, int n, float apf_added_radius) {
  if (!h || n < 0 || (n > 0 && (!boxes || !conf))) return fail(HASTAR_EINVAL, "bad argument");
  return update_boxes_impl(&h, 1, boxes, conf, &n, apf_added_radius);
}

// The same update through the per-planner raster kernel with a device-wide hit-counter map
// (DC.cnt): used for boxes whose footprint exceeds the LDS counters of the batched kernel.
static int update_boxes_legacy(hastar_handle h, const float* boxes, const float* conf, int n, float apf_added_radius) {
  HIPCHK(hipSetDevice(h->device));
  DeviceCtx& DC = *h->dc;
  PlannerDev& D = h->desc;
  const float gh = h->grid_heading;
  std::vector<float> apf((size_t)std::max(n, 1) * 3);
  std::vector<int> rp((size_t)std::max(n, 1) * 4);
  std::vector<float> dl((size_t)std::max(n, 1));
  for (int k = 0; k < n; ++k) {
    const float ox = boxes[4 * k], oy = boxes[4 * k + 1], dx = boxes[4 * k + 2], dy = boxes[4 * k + 3];
    V2 pp = rot2(ox - h->goal3x, oy - h->goal3y, gh);
    pp.x += D.n45 * D.res;
    pp.y += D.n2 * D.res;
    apf[3 * k] = pp.x;
    apf[3 * k + 1] = pp.y;
    apf[3 * k + 2] = std::max(dx, dy) / 2 + apf_added_radius;
    const V2 bl = rot2((ox - dx / 2) - h->goal2x, (oy - dy / 2) - h->goal2y, gh);
    rp[4 * k] = gmath::x86_trunc_int(std::round(bl.x / D.res) + (float)D.n45);
    rp[4 * k + 1] = gmath::x86_trunc_int(std::round(bl.y / D.res) + (float)D.n2);
    rp[4 * k + 2] = std::max(0, 2 * gmath::x86_trunc_int(std::ceil(dx / D.res)));
    rp[4 * k + 3] = std::max(0, 2 * gmath::x86_trunc_int(std::ceil(dy / D.res)));
    const float lc = (float)std::log((double)conf[k] / (1.0 - (double)conf[k]));
    dl[k] = lc - h->lp_free;
  }
  if (n > h->apf_cap || n > h->rp_cap) {
    HIPCHK(hipStreamSynchronize(DC.stream));  // buffers may still be read by queued work
    if (n > h->apf_cap) {
      side_free(DC, D.apf, (size_t)h->apf_cap * 3);
      D.apf = nullptr;
      h->apf_cap = 0;
      HIPCHK(side_alloc(DC, &D.apf, (size_t)n * 3));
      h->apf_cap = n;
    }
    if (n > h->rp_cap) {
      side_free(DC, h->d_rp, (size_t)h->rp_cap * 4);
      side_free(DC, h->d_dl, (size_t)h->rp_cap);
      h->d_rp = nullptr;
      h->d_dl = nullptr;
      h->rp_cap = 0;
      HIPCHK(side_alloc(DC, &h->d_rp, (size_t)n * 4));
      HIPCHK(side_alloc(DC, &h->d_dl, (size_t)n));
      h->rp_cap = n;
    }
  }
  D.n_apf = n;
  if (n > 0) {
    // pageable sources: hipMemcpyAsync returns after staging, so the vectors may go
    HIPCHK(hipMemcpyAsync(D.apf, apf.data(), (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice, DC.stream));
    HIPCHK(hipMemcpyAsync(h->d_rp, rp.data(), (size_t)n * 4 * sizeof(int), hipMemcpyHostToDevice, DC.stream));
    HIPCHK(hipMemcpyAsync(h->d_dl, dl.data(), (size_t)n * sizeof(float), hipMemcpyHostToDevice, DC.stream));
    // Layers: box k goes one layer above every earlier box whose cell footprint it may
    // share, so boxes within a layer touch disjoint cells (applied concurrently) and
    // overlapping boxes are applied in the reference's order (Grid2D.cpp:99-139 loops
    // over obstacles in sequence).  Footprints: the rotated sub-sample rectangle's
    // bounds plus a 2-cell margin for rounding.
    const float cg = g_cosf(gh), sg = g_sinf(gh);
    std::vector<int> bb((size_t)n * 4), layer(n, 0);
    int n_layers = 0;
    for (int k = 0; k < n; ++k) {
      const float X = (rp[4 * k + 2] - 1) * 0.5f, Y = (rp[4 * k + 3] - 1) * 0.5f;
      const float xs[4] = {0.0f, X * cg, Y * sg, X * cg + Y * sg};
      const float ys[4] = {0.0f, -X * sg, Y * cg, -X * sg + Y * cg};
      bb[4 * k] = rp[4 * k] + (int)std::floor(*std::min_element(xs, xs + 4)) - 2;
      bb[4 * k + 1] = rp[4 * k] + (int)std::ceil(*std::max_element(xs, xs + 4)) + 2;
      bb[4 * k + 2] = rp[4 * k + 1] + (int)std::floor(*std::min_element(ys, ys + 4)) - 2;
      bb[4 * k + 3] = rp[4 * k + 1] + (int)std::ceil(*std::max_element(ys, ys + 4)) + 2;
      int l = 0;
      for (int j = 0; j < k; ++j)
        if (layer[j] >= l && bb[4 * j] <= bb[4 * k + 1] && bb[4 * k] <= bb[4 * j + 1] && bb[4 * j + 2] <= bb[4 * k + 3] &&
            bb[4 * k + 2] <= bb[4 * j + 3])
          l = layer[j] + 1;
      layer[k] = l;
      n_layers = std::max(n_layers, l + 1);
    }
    std::vector<int> ids;
    std::vector<int> first(n_layers + 1, 0);
    ids.reserve(n);
    for (int l = 0; l < n_layers; ++l) {
      first[l] = (int)ids.size();
      for (int k = 0; k < n; ++k)
        if (layer[k] == l) ids.push_back(k);
    }
    first[n_layers] = n;
    if (n > h->ids_cap) {
      HIPCHK(hipStreamSynchronize(DC.stream));
      side_free(DC, h->d_ids, (size_t)h->ids_cap);
      h->d_ids = nullptr;
      h->ids_cap = 0;
      HIPCHK(side_alloc(DC, &h->d_ids, (size_t)n));
      h->ids_cap = n;
    }
    HIPCHK(hipMemcpyAsync(h->d_ids, ids.data(), (size_t)n * sizeof(int), hipMemcpyHostToDevice, DC.stream));
    std::lock_guard<std::mutex> lk(DC.mu);
    if (int rc = scratch_acquire(DC, (size_t)D.N * D.N)) return rc;
    for (int l = 0; l < n_layers; ++l)
      HIPCHK(launch_raster_boxes(D.occ, DC.cnt, D.N, h->d_rp, h->d_dl, h->d_ids + first[l], first[l + 1] - first[l], cg,
                                 sg, h->lp_min, h->lp_max, h->row0, h->row1, DC.stream));
  }
  return HASTAR_OK;
}

// Grid2D::update_obstacles(lines) (Grid2D.cpp:142-194)
int hastar_update_lines(hastar_handle h, const float* lines, const float* conf, int n, float width) {
  if (!h || n < 0 || (n > 0 && (!lines || !conf))) return fail(HASTAR_EINVAL, "bad argument");
  HIPCHK(hipSetDevice(h->device));
  DeviceCtx& DC = *h->dc;
  PlannerDev& D = h->desc;
  if (n == 0) return HASTAR_OK;
  const float gh = h->grid_heading;
  // prog_width sequence (shared by all lines of the call)
  std::vector<float> wid;
  for (float pw = 0.0f; pw <= width; pw += D.res) {
    wid.push_back(pw);
    if (wid.size() > (1u << 20)) return fail(HASTAR_EINVAL, "line_width / resolution too large");
  }
  const int stride = 100;
  std::vector<float> lp((size_t)n * 9), seq((size_t)n * stride);
  for (int k = 0; k < n; ++k) {
    const V2 a = rot2(lines[4 * k] - h->goal2x, lines[4 * k + 1] - h->goal2y, gh);
    const V2 b = rot2(lines[4 * k + 2] - h->goal2x, lines[4 * k + 3] - h->goal2y, gh);
    V2 d{b.x - a.x, b.y - a.y};
    const float len = g_hypotf(d.x, d.y);
    const V2 nrm{-d.y / len, d.x / len};
    d = {d.x / len, d.y / len};
    const float lc = (float)std::log((double)conf[k] / (1.0 - (double)conf[k]));
    int cntl = 0;
    float pl = 0.0f;
    for (; pl <= len && cntl < 100; ++cntl, pl += D.res) seq[(size_t)k * stride + cntl] = pl;
    float* L = &lp[(size_t)k * 9];
    L[0] = a.x;
    L[1] = a.y;
    L[2] = d.x;
    L[3] = d.y;
    L[4] = nrm.x;
    L[5] = nrm.y;
    L[6] = lc - h->lp_free;
    L[7] = (float)cntl;
    L[8] = (float)wid.size();
  }
  if (wid.empty()) return HASTAR_OK;
  if (n > h->lp_cap || (int)wid.size() > h->wid_cap) {
    HIPCHK(hipStreamSynchronize(DC.stream));
    if (n > h->lp_cap) {
      side_free(DC, h->d_lp, (size_t)h->lp_cap * 9);
      side_free(DC, h->d_seq, (size_t)h->lp_cap * stride);
      h->d_lp = nullptr;
      h->d_seq = nullptr;
      h->lp_cap = 0;
      HIPCHK(side_alloc(DC, &h->d_lp, (size_t)n * 9));
      HIPCHK(side_alloc(DC, &h->d_seq, (size_t)n * stride));
      h->lp_cap = n;
    }
    if ((int)wid.size() > h->wid_cap) {
      side_free(DC, h->d_wid, (size_t)h->wid_cap);
      h->d_wid = nullptr;
      h->wid_cap = 0;
      HIPCHK(side_alloc(DC, &h->d_wid, wid.size()));
      h->wid_cap = (int)wid.size();
    }
  }
  HIPCHK(hipMemcpyAsync(h->d_lp, lp.data(), lp.size() * sizeof(float), hipMemcpyHostToDevice, DC.stream));
  HIPCHK(hipMemcpyAsync(h->d_seq, seq.data(), seq.size() * sizeof(float), hipMemcpyHostToDevice, DC.stream));
  HIPCHK(hipMemcpyAsync(h->d_wid, wid.data(), wid.size() * sizeof(float), hipMemcpyHostToDevice, DC.stream));
  std::lock_guard<std::mutex> lk(DC.mu);
  if (int rc = scratch_acquire(DC, (size_t)D.N * D.N)) return rc;
  HIPCHK(launch_raster_lines(D.occ, DC.cnt, D.N, D.n45, D.n2, D.res, h->d_lp, h->d_seq, h->d_wid, stride, n, h->lp_min,
                             h->lp_max, h->row0, h->row1, DC.stream));
  return HASTAR_OK;
}

// Row-block sharding of the map build.  Grid2D::_grid[i][j] is
// stored row-major (i * N + j); the window limits decay and the box/line rasters to the rows
// i in [row0, row1).  Every cell's update sequence is the reference's, restricted to the
// window, so the union of disjoint windows built by different ranks equals the full build
// bit for bit.  relocate (hastar_update_goal) stays global: call it before sharding.
int hastar_set_row_window(hastar_handle h, int row0, int row1) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  if (row0 < 0 || row1 < row0 || row1 > h->desc.N) return fail(HASTAR_EINVAL, "row window must satisfy 0 <= row0 <= row1 <= N");
  h->row0 = row0;
  h->row1 = row1;
  return HASTAR_OK;
}

// Device-to-device copy of log-odds rows [row0, row1) into `dst` (N floats per row, a device
// pointer on the planner's device).  Returns after the copy has completed.
int hastar_export_rows(hastar_handle h, int row0, int row1, float* dst) {
  if (!h || (!dst && row1 > row0)) return fail(HASTAR_EINVAL, "bad argument");
  if (row0 < 0 || row1 < row0 || row1 > h->desc.N) return fail(HASTAR_EINVAL, "rows must satisfy 0 <= row0 <= row1 <= N");
  HIPCHK(hipSetDevice(h->device));
  const size_t N = (size_t)h->desc.N;
  if (row1 > row0)
    HIPCHK(hipMemcpyAsync(dst, h->desc.occ + (size_t)row0 * N, (size_t)(row1 - row0) * N * sizeof(float),
                          hipMemcpyDeviceToDevice, h->dc->stream));
  HIPCHK(hipStreamSynchronize(h->dc->stream));
  return HASTAR_OK;
}

// Overwrites log-odds rows [row0, row1) from `src` (device pointer, N floats per row; e.g. the
// all-gathered map).  Returns after the copy has completed, so `src` may be reused at once.
int hastar_import_rows(hastar_handle h, int row0, int row1, const float* src) {
  if (!h || (!src && row1 > row0)) return fail(HASTAR_EINVAL, "bad argument");
  if (row0 < 0 || row1 < row0 || row1 > h->desc.N) return fail(HASTAR_EINVAL, "rows must satisfy 0 <= row0 <= row1 <= N");
  HIPCHK(hipSetDevice(h->device));
  const size_t N = (size_t)h->desc.N;
  if (row1 > row0)
    HIPCHK(hipMemcpyAsync(h->desc.occ + (size_t)row0 * N, src, (size_t)(row1 - row0) * N * sizeof(float),
                          hipMemcpyDeviceToDevice, h->dc->stream));
  HIPCHK(hipStreamSynchronize(h->dc->stream));
  return HASTAR_OK;
}

// ---- the backward grid-distance field (csrc/hastar_field.hip; include/hastar.h) ----------
// Relaxes rows [r0, r1) of the field buffer (r1 - r0 + 2 rows of N floats: halo row r0 - 1,
// the block, halo row r1) to convergence for its current halo rows.  Caller holds DC.mu.
static int field_rows_locked(hastar_handle h, float* field, int r0, int r1, int init, int halo_changed, int* changed,
                             int* passes) {
  const PlannerDev& D = h->desc;
  DeviceCtx& DC = *h->dc;
  hipStream_t st = DC.stream;
  int ntx = 0, nty = 0;
  const int nt = field_tiles(D.N, r0, r1, &ntx, &nty);
  int* buf = nullptr;  // act[nt], nxt[nt], flags, pending
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&buf), (2 * (size_t)nt + 2) * sizeof(int)));
  struct Release {
    int* p;
    ~Release() { hipFree(p); }
  } release{buf};
  int* act = buf;
  int* nxt = buf + nt;
  int* flags = buf + 2 * nt;
  int* pending = flags + 1;
  HIPCHK(hipMemsetAsync(buf, 0, (2 * (size_t)nt + 2) * sizeof(int), st));
  if (init) {
    HIPCHK(launch_field_init(field, D.N, r0, r1, D.goal_cx, D.goal_cy, st));
    HIPCHK(launch_field_activate(act, ntx, nty, 0, pending, st));
  } else {
    // a halo row that changed can lower the block's first / last tile row
    if (halo_changed & 1) HIPCHK(launch_field_activate(act, ntx, nty, 1, pending, st));
    if (halo_changed & 2) HIPCHK(launch_field_activate(act, ntx, nty, 2, pending, st));
  }
  int pend = 0, np = 0;
  HIPCHK(hipMemcpyAsync(&pend, pending, sizeof(int), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  // every pass lowers at least one value or activates nothing, and values only fall through
  // finitely many floats, so the loop ends; the bound only guards against a broken device.
  // Passes are queued FIELD_BATCH at a time between host checks: a pass after the last
  // productive one finds no active tile and ends at once, so only the check's round trip is
  // saved, not work added.
  constexpr int FIELD_BATCH = 8;
  const long long max_passes = 64LL * ((long long)D.N * D.N + 64);
  while (pend > 0) {
    if ((np += FIELD_BATCH) > max_passes) return fail(HASTAR_EDEVICE, "field relaxation did not converge");
    for (int b = 0; b < FIELD_BATCH; ++b) {
      HIPCHK(hipMemsetAsync(pending, 0, sizeof(int), st));
      HIPCHK(launch_field_pass(D, field, r0, r1, act, nxt, flags, pending, st));
      HIPCHK(hipMemsetAsync(act, 0, (size_t)nt * sizeof(int), st));
      std::swap(act, nxt);
    }
    // the last pass's activations: none means the queued passes reached the fixed point
    HIPCHK(hipMemcpyAsync(&pend, pending, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  int fl = 0;
  HIPCHK(hipMemcpyAsync(&fl, flags, sizeof(int), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (changed) *changed = fl;
  if (passes) *passes = np;
  return HASTAR_OK;
}

int hastar_field_rows(hastar_handle h, float* field, int r0, int r1, int init, int halo_changed, int* changed,
                      int* passes) {
  if (!h || !field) return fail(HASTAR_EINVAL, "null argument");
  if (!h->goal_set) return fail(HASTAR_EINVAL, "update_goal must be called before the field");
  if (r0 < 0 || r1 <= r0 || r1 > h->desc.N) return fail(HASTAR_EINVAL, "rows must satisfy 0 <= r0 < r1 <= N");
  HIPCHK(hipSetDevice(h->device));
  std::lock_guard<std::mutex> lk(h->dc->mu);
  return field_rows_locked(h, field, r0, r1, init, halo_changed, changed, passes);
}

int hastar_heuristic_field(hastar_handle h, float* dst, int* passes) {
  if (!h || !dst) return fail(HASTAR_EINVAL, "null argument");
  if (!h->goal_set) return fail(HASTAR_EINVAL, "update_goal must be called before the field");
  HIPCHK(hipSetDevice(h->device));
  std::lock_guard<std::mutex> lk(h->dc->mu);
  const size_t N = (size_t)h->desc.N;
  float* buf = nullptr;  // halo row, N rows, halo row
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&buf), (N + 2) * N * sizeof(float)));
  struct Release {
    float* p;
    ~Release() { hipFree(p); }
  } release{buf};
  if (int rc = field_rows_locked(h, buf, 0, (int)N, 1, 0, nullptr, passes)) return rc;
  HIPCHK(hipMemcpyAsync(dst, buf + N, N * N * sizeof(float), hipMemcpyDeviceToDevice, h->dc->stream));
  HIPCHK(hipStreamSynchronize(h->dc->stream));
  return HASTAR_OK;
}

int hastar_relaxed_set_field(hastar_handle h, const float* src) {
  if (!h || !src) return fail(HASTAR_EINVAL, "null argument");
  if (!h->goal_set) return fail(HASTAR_EINVAL, "update_goal must be called before the field");
  HIPCHK(hipSetDevice(h->device));
  std::lock_guard<std::mutex> lk(h->dc->mu);
  const size_t NN = (size_t)h->desc.N * h->desc.N;
  if (!h->rfield && hipMalloc(reinterpret_cast<void**>(&h->rfield), NN * sizeof(float)) != hipSuccess) {
    h->rfield = nullptr;
    return fail(HASTAR_ENOMEM, "heuristic field allocation failed");
  }
  HIPCHK(hipMemcpyAsync(h->rfield, src, NN * sizeof(float), hipMemcpyDeviceToDevice, h->dc->stream));
  HIPCHK(hipStreamSynchronize(h->dc->stream));
  // a full field: every reachable cell settled, no ellipse bound (unreachable cells: h = 0)
  h->rhlim = 0.0f;
  h->rstart = 0;
  h->rcoarse = 1;
  h->rvalid = true;
  return HASTAR_OK;
}

int hastar_get_obstacles(hastar_handle h, float* out) {
  if (!h || !out) return fail(HASTAR_EINVAL, "null argument");
  HIPCHK(hipSetDevice(h->device));
  const size_t NN = (size_t)h->desc.N * h->desc.N;
  HIPCHK(hipMemcpyAsync(out, h->desc.occ, NN * sizeof(float), hipMemcpyDeviceToHost, h->dc->stream));
  HIPCHK(hipStreamSynchronize(h->dc->stream));
  return HASTAR_OK;
}

}  // extern "C"

// Cold-order key of a planner with no search history and no caller hint: obstacles close to the
// straight start-goal route are what make a search long (its holonomic A* has to work around
// them and its Dubins shots fail), so the key sums (1 + t) / (1 + d)^3 over the last boxes,
// d = the distance (m) between the box and the start-goal segment (0 when the segment crosses
// it), t = the box centre's position along the route (0 at the start, 1 at the goal).  Scaled
// to s_memrealtime ticks (only the order matters unless history and cold planners share a
// batch).  Over the 23,552 cfg3 queries and their measured search times, list scheduling in
// this order gives a step of 2.95 s against 3.05 s for sum 1 / (1 + d)^2, 3.74 s for round 2's
// nearest-box clearance and 2.67 s for perfect foreknowledge.
static double seg_box_dist(double ax, double ay, double bx, double by, double x0, double y0, double x1, double y1) {
  // does the segment cross the box? (slab test)
  double t0 = 0.0, t1 = 1.0;
  const double d[2] = {bx - ax, by - ay}, o[2] = {ax, ay}, lo[2] = {x0, y0}, hi[2] = {x1, y1};
  bool hit = true;
  for (int k = 0; k < 2 && hit; ++k) {
    if (std::fabs(d[k]) < 1e-12) {
      if (o[k] < lo[k] || o[k] > hi[k]) hit = false;
    } else {
      double ta = (lo[k] - o[k]) / d[k], tb = (hi[k] - o[k]) / d[k];
      if (ta > tb) std::swap(ta, tb);
      t0 = std::max(t0, ta);
      t1 = std::min(t1, tb);
      if (t0 > t1) hit = false;
    }
  }
  if (hit) return 0.0;
  // squared distances: the segment's end points to the box, the box corners to the segment
  auto pt_box2 = [&](double px, double py) {
    const double dx = std::max(std::max(x0 - px, px - x1), 0.0), dy = std::max(std::max(y0 - py, py - y1), 0.0);
    return dx * dx + dy * dy;
  };
  const double L2 = d[0] * d[0] + d[1] * d[1];
  auto pt_seg2 = [&](double px, double py) {
    double t = L2 > 0 ? ((px - ax) * d[0] + (py - ay) * d[1]) / L2 : 0.0;
    t = std::min(1.0, std::max(0.0, t));
    const double ex = ax + t * d[0] - px, ey = ay + t * d[1] - py;
    return ex * ex + ey * ey;
  };
  double m = std::min(pt_box2(ax, ay), pt_box2(bx, by));
  m = std::min(m, std::min(pt_seg2(x0, y0), pt_seg2(x1, y0)));
  m = std::min(m, std::min(pt_seg2(x0, y1), pt_seg2(x1, y1)));
  return std::sqrt(m);
}
static double route_score(const float* boxes, int n, float sx, float sy, float gx, float gy) {
  const double ux = (double)gx - sx, uy = (double)gy - sy, L2 = ux * ux + uy * uy;
  double sc = 0.0;
  for (int k = 0; k < n; ++k) {
    const double ox = boxes[4 * k], oy = boxes[4 * k + 1], hx = boxes[4 * k + 2] * 0.5, hy = boxes[4 * k + 3] * 0.5;
    const double d = seg_box_dist(sx, sy, gx, gy, ox - hx, oy - hy, ox + hx, oy + hy);
    // t: the box centre's position along the route (0 at the start, 1 at the goal); a box near
    // the goal weighs up to twice as much (the goal heading and the Dubins shots meet it)
    const double t = L2 > 0 ? std::min(1.0, std::max(0.0, ((ox - sx) * ux + (oy - sy) * uy) / L2)) : 0.0;
    const double q = 1.0 + d;
    sc += (1.0 + t) / (q * q * q);
  }
  return sc;
}
static long long cold_key(hastar_handle h, const float start[3]) {
  const double sc = route_score(h->boxes_w.data(), (int)(h->boxes_w.size() / 4), start[0], start[1],
                                h->desc.world_goal_x, h->desc.world_goal_y);
  return 1 + (long long)(12.6e6 + 9.1e6 * sc);
}

// Grid3D::set_start_node (Grid3D.cpp:127-160) + HybridAStar::find_path (HybridAStar.cpp:71-74)
static void prepare_start(hastar_handle h, float vel, const float start[3]) {
  PlannerDev& D = h->desc;
  const float gh = h->grid_heading;
  const float c = g_cosf(gh), s = g_sinf(gh);
  const float dx = start[0] - h->goal3x, dy = start[1] - h->goal3y;
  const float rx = dx * c + dy * s, ry = -dx * s + dy * c;
  const float rh = wrap_pi_h(start[2] - gh);
  const float px = rx + D.n45 * D.res, py = ry + D.n2 * D.res, ph = rh;
  const int i = gmath::x86_trunc_int(px / D.res), j = gmath::x86_trunc_int(py / D.res);
  if (i > -1 && i < D.N && j > -1 && j < D.N) {
    D.start_x = px;
    D.start_y = py;
    D.start_h = ph;
    D.start_cx = i;
    D.start_cy = j;
  } else {
    D.start_x = D.start_y = D.start_h = 0.0f;
    D.start_cx = D.start_cy = 0;
  }
  D.start_bin = heading_bin_h(D.start_h, D.prec);
  D.start_ci = D.nsteer / 2;
  D.start_vmin = vel * vel;
}

static void fill_stats(const SearchResult& R, hastar_stats* st) {
  if (!st) return;
  st->pops = R.pops;
  st->successors = R.successors;
  st->astar_pops = R.astar_pops;
  st->astar_searches = R.astar_searches;
  st->shots = R.shots;
  st->closed_size = R.closed_size;
  st->pop_digest = R.pop_digest;
  st->closed_digest = R.closed_digest;
  st->via_shot = R.via_shot;
  st->status = R.status;
  st->parks = R.parks;
  st->pad = 0;
}

static int copy_path_out(hastar_handle h, float* xyh, float* curv, int cap, int* len, hipStream_t st) {
  const int n = h->last.path_len;
  if (len) *len = n;
  if (n > cap) return fail(HASTAR_ENOSPC, "path buffer too small");
  if (n > 0) {
    HIPCHK(hipMemcpyAsync(xyh, h->desc.out_xyh, (size_t)n * 3 * sizeof(float), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(curv, h->desc.out_curv, (size_t)n * sizeof(float), hipMemcpyDeviceToHost, st));
  }
  return 0;
}

// per-batch device/pinned buffers (descriptors, order, results, path offsets), grown on demand
// The arena requirement of a batch (every planner's), after checking the handles.
static int batch_need(const hastar_handle* hs, int n, ArenaReq* need) {
  const int dev = hs[0] ? hs[0]->device : -1;
  for (int i = 0; i < n; ++i) {
    if (!hs[i] || hs[i]->device != dev) return fail(HASTAR_EINVAL, "null handle or handles on different devices");
    if (!hs[i]->goal_set) return fail(HASTAR_EINVAL, "update_goal must be called before find_path");
    need->merge(hs[i]->areq);
  }
  return 0;
}

// How a batch of n planners is launched, and the slot arenas it needs (W).
struct BatchShape {
  bool wide, split;
  int head, per_cu, W;
};
static BatchShape batch_shape(const DeviceCtx& DC, int n) {
  BatchShape b{};
  // A batch no larger than the CU count runs on the latency kernel: one search per CU with the
  // CU's whole LDS (outer open tree, 2048-node holonomic pool) and its SIMD to itself.  Larger
  // batches fill every CU with 8 searches (the batch kernel).  HASTAR_WIDE=0/1 forces either.
  b.wide = n <= DC.n_cu;
  if (const char* e = std::getenv("HASTAR_WIDE")) b.wide = std::atoi(e) != 0;
  // A batch many times the CU count splits: its head (the longest expected searches, first in
  // the queue) on `head_cus` latency CUs, the bulk on the batch kernel beside them.
  // HASTAR_SPLIT=0/1 forces it off/on.
  b.split = !b.wide && DC.head_cus > 0 && n > 4 * DC.n_cu;
  if (const char* e = std::getenv("HASTAR_SPLIT")) b.split = !b.wide && DC.head_cus > 0 && std::atoi(e) != 0;
  // the head grows by the searches that parked in the last split launch (they get head arenas
  // and a CU each from the start: cfg4's > 262 k-pop replans), up to one CU in 8
  // (only for a batch many times the CU count: a forced split of a small batch keeps head_cus)
  const int extra = n > 4 * DC.n_cu ? DC.head_extra : 0;
  b.head = b.split ? std::min(std::min(DC.head_cus + extra, DC.n_cu / 8), n) : 0;
  b.per_cu = DC.resident_slots / DC.n_cu;  // batch-kernel waves per CU
  b.W = std::max(1, std::min(n, b.wide ? DC.n_cu : b.split ? b.head + (DC.n_cu - b.head) * b.per_cu
                                                           : DC.resident_slots));
  if (const char* e = std::getenv("HASTAR_SLOTS")) b.W = std::max(1, std::min(b.W, std::atoi(e)));
  return b;
}

// Room for `pts` packed path points of a batch (device and pinned host copies).
static hipError_t points_acquire(DeviceCtx& DC, size_t pts) {
  if (pts <= DC.pts_cap) return hipSuccess;
  if (DC.d_pxyh) hipFree(DC.d_pxyh);
  if (DC.d_pcurv) hipFree(DC.d_pcurv);
  if (DC.h_pxyh) hipHostFree(DC.h_pxyh);
  if (DC.h_pcurv) hipHostFree(DC.h_pcurv);
  DC.d_pxyh = DC.d_pcurv = DC.h_pxyh = DC.h_pcurv = nullptr;
  DC.pts_cap = 0;
  hipError_t e = dalloc(&DC.d_pxyh, pts * 3);
  if (e == hipSuccess) e = dalloc(&DC.d_pcurv, pts);
  if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&DC.h_pxyh), pts * 3 * sizeof(float));
  if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&DC.h_pcurv), pts * sizeof(float));
  if (e == hipSuccess) DC.pts_cap = pts;
  return e;
}

static int batch_acquire(DeviceCtx& DC, int n) {
  hipStream_t st = DC.stream;
  if (n <= DC.batch_cap) return 0;
  {
    HIPCHK(hipStreamSynchronize(st));
    if (DC.d_descs) hipFree(DC.d_descs);
    if (DC.d_order) hipFree(DC.d_order);
    if (DC.d_results) hipFree(DC.d_results);
    if (DC.d_off) hipFree(DC.d_off);
    if (DC.d_len) hipFree(DC.d_len);
    if (DC.h_results) hipHostFree(DC.h_results);
    if (DC.h_offlen) hipHostFree(DC.h_offlen);
    DC.d_descs = nullptr;
    DC.d_order = nullptr;
    DC.d_results = nullptr;
    DC.d_off = nullptr;
    DC.d_len = nullptr;
    DC.h_results = nullptr;
    DC.h_offlen = nullptr;
    DC.batch_cap = 0;
    HIPCHK(dalloc(&DC.d_descs, (size_t)n));
    HIPCHK(dalloc(&DC.d_order, (size_t)n));
    HIPCHK(dalloc(&DC.d_results, (size_t)n));
    HIPCHK(dalloc(&DC.d_off, (size_t)n + 1));
    HIPCHK(dalloc(&DC.d_len, (size_t)n));
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&DC.h_results), (size_t)n * sizeof(SearchResult)));
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&DC.h_offlen), ((size_t)n * 2 + 1) * sizeof(long long)));
    DC.batch_cap = n;
  }
  return 0;
}

// Hand a finished batch back: per-planner outcome (stats[i].status), then every path packed on
// the device by one gather kernel (kept there for hastar_velocity_profile_last_batch) and one
// copy to the caller's buffers of the paths that fit its cap.  lpt: record each search's
// duration as the planner's longest-first key (exact mode only).
static bool lpt_work_key() {
  static const bool on = [] {
    const char* e = std::getenv("HASTAR_LPT_WORK");
    return e && std::atoi(e) != 0;
  }();
  return on;
}

static int finish_batch(DeviceCtx& DC, const hastar_handle* hs, int n, float* xyh, float* curv, int cap, int* len,
                        float* cost, int* ok, hastar_stats* stats, bool lpt) {
  hipStream_t st = DC.stream;
  int rc = HASTAR_OK;
  // pack the paths that fit the caller's buffers: offsets, one gather kernel, one copy.
  // Every planner reports its own outcome in stats[i].status: 0, HASTAR_EOVERFLOW (the
  // search needed more device memory than it could get, or hit HASTAR_MAX_POPS_HARD),
  // HASTAR_ENOSPC (kernel: path longer than the planner's output buffer; host: longer than
  // `cap` — then len[i] is the length needed and hastar_copy_path fetches it).  The return
  // code is the first ENOSPC, else the first EOVERFLOW.
  long long* h_off = DC.h_offlen;
  int* h_len = reinterpret_cast<int*>(DC.h_offlen + n + 1);
  long long total = 0;
  int rc_over = HASTAR_OK;
  for (int i = 0; i < n; ++i) {
    SearchResult& R = DC.h_results[i];
    hastar_handle h = hs[i];
    if (R.status == -75) R.ok = 0;
    h->last = R;
    h->have_last = true;
    // longest-first key: the search's own duration (s_memrealtime ticks) — it weighs outer
    // pops, inner A* pops and shots by what they cost where the search ran.  (A schedule-free
    // work key, 1566 x pops + 1058 x inner pops from a fit of the cfg3 durations, settled the
    // steps at 3.03 s against 2.74 s: profiles/r03h_bench_long.json; HASTAR_LPT_WORK=1.)
    if (lpt) h->prev_pops = h->last_pops;
    if (lpt) h->last_pops = (lpt_work_key() || R.t_end <= R.t_start)
                                ? 1 + 1566LL * (long long)R.pops + 1058LL * (long long)R.astar_pops
                                : (long long)(R.t_end - R.t_start);
    ok[i] = R.ok;
    cost[i] = R.ok ? R.cost : FLT_MAX;
    fill_stats(R, stats ? &stats[i] : nullptr);
    len[i] = R.path_len;
    if (R.status == -75 && rc_over == HASTAR_OK) {
      rc_over = HASTAR_EOVERFLOW;
      g_err = "search ended by an arena overflow (device memory) or HASTAR_MAX_POPS_HARD";
    } else if (R.status == -28 && rc == HASTAR_OK) {
      rc = fail(HASTAR_ENOSPC, "path longer than the planner's output buffer");
    }
    // every path is packed on the device whatever `cap` is (the device-resident velocity
    // profile of this batch reads len[i] points at offset i); only the host copy is limited
    // to the caller's buffer
    if (R.path_len > cap) {
      if (stats) stats[i].status = HASTAR_ENOSPC;  // the caller fetches it with hastar_copy_path
      if (rc == HASTAR_OK) rc = fail(HASTAR_ENOSPC, "path buffer too small");
    }
    h_off[i] = total;
    h_len[i] = R.path_len;
    total += R.path_len;
  }
  if (rc == HASTAR_OK && rc_over != HASTAR_OK) rc = rc_over;
  h_off[n] = total;
  DC.last_n = n;
  DC.last_total = total;
  // the offsets go to the device even when no path came back, so that a velocity profile of
  // this batch never reads a previous batch's offsets
  HIPCHK(hipMemcpyAsync(DC.d_off, h_off, ((size_t)n + 1) * sizeof(long long), hipMemcpyHostToDevice, st));
  if (total > 0) {
    if ((size_t)total > DC.pts_cap) HIPCHK(points_acquire(DC, (size_t)total + (size_t)total / 2 + 1024));
    HIPCHK(hipMemcpyAsync(DC.d_len, h_len, (size_t)n * sizeof(int), hipMemcpyHostToDevice, st));
    HIPCHK(launch_gather_paths(DC.d_descs, DC.d_off, DC.d_len, n, DC.d_pxyh, DC.d_pcurv, st));
    HIPCHK(hipMemcpyAsync(DC.h_pxyh, DC.d_pxyh, (size_t)total * 3 * sizeof(float), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(DC.h_pcurv, DC.d_pcurv, (size_t)total * sizeof(float), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (int i = 0; i < n; ++i) {
      if (h_len[i] == 0 || h_len[i] > cap) continue;
      std::memcpy(xyh + (size_t)i * cap * 3, DC.h_pxyh + 3 * h_off[i], (size_t)h_len[i] * 3 * sizeof(float));
      std::memcpy(curv + (size_t)i * cap, DC.h_pcurv + h_off[i], (size_t)h_len[i] * sizeof(float));
    }
  }
  return rc;
}

extern "C" {

double hastar_test_route_score(const float* boxes, int n, const float start[2], const float goal[2]) {
  return route_score(boxes, n, start[0], start[1], goal[0], goal[1]);
}

int hastar_reserve(const hastar_handle* hs, int n, long long path_points) {
  if (!hs || n <= 0 || path_points < 0) return fail(HASTAR_EINVAL, "bad argument");
  ArenaReq need;
  if (int rc = batch_need(hs, n, &need)) return rc;
  HIPCHK(hipSetDevice(hs[0]->device));
  DeviceCtx& DC = *hs[0]->dc;
  std::lock_guard<std::mutex> lk(DC.mu);
  if (int rc = arenas_acquire(DC, need, batch_shape(DC, n).W)) return rc;
  if (int rc = batch_acquire(DC, n)) return rc;
  if (path_points > 0) HIPCHK(points_acquire(DC, (size_t)path_points));
  // both search kernels once on an empty queue (every wave exits at its first queue read), so
  // that their code objects are loaded here and not in the batch's first call
  if (!DC.kernels_warm) {
    HIPCHK(launch_search(DC.d_descs, 0, DC.d_arenas, 1, DC.d_order, 0, DC.d_next, 0, DC.stream));
    HIPCHK(launch_search_wide(DC.d_descs, 0, DC.d_arenas, 1, DC.d_order, DC.d_next, 0, DC.stream, 0));
    HIPCHK(hipStreamSynchronize(DC.stream));
    DC.kernels_warm = true;
  }
  return 0;
}

int hastar_find_path(hastar_handle h, float vel, const float start[3], float* xyh, float* curv, int cap, int* len,
                     float* cost, int* ok, hastar_stats* stats) {
  return hastar_find_path_batch(&h, 1, &vel, start, xyh, curv, cap, len, cost, ok, stats);
}

int hastar_find_path_batch(const hastar_handle* hs, int n, const float* vel, const float* starts, float* xyh,
                           float* curv, int cap, int* len, float* cost, int* ok, hastar_stats* stats) {
  if (!hs || n <= 0 || !vel || !starts || !len || !cost || !ok || cap < 0 || (cap > 0 && (!xyh || !curv)))
    return fail(HASTAR_EINVAL, "bad argument");
  ArenaReq need;
  if (int rc = batch_need(hs, n, &need)) return rc;
  HIPCHK(hipSetDevice(hs[0]->device));
  DeviceCtx& DC = *hs[0]->dc;
  std::lock_guard<std::mutex> lk(DC.mu);
  hipStream_t st = DC.stream;
  const BatchShape bs = batch_shape(DC, n);
  const bool wide = bs.wide, split = bs.split;
  const int head = bs.head, per_cu = bs.per_cu, W = bs.W;
  if (int rc = arenas_acquire(DC, need, W)) return rc;
  const int slots = std::min(W, DC.n_arenas);
  if (int rc = batch_acquire(DC, n)) return rc;
  // HASTAR_SPLIT_MODE=2: the head searches run on head workgroups of the batch kernel itself
  // (wave 0 alone on its CU, the batch kernel's code and LDS layout) instead of the latency kernel
  const char* sm_env = std::getenv("HASTAR_SPLIT_MODE");
  const int split_mode = sm_env && std::atoi(sm_env) == 2 ? 2 : 1;
  const bool split2 = split && slots > head && split_mode == 2;
  const bool split1 = split && slots > head && !split2;
  {
    // head arenas (DeviceCtx::head_k) only for the latency kernel's head of a split launch
    int span = 2;
    for (int i = 0; i < n; ++i) span = std::max(span, hs[i]->span);
    if (int rc = split1 ? head_acquire(DC, head, span, slots) : head_release(DC)) return rc;
  }
  // pool arenas [0, hoff) carved into head arenas
  const int hoff = DC.head_k > 0 ? DC.head_n * DC.head_k : 0;
  std::vector<PlannerDev> descs(n);
  for (int i = 0; i < n; ++i) {
    prepare_start(hs[i], vel[i], starts + 3 * i);
    descs[i] = hs[i]->desc;
    descs[i].result = DC.d_results + i;
  }
  // longest-expected-first: planners ordered by the work of their previous search
  // (a planner with no history and no hint is keyed by its obstacles near the route, cold_key)
  std::vector<long long> key(n);
  int n_cold = 0;
  for (int i = 0; i < n; ++i) {
    // the longer of the planner's last two searches (cfg4's longest queries alternate long and
    // short replans; keyed by the last one alone, a long one ran in the bulk and parked there)
    key[i] = hs[i]->last_pops > 0 ? std::max(hs[i]->last_pops, hs[i]->prev_pops) : 0;
    n_cold += key[i] <= 0;
  }
  if (n_cold > 0)
    host_parallel(n_cold >= 256 ? n : 1, [&](int a, int b) {
      if (n_cold < 256) a = 0, b = n;
      for (int i = a; i < b; ++i)
        if (key[i] <= 0) key[i] = cold_key(hs[i], starts + 3 * i);
    });
  std::vector<int> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return key[a] > key[b]; });
  HIPCHK(hipMemcpyAsync(DC.d_descs, descs.data(), (size_t)n * sizeof(PlannerDev), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(DC.d_order, order.data(), (size_t)n * sizeof(int), hipMemcpyHostToDevice, st));
  // raised issue priority for the head of the longest-first queue (HASTAR_PRIO_N overrides)
  int n_prio = std::max(1, slots / 8);
  if (const char* e = std::getenv("HASTAR_PRIO_N")) n_prio = std::atoi(e);
  // an explicit pop budget (0 = none: a search runs until the reference's loop would end)
  long long hard_pops = 0;
  if (const char* e = std::getenv("HASTAR_MAX_POPS_HARD")) hard_pops = std::atoll(e);
  // a split launch's batch-kernel search is offered to free latency CUs after this many pops
  // (DESIGN.md §4.1 "Handoff"): a remedy for a queue ordered without history, where the cold key
  // can rank a long search far down the queue, onto a batch slot.  With the measured pops of
  // the planners' last searches the longest ones start on the latency CUs, and handoffs measured
  // 1 % slower (profiles/r05k_handoff_ab.jsonl): on only when more than an eighth of the batch
  // has no history (HASTAR_HANDOFF_WARM=1: always)
  int handoff_pops = 32768;
  if (const char* e = std::getenv("HASTAR_HANDOFF_POPS")) handoff_pops = std::atoi(e);
  const char* hw_env = std::getenv("HASTAR_HANDOFF_WARM");
  if (!(hw_env && std::atoi(hw_env) != 0) && (long long)n_cold * 8 <= (long long)n) handoff_pops = 0;
  // every result starts as "not run" (a wave that parks a search stops taking work, so a
  // launch can end with queue entries nobody took)
  HIPCHK(hipMemsetAsync(DC.d_results, 0xff, (size_t)n * sizeof(SearchResult), st));
  float ms_total = 0.0f;
  auto timed = [&](auto&& launch) -> int {
    HIPCHK(hipEventRecord(DC.ev0, st));
    HIPCHK(launch());
    HIPCHK(hipEventRecord(DC.ev1, st));
    HIPCHK(hipMemcpyAsync(DC.h_results, DC.d_results, (size_t)n * sizeof(SearchResult), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    float ms = 0.0f;
    hipEventElapsedTime(&ms, DC.ev0, DC.ev1);
    ms_total += ms;
    return 0;
  };
  if (int r = timed([&]() -> hipError_t {
        if (split2)
          return launch_search(DC.d_descs, n, DC.d_arenas, slots, DC.d_order, n_prio, DC.d_next, hard_pops, st, 0, -1,
                               head);
        if (split1) {
          // the head's queue entries 0 .. head-1 are taken statically by the latency workgroups
          // (arenas 0 .. head-1, or the head arenas); the batch kernel's waves count on from
          // `head` (pool arenas from max(head, hoff))
          const int init[4] = {head, 0, 0, 0};
          hipError_t e = hipMemcpyAsync(DC.d_next, init, sizeof(init), hipMemcpyHostToDevice, st);
          // the handoff board: every entry empty, enabled with the offer threshold (pops) unless
          // HASTAR_HANDOFF_POPS=0
          if (e == hipSuccess) e = hipMemsetAsync(DC.d_board, 0, offsetof(HandoffBoard, entry), st);
          if (e == hipSuccess && handoff_pops > 0) {
            // the header alone (the words before `state`), staged like `init` above
            alignas(16) unsigned char hdr[offsetof(HandoffBoard, state)] = {};
            HandoffBoard* H = reinterpret_cast<HandoffBoard*>(hdr);
            H->enabled = 1;
            H->thr = handoff_pops;
            H->n = std::min(DC.n_arenas, HANDOFF_CAP);
            H->pool = DC.d_arenas;
            e = hipMemcpyAsync(DC.d_board, hdr, sizeof(hdr), hipMemcpyHostToDevice, st);
          }
          if (e == hipSuccess) e = hipEventRecord(DC.ev_fork, st);
          if (e == hipSuccess) e = hipStreamWaitEvent(DC.head_st, DC.ev_fork, 0);
          if (e == hipSuccess) e = hipStreamWaitEvent(DC.bulk_st, DC.ev_fork, 0);
          if (e == hipSuccess) e = hipEventRecord(DC.ev_hs, DC.head_st);
          if (e == hipSuccess) e = hipEventRecord(DC.ev_bs, DC.bulk_st);
          const int boff = std::max(head, hoff);
          if (e == hipSuccess)
            e = DC.head_n > 0 ? launch_search_wide(DC.d_descs, n, DC.d_head, head, DC.d_order, DC.d_next, hard_pops,
                                                   DC.head_st, 1, DC.n_arenas)
                              : launch_search_wide(DC.d_descs, n, DC.d_arenas, head, DC.d_order, DC.d_next, hard_pops,
                                                   DC.head_st, 1);
          if (e == hipSuccess)
            e = launch_search(DC.d_descs, n, DC.d_arenas + boff, std::min(slots - boff, (DC.n_cu - head) * per_cu),
                              DC.d_order, n_prio, DC.d_next, hard_pops, DC.bulk_st, boff, -1);
          if (e == hipSuccess) e = hipEventRecord(DC.ev_head, DC.head_st);
          if (e == hipSuccess) e = hipEventRecord(DC.ev_bulk, DC.bulk_st);
          if (e == hipSuccess) e = hipStreamWaitEvent(st, DC.ev_head, 0);
          if (e == hipSuccess) e = hipStreamWaitEvent(st, DC.ev_bulk, 0);
          return e;
        }
        return wide ? launch_search_wide(DC.d_descs, n, DC.d_arenas, slots, DC.d_order, DC.d_next, hard_pops, st)
                    : launch_search(DC.d_descs, n, DC.d_arenas, slots, DC.d_order, n_prio, DC.d_next, hard_pops, st);
      })) {
    // a failed split launch must not leave the board enabled: later launches through the same
    // pool arenas (resumes, unsplit batches) would post offers no latency wave claims.  The
    // header is cleared synchronously, whatever state the streams are in (best effort: the
    // launch's own error is the one reported).
    if (split1) {
      (void)hipDeviceSynchronize();
      (void)hipMemset(DC.d_board, 0, offsetof(HandoffBoard, state));
      (void)hipDeviceSynchronize();
    }
    return r;
  }
  if (split1) {
    // the board is read back and disabled before any other launch (resume passes run the
    // batch kernel without it)
    int hdr[6] = {0, 0, 0, 0, 0, 0};
    HIPCHK(hipMemcpy(hdr, DC.d_board, sizeof(hdr), hipMemcpyDeviceToHost));
    DC.handoffs = hdr[5];
    HIPCHK(hipMemsetAsync(DC.d_board, 0, offsetof(HandoffBoard, state), st));
    hipEventElapsedTime(&DC.split_ms[0], DC.ev0, DC.ev_hs);
    hipEventElapsedTime(&DC.split_ms[1], DC.ev0, DC.ev_head);
    hipEventElapsedTime(&DC.split_ms[2], DC.ev0, DC.ev_bs);
    hipEventElapsedTime(&DC.split_ms[3], DC.ev0, DC.ev_bulk);
  }
  // Parked searches (their arena could not take one more pop) continue in larger arenas,
  // planners no wave took run in a new queue pass: until every search has ended.
  {
    std::vector<char> in_resume(n, 0);      // 1: the planner's last launch was a resume launch
    std::vector<int> pool_used;             // {first, count} of pool arenas lent to resume arenas
    const char* rp_env = std::getenv("HASTAR_RESUME_POOL");
    const bool pool_first = rp_env && std::atoi(rp_env) != 0;
    std::vector<ResumeArena> cur, nxt;      // resume arenas of the last resume launch, by index
    std::vector<int> notrun, parked;
    for (;;) {
      notrun.clear();
      parked.clear();
      for (int i = 0; i < n; ++i) {
        const int stt = DC.h_results[i].status;
        if (stt == SEARCH_NOT_RUN) notrun.push_back(i);
        else if (stt == SEARCH_PARKED) parked.push_back(i);
      }
      if (notrun.empty() && parked.empty()) break;
      // 1. move every parked search into an arena 4x its current outer capacity: its own
      // allocation, or (when that fails, or HASTAR_RESUME_POOL=1 asks for it first) idle slot
      // arenas of the pool.  Not idle: the arenas this round's queue pass will use (the first
      // min(slots, not-run planners)), those that hold a parked state, and those lent to a live
      // resume arena.
      nxt.clear();
      std::vector<char> pool_busy((size_t)DC.n_arenas, 0);
      const int wq = notrun.empty() ? 0 : std::min<int>(slots - hoff, (int)notrun.size());
      for (int q = 0; q < hoff + wq && q < DC.n_arenas; ++q) pool_busy[(size_t)q] = 1;
      for (int i : parked)
        if (!in_resume[i] && DC.h_results[i].park_arena >= 0 && DC.h_results[i].park_arena < DC.n_arenas)
          pool_busy[(size_t)DC.h_results[i].park_arena] = 1;
      for (const ResumeArena& ra : cur)
        for (int q = 0; q < ra.pool_count; ++q) pool_busy[(size_t)(ra.pool_first + q)] = 1;
      auto carve_from_pool = [&](size_t bytes, ResumeArena& ra) -> bool {
        if (DC.arena_bytes == 0) return false;
        const int k = (int)((bytes + DC.arena_bytes - 1) / DC.arena_bytes);
        for (int j = 0, run = 0; j < DC.n_arenas; ++j) {
          run = pool_busy[(size_t)j] ? 0 : run + 1;
          if (run == k) {
            ra.pool_first = j - k + 1;
            ra.pool_count = k;
            for (int q = ra.pool_first; q <= j; ++q) pool_busy[(size_t)q] = 1;
            pool_used.push_back(ra.pool_first);
            pool_used.push_back(k);
            ++g_pooled_resumes;
            return true;
          }
        }
        return false;
      };
      for (int i : parked) {
        const SearchResult& R = DC.h_results[i];
        const SlotArena* from = nullptr;
        SlotArena host_from;
        if (in_resume[i]) {
          from = &cur[(size_t)R.park_arena].desc;
        } else if (R.park_arena >= DC.n_arenas) {  // a head arena (slot ids n_arenas + b)
          from = &DC.h_head[(size_t)(R.park_arena - DC.n_arenas)];
        } else {
          HIPCHK(hipMemcpy(&host_from, DC.d_arenas + R.park_arena, sizeof(SlotArena), hipMemcpyDeviceToHost));
          from = &host_from;
        }
        // the planner's capacity after R.parks parks (4x each), as the kernel computes it
        const long long was = std::min((long long)hs[i]->max_pops << (2 * std::min(R.parks - 1, 12)),
                                       (long long)SLOT3_IDX_MASK - 1);
        const long long pops = std::min((long long)hs[i]->max_pops << (2 * std::min(R.parks, 12)),
                                        (long long)SLOT3_IDX_MASK - 1);
        ArenaReq r = need;
        size_outer(r, pops, hs[i]->span);
        ResumeArena ra;
        const size_t bytes = arena_layout(r).total();
        bool have = false;
        if (pops > was) {
          if (pool_first) have = carve_from_pool(bytes, ra);
          size_t fr = 0, tot = 0;
          if (!have && hipMemGetInfo(&fr, &tot) == hipSuccess && fr < bytes + kHeadroom)
            have = carve_from_pool(bytes, ra);  // an allocation would eat the runtime's headroom
          if (!have) {
            have = hipMalloc(&ra.slab, bytes) == hipSuccess;
            if (!have) {
              ra.slab = nullptr;
              have = carve_from_pool(bytes, ra);
            }
          }
        }
        if (!have) {
          // no larger arena can be had: this search ends here, reported as an overflow
          DC.h_results[i].status = HASTAR_EOVERFLOW;
          DC.h_results[i].ok = 0;
          DC.h_results[i].path_len = 0;
          HIPCHK(hipMemcpyAsync(DC.d_results + i, DC.h_results + i, sizeof(SearchResult), hipMemcpyHostToDevice, st));
          continue;
        }
        char* where = ra.slab ? static_cast<char*>(ra.slab)
                              : static_cast<char*>(DC.slab) + DC.arena_bytes * (size_t)ra.pool_first;
        HIPCHK(carve_arena(where, r, arena_layout(r), &ra.desc, st));
        HIPCHK(hipMemcpyAsync(ra.desc.open3, from->open3, (size_t)R.ps3_next * sizeof(Node3), hipMemcpyDeviceToDevice, st));
        HIPCHK(hipMemcpyAsync(ra.desc.closed3, from->closed3, (size_t)R.n_closed3 * sizeof(Closed3),
                              hipMemcpyDeviceToDevice, st));
        ra.planner = i;
        nxt.push_back(ra);
      }
      HIPCHK(hipStreamSynchronize(st));
      for (ResumeArena& ra : cur)
        if (ra.slab) hipFree(ra.slab);  // their states have been copied out
      cur.swap(nxt);
      // 2. planners no wave took: a new queue pass over the slot arenas (free again)
      if (!notrun.empty()) {
        HIPCHK(hipMemcpyAsync(DC.d_order, notrun.data(), notrun.size() * sizeof(int), hipMemcpyHostToDevice, st));
        for (int i : notrun) in_resume[i] = 0;
        const int w = std::min<int>(slots - hoff, (int)notrun.size());
        if (int r = timed([&] {
              return wide ? launch_search_wide(DC.d_descs, (int)notrun.size(), DC.d_arenas + hoff, w, DC.d_order,
                                               DC.d_next, hard_pops, st, 0, hoff)
                          : launch_search(DC.d_descs, (int)notrun.size(), DC.d_arenas + hoff, w, DC.d_order, 0,
                                          DC.d_next, hard_pops, st, hoff);
            }))
          return r;
      }
      // 3. the parked searches continue, one wave each
      if (!cur.empty()) {
        std::vector<SlotArena> descs_r(cur.size());
        std::vector<int> ord(cur.size());
        for (size_t k = 0; k < cur.size(); ++k) {
          descs_r[k] = cur[k].desc;
          ord[k] = cur[k].planner;
          in_resume[cur[k].planner] = 1;
        }
        if (cur.size() > DC.resume_cap) {
          if (DC.d_resume) hipFree(DC.d_resume);
          if (DC.d_resume_order) hipFree(DC.d_resume_order);
          DC.d_resume = nullptr;
          DC.d_resume_order = nullptr;
          DC.resume_cap = 0;
          HIPCHK(dalloc(&DC.d_resume, cur.size()));
          HIPCHK(dalloc(&DC.d_resume_order, cur.size()));
          DC.resume_cap = cur.size();
        }
        HIPCHK(hipMemcpyAsync(DC.d_resume, descs_r.data(), cur.size() * sizeof(SlotArena), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(DC.d_resume_order, ord.data(), ord.size() * sizeof(int), hipMemcpyHostToDevice, st));
        if (int r = timed([&] { return launch_resume(DC.d_descs, (int)cur.size(), DC.d_resume, DC.d_resume_order,
                                                     hard_pops, st); }))
          return r;
      } else if (notrun.empty()) {
        break;
      }
    }
    for (ResumeArena& ra : cur)
      if (ra.slab) hipFree(ra.slab);
    // pool arenas lent to resume arenas get their generation-stamped tables back to a fresh
    // arena's state (same layout, so the device descriptors stay valid)
    if (!pool_used.empty()) {
      const ArenaLayout lay = arena_layout(DC.areq);
      for (size_t u = 0; u < pool_used.size(); u += 2)
        for (int q = pool_used[u]; q < pool_used[u] + pool_used[u + 1]; ++q) {
          SlotArena tmp;
          HIPCHK(carve_arena(static_cast<char*>(DC.slab) + DC.arena_bytes * (size_t)q, DC.areq, lay, &tmp, st));
        }
      HIPCHK(hipStreamSynchronize(st));
    }
  }
  // a search that parked in a split launch sizes the next split launches' head arenas
  if (split1) {
    // searches that outgrew their plain arena (parked, or ran through on a head arena's grant):
    // the next split launches give the head arenas room for the longest of them and widen the
    // head by their number, as long as one of the last kHeadWindow split launches had any
    long long want = 0;
    int big = 0;
    for (int i = 0; i < n; ++i)
      if (DC.h_results[i].parks > 0 || DC.h_results[i].pops > (long long)hs[i]->max_pops) {
        want = std::max(want, (long long)DC.h_results[i].pops);
        ++big;
      }
    constexpr int kHeadWindow = 8;
    DC.head_win_pops[DC.head_win_at] = want;
    DC.head_win_cnt[DC.head_win_at] = std::min(big, DC.n_cu / 8);
    DC.head_win_at = (DC.head_win_at + 1) % kHeadWindow;
    DC.head_want = 0;
    DC.head_extra = 0;
    for (int w = 0; w < kHeadWindow; ++w) {
      DC.head_want = std::max(DC.head_want, DC.head_win_pops[w]);
      DC.head_extra = std::max(DC.head_extra, DC.head_win_cnt[w]);
    }
  }
  g_last_ms = ms_total;
  return finish_batch(DC, hs, n, xyh, curv, cap, len, cost, ok, stats, true);
}

}  // extern "C"

// ---- RELAXED mode (hastar_relaxed.hip): non-parity by design ----
namespace {
size_t relax_bytes(int N, int nodes, RelaxArena* A, char* q) {
  const size_t NN = (size_t)N * N;
  const int bcap = 32 * N;
  uint32_t slots = 1;
  while (slots < 2u * (uint32_t)nodes + 64) slots <<= 1;
  const int dub_cap = 4 * N + 64;  // Dubins samples of one shot (as ArenaReq::dub)
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = q ? q + off : nullptr;
    off += align256(bytes);
    return p;
  };
  char* dist = take(NN * 4);
  char* bucket = take((size_t)8 * bcap * sizeof(BucketEntry));
  char* table = take((size_t)slots * sizeof(RelaxSlot));
  char* nodes_p = take((size_t)nodes * sizeof(Node3));
  char* lists = take((size_t)3 * nodes * 8);
  char* dxyh = take((size_t)relaxed_waves() * dub_cap * 12);
  char* dcurv = take((size_t)relaxed_waves() * dub_cap * 4);
  char* chain = take((size_t)(nodes + 2) * 4);
  if (A) {
    std::memset(A, 0, sizeof(*A));
    A->dist = reinterpret_cast<float*>(dist);
    A->bucket = reinterpret_cast<BucketEntry*>(bucket);
    A->bcap = bcap;
    A->table = reinterpret_cast<RelaxSlot*>(table);
    A->tmask = slots - 1;
    A->nodes = reinterpret_cast<Node3*>(nodes_p);
    A->node_cap = nodes;
    A->lists = reinterpret_cast<int*>(lists);
    A->list_cap = nodes;
    A->dub_xyh = reinterpret_cast<float*>(dxyh);
    A->dub_curv = reinterpret_cast<float*>(dcurv);
    A->dub_cap = dub_cap;
    A->chain = reinterpret_cast<int*>(chain);
    A->chain_cap = nodes + 2;
    A->cells = NN;
  }
  return off;
}
// debug: per-wave progress words of the relaxed kernel in pinned host memory, readable while
// a launch runs (HASTAR_RELAXED_PROGRESS set; hastar_debug_relaxed_progress)
unsigned* relaxed_progress() {
  static unsigned* words = nullptr;
  static bool tried = false;
  if (!tried) {
    tried = true;
    if (std::getenv("HASTAR_RELAXED_PROGRESS") &&
        hipHostMalloc(reinterpret_cast<void**>(&words), 4096 * 64 * sizeof(unsigned), hipHostMallocCoherent) != hipSuccess)
      words = nullptr;
    if (words) std::memset(words, 0, 4096 * 64 * sizeof(unsigned));
  }
  return words;
}
int relax_acquire(DeviceCtx& D, int N, int nodes, int want) {
  // the pool serves a call whose arenas it covers, with as many workgroups as it was sized for
  // (a pool capped by free HBM is not reallocated by every call that asks for more)
  if (D.n_rarenas > 0 && D.r_N >= N && D.r_nodes >= nodes && (D.n_rarenas >= want || D.r_asked >= want)) return 0;
  HIPCHK(hipStreamSynchronize(D.stream));
  if (D.rslab) hipFree(D.rslab);
  if (D.d_rarenas) hipFree(D.d_rarenas);
  D.rslab = nullptr;
  D.d_rarenas = nullptr;
  D.n_rarenas = 0;
  // sized for this call (a smaller node capacity gives smaller arenas and more workgroups)
  const size_t per = relax_bytes(N, nodes, nullptr, nullptr);
  size_t fr = 0, tot = 0;
  HIPCHK(hipMemGetInfo(&fr, &tot));
  const int n = (int)std::max<size_t>(1, std::min<size_t>((size_t)want, (size_t)(0.5 * (double)fr) / per));
  if (hipMalloc(&D.rslab, per * (size_t)n) != hipSuccess) {
    D.rslab = nullptr;
    return fail(HASTAR_ENOMEM, "relaxed arenas: hipMalloc failed");
  }
  std::vector<RelaxArena> host(n);
  for (int i = 0; i < n; ++i) {
    relax_bytes(N, nodes, &host[i], static_cast<char*>(D.rslab) + per * (size_t)i);
    // the best-g tables start empty; every search leaves its table empty again
    HIPCHK(hipMemsetAsync(host[i].table, 0xff, ((size_t)host[i].tmask + 1) * sizeof(RelaxSlot), D.stream));
  }
  HIPCHK(dalloc(&D.d_rarenas, (size_t)n));
  HIPCHK(hipMemcpyAsync(D.d_rarenas, host.data(), (size_t)n * sizeof(RelaxArena), hipMemcpyHostToDevice, D.stream));
  HIPCHK(hipStreamSynchronize(D.stream));
  D.n_rarenas = n;
  D.r_asked = want;
  D.r_N = N;
  D.r_nodes = nodes;
  return 0;
}
}  // namespace

extern "C" int hastar_find_path_relaxed_batch(const hastar_handle* hs, int n, const float* vel, const float* starts,
                                              float* xyh, float* curv, int cap, int* len, float* cost, int* ok,
                                              hastar_stats* stats, const hastar_relaxed_opts* opts) {
  return hastar_find_path_relaxed_batch_dir(hs, n, vel, starts, xyh, curv, nullptr, cap, len, cost, ok, stats, opts);
}

extern "C" int hastar_find_path_relaxed_batch_dir(const hastar_handle* hs, int n, const float* vel, const float* starts,
                                                  float* xyh, float* curv, signed char* dir, int cap, int* len,
                                                  float* cost, int* ok, hastar_stats* stats,
                                                  const hastar_relaxed_opts* opts) {
  if (!hs || n <= 0 || !vel || !starts || !len || !cost || !ok || cap < 0 || (cap > 0 && (!xyh || !curv)))
    return fail(HASTAR_EINVAL, "bad argument");
  const int dev = hs[0] ? hs[0]->device : -1;
  int N = 0;
  for (int i = 0; i < n; ++i) {
    if (!hs[i] || hs[i]->device != dev) return fail(HASTAR_EINVAL, "null handle or handles on different devices");
    if (!hs[i]->goal_set) return fail(HASTAR_EINVAL, "update_goal must be called before find_path");
    N = std::max(N, hs[i]->desc.N);
  }
  RelaxParams rp{};
  rp.delta = opts && opts->delta > 0.0f ? opts->delta : 0.25f;
  rp.h_stop = opts && opts->h_stop >= 1.0f ? opts->h_stop : 1.2f;
  rp.max_rounds = opts && opts->max_rounds > 0 ? opts->max_rounds : (1 << 20);
  rp.h_weight = opts && opts->h_weight > 0.0f ? opts->h_weight : 1.35f;
  rp.h_coarse = opts && opts->h_coarse > 0 ? opts->h_coarse : 2;
  if (rp.h_coarse != 1 && rp.h_coarse != 2 && rp.h_coarse != 4) return fail(HASTAR_EINVAL, "h_coarse must be 1, 2 or 4");
  rp.rev_cost = opts && opts->reverse_cost > 0.0f ? opts->reverse_cost : 0.0f;
  rp.gear_cost = opts && opts->reverse_cost > 0.0f && opts->gear_cost > 0.0f ? opts->gear_cost : 0.0f;
  if (opts && (!(opts->reverse_cost >= 0.0f) || !(opts->gear_cost >= 0.0f)))
    return fail(HASTAR_EINVAL, "reverse_cost and gear_cost must be >= 0");
  const int nodes = opts && opts->max_nodes > 0 ? opts->max_nodes : (1 << 18);
  HIPCHK(hipSetDevice(dev));
  DeviceCtx& DC = *hs[0]->dc;
  std::lock_guard<std::mutex> lk(DC.mu);
  hipStream_t st = DC.stream;
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, dev));
  int want = std::min(n, prop.multiProcessorCount);  // one 8-wave workgroup per CU (230 VGPRs)
  if (const char* e = std::getenv("HASTAR_RELAXED_GROUPS")) want = std::max(1, std::min(want, std::atoi(e)));
  if (int rc = relax_acquire(DC, N, nodes, want)) return rc;
  if (int rc = batch_acquire(DC, n)) return rc;
  std::vector<PlannerDev> descs(n);
  for (int i = 0; i < n; ++i) {
    prepare_start(hs[i], vel[i], starts + 3 * i);
    descs[i] = hs[i]->desc;
    descs[i].result = DC.d_results + i;
  }
  HIPCHK(hipMemcpyAsync(DC.d_descs, descs.data(), (size_t)n * sizeof(PlannerDev), hipMemcpyHostToDevice, st));
  // planners that keep their heuristic field: allocate it on first use
  const bool reuse = opts && opts->reuse_heuristic;
  std::vector<RelaxField> fields;
  if (reuse) {
    fields.resize(n);
    for (int i = 0; i < n; ++i) {
      hastar_handle h = hs[i];
      const size_t NN = (size_t)h->desc.N * h->desc.N;
      if (!h->rfield && hipMalloc(reinterpret_cast<void**>(&h->rfield), NN * sizeof(float)) != hipSuccess) {
        h->rfield = nullptr;
        return fail(HASTAR_ENOMEM, "relaxed heuristic field: hipMalloc failed");
      }
      fields[i] = RelaxField{h->rfield, h->rhlim, h->rvalid && h->rcoarse == rp.h_coarse ? 1 : 0, h->rstart};
    }
    if ((size_t)n > DC.rfields_cap) {
      HIPCHK(hipStreamSynchronize(st));
      if (DC.d_rfields) hipFree(DC.d_rfields);
      DC.d_rfields = nullptr;
      DC.rfields_cap = 0;
      HIPCHK(dalloc(&DC.d_rfields, (size_t)n));
      DC.rfields_cap = n;
    }
    HIPCHK(hipMemcpyAsync(DC.d_rfields, fields.data(), (size_t)n * sizeof(RelaxField), hipMemcpyHostToDevice, st));
  }
  rp.progress = relaxed_progress();
  // per-pose directions: a device slab of n x (the largest output buffer), copied out below
  int dstride = 0;
  if (dir && cap > 0) {
    for (int i = 0; i < n; ++i) dstride = std::max(dstride, hs[i]->desc.out_cap);
    const size_t bytes = (size_t)n * dstride;
    if (bytes > DC.dir_cap) {
      HIPCHK(hipStreamSynchronize(st));
      if (DC.d_dir) hipFree(DC.d_dir);
      DC.d_dir = nullptr;
      DC.dir_cap = 0;
      if (hipMalloc(reinterpret_cast<void**>(&DC.d_dir), bytes) != hipSuccess) {
        DC.d_dir = nullptr;
        return fail(HASTAR_ENOMEM, "relaxed directions: hipMalloc failed");
      }
      DC.dir_cap = bytes;
    }
    rp.dir_out = DC.d_dir;
    rp.dir_stride = dstride;
  }
  HIPCHK(hipEventRecord(DC.ev0, st));
  HIPCHK(launch_relaxed(DC.d_descs, n, DC.d_rarenas, std::min(want, DC.n_rarenas), DC.d_next, rp,
                        reuse ? DC.d_rfields : nullptr, st));
  HIPCHK(hipEventRecord(DC.ev1, st));
  HIPCHK(hipMemcpyAsync(DC.h_results, DC.d_results, (size_t)n * sizeof(SearchResult), hipMemcpyDeviceToHost, st));
  if (reuse)
    HIPCHK(hipMemcpyAsync(fields.data(), DC.d_rfields, (size_t)n * sizeof(RelaxField), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  for (int i = 0; reuse && i < n; ++i) {
    hs[i]->rvalid = fields[i].valid != 0;
    hs[i]->rhlim = fields[i].hlim;
    hs[i]->rstart = fields[i].start_ij;
    hs[i]->rcoarse = rp.h_coarse;
  }
  float ms = 0.0f;
  hipEventElapsedTime(&ms, DC.ev0, DC.ev1);
  g_last_ms = ms;
  const int rc = finish_batch(DC, hs, n, xyh, curv, cap, len, cost, ok, stats, false);
  if (rp.dir_out) {
    std::vector<signed char> hd((size_t)n * dstride);
    HIPCHK(hipMemcpy(hd.data(), DC.d_dir, hd.size(), hipMemcpyDeviceToHost));
    for (int i = 0; i < n; ++i) {
      const int k = std::min(std::min(len[i], cap), dstride);
      std::memcpy(dir + (size_t)i * cap, hd.data() + (size_t)i * dstride, (size_t)std::max(k, 0));
    }
  }
  return rc;
}

extern "C" {

const unsigned* hastar_debug_relaxed_progress(void) { return relaxed_progress(); }

int hastar_copy_path(hastar_handle h, float* xyh, float* curv, int cap, int* len) {
  if (!h || !h->have_last) return fail(HASTAR_EINVAL, "no search result");
  HIPCHK(hipSetDevice(h->device));
  int r = copy_path_out(h, xyh, curv, cap, len, h->dc->stream);
  HIPCHK(hipStreamSynchronize(h->dc->stream));
  return r;
}

// VelocityGenerator<float> (VelocityGenerator.cpp:7-84) over a batch of paths: inputs are
// packed into one device slab, profiled by k_velocity_profile (one thread per path) on the
// device context's stream, and copied back.
int hastar_velocity_profile_batch(int device, const hastar_velocity_params* vp, int n, const long long* offsets,
                                  const float* xyh, const float* curv, const float* vel_init,
                                  const float* max_velocity_curr, const unsigned char* flags, float* velocity,
                                  unsigned char* feasible) {
  if (!vp || n < 0 || (n > 0 && (!offsets || !xyh || !curv || !vel_init || !max_velocity_curr || !flags ||
                                 !velocity || !feasible)))
    return fail(HASTAR_EINVAL, "velocity_profile: null argument");
  if (n == 0) return HASTAR_OK;
  if (offsets[0] != 0) return fail(HASTAR_EINVAL, "velocity_profile: offsets[0] must be 0");
  for (int p = 0; p < n; ++p)
    if (offsets[p + 1] <= offsets[p]) return fail(HASTAR_EINVAL, "velocity_profile: path " + std::to_string(p) + " is empty");
  const size_t pts = (size_t)offsets[n];
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev || device > 63)
    return fail(HASTAR_EDEVICE, "velocity_profile: no HIP device " + std::to_string(device));
  std::lock_guard<std::mutex> lk(g_dev[device].mu);  // the device context and its stream
  DeviceCtx* D = nullptr;
  if (int r = device_ctx(device, &D)) return r;
  HIPCHK(hipSetDevice(device));
  const size_t b_off = align256((n + 1) * sizeof(long long)), b_xyh = align256(3 * pts * sizeof(float)),
               b_pt = align256(pts * sizeof(float)), b_pf = align256(n * sizeof(float)), b_pb = align256(n);
  const size_t total = b_off + b_xyh + 2 * b_pt + 2 * b_pf + 2 * b_pb;
  hipStream_t st = D->stream;
  if (int r = vel_slab_acquire(*D, total)) return r;
  char* q = D->vel_slab;
  auto take = [&](size_t b) { char* r = q; q += b; return r; };
  long long* d_off = reinterpret_cast<long long*>(take(b_off));
  float* d_xyh = reinterpret_cast<float*>(take(b_xyh));
  float* d_curv = reinterpret_cast<float*>(take(b_pt));
  float* d_vel = reinterpret_cast<float*>(take(b_pt));
  float* d_v0 = reinterpret_cast<float*>(take(b_pf));
  float* d_vmax = reinterpret_cast<float*>(take(b_pf));
  unsigned char* d_flags = reinterpret_cast<unsigned char*>(take(b_pb));
  unsigned char* d_feas = reinterpret_cast<unsigned char*>(take(b_pb));
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) { if (e == hipSuccess) e = x; };
  chk(hipMemcpyAsync(d_off, offsets, (n + 1) * sizeof(long long), hipMemcpyHostToDevice, st));
  chk(hipMemcpyAsync(d_xyh, xyh, 3 * pts * sizeof(float), hipMemcpyHostToDevice, st));
  chk(hipMemcpyAsync(d_curv, curv, pts * sizeof(float), hipMemcpyHostToDevice, st));
  chk(hipMemcpyAsync(d_v0, vel_init, n * sizeof(float), hipMemcpyHostToDevice, st));
  chk(hipMemcpyAsync(d_vmax, max_velocity_curr, n * sizeof(float), hipMemcpyHostToDevice, st));
  chk(hipMemcpyAsync(d_flags, flags, n, hipMemcpyHostToDevice, st));
  const hastar::VelParams P{vp->max_velocity, vp->coast_velocity, vp->max_lat_acc, vp->max_lat_acc * vp->max_lat_acc,
                            vp->max_long_acc, vp->max_long_dec};
  if (e == hipSuccess) chk(hastar::launch_velocity_profile(P, n, d_off, d_xyh, d_curv, d_v0, d_vmax, d_flags, d_vel, d_feas, st));
  chk(hipMemcpyAsync(velocity, d_vel, pts * sizeof(float), hipMemcpyDeviceToHost, st));
  chk(hipMemcpyAsync(feasible, d_feas, n, hipMemcpyDeviceToHost, st));
  chk(hipStreamSynchronize(st));
  if (e != hipSuccess) return fail(HASTAR_EDEVICE, std::string("velocity_profile: ") + hipGetErrorString(e));
  return HASTAR_OK;
}

// VelocityGenerator over the paths of the device's last hastar_find_path_batch, which are
// still packed in HBM (local_planner.cpp:316-323 profiles the search's own output): no
// path upload.  Path i is the batch's planner i with len[i] points at the offsets the
// batch packed (a planner with len 0 gets feasible 0 and no velocities).
int hastar_velocity_profile_last_batch(int device, const hastar_velocity_params* vp, int n, const float* vel_init,
                                       const float* max_velocity_curr, const unsigned char* flags, float* velocity,
                                       unsigned char* feasible) {
  if (!vp || n < 0 || (n > 0 && (!vel_init || !max_velocity_curr || !flags || !feasible)))
    return fail(HASTAR_EINVAL, "velocity_profile_last_batch: null argument");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev || device > 63)
    return fail(HASTAR_EDEVICE, "velocity_profile_last_batch: no HIP device " + std::to_string(device));
  std::lock_guard<std::mutex> lk(g_dev[device].mu);
  DeviceCtx* D = nullptr;
  if (int r = device_ctx(device, &D)) return r;
  if (n != D->last_n) return fail(HASTAR_EINVAL, "velocity_profile_last_batch: n differs from the last batch");
  if (n == 0) return HASTAR_OK;
  const size_t pts = (size_t)D->last_total;
  if (pts == 0) {  // the last batch returned no path: nothing to profile, nothing feasible
    std::memset(feasible, 0, (size_t)n);
    return HASTAR_OK;
  }
  if (!velocity) return fail(HASTAR_EINVAL, "velocity_profile_last_batch: null velocity");
  HIPCHK(hipSetDevice(device));
  const size_t b_pt = align256(std::max<size_t>(pts, 1) * sizeof(float)), b_pf = align256(n * sizeof(float)),
               b_pb = align256(n);
  if (int r = vel_slab_acquire(*D, b_pt + 2 * b_pf + 2 * b_pb)) return r;
  char* q = D->vel_slab;
  float* d_vel = reinterpret_cast<float*>(q); q += b_pt;
  float* d_v0 = reinterpret_cast<float*>(q); q += b_pf;
  float* d_vmax = reinterpret_cast<float*>(q); q += b_pf;
  unsigned char* d_flags = reinterpret_cast<unsigned char*>(q); q += b_pb;
  unsigned char* d_feas = reinterpret_cast<unsigned char*>(q);
  hipStream_t st = D->stream;
  HIPCHK(hipMemcpyAsync(d_v0, vel_init, n * sizeof(float), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(d_vmax, max_velocity_curr, n * sizeof(float), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(d_flags, flags, n, hipMemcpyHostToDevice, st));
  const hastar::VelParams P{vp->max_velocity, vp->coast_velocity, vp->max_lat_acc, vp->max_lat_acc * vp->max_lat_acc,
                            vp->max_long_acc, vp->max_long_dec};
  HIPCHK(hastar::launch_velocity_profile(P, n, D->d_off, D->d_pxyh, D->d_pcurv, d_v0, d_vmax, d_flags, d_vel, d_feas, st));
  if (pts > 0) HIPCHK(hipMemcpyAsync(velocity, d_vel, pts * sizeof(float), hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(feasible, d_feas, n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return HASTAR_OK;
}

// ------------------------------------------- AStar<float> / Grid2D<float> on a handle ---
// The reference's AStar class owns a plain Grid2D (AStar.h:63-66 without
// STORE_GRID_AS_REFERENCE): its goal change only re-orients the frame (no relocation,
// Grid2D.cpp:260-266) and its start cell truncates the rotated offset before adding the
// goal cell (Grid2D.cpp:270-290).  These entry points give a planner handle those
// semantics; map updates, reset and get_obstacles are the planner's own.
int hastar_grid2d_update_goal_heading(hastar_handle h, const float goal[2], const float start[2]) {
  if (!h || !goal || !start) return fail(HASTAR_EINVAL, "null argument");
  h->goal2x = goal[0];
  h->goal2y = goal[1];
  h->grid_heading = g_atan2f(goal[1] - start[1], goal[0] - start[0]);
  PlannerDev& D = h->desc;
  D.goal_cx = D.n45;
  D.goal_cy = D.n2;
  D.grid_heading = h->grid_heading;
  h->goal_set = true;
  h->rvalid = false;
  return HASTAR_OK;
}

static float euclid_h_host(const PlannerDev& P, int i, int j) {  // Grid2D.cpp:303-316, as euclid_h
  const float dx = (float)(P.n45 - i) * P.res;
  const float dx2 = dx * dx;
  const float dy = (float)(P.n2 - j) * P.res;
  const float dy2 = dy * dy;
  return std::sqrt(dx2 + dy2);
}

// Node2D::soft_reset of cell (i, j) (Grid2D.cpp:294-299): its f becomes its h
int hastar_grid2d_set_start_node_grid(hastar_handle h, int i, int j) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  const PlannerDev& D = h->desc;
  if (i < 0 || i >= D.N || j < 0 || j >= D.N) return fail(HASTAR_EINVAL, "cell outside the grid");
  HIPCHK(hipSetDevice(h->device));
  const float f = euclid_h_host(D, i, j);
  HIPCHK(hipMemcpyAsync(D.nm_f + (size_t)i * D.N + j, &f, sizeof(float), hipMemcpyHostToDevice, h->dc->stream));
  HIPCHK(hipStreamSynchronize(h->dc->stream));
  return HASTAR_OK;
}

// Grid2D::set_start_node(start) (Grid2D.cpp:270-290): cell[0..1] = the start cell
int hastar_grid2d_set_start_node(hastar_handle h, const float start[2], int cell[2]) {
  if (!h || !start || !cell) return fail(HASTAR_EINVAL, "null argument");
  const PlannerDev& D = h->desc;
  const float gh = h->grid_heading, c = g_cosf(gh), s = g_sinf(gh);
  const float dx = start[0] - h->goal2x, dy = start[1] - h->goal2y;
  const float rx = dx * c + dy * s, ry = -dx * s + dy * c;
  int i = gmath::x86_trunc_int(rx / D.res) + D.n45, j = gmath::x86_trunc_int(ry / D.res) + D.n2;
  if (!(i > -1 && i < D.N && j > -1 && j < D.N)) i = j = 0;
  cell[0] = i;
  cell[1] = j;
  return hastar_grid2d_set_start_node_grid(h, i, j);
}

// ---- Grid3D<float> on a handle (Grid3D.h:14-46) ----
// Grid3D::set_start_node (Grid3D.cpp:127-160): the start node in the grid frame and its
// cell, whose node is soft-reset; default action, velocity 0 (find_path sets its own)
int hastar_grid3d_set_start_node(hastar_handle h, const float start[3], hastar_node3_f32* node, int cell[2]) {
  if (!h || !start || !node || !cell) return fail(HASTAR_EINVAL, "null argument");
  if (!h->goal_set) return fail(HASTAR_EINVAL, "update_goal must come first");
  prepare_start(h, 0.0f, start);
  const PlannerDev& D = h->desc;
  node->x = D.start_x;
  node->y = D.start_y;
  node->heading = D.start_h;
  node->g = 0.0f;
  node->vmin_sqr = 0.0f;
  node->curvature_index = D.start_ci;
  node->angle_bin = D.start_bin;
  cell[0] = D.start_cx;
  cell[1] = D.start_cy;
  return hastar_grid2d_set_start_node_grid(h, D.start_cx, D.start_cy);
}

// the goal node of Grid3D::update_goal_heading (Grid3D.cpp:115-123)
int hastar_grid3d_goal_node(hastar_handle h, hastar_node3_f32* node) {
  if (!h || !node) return fail(HASTAR_EINVAL, "null argument");
  const PlannerDev& D = h->desc;
  node->x = D.goal_x;
  node->y = D.goal_y;
  node->heading = D.goal_h;
  node->g = 0.0f;
  node->vmin_sqr = 0.0f;
  node->curvature_index = 0;
  node->angle_bin = D.goal_bin;
  return HASTAR_OK;
}

// Grid3D::get_neighbors (Grid3D.cpp:47-74) of one node on the device
int hastar_grid3d_neighbors(hastar_handle h, const hastar_node3_f32* node, int cap, hastar_node3_f32* out, int* cells,
                            int* count, int* neglect) {
  if (!h || !node || !count || !neglect || cap < 0 || (cap > 0 && (!out || !cells)))
    return fail(HASTAR_EINVAL, "bad argument");
  const PlannerDev& D = h->desc;
  if (node->angle_bin < 0 || node->angle_bin > D.bins || node->curvature_index < 0 || node->curvature_index >= D.nsteer)
    return fail(HASTAR_EINVAL, "node angle bin / curvature index out of range");
  HIPCHK(hipSetDevice(h->device));
  DeviceCtx& DC = *h->dc;
  std::lock_guard<std::mutex> lk(DC.mu);
  const int oc = std::max(cap, 1);
  const size_t b_desc = align256(sizeof(PlannerDev)), b_out = align256((size_t)oc * 7 * sizeof(float));
  const size_t b_cells = align256((size_t)oc * 2 * sizeof(int));
  if (int rc = stage_acquire(DC, b_desc + b_out + b_cells + 256)) return rc;
  char* q = DC.stage;
  PlannerDev* d_desc = reinterpret_cast<PlannerDev*>(q);
  float* d_out = reinterpret_cast<float*>(q + b_desc);
  int* d_cells = reinterpret_cast<int*>(q + b_desc + b_out);
  int* d_cnt = reinterpret_cast<int*>(q + b_desc + b_out + b_cells);
  HIPCHK(hipMemcpyAsync(d_desc, &D, sizeof(PlannerDev), hipMemcpyHostToDevice, DC.stream));
  const float nd[5] = {node->x, node->y, node->heading, node->g, node->vmin_sqr};
  HIPCHK(launch_grid3d_neighbors(d_desc, nd, node->curvature_index, node->angle_bin, d_out, d_cells, cap, d_cnt,
                                 d_cnt + 1, DC.stream));
  int cn[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(cn, d_cnt, sizeof(cn), hipMemcpyDeviceToHost, DC.stream));
  HIPCHK(hipStreamSynchronize(DC.stream));
  *count = cn[0];
  *neglect = cn[1];
  const int k = std::min(cn[0], cap);
  if (k > 0) {
    std::vector<float> o((size_t)k * 7);
    HIPCHK(hipMemcpy(o.data(), d_out, o.size() * sizeof(float), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(cells, d_cells, (size_t)k * 2 * sizeof(int), hipMemcpyDeviceToHost));
    for (int i = 0; i < k; ++i) {
      const float* r = &o[(size_t)7 * i];
      out[i].x = r[0];
      out[i].y = r[1];
      out[i].heading = r[2];
      out[i].g = r[3];
      out[i].vmin_sqr = r[4];
      std::memcpy(&out[i].curvature_index, &r[5], 4);
      std::memcpy(&out[i].angle_bin, &r[6], 4);
    }
  }
  if (cn[0] > cap) return fail(HASTAR_ENOSPC, "neighbor buffer too small (*count = required)");
  return HASTAR_OK;
}

// Grid3D::check_path (Grid3D.cpp:78-93): *is_free = 1 when every sample's rounded cell is
// inside the grid and below the threshold
int hastar_grid3d_check_path(hastar_handle h, const float* xyh, int n, int* is_free) {
  if (!h || !is_free || n < 0 || (n > 0 && !xyh)) return fail(HASTAR_EINVAL, "bad argument");
  HIPCHK(hipSetDevice(h->device));
  DeviceCtx& DC = *h->dc;
  std::lock_guard<std::mutex> lk(DC.mu);
  const size_t b_desc = align256(sizeof(PlannerDev)), b_path = align256((size_t)std::max(n, 1) * 3 * sizeof(float));
  if (int rc = stage_acquire(DC, b_desc + b_path + 256)) return rc;
  char* q = DC.stage;
  PlannerDev* d_desc = reinterpret_cast<PlannerDev*>(q);
  float* d_path = reinterpret_cast<float*>(q + b_desc);
  int* d_free = reinterpret_cast<int*>(q + b_desc + b_path);
  HIPCHK(hipMemcpyAsync(d_desc, &h->desc, sizeof(PlannerDev), hipMemcpyHostToDevice, DC.stream));
  if (n > 0) HIPCHK(hipMemcpyAsync(d_path, xyh, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice, DC.stream));
  HIPCHK(launch_grid3d_check_path(d_desc, d_path, n, d_free, DC.stream));
  HIPCHK(hipMemcpyAsync(is_free, d_free, sizeof(int), hipMemcpyDeviceToHost, DC.stream));
  HIPCHK(hipStreamSynchronize(DC.stream));
  return HASTAR_OK;
}

// Grid2D::clear_obstacles (Grid2D.cpp:66-71): every log-odds cell back to 0
int hastar_grid2d_clear(hastar_handle h) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipMemsetAsync(h->desc.occ, 0, (size_t)h->desc.N * h->desc.N * sizeof(float), h->dc->stream));
  return HASTAR_OK;
}

// AStar::update_goal_node (AStar.cpp:24-28): searches end at this cell
int hastar_astar_set_goal_cell(hastar_handle h, int i, int j) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  if (i < 0 || i >= h->desc.N || j < 0 || j >= h->desc.N) return fail(HASTAR_EINVAL, "cell outside the grid");
  h->desc.goal_cx = i;
  h->desc.goal_cy = j;
  return HASTAR_OK;
}

// Grid2D::get_node_total_cost (Grid2D.cpp:229-233)
int hastar_grid2d_node_cost(hastar_handle h, int i, int j, float* f) {
  if (!h || !f) return fail(HASTAR_EINVAL, "null argument");
  const PlannerDev& D = h->desc;
  if (i < 0 || i >= D.N || j < 0 || j >= D.N) return fail(HASTAR_EINVAL, "cell outside the grid");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipMemcpyAsync(f, D.nm_f + (size_t)i * D.N + j, sizeof(float), hipMemcpyDeviceToHost, h->dc->stream));
  HIPCHK(hipStreamSynchronize(h->dc->stream));
  return HASTAR_OK;
}

// One holonomic search on the device (k_astar_query).  mode: 1 memo test of the start,
// 2 get_cost_only, 4 path (cap points of xy, world frame, goal's predecessor first).
static int astar_run(hastar_handle h, int si, int sj, int mode, const float goal_w[2], float* cost, float* xy, int cap,
                     int* n) {
  const PlannerDev& D = h->desc;
  if (si < 0 || si >= D.N || sj < 0 || sj >= D.N) return fail(HASTAR_EINVAL, "cell outside the grid");
  if (!h->goal_set) return fail(HASTAR_EINVAL, "update_goal / update_goal_start must come first");
  HIPCHK(hipSetDevice(h->device));
  DeviceCtx& DC = *h->dc;
  std::lock_guard<std::mutex> lk(DC.mu);
  if (int rc = arenas_acquire(DC, h->areq, 1)) return rc;
  if (int rc = head_release(DC)) return rc;
  const int pcap = std::max(cap, 1);
  const size_t bytes = align256(sizeof(PlannerDev)) + 256 + align256((size_t)pcap * 2 * sizeof(float)) + 256;
  if (int rc = stage_acquire(DC, bytes)) return rc;
  char* q = DC.stage;
  PlannerDev* d_desc = reinterpret_cast<PlannerDev*>(q);
  float* d_cost = reinterpret_cast<float*>(q + align256(sizeof(PlannerDev)));
  int* d_n = reinterpret_cast<int*>(q + align256(sizeof(PlannerDev)) + 16);
  float* d_xy = reinterpret_cast<float*>(q + align256(sizeof(PlannerDev)) + 256);
  HIPCHK(hipMemcpyAsync(d_desc, &D, sizeof(PlannerDev), hipMemcpyHostToDevice, DC.stream));
  const float ang = -h->grid_heading;
  HIPCHK(launch_astar_query(d_desc, DC.d_arenas, si, sj, mode, goal_w ? goal_w[0] : 0.0f, goal_w ? goal_w[1] : 0.0f,
                            g_cosf(ang), g_sinf(ang), d_cost, d_xy, cap, d_n, DC.stream));
  int nn = 0;
  HIPCHK(hipMemcpyAsync(cost, d_cost, sizeof(float), hipMemcpyDeviceToHost, DC.stream));
  HIPCHK(hipMemcpyAsync(&nn, d_n, sizeof(int), hipMemcpyDeviceToHost, DC.stream));
  HIPCHK(hipStreamSynchronize(DC.stream));
  if (nn == -2) return fail(HASTAR_EOVERFLOW, "holonomic search outgrew its open-set arena (max_astar_nodes)");
  if (n) *n = nn;
  if (nn == -1) return fail(HASTAR_ENOSPC, "path buffer too small");
  if (nn > 0 && xy) HIPCHK(hipMemcpy(xy, d_xy, (size_t)nn * 2 * sizeof(float), hipMemcpyDeviceToHost));
  return HASTAR_OK;
}

// AStar::find_path(int, int) (AStar.cpp:100-113): memo test, then a cost-only search
int hastar_astar_cost(hastar_handle h, int i, int j, float* cost) {
  if (!h || !cost) return fail(HASTAR_EINVAL, "null argument");
  return astar_run(h, i, j, 1 | 2, nullptr, cost, nullptr, 0, nullptr);
}

// AStar::find_path(goal, start, get_cost_only) and find_path(goal, start, path)
// (AStar.cpp:70-97): re-orient the frame (no relocation), soft-reset the start cell, search.
// With path != NULL (cap points), *n points of the predecessor chain follow the goal (the
// reference's path = goal, then these).
int hastar_astar_find_path(hastar_handle h, const float goal[2], const float start[2], int cost_only, float* cost,
                           float* xy, int cap, int* n) {
  if (!h || !goal || !start || !cost) return fail(HASTAR_EINVAL, "null argument");
  if (int rc = hastar_grid2d_update_goal_heading(h, goal, start)) return rc;
  int cell[2];
  if (int rc = hastar_grid2d_set_start_node(h, start, cell)) return rc;
  const int mode = cost_only ? 2 : (xy ? 4 : 0);
  return astar_run(h, cell[0], cell[1], mode, goal, cost, xy, cap, n);
}

// ---------------------------------------------------------------- test hooks --------
int hastar_test_math(int fn, const float* a, const float* b, float* out, int n) {
  if (n <= 0) return HASTAR_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(HASTAR_EDEVICE, "no HIP device");
  float *da = nullptr, *db = nullptr, *dout = nullptr;
  HIPCHK(dalloc(&da, n));
  HIPCHK(dalloc(&db, n));
  HIPCHK(dalloc(&dout, n));
  HIPCHK(hipMemcpy(da, a, n * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(db, b ? b : a, n * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(launch_test_math(fn, da, db, dout, n, nullptr));
  HIPCHK(hipMemcpy(out, dout, n * sizeof(float), hipMemcpyDeviceToHost));
  hipFree(da);
  hipFree(db);
  hipFree(dout);
  return HASTAR_OK;
}

int hastar_test_field(hastar_handle h, const float* poses, int n, float* out) {
  if (!h || n < 0) return fail(HASTAR_EINVAL, "bad argument");
  if (n == 0) return HASTAR_OK;
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->dc->stream));
  float *dp = nullptr, *dout = nullptr;
  HIPCHK(dalloc(&dp, (size_t)n * 3));
  HIPCHK(dalloc(&dout, (size_t)n));
  HIPCHK(hipMemcpy(dp, poses, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(launch_test_field(h->desc, dp, n, dout, nullptr));
  HIPCHK(hipMemcpy(out, dout, (size_t)n * sizeof(float), hipMemcpyDeviceToHost));
  hipFree(dp);
  hipFree(dout);
  return HASTAR_OK;
}

int hastar_test_dubins_len(float r, const float* starts, int n, const float goal[3], float* out, int* word) {
  if (n <= 0) return HASTAR_OK;
  float *ds = nullptr, *dout = nullptr;
  int* dw = nullptr;
  HIPCHK(dalloc(&ds, (size_t)n * 3));
  HIPCHK(dalloc(&dout, (size_t)n));
  HIPCHK(dalloc(&dw, (size_t)n));
  HIPCHK(hipMemcpy(ds, starts, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(launch_test_dubins_len(r, ds, n, goal[0], goal[1], goal[2], dout, dw, nullptr));
  HIPCHK(hipMemcpy(out, dout, (size_t)n * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(word, dw, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
  hipFree(ds);
  hipFree(dout);
  hipFree(dw);
  return HASTAR_OK;
}

int hastar_test_reeds_shepp(float r, const float* starts, int n, const float goal[3], float* len, int* word, float* seg,
                            float* len_groups) {
  if (n <= 0) return HASTAR_OK;
  if (!starts || !goal || !len || !word || !seg || !len_groups || !(r > 0.0f)) return fail(HASTAR_EINVAL, "bad argument");
  float *ds = nullptr, *dl = nullptr, *dseg = nullptr, *dg = nullptr;
  int* dw = nullptr;
  HIPCHK(dalloc(&ds, (size_t)n * 3));
  HIPCHK(dalloc(&dl, (size_t)n));
  HIPCHK(dalloc(&dseg, (size_t)n * 5));
  HIPCHK(dalloc(&dg, (size_t)n * 2));
  HIPCHK(dalloc(&dw, (size_t)n));
  HIPCHK(hipMemcpy(ds, starts, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(launch_test_rs(r, ds, n, goal[0], goal[1], goal[2], dl, dw, dseg, dg, nullptr));
  HIPCHK(hipMemcpy(len, dl, (size_t)n * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(word, dw, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(seg, dseg, (size_t)n * 5 * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(len_groups, dg, (size_t)n * 2 * sizeof(float), hipMemcpyDeviceToHost));
  hipFree(ds);
  hipFree(dl);
  hipFree(dseg);
  hipFree(dg);
  hipFree(dw);
  return HASTAR_OK;
}

int hastar_test_dubins_path(hastar_handle h, const float start[3], float* xyh, float* curv, int cap, int* n,
                            float* length, int* first_arc_gt_90) {
  if (!h || !h->goal_set) return fail(HASTAR_EINVAL, "bad handle / no goal");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->dc->stream));
  float *dx = nullptr, *dc = nullptr, *dl = nullptr;
  int *dn = nullptr, *df = nullptr;
  HIPCHK(dalloc(&dx, (size_t)cap * 3));
  HIPCHK(dalloc(&dc, (size_t)cap));
  HIPCHK(dalloc(&dl, 1));
  HIPCHK(dalloc(&dn, 1));
  HIPCHK(dalloc(&df, 1));
  HIPCHK(launch_test_dubins_path(h->desc, start[0], start[1], start[2], dx, dc, cap, dn, dl, df, nullptr));
  HIPCHK(hipMemcpy(n, dn, sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(length, dl, sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(first_arc_gt_90, df, sizeof(int), hipMemcpyDeviceToHost));
  if (*n > 0 && *n <= cap) {
    HIPCHK(hipMemcpy(xyh, dx, (size_t)(*n) * 3 * sizeof(float), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(curv, dc, (size_t)(*n) * sizeof(float), hipMemcpyDeviceToHost));
  }
  hipFree(dx);
  hipFree(dc);
  hipFree(dl);
  hipFree(dn);
  hipFree(df);
  return HASTAR_OK;
}

int hastar_debug_memo(hastar_handle h, float* f_out, unsigned char* visited_out) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->dc->stream));
  const size_t NN = (size_t)h->desc.N * h->desc.N;
  HIPCHK(hipMemcpy(f_out, h->desc.nm_f, NN * sizeof(float), hipMemcpyDeviceToHost));
  std::vector<uint32_t> bits(bitmap_words(NN));
  HIPCHK(hipMemcpy(bits.data(), h->desc.visited, bits.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < NN; ++i) visited_out[i] = (bits[i >> 5] >> (i & 31)) & 1u;
  return HASTAR_OK;
}

int hastar_debug_apf(hastar_handle h, float* out, int cap) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  const int n = h->desc.n_apf;
  if (n > cap) return n;
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->dc->stream));
  if (n) HIPCHK(hipMemcpy(out, h->desc.apf, (size_t)n * 3 * sizeof(float), hipMemcpyDeviceToHost));
  return n;
}

int hastar_debug_motion(hastar_handle h, float* off, float* dth, float* cost, float* curv_abs, float* prec,
                        float* r_min) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->dc->stream));
  const PlannerDev& D = h->desc;
  const int ns = D.nsteer;
  HIPCHK(hipMemcpy(off, D.off, (size_t)ns * (D.bins + 1) * 2 * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(dth, D.dth, ns * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(cost, D.act_cost, ns * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(curv_abs, D.curv_abs, ns * sizeof(float), hipMemcpyDeviceToHost));
  *prec = D.prec;
  *r_min = D.r_min;
  return HASTAR_OK;
}

int hastar_debug_cycles(hastar_handle h, unsigned long long* out8) {
  if (!h || !h->have_last) return fail(HASTAR_EINVAL, "no search result");
  for (int q = 0; q < NSTAMP; ++q) out8[q] = h->last.cycles[q];
  return HASTAR_OK;
}

int hastar_debug_timing(hastar_handle h, unsigned long long* out3) {
  if (!h || !h->have_last) return fail(HASTAR_EINVAL, "no search result");
  out3[0] = h->last.t_start;
  out3[1] = h->last.t_end;
  out3[2] = (unsigned long long)h->last.slot;
  return HASTAR_OK;
}

int hastar_debug_hw_id(hastar_handle h, int* out) {
  if (!h || !out || !h->have_last) return fail(HASTAR_EINVAL, "no search result");
  *out = h->last.hw_id;
  return HASTAR_OK;
}

// Search-slot pool of the handle's device: {resident wavefronts (occupancy x CUs), search
// waves per CU, arenas in the pool, MiB per arena}.
int hastar_debug_pooled_resumes(long long* out) {
  if (!out) return fail(HASTAR_EINVAL, "null output");
  *out = g_pooled_resumes.load();
  return HASTAR_OK;
}

int hastar_debug_relaxed_pool(hastar_handle h, long long* out2) {
  if (!h || !h->dc || !out2) return fail(HASTAR_EINVAL, "bad argument");
  out2[0] = h->dc->n_rarenas;
  out2[1] = h->dc->n_rarenas > 0 ? (long long)(relax_bytes(h->dc->r_N, h->dc->r_nodes, nullptr, nullptr) >> 20) : 0;
  return 0;
}

int hastar_debug_split(hastar_handle h, float* out4) {
  if (!h || !h->dc || !out4) return fail(HASTAR_EINVAL, "bad argument");
  for (int i = 0; i < 4; ++i) out4[i] = h->dc->split_ms[i];
  return 0;
}

int hastar_debug_handoffs(hastar_handle h, int* out) {
  if (!h || !h->dc || !out) return fail(HASTAR_EINVAL, "bad argument");
  *out = h->dc->handoffs;
  return 0;
}

int hastar_debug_slots(hastar_handle h, long long* out5) {
  if (!h || !h->dc) return fail(HASTAR_EINVAL, "bad handle");
  const DeviceCtx& D = *h->dc;
  out5[0] = D.resident_slots;
  out5[1] = search_slots_per_cu();
  out5[2] = D.n_arenas;
  out5[3] = (long long)(D.arena_bytes >> 20);
  out5[4] = D.head_cus;
  return HASTAR_OK;
}

int hastar_debug_head_arenas(hastar_handle h, long long* out3) {
  if (!h || !h->dc || !out3) return fail(HASTAR_EINVAL, "bad handle");
  const DeviceCtx& D = *h->dc;
  out3[0] = D.head_n;
  out3[1] = D.head_k;
  out3[2] = D.head_grant;
  return HASTAR_OK;
}

int hastar_debug_astar_modes(hastar_handle h, long long* out2) {
  if (!h || !h->have_last) return fail(HASTAR_EINVAL, "no search result");
  out2[0] = h->last.astar_migrations;
  out2[1] = h->last.astar_pops_hbm;
  return HASTAR_OK;
}

// Closed-set keys of the last search.  The closed records live in the slot arena that
// ran it, so this hook is only meaningful right after a single-planner find_path.
int hastar_debug_closed_keys(hastar_handle h, int* out, int cap) {
  if (!h || !h->have_last) return fail(HASTAR_EINVAL, "no search result");
  HIPCHK(hipSetDevice(h->device));
  DeviceCtx& DC = *h->dc;
  std::lock_guard<std::mutex> lk(DC.mu);
  HIPCHK(hipStreamSynchronize(DC.stream));
  if (DC.n_arenas < 1) return fail(HASTAR_EINVAL, "no arena");
  SlotArena A0;
  HIPCHK(hipMemcpy(&A0, DC.d_arenas, sizeof(SlotArena), hipMemcpyDeviceToHost));
  const int n = (int)h->last.closed_size;
  std::vector<Closed3> rec(n);
  if (n) HIPCHK(hipMemcpy(rec.data(), A0.closed3, (size_t)n * sizeof(Closed3), hipMemcpyDeviceToHost));
  std::vector<long long> k(n);
  for (int i = 0; i < n; ++i) {
    const uint32_t kk = rec[i].key;
    k[i] = ((long long)(kk >> 20) << 40) | ((long long)((kk >> 8) & 0xfff) << 16) | (kk & 0xff);
  }
  std::sort(k.begin(), k.end());
  for (int i = 0; i < n && i < cap; ++i) {
    out[3 * i] = (int)(k[i] >> 40);
    out[3 * i + 1] = (int)((k[i] >> 16) & 0xffffff);
    out[3 * i + 2] = (int)(k[i] & 0xffff);
  }
  return n;
}

}  // extern "C"
