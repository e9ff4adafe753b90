// hastar_f64.cpp — host runtime of the double planner (include/hastar_f64.h):
// HybridAStar<double> and VelocityGenerator<double> (HybridAStar.cpp:285-286,
// VelocityGenerator.cpp:88-89) over the kernels of hastar_f64.hip.
//
// Scalar preparation (constructor tables, grid frame, raster parameters, start node) runs
// here with the reference's double arithmetic and the host's glibc libm — the same calls the
// reference makes, so these values are the reference's bit for bit; every per-cell and
// per-expansion operation runs on the GPU.  Each handle owns one HIP stream and its search
// arena.  A search that outgrows its arena is re-run from the same memo state in a 4x larger
// one (the reference's sets have no limit, HybridAStar.cpp:107), so arena sizes never change
// a result.  There is no CPU fallback.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hastar_f64.h"
#include "glibc_mathf.h"
#include "hastar_f64_kernels.h"
#include "hastar_f64_layout.h"

namespace hastar {
int set_last_error(int code, const std::string& msg);  // hastar_capi.cpp (hastar_last_error)
}

using namespace hastar;

namespace {

int fail64(int code, const std::string& msg) { return set_last_error(code, msg); }

#define HIPCHK64(expr)                                                                                    \
  do {                                                                                                    \
    hipError_t e_ = (expr);                                                                               \
    if (e_ != hipSuccess) return fail64(HASTAR_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// common.h helpers with T = double (host glibc libm, as the reference)
double wrap_pi64(double a) {
  const double w = std::fmod(a, 2 * M_PI);
  if (w > M_PI) return w - 2 * M_PI;
  if (w < -M_PI) return w + 2 * M_PI;
  return w;
}
int heading_bin64(double h, double prec) {
  const double r = std::round(h / prec) * prec;
  return gmath::x86_trunc_int((r + M_PI) / prec);
}
struct V2d {
  double x, y;
};
V2d rot2d(double x, double y, double ang) {  // Vector2D::get_rotated_vector (common.h:55-61)
  const double c = std::cos(ang), s = std::sin(ang);
  return {x * c + y * s, -x * s + y * c};
}
double logodds(double p) { return std::log(p / (1.0 - p)); }  // Grid2D.cpp:11-14
size_t bitmap_words64(size_t NN) { return ((NN + 31) / 32 + 3) & ~(size_t)3; }
size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace

struct hastar64_s {
  int device = 0;
  hipStream_t st = nullptr;
  Planner64Dev D{};            // host copy of the descriptor
  Planner64Dev* d_desc = nullptr;
  Result64* d_res = nullptr;
  double lp_min = 0, lp_max = 0, lp_free = 0;
  double grid_heading = 0, goal2x = 0, goal2y = 0, goal3x = 0, goal3y = 0, goal3h = 0;
  int span = 3;
  // persistent state: maps, memo, tables, APF list, map scratch, memo snapshot
  void* slab = nullptr;
  double* tmp = nullptr;       // N*N relocation target
  int* winner = nullptr;       // N*N, kept at -1
  int* cnt = nullptr;          // N*N raster hit counters, kept at 0
  double* snap_f = nullptr;    // memo snapshot (a re-run starts from it)
  uint32_t* snap_vis = nullptr;
  double* apf = nullptr;
  int apf_cap = 0;
  // raster staging
  void* stage = nullptr;
  size_t stage_cap = 0;
  // search arena
  void* arena = nullptr;
  long long pops_cap = 0;
  int astar_cap = 0, dub_cap = 0;
  // output
  double* out = nullptr;
  int out_cap = 0;
  std::vector<double> last_xyh, last_curv;
  int last_len = 0, reruns = 0;
};

namespace {

void free64(hastar64_handle h) {
  if (!h) return;
  hipSetDevice(h->device);
  if (h->st) hipStreamSynchronize(h->st);
  for (void* p : {(void*)h->d_desc, (void*)h->d_res, h->slab, h->apf ? (void*)h->apf : nullptr, h->stage, h->arena,
                  (void*)h->out})
    if (p) hipFree(p);
  if (h->st) hipStreamDestroy(h->st);
  delete h;
}

// (re)carve the search arena for pops_cap / astar_cap / dub_cap
int arena_alloc(hastar64_handle h) {
  Planner64Dev& D = h->D;
  const size_t NN = (size_t)D.N * D.N;
  const long long open3 = (long long)(h->span - 1) * h->pops_cap + 66, closed3 = h->pops_cap + 1;
  uint32_t slots = 1;
  while (slots < 2 * (uint64_t)closed3 + 64) slots <<= 1;
  if (open3 > (1ll << 30) || closed3 > (1ll << 30) || h->astar_cap > (1 << 30) || h->dub_cap > (1 << 28))
    return fail64(HASTAR_EOVERFLOW, "search arena beyond 2^30 records");
  const size_t b3 = al256((size_t)open3 * sizeof(Node3d)), bc = al256((size_t)closed3 * sizeof(Closed3d)),
               bs = al256((size_t)slots * sizeof(Slot3d)), b2 = al256(((size_t)h->astar_cap + 1) * sizeof(Node2d)),
               bcell = al256(NN * sizeof(Cell2d)), bd = al256((size_t)h->dub_cap * 3 * sizeof(double)),
               bdc = al256((size_t)h->dub_cap * sizeof(double)), bch = al256((size_t)closed3 * sizeof(int)),
               bg = 256;
  const size_t total = b3 + bc + bs + b2 + bcell + bd + bdc + bch + bg;
  // the new arena is allocated before the old one is freed, so that a failed growth leaves the
  // planner its current arena; when both do not fit at once, the old one is freed first and the
  // allocation retried (peak = the larger arena alone).  If that fails too, h->arena is null and
  // the caller restores the caps and carves the old size again (arena_restore).
  void* fresh = nullptr;
  if (hipMalloc(&fresh, total) != hipSuccess) {
    (void)hipGetLastError();
    if (!h->arena)
      return fail64(HASTAR_EOVERFLOW, "search arena of " + std::to_string(total >> 20) + " MiB cannot be allocated");
    HIPCHK64(hipStreamSynchronize(h->st));
    hipFree(h->arena);
    h->arena = nullptr;
    if (hipMalloc(&fresh, total) != hipSuccess) {
      (void)hipGetLastError();
      return fail64(HASTAR_EOVERFLOW, "search arena of " + std::to_string(total >> 20) + " MiB cannot be allocated");
    }
  }
  HIPCHK64(hipStreamSynchronize(h->st));
  if (h->arena) hipFree(h->arena);
  h->arena = fresh;
  char* q = static_cast<char*>(h->arena);
  D.open3 = reinterpret_cast<Node3d*>(q); q += b3;
  D.open3_cap = (int)open3;
  D.closed3 = reinterpret_cast<Closed3d*>(q); q += bc;
  D.closed3_cap = (int)closed3;
  D.slots3 = reinterpret_cast<Slot3d*>(q); q += bs;
  D.slots3_mask = slots - 1;
  D.open2 = reinterpret_cast<Node2d*>(q); q += b2;
  D.open2_cap = h->astar_cap + 1;
  D.cell2 = reinterpret_cast<Cell2d*>(q); q += bcell;
  D.dub_xyh = reinterpret_cast<double*>(q); q += bd;
  D.dub_curv = reinterpret_cast<double*>(q); q += bdc;
  D.dub_cap = h->dub_cap;
  D.chain = reinterpret_cast<int*>(q); q += bch;
  D.gens = reinterpret_cast<uint32_t*>(q);
  // fresh tables: every generation stamp 0, the counters at 0
  HIPCHK64(hipMemsetAsync(D.slots3, 0, bs, h->st));
  HIPCHK64(hipMemsetAsync(D.cell2, 0, bcell, h->st));
  HIPCHK64(hipMemsetAsync(D.gens, 0, bg, h->st));
  return HASTAR_OK;
}

int stage_need(hastar64_handle h, size_t bytes) {
  if (bytes <= h->stage_cap) return HASTAR_OK;
  HIPCHK64(hipStreamSynchronize(h->st));
  if (h->stage) hipFree(h->stage);
  h->stage = nullptr;
  h->stage_cap = 0;
  HIPCHK64(hipMalloc(&h->stage, bytes));
  h->stage_cap = bytes;
  return HASTAR_OK;
}

int check64(const hastar_params_f64* p) {
  if (p->grid_size < 2 || p->grid_size > 4095) return fail64(HASTAR_EINVAL, "grid_size must be in [2, 4095]");
  if (p->num_angle_bins < 1 || p->num_angle_bins > 254) return fail64(HASTAR_EINVAL, "num_angle_bins must be in [1, 254]");
  if (p->num_steering < 1 || p->num_steering > 16 || !p->steering || !p->curvature_weights)
    return fail64(HASTAR_EINVAL, "num_steering must be in [1, 16] with steering/curvature_weights arrays");
  if (p->num_actions < 0 || p->max_pops < 0 || p->max_astar_nodes < 0 || p->max_dubins_samples < 0)
    return fail64(HASTAR_EINVAL, "negative count");
  if (!(p->grid_resolution > 0) || !(p->step_size > 0)) return fail64(HASTAR_EINVAL, "resolution/step must be > 0");
  return 0;
}

}  // namespace

extern "C" {

// HybridAStar<double>::HybridAStar (HybridAStar.cpp:7-24): Grid2D (Grid2D.cpp:7-62),
// VehicleModel (VehicleModel.cpp:7-47), Dubins radius (HybridAStar.cpp:22-24, HybridAStar.h:20-25)
int hastar64_create(const hastar_params_f64* p, int device, hastar64_handle* out) {
  if (!p || !out) return fail64(HASTAR_EINVAL, "null argument");
  *out = nullptr;
  if (int rc = check64(p)) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail64(HASTAR_EDEVICE, "no HIP device available (this library has no CPU path)");
  if (device < 0 || device >= ndev) return fail64(HASTAR_EINVAL, "device ordinal out of range");
  HIPCHK64(hipSetDevice(device));
  hastar64_handle h = new hastar64_s();
  h->device = device;
  if (hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking) != hipSuccess) {
    h->st = nullptr;
    free64(h);
    return fail64(HASTAR_EDEVICE, "stream creation failed");
  }
  Planner64Dev& D = h->D;
  const int N = p->grid_size;
  D.N = N;
  D.n2 = (int)std::round(N * 0.5);
  D.n45 = (int)std::round(N * 0.8);
  D.diag = p->grid_2d_allow_diag_moves ? 1 : 0;
  D.bins = p->num_angle_bins;
  D.nsteer = p->num_steering;
  D.na = p->num_actions;
  D.shot_interval = p->dubins_shot_interval;
  D.shot_decay = p->dubins_shot_interval_decay;
  D.res = p->grid_resolution;
  D.thr = logodds(p->obstacle_threshold);
  h->lp_min = logodds(p->obstacle_prob_min);
  h->lp_max = logodds(p->obstacle_prob_max);
  h->lp_free = logodds(p->obstacle_prob_free);
  D.apf_rep = p->apf_rep_constant;
  D.apf_ang = p->apf_active_angle;
  D.act_cost_axis = D.res * std::sqrt(1.0);
  D.act_cost_diag = D.res * std::sqrt(2.0);
  D.ts = p->step_size;
  D.a_lat = p->max_lat_acc;
  D.a_lat2 = p->max_lat_acc * p->max_lat_acc;
  D.prec = 2 * M_PI / D.bins;
  const int ns = D.nsteer, bins = D.bins;
  std::vector<double> beta(ns), curv(ns), dth(ns), cost(ns), ca(ns), off((size_t)ns * (bins + 1) * 2, 0.0);
  for (int i = 0; i < ns; ++i) {
    beta[i] = std::atan2(p->rear_to_cg * std::tan(p->steering[i]), p->wheelbase);
    curv[i] = std::cos(beta[i]) * std::tan(p->steering[i]) / p->wheelbase;
  }
  for (int i = 0; i < ns; ++i) {
    dth[i] = D.ts * curv[i];
    cost[i] = D.ts + p->curvature_weights[i] * std::abs(curv[i]);
    for (int j = 0; j < bins; ++j) {  // calculate_offset (VehicleModel.cpp:147-164)
      const double head = -M_PI + j * D.prec;
      const double dt = 0.001;
      double ox = 0, oy = 0, hh = head;
      const int nup = (int)(D.ts / dt);
      for (int k = 0; k < nup; ++k) {
        ox += dt * std::cos(beta[i] + hh);
        oy += dt * std::sin(beta[i] + hh);
        hh += dt * curv[i];
      }
      off[2 * ((size_t)i * (bins + 1) + j)] = ox;
      off[2 * ((size_t)i * (bins + 1) + j) + 1] = oy;
    }
    // row `bins` stays (0, 0): the reference's one-past-the-end read (VehicleModel.cpp:145)
  }
  for (int i = 0; i < ns; ++i) ca[i] = std::abs(curv[i]);
  const double tm = std::tan(*std::max_element(p->steering, p->steering + ns));
  D.r_min = p->wheelbase / (std::cos(std::atan2(p->rear_to_cg * tm, p->wheelbase)) * tm);
  D.step = p->step_size;
  D.ang_step = p->step_size / D.r_min;
  h->span = std::max(2, std::min(2 * D.na + 1, D.nsteer));
  // persistent device state
  const size_t NN = (size_t)N * N;
  const size_t b_map = al256(NN * sizeof(double)), b_vis = al256(bitmap_words64(NN) * sizeof(uint32_t)),
               b_int = al256(NN * sizeof(int)), b_off = al256(off.size() * sizeof(double)),
               b_s = al256((size_t)ns * sizeof(double));
  const size_t total = 4 * b_map + 2 * b_vis + 2 * b_int + b_off + 3 * b_s + b_s;
  if (hipMalloc(&h->slab, total) != hipSuccess || hipMalloc(reinterpret_cast<void**>(&h->d_desc), sizeof(Planner64Dev)) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&h->d_res), sizeof(Result64)) != hipSuccess) {
    free64(h);
    return fail64(HASTAR_ENOMEM, "planner state allocation failed");
  }
  char* q = static_cast<char*>(h->slab);
  D.occ = reinterpret_cast<double*>(q); q += b_map;
  D.nm_f = reinterpret_cast<double*>(q); q += b_map;
  h->tmp = reinterpret_cast<double*>(q); q += b_map;
  h->snap_f = reinterpret_cast<double*>(q); q += b_map;
  D.visited = reinterpret_cast<uint32_t*>(q); q += b_vis;
  h->snap_vis = reinterpret_cast<uint32_t*>(q); q += b_vis;
  h->winner = reinterpret_cast<int*>(q); q += b_int;
  h->cnt = reinterpret_cast<int*>(q); q += b_int;
  D.off = reinterpret_cast<double*>(q); q += b_off;
  D.dth = reinterpret_cast<double*>(q); q += b_s;
  D.act_cost = reinterpret_cast<double*>(q); q += b_s;
  D.curv_abs = reinterpret_cast<double*>(q); q += b_s;
  D.result = h->d_res;
  // arena defaults (include/hastar_f64.h)
  h->pops_cap = p->max_pops > 0 ? p->max_pops : 65536;
  h->astar_cap = p->max_astar_nodes > 0 ? p->max_astar_nodes : (int)std::min<size_t>(NN + 16, 65536);
  h->dub_cap = p->max_dubins_samples > 0 ? p->max_dubins_samples
                                         : (int)(2.0 * N * D.res / D.step) + 2 * (int)(2 * M_PI / D.ang_step + 2) + 64;
  hipStream_t st = h->st;
  hipError_t he = hipMemsetAsync(D.occ, 0, NN * sizeof(double), st);
  if (he == hipSuccess) he = hipMemsetAsync(D.visited, 0, bitmap_words64(NN) * sizeof(uint32_t), st);
  if (he == hipSuccess) he = hipMemsetAsync(h->winner, 0xff, NN * sizeof(int), st);
  if (he == hipSuccess) he = hipMemsetAsync(h->cnt, 0, NN * sizeof(int), st);
  if (he == hipSuccess) he = hipMemcpyAsync(D.off, off.data(), off.size() * sizeof(double), hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = hipMemcpyAsync(D.dth, dth.data(), ns * sizeof(double), hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = hipMemcpyAsync(D.act_cost, cost.data(), ns * sizeof(double), hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = hipMemcpyAsync(D.curv_abs, ca.data(), ns * sizeof(double), hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = hipMemcpyAsync(h->d_desc, &D, sizeof(D), hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = launch64_init_nodemap(h->d_desc, N, st);
  if (he == hipSuccess) he = hipStreamSynchronize(st);  // the host vectors go out of scope
  if (he != hipSuccess) {
    free64(h);
    return fail64(HASTAR_EDEVICE, std::string("init: ") + hipGetErrorString(he));
  }
  if (int rc = arena_alloc(h)) {
    free64(h);
    return rc;
  }
  *out = h;
  return HASTAR_OK;
}

int hastar64_destroy(hastar64_handle h) {
  if (!h) return fail64(HASTAR_EINVAL, "null handle");
  free64(h);
  return HASTAR_OK;
}

int hastar64_grid_size(hastar64_handle h) { return h ? h->D.N : HASTAR_EINVAL; }

// update_goal: Grid3D::update_goal_heading + relocate_obstacles (Grid3D.cpp:102-124, 169-203)
int hastar64_update_goal(hastar64_handle h, const double goal[3], const double start[3]) {
  if (!h || !goal || !start) return fail64(HASTAR_EINVAL, "null argument");
  HIPCHK64(hipSetDevice(h->device));
  Planner64Dev& D = h->D;
  const double gh_prev = h->grid_heading;
  const double g3px = h->goal3x, g3py = h->goal3y;
  h->goal2x = goal[0];
  h->goal2y = goal[1];
  h->grid_heading = std::atan2(goal[1] - start[1], goal[0] - start[0]);
  h->goal3x = goal[0];
  h->goal3y = goal[1];
  h->goal3h = goal[2];
  const double gh = h->grid_heading, dh = gh - gh_prev;
  const V2d gp = rot2d((double)D.n45, (double)D.n2, dh);
  const V2d gno = rot2d(g3px - h->goal3x, g3py - h->goal3y, gh);
  V2d org{(double)D.n45 + gno.x / D.res, (double)D.n2 + gno.y / D.res};
  org = {org.x - gp.x, org.y - gp.y};
  const size_t NN = (size_t)D.N * D.N;
  HIPCHK64(launch64_relocate(D.N, std::cos(dh), std::sin(dh), org.x, org.y, D.occ, h->tmp, h->winner, h->st));
  HIPCHK64(hipMemcpyAsync(D.occ, h->tmp, NN * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  // the goal node (Grid3D.cpp:115-123)
  D.goal_x = D.n45 * D.res;
  D.goal_y = D.n2 * D.res;
  D.goal_h = wrap_pi64(goal[2] - gh);
  D.goal_bin = heading_bin64(D.goal_h, D.prec);
  D.goal_cx = D.n45;
  D.goal_cy = D.n2;
  D.world_goal_x = goal[0];
  D.world_goal_y = goal[1];
  D.neg_heading = -gh;
  D.rot_c = std::cos(-gh);
  D.rot_s = std::sin(-gh);
  return HASTAR_OK;
}

// reset() -> AStar::reset (AStar.cpp:56-60)
int hastar64_reset(hastar64_handle h) {
  if (!h) return fail64(HASTAR_EINVAL, "null handle");
  HIPCHK64(hipSetDevice(h->device));
  HIPCHK64(hipMemsetAsync(h->D.visited, 0, bitmap_words64((size_t)h->D.N * h->D.N) * sizeof(uint32_t), h->st));
  return HASTAR_OK;
}

// update_obstacles() (Grid2D.cpp:197-208)
int hastar64_decay(hastar64_handle h) {
  if (!h) return fail64(HASTAR_EINVAL, "null handle");
  HIPCHK64(hipSetDevice(h->device));
  HIPCHK64(launch64_decay(h->D.occ, (size_t)h->D.N * h->D.N, h->lp_free, h->lp_min, h->lp_max, h->st));
  return HASTAR_OK;
}

// update_obstacles(boxes) (Grid3D.cpp:22-44 + Grid2D.cpp:99-139)
int hastar64_update_boxes(hastar64_handle h, const double* boxes, const double* conf, int n, double apf_r) {
  if (!h || n < 0 || (n > 0 && (!boxes || !conf))) return fail64(HASTAR_EINVAL, "bad argument");
  HIPCHK64(hipSetDevice(h->device));
  Planner64Dev& D = h->D;
  const double gh = h->grid_heading;
  std::vector<double> apf((size_t)n * 3), dl((size_t)n);
  std::vector<int> rp((size_t)n * 4);
  for (int k = 0; k < n; ++k) {
    const double ox = boxes[4 * k], oy = boxes[4 * k + 1], dx = boxes[4 * k + 2], dy = boxes[4 * k + 3];
    V2d pp = rot2d(ox - h->goal3x, oy - h->goal3y, gh);
    pp.x += D.n45 * D.res;
    pp.y += D.n2 * D.res;
    apf[3 * k] = pp.x;
    apf[3 * k + 1] = pp.y;
    apf[3 * k + 2] = std::max(dx, dy) / 2 + apf_r;
    const V2d bl = rot2d((ox - dx / 2) - h->goal2x, (oy - dy / 2) - h->goal2y, gh);
    rp[4 * k] = gmath::x86_trunc_int(std::round(bl.x / D.res) + D.n45);
    rp[4 * k + 1] = gmath::x86_trunc_int(std::round(bl.y / D.res) + D.n2);
    rp[4 * k + 2] = std::max(0, 2 * gmath::x86_trunc_int(std::ceil(dx / D.res)));
    rp[4 * k + 3] = std::max(0, 2 * gmath::x86_trunc_int(std::ceil(dy / D.res)));
    dl[k] = logodds(conf[k]) - h->lp_free;
  }
  // the APF list replaces the previous one (Grid3D.cpp:26-27)
  if (n > h->apf_cap) {
    HIPCHK64(hipStreamSynchronize(h->st));
    if (h->apf) hipFree(h->apf);
    h->apf = nullptr;
    h->apf_cap = 0;
    HIPCHK64(hipMalloc(reinterpret_cast<void**>(&h->apf), (size_t)n * 3 * sizeof(double)));
    h->apf_cap = n;
  }
  D.apf = h->apf;
  D.n_apf = n;
  if (n == 0) return HASTAR_OK;
  const size_t b_rp = al256(rp.size() * sizeof(int)), b_dl = al256(dl.size() * sizeof(double));
  if (int rc = stage_need(h, b_rp + b_dl)) return rc;
  HIPCHK64(hipStreamSynchronize(h->st));  // the staging buffer may still feed an earlier launch
  int* d_rp = static_cast<int*>(h->stage);
  double* d_dl = reinterpret_cast<double*>(static_cast<char*>(h->stage) + b_rp);
  HIPCHK64(hipMemcpyAsync(h->apf, apf.data(), apf.size() * sizeof(double), hipMemcpyHostToDevice, h->st));
  HIPCHK64(hipMemcpyAsync(d_rp, rp.data(), rp.size() * sizeof(int), hipMemcpyHostToDevice, h->st));
  HIPCHK64(hipMemcpyAsync(d_dl, dl.data(), dl.size() * sizeof(double), hipMemcpyHostToDevice, h->st));
  HIPCHK64(launch64_raster_boxes(D.occ, h->cnt, D.N, d_rp, d_dl, n, std::cos(gh), std::sin(gh), h->lp_min, h->lp_max,
                                 h->st));
  HIPCHK64(hipStreamSynchronize(h->st));  // pageable host vectors
  return HASTAR_OK;
}

// update_obstacles(lines) (Grid2D.cpp:142-194)
int hastar64_update_lines(hastar64_handle h, const double* lines, const double* conf, int n, double width) {
  if (!h || n < 0 || (n > 0 && (!lines || !conf))) return fail64(HASTAR_EINVAL, "bad argument");
  HIPCHK64(hipSetDevice(h->device));
  if (n == 0) return HASTAR_OK;
  Planner64Dev& D = h->D;
  const double gh = h->grid_heading;
  std::vector<double> wid;
  for (double pw = 0; pw <= width; pw += D.res) {
    wid.push_back(pw);
    if (wid.size() > (1u << 20)) return fail64(HASTAR_EINVAL, "line_width / resolution too large");
  }
  if (wid.empty()) return HASTAR_OK;
  const int stride = 100;
  std::vector<double> lp((size_t)n * 9), seq((size_t)n * stride);
  for (int k = 0; k < n; ++k) {
    const V2d a = rot2d(lines[4 * k] - h->goal2x, lines[4 * k + 1] - h->goal2y, gh);
    const V2d b = rot2d(lines[4 * k + 2] - h->goal2x, lines[4 * k + 3] - h->goal2y, gh);
    V2d d{b.x - a.x, b.y - a.y};
    const double len = std::hypot(d.x, d.y);
    const V2d nrm{-d.y / len, d.x / len};
    d = {d.x / len, d.y / len};
    int cntl = 0;
    double pl = 0;
    for (; pl <= len && cntl < 100; ++cntl, pl += D.res) seq[(size_t)k * stride + cntl] = pl;
    double* L = &lp[(size_t)k * 9];
    L[0] = a.x;
    L[1] = a.y;
    L[2] = d.x;
    L[3] = d.y;
    L[4] = nrm.x;
    L[5] = nrm.y;
    L[6] = logodds(conf[k]) - h->lp_free;
    L[7] = cntl;
    L[8] = (double)wid.size();
  }
  const size_t b_lp = al256(lp.size() * sizeof(double)), b_seq = al256(seq.size() * sizeof(double)),
               b_wid = al256(wid.size() * sizeof(double));
  if (int rc = stage_need(h, b_lp + b_seq + b_wid)) return rc;
  HIPCHK64(hipStreamSynchronize(h->st));
  char* s = static_cast<char*>(h->stage);
  double* d_lp = reinterpret_cast<double*>(s);
  double* d_seq = reinterpret_cast<double*>(s + b_lp);
  double* d_wid = reinterpret_cast<double*>(s + b_lp + b_seq);
  HIPCHK64(hipMemcpyAsync(d_lp, lp.data(), lp.size() * sizeof(double), hipMemcpyHostToDevice, h->st));
  HIPCHK64(hipMemcpyAsync(d_seq, seq.data(), seq.size() * sizeof(double), hipMemcpyHostToDevice, h->st));
  HIPCHK64(hipMemcpyAsync(d_wid, wid.data(), wid.size() * sizeof(double), hipMemcpyHostToDevice, h->st));
  HIPCHK64(launch64_raster_lines(D.occ, h->cnt, D.N, D.n45, D.n2, D.res, d_lp, d_seq, d_wid, stride, n, h->lp_min,
                                 h->lp_max, h->st));
  HIPCHK64(hipStreamSynchronize(h->st));
  return HASTAR_OK;
}

int hastar64_get_obstacles(hastar64_handle h, double* out) {
  if (!h || !out) return fail64(HASTAR_EINVAL, "null argument");
  HIPCHK64(hipSetDevice(h->device));
  HIPCHK64(hipMemcpyAsync(out, h->D.occ, (size_t)h->D.N * h->D.N * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK64(hipStreamSynchronize(h->st));
  return HASTAR_OK;
}

// find_path (HybridAStar.cpp:68-88): set_start_node (Grid3D.cpp:127-160) here, the search and
// reconstruct_path (HybridAStar.cpp:93-262) on the device
int hastar64_find_path(hastar64_handle h, double vel, const double start[3], double* xyh, double* curv, int cap,
                       int* len, double* cost, int* ok, hastar_stats* stats) {
  if (!h || !start || !len || !cost || !ok || cap < 0 || (cap > 0 && (!xyh || !curv)))
    return fail64(HASTAR_EINVAL, "bad argument");
  HIPCHK64(hipSetDevice(h->device));
  Planner64Dev& D = h->D;
  *len = 0;
  *cost = DBL_MAX;
  *ok = 0;
  h->last_len = 0;
  if (!h->arena) return fail64(HASTAR_ENOMEM, "the planner has no search arena");
  // Vector3D::get_rotated_vector (common.h:162-169) of the start relative to the goal
  const double rx = start[0] - h->goal3x, ry = start[1] - h->goal3y;
  const double c = std::cos(h->grid_heading), s = std::sin(h->grid_heading);
  const double px = (rx * c + ry * s) + D.n45 * D.res, py = (-rx * s + ry * c) + D.n2 * D.res;
  const double ph = wrap_pi64(start[2] - h->grid_heading);
  const int i = gmath::x86_trunc_int(px / D.res), j = gmath::x86_trunc_int(py / D.res);
  if (i > -1 && i < D.N && j > -1 && j < D.N) {
    D.start_x = px;
    D.start_y = py;
    D.start_h = ph;
    D.start_cx = i;
    D.start_cy = j;
  } else {
    D.start_x = D.start_y = D.start_h = 0.0;
    D.start_cx = D.start_cy = 0;
  }
  D.start_bin = heading_bin64(D.start_h, D.prec);
  D.start_ci = D.nsteer / 2;  // VehicleModel::get_default_action_index (VehicleModel.cpp:57-60)
  D.start_vmin = vel * vel;
  const size_t NN = (size_t)D.N * D.N, vis_bytes = bitmap_words64(NN) * sizeof(uint32_t);
  // the memo before the search: a re-run in a larger arena starts from it again
  HIPCHK64(hipMemcpyAsync(h->snap_f, D.nm_f, NN * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  HIPCHK64(hipMemcpyAsync(h->snap_vis, D.visited, vis_bytes, hipMemcpyDeviceToDevice, h->st));
  Result64 R{};
  h->reruns = 0;
  int status = 0;
  for (;;) {
    HIPCHK64(hipMemcpyAsync(h->d_desc, &D, sizeof(D), hipMemcpyHostToDevice, h->st));
    HIPCHK64(launch64_search(h->d_desc, 1, h->st));
    HIPCHK64(hipMemcpyAsync(&R, h->d_res, sizeof(R), hipMemcpyDeviceToHost, h->st));
    HIPCHK64(hipStreamSynchronize(h->st));
    if (!R.need) break;
    HIPCHK64(hipMemcpyAsync(D.nm_f, h->snap_f, NN * sizeof(double), hipMemcpyDeviceToDevice, h->st));
    HIPCHK64(hipMemcpyAsync(D.visited, h->snap_vis, vis_bytes, hipMemcpyDeviceToDevice, h->st));
    const int was_pops = h->pops_cap, was_astar = h->astar_cap, was_dub = h->dub_cap;
    if (R.need & NEED_OUTER) h->pops_cap = (int)std::min<long long>(4ll * h->pops_cap, 1ll << 30);
    if (R.need & NEED_INNER) h->astar_cap = (int)std::min<long long>(4ll * h->astar_cap, 1ll << 30);
    if (R.need & NEED_SHOT) h->dub_cap = (int)std::min<long long>(4ll * h->dub_cap, 1ll << 28);
    ++h->reruns;
    if (int rc = arena_alloc(h)) {  // no larger arena: the reference's failure pair, status EOVERFLOW
      status = rc;
      // the planner keeps the capacities of its current arena; arena_alloc kept that arena unless
      // it had to free it to retry, and then it is carved again at the old size
      h->pops_cap = was_pops;
      h->astar_cap = was_astar;
      h->dub_cap = was_dub;
      if (!h->arena) {
        if (int rc2 = arena_alloc(h)) status = rc2;
      }
      break;
    }
  }
  if (stats) {
    *stats = hastar_stats{};
    stats->pops = R.pops;
    stats->successors = R.successors;
    stats->astar_pops = R.astar_pops;
    stats->astar_searches = R.astar_searches;
    stats->shots = R.shots;
    stats->closed_size = R.closed_size;
    stats->pop_digest = R.pop_digest;
    stats->closed_digest = R.closed_digest;
    stats->via_shot = R.via_shot;
    stats->status = status;
    stats->parks = h->reruns;
  }
  if (status) return status;
  *cost = R.cost;
  *ok = R.ok;
  if (!R.ok) return HASTAR_OK;
  const int L = R.path_len;
  if (L > h->out_cap) {
    HIPCHK64(hipStreamSynchronize(h->st));
    if (h->out) hipFree(h->out);
    h->out = nullptr;
    h->out_cap = 0;
    const int nc = std::max(L, 1024);
    HIPCHK64(hipMalloc(reinterpret_cast<void**>(&h->out), (size_t)nc * 4 * sizeof(double)));
    h->out_cap = nc;
  }
  D.out_xyh = h->out;
  D.out_curv = h->out + 3 * (size_t)h->out_cap;
  D.out_cap = h->out_cap;
  HIPCHK64(hipMemcpyAsync(h->d_desc, &D, sizeof(D), hipMemcpyHostToDevice, h->st));
  HIPCHK64(launch64_reconstruct(h->d_desc, 1, h->st));
  h->last_xyh.resize((size_t)L * 3);
  h->last_curv.resize((size_t)L);
  HIPCHK64(hipMemcpyAsync(h->last_xyh.data(), D.out_xyh, (size_t)L * 3 * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK64(hipMemcpyAsync(h->last_curv.data(), D.out_curv, (size_t)L * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK64(hipStreamSynchronize(h->st));
  h->last_len = L;
  *len = L;
  if (L > cap) {
    if (stats) stats->status = HASTAR_ENOSPC;
    return fail64(HASTAR_ENOSPC, "path longer than the caller's buffer (*len = poses needed)");
  }
  std::memcpy(xyh, h->last_xyh.data(), (size_t)L * 3 * sizeof(double));
  std::memcpy(curv, h->last_curv.data(), (size_t)L * sizeof(double));
  return HASTAR_OK;
}

int hastar64_copy_path(hastar64_handle h, double* xyh, double* curv, int cap, int* len) {
  if (!h || !len || cap < 0 || (cap > 0 && (!xyh || !curv))) return fail64(HASTAR_EINVAL, "bad argument");
  *len = h->last_len;
  if (h->last_len > cap) return fail64(HASTAR_ENOSPC, "path longer than the caller's buffer");
  std::memcpy(xyh, h->last_xyh.data(), (size_t)h->last_len * 3 * sizeof(double));
  std::memcpy(curv, h->last_curv.data(), (size_t)h->last_len * sizeof(double));
  return HASTAR_OK;
}

}  // extern "C"

namespace {
// velocity-profile staging of one device (hastar_velocity_profile_batch_f64)
struct VelStage64 {
  std::mutex mu;
  hipStream_t st = nullptr;
  char* base = nullptr;
  size_t cap = 0;
};
VelStage64& vel_stage64(int device) {
  static std::mutex mu;
  static std::map<int, std::unique_ptr<VelStage64>> all;
  std::lock_guard<std::mutex> lk(mu);
  std::unique_ptr<VelStage64>& p = all[device];
  if (!p) p.reset(new VelStage64());
  return *p;
}
}  // namespace

extern "C" {

// VelocityGenerator<double> (VelocityGenerator.cpp:7-84) over n paths, host buffers in and out
int hastar_velocity_profile_batch_f64(int device, const hastar_velocity_params_f64* vp, int n, const long long* offsets,
                                      const double* xyh, const double* curv, const double* vel_init,
                                      const double* vmax_curr, const unsigned char* flags, double* velocity,
                                      unsigned char* feasible) {
  if (!vp || n < 0 || (n > 0 && (!offsets || !vel_init || !vmax_curr || !flags || !feasible)))
    return fail64(HASTAR_EINVAL, "bad argument");
  if (n == 0) return HASTAR_OK;
  for (int i = 0; i < n; ++i)
    if (offsets[i + 1] <= offsets[i]) return fail64(HASTAR_EINVAL, "empty path (undefined in the reference)");
  const long long pts = offsets[n] - offsets[0];
  if (offsets[0] != 0 || !xyh || !curv || !velocity) return fail64(HASTAR_EINVAL, "bad path buffers");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail64(HASTAR_EDEVICE, "no HIP device available (this library has no CPU path)");
  if (device < 0 || device >= ndev) return fail64(HASTAR_EINVAL, "device ordinal out of range");
  HIPCHK64(hipSetDevice(device));
  const size_t b_off = al256((size_t)(n + 1) * 8), b_x = al256((size_t)pts * 3 * 8), b_c = al256((size_t)pts * 8),
               b_v = al256((size_t)n * 8), b_f = al256((size_t)n);
  const size_t total = b_off + b_x + 2 * b_c + 2 * b_v + 2 * b_f;
  // one staging slab and stream per device, grown and reused (LocalPlanner<double> profiles
  // one path per tick): no allocation or device-wide synchronisation per call
  VelStage64& S = vel_stage64(device);
  std::lock_guard<std::mutex> lk(S.mu);
  if (!S.st) HIPCHK64(hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking));
  if (total > S.cap) {
    HIPCHK64(hipStreamSynchronize(S.st));
    if (S.base) hipFree(S.base);
    S.base = nullptr;
    S.cap = 0;
    HIPCHK64(hipMalloc(reinterpret_cast<void**>(&S.base), total + total / 2));
    S.cap = total + total / 2;
  }
  char* q = S.base;
  long long* d_off = reinterpret_cast<long long*>(q); q += b_off;
  double* d_x = reinterpret_cast<double*>(q); q += b_x;
  double* d_c = reinterpret_cast<double*>(q); q += b_c;
  double* d_vel = reinterpret_cast<double*>(q); q += b_c;
  double* d_v0 = reinterpret_cast<double*>(q); q += b_v;
  double* d_vm = reinterpret_cast<double*>(q); q += b_v;
  unsigned char* d_fl = reinterpret_cast<unsigned char*>(q); q += b_f;
  unsigned char* d_feas = reinterpret_cast<unsigned char*>(q);
  hipStream_t st = S.st;
  HIPCHK64(hipMemcpyAsync(d_off, offsets, (size_t)(n + 1) * 8, hipMemcpyHostToDevice, st));
  HIPCHK64(hipMemcpyAsync(d_x, xyh, (size_t)pts * 3 * 8, hipMemcpyHostToDevice, st));
  HIPCHK64(hipMemcpyAsync(d_c, curv, (size_t)pts * 8, hipMemcpyHostToDevice, st));
  HIPCHK64(hipMemcpyAsync(d_v0, vel_init, (size_t)n * 8, hipMemcpyHostToDevice, st));
  HIPCHK64(hipMemcpyAsync(d_vm, vmax_curr, (size_t)n * 8, hipMemcpyHostToDevice, st));
  HIPCHK64(hipMemcpyAsync(d_fl, flags, (size_t)n, hipMemcpyHostToDevice, st));
  const VelParams64 P{vp->max_velocity, vp->coast_velocity, vp->max_lat_acc, vp->max_lat_acc * vp->max_lat_acc,
                      vp->max_long_acc, vp->max_long_dec};
  HIPCHK64(launch64_velocity(P, n, d_off, d_x, d_c, d_v0, d_vm, d_fl, d_vel, d_feas, st));
  HIPCHK64(hipMemcpyAsync(velocity, d_vel, (size_t)pts * 8, hipMemcpyDeviceToHost, st));
  HIPCHK64(hipMemcpyAsync(feasible, d_feas, (size_t)n, hipMemcpyDeviceToHost, st));
  HIPCHK64(hipStreamSynchronize(st));
  return HASTAR_OK;
}

// ---- test hooks ----
int hastar64_debug_memo(hastar64_handle h, double* f_out, unsigned char* visited_out) {
  if (!h || !f_out || !visited_out) return fail64(HASTAR_EINVAL, "bad argument");
  HIPCHK64(hipSetDevice(h->device));
  const size_t NN = (size_t)h->D.N * h->D.N;
  std::vector<uint32_t> bits(bitmap_words64(NN));
  HIPCHK64(hipMemcpyAsync(f_out, h->D.nm_f, NN * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK64(hipMemcpyAsync(bits.data(), h->D.visited, bits.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, h->st));
  HIPCHK64(hipStreamSynchronize(h->st));
  for (size_t c = 0; c < NN; ++c) visited_out[c] = (bits[c >> 5] >> (c & 31)) & 1u;
  return HASTAR_OK;
}

int hastar64_debug_closed_keys(hastar64_handle h, int* out, int cap) {
  if (!h || (cap > 0 && !out)) return fail64(HASTAR_EINVAL, "bad argument");
  HIPCHK64(hipSetDevice(h->device));
  Result64 R{};
  HIPCHK64(hipMemcpyAsync(&R, h->d_res, sizeof(R), hipMemcpyDeviceToHost, h->st));
  HIPCHK64(hipStreamSynchronize(h->st));
  const int n = (int)R.closed_size;
  std::vector<Closed3d> rec((size_t)n);
  if (n > 0) HIPCHK64(hipMemcpy(rec.data(), h->D.closed3, (size_t)n * sizeof(Closed3d), hipMemcpyDeviceToHost));
  std::vector<long long> k((size_t)n);
  for (int i = 0; i < n; ++i) {
    const uint32_t key = rec[i].key;
    k[i] = ((long long)(key >> 20) << 40) | ((long long)((key >> 8) & 0xfff) << 16) | (key & 0xff);
  }
  std::sort(k.begin(), k.end());
  for (int i = 0; i < n && i < cap; ++i) {
    out[3 * i] = (int)(k[i] >> 40);
    out[3 * i + 1] = (int)((k[i] >> 16) & 0xffffff);
    out[3 * i + 2] = (int)(k[i] & 0xffff);
  }
  return n;
}

int hastar64_debug_arena(hastar64_handle h, long long* out4) {
  if (!h || !out4) return fail64(HASTAR_EINVAL, "bad argument");
  out4[0] = h->D.open3_cap;
  out4[1] = h->D.open2_cap;
  out4[2] = h->D.dub_cap;
  out4[3] = h->reruns;
  return HASTAR_OK;
}

}  // extern "C"
