// hastar_capi.cpp — host runtime behind include/hastar.h (the drop-in C ABI).
//
// Each hastar_handle owns one planner's device state (maps, memo, search arenas) and a
// HIP stream.  Per-call scalar preparation (rotations of the call's inputs into the
// goal-centred grid frame, per-box/per-line raster parameters, the start node) is done
// here with the same float arithmetic as the reference and the bit-faithful libm ports;
// every per-cell and per-expansion operation runs in the HIP kernels.  There is no CPU
// fallback: without a usable gfx950 device every call returns HASTAR_EDEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <mutex>
#include <vector>

#include "../../include/hastar.h"
#include "../../include/hastar_test.h"
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
float stl_max(float a, float b) { return (a < b) ? b : a; }

template <class T>
hipError_t dalloc(T** p, size_t n) {
  return hipMalloc(reinterpret_cast<void**>(p), std::max<size_t>(n, 1) * sizeof(T));
}

// Map-update scratch shared by every planner of a device (relocation target + claim
// table, raster hit counters): N*N floats/ints each, grown to the largest grid seen.
// Map updates of different handles on one device are serialised by its mutex.
struct DeviceScratch {
  std::mutex mu;
  size_t cap = 0;
  float* tmp = nullptr;
  int* winner = nullptr;  // kept at -1 between uses
  int* cnt = nullptr;     // kept at 0 between uses
};
DeviceScratch g_scratch[64];

int scratch_acquire(int dev, size_t NN, hipStream_t st, DeviceScratch** out) {
  DeviceScratch& S = g_scratch[dev & 63];
  if (S.cap < NN) {
    if (S.tmp) hipFree(S.tmp);
    if (S.winner) hipFree(S.winner);
    if (S.cnt) hipFree(S.cnt);
    S.tmp = nullptr;
    S.winner = S.cnt = nullptr;
    S.cap = 0;
    if (dalloc(&S.tmp, NN) != hipSuccess || dalloc(&S.winner, NN) != hipSuccess || dalloc(&S.cnt, NN) != hipSuccess)
      return fail(HASTAR_ENOMEM, "map scratch allocation failed");
    if (hipMemsetAsync(S.winner, 0xff, NN * sizeof(int), st) != hipSuccess ||
        hipMemsetAsync(S.cnt, 0, NN * sizeof(int), st) != hipSuccess)
      return fail(HASTAR_EDEVICE, "map scratch init failed");
    S.cap = NN;
  }
  *out = &S;
  return 0;
}

}  // namespace

struct hastar_handle_s {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  PlannerDev desc{};            // host copy of the descriptor
  PlannerDev* d_desc = nullptr; // device copy
  float lp_min = 0, lp_max = 0, lp_free = 0;
  int max_pops = 0;
  std::vector<float> curv_abs;
  // grid-frame state (Grid2D::_grid_heading/_goal_location, Grid3D::_goal_location3D)
  float grid_heading = 0, goal2x = 0, goal2y = 0, goal3x = 0, goal3y = 0, goal3h = 0;
  bool goal_set = false;
  // device buffers not referenced by the descriptor
  int apf_cap = 0;
  int* d_rp = nullptr;
  float* d_dl = nullptr;
  int rp_cap = 0;
  float* d_lp = nullptr;
  float* d_seq = nullptr;
  float* d_wid = nullptr;
  int lp_cap = 0, seq_cap = 0, wid_cap = 0;
  SearchResult last{};
  bool have_last = false;
  std::vector<void*> owned;
};

static void free_handle(hastar_handle h) {
  if (!h) return;
  if (h->device >= 0) hipSetDevice(h->device);
  for (void* p : h->owned) hipFree(p);
  if (h->d_rp) hipFree(h->d_rp);
  if (h->d_dl) hipFree(h->d_dl);
  if (h->d_lp) hipFree(h->d_lp);
  if (h->d_seq) hipFree(h->d_seq);
  if (h->d_wid) hipFree(h->d_wid);
  if (h->desc.apf) hipFree(h->desc.apf);
  if (h->ev0) hipEventDestroy(h->ev0);
  if (h->ev1) hipEventDestroy(h->ev1);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
}

template <class T>
static int own_alloc(hastar_handle h, T** p, size_t n) {
  hipError_t e = dalloc(p, n);
  if (e != hipSuccess) return fail(HASTAR_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  h->owned.push_back(*p);
  return 0;
}

static int push_desc(hastar_handle h) {
  HIPCHK(hipMemcpyAsync(h->d_desc, &h->desc, sizeof(PlannerDev), hipMemcpyHostToDevice, h->stream));
  return 0;
}

extern "C" {

const char* hastar_last_error(void) { return g_err.c_str(); }
float hastar_last_search_ms(void) { return g_last_ms; }
int hastar_grid_size(hastar_handle h) { return h ? h->desc.N : HASTAR_EINVAL; }

// HybridAStar::HybridAStar (HybridAStar.cpp:7-24) and the member constructors it runs:
// Grid2D (Grid2D.cpp:7-62), VehicleModel (VehicleModel.cpp:7-47), Dubins (Dubins.cpp:7-16).
int hastar_create_f32(const hastar_params* p, int device, hastar_handle* out) {
  if (!p || !out) return fail(HASTAR_EINVAL, "null argument");
  *out = nullptr;
  if (p->grid_size < 2 || p->grid_size > 4095) return fail(HASTAR_EINVAL, "grid_size must be in [2, 4095]");
  if (p->num_angle_bins < 1 || p->num_angle_bins > 254) return fail(HASTAR_EINVAL, "num_angle_bins must be in [1, 254]");
  if (p->num_steering < 1 || p->num_steering > 16 || !p->steering || !p->curvature_weights)
    return fail(HASTAR_EINVAL, "num_steering must be in [1, 16] with steering/curvature_weights arrays");
  if (p->num_actions < 0) return fail(HASTAR_EINVAL, "num_actions must be >= 0");
  if (!(p->grid_resolution > 0) || !(p->step_size > 0)) return fail(HASTAR_EINVAL, "resolution/step must be > 0");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(HASTAR_EDEVICE, "no HIP device available (this library has no CPU path)");
  if (device < 0 || device >= ndev) return fail(HASTAR_EINVAL, "device ordinal out of range");
  if (hipSetDevice(device) != hipSuccess) return fail(HASTAR_EDEVICE, "hipSetDevice failed");

  hastar_handle h = new hastar_handle_s();
  h->device = device;
  PlannerDev& D = h->desc;
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
  std::vector<float> beta(ns), curv(ns), dth(ns), cost(ns), off((size_t)ns * (bins + 1) * 2, 0.0f);
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
  // Dubins radius (HybridAStar.cpp:22-24, tan_max HybridAStar.h:20-25)
  const float tmax = std::tan(*std::max_element(p->steering, p->steering + ns));
  D.r_min = p->wheelbase / (g_cosf(g_atan2f(p->rear_to_cg * tmax, p->wheelbase)) * tmax);
  D.step = p->step_size;
  D.ang_step = p->step_size / D.r_min;

  // arena sizes
  h->max_pops = p->max_pops > 0 ? p->max_pops : 262144;
  const size_t NN = (size_t)N * N;
  const int open3_cap = 3 * h->max_pops + 64;
  uint32_t slots = 1;
  while (slots < 2u * (uint32_t)h->max_pops + 64) slots <<= 1;
  const int astar_cap = p->max_astar_nodes > 0 ? p->max_astar_nodes : (int)std::min<size_t>(NN + 16, 1u << 30);
  int dub_cap = p->max_dubins_samples;
  if (dub_cap <= 0) {
    const double span = 2.0 * N * D.res;
    dub_cap = (int)(span / D.step) + 2 * (int)(2 * M_PI / D.ang_step + 2) + 64;
  }
  D.open3_cap = open3_cap;
  D.closed3_cap = h->max_pops + 1;
  D.slots3_mask = slots - 1;
  D.open2_cap = astar_cap + 1;
  D.closed2_cap = (int)std::min<size_t>(NN, (size_t)astar_cap);
  D.dub_cap = dub_cap;
  D.out_cap = dub_cap + h->max_pops + 2;

  int rc = 0;
  hipError_t he = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  if (he == hipSuccess) he = hipEventCreate(&h->ev0);
  if (he == hipSuccess) he = hipEventCreate(&h->ev1);
  if (he != hipSuccess) {
    free_handle(h);
    return fail(HASTAR_EDEVICE, std::string("stream/event: ") + hipGetErrorString(he));
  }
#define OWN(ptr, n) do { if ((rc = own_alloc(h, &(ptr), (n))) != 0) { free_handle(h); return rc; } } while (0)
  OWN(D.occ, NN);
  OWN(D.nm_f, NN);
  OWN(D.visited, NN);
  OWN(D.off, off.size());
  OWN(D.dth, (size_t)ns);
  OWN(D.act_cost, (size_t)ns);
  OWN(D.curv_abs, (size_t)ns);
  OWN(D.open3, (size_t)open3_cap);
  OWN(D.closed3, (size_t)D.closed3_cap);
  OWN(D.slots3, (size_t)slots);
  OWN(D.open2, (size_t)D.open2_cap);
  OWN(D.closed2, (size_t)D.closed2_cap);
  OWN(D.cgen2, NN);
  OWN(D.cidx2, NN);
  OWN(D.gens, (size_t)4);
  OWN(D.dub_xyh, (size_t)dub_cap * 3);
  OWN(D.dub_curv, (size_t)dub_cap);
  OWN(D.out_xyh, (size_t)D.out_cap * 3);
  OWN(D.out_curv, (size_t)D.out_cap);
  OWN(D.out_chain, (size_t)D.out_cap);
  OWN(D.result, (size_t)1);
  OWN(h->d_desc, (size_t)1);
#undef OWN
  D.apf = nullptr;
  D.n_apf = 0;
  hipStream_t st = h->stream;
  he = hipMemsetAsync(D.occ, 0, NN * sizeof(float), st);
  if (he == hipSuccess) he = hipMemsetAsync(D.visited, 0, NN, st);
  if (he == hipSuccess) he = hipMemsetAsync(D.slots3, 0, (size_t)slots * sizeof(Slot3), st);
  if (he == hipSuccess) he = hipMemsetAsync(D.cgen2, 0, NN * sizeof(uint32_t), st);
  if (he == hipSuccess) he = hipMemsetAsync(D.gens, 0, 4 * sizeof(uint32_t), st);
  if (he == hipSuccess) he = hipMemcpyAsync(D.off, off.data(), off.size() * sizeof(float), hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = hipMemcpyAsync(D.dth, dth.data(), ns * sizeof(float), hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = hipMemcpyAsync(D.act_cost, cost.data(), ns * sizeof(float), hipMemcpyHostToDevice, st);
  if (he == hipSuccess)
    he = hipMemcpyAsync(D.curv_abs, h->curv_abs.data(), ns * sizeof(float), hipMemcpyHostToDevice, st);
  if (he == hipSuccess) he = launch_init_nodemap(D, st);
  if (he == hipSuccess) he = hipStreamSynchronize(st);
  if (he != hipSuccess) {
    free_handle(h);
    return fail(HASTAR_EDEVICE, std::string("init: ") + hipGetErrorString(he));
  }
  *out = h;
  return HASTAR_OK;
}

int hastar_destroy(hastar_handle h) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  free_handle(h);
  return HASTAR_OK;
}

// HybridAStar::update_goal -> Grid3D::update_goal_heading + relocate_obstacles
// (Grid3D.cpp:102-124, 169-203); AStar::update_goal_node takes the goal cell.
int hastar_update_goal(hastar_handle h, const float goal[3], const float start[3]) {
  if (!h || !goal || !start) return fail(HASTAR_EINVAL, "null argument");
  HIPCHK(hipSetDevice(h->device));
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
  {
    std::lock_guard<std::mutex> lk(g_scratch[h->device & 63].mu);
    DeviceScratch* S = nullptr;
    const size_t NN = (size_t)D.N * D.N;
    if (int rc = scratch_acquire(h->device, NN, h->stream, &S)) return rc;
    HIPCHK(launch_relocate(D.N, g_cosf(dh), g_sinf(dh), org.x, org.y, D.occ, S->tmp, S->winner, h->stream));
    HIPCHK(hipMemcpyAsync(D.occ, S->tmp, NN * sizeof(float), hipMemcpyDeviceToDevice, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
  }
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
  HIPCHK(hipStreamSynchronize(h->stream));
  return HASTAR_OK;
}

// HybridAStar::reset -> AStar::reset (AStar.cpp:56-60)
int hastar_reset(hastar_handle h) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipMemsetAsync(h->desc.visited, 0, (size_t)h->desc.N * h->desc.N, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return HASTAR_OK;
}

// Grid2D::update_obstacles() (Grid2D.cpp:197-208)
int hastar_decay(hastar_handle h) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(launch_decay(h->desc.occ, (size_t)h->desc.N * h->desc.N, h->lp_free, h->lp_min, h->lp_max, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return HASTAR_OK;
}

// Grid3D::update_obstacles(boxes) (Grid3D.cpp:22-44) + Grid2D boxes (Grid2D.cpp:99-139)
int hastar_update_boxes(hastar_handle h, const float* boxes, const float* conf, int n, float apf_added_radius) {
  if (!h || n < 0 || (n > 0 && (!boxes || !conf))) return fail(HASTAR_EINVAL, "bad argument");
  HIPCHK(hipSetDevice(h->device));
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
    rp[4 * k + 2] = 2 * gmath::x86_trunc_int(std::ceil(dx / D.res));
    rp[4 * k + 3] = 2 * gmath::x86_trunc_int(std::ceil(dy / D.res));
    if (rp[4 * k + 2] < 0) rp[4 * k + 2] = 0;
    if (rp[4 * k + 3] < 0) rp[4 * k + 3] = 0;
    const float lc = (float)std::log((double)conf[k] / (1.0 - (double)conf[k]));
    dl[k] = lc - h->lp_free;
  }
  if (n > h->apf_cap) {
    if (D.apf) hipFree(D.apf);
    D.apf = nullptr;
    h->apf_cap = 0;
    HIPCHK(dalloc(&D.apf, (size_t)n * 3));
    h->apf_cap = n;
  }
  if (n > h->rp_cap) {
    if (h->d_rp) hipFree(h->d_rp);
    if (h->d_dl) hipFree(h->d_dl);
    h->d_rp = nullptr;
    h->d_dl = nullptr;
    h->rp_cap = 0;
    HIPCHK(dalloc(&h->d_rp, (size_t)n * 4));
    HIPCHK(dalloc(&h->d_dl, (size_t)n));
    h->rp_cap = n;
  }
  D.n_apf = n;
  if (n > 0) {
    HIPCHK(hipMemcpyAsync(D.apf, apf.data(), (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->d_rp, rp.data(), (size_t)n * 4 * sizeof(int), hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->d_dl, dl.data(), (size_t)n * sizeof(float), hipMemcpyHostToDevice, h->stream));
    std::lock_guard<std::mutex> lk(g_scratch[h->device & 63].mu);
    DeviceScratch* S = nullptr;
    if (int rc = scratch_acquire(h->device, (size_t)D.N * D.N, h->stream, &S)) return rc;
    HIPCHK(launch_raster_boxes(D.occ, S->cnt, D.N, h->d_rp, h->d_dl, n, g_cosf(gh), g_sinf(gh), h->lp_min,
                               h->lp_max, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  HIPCHK(hipStreamSynchronize(h->stream));
  return HASTAR_OK;
}

// Grid2D::update_obstacles(lines) (Grid2D.cpp:142-194)
int hastar_update_lines(hastar_handle h, const float* lines, const float* conf, int n, float width) {
  if (!h || n < 0 || (n > 0 && (!lines || !conf))) return fail(HASTAR_EINVAL, "bad argument");
  HIPCHK(hipSetDevice(h->device));
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
  if (n > h->lp_cap) {
    if (h->d_lp) hipFree(h->d_lp);
    if (h->d_seq) hipFree(h->d_seq);
    h->d_lp = nullptr;
    h->d_seq = nullptr;
    h->lp_cap = 0;
    HIPCHK(dalloc(&h->d_lp, (size_t)n * 9));
    HIPCHK(dalloc(&h->d_seq, (size_t)n * stride));
    h->lp_cap = n;
  }
  if ((int)wid.size() > h->wid_cap) {
    if (h->d_wid) hipFree(h->d_wid);
    h->d_wid = nullptr;
    h->wid_cap = 0;
    HIPCHK(dalloc(&h->d_wid, wid.size()));
    h->wid_cap = (int)wid.size();
  }
  HIPCHK(hipMemcpyAsync(h->d_lp, lp.data(), lp.size() * sizeof(float), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->d_seq, seq.data(), seq.size() * sizeof(float), hipMemcpyHostToDevice, h->stream));
  if (!wid.empty())
    HIPCHK(hipMemcpyAsync(h->d_wid, wid.data(), wid.size() * sizeof(float), hipMemcpyHostToDevice, h->stream));
  if (!wid.empty()) {
    std::lock_guard<std::mutex> lk(g_scratch[h->device & 63].mu);
    DeviceScratch* S = nullptr;
    if (int rc = scratch_acquire(h->device, (size_t)D.N * D.N, h->stream, &S)) return rc;
    HIPCHK(launch_raster_lines(D.occ, S->cnt, D.N, D.n45, D.n2, D.res, h->d_lp, h->d_seq, h->d_wid, stride, n,
                               h->lp_min, h->lp_max, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  HIPCHK(hipStreamSynchronize(h->stream));
  return HASTAR_OK;
}

int hastar_get_obstacles(hastar_handle h, float* out) {
  if (!h || !out) return fail(HASTAR_EINVAL, "null argument");
  HIPCHK(hipSetDevice(h->device));
  const size_t NN = (size_t)h->desc.N * h->desc.N;
  HIPCHK(hipMemcpyAsync(out, h->desc.occ, NN * sizeof(float), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return HASTAR_OK;
}

}  // extern "C"

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

extern "C" {

int hastar_find_path(hastar_handle h, float vel, const float start[3], float* xyh, float* curv, int cap, int* len,
                     float* cost, int* ok, hastar_stats* stats) {
  return hastar_find_path_batch(&h, 1, &vel, start, xyh, curv, cap, len, cost, ok, stats);
}

int hastar_find_path_batch(const hastar_handle* hs, int n, const float* vel, const float* starts, float* xyh,
                           float* curv, int cap, int* len, float* cost, int* ok, hastar_stats* stats) {
  if (!hs || n <= 0 || !vel || !starts || !len || !cost || !ok || cap < 0 || (cap > 0 && (!xyh || !curv)))
    return fail(HASTAR_EINVAL, "bad argument");
  const int dev = hs[0] ? hs[0]->device : -1;
  int max_pops = 0;
  for (int i = 0; i < n; ++i) {
    if (!hs[i] || hs[i]->device != dev) return fail(HASTAR_EINVAL, "null handle or handles on different devices");
    if (!hs[i]->goal_set) return fail(HASTAR_EINVAL, "update_goal must be called before find_path");
    max_pops = std::max(max_pops, hs[i]->max_pops);
  }
  HIPCHK(hipSetDevice(dev));
  hastar_handle h0 = hs[0];
  hipStream_t st = h0->stream;
  // descriptors of all planners, contiguous on the device
  static thread_local PlannerDev* d_batch = nullptr;
  static thread_local int d_batch_cap = 0;
  static thread_local int d_batch_dev = -1;
  std::vector<PlannerDev> descs(n);
  for (int i = 0; i < n; ++i) {
    prepare_start(hs[i], vel[i], starts + 3 * i);
    descs[i] = hs[i]->desc;
  }
  if (n > d_batch_cap || d_batch_dev != dev) {
    if (d_batch) hipFree(d_batch);
    d_batch = nullptr;
    d_batch_cap = 0;
    HIPCHK(dalloc(&d_batch, (size_t)n));
    d_batch_cap = n;
    d_batch_dev = dev;
  }
  HIPCHK(hipMemcpyAsync(d_batch, descs.data(), (size_t)n * sizeof(PlannerDev), hipMemcpyHostToDevice, st));
  HIPCHK(hipEventRecord(h0->ev0, st));
  HIPCHK(launch_search(d_batch, n, max_pops, st));
  HIPCHK(hipEventRecord(h0->ev1, st));
  std::vector<SearchResult> res(n);
  for (int i = 0; i < n; ++i)
    HIPCHK(hipMemcpyAsync(&res[i], hs[i]->desc.result, sizeof(SearchResult), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  float ms = 0.0f;
  hipEventElapsedTime(&ms, h0->ev0, h0->ev1);
  g_last_ms = ms;
  int rc = HASTAR_OK;
  for (int i = 0; i < n; ++i) {
    hs[i]->last = res[i];
    hs[i]->have_last = true;
    ok[i] = res[i].ok;
    cost[i] = res[i].ok ? res[i].cost : FLT_MAX;
    fill_stats(res[i], stats ? &stats[i] : nullptr);
    if (res[i].status != 0 && rc == HASTAR_OK) {
      rc = res[i].status == -75 ? HASTAR_EOVERFLOW : HASTAR_EDEVICE;
      g_err = "search arena overflow (raise max_pops / max_astar_nodes)";
    }
    int r = copy_path_out(hs[i], xyh ? xyh + (size_t)i * cap * 3 : nullptr, curv ? curv + (size_t)i * cap : nullptr,
                          cap, &len[i], st);
    if (r != 0 && rc == HASTAR_OK) rc = r;
  }
  HIPCHK(hipStreamSynchronize(st));
  return rc;
}

int hastar_copy_path(hastar_handle h, float* xyh, float* curv, int cap, int* len) {
  if (!h || !h->have_last) return fail(HASTAR_EINVAL, "no search result");
  HIPCHK(hipSetDevice(h->device));
  int r = copy_path_out(h, xyh, curv, cap, len, h->stream);
  HIPCHK(hipStreamSynchronize(h->stream));
  return r;
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

int hastar_test_dubins_path(hastar_handle h, const float start[3], float* xyh, float* curv, int cap, int* n,
                            float* length, int* first_arc_gt_90) {
  if (!h || !h->goal_set) return fail(HASTAR_EINVAL, "bad handle / no goal");
  HIPCHK(hipSetDevice(h->device));
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
  const size_t NN = (size_t)h->desc.N * h->desc.N;
  HIPCHK(hipMemcpy(f_out, h->desc.nm_f, NN * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(visited_out, h->desc.visited, NN, hipMemcpyDeviceToHost));
  return HASTAR_OK;
}

int hastar_debug_apf(hastar_handle h, float* out, int cap) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  const int n = h->desc.n_apf;
  if (n > cap) return n;
  HIPCHK(hipSetDevice(h->device));
  if (n) HIPCHK(hipMemcpy(out, h->desc.apf, (size_t)n * 3 * sizeof(float), hipMemcpyDeviceToHost));
  return n;
}

int hastar_debug_motion(hastar_handle h, float* off, float* dth, float* cost, float* curv_abs, float* prec,
                        float* r_min) {
  if (!h) return fail(HASTAR_EINVAL, "null handle");
  HIPCHK(hipSetDevice(h->device));
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
  for (int q = 0; q < 8; ++q) out8[q] = h->last.cycles[q];
  return HASTAR_OK;
}

int hastar_debug_astar_modes(hastar_handle h, long long* out2) {
  if (!h || !h->have_last) return fail(HASTAR_EINVAL, "no search result");
  out2[0] = h->last.astar_migrations;
  out2[1] = h->last.astar_pops_hbm;
  return HASTAR_OK;
}

int hastar_debug_closed_keys(hastar_handle h, int* out, int cap) {
  if (!h || !h->have_last) return fail(HASTAR_EINVAL, "no search result");
  HIPCHK(hipSetDevice(h->device));
  const int n = (int)h->last.closed_size;
  std::vector<Closed3> rec(n);
  if (n) HIPCHK(hipMemcpy(rec.data(), h->desc.closed3, (size_t)n * sizeof(Closed3), hipMemcpyDeviceToHost));
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
