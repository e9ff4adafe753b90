// hastar_f64.hip — HybridAStar<double> and VelocityGenerator<double> on the GPU (gfx950).
//
// The reference instantiates its planner for double too (HybridAStar.cpp:285-286), and its
// ROS node's LocalPlanner<double> specialization constructs and calls it
// (local_planner.cpp:158-166, 378-500).  This file is that instantiation on the device:
//
//   k64_search        one wavefront per planner: HybridAStar::hybrid_a_star_search
//                     (HybridAStar.cpp:93-199) with the lazy holonomic A* (AStar.cpp:100-218)
//                     nested in it.  The open sets are the libstdc++ RB-tree replica of
//                     rbtree_dev.h over double f (its equal-f drops and shape-dependent finds
//                     are what the reference's non-strict comparator does, Node3D.h:50-54,
//                     Node2D.h:41-45); the closed sets are generation-stamped tables.  Lanes
//                     take the data-parallel parts: a successor each (VehicleModel.cpp:63-105,
//                     Grid3D.cpp:47-74, its APF sum in obstacle order, Grid3D.cpp:206-227, and
//                     its Dubins length, Dubins.cpp:19-69), a holonomic neighbour each
//                     (Grid2D.cpp:72-96), a shot sample each (Grid3D.cpp:78-93).
//   k64_reconstruct   HybridAStar::reconstruct_path (HybridAStar.cpp:208-262), a pose per lane.
//   map kernels       Grid2D / Grid3D map upkeep in double (Grid2D.cpp:99-208, 303-316,
//                     Grid3D.cpp:169-203).
//   k64_velocity      VelocityGenerator<double>::generate_velocity_profile
//                     (VelocityGenerator.cpp:19-84), one thread per path.
//
// Expressions keep the reference's double arithmetic (-ffp-contract=off).  sin, cos, atan2, acos
// and hypot are ports of glibc 2.35's routines (hastar_libm64.h), bit for bit the host libm's on
// every argument sampled in the planner's ranges (sin/cos: |x| < 2^27 * pi/2, beyond which
// glibc's __branred reduction is not ported; the planner's angles are wrapped to [-pi, pi]), so
// this planner reproduces the reference bit for bit (include/hastar_f64.h).
#include <hip/hip_runtime.h>
#include <cfloat>
#include "hastar_device.h"
#include "hastar_dubins_f64.h"
#include "hastar_f64_layout.h"
#include "hastar_f64_kernels.h"

namespace hastar {
namespace {

// ---- wave-uniform doubles and cross-lane reads ------------------------------------------
__device__ __forceinline__ double ufd(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double rld(double v, int l) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ int rli(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ double stl_maxd(double a, double b) { return (a < b) ? b : a; }
__device__ __forceinline__ double stl_mind(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ uint64_t dbits(double v) { return (uint64_t)__double_as_longlong(v); }

// common.h:31-36 with T = double
__device__ __forceinline__ int heading_bin_d(double h, double prec) {
  const double r = ::round(h / prec) * prec;
  return x86_trunc_int((r + M_PI) / prec);
}
// Grid2D::compute_heuristic (Grid2D.cpp:303-316), T = double
__device__ __forceinline__ double euclid_h64(const Planner64Dev& P, int i, int j) {
  const double dx = (P.n45 - i) * P.res;
  const double dx2 = dx * dx;
  const double dy = (P.n2 - j) * P.res;
  const double dy2 = dy * dy;
  return ::sqrt(dx2 + dy2);
}
__device__ __forceinline__ uint32_t slot_hash64(uint32_t k) {
  k ^= k >> 16;
  k *= 0x7feb352du;
  k ^= k >> 15;
  k *= 0x846ca68bu;
  k ^= k >> 16;
  return k;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o, 64);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

// ---- the open sets: rbtree_dev.h's libstdc++ replica over HBM records with double f --------
template <class NodeT>
struct Acc64 {
  static constexpr bool kPathWalk = false;
  using FT = double;
  GAS NodeT* t;
  __device__ __forceinline__ int L(int x) const { return ufi(t[x].l); }
  __device__ __forceinline__ int R(int x) const { return ufi(t[x].r); }
  __device__ __forceinline__ int P(int x) const { return ufi(t[x].p); }
  __device__ __forceinline__ int C(int x) const { return ufi(t[x].color); }
  __device__ __forceinline__ void sL(int x, int v) { t[x].l = v; }
  __device__ __forceinline__ void sR(int x, int v) { t[x].r = v; }
  __device__ __forceinline__ void sP(int x, int v) { t[x].p = v; }
  __device__ __forceinline__ void sC(int x, int v) { t[x].color = v; }
  __device__ __forceinline__ uint32_t K(int x) const { return ufu(t[x].key); }
  __device__ __forceinline__ double F(int x) const { return ufd(t[x].f); }
  __device__ __forceinline__ QuadT<double> quad_at(int x, int) const {
    QuadT<double> q;
    q.key = ufu(t[x].key);
    q.f = ufd(t[x].f);
    q.l = ufi(t[x].l);
    q.r = ufi(t[x].r);
    return q;
  }
  __device__ __forceinline__ void leaf(int x, int p) {
    t[x].p = p;
    t[x].l = NIL;
    t[x].r = NIL;
    t[x].color = RB_RED;
  }
};
using Tree3 = RBT<Acc64<Node3d>>;
using Tree2 = RBT<Acc64<Node2d>>;

struct Ctx64 {
  const Planner64Dev* P;
  int lane, N;
  double thr;
  GAS double* occ;
  GAS double* nm_f;
  GAS uint32_t* vis;
  GAS Cell2d* cell2;
  uint32_t gen3, gen2;
  long long succ, apops, asearch;
  int need;  // NEED_* bits: the search stopped for a larger arena
};

__device__ __forceinline__ bool inside(const Ctx64& c, int i, int j) { return i > -1 && i < c.N && j > -1 && j < c.N; }
__device__ __forceinline__ bool vis_get(const Ctx64& c, size_t cell) {
  return (ufu(c.vis[cell >> 5]) >> (cell & 31)) & 1u;
}
__device__ __forceinline__ void vis_set(Ctx64& c, size_t cell) {
  const uint32_t w = ufu(c.vis[cell >> 5]);
  c.vis[cell >> 5] = w | (1u << (cell & 31));
}

// AStar::update_visted + Grid2D::update_costs (AStar.cpp:209-218, Grid2D.cpp:219-227): the
// chain of closed records from `cell` back to the inner search's start
__device__ void memoise64(Ctx64& c, double total, int cell) {
  for (int p = cell; p != NIL; p = ufi(c.cell2[p].prev)) vis_set(c, (size_t)p);
  for (int p = cell; p != NIL; p = ufi(c.cell2[p].prev)) c.nm_f[p] = total - ufd(c.cell2[p].g);
}

__device__ __forceinline__ bool tree2_insert(Ctx64& c, Tree2& T, PoolState& ps, int cap, uint32_t key, double f,
                                             double g, int prev) {
  bool left = false;
  const int pos = T.insert_pos(key, f, &left);
  if (pos == -2) return true;  // an "equivalent" node is open: std::set::insert drops it
  const int x = tpool_alloc(T, ps, cap);
  if (x == NIL) {
    c.need |= NEED_INNER;
    return false;
  }
  GAS Node2d* n = &T.t[x];
  n->key = key;
  n->f = f;
  n->g = g;
  n->prev = prev;
  T.link(left, x, pos);
  return true;
}

// AStar::find_path(int, int) with get_cost_only (AStar.cpp:100-113) after a memo miss:
// a_star_search from the soft-reset start (AStar.cpp:118-186).  Returns the cost (DBL_MAX if
// the goal cell is unreachable); c.need != 0 means the search stopped for a larger arena.
__device__ double a_star64(Ctx64& c, const Planner64Dev& P, int si, int sj) {
  const int N = c.N, lane = c.lane;
  const size_t s0 = (size_t)si * N + sj;
  c.nm_f[s0] = euclid_h64(P, si, sj);  // Node2D::soft_reset (via Grid2D::set_start_node_grid)
  c.asearch++;
  c.gen2 = c.gen2 + 1;
  if (c.gen2 == 0) {  // the 32-bit generation wrapped: clear every cell's stamp
    for (size_t t = lane; t < (size_t)N * N; t += 64) c.cell2[t].gen = 0;
    wave_lds_sync();
    c.gen2 = 1;
  }
  Tree2 T;
  T.t = gp(P.open2);
  T.clear();
  PoolState ps{1, NIL};
  const int cap = P.open2_cap;
  if (!tree2_insert(c, T, ps, cap, ((uint32_t)si << 16) | (uint32_t)sj, ufd(c.nm_f[s0]), 0.0, NIL)) return DBL_MAX;
  const bool diag = P.diag != 0;
  const int nact = diag ? 8 : 4;
  // Grid2D's actions (Grid2D.cpp:32-51) and their costs (:54-58)
  int adx = 0, ady = 0;
  if (diag) {
    const int d8x[8] = {0, 1, 1, 1, 0, -1, -1, -1}, d8y[8] = {-1, -1, 0, 1, 1, 1, 0, -1};
    adx = d8x[lane & 7];
    ady = d8y[lane & 7];
  } else {
    const int d4x[4] = {0, 1, 0, -1}, d4y[4] = {-1, 0, 1, 0};
    adx = d4x[lane & 3];
    ady = d4y[lane & 3];
  }
  const double acost = (adx != 0 && ady != 0) ? P.act_cost_diag : P.act_cost_axis;
  while (!T.empty()) {
    const int x = T.begin();
    const uint32_t key = ufu(T.t[x].key);
    const double nf = ufd(T.t[x].f), ng = ufd(T.t[x].g);
    const int nprev = ufi(T.t[x].prev);
    const int ci = (int)(key >> 16), cj = (int)(key & 0xffffu);
    const int cell = ci * N + cj;
    // closed-set insert (AStar.cpp:127-129): an already closed cell returns its OLD record
    double cg = ng;
    if (ufu(c.cell2[cell].gen) != c.gen2) {
      Cell2d r;
      r.gen = c.gen2;
      r.prev = nprev;
      r.g = ng;
      gstore(&c.cell2[cell], r);
    } else {
      cg = ufd(c.cell2[cell].g);
    }
    T.unlink(x);
    tpool_free(T, ps, x);
    c.apops++;
    if (ci == P.n45 && cj == P.n2) {  // the goal cell (AStar::update_goal_node: the grid's goal)
      memoise64(c, nf, cell);         // first pop of the goal cell: the record is the popped node
      return nf;
    }
    // every neighbour's probes at once (lane k = action k): bounds, occupancy, memo flag,
    // node-map f, closed stamp.  A neighbour's own processing is the only writer of its f,
    // and only pops close cells, so the probes stay valid through the sequential loop below.
    const int ni = ci + adx, nj = cj + ady;
    bool ok = false, vis = false, closed = false;
    double pf = 0.0;
    if (lane < nact && inside(c, ni, nj)) {
      const size_t nc = (size_t)ni * N + nj;
      ok = c.occ[nc] < c.thr;
      if (ok) {
        vis = (c.vis[nc >> 5] >> (nc & 31)) & 1u;
        pf = c.nm_f[nc];
        closed = c.cell2[nc].gen == c.gen2;
      }
    }
    const uint64_t okm = __ballot(ok), vism = __ballot(vis), clm = __ballot(closed);
    for (int k = 0; k < nact; ++k) {
      if (!((okm >> k) & 1ull)) continue;
      const int ki = rli(ni, k), kj = rli(nj, k);
      const size_t nc = (size_t)ki * N + kj;
      const double kcost = rld(acost, k);
      if ((vism >> k) & 1ull) {  // memo hit (AStar.cpp:150-157)
        const double tot = rld(pf, k) + cg + kcost;
        memoise64(c, tot, cell);
        return tot;
      }
      if ((clm >> k) & 1ull) continue;
      const uint32_t kkey = ((uint32_t)ki << 16) | (uint32_t)kj;
      const int hit = T.find(kkey, rld(pf, k));
      const double gn = cg + kcost;
      if (hit == 0) {
        const double f = gn + euclid_h64(P, ki, kj);
        c.nm_f[nc] = f;
        if (!tree2_insert(c, T, ps, cap, kkey, f, gn, cell)) return DBL_MAX;
      } else if (gn < ufd(T.t[hit].g)) {
        T.unlink(hit);
        tpool_free(T, ps, hit);
        const double f = gn + euclid_h64(P, ki, kj);
        c.nm_f[nc] = f;
        if (!tree2_insert(c, T, ps, cap, kkey, f, gn, cell)) return DBL_MAX;
      }
    }
  }
  return DBL_MAX;
}

// AStar::find_path(int, int) (AStar.cpp:100-113): the memoised value, or a search
__device__ __forceinline__ double holonomic64(Ctx64& c, const Planner64Dev& P, int i, int j) {
  const size_t cell = (size_t)i * c.N + j;
  if (vis_get(c, cell)) return ufd(c.nm_f[cell]);
  return a_star64(c, P, i, j);
}

// Grid3D::get_field_intensity (Grid3D.cpp:206-227) of one pose, obstacles in order.  A term
// with distance >= radius (or NaN) is the reference's 0, and acc + 0.0 == acc (acc starts at
// +0.0), so such obstacles are skipped without their atan2.
__device__ double apf_field64(const Planner64Dev& P, const GAS double* apf, double px, double py, double ph) {
  double acc = 0.0;
  for (int k = 0; k < P.n_apf; ++k) {
    const double ox = apf[3 * k], oy = apf[3 * k + 1], orad = apf[3 * k + 2];
    const double d = gm64::hypot(ox - px, oy - py);
    if (d < orad) {
      double ang = ::fabs(wrap_pi_d(ph - gm64::atan2(oy - py, ox - px)));
      ang = stl_maxd(P.apf_ang - ang, 0.0);
      const double t = 1.0 / d - 1.0 / orad;
      double fp = P.apf_rep * (t * t);  // std::pow(t, 2)
      fp = fp * ang / P.apf_ang;
      acc = acc + fp;
    }
  }
  return acc;
}

__device__ __forceinline__ Closed3d node_to_closed(uint32_t key, int prev, int ci, double g, double vmin, double x,
                                                   double y, double h) {
  Closed3d r;
  r.key = key;
  r.prev = prev;
  r.ci = ci;
  r.pad = 0;
  r.g = g;
  r.vmin = vmin;
  r.x = x;
  r.y = y;
  r.h = h;
  r.pad2 = 0.0;
  return r;
}

}  // namespace

// HybridAStar<double>::find_path's search (HybridAStar.cpp:93-199): one wavefront, one planner
__global__ __launch_bounds__(64) void k64_search(const Planner64Dev* __restrict__ descs) {
  const Planner64Dev& P = descs[blockIdx.x];
  const int lane = threadIdx.x;
  Ctx64 c;
  c.P = &P;
  c.lane = lane;
  c.N = P.N;
  c.thr = P.thr;
  c.occ = gp(P.occ);
  c.nm_f = gp(P.nm_f);
  c.vis = gp(P.visited);
  c.cell2 = gp(P.cell2);
  c.succ = c.apops = c.asearch = 0;
  c.need = 0;
  GAS uint32_t* gens = gp(P.gens);
  GAS Slot3d* slots = gp(P.slots3);
  GAS Closed3d* closed = gp(P.closed3);
  const uint32_t smask = P.slots3_mask;
  c.gen3 = ufu(gens[0]) + 1;
  c.gen2 = ufu(gens[1]);
  if (c.gen3 == 0) {
    for (size_t t = lane; t <= (size_t)smask; t += 64) slots[t].gen = 0;
    wave_lds_sync();
    c.gen3 = 1;
  }
  const int N = c.N;
  // Grid3D::set_start_node (Grid3D.cpp:127-160): the start cell's node is soft-reset
  c.nm_f[(size_t)P.start_cx * N + P.start_cy] = euclid_h64(P, P.start_cx, P.start_cy);

  Tree3 T;
  T.t = gp(P.open3);
  T.clear();
  PoolState ps{1, NIL};
  const int cap3 = P.open3_cap;
  int n_closed = 0;
  long long pops = 0, shots = 0;
  uint64_t dig = 0x243f6a8885a308d3ull;
  int counter = 0, interval = P.shot_interval;
  bool shot_allowed = false;
  int ok = 0, via_shot = 0, terminal = NIL, dub_len = 0;
  double cost = DBL_MAX;
  {
    const int x = tpool_alloc(T, ps, cap3);  // the start node (HybridAStar.cpp:68-88): f = max
    GAS Node3d* n = &T.t[x];
    n->key = key3(P.start_cx, P.start_cy, P.start_bin);
    n->f = DBL_MAX;
    n->g = 0.0;
    n->vmin = P.start_vmin;
    n->x = P.start_x;
    n->y = P.start_y;
    n->h = P.start_h;
    n->ci = P.start_ci;
    n->prev = NIL;
    T.link(true, x, 0);
  }
  const int na = P.na, nsteer = P.nsteer;
  while (!T.empty()) {
    const int x = T.begin();
    const GAS Node3d* on = &T.t[x];
    const uint32_t key = ufu(on->key);
    // unordered_set::insert(*it).first (HybridAStar.cpp:110-111): the OLD record of a closed key
    uint32_t h = slot_hash64(key) & smask;
    int idx = -1;
    for (;;) {
      const uint32_t sg = ufu(slots[h].gen);
      if (sg != c.gen3) break;
      if (ufu(slots[h].key) == key) {
        idx = ufi(slots[h].idx);
        break;
      }
      h = (h + 1) & smask;
    }
    if (idx < 0) {
      if (n_closed >= P.closed3_cap) {
        c.need |= NEED_OUTER;
        break;
      }
      idx = n_closed++;
      gstore(&closed[idx], node_to_closed(key, ufi(on->prev), ufi(on->ci), ufd(on->g), ufd(on->vmin), ufd(on->x),
                                          ufd(on->y), ufd(on->h)));
      Slot3d sl;
      sl.key = key;
      sl.gen = c.gen3;
      sl.idx = idx;
      sl.pad = 0;
      gstore(&slots[h], sl);
    }
    T.unlink(x);
    tpool_free(T, ps, x);
    pops++;
    const GAS Closed3d* cur = &closed[idx];
    const double cg = ufd(cur->g), cvm = ufd(cur->vmin), cx = ufd(cur->x), cy = ufd(cur->y), ch = ufd(cur->h);
    const int cci = ufi(cur->ci);
    dig = mix64(dig ^ digest_key(key)) + dbits(cg);
    const int kx = key3_x(key), ky = key3_y(key);
    if (kx == P.goal_cx && ky == P.goal_cy) {  // HybridAStar.cpp:113-117
      terminal = idx;
      ok = 1;
      cost = cg;
      break;
    }
    if (shot_allowed) {  // HybridAStar.cpp:118-154
      if (++counter == interval) {
        shots++;
        int n = 0, flag = 0;
        double len = 0.0;
        if (lane == 0) {
          DubD D;
          D.r = P.r_min;
          D.step = P.step;
          D.ang_step = P.ang_step;
          len = dub_shortest_d(D, cx, cy, ch, P.goal_x, P.goal_y, P.goal_h);
          n = dub_sample_d(D, P.dub_xyh, P.dub_curv, P.dub_cap);
          flag = ::fabs(D.prm[1]) > M_PI_2;  // Dubins.cpp:149: first arc longer than 90 degrees
        }
        n = rli(n, 0);
        flag = rli(flag, 0);
        len = rld(len, 0);
        if (n < 0) {
          c.need |= NEED_SHOT;
          break;
        }
        wave_lds_sync();  // lane 0's samples, read by every lane below
        bool blocked = false;
        if (!flag) {  // Grid3D::check_path (Grid3D.cpp:78-93)
          const GAS double* sx = gp(P.dub_xyh);
          for (int i = lane; i < n; i += 64) {
            const int i1 = x86_trunc_int(::round(sx[3 * i] / P.res)), j1 = x86_trunc_int(::round(sx[3 * i + 1] / P.res));
            if (i1 < 0 || i1 >= N || j1 < 0 || j1 >= N || c.occ[(size_t)i1 * N + j1] >= c.thr) blocked = true;
          }
        }
        if (!flag && !__ballot(blocked)) {
          terminal = ufi(cur->prev);
          ok = 1;
          via_shot = 1;
          dub_len = n;
          cost = cg + len;
          break;
        }
        counter = 0;
        interval = interval - P.shot_decay > 50 ? interval - P.shot_decay : 50;
      }
    }
    // Grid3D::get_neighbors (Grid3D.cpp:47-74) over VehicleModel::get_neighbors
    // (VehicleModel.cpp:63-105): lane i takes action lo + i of the window
    const bool slow = cvm < 1.0;
    int lo = cci - na;
    lo = lo < 0 ? 0 : lo;
    int hi = lo + 2 * na + 1;
    hi = hi < nsteer ? hi : nsteer;
    const int cnt = hi - lo;
    const int cbin = key3_bin(key);
    bool sv = false;
    double sx = 0, sy = 0, sh = 0, sg = 0, svm = 0, sdub = 0;
    int sbin = 0, scx = 0, scy = 0;
    if (lane < cnt) {
      const int a = lo + lane;
      bool feasible = true;
      double vm = 0.0;
      if (!slow) {
        const double lat = cvm * P.curv_abs[a];
        if (lat > P.a_lat) feasible = false;
        const double al = ::sqrt(1.0 - ((lat * lat) / P.a_lat2));
        vm = cvm - 2 * al * P.ts;
      }
      if (feasible) {
        const GAS double* o = gp(P.off) + 2 * ((size_t)a * (P.bins + 1) + cbin);
        sx = cx + o[0];
        sy = cy + o[1];
        sh = wrap_pi_d(ch + P.dth[a]);
        sg = cg + P.act_cost[a];
        svm = vm;
        sbin = heading_bin_d(sh, P.prec);
        scx = x86_trunc_int(sx / P.res);
        scy = x86_trunc_int(sy / P.res);
        if (scx > -1 && scx < N && scy > -1 && scy < N && c.occ[(size_t)scx * N + scy] < c.thr) {
          sv = true;
          sg = sg + apf_field64(P, gp(P.apf), sx, sy, sh);  // _cost_g += field (f likewise: f == g here)
          DubD D;  // the successor's Dubins length (HybridAStar.cpp:170), used if it is inserted
          D.r = P.r_min;
          D.step = P.step;
          D.ang_step = P.ang_step;
          sdub = dub_shortest_d(D, sx, sy, sh, P.goal_x, P.goal_y, P.goal_h);
        }
      }
    }
    const uint64_t vm_mask = __ballot(sv);
    c.succ += __popcll(vm_mask);
    shot_allowed = slow;
    for (int i = 0; i < cnt; ++i) {  // HybridAStar.cpp:157-194, successors in action order
      if (!((vm_mask >> i) & 1ull)) continue;
      const int kcx = rli(scx, i), kcy = rli(scy, i), kbin = rli(sbin, i);
      const uint32_t skey = key3(kcx, kcy, kbin);
      // closed-set membership
      bool is_closed = false;
      for (uint32_t q = slot_hash64(skey) & smask;; q = (q + 1) & smask) {
        if (ufu(slots[q].gen) != c.gen3) break;
        if (ufu(slots[q].key) == skey) {
          is_closed = true;
          break;
        }
      }
      if (is_closed) continue;
      const double g = rld(sg, i);
      const int hit = T.find(skey, g);  // probe with f == g (HybridAStar.cpp:162)
      if (hit != 0) {
        if (!(g < ufd(T.t[hit].g))) continue;
        T.unlink(hit);
        tpool_free(T, ps, hit);
      }
      const double h1 = holonomic64(c, P, kcx, kcy);
      if (c.need) break;
      const double h2 = rld(sdub, i);
      const double f = g + stl_maxd(h1, h2);
      bool left = false;
      const int pos = T.insert_pos(skey, f, &left);
      if (pos == -2) continue;
      const int nx = tpool_alloc(T, ps, cap3);
      if (nx == NIL) {
        c.need |= NEED_OUTER;
        break;
      }
      GAS Node3d* n = &T.t[nx];
      n->key = skey;
      n->f = f;
      n->g = g;
      n->vmin = rld(svm, i);
      n->x = rld(sx, i);
      n->y = rld(sy, i);
      n->h = rld(sh, i);
      n->ci = lo + i;
      n->prev = idx;
      T.link(left, nx, pos);
    }
    if (c.need) break;
  }
  gens[0] = c.gen3;
  gens[1] = c.gen2;
  // statistics (hastar_stats) and the closed digest (sum over records, order-free)
  uint64_t cd = 0;
  for (int i = lane; i < n_closed; i += 64) cd += mix64(digest_key(closed[i].key));
  cd = wave_sum64(cd);
  int chain = 0;
  if (ok) {
    for (int p = terminal; p != NIL; p = ufi(closed[p].prev)) ++chain;
  }
  if (lane == 0) {
    Result64* R = P.result;
    R->pops = pops;
    R->successors = c.succ;
    R->astar_pops = c.apops;
    R->astar_searches = c.asearch;
    R->shots = shots;
    R->closed_size = n_closed;
    R->pop_digest = dig;
    R->closed_digest = cd;
    R->ok = c.need ? 0 : ok;
    R->via_shot = via_shot;
    R->need = c.need;
    R->cost = c.need ? DBL_MAX : cost;
    R->terminal = terminal;
    R->dubins_len = via_shot ? dub_len : 0;
    R->chain_len = chain;
    R->path_len = ok ? (via_shot ? dub_len : 0) + chain : 0;
  }
}

// HybridAStar::reconstruct_path (HybridAStar.cpp:208-262) into the planner's output buffers:
// the shot's samples last-to-first, then the closed chain terminal -> start, every pose
// rotated back into the world frame; curvature: 0, the shot's curvatures, the chain's
// |curvature| of its actions, minus the last entry (HybridAStar.cpp:78-84).
__global__ __launch_bounds__(64) void k64_reconstruct(const Planner64Dev* __restrict__ descs) {
  const Planner64Dev& P = descs[blockIdx.x];
  const Result64* R = P.result;
  const int lane = threadIdx.x;
  if (!R->ok) return;
  const int D = R->dubins_len, C = R->chain_len, L = D + C;
  if (L > P.out_cap) return;  // the host checked; kept for safety
  GAS int* chain = gp(P.chain);
  GAS const Closed3d* closed = gp(P.closed3);
  if (lane == 0) {
    int k = 0;
    for (int p = R->terminal; p != NIL && k < C; p = closed[p].prev) chain[k++] = p;
  }
  wave_lds_sync();
  const double gx = P.goal_x, gy = P.goal_y, rc = P.rot_c, rs = P.rot_s;
  GAS double* ox = gp(P.out_xyh);
  GAS double* oc = gp(P.out_curv);
  for (int t = lane; t < L; t += 64) {
    double x, y, h;
    if (t < D) {
      const int q = D - 1 - t;
      x = P.dub_xyh[3 * q];
      y = P.dub_xyh[3 * q + 1];
      h = P.dub_xyh[3 * q + 2];
    } else {
      const int r = chain[t - D];
      x = closed[r].x;
      y = closed[r].y;
      h = closed[r].h;
    }
    // Vector3D::get_rotated_vector(-grid_heading) of (pose - goal node) + goal location
    const double dx = x - gx, dy = y - gy;
    ox[3 * t] = (dx * rc + dy * rs) + P.world_goal_x;
    ox[3 * t + 1] = (-dx * rs + dy * rc) + P.world_goal_y;
    ox[3 * t + 2] = wrap_pi_d(h - P.neg_heading);
    double k;
    if (t == 0) k = 0.0;
    else if (t <= D) k = P.dub_curv[D - t];
    else k = P.curv_abs[closed[chain[t - D - 1]].ci];
    oc[t] = k;
  }
}

// ------------------------------------------------------------- map kernels (double) -----
// Grid2D ctor + compute_heuristic (Grid2D.cpp:7-62, 303-316): node-map f = h
__global__ __launch_bounds__(256) void k64_init_nodemap(const Planner64Dev* __restrict__ descs) {
  const Planner64Dev& P = descs[0];
  const int N = P.N;
  GAS double* f = gp(P.nm_f);
  for (int i = blockIdx.x; i < N; i += gridDim.x)
    for (int j = threadIdx.x; j < N; j += blockDim.x) f[(size_t)i * N + j] = euclid_h64(P, i, j);
}
// Grid2D::update_obstacles() (Grid2D.cpp:197-208)
__global__ __launch_bounds__(256) void k64_decay(double* __restrict__ occ, size_t NN, double fr, double mn, double mx) {
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < NN; t += (size_t)gridDim.x * blockDim.x)
    occ[t] = stl_maxd(stl_mind(occ[t] + fr, mx), mn);
}
// Grid3D::relocate_obstacles (Grid3D.cpp:169-203): the reference's row-major loop lets the
// last writer (largest source index) win; atomicMax claims make that order-free
__global__ __launch_bounds__(256) void k64_relocate_claim(int N, double c, double s, double ox, double oy,
                                                          int* __restrict__ winner) {
  const size_t NN = (size_t)N * N;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < NN; t += (size_t)gridDim.x * blockDim.x) {
    const double fi = (double)(int)(t / N), fj = (double)(int)(t % N);
    const double x = (fi * c + fj * s) + ox;
    const double y = (-fi * s + fj * c) + oy;
    const int a = x86_trunc_int(::round(x)), b = x86_trunc_int(::round(y));
    if (a > -1 && a < N && b > -1 && b < N) atomicMax(&winner[(size_t)a * N + b], (int)t);
  }
}
__global__ __launch_bounds__(256) void k64_relocate_gather(size_t NN, const double* __restrict__ src,
                                                           int* __restrict__ winner, double* __restrict__ dst) {
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < NN; t += (size_t)gridDim.x * blockDim.x) {
    const int w = winner[t];
    dst[t] = (w >= 0) ? src[w] : 0.0;
    winner[t] = -1;
  }
}
// Grid2D::update_obstacles(boxes) (Grid2D.cpp:99-139): boxes in the reference's order, one
// workgroup; within a box every sub-sample adds the same delta and clamps, so a cell's hits
// are counted and applied in a row.  rp: {start_i, start_j, 2 end_i, 2 end_j}; dl: delta.
__global__ __launch_bounds__(1024) void k64_raster_boxes(double* __restrict__ occ, int* __restrict__ cnt, int N,
                                                         const int* __restrict__ rp, const double* __restrict__ dl,
                                                         int nbox, double c, double s, double mn, double mx) {
  for (int k = 0; k < nbox; ++k) {
    const int si = rp[4 * k], sj = rp[4 * k + 1], ni = rp[4 * k + 2], nj = rp[4 * k + 3];
    const double d = dl[k];
    const long long total = (long long)ni * nj;
    for (int pass = 0; pass < 2; ++pass) {
      for (long long t = threadIdx.x; t < total; t += blockDim.x) {
        const int i = (int)(t / nj), j = (int)(t % nj);
        const double x0 = i * 0.5, y0 = j * 0.5;  // Vector2D<T> offset(i * 0.5, j * 0.5), rotated
        const double x = x0 * c + y0 * s;
        const double y = -x0 * s + y0 * c;
        const int ip = si + x86_trunc_int(::round(x)), jp = sj + x86_trunc_int(::round(y));
        if (ip > -1 && ip < N && jp > -1 && jp < N) {
          const size_t cell = (size_t)ip * N + jp;
          if (pass == 0) {
            atomicAdd(&cnt[cell], 1);
          } else {
            const int m = atomicExch(&cnt[cell], 0);
            if (m) {
              double v = occ[cell];
              for (int r = 0; r < m; ++r) v = stl_maxd(stl_mind(v + d, mx), mn);
              occ[cell] = v;
            }
          }
        }
      }
      __syncthreads();
    }
  }
}
// Grid2D::update_obstacles(lines) (Grid2D.cpp:142-194).  lp: per line {ax, ay, dx, dy, nx, ny,
// delta, n_len, n_wid}; seq_len / seq_wid: the reference's accumulated progress values
// (prog_length, prog_width), computed on the host.
__global__ __launch_bounds__(1024) void k64_raster_lines(double* __restrict__ occ, int* __restrict__ cnt, int N, int n45,
                                                         int n2, double res, const double* __restrict__ lp,
                                                         const double* __restrict__ seq_len,
                                                         const double* __restrict__ seq_wid, int seq_stride, int nline,
                                                         double mn, double mx) {
  for (int k = 0; k < nline; ++k) {
    const double* L = lp + 9 * k;
    const double ax = L[0], ay = L[1], dx = L[2], dy = L[3], nx = L[4], ny = L[5], d = L[6];
    const int nlen = (int)L[7], nwid = (int)L[8];
    const double* sl = seq_len + (size_t)k * seq_stride;
    const int total = nlen * nwid;
    for (int pass = 0; pass < 2; ++pass) {
      for (int t = threadIdx.x; t < total; t += blockDim.x) {
        const int a = t / nwid, b = t % nwid;
        const double pl = sl[a], pw = seq_wid[b];
        const double cx = ax + dx * pl, cy = ay + dy * pl;  // start_point + delta * prog_length
        const double p1x = cx + nx * pw, p1y = cy + ny * pw;
        const double p2x = cx - nx * pw, p2y = cy - ny * pw;
        const int i1 = x86_trunc_int(::round(p1x / res)) + n45, i2 = x86_trunc_int(::round(p2x / res)) + n45;
        const int j1 = x86_trunc_int(::round(p1y / res)) + n2, j2 = x86_trunc_int(::round(p2y / res)) + n2;
        for (int e = 0; e < 2; ++e) {
          const int ii = e ? i2 : i1, jj = e ? j2 : j1;
          if (ii > -1 && ii < N && jj > -1 && jj < N) {
            const size_t cell = (size_t)ii * N + jj;
            if (pass == 0) {
              atomicAdd(&cnt[cell], 1);
            } else {
              const int m = atomicExch(&cnt[cell], 0);
              if (m) {
                double v = occ[cell];
                for (int q = 0; q < m; ++q) v = stl_maxd(stl_mind(v + d, mx), mn);
                occ[cell] = v;
              }
            }
          }
        }
      }
      __syncthreads();
    }
  }
}

// --------------------------------------------- VelocityGenerator<double> (post-search) -----
// VelocityGenerator.cpp:19-84 with T = double, one thread per path (the passes are sequential
// along a path; paths are independent).
__global__ __launch_bounds__(64) void k64_velocity(VelParams64 vp, int n, const long long* __restrict__ off,
                                                   const double* __restrict__ xyh, const double* __restrict__ curv,
                                                   const double* __restrict__ vel_init,
                                                   const double* __restrict__ vmax_curr,
                                                   const unsigned char* __restrict__ flags, double* vel,
                                                   unsigned char* __restrict__ feasible) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const long long o = off[p];
  const long long S = off[p + 1] - o;
  if (S <= 0) {
    feasible[p] = 0;
    return;
  }
  const double* X = xyh + 3 * o;
  const double* K = curv + o;
  double* V = vel + o;  // velocity_sqr, then velocity, in place
  const unsigned char fl = flags[p];
  double vmax = (fl & 1u) ? vp.coast_velocity : vp.max_velocity;
  vmax = stl_mind(vmax, vmax_curr[p]);
  const double vmax2 = vmax * vmax;
  const double v0 = vel_init[p];
  auto step = [X](long long a, long long b) { return gm64::hypot(X[3 * a] - X[3 * b], X[3 * a + 1] - X[3 * b + 1]); };
  V[0] = v0 * v0;
  double mcur = V[0];
  for (long long i = 0; i < S - 1; ++i) {  // initial profile (VelocityGenerator.cpp:34-49)
    const long long pi = S - i - 1;
    const double st = step(pi - 1, pi);
    const double lat = V[i] * K[pi];
    const double rem = vp.max_long_dec * ::sqrt(1.0 - (lat * lat) / vp.max_lat_acc_sqr);
    mcur = stl_maxd(mcur - 2 * rem * st, vmax2);
    V[i + 1] = (K[pi - 1] != 0) ? stl_mind(vp.max_lat_acc / K[pi - 1], mcur) : mcur;
  }
  if (fl & 2u) V[S - 1] = 0;  // (51-52)
  for (long long i = 0; i < S - 1; ++i) {  // forward pass (54-64)
    const long long pi = S - i - 1;
    const double st = step(pi - 1, pi);
    const double lat = V[i] * K[pi];
    const double rem = vp.max_long_acc * ::sqrt(1.0 - (lat * lat) / vp.max_lat_acc_sqr);
    V[i + 1] = stl_mind(V[i] + 2 * rem * st, V[i + 1]);
  }
  // backward pass (66-77): velocity[i - 1] = sqrt(v²[i - 1]) overwrites v²[i - 1] after its
  // last read; v²[S - 1] is kept until the end (79-82)
  const double last = V[S - 1];
  double vs = last;  // v²[i]
  for (long long i = S - 1; i > 0; --i) {
    const long long pi = S - i - 1;
    const double st = step(pi + 1, pi);
    const double lat = vs * K[pi];
    const double rem = vp.max_long_dec * ::sqrt(1.0 - (lat * lat) / vp.max_lat_acc_sqr);
    const double nv = stl_mind(vs + 2 * rem * st, V[i - 1]);
    V[i - 1] = ::sqrt(nv);
    vs = nv;
  }
  V[S - 1] = ::sqrt(last);
  feasible[p] = (v0 < (V[0] + 0.25)) ? 1 : 0;
}

// ------------------------------------------------------------------ launchers -------------
hipError_t launch64_search(const Planner64Dev* d_desc, int n, hipStream_t st) {
  hipLaunchKernelGGL(k64_search, dim3(n), dim3(64), 0, st, d_desc);
  return hipGetLastError();
}
hipError_t launch64_reconstruct(const Planner64Dev* d_desc, int n, hipStream_t st) {
  hipLaunchKernelGGL(k64_reconstruct, dim3(n), dim3(64), 0, st, d_desc);
  return hipGetLastError();
}
hipError_t launch64_init_nodemap(const Planner64Dev* d_desc, int N, hipStream_t st) {
  hipLaunchKernelGGL(k64_init_nodemap, dim3(N < 4096 ? N : 4096), dim3(256), 0, st, d_desc);
  return hipGetLastError();
}
hipError_t launch64_decay(double* occ, size_t NN, double fr, double mn, double mx, hipStream_t st) {
  if (NN == 0) return hipSuccess;
  const size_t b = (NN + 255) / 256;
  hipLaunchKernelGGL(k64_decay, dim3((unsigned)(b < 4096 ? b : 4096)), dim3(256), 0, st, occ, NN, fr, mn, mx);
  return hipGetLastError();
}
hipError_t launch64_relocate(int N, double c, double s, double ox, double oy, const double* src, double* dst, int* winner,
                             hipStream_t st) {
  const size_t NN = (size_t)N * N, b = (NN + 255) / 256;
  const dim3 g((unsigned)(b < 4096 ? b : 4096));
  hipLaunchKernelGGL(k64_relocate_claim, g, dim3(256), 0, st, N, c, s, ox, oy, winner);
  hipLaunchKernelGGL(k64_relocate_gather, g, dim3(256), 0, st, NN, src, winner, dst);
  return hipGetLastError();
}
hipError_t launch64_raster_boxes(double* occ, int* cnt, int N, const int* rp, const double* dl, int nbox, double c,
                                 double s, double mn, double mx, hipStream_t st) {
  if (nbox <= 0) return hipSuccess;
  hipLaunchKernelGGL(k64_raster_boxes, dim3(1), dim3(1024), 0, st, occ, cnt, N, rp, dl, nbox, c, s, mn, mx);
  return hipGetLastError();
}
hipError_t launch64_raster_lines(double* occ, int* cnt, int N, int n45, int n2, double res, const double* lp,
                                 const double* seq_len, const double* seq_wid, int stride, int nline, double mn,
                                 double mx, hipStream_t st) {
  if (nline <= 0) return hipSuccess;
  hipLaunchKernelGGL(k64_raster_lines, dim3(1), dim3(1024), 0, st, occ, cnt, N, n45, n2, res, lp, seq_len, seq_wid,
                     stride, nline, mn, mx);
  return hipGetLastError();
}
hipError_t launch64_velocity(const VelParams64& vp, int n, const long long* off, const double* xyh, const double* curv,
                             const double* vel_init, const double* vmax_curr, const unsigned char* flags, double* vel,
                             unsigned char* feasible, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k64_velocity, dim3((n + 63) / 64), dim3(64), 0, st, vp, n, off, xyh, curv, vel_init, vmax_curr,
                     flags, vel, feasible);
  return hipGetLastError();
}

}  // namespace hastar
