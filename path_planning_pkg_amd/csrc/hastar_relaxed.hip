// hastar_relaxed.hip — the RELAXED search mode: a frontier-parallel
// Hybrid A* with a backward-Dijkstra heuristic, for one planner per workgroup.
//
// NOT bit-exact with the reference, on purpose.  The exact mode (hastar_search_kernel) keeps
// the reference's sequential pop order (HybridAStar.cpp:107-194) and its lazy per-cell A*
// heuristic (AStar.cpp:118-186), which leaves one wavefront per query.  This mode trades that
// order for parallelism inside one query:
//   1. heuristic: the 8-connected (4 when diag is off) grid distance to the goal cell over the
//      traversable cells, i.e. the converged value of the reference's lazy A* for every cell
//      at once (Grid2D.cpp:219-316 move costs act_cost_axis / act_cost_diag), computed by a
//      Dial-bucket Dijkstra: buckets of width act_cost_axis (the smallest move), so every move
//      leaves its bucket and a whole bucket is settled in parallel by the workgroup;
//   2. search: Δ-stepping over f.  Each round expands EVERY open node with f <= min f + delta,
//      one wavefront per node (the same fused successor / APF / Dubins-length code as the
//      exact kernel: VehicleModel.cpp:63-105, Grid3D.cpp:47-74, 206-227, Dubins.cpp:19-69);
//      duplicates are resolved by a best-g table per node key (atomicMin), not a closed set;
//   3. termination as in the reference: the goal cell is reached (Node3D::operator==,
//      Node3D.h:42) or an analytic Dubins shot is collision-free (HybridAStar.cpp:115-154,
//      the same interval / decay schedule counted over the workgroup's expansions); the
//      cheapest candidate of the round in which the first one appears wins;
//   4. reconstruction and output format as the exact mode (HybridAStar.cpp:208-262).
// Costs keep the reference's definitions (g = action costs + APF field, f = g + max(h, Dubins
// length)), so results are comparable: tests check validity (collision-free, continuous, ends at
// start and goal) and report the cost ratio against the exact mode, not bit parity.
#include <hip/hip_runtime.h>

#include "hastar_device.h"
#include "hastar_kernels.h"
#include "hastar_rs.h"

namespace hastar {

constexpr int RW = 8;                        // wavefronts per planner workgroup
constexpr int DU = 4;                        // Dijkstra bucket entries per thread in flight
constexpr int BL = 1536;                     // Dijkstra bucket entries per ring slot held in LDS
// The bucket ring lives in dynamic LDS (8 x BL entries, 96 KiB: one 8-wave workgroup per CU
// leaves the LDS to it); entries past BL of a slot spill to the arena's HBM lists.
constexpr size_t RELAX_DYN_LDS = (size_t)8 * BL * sizeof(BucketEntry);
__device__ __forceinline__ BucketEntry bucket_get(const RelaxArena& A, const BucketEntry* lds, int slot, int e) {
  return e < BL ? lds[slot * BL + e] : A.bucket[(size_t)slot * A.bcap + (e - BL)];
}
__device__ __forceinline__ bool bucket_put(const RelaxArena& A, BucketEntry* lds, int slot, int e, BucketEntry v) {
  if (e < BL) {
    lds[slot * BL + e] = v;
    return true;
  }
  if (e - BL >= A.bcap) return false;
  A.bucket[(size_t)slot * A.bcap + (e - BL)] = v;
  return true;
}

// diagnostic build (-DRELAX_STAMPS): per-phase cycles of the Dijkstra's bucket loop, thread 0
#ifdef RELAX_STAMPS
#define RSTAMP_BEGIN() unsigned long long rt0 = (__builtin_amdgcn_s_waitcnt(0), __builtin_amdgcn_s_memtime())
#define RSTAMP(k)                                                              \
  do {                                                                         \
    __builtin_amdgcn_s_waitcnt(0);                                             \
    const unsigned long long rt1 = __builtin_amdgcn_s_memtime();               \
    rst[k] += rt1 - rt0;                                                       \
    rt0 = rt1;                                                                 \
  } while (0)
#else
#define RSTAMP_BEGIN() (void)0
#define RSTAMP(k) (void)0
#endif
constexpr float SHOT_ADVANCE = 0.8f;  // an extra shot once the frontier's best f - g falls to 0.8x the last shooter's
constexpr unsigned long long RELAX_WATCHDOG = 1000000000ull;  // 10 s of s_memrealtime (100 MHz)
constexpr uint32_t EMPTY_KEY = 0xffffffffu;  // no node key has all bits set (x < 4096, bin < 256 with y < 4096)

// debug progress words (RelaxParams::progress): workgroup b, wave w -> words [(b * RW + w) * 4, +4)
#define RPROG(k, v)                                                                                   \
  do {                                                                                                \
    if (rp.progress && lane == 0)                                                                     \
      __hip_atomic_store(rp.progress + ((size_t)blockIdx.x * RW + wv) * 4 + (k), (unsigned)(v),         \
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);                                  \
  } while (0)

// L1-bypassing loads of words other waves update with atomics
__device__ __forceinline__ uint32_t ld_sync(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_dist(const float* d, size_t c) {
  return __uint_as_float(ld_sync(reinterpret_cast<const uint32_t*>(d) + c));
}
__device__ __forceinline__ void block_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ uint32_t rx_hash(uint32_t k) {
  k ^= k >> 16;
  k *= 0x7feb352dU;
  k ^= k >> 15;
  k *= 0x846ca68bU;
  return k ^ (k >> 16);
}
// best-g table: lower the key's best to v = g bits << 32 | tie; true when v is the new best
// (*slot: the key's slot, kept in the node so the search can clear exactly the slots it used).
// *full is set when the table has no room left.
__device__ __forceinline__ bool table_lower(const RelaxArena& A, uint32_t key, unsigned long long v, bool* full,
                                            uint32_t* slot) {
  uint32_t h = rx_hash(key) & A.tmask;
  for (uint32_t probe = 0; probe <= A.tmask; ++probe) {
    RelaxSlot* s = &A.table[h];
    uint32_t k = ld_sync(&s->key);
    if (k == EMPTY_KEY) {
      const uint32_t prev = atomicCAS(&s->key, EMPTY_KEY, key);
      k = prev == EMPTY_KEY ? key : prev;
    }
    *slot = h;
    if (k == key) return atomicMin(&s->best, v) > v;
    h = (h + 1) & A.tmask;
  }
  *full = true;
  return false;
}
// A node is current iff it still holds its key's best {g, tie}.  Only asked between rounds,
// when the table is final for the round, so the answer does not depend on wavefront timing.
__device__ __forceinline__ bool node_current(const RelaxArena& A, int idx, float* vmin = nullptr,
                                             float* g = nullptr, uint32_t* tie = nullptr) {
  const int4 q0 = *reinterpret_cast<const int4*>(&A.nodes[idx]);      // key, f, l, r
  const float4 q1 = *(reinterpret_cast<const float4*>(&A.nodes[idx]) + 1);  // p, cc, g, vmin
  if (vmin) *vmin = q1.w;
  if (g) *g = q1.z;
  if (tie) *tie = (uint32_t)q0.w;
  const unsigned long long mine = ((unsigned long long)__float_as_uint(q1.z) << 32) | (uint32_t)q0.w;
  return __hip_atomic_load(&A.table[(uint32_t)q0.z].best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == mine;
}
// a shooter's rank among the round's allowed nodes: the nearest to the goal by the heuristic
// part of f (f - g), then the tie.  The round's nodes share f to within delta, so this picks
// the frontier's most advanced nodes, whose shots are the likeliest to be free.
__device__ __forceinline__ unsigned long long shot_key(float f, float g, uint32_t tie) {
  return ((unsigned long long)__float_as_uint(fmaxf(f - g, 0.0f)) << 32) | tie;
}
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long w = ((unsigned long long)(uint32_t)__shfl_xor((int)(v >> 32), o, 64) << 32) |
                                 (uint32_t)__shfl_xor((int)(uint32_t)v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

struct RelaxShared {
  ApfStage apf[RW];
  int planner;
  int cnt[8];               // Dijkstra bucket fill counts (ring of 8)
  int overflow, hover;
  int settled;              // cells settled (diagnostic: astar_pops)
  int buckets;              // Dijkstra buckets processed
  int nA, nB, nE, nN, eNext, nodes, nE_last, n_allowed;
  uint32_t fmin, fnext;     // float bits of the open list's min f, and of the next open list's
  unsigned long long best;  // cheapest solution candidate: cost bits << 32 | tag
  int since_shot, interval;
  int pops, succ, shots, rounds;
  int n_sel;                     // shots of this round
  float last_shot_h;             // f - g of the last shooter
  unsigned long long sel[RW];    // their shooters' shot_key, lowest first
  int shot_term[RW], shot_n[RW];
  unsigned long long stamp[6];
};

// Phase 1: Dial-bucket Dijkstra from the goal cell into `dist`, restricted to the ellipse
// d(c) + |c - start| <= bound (bound = h_stop x |goal - start| + 64 moves); returns the
// bound.  A cell left unsettled gets the lower bound bound - |c - start| (relaxed_h).
// Bucket entries are {cell, distance bits}: an entry is live iff the cell's distance is still
// the one it was pushed with (a cell improves only by a strictly smaller push), so no settled
// flags are needed.  Moves cost >= wb, so iteration `cur` pushes only into buckets cur+1 ..
// cur+3 of a ring of 8: one barrier per bucket suffices — a bucket's count is final when its
// iteration starts, and slot (cur-1) & 7 is recycled (reset) long before it is pushed again.
// The run ends after 3 empty buckets in a row (nothing can be pushed past them) or at the
// early stop; both decisions use values every thread reads identically.
// The field is over blocks of K x K map cells (K = rp.h_coarse: 1, 2 or 4): a block is
// passable when any of its cells is (so no passage of the map closes), its moves cost K x the
// cell moves, and a cell's heuristic is its block's distance (relaxed_h).  K = 2 settles a
// quarter of the cells in half the buckets: the bucket loop's dependent round trips, and in a
// batch the field's scattered traffic, fall with it.
__device__ float relaxed_heuristic(const PlannerDev& P, const RelaxArena& A, RelaxShared& S, const RelaxParams& rp,
                                   float* dist_f, BucketEntry* bl) {
  const int tid = threadIdx.x, NT = blockDim.x;
  const int K = rp.h_coarse;
  const int N = (P.N + K - 1) / K;  // blocks per side
  const float wb = P.act_cost_axis * (float)K;
  const float cd = P.act_cost_diag * (float)K;
  const int nact = P.diag ? 8 : 4;
  uint32_t* dist = reinterpret_cast<uint32_t*>(dist_f);
  const size_t NN = (size_t)N * N;
  for (size_t i = tid; i < NN; i += NT) dist[i] = 0x7f800000u;
  // entries name blocks as (i << 16 | j): no integer division per entry
  const int gbx = P.goal_cx / K, gby = P.goal_cy / K, sbx = P.start_cx / K, sby = P.start_cy / K;
  const uint32_t goal_ij = ((uint32_t)gbx << 16) | (uint32_t)gby;
  const float inv_wb = 1.0f / wb;  // bucket index only: rounding is absorbed by the clamp below
  const float bres = P.res * (float)K;
  // relax only inside the ellipse d(c) + |c - start| <= bound around the goal-start segment
  const float gsx = (float)(P.goal_cx - P.start_cx), gsy = (float)(P.goal_cy - P.start_cy);
  const float bound = rp.h_stop * P.res * sqrtf(gsx * gsx + gsy * gsy) + 64.0f * P.act_cost_axis;
  block_sync();
  if (tid == 0) {
    dist[(size_t)gbx * N + gby] = 0u;
    bl[0] = BucketEntry{goal_ij, 0u};
    for (int k = 0; k < 8; ++k) S.cnt[k] = k == 0 ? 1 : 0;
    S.overflow = 0;
    S.settled = 0;
  }
  block_sync();
  const int max_b = 4 * N + 64;
  int cur = 0, empty_run = 0;
  const int cap = BL + A.bcap;
#ifdef RELAX_STAMPS
  unsigned long long rst[6] = {0, 0, 0, 0, 0, 0};
#endif
  for (; cur < max_b; ++cur) {
    const int slot = cur & 7;
    const int m = min(S.cnt[slot], cap);
    if (tid == 0) S.cnt[(cur - 1) & 7] = 0;  // recycled: pushed again no earlier than iteration cur + 4
    empty_run = m == 0 ? empty_run + 1 : 0;
    if (empty_run >= 3) break;
    // DU entries per thread at a time, phase by phase (entries, then distances and occupancy,
    // then every relaxation's atomicMin, then the pushes), so the dependent global round trips
    // of DU entries overlap instead of queueing one entry after the other
    int settled = 0;
    RSTAMP_BEGIN();
    for (int e0 = tid; e0 < m; e0 += NT * DU) {
      BucketEntry en[DU];
      uint32_t dc[DU];
      float oc[DU];
#pragma unroll
      for (int u = 0; u < DU; ++u) {
        const int e = e0 + u * NT;
        en[u] = e < m ? bucket_get(A, bl, slot, e) : BucketEntry{0xffffffffu, 0u};
      }
      RSTAMP(0);
#pragma unroll
      for (int u = 0; u < DU; ++u) {
        dc[u] = 0u;
        oc[u] = 0.0f;
        if (en[u].cell != 0xffffffffu) {
          const uint32_t bi = en[u].cell >> 16, bj = en[u].cell & 0xffffu;
          dc[u] = ld_sync(&dist[bi * (uint32_t)N + bj]);
          // the block's least occupancy (passable when any of its cells is)
          float o = FLT_MAX;
          for (int di = 0; di < K; ++di)
            for (int dj = 0; dj < K; ++dj) {
              const uint32_t ci = bi * K + di, cj = bj * K + dj;
              if (ci < (uint32_t)P.N && cj < (uint32_t)P.N) o = fminf(o, gp(P.occ)[ci * (uint32_t)P.N + cj]);
            }
          oc[u] = o;
        }
      }
      RSTAMP(1);
      uint32_t old[DU][8];
      uint32_t nbv[DU][8];
#pragma unroll
      for (int u = 0; u < DU; ++u) {
        const uint32_t cij = en[u].cell;
        // live: still the cell's distance (else a shorter push settles it); expanding: enterable
        const bool live = cij != 0xffffffffu && dc[u] == en[u].d;
        if (live) ++settled;
        const bool expand = live && (cij == goal_ij || oc[u] < P.thr);
        const float d = __uint_as_float(dc[u]);
        const int ci = (int)(cij >> 16), cj = (int)(cij & 0xffffu);
        // the neighbours' current distances first (all in flight together):
        // most are already at or below the offer, and only the others take an atomic — the
        // atomics of one wavefront front hit few cache lines and serialise in L2
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          // the 8 moves (Grid2D.cpp:22-40), axis moves first
          const int di = a < 4 ? ((a & 1) ? 0 : (a == 0 ? 1 : -1)) : ((a & 1) ? 1 : -1);
          const int dj = a < 4 ? ((a & 1) ? (a == 1 ? 1 : -1) : 0) : ((a & 2) ? 1 : -1);
          const int pi = ci + di, pj = cj + dj;
          const bool ok = expand && a < nact && pi >= 0 && pi < N && pj >= 0 && pj < N;
          const uint32_t nb = __float_as_uint(d + (a < 4 ? wb : cd));
          nbv[u][a] = nb;
          // a plain (possibly L1-stale) load: distances only fall, so a stale value only
          // costs an extra atomic, never a missed relaxation
          old[u][a] = ok ? gp(dist)[(uint32_t)pi * (uint32_t)N + (uint32_t)pj] : nb;
        }
      }
      RSTAMP(2);
#pragma unroll
      for (int u = 0; u < DU; ++u) {
        const uint32_t cij = en[u].cell;
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          if (old[u][a] <= nbv[u][a]) continue;
          const int di = a < 4 ? ((a & 1) ? 0 : (a == 0 ? 1 : -1)) : ((a & 1) ? 1 : -1);
          const int dj = a < 4 ? ((a & 1) ? (a == 1 ? 1 : -1) : 0) : ((a & 2) ? 1 : -1);
          const uint32_t pidx = (uint32_t)((int)(cij >> 16) + di) * (uint32_t)N + (uint32_t)((int)(cij & 0xffffu) + dj);
          old[u][a] = atomicMin(&dist[pidx], nbv[u][a]);
        }
      }
      RSTAMP(3);
#pragma unroll
      for (int u = 0; u < DU; ++u) {
        const uint32_t cij = en[u].cell;
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          const uint32_t nb = nbv[u][a];
          if (old[u][a] <= nb) continue;  // no improvement (or not relaxed at all)
          const int di = a < 4 ? ((a & 1) ? 0 : (a == 0 ? 1 : -1)) : ((a & 1) ? 1 : -1);
          const int dj = a < 4 ? ((a & 1) ? (a == 1 ? 1 : -1) : 0) : ((a & 2) ? 1 : -1);
          const int pi = (int)(cij >> 16) + di, pj = (int)(cij & 0xffffu) + dj;
          // the ellipse: a cell whose distance plus its straight-line distance to the start
          // exceeds the bound cannot lie on a path the search needs; it stays unsettled
          const float es = bres * sqrtf((float)((pi - sbx) * (pi - sbx) + (pj - sby) * (pj - sby)));
          if (__uint_as_float(nb) + es > bound) continue;
          const uint32_t pij = (uint32_t)pi << 16 | (uint32_t)pj;
          int kb = (int)(__uint_as_float(nb) * inv_wb);
          kb = max(kb, cur + 1);
          kb = min(kb, cur + 3);
          const int pos = atomicAdd(&S.cnt[kb & 7], 1);
          if (!bucket_put(A, bl, kb & 7, pos, BucketEntry{pij, nb})) S.overflow = 1;
        }
      }
    }
    RSTAMP(4);
    if (settled) atomicAdd(&S.settled, settled);
    block_sync();
    RSTAMP(5);
  }
  block_sync();
  if (tid == 0) S.buckets = cur;
#ifdef RELAX_STAMPS
  if (tid == 0)
    for (int k = 0; k < 6; ++k) S.stamp[k] = rst[k];
#endif
  return (float)cur * wb;
}

// The heuristic of cell (i, j): its block's Dijkstra distance, or for a block the ellipse left
// unsettled the bound minus the cell's straight-line distance to the field's start cell.
__device__ __forceinline__ float relaxed_h(const PlannerDev& P, const float* dist, int K, int i, int j, float bound,
                                          int sx, int sy) {
  const int nb = (P.N + K - 1) / K;
  const float d = ld_dist(dist, (size_t)(i / K) * nb + (j / K));
  if (d < FLT_MAX) return d;
  const float es = P.res * sqrtf((float)((i - sx) * (i - sx) + (j - sy) * (j - sy)));
  return fmaxf(bound - es, 0.0f);
}

// One expansion by one wavefront: the exact kernel's fused successor block without the
// closed set and the lazy A* (the heuristic is the Dijkstra field).  Every decision is keyed by
// values (g, f and the node's tie), never by the order in which the round's wavefronts run, so
// a query gives the same path on every run.
// RS sampling of a Reeds-Shepp shot (reversing model): poses every P.step metres of arc along
// the path's segments from (x0, y0, h0), sample 0 the shooter's own pose; curv[i] carries the
// segment's curvature with the sign of its direction of travel (-0.0f: a reverse straight);
// sample 0 carries d_start, the direction that reached the shooter.
// Returns the sample count, -1 when the scratch is too small, -2 at the first blocked chunk.
__device__ inline int rs_sample(const PlannerDev& P, const RSPath& rp, float x0, float y0, float h0, float d_start,
                                GAS float* xyh, GAS float* curv, int cap, int lane) {
  const float r = P.r_min, st = P.step;
  int cnt[5], base[5];
  float sx[5], sy[5], sh[5];
  int n = 1;
  float x = x0, y = y0, h = h0;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int kind = rs_kind(rp.word, k);
    const float a = rp.seg[k];
    const bool on = kind != RS_N && fabsf(a) > 1e-6f;
    cnt[k] = on ? max(1, (int)ceilf(fabsf(a) * r / st)) : 0;
    base[k] = n;
    n += cnt[k];
    sx[k] = x;
    sy[k] = y;
    sh[k] = h;
    if (on) rs_step(kind, r, x, y, h, a, &x, &y, &h);
  }
  if (n > cap) return -1;
  for (int b0 = 0; b0 < n; b0 += 64) {
    const int i = b0 + lane;
    bool bad = false;
    if (i < n) {
      float px = x0, py = y0, ph = h0, kc = 0.0f, d = d_start;
      if (i > 0) {
        // the segment holding sample i (constant indices after unrolling: no private arrays)
#pragma unroll
        for (int q = 0; q < 5; ++q) {
          if (cnt[q] > 0 && i >= base[q] && i < base[q] + cnt[q]) {
            const int kind = rs_kind(rp.word, q);
            const float a = rp.seg[q] * (float)(i - base[q] + 1) / (float)cnt[q];
            rs_step(kind, r, sx[q], sy[q], sh[q], a, &px, &py, &ph);
            kc = kind == RS_S ? 0.0f : 1.0f / r;
            d = rp.seg[q] < 0.0f ? -1.0f : 1.0f;
          }
        }
      } else {
        kc = rs_kind(rp.word, 0) == RS_S ? 0.0f : 1.0f / r;
      }
      xyh[3 * i] = px;
      xyh[3 * i + 1] = py;
      xyh[3 * i + 2] = wrap_pi_f(ph);
      curv[i] = copysignf(kc, d);
      bad = sample_blocked(P, px, py);
    }
    if (__ballot(bad)) return -2;
  }
  return n;
}
// the cost of a Reeds-Shepp shot from a node travelling in direction cdir (1: reverse): forward
// arc length, reverse arc length x rev_cost, and gear_cost per change of direction
__device__ __forceinline__ float rs_cost(const RSPath& p, float r, float rev_cost, float gear_cost, int cdir) {
  float c = 0.0f;
  int d = cdir;
  for (int k = 0; k < 5; ++k) {
    const float a = p.seg[k];
    if (rs_kind(p.word, k) == RS_N || fabsf(a) <= 1e-6f) continue;
    const int dk = a < 0.0f ? 1 : 0;
    c += fabsf(a) * r * (dk ? rev_cost : 1.0f) + (dk != d ? gear_cost : 0.0f);
    d = dk;
  }
  return c;
}

__device__ __forceinline__ void relaxed_expand(const PlannerDev& P, const RelaxArena& A, RelaxShared& S, ApfStage& apfs,
                               const GoalC& GC, const float* dist, int hk, float hlim, int hs_x, int hs_y, float hw, int idx,
                               int lane, uint2* list_n, const RelaxParams& rp) {
  const bool rev = rp.rev_cost > 0.0f;
  const Node3 cur = gload(&A.nodes[idx]);
  const uint32_t key = ufu(cur.key), tie = ufu((uint32_t)cur.r);
  const float cg = uff(cur.g), cf = uff(cur.f), cxp = uff(cur.x), cyp = uff(cur.y), chd = uff(cur.h),
              cvm = uff(cur.vmin);
  const int cci = ufi((int)(cur.cc >> 8));
  const int cdir = ufi((int)(cur.cc & 1u));  // 1: the node was reached in reverse
  const int cx = key3_x(key), cy = key3_y(key), cbin = key3_bin(key);
  if (lane == 0) atomicAdd(&S.pops, 1);
  // goal test (Node3D::operator==: the cell only, Node3D.h:42).  The stages below run under
  // wave-uniform flags, with no early return out of divergent code.
  int done = 0;
  if (cx == P.goal_cx && cy == P.goal_cy) {
    if (lane == 0) atomicMin(&S.best, ((unsigned long long)__float_as_uint(cg) << 32) | (tie & 0x7fffffffu));
    done = 1;
  }
  // Dubins shot (HybridAStar.cpp:115-154): the round's shooters were chosen between rounds
  const bool allowed = cvm < 1.0f;
  int shot = -1;
  if (!done && allowed) {
    const unsigned long long v = shot_key(cf, cg, tie);
    for (int q = 0; q < S.n_sel; ++q)
      if (S.sel[q] == v) shot = q;
  }
  shot = ufi(shot);
  if (shot >= 0) {
    if (lane == 0) atomicAdd(&S.shots, 1);
    const float r = P.r_min;
    GAS float* xyh = gp(A.dub_xyh) + (size_t)shot * A.dub_cap * 3;
    GAS float* curv = gp(A.dub_curv) + (size_t)shot * A.dub_cap;
    float L;
    int n;
    if (rev) {  // Reeds-Shepp shot: the shortest of its 44 candidates, sampled and checked
      const RSPath rsp = rs_best(r, cxp, cyp, chd, P.goal_x, P.goal_y, P.goal_h, lane);
      L = rs_cost(rsp, r, rp.rev_cost, rp.gear_cost, cdir);
      n = rsp.L < RS_INF ? ufi(rs_sample(P, rsp, cxp, cyp, chd, cdir ? -1.0f : 1.0f, xyh, curv, A.dub_cap, lane)) : -1;
    } else {
      int word = 0;
      float prm[4];
      L = dubins_shortest(r, cxp, cyp, chd, P.goal_x, P.goal_y, P.goal_h, &word, prm);
      const Centres C = dubins_centres(r, cxp, cyp, chd, P.goal_x, P.goal_y, P.goal_h);
      // sampled and checked chunk by chunk: a blocked shot stops at its first blocked chunk
      const int first_arc_long = ufi(fabsf(prm[1]) > (float)M_PI_2 ? 1 : 0);
      n = first_arc_long ? -1 : ufi(dubins_sample<1>(P, C, word, prm, xyh, curv, A.dub_cap, lane));
    }
    wave_lds_sync();
    if (n > 0) {
      const int term = ufi(cur.prev);
      if (lane == 0) {
        S.shot_term[shot] = term;
        S.shot_n[shot] = n;
        atomicMin(&S.best, ((unsigned long long)__float_as_uint(cg + L) << 32) | 0x80000000u | (unsigned)shot);
      }
      done = 1;
    }
  }
  done = ufi(done);
  if (done) return;
  // successors (VehicleModel.cpp:63-105) in groups of gs lanes, as in the exact kernel; with
  // the reversing model every steering also gets a reverse arc (candidates span .. 2 span - 1)
  const int span = 2 * P.na + 1;
  const int gsh = (span <= 4 && !rev) ? 4 : 2, gs = 1 << gsh;
  int lo = cci - P.na;
  lo = lo < 0 ? 0 : lo;
  const int ca = lane >> gsh, sub = lane & (gs - 1);
  const bool back = rev && ca >= span;
  const int ai = lo + (back ? ca - span : ca);
  bool cand = ca < (rev ? 2 * span : span) && ai < P.nsteer;
  const int ia = cand ? ai : lo;
  const float cabs = gp(P.curv_abs)[ia];
  const float odth = gp(P.dth)[ia];
  // a reverse arc is a forward arc driven backwards: it starts at the heading h0 = h - dth whose
  // forward arc ends at h, and moves by minus that arc's offset (the offset of h0's bin)
  const float h_rev = wrap_pi_f(chd - odth);
  const int obin = back ? heading_bin(h_rev, P.prec) : cbin;
  const GAS float* ofs = &gp(P.off)[2 * ((size_t)ia * (P.bins + 1) + obin)];
  const float ofx = ofs[0], ofy = ofs[1];
  const float oact = gp(P.act_cost)[ia] * (back ? rp.rev_cost : 1.0f) + ((back ? 1 : 0) != cdir ? rp.gear_cost : 0.0f);
  float vm = 0.0f;
  if (cand && !allowed) {
    const float lat = cvm * cabs;
    if (lat > P.a_lat) cand = false;
    const float al = (float)sqrt(1.0 - (double)((lat * lat) / P.a_lat2));
    vm = cvm - 2.0f * al * P.ts;
  }
  float sx = 0.0f, sy = 0.0f, sh = 0.0f, sg = 0.0f;
  int sbin = 0, scx = 0, scy = 0;
  bool inb = false;
  if (cand) {
    sx = back ? cxp - ofx : cxp + ofx;
    sy = back ? cyp - ofy : cyp + ofy;
    sh = back ? h_rev : wrap_pi_f(chd + odth);
    sg = cg + oact;
    sbin = heading_bin(sh, P.prec);
    scx = trunc_f(sx / P.res);
    scy = trunc_f(sy / P.res);
    inb = scx > -1 && scx < P.N && scy > -1 && scy < P.N;
  }
  const bool lead = inb && sub == 0;
  float occv = 0.0f, h2 = 0.0f;
  if (lead) {
    const size_t cell = (size_t)scx * P.N + scy;
    occv = gp(P.occ)[cell];
    h2 = relaxed_h(P, dist, hk, scx, scy, hlim, hs_x, hs_y);
  }
  const float dub = rev ? rs_length_group(P.r_min, sx, sy, sh, P.goal_x, P.goal_y, P.goal_h, gs, lane)
                        : cand_dubins(P.r_min, GC, P.goal_h, sx, sy, sh, gs, lane);
  const float fc = apf_fused(P, apfs, cxp, cyp, sx, sy, sh, __ballot(lead), gs, lane);
  const bool kept = lead && occv < P.thr;
  const uint64_t km = __ballot(kept);
  if (lane == 0) atomicAdd(&S.succ, __popcll(km));
  if (kept) {
    const float g = sg + fc;  // Grid3D.cpp:66-69
    const float f = g + hw * stl_max(h2, dub);
    const uint32_t skey = key3(scx, scy, sbin);
    // equal-g offers for one key resolve by this tie, a hash of (parent key, action)
    const uint32_t stie = rx_hash(key * 0x9e3779b1u + (uint32_t)ai + (back ? 0x10000u : 0u));
    bool full = false;
    uint32_t tslot = 0;
    if (table_lower(A, skey, ((unsigned long long)__float_as_uint(g) << 32) | stie, &full, &tslot)) {
      const int n = atomicAdd(&S.nodes, 1);
      const int pos = atomicAdd(&S.nN, 1);
      if (n < A.node_cap && pos < A.list_cap) {
        Node3 d;
        d.key = skey;
        d.f = f;
        d.l = (int)tslot;
        d.r = (int)stie;
        d.p = NIL;
        d.cc = ((uint32_t)ai << 8) | (back ? 1u : 0u);
        d.g = g;
        d.vmin = vm;
        d.x = sx;
        d.y = sy;
        d.h = sh;
        d.prev = idx;
        gstore(&A.nodes[n], d);
        list_n[pos] = make_uint2(__float_as_uint(f), (uint32_t)n);
      } else {
        S.overflow = 1;
      }
    }
    if (full) S.overflow = 1;
  }
}

__device__ void relaxed_one(const PlannerDev& P, const RelaxArena& A, RelaxShared& S, const RelaxParams& rp,
                            RelaxField* F, BucketEntry* bl, int pi) {
  const int tid = threadIdx.x, NT = blockDim.x, wv = tid >> 6, lane = tid & 63;
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  RPROG(0, 1);
  // the heuristic field: the planner's own (kept across calls until reset / update_goal, like
  // the reference's A* memo) or the arena's scratch
  float* dist = (F && F->dist) ? F->dist : A.dist;
  float hlim;
  int hs_x = P.start_cx, hs_y = P.start_cy;  // the start cell the field's ellipse was built around
  if (F && F->dist && F->valid) {
    hlim = F->hlim;
    hs_x = F->start_ij >> 16;
    hs_y = F->start_ij & 0xffff;
    if (tid == 0) {
      S.buckets = 0;
      S.settled = 0;
      S.overflow = 0;
    }
  } else {
    hlim = relaxed_heuristic(P, A, S, rp, dist, bl);
    if (tid == 0 && F && F->dist) {
      F->hlim = hlim;
      F->start_ij = (P.start_cx << 16) | P.start_cy;
      F->valid = 1;
    }
  }
  const unsigned long long t_heur = __builtin_amdgcn_s_memrealtime();
  RPROG(0, 2);
  // ---- the frontier-parallel search
  apf_stage(P, S.apf[wv], lane);
  const GoalC GC = goal_centres(P.r_min, P.goal_x, P.goal_y, P.goal_h);
  if (tid == 0) {
    Node3 s0;
    s0.key = key3(P.start_cx, P.start_cy, P.start_bin);
    const float h0 = relaxed_h(P, dist, rp.h_coarse, P.start_cx, P.start_cy, hlim, hs_x, hs_y);
    s0.f = h0;
    s0.l = s0.p = NIL;
    s0.r = 0;
    s0.cc = (uint32_t)P.start_ci << 8;
    s0.g = 0.0f;
    s0.vmin = P.start_vmin;
    s0.x = P.start_x;
    s0.y = P.start_y;
    s0.h = P.start_h;
    s0.prev = NIL;
    gstore(&A.nodes[0], s0);
    bool full = false;
    uint32_t tslot = 0;
    table_lower(A, s0.key, 0ull, &full, &tslot);
    A.nodes[0].l = (int)tslot;  // tie 0: s0.r
    reinterpret_cast<uint2*>(A.lists)[0] = make_uint2(__float_as_uint(s0.f), 0u);
    S.nA = 1;
    S.nB = 0;
    S.nE = 0;
    S.nN = 0;
    S.nE_last = 0;
    S.n_allowed = 0;
    S.n_sel = 0;
    for (int q = 0; q < RW; ++q) S.sel[q] = ~0ull;
    S.last_shot_h = FLT_MAX;
    S.eNext = 0;
    S.nodes = 1;
    S.best = ~0ull;
    S.since_shot = 0;
    S.interval = P.shot_interval;
    S.pops = S.succ = S.shots = S.rounds = 0;
    S.fmin = __float_as_uint(s0.f);
    S.fnext = 0x7f800000u;
    S.hover = S.overflow;  // a bucket overflow only weakens the heuristic: reported, not fatal
    S.overflow = 0;
  }
  if (lane == 0) {
    S.shot_n[wv] = 0;
    S.shot_term[wv] = NIL;
  }
  block_sync();
  // lists L[a]: the open list; L[a ^ 1]: the next open list; LE: the round's expansion set.
  // A round: split the open list (f <= min f + delta and still current -> LE, f above -> next),
  // choose the round's shooters, expand LE (raw successors -> the free L[a]), then keep the
  // successors still current at the round's end.  Every choice is made between rounds from
  // values, so the rounds — and the path — do not depend on wavefront timing.
  uint2* const L0 = reinterpret_cast<uint2*>(A.lists);
  int* const LE = reinterpret_cast<int*>(L0 + (size_t)2 * A.list_cap);
  int a = 0;
  int status = 0;
  for (int round = 0;; ++round) {
    uint2* LA = L0 + (size_t)a * A.list_cap;
    uint2* LB = L0 + (size_t)(a ^ 1) * A.list_cap;
    const int nA = S.nA;
    const float thr = __uint_as_float(S.fmin) + rp.delta;
    if (nA == 0 || S.best != ~0ull) break;
    if (round >= rp.max_rounds || S.overflow) {
      status = -75;
      break;
    }
    RPROG(0, 3);
    RPROG(1, round);
    // split; a candidate no longer current (a cheaper node of its key exists) is dropped.  The
    // split also ranks the round's shot-allowed candidates (shot_key) for the first shooter.
    uint32_t fm = 0x7f800000u;
    int allowed = 0;
    unsigned long long mk = ~0ull;
    for (int e = tid; e < nA; e += NT) {
      const uint2 en = LA[e];
      if (__uint_as_float(en.x) <= thr) {
        float vm, g;
        uint32_t tie;
        if (node_current(A, (int)en.y, &vm, &g, &tie)) {
          LE[atomicAdd(&S.nE, 1)] = (int)en.y;
          if (vm < 1.0f) {
            ++allowed;
            const unsigned long long v = shot_key(__uint_as_float(en.x), g, tie);
            mk = v < mk ? v : mk;
          }
        }
      } else {
        LB[atomicAdd(&S.nB, 1)] = en;
        fm = min(fm, en.x);
      }
    }
    fm = wave_min_u32(fm);
    if (lane == 0 && fm != 0x7f800000u) atomicMin(&S.fnext, fm);
    if (allowed) atomicAdd(&S.n_allowed, allowed);
    mk = wave_min_u64(mk);
    if (lane == 0 && mk != ~0ull) atomicMin(&S.sel[0], mk);
    block_sync();
    // the shot schedule (HybridAStar.cpp:115-154): the counter advances by the round's
    // shot-allowed expansions; each time it reaches the interval one shot is due and the
    // interval decays.  The due shots go to the round's allowed nodes of lowest shot_key.
    // Besides those, one shot goes to the frontier's most advanced node whenever its f - g has
    // fallen to SHOT_ADVANCE of the last shooter's (a shot costs one wavefront for a few
    // microseconds; a round without one can cost the search many rounds).
    if (tid == 0) {
      int c = S.since_shot + S.n_allowed, k = 0;
      while (c >= S.interval && k < RW) {
        c -= S.interval;
        S.interval = max(S.interval - P.shot_decay, 50);
        ++k;
      }
      S.since_shot = k == RW ? 0 : c;
      const unsigned long long s0 = S.sel[0];
      const float h0 = __uint_as_float((uint32_t)(s0 >> 32));
      const bool advance = s0 != ~0ull && h0 <= SHOT_ADVANCE * S.last_shot_h;
      if (s0 != ~0ull && (advance || k > 0)) S.last_shot_h = h0;
      S.n_sel = k > 0 ? k : (advance ? 1 : 0);
    }
    block_sync();
    const int nE = S.nE, n_sel = S.n_sel;
    RPROG(0, 4);
    RPROG(2, nE);
    // further due shooters (rare: more than one due in a round), next-lowest shot_key each
    unsigned long long prev_sel = S.sel[0];
    for (int q = 1; q < n_sel; ++q) {
      unsigned long long m = ~0ull;
      for (int e = tid; e < nE; e += NT) {
        const Node3* nd = &A.nodes[LE[e]];
        const int4 q0 = *reinterpret_cast<const int4*>(nd);
        const float4 q1 = *(reinterpret_cast<const float4*>(nd) + 1);  // p, cc, g, vmin
        if (q1.w >= 1.0f) continue;
        const unsigned long long v = shot_key(__int_as_float(q0.y), q1.z, (uint32_t)q0.w);
        if (v > prev_sel && v < m) m = v;
      }
      m = wave_min_u64(m);
      if (lane == 0 && m != ~0ull) atomicMin(&S.sel[q], m);
      block_sync();
      prev_sel = S.sel[q];
    }
    // one wavefront per expanded node
    for (;;) {
      int e = 0;
      if (lane == 0) e = atomicAdd(&S.eNext, 1);
      e = ufi(e);
      if (e >= nE) break;
      RPROG(0, 5);
      RPROG(3, e);
      relaxed_expand(P, A, S, S.apf[wv], GC, dist, rp.h_coarse, hlim, hs_x, hs_y, rp.h_weight, LE[e], lane, LA, rp);
    }
    RPROG(0, 6);
    block_sync();
    // the round's successors that are still their key's best join the next open list
    const int nN = min(S.nN, A.list_cap);
    fm = 0x7f800000u;
    for (int e = tid; e < nN; e += NT) {
      const uint2 en = LA[e];
      if (!node_current(A, (int)en.y)) continue;
      const int pos = atomicAdd(&S.nB, 1);
      if (pos < A.list_cap) {
        LB[pos] = en;
        fm = min(fm, en.x);
      } else {
        S.overflow = 1;
      }
    }
    fm = wave_min_u32(fm);
    if (lane == 0 && fm != 0x7f800000u) atomicMin(&S.fnext, fm);
    RPROG(0, 7);
    block_sync();
    if (tid == 0) {
      S.nA = min(S.nB, A.list_cap);
      S.nB = 0;
      S.nE_last = nE;
      S.nE = 0;
      S.nN = 0;
      S.n_allowed = 0;
      S.n_sel = 0;
      for (int q = 0; q < RW; ++q) S.sel[q] = ~0ull;
      S.eNext = 0;
      S.fmin = S.fnext;
      S.fnext = 0x7f800000u;
      S.rounds = round + 1;
      // watchdog: a search still running after RELAX_WATCHDOG ticks ends as an overflow
      if (__builtin_amdgcn_s_memrealtime() - t_start > RELAX_WATCHDOG) S.overflow = 2;
    }
    block_sync();
    a ^= 1;  // the next open list becomes the open list
  }
  RPROG(0, 8);
  block_sync();
  // ---- result and reconstruction (HybridAStar.cpp:208-262, as the exact kernel), by wave 0
  const unsigned long long best = S.best;
  const bool found = best != ~0ull && status == 0;
  if (wv == 0) {
    int ok = found ? 1 : 0, via_shot = 0, terminal = NIL, dub_n = 0, sw = 0;
    float cost = FLT_MAX;
    if (found) {
      const uint32_t tag = (uint32_t)best;
      cost = __uint_as_float((uint32_t)(best >> 32));
      if (tag & 0x80000000u) {
        via_shot = 1;
        sw = (int)(tag & 0xffu);
        terminal = S.shot_term[sw];
        dub_n = S.shot_n[sw];
      } else {
        // the goal node of the last round whose {g, tie} won (its LE is still intact)
        int t = 0x7fffffff;
        for (int e = lane; e < S.nE_last; e += 64) {
          const int idx = LE[e];
          const Node3 nd = A.nodes[idx];
          if (key3_x(nd.key) == P.goal_cx && key3_y(nd.key) == P.goal_cy &&
              (((unsigned long long)__float_as_uint(nd.g) << 32) | ((uint32_t)nd.r & 0x7fffffffu)) == best)
            t = min(t, idx);
        }
        terminal = (int)wave_min_u32((uint32_t)t);
        if (terminal == 0x7fffffff) {
          ok = 0;
          status = -75;
        }
      }
    }
    int path_len = 0;
    if (ok) {
      int L = 0;
      for (int i = terminal; i != NIL; i = A.nodes[i].prev) {
        if (dub_n + L >= P.out_cap || L >= A.chain_cap) {
          status = -28;
          break;
        }
        if (lane == 0) A.chain[L] = i;
        ++L;
      }
      wave_lds_sync();
      if (status == 0) {
        const GAS float* dxyh = gp(A.dub_xyh) + (size_t)sw * A.dub_cap * 3;
        const GAS float* dcurv = gp(A.dub_curv) + (size_t)sw * A.dub_cap;
        const float cs = P.rot_c, sn = P.rot_s, ang = -P.grid_heading;
        path_len = dub_n + L;
        signed char* dout = rp.dir_out ? rp.dir_out + (size_t)pi * rp.dir_stride : nullptr;
        for (int k = lane; k < path_len; k += 64) {
          float px, py, ph, kc = 0.0f;
          bool has_curv = true;
          int dir = 1;
          if (k < dub_n) {
            const int q = dub_n - 1 - k;
            px = dxyh[3 * q];
            py = dxyh[3 * q + 1];
            ph = dxyh[3 * q + 2];
            kc = dcurv[q];
            dir = signbit(kc) ? -1 : 1;  // a Reeds-Shepp sample's direction (rs_sample)
            kc = fabsf(kc);
          } else {
            const int m = k - dub_n;
            const Node3 nd = gload(&A.nodes[A.chain[m]]);
            px = nd.x;
            py = nd.y;
            ph = nd.h;
            kc = gp(P.curv_abs)[nd.cc >> 8];
            dir = (nd.cc & 1u) ? -1 : 1;
            has_curv = (m < L - 1);
          }
          if (dout && k < rp.dir_stride) dout[k] = (signed char)dir;
          const float x0 = px - P.goal_x, y0 = py - P.goal_y;
          float xr = x0 * cs + y0 * sn;
          float yr = -x0 * sn + y0 * cs;
          const float hr = wrap_pi_f(ph - ang);
          xr += P.world_goal_x;
          yr += P.world_goal_y;
          gp(P.out_xyh)[3 * k] = xr;
          gp(P.out_xyh)[3 * k + 1] = yr;
          gp(P.out_xyh)[3 * k + 2] = hr;
          if (has_curv) gp(P.out_curv)[k + 1] = kc;
        }
        if (lane == 0) gp(P.out_curv)[0] = 0.0f;
      } else {
        ok = 0;
      }
    }
    if (lane == 0) {
      SearchResult* R = P.result;
      R->pops = S.pops;
      R->successors = S.succ;
      R->astar_pops = S.settled;      // cells the Dijkstra settled
      R->astar_searches = 1;
      R->shots = S.shots;
      R->closed_size = min(S.nodes, A.node_cap);  // nodes generated
      R->pop_digest = (unsigned long long)S.rounds;
      R->closed_digest = 0;
      R->ok = ok;
      R->via_shot = via_shot;
      R->status = status;
      R->path_len = ok ? path_len : 0;
      R->cost = ok ? cost : FLT_MAX;
      R->terminal = terminal;
      R->dubins_len = dub_n;
      R->astar_migrations = S.hover;  // 1: the Dijkstra's bucket ring overflowed
      R->astar_pops_hbm = 0;
      R->t_start = t_start;
      R->t_end = __builtin_amdgcn_s_memrealtime();
      R->slot = (int)blockIdx.x;
      R->parks = 0;
      // phase split (s_memrealtime, 100 MHz; hastar_debug_cycles): clear + Dijkstra, search
      // rounds + reconstruction, Dijkstra buckets, search rounds
      for (int q = 0; q < NSTAMP; ++q) R->cycles[q] = 0;
      R->cycles[0] = t_heur - t_start;
      R->cycles[1] = R->t_end - t_heur;
      R->cycles[2] = (unsigned long long)S.buckets;
      R->cycles[3] = (unsigned long long)S.rounds;
      R->cycles[4] = (unsigned long long)S.overflow;
      R->cycles[5] = (unsigned long long)S.nA;
      R->cycles[6] = (unsigned long long)S.nE_last;
      R->cycles[7] = (unsigned long long)S.fmin;
#ifdef RELAX_STAMPS
      for (int k = 0; k < 6; ++k) R->cycles[8 + k] = S.stamp[k];
#endif
    }
  }
  RPROG(0, 9);
  // leave the best-g table empty for the next planner: the slots this search claimed (kept in
  // its nodes), or the whole table when an overflow may have left claimed slots without a node
  if (S.overflow) {
    for (size_t i = tid; i <= A.tmask; i += NT) {
      A.table[i].key = EMPTY_KEY;
      A.table[i].best = ~0ull;
    }
  } else {
    const int nn = min(S.nodes, A.node_cap);
    for (int n = tid; n < nn; n += NT) {
      const uint32_t t = (uint32_t)A.nodes[n].l;
      A.table[t].key = EMPTY_KEY;
      A.table[t].best = ~0ull;
    }
  }
  block_sync();
  RPROG(0, 10);
}

// Persistent: grid = resident relaxed arenas; each workgroup pulls planners from *next.
__global__ __launch_bounds__(RW * 64) void k_relaxed_search(const PlannerDev* __restrict__ descs, int n,
                                                           const RelaxArena* __restrict__ arenas, int* next,
                                                           RelaxParams rp, RelaxField* fields) {
  __shared__ RelaxShared S;
  extern __shared__ BucketEntry relax_dyn_lds[];
  const RelaxArena A = arenas[blockIdx.x];
  for (;;) {
    if (threadIdx.x == 0) S.planner = atomicAdd(next, 1);
    block_sync();
    const int pi = S.planner;
    block_sync();
    if (pi >= n) break;
    relaxed_one(descs[pi], A, S, rp, fields ? &fields[pi] : nullptr, relax_dyn_lds, pi);
  }
}

hipError_t launch_relaxed(const PlannerDev* d_descs, int n, const RelaxArena* d_arenas, int n_arenas, int* d_next,
                          const RelaxParams& rp, RelaxField* d_fields, hipStream_t st) {
  hipError_t e = hipMemsetAsync(d_next, 0, sizeof(int), st);
  if (e != hipSuccess) return e;
  // the dynamic-LDS opt-in, once per device (callers hold the device context's lock)
  static bool attr[64] = {};
  int dev = 0;
  hipError_t a = hipGetDevice(&dev);
  if (a != hipSuccess) return a;
  if (!attr[dev & 63]) {
    a = hipFuncSetAttribute(reinterpret_cast<const void*>(k_relaxed_search), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)RELAX_DYN_LDS);
    if (a != hipSuccess) return a;
    attr[dev & 63] = true;
  }
  hipLaunchKernelGGL(k_relaxed_search, dim3(n_arenas), dim3(RW * 64), RELAX_DYN_LDS, st, d_descs, n, d_arenas, d_next,
                     rp, d_fields);
  return hipGetLastError();
}
int relaxed_waves() { return RW; }

// unit test of the Reeds-Shepp code (hastar_test_reeds_shepp): one wavefront per start pose:
// rs_best's length (metres), word and segments (radius units), and rs_length_group's length with
// groups of 4 and of 16 lanes
__global__ __launch_bounds__(64) void k_test_rs(float r, const float* __restrict__ starts, int n, float gx, float gy,
                                                float gh, float* __restrict__ len, int* __restrict__ word,
                                                float* __restrict__ seg, float* __restrict__ len_groups) {
  const int lane = (int)threadIdx.x, i = (int)blockIdx.x;
  if (i >= n) return;
  const float sx = starts[3 * i], sy = starts[3 * i + 1], sh = starts[3 * i + 2];
  const RSPath p = rs_best(r, sx, sy, sh, gx, gy, gh, lane);
  const float l4 = rs_length_group(r, sx, sy, sh, gx, gy, gh, 4, lane);
  const float l16 = rs_length_group(r, sx, sy, sh, gx, gy, gh, 16, lane);
  if (lane == 0) {
    len[i] = p.L * r;
    word[i] = p.word;
    for (int k = 0; k < 5; ++k) seg[5 * i + k] = p.seg[k];
    len_groups[2 * i] = l4;
    len_groups[2 * i + 1] = l16;
  }
}
hipError_t launch_test_rs(float r, const float* starts, int n, float gx, float gy, float gh, float* len, int* word,
                          float* seg, float* len_groups, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_test_rs, dim3((unsigned)n), dim3(64), 0, st, r, starts, n, gx, gy, gh, len, word, seg, len_groups);
  return hipGetLastError();
}

}  // namespace hastar
