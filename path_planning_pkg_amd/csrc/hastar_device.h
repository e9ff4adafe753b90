// hastar_device.h — device-side building blocks of the search (HIP, gfx950).
//
// Every function restates one reference expression with the reference's exact float /
// double promotions (compiled with -ffp-contract=off; the only fused multiply-adds are
// the explicit fma() calls inside glibc_mathf.h that mirror glibc's FMA build).
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>
#include "hastar_layout.h"
#include "glibc_mathf.h"
#include "rbtree_dev.h"

namespace hastar {
using namespace gmath;

// Pointers loaded from the descriptor are generic (flat) to the compiler; every access
// through them would be a flat_load/flat_store with vmcnt+lgkmcnt waits.  They all point
// to hipMalloc'ed HBM, so the kernels view them as address_space(1) (global).
#define GAS __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ GAS T* gp(T* p) {
  return (GAS T*)p;
}

// Wave-uniform value into an SGPR (values every lane loaded from the same address).
__device__ __forceinline__ int ufi(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t ufu(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ float uff(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// Cross-lane hand-off through LDS/HBM inside ONE wavefront: the wave's memory operations
// stay in order in hardware (LLVM AMDGPU memory model: wavefront scope needs no cache or
// counter action), so this is only a compiler barrier — unlike __syncthreads, which also
// drains every outstanding global load and store (s_waitcnt vmcnt(0)).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// whole-record copies to/from HBM in 16-byte pieces (records are 16-byte aligned)
typedef int v4i __attribute__((ext_vector_type(4)));
template <class T>
__device__ __forceinline__ T gload(const GAS T* p) {
  static_assert(sizeof(T) % 16 == 0, "record size");
  union U { T v; v4i q[sizeof(T) / 16]; } u;
  const GAS v4i* src = (const GAS v4i*)p;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 16); ++i) u.q[i] = src[i];
  return u.v;
}
template <class T>
__device__ __forceinline__ void gstore(GAS T* p, const T& v) {
  static_assert(sizeof(T) % 16 == 0, "record size");
  union U { T v; v4i q[sizeof(T) / 16]; } u;
  u.v = v;
  GAS v4i* dst = (GAS v4i*)p;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 16); ++i) dst[i] = u.q[i];
}
// the same for LDS / generic pointers
template <class T>
__device__ __forceinline__ T gload(const T* p) {
  return *p;
}
template <class T>
__device__ __forceinline__ void gstore(T* p, const T& v) {
  *p = v;
}

// common.h:15-29 for T = float: fmod in double, compare against M_PI in double.
__device__ __forceinline__ float wrap_pi_f(float a) {
  const float w = (float)fmod_2pi((double)a);
  if ((double)w > M_PI) return (float)((double)w - 2 * M_PI);
  if ((double)w < -M_PI) return (float)((double)w + 2 * M_PI);
  return w;
}
// common.h:15-29 instantiated with T = double (Dubins.cpp sampling: wrap_pi(theta - M_PI_2)).
__device__ __forceinline__ double wrap_pi_d(double a) {
  const double w = fmod_2pi(a);
  if (w > M_PI) return w - 2 * M_PI;
  if (w < -M_PI) return w + 2 * M_PI;
  return w;
}
// common.h:31-36: round_to_nearest in float, index in double, truncation.
__device__ __forceinline__ int heading_bin(float h, float prec) {
  const float r = roundf(h / prec) * prec;
  return x86_trunc_int(((double)r + M_PI) / (double)prec);
}
__device__ __forceinline__ int trunc_f(float v) { return x86_trunc_int((double)v); }

__device__ __forceinline__ uint32_t key3(int cx, int cy, int bin) {
  return ((uint32_t)cx << 20) | ((uint32_t)cy << 8) | (uint32_t)bin;
}
__device__ __forceinline__ int key3_x(uint32_t k) { return (int)(k >> 20); }
__device__ __forceinline__ int key3_y(uint32_t k) { return (int)((k >> 8) & 0xfffu); }
__device__ __forceinline__ int key3_bin(uint32_t k) { return (int)(k & 0xffu); }
__device__ __forceinline__ uint64_t digest_key(uint32_t k) {
  return ((uint64_t)(uint32_t)key3_x(k) << 40) | ((uint64_t)(uint32_t)key3_y(k) << 16) | (uint64_t)key3_bin(k);
}
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// std::max / std::min as libstdc++ defines them
__device__ __forceinline__ float stl_max(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ float stl_min(float a, float b) { return (b < a) ? b : a; }

// Grid2D::compute_heuristic (Grid2D.cpp:303-316): Euclidean distance to the goal cell.
__device__ __forceinline__ float euclid_h(const PlannerDev& P, int i, int j) {
  const float dx = (float)(P.n45 - i) * P.res;
  const float dx2 = dx * dx;
  const float dy = (float)(P.n2 - j) * P.res;
  const float dy2 = dy * dy;
  return sqrtf(dx2 + dy2);
}

// ------------------------------------------------------------- Dubins (Dubins.cpp) --
struct Centres { float srx, sry, slx, sly, grx, gry, glx, gly; };

// Dubins.cpp:19-32: circle centres of a start and a goal pose.  The goal half is the same
// for every evaluation of one search, so it is computed once (GoalC).
struct GoalC { float grx, gry, glx, gly; };
__device__ __forceinline__ GoalC goal_centres(float r, float gx, float gy, float gh) {
  const float sg = g_sinf(gh), cg = g_cosf(gh);
  return GoalC{gx + r * sg, gy - r * cg, gx - r * sg, gy + r * cg};
}
// start half from sin/cos of the start heading
__device__ __forceinline__ Centres centres_from(float r, float sx, float sy, float ss, float cs, const GoalC& G) {
  Centres c;
  c.srx = sx + r * ss;
  c.sry = sy - r * cs;
  c.slx = sx - r * ss;
  c.sly = sy + r * cs;
  c.grx = G.grx;
  c.gry = G.gry;
  c.glx = G.glx;
  c.gly = G.gly;
  return c;
}
__device__ __forceinline__ Centres dubins_centres_g(float r, float sx, float sy, float sh, const GoalC& G) {
  return centres_from(r, sx, sy, g_sinf(sh), g_cosf(sh), G);
}
__device__ __forceinline__ Centres dubins_centres(float r, float sx, float sy, float sh, float gx, float gy,
                                                  float gh) {
  return dubins_centres_g(r, sx, sy, sh, goal_centres(r, gx, gy, gh));
}

// Dubins.cpp:180-323 — CSC word w (0 RSR, 1 RSL, 2 LSR, 3 LSL) in stages, so that a
// wavefront can spread one word's libm calls over several lanes:
//   word_geo      centre-to-centre vector of the word's circles;
//   (caller)      th = atan2f(dy, dx); for RSL/LSR ac = acosf(2r / dist);
//   word_arcs     the tangent angles t1 and q[2] of RSL/LSR;
//   (caller)      cos/sin of t1 and q[2] for RSL/LSR;
//   word_len      params and length.
struct WordGeo { float csx, csy, cgx, cgy, dx, dy, dist; };
__device__ __forceinline__ WordGeo word_geo(int w, const Centres& C) {
  WordGeo g;
  g.csx = (w < 2) ? C.srx : C.slx;
  g.csy = (w < 2) ? C.sry : C.sly;
  g.cgx = (w == 0 || w == 2) ? C.grx : C.glx;
  g.cgy = (w == 0 || w == 2) ? C.gry : C.gly;
  g.dx = g.cgx - g.csx;
  g.dy = g.cgy - g.csy;
  g.dist = sqrtf(g.dx * g.dx + g.dy * g.dy);
  return g;
}
__device__ __forceinline__ float word_acos_arg(float r, const WordGeo& g) { return 2.0f * r / g.dist; }
__device__ __forceinline__ void word_arcs(int w, float th, float ac, float* t1, float* q2) {
  if (w == 1) {
    *t1 = ac + th;
    *q2 = (float)((double)*t1 - M_PI);
  } else {
    *t1 = -ac + th;
    *q2 = (float)((double)*t1 + M_PI);
  }
}
__device__ __forceinline__ float word_len(int w, float r, const WordGeo& g, float sh, float gh, float th, float t1,
                                          float ct1, float st1, float cq2, float sq2, float q[4]) {
  if (w == 0 || w == 3) {
    if (w == 0) {
      q[0] = (float)(M_PI_2 + (double)sh);
      const float a1 = (float)(M_PI_2 + (double)th);
      q[2] = a1;
      const float tg = (float)(M_PI_2 + (double)gh);
      q[1] = a1 - q[0];
      if (q[1] > 0) q[1] = (float)((double)q[1] - 2 * M_PI);
      q[3] = tg - q[2];
      if (q[3] > 0) q[3] = (float)((double)q[3] - 2 * M_PI);
    } else {
      q[0] = (float)(-M_PI_2 + (double)sh);
      const float a1 = (float)(-M_PI_2 + (double)th);
      q[2] = a1;
      const float tg = (float)(-M_PI_2 + (double)gh);
      q[1] = a1 - q[0];
      if (q[1] < 0) q[1] = (float)((double)q[1] + 2 * M_PI);
      q[3] = tg - q[2];
      if (q[3] < 0) q[3] = (float)((double)q[3] + 2 * M_PI);
    }
    return (w == 0) ? g.dist + r * -(q[1] + q[3]) : g.dist + r * (q[1] + q[3]);
  }
  if (w == 1) {
    q[0] = (float)(M_PI_2 + (double)sh);
    q[2] = (float)((double)t1 - M_PI);
    const float tg = (float)(-M_PI_2 + (double)gh);
    q[1] = t1 - q[0];
    if (q[1] > 0) q[1] = (float)((double)q[1] - 2 * M_PI);
    q[3] = tg - q[2];
    if (q[3] < 0) q[3] = (float)((double)q[3] + 2 * M_PI);
  } else {
    q[0] = (float)(-M_PI_2 + (double)sh);
    q[2] = (float)((double)t1 + M_PI);
    const float tg = (float)(M_PI_2 + (double)gh);
    q[1] = t1 - q[0];
    if (q[1] < 0) q[1] = (float)((double)q[1] + 2 * M_PI);
    q[3] = tg - q[2];
    if (q[3] > 0) q[3] = (float)((double)q[3] - 2 * M_PI);
  }
  float ax = g.csx, ay = g.csy, bx = g.cgx, by = g.cgy;
  ax += r * ct1;
  ay += r * st1;
  bx += r * cq2;
  by += r * sq2;
  const float ex = bx - ax, ey = by - ay;
  const float dst = sqrtf(ex * ex + ey * ey);
  return (w == 1) ? dst + r * (-q[1] + q[3]) : dst + r * (q[1] - q[3]);
}

// One lane evaluates the whole word.
__device__ __forceinline__ float dubins_word(int w, float r, const Centres& C, float sh, float gh, float q[4]) {
  const WordGeo g = word_geo(w, C);
  const float th = g_atan2f(g.dy, g.dx);
  float t1 = 0.0f, q2 = 0.0f, ct1 = 0.0f, st1 = 0.0f, cq2 = 0.0f, sq2 = 0.0f;
  if (w == 1 || w == 2) {
    word_arcs(w, th, g_acosf(word_acos_arg(r, g)), &t1, &q2);
    ct1 = g_cosf(t1);
    st1 = g_sinf(t1);
    cq2 = g_cosf(q2);
    sq2 = g_sinf(q2);
  }
  return word_len(w, r, g, sh, gh, th, t1, ct1, st1, cq2, sq2, q);
}

// Dubins.cpp:19-69: shortest of the four words in RSR, RSL, LSR, LSL order (strict <).
__device__ __forceinline__ float dubins_shortest(float r, float sx, float sy, float sh, float gx, float gy, float gh,
                                                 int* word, float prm[4]) {
  const Centres C = dubins_centres(r, sx, sy, sh, gx, gy, gh);
  float best = 0.0f;
  for (int w = 0; w < 4; ++w) {
    float q[4];
    const float len = dubins_word(w, r, C, sh, gh, q);
    if (w == 0 || len < best) {
      best = len;
      *word = w;
      prm[0] = q[0];
      prm[1] = q[1];
      prm[2] = q[2];
      prm[3] = q[3];
    }
  }
  return best;
}

// ------------------------------------------------------------ wave helpers ----------
__device__ __forceinline__ float shfl_f(float v, int src) { return __shfl(v, src, 64); }
__device__ __forceinline__ int shfl_i(int v, int src) { return __shfl(v, src, 64); }
// lane L's value as a wave-uniform (scalar) value
__device__ __forceinline__ float rl_f(float v, int L) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), L));
}
__device__ __forceinline__ int rl_i(int v, int L) { return __builtin_amdgcn_readlane(v, L); }

// Dubins::get_shortest_path_length (Dubins.cpp:19-69) of every candidate successor of an
// expansion: candidate a's pose (sx, sy, sh) is held by all lanes of its group
// [a * gs, (a + 1) * gs); every lane of the group returns the candidate's length, the
// minimum of the four CSC words in RSR, RSL, LSR, LSL order (strict <).
//   gs = 16: the libm calls of one candidate are spread over its group — lanes 0/1 take
//            sin/cos of the heading, word lanes 0..3 atan2f/acosf, lanes 4..11 the cos/sin
//            of the RSL and LSR tangent angles — so the dependent chain is 4 calls long;
//   gs = 4:  lane w of the group evaluates word w alone.
// Lane L of each row of 16 lanes, to the whole row (DPP row_newbcast, a VALU move: no LDS
// round trip).  The caller runs it with every lane of the wave active: a DPP move reads
// `old` (here 0) from a source lane that is off in EXEC, where a ds_bpermute reads 0 too —
// both only give the row's value under a full mask.
template <int L>
__device__ __forceinline__ float row_bcast(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 | L, 0xf, 0xf, false));
}
// Lane L or M of each row, per lane (sel): both broadcasts are materialised before the select.
// Without the empty asm the compiler turns `sel ? bcast<L> : bcast<M>` into an if/else whose
// arms run the moves under a partial EXEC, where a source lane of the other arm reads as 0
// (the cause of the round-2 parity failure of this change: ISA inspection).
template <int L, int M>
__device__ __forceinline__ float row_bcast_sel(bool sel, float v) {
  float a = row_bcast<L>(v), b = row_bcast<M>(v);
  asm volatile("" : "+v"(a), "+v"(b));
  return sel ? a : b;
}

// Called with every lane active (the row broadcasts of the 16-lane case read other lanes).
__device__ __forceinline__ float cand_dubins(float r, const GoalC& GC, float gh, float sx, float sy, float sh, int gs,
                                            int lane) {
  const int base = lane & ~(gs - 1), sub = lane & (gs - 1), w = sub & 3;
  if (gs == 16) {  // a group is a DPP row
    const float t0 = g_sincosf_sel(sh, (sub & 1) != 0);
    float c0 = row_bcast<0>(t0), s0 = row_bcast<1>(t0);
    asm volatile("" : "+v"(c0), "+v"(s0));
    const Centres C = centres_from(r, sx, sy, c0, s0, GC);
    const WordGeo g = word_geo(w, C);
    const float th = g_atan2f(g.dy, g.dx);
    const float ac = g_acosf(word_acos_arg(r, g));  // used by RSL / LSR only
    float t1, q2;
    word_arcs(w == 2 ? 2 : 1, th, ac, &t1, &q2);
    // lanes 4..7: cos t1, sin t1, cos q2, sin q2 of RSL (word lane 1); lanes 8..11: of LSR
    // (word lane 2); every broadcast is taken by every lane, then selected
    const bool lsr = (sub >> 2) == 2;
    const float t1s = row_bcast_sel<2, 1>(lsr, t1);
    const float q2s = row_bcast_sel<2, 1>(lsr, q2);
    const float at = (sub & 3) < 2 ? t1s : q2s;
    const float tv = g_sincosf_sel(at, (sub & 1) == 0);
    const bool w2 = w == 2;
    const float c1 = row_bcast_sel<8, 4>(w2, tv), s1 = row_bcast_sel<9, 5>(w2, tv);
    const float c2 = row_bcast_sel<10, 6>(w2, tv), s2 = row_bcast_sel<11, 7>(w2, tv);
    float q[4];
    const float len = word_len(w, r, g, sh, gh, th, t1, c1, s1, c2, s2, q);
    float l0 = row_bcast<0>(len), l1 = row_bcast<1>(len), l2 = row_bcast<2>(len), l3 = row_bcast<3>(len);
    asm volatile("" : "+v"(l0), "+v"(l1), "+v"(l2), "+v"(l3));
    float best = l0;
    if (l1 < best) best = l1;
    if (l2 < best) best = l2;
    if (l3 < best) best = l3;
    return best;
  }
  float q[4];
  const float len = dubins_word(w, r, dubins_centres_g(r, sx, sy, sh, GC), sh, gh, q);
  float best = shfl_f(len, base);
  for (int w2 = 1; w2 < 4; ++w2) {
    const float v = shfl_f(len, base + w2);
    if (v < best) best = v;
  }
  return best;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)v, o, 64), hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

// Grid3D::get_field_intensity (Grid3D.cpp:206-227) for one pose, wave-parallel over the
// obstacle list.  Terms of obstacles farther than their radius are exactly +0.0f in
// the reference, so only in-radius terms are accumulated — in obstacle order, one at a
// time, exactly like std::accumulate.
// The first APF_LDS_CAP obstacles of a planner are staged in LDS for the whole search
// (loaded once); any further ones are read from HBM per call.
constexpr int APF_LDS_CAP = 256;
constexpr int APF_MAXC = 64;  // obstacles kept by the per-expansion cull (more: per-candidate fallback)
struct ApfCand { float x, y, r; };
struct ApfStage {
  ApfCand obs[APF_LDS_CAP];
  ApfCand kept[APF_MAXC];
};
__device__ __forceinline__ void apf_stage(const PlannerDev& P, ApfStage& S, int lane) {
  const GAS float* apf = gp(P.apf);
  const int n = P.n_apf < APF_LDS_CAP ? P.n_apf : APF_LDS_CAP;
  for (int k = lane; k < n; k += 64) S.obs[k] = ApfCand{apf[3 * k], apf[3 * k + 1], apf[3 * k + 2]};
  wave_lds_sync();
}
__device__ __forceinline__ ApfCand apf_obstacle(const PlannerDev& P, const ApfStage& S, int k) {
  if (k < APF_LDS_CAP) return S.obs[k];
  const GAS float* apf = gp(P.apf);
  return ApfCand{apf[3 * k], apf[3 * k + 1], apf[3 * k + 2]};
}

// the in-radius term of one obstacle (Grid3D.cpp:212-223), d = hypotf(dx, dy) < orad
__device__ __forceinline__ float apf_term(const PlannerDev& P, float dx, float dy, float d, float orad, float ph) {
  float ang = fabsf(wrap_pi_f(ph - g_atan2f(dy, dx)));
  ang = stl_max(P.apf_ang - ang, 0.0f);
  const double t = 1.0 / (double)d - 1.0 / (double)orad;
  float fp = (float)((double)P.apf_rep * (t * t));  // std::pow(t, 2) folded to t*t (GCC)
  fp = fp * ang / P.apf_ang;
  return fp;
}

__device__ __forceinline__ float apf_field(const PlannerDev& P, const ApfStage& S, float px, float py, float ph,
                                           int lane) {
  float acc = 0.0f;
  for (int base = 0; base < P.n_apf; base += 64) {
    const int k = base + lane;
    float term = 0.0f;
    bool near = false;
    const ApfCand o = apf_obstacle(P, S, k < P.n_apf ? k : 0);
    const float ox = o.x, oy = o.y, orad = o.r;
    const float dx = ox - px, dy = oy - py;
    // exact pre-test: the correctly rounded hypotf(dx, dy) >= max(|dx|, |dy|), so an
    // obstacle outside the axis-aligned square of half-width r cannot have d < r
    if (k < P.n_apf && fabsf(dx) < orad && fabsf(dy) < orad) {
      const float d = g_hypotf(dx, dy);
      if (d < orad) {
        near = true;
        term = apf_term(P, dx, dy, d, orad, ph);
      }
    }
    uint64_t m = __ballot(near);
    while (m) {
      const int b = __ffsll((unsigned long long)m) - 1;
      acc = acc + shfl_f(term, b);
      m &= m - 1;
    }
  }
  return acc;
}

// APF fields of all candidate successors of one expansion at once.  Candidate a of the
// window sits in lane a * gs (its pose in sx/sy/sh there); cmask has bit a * gs set for
// every candidate to evaluate; the result is in lane a * gs.  Every successor lies within
// P.apf_reach (per axis) of the expanded pose (cx, cy), so an obstacle whose square of
// half-width r + apf_reach around it misses (cx, cy) cannot pass the exact pre-test of any
// successor: the obstacle list is culled once, then lanes run over (candidate, kept
// obstacle) pairs, and every successor's in-radius terms are summed in obstacle order.
// kStageKept: the cull list is the stage's own (S.kept); else `kept_arg` (a helper wave's)
template <bool kStageKept>
__device__ __forceinline__ float apf_fused_t(const PlannerDev& P, ApfStage& S, ApfCand* kept_arg, float cx, float cy,
                                             float sx, float sy, float sh, uint64_t cmask, int gs, int lane) {
  ApfCand* __restrict__ kept = kStageKept ? S.kept : kept_arg;
  float fc = 0.0f;
  if (cmask == 0) return fc;
  int C = APF_MAXC + 1;
#ifdef HASTAR_DBG_APFOLD
  if (false) {
#else
  if (P.n_apf <= APF_LDS_CAP) {
#endif
    C = 0;
#pragma unroll
    for (int u = 0; u < APF_LDS_CAP / 64; ++u) {
      const ApfCand o = S.obs[64 * u + lane];
      const float lim = o.r + P.apf_reach;
      const bool in = 64 * u + lane < P.n_apf && fabsf(o.x - cx) < lim && fabsf(o.y - cy) < lim;
      const uint64_t bm = __ballot(in);
      const int pos = C + __popcll(bm & ((1ull << lane) - 1));
      if (in && pos < APF_MAXC) kept[pos] = o;
      C += __popcll(bm);
    }
    if (C == 0) return 0.0f;
  }
  if (C > APF_MAXC) {  // many obstacles near: one candidate at a time over the whole list
    for (uint64_t m = cmask; m; m &= m - 1) {
      const int L = __ffsll((unsigned long long)m) - 1;
      const float f = apf_field(P, S, uff(shfl_f(sx, L)), uff(shfl_f(sy, L)), uff(shfl_f(sh, L)), lane);
      if (lane == L) fc = f;
    }
    return fc;
  }
  wave_lds_sync();
  const int na = (63 - __builtin_clzll(cmask)) / gs + 1;  // candidates 0 .. na-1
  const int npair = na * C;
  for (int base = 0; base < npair; base += 64) {
    const int p = base + lane;
    const bool act = p < npair;
    const int a = act ? p / C : 0;
    const int j = act ? p - a * C : 0;
    const float px = shfl_f(sx, a * gs), py = shfl_f(sy, a * gs), ph = shfl_f(sh, a * gs);
    float term = 0.0f;
    bool near = false;
    if (act && ((cmask >> (a * gs)) & 1ull)) {
      const ApfCand o = kept[j];
      const float dx = o.x - px, dy = o.y - py;
      if (fabsf(dx) < o.r && fabsf(dy) < o.r) {
        const float d = g_hypotf(dx, dy);
        if (d < o.r) {
          near = true;
          term = apf_term(P, dx, dy, d, o.r, ph);
        }
      }
    }
    // pairs are candidate-major, obstacles ascending: lane order is summation order
    uint64_t m = __ballot(near);
    while (m) {
      const int b = __ffsll((unsigned long long)m) - 1;
      const float t = shfl_f(term, b);
      const int ab = __builtin_amdgcn_readlane(a, b);
      if (lane == ab * gs) fc = fc + t;
      m &= m - 1;
    }
  }
  wave_lds_sync();
  return fc;
}
__device__ __forceinline__ float apf_fused(const PlannerDev& P, ApfStage& S, float cx, float cy, float sx, float sy,
                                           float sh, uint64_t cmask, int gs, int lane) {
  return apf_fused_t<true>(P, S, nullptr, cx, cy, sx, sy, sh, cmask, gs, lane);
}
// the same with a cull buffer of the caller's (a helper wave of the latency kernel brings its own)
__device__ __forceinline__ float apf_fused_k(const PlannerDev& P, ApfStage& S, ApfCand* kept, float cx, float cy,
                                             float sx, float sy, float sh, uint64_t cmask, int gs, int lane) {
  return apf_fused_t<false>(P, S, kept, cx, cy, sx, sy, sh, cmask, gs, lane);
}

// Dubins.cpp:326-563 sampling of the chosen word, wave-parallel (64 samples per step).
// Angles and distances accumulate sequentially exactly like the reference loops; each
// lane keeps the value of its own sample index.  Returns the sample count or -1 when
// the scratch is too small.
// MODE 0: sample only.  MODE 1: also check every sample as Grid3D::check_path does
// (path_is_free's cell rule) chunk by chunk and return -2 at the first blocked chunk, so a failed
// shot stops early; a non-negative result then means the whole path is free.  MODE 2: count
// only (the scratch-size check of MODE 0, no samples written).
__device__ __forceinline__ bool sample_blocked(const PlannerDev& P, float x, float y) {
  const int ci = trunc_f(roundf(x / P.res));
  const int cj = trunc_f(roundf(y / P.res));
  return ci < 0 || ci >= P.N || cj < 0 || cj >= P.N || gp(P.occ)[(size_t)ci * P.N + cj] >= P.thr;
}
template <int MODE = 0>
__device__ inline int dubins_sample(const PlannerDev& P, const Centres& C, int word, const float prm[4], GAS float* xyh,
                                    GAS float* curv, int cap, int lane) {
  const float r = P.r_min, as = P.ang_step, st = P.step;
  const bool s_right = (word == 0 || word == 1), g_right = (word == 0 || word == 2);
  const float csx = s_right ? C.srx : C.slx, csy = s_right ? C.sry : C.sly;
  const float cgx = g_right ? C.grx : C.glx, cgy = g_right ? C.gry : C.gly;
  float ax = csx, ay = csy, bx = cgx, by = cgy;
  ax += r * g_cosf(prm[0] + prm[1]);
  ay += r * g_sinf(prm[0] + prm[1]);
  bx += r * g_cosf(prm[2]);
  by += r * g_sinf(prm[2]);
  const float ex = bx - ax, ey = by - ay;
  const float lst = sqrtf(ex * ex + ey * ey);
  const int n1 = trunc_f(floorf((s_right ? -prm[1] : prm[1]) / as));
  const int n2 = n1 + trunc_f(floorf(lst / st));
  const int n3 = n2 + trunc_f(floorf((g_right ? -prm[3] : prm[3]) / as));
  if (n1 < 0 || n2 < n1 || n3 < n2 || n3 + 1 > cap) return -1;
  if (MODE == 2) return n3 + 1;
  const float k = 1.0f / r;
  // first arc
  float th = prm[0];
  for (int base = 0; base < n1; base += 64) {
    float mine = 0.0f;
    for (int q = 0; q < 64 && base + q < n1; ++q) {
      if (lane == q) mine = th;
      th = s_right ? th - as : th + as;
    }
    const int i = base + lane;
    bool bad = false;
    if (i < n1) {
      const float x = csx + r * g_cosf(mine), y = csy + r * g_sinf(mine);
      xyh[3 * i] = x;
      xyh[3 * i + 1] = y;
      xyh[3 * i + 2] = (float)(s_right ? wrap_pi_d((double)mine - M_PI_2) : wrap_pi_d((double)mine + M_PI_2));
      curv[i] = k;
      if (MODE == 1) bad = sample_blocked(P, x, y);
    }
    if (MODE == 1 && __ballot(bad)) return -2;
  }
  // straight segment
  const float ts = g_atan2f(ey, ex);
  const float ct = g_cosf(ts), sn = g_sinf(ts);
  float dd = 0.0f;
  for (int base = n1; base < n2; base += 64) {
    float mine = 0.0f;
    for (int q = 0; q < 64 && base + q < n2; ++q) {
      if (lane == q) mine = dd;
      dd += st;
    }
    const int i = base + lane;
    bool bad = false;
    if (i < n2) {
      const float x = ax + mine * ct, y = ay + mine * sn;
      xyh[3 * i] = x;
      xyh[3 * i + 1] = y;
      xyh[3 * i + 2] = ts;
      curv[i] = 0.0f;
      if (MODE == 1) bad = sample_blocked(P, x, y);
    }
    if (MODE == 1 && __ballot(bad)) return -2;
  }
  // second arc
  th = prm[2];
  for (int base = n2; base < n3; base += 64) {
    float mine = 0.0f;
    for (int q = 0; q < 64 && base + q < n3; ++q) {
      if (lane == q) mine = th;
      th = g_right ? th - as : th + as;
    }
    const int i = base + lane;
    bool bad = false;
    if (i < n3) {
      const float x = cgx + r * g_cosf(mine), y = cgy + r * g_sinf(mine);
      xyh[3 * i] = x;
      xyh[3 * i + 1] = y;
      xyh[3 * i + 2] = (float)(g_right ? wrap_pi_d((double)mine - M_PI_2) : wrap_pi_d((double)mine + M_PI_2));
      curv[i] = k;
      if (MODE == 1) bad = sample_blocked(P, x, y);
    }
    if (MODE == 1 && __ballot(bad)) return -2;
  }
  bool bad = false;
  if (lane == 0) {
    const float e = prm[2] + prm[3];
    const float x = cgx + r * g_cosf(e), y = cgy + r * g_sinf(e);
    xyh[3 * n3] = x;
    xyh[3 * n3 + 1] = y;
    xyh[3 * n3 + 2] = (float)(g_right ? wrap_pi_d((double)e - M_PI_2) : wrap_pi_d((double)e + M_PI_2));
    curv[n3] = 0.0f;
    if (MODE == 1) bad = sample_blocked(P, x, y);
  }
  if (MODE == 1 && __ballot(bad)) return -2;
  return n3 + 1;
}

// Grid3D::check_path (Grid3D.cpp:78-93), wave-parallel.  Reads samples written by other
// lanes: caller must order (block barrier) before calling.
__device__ __forceinline__ bool path_is_free(const PlannerDev& P, const GAS float* xyh, int n, int lane) {
  bool bad = false;
  for (int i = lane; i < n; i += 64)
    if (sample_blocked(P, xyh[3 * i], xyh[3 * i + 1])) bad = true;
  return __ballot(bad) == 0;
}

}  // namespace hastar
