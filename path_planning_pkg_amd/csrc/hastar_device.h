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

// Dubins.cpp:19-32: circle centres of a start and a goal pose
__device__ __forceinline__ Centres dubins_centres(float r, float sx, float sy, float sh, float gx, float gy,
                                                  float gh) {
  Centres c;
  const float ss = g_sinf(sh), cs = g_cosf(sh), sg = g_sinf(gh), cg = g_cosf(gh);
  c.srx = sx + r * ss;
  c.sry = sy - r * cs;
  c.slx = sx - r * ss;
  c.sly = sy + r * cs;
  c.grx = gx + r * sg;
  c.gry = gy - r * cg;
  c.glx = gx - r * sg;
  c.gly = gy + r * cg;
  return c;
}

// Dubins.cpp:180-323 — length of CSC word w (0 RSR, 1 RSL, 2 LSR, 3 LSL) and its params.
__device__ __forceinline__ float dubins_word(int w, float r, const Centres& C, float sh, float gh, float q[4]) {
  const float csx = (w < 2) ? C.srx : C.slx, csy = (w < 2) ? C.sry : C.sly;
  const float cgx = (w == 0 || w == 2) ? C.grx : C.glx, cgy = (w == 0 || w == 2) ? C.gry : C.gly;
  const float dx = cgx - csx, dy = cgy - csy;
  if (w == 0 || w == 3) {
    const float th = g_atan2f(dy, dx);
    if (w == 0) {
      q[0] = (float)(M_PI_2 + (double)sh);
      const float t1 = (float)(M_PI_2 + (double)th);
      q[2] = t1;
      const float tg = (float)(M_PI_2 + (double)gh);
      q[1] = t1 - q[0];
      if (q[1] > 0) q[1] = (float)((double)q[1] - 2 * M_PI);
      q[3] = tg - q[2];
      if (q[3] > 0) q[3] = (float)((double)q[3] - 2 * M_PI);
    } else {
      q[0] = (float)(-M_PI_2 + (double)sh);
      const float t1 = (float)(-M_PI_2 + (double)th);
      q[2] = t1;
      const float tg = (float)(-M_PI_2 + (double)gh);
      q[1] = t1 - q[0];
      if (q[1] < 0) q[1] = (float)((double)q[1] + 2 * M_PI);
      q[3] = tg - q[2];
      if (q[3] < 0) q[3] = (float)((double)q[3] + 2 * M_PI);
    }
    const float dst = sqrtf(dx * dx + dy * dy);
    return (w == 0) ? dst + r * -(q[1] + q[3]) : dst + r * (q[1] + q[3]);
  }
  const float dist = sqrtf(dx * dx + dy * dy);
  const float th = g_atan2f(dy, dx);
  float t1;
  if (w == 1) {
    q[0] = (float)(M_PI_2 + (double)sh);
    t1 = g_acosf(2.0f * r / dist) + th;
    q[2] = (float)((double)t1 - M_PI);
    const float tg = (float)(-M_PI_2 + (double)gh);
    q[1] = t1 - q[0];
    if (q[1] > 0) q[1] = (float)((double)q[1] - 2 * M_PI);
    q[3] = tg - q[2];
    if (q[3] < 0) q[3] = (float)((double)q[3] + 2 * M_PI);
  } else {
    q[0] = (float)(-M_PI_2 + (double)sh);
    t1 = -g_acosf(2.0f * r / dist) + th;
    q[2] = (float)((double)t1 + M_PI);
    const float tg = (float)(M_PI_2 + (double)gh);
    q[1] = t1 - q[0];
    if (q[1] < 0) q[1] = (float)((double)q[1] + 2 * M_PI);
    q[3] = tg - q[2];
    if (q[3] > 0) q[3] = (float)((double)q[3] - 2 * M_PI);
  }
  float ax = csx, ay = csy, bx = cgx, by = cgy;
  ax += r * g_cosf(t1);
  ay += r * g_sinf(t1);
  bx += r * g_cosf(q[2]);
  by += r * g_sinf(q[2]);
  const float ex = bx - ax, ey = by - ay;
  const float dst = sqrtf(ex * ex + ey * ey);
  return (w == 1) ? dst + r * (-q[1] + q[3]) : dst + r * (q[1] - q[3]);
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
// The first APF_REG_ROUNDS x 64 obstacles of a planner are held in registers for the
// whole search (loaded once); any further ones are read from HBM per call.
constexpr int APF_REG_ROUNDS = 4;
struct ApfRegs {
  float ox[APF_REG_ROUNDS], oy[APF_REG_ROUNDS], orad[APF_REG_ROUNDS];
};
__device__ __forceinline__ void apf_load_regs(const PlannerDev& P, ApfRegs& R, int lane) {
  const GAS float* apf = gp(P.apf);
#pragma unroll
  for (int q = 0; q < APF_REG_ROUNDS; ++q) {
    const int k = 64 * q + lane;
    const bool in = k < P.n_apf;
    R.ox[q] = in ? apf[3 * k] : 0.0f;
    R.oy[q] = in ? apf[3 * k + 1] : 0.0f;
    R.orad[q] = in ? apf[3 * k + 2] : 0.0f;
  }
}

__device__ __forceinline__ float apf_field(const PlannerDev& P, const ApfRegs& R, float px, float py, float ph,
                                           int lane) {
  float acc = 0.0f;
  for (int base = 0, q = 0; base < P.n_apf; base += 64, ++q) {
    const int k = base + lane;
    float term = 0.0f;
    bool near = false;
    float ox, oy, orad;
    if (q < APF_REG_ROUNDS) {
      // static register index: select through the unrolled rounds
      ox = R.ox[0];
      oy = R.oy[0];
      orad = R.orad[0];
#pragma unroll
      for (int u = 1; u < APF_REG_ROUNDS; ++u)
        if (q == u) {
          ox = R.ox[u];
          oy = R.oy[u];
          orad = R.orad[u];
        }
    } else {
      const GAS float* apf = gp(P.apf);
      ox = k < P.n_apf ? apf[3 * k] : 0.0f;
      oy = k < P.n_apf ? apf[3 * k + 1] : 0.0f;
      orad = k < P.n_apf ? apf[3 * k + 2] : 0.0f;
    }
    const float dx = ox - px, dy = oy - py;
    // exact pre-test: the correctly rounded hypotf(dx, dy) >= max(|dx|, |dy|), so an
    // obstacle outside the axis-aligned square of half-width r cannot have d < r
    if (k < P.n_apf && fabsf(dx) < orad && fabsf(dy) < orad) {
      const float d = g_hypotf(dx, dy);
      if (d < orad) {
        near = true;
        float ang = fabsf(wrap_pi_f(ph - g_atan2f(dy, dx)));
        ang = stl_max(P.apf_ang - ang, 0.0f);
        const double t = 1.0 / (double)d - 1.0 / (double)orad;
        float fp = (float)((double)P.apf_rep * (t * t));  // std::pow(t, 2) folded to t*t (GCC)
        fp = fp * ang / P.apf_ang;
        term = fp;
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

// Dubins.cpp:326-563 sampling of the chosen word, wave-parallel (64 samples per step).
// Angles and distances accumulate sequentially exactly like the reference loops; each
// lane keeps the value of its own sample index.  Returns the sample count or -1 when
// the scratch is too small.
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
    if (i < n1) {
      xyh[3 * i] = csx + r * g_cosf(mine);
      xyh[3 * i + 1] = csy + r * g_sinf(mine);
      xyh[3 * i + 2] = (float)(s_right ? wrap_pi_d((double)mine - M_PI_2) : wrap_pi_d((double)mine + M_PI_2));
      curv[i] = k;
    }
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
    if (i < n2) {
      xyh[3 * i] = ax + mine * ct;
      xyh[3 * i + 1] = ay + mine * sn;
      xyh[3 * i + 2] = ts;
      curv[i] = 0.0f;
    }
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
    if (i < n3) {
      xyh[3 * i] = cgx + r * g_cosf(mine);
      xyh[3 * i + 1] = cgy + r * g_sinf(mine);
      xyh[3 * i + 2] = (float)(g_right ? wrap_pi_d((double)mine - M_PI_2) : wrap_pi_d((double)mine + M_PI_2));
      curv[i] = k;
    }
  }
  if (lane == 0) {
    const float e = prm[2] + prm[3];
    xyh[3 * n3] = cgx + r * g_cosf(e);
    xyh[3 * n3 + 1] = cgy + r * g_sinf(e);
    xyh[3 * n3 + 2] = (float)(g_right ? wrap_pi_d((double)e - M_PI_2) : wrap_pi_d((double)e + M_PI_2));
    curv[n3] = 0.0f;
  }
  return n3 + 1;
}

// Grid3D::check_path (Grid3D.cpp:78-93), wave-parallel.  Reads samples written by other
// lanes: caller must order (block barrier) before calling.
__device__ __forceinline__ bool path_is_free(const PlannerDev& P, const GAS float* xyh, int n, int lane) {
  bool bad = false;
  for (int i = lane; i < n; i += 64) {
    const int ci = trunc_f(roundf(xyh[3 * i] / P.res));
    const int cj = trunc_f(roundf(xyh[3 * i + 1] / P.res));
    if (ci < 0 || ci >= P.N || cj < 0 || cj >= P.N || gp(P.occ)[(size_t)ci * P.N + cj] >= P.thr) bad = true;
  }
  return __ballot(bad) == 0;
}

}  // namespace hastar
