// hastar_rs.h — Reeds-Shepp shortest paths on the device, for the RELAXED mode's optional
// reversing motion model (hastar_relaxed_opts::reverse_cost > 0).  NOT part of the exact mode:
// the reference's vehicle model drives forward only (VehicleModel.cpp:97-101) and its analytic
// expansion is forward CSC Dubins (Dubins.h:13-19), so nothing here has a reference to match
// bit for bit ("parity unpinned"; BASELINE.json configs[2] asks for Reeds-Shepp reversals).
//
// The algorithm is the published one (Reeds & Shepp 1990, formulas 8.1-8.11: the families CSC,
// CCC, CCCC, CCSC and CCSCC under the time-flip / reflection / backwards symmetries, 44
// candidates over 18 words).  oracle/reeds_shepp.py restates it in double precision and is
// the checker (tests/test_reeds_shepp.py): every candidate the device returns must integrate to
// the goal, and the device's shortest length must equal the restatement's to float precision.
//
// Wave mapping: a candidate is (family group g in 0..10, symmetry s in 0..3).  For the
// heuristic of a successor group of gs >= 4 lanes, lane sub of the group takes symmetry sub & 3
// and the groups g = sub >> 2, sub >> 2 + gs / 4, ...; a shuffle reduction takes the minimum.
// For a shot, lanes 0..43 take one candidate each and the shortest wins (rs_best).
#pragma once
#include <hip/hip_runtime.h>

namespace hastar {

constexpr float RS_ZERO = 1e-5f;  // slack of the family conditions, in turning radii (float)
constexpr float RS_INF = 3.0e38f;
enum : int { RS_L = 1, RS_S = 0, RS_R = -1, RS_N = 2 };

// the 18 words' segment kinds (oracle/reeds_shepp.py WORDS), five 2-bit codes per word:
// code 0 straight, 1 left, 2 right, 3 none
__device__ __forceinline__ int rs_kind(int word, int k) {
  // six 10-bit words per 64-bit constant (selected, not indexed: no table in memory)
  const int q = word / 6;
  const unsigned long long W = q == 0 ? 0xe1b49d9b99f9bd9ull : q == 1 ? 0xe4762d1b89e4b61ull : 0x61a49f8bd1f4be1ull;
  const unsigned c = (unsigned)(W >> (10 * (word - 6 * q) + 2 * k)) & 3u;
  return c == 0 ? RS_S : c == 1 ? RS_L : c == 2 ? RS_R : RS_N;
}

__device__ __forceinline__ float rs_mod2pi(float x) {
  const float TWO_PI = 6.28318530717958648f, PI = 3.14159265358979324f;
  float v = fmodf(x, TWO_PI);
  if (v < -PI) v += TWO_PI;
  else if (v > PI) v -= TWO_PI;
  return v;
}

// one candidate: family group g (0..10) under symmetry s (0 identity, 1 time-flip, 2 reflection,
// 3 both) for the goal (x, y, phi) in the start's frame, radius units.  Returns the length
// (RS_INF when the family has no solution) with the word and its signed segment lengths.
__device__ inline float rs_candidate(int g, int s, float x, float y, float phi, int* word, float seg[5]) {
  const float PI = 3.14159265358979324f, HP = 1.57079632679489662f;
  const bool back = g == 3 || g == 8 || g == 9;
  float xx = x, yy = y;
  if (back) {  // the backwards symmetry: the goal seen from the goal, driven in reverse order
    const float c = cosf(phi), sn = sinf(phi);
    xx = x * c + y * sn;
    yy = x * sn - y * c;
  }
  const float X = (s & 1) ? -xx : xx, Y = (s & 2) ? -yy : yy, F = (s == 1 || s == 2) ? -phi : phi;
  const float sg = (s & 1) ? -1.0f : 1.0f;
  const int refl = s >> 1;
  float t = 0.0f, u = 0.0f, v = 0.0f;
  bool ok = false;
  const float sF = sinf(F), cF = cosf(F);
  switch (g) {
    case 0: {  // 8.1 L+S+L+
      const float a = X - sF, b = Y - 1.0f + cF;
      u = sqrtf(a * a + b * b);
      t = atan2f(b, a);
      if (t >= -RS_ZERO) {
        v = rs_mod2pi(F - t);
        ok = v >= -RS_ZERO;
      }
      break;
    }
    case 1: {  // 8.2 L+S+R+
      const float a = X + sF, b = Y - 1.0f - cF;
      const float u1 = a * a + b * b, t1 = atan2f(b, a);
      if (u1 >= 4.0f) {
        u = sqrtf(u1 - 4.0f);
        t = rs_mod2pi(t1 + atan2f(2.0f, u));
        v = rs_mod2pi(t - F);
        ok = t >= -RS_ZERO && v >= -RS_ZERO;
      }
      break;
    }
    case 2:
    case 3: {  // 8.3 / 8.4 L+R-L
      const float xi = X - sF, eta = Y - 1.0f + cF;
      const float u1 = sqrtf(xi * xi + eta * eta), th = atan2f(eta, xi);
      if (u1 <= 4.0f) {
        u = -2.0f * asinf(0.25f * u1);
        t = rs_mod2pi(th + 0.5f * u + PI);
        v = rs_mod2pi(F - t + u);
        ok = t >= -RS_ZERO && u <= RS_ZERO;
      }
      break;
    }
    case 4:
    case 5: {  // 8.7 L+R+L-R-, 8.8 L+R-L-R+
      const float xi = X + sF, eta = Y - 1.0f - cF;
      float uu = 0.0f;
      bool pre = false;
      if (g == 4) {
        const float rho = 0.25f * (2.0f + sqrtf(xi * xi + eta * eta));
        if (rho <= 1.0f) {
          uu = acosf(rho);
          pre = true;
        }
      } else {
        const float rho = (20.0f - xi * xi - eta * eta) / 16.0f;
        if (rho >= 0.0f && rho <= 1.0f) {
          uu = -acosf(rho);
          pre = uu >= -HP;
        }
      }
      if (pre) {
        const float vv = g == 4 ? -uu : uu;
        const float delta = rs_mod2pi(uu - vv);
        const float A = sinf(uu) - sinf(delta), B = cosf(uu) - cosf(delta) - 1.0f;
        const float t1 = atan2f(eta * A - xi * B, xi * A + eta * B);
        const float t2 = 2.0f * (cosf(delta) - cosf(vv) - cosf(uu)) + 3.0f;
        t = t2 < 0.0f ? rs_mod2pi(t1 + PI) : rs_mod2pi(t1);
        v = rs_mod2pi(t - uu + vv - F);
        u = uu;
        ok = t >= -RS_ZERO && (g == 4 ? v <= RS_ZERO : v >= -RS_ZERO);
      }
      break;
    }
    case 6:
    case 8: {  // 8.9 L+R-S-L-
      const float xi = X - sF, eta = Y - 1.0f + cF;
      const float rho = sqrtf(xi * xi + eta * eta), th = atan2f(eta, xi);
      if (rho >= 2.0f) {
        const float r = sqrtf(rho * rho - 4.0f);
        u = 2.0f - r;
        t = rs_mod2pi(th + atan2f(r, -2.0f));
        v = rs_mod2pi(F - HP - t);
        ok = t >= -RS_ZERO && u <= RS_ZERO && v <= RS_ZERO;
      }
      break;
    }
    case 7:
    case 9: {  // 8.10 L+R-S-R-
      const float xi = X + sF, eta = Y - 1.0f - cF;
      const float rho = sqrtf(xi * xi + eta * eta), th = atan2f(xi, -eta);
      if (rho >= 2.0f) {
        t = th;
        u = 2.0f - rho;
        v = rs_mod2pi(t + HP - F);
        ok = t >= -RS_ZERO && u <= RS_ZERO && v <= RS_ZERO;
      }
      break;
    }
    default: {  // 10: 8.11 L+R-S-L-R+
      const float xi = X + sF, eta = Y - 1.0f - cF;
      const float rho = sqrtf(xi * xi + eta * eta);
      if (rho >= 2.0f) {
        u = 4.0f - sqrtf(rho * rho - 4.0f);
        if (u <= RS_ZERO) {
          t = rs_mod2pi(atan2f((4.0f - u) * xi - 2.0f * eta, -2.0f * xi + (u - 4.0f) * eta));
          v = rs_mod2pi(t - F);
          ok = t >= -RS_ZERO && v >= -RS_ZERO;
        }
      }
      break;
    }
  }
  if (!ok) return RS_INF;
  float a0 = t, a1 = u, a2 = v, a3 = 0.0f, a4 = 0.0f;
  int w;
  switch (g) {
    case 0: w = 14; break;
    case 1: w = 12; break;
    case 2: w = 0; break;
    case 3: w = 0; a0 = v; a2 = t; break;
    case 4: w = 2; a2 = -u; a3 = v; break;
    case 5: w = 2; a2 = u; a3 = v; break;
    case 6: w = 4; a1 = -HP; a2 = u; a3 = v; break;
    case 7: w = 8; a1 = -HP; a2 = u; a3 = v; break;
    case 8: w = 6; a0 = v; a1 = u; a2 = -HP; a3 = t; break;
    case 9: w = 10; a0 = v; a1 = u; a2 = -HP; a3 = t; break;
    default: w = 16; a1 = -HP; a2 = u; a3 = -HP; a4 = v; break;
  }
  *word = w + refl;
  seg[0] = sg * a0;
  seg[1] = sg * a1;
  seg[2] = sg * a2;
  seg[3] = sg * a3;
  seg[4] = sg * a4;
  return fabsf(a0) + fabsf(a1) + fabsf(a2) + fabsf(a3) + fabsf(a4);
}

// the goal pose in the frame of (sx, sy, sh), in units of r
__device__ __forceinline__ void rs_local(float r, float sx, float sy, float sh, float gx, float gy, float gh, float* x,
                                         float* y, float* phi) {
  const float dx = gx - sx, dy = gy - sy, c = cosf(sh), s = sinf(sh);
  *x = (c * dx + s * dy) / r;
  *y = (-s * dx + c * dy) / r;
  *phi = gh - sh;
}

// shortest length (metres) from each lane group's pose to the goal; groups of gs >= 4 aligned
// lanes share one pose (see the header comment)
__device__ inline float rs_length_group(float r, float sx, float sy, float sh, float gx, float gy, float gh, int gs,
                                        int lane) {
  float x, y, phi;
  rs_local(r, sx, sy, sh, gx, gy, gh, &x, &y, &phi);
  const int sub = lane & (gs - 1), s = sub & 3;
  float best = RS_INF;
  int w;
  float seg[5];
  for (int g = sub >> 2; g < 11; g += gs >> 2) best = fminf(best, rs_candidate(g, s, x, y, phi, &w, seg));
  for (int m = 1; m < gs; m <<= 1) best = fminf(best, __shfl_xor(best, m, 64));
  return best * r;
}

struct RSPath {
  float L;  // radius units
  int word;
  float seg[5];
};
// the shortest path from (sx, sy, sh) to the goal, wave-wide (every lane gets it); L = RS_INF
// when no candidate exists (not expected: some family always solves)
__device__ inline RSPath rs_best(float r, float sx, float sy, float sh, float gx, float gy, float gh, int lane) {
  float x, y, phi;
  rs_local(r, sx, sy, sh, gx, gy, gh, &x, &y, &phi);
  RSPath p;
  p.L = RS_INF;
  p.word = 0;
  for (int k = 0; k < 5; ++k) p.seg[k] = 0.0f;
  if (lane < 44) p.L = rs_candidate(lane >> 2, lane & 3, x, y, phi, &p.word, p.seg);
  unsigned long long key = ((unsigned long long)__float_as_uint(p.L) << 32) | (unsigned)lane;
  for (int m = 32; m >= 1; m >>= 1) {
    const unsigned long long o = __shfl_xor(key, m, 64);
    key = o < key ? o : key;
  }
  const int win = (int)(key & 63u);
  RSPath q;
  q.L = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.L), win));
  q.word = __builtin_amdgcn_readlane(p.word, win);
  for (int k = 0; k < 5; ++k) q.seg[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.seg[k]), win));
  return q;
}

// pose at signed arc a (radius units) along a segment of kind `kind` from (x, y, h), radius r
__device__ __forceinline__ void rs_step(int kind, float r, float x, float y, float h, float a, float* ox, float* oy,
                                        float* oh) {
  if (kind == RS_L) {
    *ox = x + r * (sinf(h + a) - sinf(h));
    *oy = y + r * (cosf(h) - cosf(h + a));
    *oh = h + a;
  } else if (kind == RS_R) {
    *ox = x + r * (sinf(h) - sinf(h - a));
    *oy = y + r * (cosf(h - a) - cosf(h));
    *oh = h - a;
  } else {
    *ox = x + r * a * cosf(h);
    *oy = y + r * a * sinf(h);
    *oh = h;
  }
}

}  // namespace hastar
