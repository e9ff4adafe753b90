// glibc_mathf.h — bit-faithful host+device ports of the glibc 2.35 (x86-64)
// float transcendental routines that the reference planner reaches through
// std::sin/std::cos/std::atan2/std::acos/std::hypot on float arguments.
//
// Why this exists: the reference (lib/*.cpp, T = float) calls glibc libm.  glibc's
// float routines are NOT correctly rounded (atan2f mismatches the correctly rounded
// value on ~16 % of inputs, acosf ~8 %, sinf/cosf ~1 %), and sinf/cosf are IFUNC
// dispatched — on an FMA+AVX2 host the `__sinf_fma`/`__cosf_fma` variants run.  A GPU
// search that must reproduce the reference's closed set bit-for-bit therefore needs
// these exact algorithms, with exactly the same roundings and the same fused
// multiply-adds, on gfx950.
//
// Provenance (algorithm + constants):
//   * g_sinf / g_cosf : optimized-routines sinf/cosf as shipped in glibc 2.35
//     (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h), FMA build
//     (sysdeps/x86_64/fpu/multiarch/s_sinf-fma.c).  Every fma() below corresponds to
//     one vfmadd/vfnmadd in the container's libm.so.6 (__sinf_fma at 0x7b2b0,
//     __cosf_fma at 0x7b4f0); the table values are the `__sincosf_table` /
//     `__inv_pio4` contents read from that binary.
//   * g_atan2f / g_atanf : fdlibm e_atan2f.c / s_atanf.c (glibc 2.35, plain SSE2 build,
//     no contraction).  Evaluation order follows the binary (__atan2f_finite 0x38be0,
//     atanf 0x3e080).
//   * g_acosf : fdlibm e_acosf.c (glibc 2.35, __acosf_finite 0x385c0).
//   * g_hypotf : glibc 2.35 sysdeps/ieee754/flt-32/e_hypotf.c (new GLIBC_2.35 symbol):
//     (float)sqrt((double)x*x + (double)y*y) for finite inputs.
// Validation: tests/test_mathf_ports.py compares every port against the live glibc
// of the container (exhaustive over the float ranges the planner reaches, plus
// random full-range samples); tools/mathf_exhaustive.cpp is the full 2^32 sweep.
//
// Compile with -ffp-contract=off on both host (g++) and device (hipcc): every
// multiply-add below that is NOT written as fma() must stay unfused.
#pragma once

#include <stdint.h>
#include <string.h>
#include <math.h>

#if defined(__HIPCC__)
#define GM_HD __host__ __device__ __forceinline__
#else
#define GM_HD static inline
#endif

namespace gmath {

GM_HD uint32_t fbits(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
GM_HD float bitsf(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }
GM_HD uint64_t dbits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
GM_HD double bitsd(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

// ---------------------------------------------------------------- sinf / cosf --
// glibc's sincos_t (sincosf.h) comes in two copies: the sine coefficients are identical,
// copy 1 negates every cosine coefficient, and sign[4] = {1, -1, -1, 1}.  fma() and the
// double -> float conversion round symmetrically, so the copy-1 cosine polynomial is
// exactly the negated copy-0 one, and sign[] only negates x (exact).  The polynomials
// below therefore take the copy-0 constants as immediates and never index a table (a
// per-lane table index would be a vector memory load on the GPU).
//   copy 0: hpi_inv 0x1.45f306dc9c883p+23, hpi 0x1.921fb54442d18p+0, c0 1, c1 -0x1.ffffffd0c621cp-2,
//   s1 -0x1.555545995a603p-3, c2 0x1.55553e1068f19p-5, s2 0x1.1107605230bc4p-7,
//   c3 -0x1.6c087e89a359dp-10, s3 -0x1.994eb3774cf24p-13, c4 0x1.99343027bf8c3p-16.
#define GM_INV_PIO4_INIT                                                                        \
  {0xa2u, 0xa2f9u, 0xa2f983u, 0xa2f9836eu, 0xf9836e4eu, 0x836e4e44u, 0x6e4e4415u, 0x4e441529u,  \
   0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u, 0x2757d1f5u, 0x57d1f534u, 0xd1f534ddu,    \
   0xf534ddc0u, 0x34ddc0dbu, 0xddc0db62u, 0xc0db6295u, 0xdb629599u, 0x6295993cu, 0x95993c43u,    \
   0x993c4390u, 0x3c439041u}

static const uint32_t kInvPio4Host[24] = GM_INV_PIO4_INIT;
#if defined(__HIPCC__)
__constant__ uint32_t kInvPio4Dev[24] = GM_INV_PIO4_INIT;
#endif

GM_HD uint32_t inv_pio4(int i) {
#if defined(__HIP_DEVICE_COMPILE__)
  return kInvPio4Dev[i];
#else
  return kInvPio4Host[i];
#endif
}

GM_HD uint32_t abstop12(float x) { return (fbits(x) >> 20) & 0x7ffu; }

// sinf_poly() with the FMA grouping of the -mfma build: odd (n even: sine) or even
// (n odd: cosine) polynomial; tab1 selects copy 1 of the table.
GM_HD float sincos_poly_t(double x, double x2, bool tab1, int n) {
  // both polynomials, selected (lanes of a wave may need different ones)
  const double x3 = x * x2;
  const double s1 = fma(x2, -0x1.994eb3774cf24p-13, 0x1.1107605230bc4p-7);
  const double x7 = x3 * x2;
  const double sp = fma(x3, -0x1.555545995a603p-3, x);
  const float vs = (float)fma(s1, x7, sp);
  const double x4 = x2 * x2;
  const double c1 = fma(x2, -0x1.ffffffd0c621cp-2, 0x1.0p+0);
  const double c2 = fma(x2, 0x1.99343027bf8c3p-16, -0x1.6c087e89a359dp-10);
  const double x6 = x4 * x2;
  const double c = fma(x4, 0x1.55553e1068f19p-5, c1);
  const float vc = (float)fma(c2, x6, c);
  if ((n & 1) == 0) return vs;
  return tab1 ? -vc : vc;
}

// reduce_large(): Payne-Hanek style reduction for |y| >= 120, 64-bit integer exact.
GM_HD double reduce_large(uint32_t xi, int* np) {
  int idx = (int)((xi >> 26) & 15u);
  int shift = (int)((xi >> 23) & 7u);
  uint32_t m = ((xi & 0xffffffu) | 0x800000u) << shift;
  uint64_t res0 = (uint32_t)(m * inv_pio4(idx));
  uint64_t res1 = (uint64_t)m * inv_pio4(idx + 4);
  uint64_t res2 = (uint64_t)m * inv_pio4(idx + 8);
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  uint64_t n = (res0 + (1ull << 61)) >> 62;
  res0 -= n << 62;
  *np = (int)n;
  return (double)(int64_t)res0 * 0x1.921fb54442d18p-62;
}

GM_HD float nan_of(float y) { return (y - y) / (y - y); }

// sinf(y) (cosine = false) or cosf(y) (cosine = true): one code path for both, so a
// wavefront whose lanes need different functions evaluates them in a single pass.
// sinf and cosf differ only in the |y| < 2^-12 result and in which polynomial an odd
// quadrant takes.
GM_HD float g_sincosf_sel(float y, bool cosine) {
  // |y| < 0.75 (glibc's small-argument path) is the |y| < 120 path with n = 0: the
  // reduction x - 0 * hpi is exact and the quadrant logic picks the same polynomial, so
  // both run as one branch-free sequence (no divergence between the lanes of a wave).
  const double x = y;
  const uint32_t t = abstop12(y);
  if (t >= 0x42fu) {  // |y| >= 120, inf, nan (the planner never gets here)
    if (t >= 0x7f8u) return nan_of(y);
    const uint32_t xi = fbits(y);
    int n;
    const double xr = reduce_large(xi, &n);
    const int ns = n + (int)(xi >> 31);
    const double x2 = xr * xr;
    const bool tab1 = (ns & 2) != 0;
    if (cosine ? ((n ^ 1) & 1) : (n & 1)) return sincos_poly_t(xr, x2, tab1, 1);
    return sincos_poly_t(((ns + 1) & 2) ? -xr : xr, x2, tab1, 0);
  }
  const double r = x * 0x1.45f306dc9c883p+23;
  const int n = (((int32_t)r) + 0x800000) >> 24;
  const double xr = fma(-(double)n, 0x1.921fb54442d18p+0, x);  // vfnmadd: x - n*hpi, one rounding
  const double x2 = xr * xr;
  const bool odd = cosine ? ((n ^ 1) & 1) : (n & 1);
  const float v = sincos_poly_t(odd ? xr : (((n + 1) & 2) ? -xr : xr), x2, (n & 2) != 0, odd ? 1 : 0);
  if (t < 0x398u) return cosine ? 1.0f : y;  // |y| < 2^-12
  return v;
}
GM_HD float g_sinf(float y) { return g_sincosf_sel(y, false); }
GM_HD float g_cosf(float y) { return g_sincosf_sel(y, true); }

// ---------------------------------------------------------------- atanf -------
// The argument-reduction cases are selected, not branched, so lanes in different ranges
// share one instruction stream; each case computes exactly the fdlibm expression.
GM_HD float g_atanf(float x) {
  const int32_t hx = (int32_t)fbits(x);
  const int32_t ix = hx & 0x7fffffff;
  if (ix >= 0x4c000000) {                         // |x| >= 2^25
    if (ix > 0x7f800000) return x + x;
    if (hx > 0) return bitsf(0x33a22168u) + bitsf(0x3fc90fdau);
    return bitsf(0xbfc90fdau) - bitsf(0x33a22168u);
  }
  const bool small = ix < 0x3ee00000;             // |x| < 0.4375: id = -1
  const float ax = fabsf(x);
  // id 0: 7/16 <= |x| < 11/16, 1: < 19/16, 2: < 2.4375, 3: >= 2.4375
  const int id = ix < 0x3f300000 ? 0 : (ix < 0x3f980000 ? 1 : (ix < 0x401c0000 ? 2 : 3));
  const float num = id == 0 ? ax + ax - 1.0f : (id == 1 ? ax - 1.0f : (id == 2 ? ax - 1.5f : -1.0f));
  const float den = id == 0 ? ax + 2.0f : (id == 1 ? ax + 1.0f : (id == 2 ? ax * 1.5f + 1.0f : ax));
  const float hi = bitsf(id == 0 ? 0x3eed6338u : (id == 1 ? 0x3f490fdau : (id == 2 ? 0x3f7b985eu : 0x3fc90fdau)));
  const float lo = bitsf(id == 0 ? 0x31ac3769u : (id == 1 ? 0x33222168u : (id == 2 ? 0x33140fb4u : 0x33a22168u)));
  const float xr = small ? x : num / den;
  const float z = xr * xr;
  const float w = z * z;
  float s1 = bitsf(0x3c8569d7u) * w + bitsf(0x3d4bda59u);
  s1 = s1 * w + bitsf(0x3d886b35u);
  s1 = s1 * w + bitsf(0x3dba2e6eu);
  s1 = s1 * w + bitsf(0x3e124925u);
  s1 = s1 * w + bitsf(0x3eaaaaabu);
  s1 = s1 * z;
  float s2 = bitsf(0xbd15a221u) * w - bitsf(0x3d6ef16bu);
  s2 = s2 * w - bitsf(0x3d9d8795u);
  s2 = s2 * w - bitsf(0x3de38e38u);
  s2 = s2 * w - bitsf(0x3e4ccccdu);
  s2 = s2 * w;
  const float t = (s1 + s2) * xr;
  const float r = hi - ((t - lo) - xr);
  if (ix < 0x31000000) return x;                  // |x| < 2^-29 (huge + x > 1 always)
  if (small) return xr - t;
  return (hx < 0) ? -r : r;
}

// ---------------------------------------------------------------- atan2f ------
GM_HD float g_atan2f(float y, float x) {
  const float tiny = bitsf(0x0da24260u);      // 1.0e-30
  const float pi = bitsf(0x40490fdbu), npi = bitsf(0xc0490fdbu);
  const float pio2 = bitsf(0x3fc90fdbu), npio2 = bitsf(0xbfc90fdbu);
  const float pio4 = bitsf(0x3f490fdbu), npio4 = bitsf(0xbf490fdbu);
  const float mpi_lo = bitsf(0x33bbbd2eu);    // -pi_lo
  const uint32_t hx = fbits(x), hy = fbits(y);
  const uint32_t ix = hx & 0x7fffffffu, iy = hy & 0x7fffffffu;
  if (ix > 0x7f800000u || iy > 0x7f800000u) return x + y;
  if (hx == 0x3f800000u) return g_atanf(y);
  const int m = (int)(((hy >> 31) & 1u) | ((hx >> 30) & 2u));
  if (iy == 0) {
    if (m == 2) return tiny + pi;
    if (m == 3) return npi - tiny;
    return y;
  }
  if (ix == 0) return ((int32_t)hy < 0) ? npio2 - tiny : tiny + pio2;
  if (ix == 0x7f800000u) {
    if (iy == 0x7f800000u) {
      if (m == 0) return tiny + pio4;
      if (m == 1) return npio4 - tiny;
      if (m == 2) return 3.0f * pio4 + tiny;
      return -3.0f * pio4 - tiny;
    }
    if (m == 0) return 0.0f;
    if (m == 1) return -0.0f;
    if (m == 2) return tiny + pi;
    return npi - tiny;
  }
  if (iy == 0x7f800000u) return ((int32_t)hy < 0) ? npio2 - tiny : tiny + pio2;
  const int32_t dk = (int32_t)iy - (int32_t)ix;
  const int32_t k = dk >> 23;
  const float za = g_atanf(fabsf(y / x));
  const float z = dk > 0x1e7fffff ? pio2 - bitsf(0x333bbd2eu)       // pi_o_2 + 0.5*pi_lo
                  : (((int32_t)hx < 0 && k < -60) ? 0.0f : za);
  const float r1 = bitsf(fbits(z) ^ 0x80000000u);
  const float r2 = pi - (mpi_lo + z);
  const float r3 = (z + mpi_lo) - pi;
  return m == 0 ? z : (m == 1 ? r1 : (m == 2 ? r2 : r3));
}

// ---------------------------------------------------------------- acosf -------
// The three argument ranges share one instruction stream (one rational approximation,
// one sqrt, the final expression selected); each range computes exactly fdlibm's value.
GM_HD float g_acosf(float x) {
  const float pio2_hi = bitsf(0x3fc90fdau), pio2_lo = bitsf(0x33a22168u);
  const float pi = bitsf(0x40490fdau);
  const int32_t hx = (int32_t)fbits(x);
  const int32_t ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) {
    if (hx > 0) return 0.0f;
    return bitsf(0x34222168u) + pi;                // pi + 2*pio2_lo
  }
  if (ix > 0x3f800000) return (x - x) / (x - x);
  const bool mid = ix < 0x3f000000;                // |x| < 0.5
  const bool neg = hx < 0;                         // x <= -0.5 (when !mid)
  const float z = mid ? x * x : (neg ? (x + 1.0f) * 0.5f : (1.0f - x) * 0.5f);
  float p = bitsf(0x3811ef08u) * z + bitsf(0x3a4f7f04u);
  p = p * z - bitsf(0x3d241146u);
  p = p * z + bitsf(0x3e4e0aa8u);
  p = p * z - bitsf(0x3ea6b090u);
  p = p * z + bitsf(0x3e2aaaabu);
  p = p * z;
  float q = bitsf(0x3d9dc62eu) * z - bitsf(0x3f303361u);
  q = q * z + bitsf(0x4001572du);
  q = q * z - bitsf(0x4019d139u);
  q = q * z + 1.0f;
  const float r = p / q;
  const float s = sqrtf(z);
  const float df = bitsf(fbits(s) & 0xfffff000u);
  const float c = (z - df * df) / (s + df);
  const float v_mid = pio2_hi - (x - (pio2_lo - r * x));
  const float v_neg = pi - (s + (r * s - pio2_lo)) * 2.0f;
  const float v_pos = (df + (r * s + c)) * 2.0f;
  if (mid && ix <= 0x32800000) return pio2_lo + pio2_hi;
  return mid ? v_mid : (neg ? v_neg : v_pos);
}

// ---------------------------------------------------------------- hypotf ------
GM_HD float g_hypotf(float x, float y) {
  const uint32_t ax = fbits(x) & 0x7fffffffu, ay = fbits(y) & 0x7fffffffu;
  if (ax >= 0x7f800000u || ay >= 0x7f800000u) {
    const bool xsig = ax > 0x7f800000u && !(ax & 0x400000u);
    const bool ysig = ay > 0x7f800000u && !(ay & 0x400000u);
    if ((ax == 0x7f800000u && !ysig) || (ay == 0x7f800000u && !xsig)) return bitsf(0x7f800000u);
    return x + y;
  }
  const double dx = x, dy = y;
  return (float)sqrt(dx * dx + dy * dy);
}

// ---------------------------------------------------------------- helpers -----
// std::fmod(a, 2*M_PI) for the reference's wrap_pi (common.h:15-29).  fmod is exact;
// the two short cases are exact by Sterbenz, the rest goes to the libm fmod.
GM_HD double fmod_2pi(double a) {
  const double c = 2.0 * M_PI;
  const double aa = fabs(a);
  if (!(aa >= c)) return a;                        // also NaN
  if (aa < 2.0 * c) return copysign(aa - c, a);
  return fmod(a, c);
}

// static_cast<int>(float/double) with x86-64 cvtt* semantics: NaN and out-of-range
// values become INT_MIN (gfx950's v_cvt_i32 would saturate / map NaN to 0).
GM_HD int x86_trunc_int(double v) {
  if (!(v > -2147483649.0 && v < 2147483648.0)) return (int)0x80000000u;
  return (int)v;
}

}  // namespace gmath
