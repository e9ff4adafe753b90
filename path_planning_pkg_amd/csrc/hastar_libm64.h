// hastar_libm64.h — the f64 libm of the double planner's device code (hastar_f64.hip,
// hastar_dubins_f64.h): sin, cos, atan2, acos and hypot as HybridAStar<double> calls them
// (Dubins.cpp:23-33, 185-263, 331-417; Grid3D.cpp:212-213; VelocityGenerator.cpp:40-84).
//
// The device libm (ocml) differs from the host's glibc 2.35 in the last bit on 3 % (sin, cos) to
// 27 % (atan2) of the planner's arguments (tools/libm64_fingerprint.hip, profiles/r05_libm64_ocml
// .jsonl), and glibc itself is not correctly rounded (a double-double evaluation rounded once
// still differed on ~0.1 % of arguments).  So these are ports of glibc 2.35's own routines, in the
// variants the x86-64 libm dispatches to on FMA hardware (__sin_fma, __cos_fma,
// __ieee754_atan2_fma, __ieee754_acos_fma; hypot has no FMA variant): the IBM Accurate
// Mathematical Library algorithms of sysdeps/ieee754/dbl-64 (s_sin.c, e_atan2.c, e_asin.c without
// their removed slow paths) and Borges' hypot (e_hypot.c), with every fused multiply-add GCC forms
// in that build written out (a product fuses into an addition or subtraction in the same basic
// block when all its uses are such).  Their accurate tables (uatan2.tbl, asncs.tbl, root.tbl) and
// the atan2/acos series constants are data read from this container's libm.so.6
// (tools/extract_glibc_{atan,acos}_table.py: the table points of Gal's accurate-table method cannot
// be recomputed); sin/cos's table and constants are recomputed (tools/gen_libm64_tables.py).
// Result: bit for bit the host glibc on 2e8 device samples per function and 5e7 host samples
// (tests/test_libm64_ports.py, profiles/r05_libm64_gm64.jsonl).
// Bit-exact range: atan2, acos and hypot on every argument (glibc 2.35's e_atan2.c / e_asin.c
// have no slow paths left); sin and cos for |x| < 0x419921FB'00000000 (~1.05e8, 2^27 * pi/2).
// Beyond that glibc reduces with __branred (multi-precision pi/2), which is NOT ported: these
// fall back to ::sin / ::cos, i.e. ocml on the device (not bit-exact there), glibc on the host.
// The planner only calls sin/cos on headings wrapped to [-pi, pi] and on arc angles below 2 pi.  Every operation is an IEEE basic
// operation or an explicit fma and the build has -ffp-contract=off, so device and host agree.
// glibc is LGPL-2.1 (NOTICE).
#pragma once
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#endif
#include <cmath>
#include <cstdint>
#include "hastar_libm64_tables.h"
#include "hastar_libm64_atan_table.h"
#include "hastar_libm64_acos_table.h"

#if defined(__HIPCC__)
#define GM64_HD __host__ __device__ __forceinline__
#else
#define GM64_HD inline
#endif

namespace gm64 {

struct dd {
  double hi, lo;
};

// ---- error-free transformations and double-double arithmetic (Dekker / Knuth) ----------
GM64_HD double fma_(double a, double b, double c) { return std::fma(a, b, c); }
GM64_HD dd two_sum(double a, double b) {
  const double s = a + b;
  const double bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
GM64_HD dd fast_two_sum(double a, double b) {  // |a| >= |b| (or a == 0)
  const double s = a + b;
  return {s, b - (s - a)};
}
GM64_HD dd two_prod(double a, double b) {
  const double p = a * b;
  return {p, fma_(a, b, -p)};
}
GM64_HD dd add(dd a, dd b) {
  dd s = two_sum(a.hi, b.hi);
  const dd t = two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = fast_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return fast_two_sum(s.hi, s.lo);
}
GM64_HD dd neg(dd a) { return {-a.hi, -a.lo}; }
GM64_HD dd sub(dd a, dd b) { return add(a, neg(b)); }
GM64_HD dd add_d(dd a, double b) {
  dd s = two_sum(a.hi, b);
  s.lo += a.lo;
  return fast_two_sum(s.hi, s.lo);
}
GM64_HD dd mul(dd a, dd b) {
  dd p = two_prod(a.hi, b.hi);
  p.lo = fma_(a.hi, b.lo, fma_(a.lo, b.hi, p.lo));
  return fast_two_sum(p.hi, p.lo);
}
GM64_HD dd mul_d(dd a, double b) {
  dd p = two_prod(a.hi, b);
  p.lo = fma_(a.lo, b, p.lo);
  return fast_two_sum(p.hi, p.lo);
}
GM64_HD dd div(dd a, dd b) {  // three quotient digits
  const double q1 = a.hi / b.hi;
  dd r = sub(a, mul_d(b, q1));
  const double q2 = r.hi / b.hi;
  r = sub(r, mul_d(b, q2));
  const double q3 = r.hi / b.hi;
  return add_d(fast_two_sum(q1, q2), q3);
}
GM64_HD dd sqrt_dd(dd a) {  // a > 0: one Newton step from the double root
  const double s = std::sqrt(a.hi);
  const dd r = sub(a, two_prod(s, s));
  return fast_two_sum(s, r.hi / (2.0 * s));
}
GM64_HD dd tab2(const double* t) { return {t[0], t[1]}; }
GM64_HD double round_dd(dd a) { return a.hi + a.lo; }

// ---- atan on [0, 1] --------------------------------------------------------------------
// atan(t) = atan(c) + atan(u), c = k / 64 nearest to t, u = (t - c) / (1 + t c), |u| <= 2^-7;
// atan(u) = u * sum_{n <= 8} (-1)^n u^(2n) / (2n + 1) (the next term is below 2^-126 of u)
GM64_HD dd atan01(dd t) {
  const int k = (int)(t.hi * 64.0 + 0.5);
  const double c = (double)k * 0.015625;
  const dd num = add_d(t, -c);
  const dd den = add_d(mul_d(t, c), 1.0);
  const dd u = div(num, den);
  const dd u2 = mul(u, u);
  dd s = tab2(kInvOdd[8]);
  for (int n = 7; n >= 0; --n) s = sub(tab2(kInvOdd[n]), mul(s, u2));  // s_n = 1/(2n+1) - u^2 s_(n+1)
  return add(tab2(kAtan64[k]), mul(u, s));
}

// ---- hypot: glibc 2.35's algorithm (sysdeps/ieee754/dbl-64/e_hypot.c, the build without
// fused multiply-add: Borges' correction of the rounded root), bit-exact with the host libm --
GM64_HD double hypot_kernel(double ax, double ay) {  // ax >= ay >= 0, no overflow or underflow
  double h = std::sqrt(ax * ax + ay * ay);
  double t1, t2;
  if (h <= 2.0 * ay) {
    const double delta = h - ay;
    t1 = ax * (2.0 * delta - ax);
    t2 = (delta - 2.0 * (ax - ay)) * delta;
  } else {
    const double delta = h - ax;
    t1 = 2.0 * delta * (ax - 2.0 * ay);
    t2 = (4.0 * delta - ay) * ay + delta * delta;
  }
  h -= (t1 + t2) / (2.0 * h);
  return h;
}
GM64_HD double hypot(double x, double y) {
  if (!std::isfinite(x) || !std::isfinite(y)) {
    if (std::isinf(x) || std::isinf(y)) return INFINITY;
    return x + y;
  }
  x = std::fabs(x);
  y = std::fabs(y);
  double ax = x < y ? y : x;
  const double ay = x < y ? x : y;
  if (ax > 0x1p+511) {
    if (ay <= ax * 0x1p-54) return ax + ay;
    return hypot_kernel(ax * 0x1p-600, ay * 0x1p-600) / 0x1p-600;
  }
  if (ay < 0x1p-511) {
    if (ax >= ay / 0x1p-54) return ax + ay;
    ax = hypot_kernel(ax / 0x1p-600, ay / 0x1p-600) * 0x1p-600;
    return ax;
  }
  if (ay <= ax * 0x1p-54) return ax + ay;
  return hypot_kernel(ax, ay);
}

// ---- atan2: glibc 2.35's algorithm (sysdeps/ieee754/dbl-64/e_atan2.c without its removed slow
// paths, the __ieee754_atan2_fma variant: dla.h's EMULV with fma, GCC's fusions written out), on
// uatan2.tbl's accurate table (hastar_libm64_atan_table.h) ------------------------------------
namespace at {
constexpr double d3 = -0x1.5555555555555p-2, d5 = 0x1.99999999997fdp-3, d7 = -0x1.24924923f7603p-3,
                 d9 = 0x1.c71c6e5129a3bp-4, d11 = -0x1.7458022b13c25p-4, d13 = 0x1.375f08b31cbcep-4;
constexpr double hpi = 0x1.921fb54442d18p+0, hpi1 = 0x1.1a62633145c07p-54, opi = 0x1.921fb54442d18p+1,
                 opi1 = 0x1.1a62633145c07p-53, qpi = 0x1.921fb54442d18p-1, tqpi = 0x1.2d97c7f3321d2p+1,
                 inv16 = 0.0625, two8 = 256.0, two52 = 0x1p52;
}  // namespace at
GM64_HD double at_poly(double v) {  // d3 + v (d5 + v (d7 + v (d9 + v (d11 + v d13))))
  double p = fma_(v, at::d13, at::d11);
  p = fma_(v, p, at::d9);
  p = fma_(v, p, at::d7);
  p = fma_(v, p, at::d5);
  return fma_(v, p, at::d3);
}
GM64_HD double at_tail(double v, int i, int from) {  // c_from + v (... + v c6)
  double q = fma_(v, kAtanCij[i][6], kAtanCij[i][5]);
  q = fma_(v, q, kAtanCij[i][4]);
  q = fma_(v, q, kAtanCij[i][3]);
  if (from == 2) q = fma_(v, q, kAtanCij[i][2]);
  return q;
}
GM64_HD int at_index(double u) { return (int)(fma_(at::two8, u, at::two52) - at::two52) - 16; }
GM64_HD uint64_t bits_of(double x) {
  uint64_t b;
  __builtin_memcpy(&b, &x, 8);
  return b;
}
GM64_HD double atan2(double y, double x) {
  const uint64_t bx = bits_of(x), by = bits_of(y);
  const uint32_t ux = (uint32_t)(bx >> 32), dx = (uint32_t)bx, uy = (uint32_t)(by >> 32), dy = (uint32_t)by;
  if ((ux & 0x7ff00000u) == 0x7ff00000u && (((ux & 0x000fffffu) | dx) != 0u)) return x + y;
  if ((uy & 0x7ff00000u) == 0x7ff00000u && (((uy & 0x000fffffu) | dy) != 0u)) return y + y;
  if (uy == 0x00000000u && dy == 0u) return (ux & 0x80000000u) == 0u ? 0.0 : at::opi;
  if (uy == 0x80000000u && dy == 0u) return (ux & 0x80000000u) == 0u ? -0.0 : -at::opi;
  if (x == 0.0) return (uy & 0x80000000u) == 0u ? at::hpi : -at::hpi;
  if (dx == 0u && (ux == 0x7ff00000u || ux == 0xfff00000u)) {
    const bool xneg = ux == 0xfff00000u;
    if (uy == 0x7ff00000u && dy == 0u) return xneg ? at::tqpi : at::qpi;
    if (uy == 0xfff00000u && dy == 0u) return xneg ? -at::tqpi : -at::qpi;
    if (xneg) return (uy & 0x80000000u) == 0u ? at::opi : -at::opi;
    return (uy & 0x80000000u) == 0u ? 0.0 : -0.0;
  }
  if (dy == 0u && uy == 0x7ff00000u) return at::hpi;
  if (dy == 0u && uy == 0xfff00000u) return -at::hpi;
  double ax = x < 0 ? -x : x, ay = y < 0 ? -y : y;
  const int de = (int)(uy & 0x7ff00000u) - (int)(ux & 0x7ff00000u);
  if (de >= 59768832) return y > 0 ? at::hpi : -at::hpi;
  if (de <= -59768832) {
    if (x > 0) return std::copysign(ay / ax, y);  // (glibc rescales a subnormal quotient)
    return y > 0 ? at::opi : -at::opi;
  }
  if (ax < 0x1p-500 || ay < 0x1p-500) {
    ax *= 0x1p500;
    ay *= 0x1p500;
  }
  if (ax > 0x1p500 || ay > 0x1p500) {
    ax *= 0x1p-500;
    ay *= 0x1p-500;
  }
  double u, du, v, vv;
  if (ay < ax) {
    u = ay / ax;
    v = ax * u;
    vv = fma_(ax, u, -v);
    du = ((ay - v) - vv) / ax;
  } else {
    u = ax / ay;
    v = ay * u;
    vv = fma_(ay, u, -v);
    du = ((ax - v) - vv) / ay;
  }
  double z;
  if (x > 0) {
    if (ay < ax) {  // (i) atan(ay / ax)
      if (u < at::inv16) {
        v = u * u;
        z = u + fma_(u * v, at_poly(v), du);
      } else {
        const int i = at_index(u);
        const double t3 = u - kAtanCij[i][0];
        const double w = t3 + du;
        const double dw = std::fabs(t3) > std::fabs(du) ? ((t3 - w) + du) : ((du - w) + t3);
        const double t1 = kAtanCij[i][1], t2 = kAtanCij[i][2];
        const double zz = fma_(w, t2, fma_(dw, t2, (w * w) * at_tail(w, i, 3)));
        z = t1 + zz;
      }
    } else {  // (ii) pi/2 - atan(ax / ay)
      if (u < at::inv16) {
        v = u * u;
        const double t2 = at::hpi - u;
        const double cor = std::fabs(at::hpi) > std::fabs(u) ? ((at::hpi - t2) - u) : (at::hpi - (u + t2));
        const double zz = (u * v) * at_poly(v);  // not fused: EADD/ESUB's branch separates it from its use
        const double t3 = ((at::hpi1 + cor) - du) - zz;
        z = t2 + t3;
      } else {
        const int i = at_index(u);
        v = (u - kAtanCij[i][0]) + du;
        const double zz = fma_(-v, at_tail(v, i, 2), at::hpi1);
        z = (at::hpi - kAtanCij[i][1]) + zz;
      }
    }
  } else if (ax < ay) {  // (iii) pi/2 + atan(ax / ay)
    if (u < at::inv16) {
      v = u * u;
      const double t2 = at::hpi + u;
      const double cor = std::fabs(at::hpi) > std::fabs(u) ? ((at::hpi - t2) + u) : ((u - t2) + at::hpi);
      const double zz = (u * v) * at_poly(v);
      const double t3 = ((at::hpi1 + cor) + du) + zz;
      z = t2 + t3;
    } else {
      const int i = at_index(u);
      v = (u - kAtanCij[i][0]) + du;
      const double zz = fma_(v, at_tail(v, i, 2), at::hpi1);
      z = (at::hpi + kAtanCij[i][1]) + zz;
    }
  } else {  // (iv) pi - atan(ay / ax)
    if (u < at::inv16) {
      v = u * u;
      const double t2 = at::opi - u;
      const double cor = std::fabs(at::opi) > std::fabs(u) ? ((at::opi - t2) - u) : (at::opi - (u + t2));
      const double zz = (u * v) * at_poly(v);
      const double t3 = ((at::opi1 + cor) - du) - zz;
      z = t2 + t3;
    } else {
      const int i = at_index(u);
      v = (u - kAtanCij[i][0]) + du;
      const double zz = fma_(-v, at_tail(v, i, 2), at::opi1);
      z = (at::opi - kAtanCij[i][1]) + zz;
    }
  }
  return std::copysign(z, y);
}

// ---- acos: glibc 2.35's algorithm (sysdeps/ieee754/dbl-64/e_asin.c without its removed slow
// paths, the __ieee754_acos_fma variant: GCC's fusions written out) on asncs.tbl / root.tbl
// (hastar_libm64_acos_table.h) --------------------------------------------------------------
namespace ac {
constexpr double hp0 = 0x1.921fb54442d18p+0, hp1 = 0x1.1a62633145c07p-54, pi = 0x1.921fb54442d18p+1, t27 = 0x1p27;
constexpr double f1 = 0x1.55555555554f9p-3, f2 = 0x1.333333336127dp-4, f3 = 0x1.6db6dae42c0e4p-5,
                 f4 = 0x1.f1c7e04f4ad99p-6, f5 = 0x1.6e442c822d419p-6, f6 = 0x1.292d80f453c72p-6;
constexpr double rt0 = 0x1.fffffffecc1ddp-1, rt1 = 0x1.fffffff757304p-2, rt2 = 0x1.800496769c91ap-2,
                 rt3 = 0x1.4006318d1dab9p-2;
}  // namespace ac
GM64_HD double ac_poly_f(double v) {  // ((((f6 v + f5) v + f4) v + f3) v + f2) v + f1
  double p = fma_(v, ac::f6, ac::f5);
  p = fma_(v, p, ac::f4);
  p = fma_(v, p, ac::f3);
  p = fma_(v, p, ac::f2);
  return fma_(v, p, ac::f1);
}
// one asncs interval: n its first entry, K the index of its last series coefficient
GM64_HD double ac_table(double x, int m_pos, int n, int K) {
  const double xx = (m_pos ? x : -x) - kAsncs[n];
  double q = kAsncs[n + K];
  for (int i = K - 1; i >= 2; --i) q = fma_(xx, q, kAsncs[n + i]);
  const double p = fma_(xx * xx, q, kAsncs[n + K + 1]);
  const double t = fma_(xx, kAsncs[n + 1], p);
  const double ya = kAsncs[n + K + 2];
  if (m_pos) return (ac::hp1 - t) + (ac::hp0 - ya);
  return (t + ac::hp1) + (ya + ac::hp0);
}
GM64_HD double acos(double x) {
  uint64_t bx;
  __builtin_memcpy(&bx, &x, 8);
  const int32_t m = (int32_t)(bx >> 32);
  const uint32_t lo = (uint32_t)bx;
  const uint32_t k = (uint32_t)m & 0x7fffffffu;
  const int pos = m > 0;
  if (k < 0x3c880000u) return ac::hp0;
  if (k < 0x3fc00000u) {  // |x| < 0.125
    const double x2 = x * x;
    const double p = ac_poly_f(x2);
    const double r = ac::hp0 - x;
    const double cor = fma_(-p, x * x2, ((ac::hp0 - r) - x) + ac::hp1);
    return r + cor;
  }
  if (k < 0x3fd00000u) return ac_table(x, pos, 11 * (int)((k >> 15) & 0x1f), 6);            // [0.125, 0.25)
  if (k < 0x3fe00000u) return ac_table(x, pos, 11 * (int)((k >> 14) & 0x3f) + 352, 6);      // [0.25, 0.5)
  if (k < 0x3fe80000u) return ac_table(x, pos, 12 * (int)((k >> 13) & 0x7f) + 1056, 7);     // [0.5, 0.75)
  if (k < 0x3fed8000u) return ac_table(x, pos, 13 * (int)((k >> 13) & 0x7f) + 992, 8);      // [0.75, 0.921875)
  if (k < 0x3fee8000u) return ac_table(x, pos, 14 * (int)((k >> 13) & 0x7f) + 884, 9);      // [0.921875, 0.953125)
  if (k < 0x3fef0000u) return ac_table(x, pos, 15 * (int)((k >> 13) & 0x7f) + 768, 10);     // [0.953125, 0.96875)
  if (k < 0x3ff00000u) {  // [0.96875, 1): 2 asin(sqrt(z)), z = (1 - |x|) / 2
    const double z = 0.5 * (pos ? (1.0 - x) : (x + 1.0));
    uint64_t bz;
    __builtin_memcpy(&bz, &z, 8);
    double t = kInroot[(int)((bz >> 46) & 0x7f)] * kPowtwo[511 - (int)(bz >> 53)];
    const double r = fma_(-(t * t), z, 1.0);
    t = t * fma_(r, fma_(r, fma_(r, ac::rt3, ac::rt2), ac::rt1), ac::rt0);
    const double c = z * t;
    const double u = fma_(-(0.5 * t), c, 1.5);
    const double y = fma_(-ac::t27, c, fma_(c, ac::t27, c));
    const double cc = fma_(-y, y, z) / fma_(u, c, y);
    const double pz = ac_poly_f(z) * z;
    const double pyc = pz * (y + cc);
    if (!pos) {
      const double cor = (ac::hp1 - cc) - pyc;
      const double res = (ac::hp0 - y) + cor;
      return res + res;
    }
    const double res = (cc + pyc) + y;
    return res + res;
  }
  if (k == 0x3ff00000u && lo == 0u) return pos ? 0.0 : ac::pi;
  if (k > 0x7ff00000u || (k == 0x7ff00000u && lo != 0u)) return x + x;
  const double zz = x - x;
  return zz / zz;
}

// ---- sin / cos: glibc 2.35's algorithm (sysdeps/ieee754/dbl-64/s_sin.c, the __sin_fma /
// __cos_fma variants the x86-64 libm dispatches to on FMA hardware).  That build lets GCC fuse
// every product whose uses are all additions or subtractions into them (-ffp-contract=fast),
// so the fused multiply-adds below are written out where GCC forms them.  The table is
// __sincostab's layout (sin and cos of i/128 split in two doubles).  Valid for |x| < 105414350
// (reduce_sincos); beyond it (never in the planner) the device libm.
namespace sc {
constexpr double s1 = -0x1.5555555555555p-3, s2 = 0.0083333333333323288, s3 = -0.00019841269834414642,
                 s4 = 2.755729806860771e-06, s5 = -2.5022014848318398e-08;
constexpr double sn3 = -1.66666666666664880952546298448555E-01, sn5 = 8.33333214285722277379541354343671E-03,
                 cs2 = 4.99999999999999999999950396842453E-01, cs4 = -4.16666666666664434524222570944589E-02,
                 cs6 = 1.38888874007937613028114285595617E-03;
constexpr double big = 0x1.8p45, hp0 = 0x1.921FB54442D18p0, hp1 = 0x1.1A62633145C07p-54,
                 mp1 = 0x1.921FB58000000p0, mp2 = -0x1.DDE973C000000p-27, pp3 = -0x1.CB3B398000000p-55,
                 pp4 = -0x1.d747f23e32ed7p-83, hpinv = 0x1.45F306DC9C883p-1, toint = 0x1.8p52;
}  // namespace sc
GM64_HD int sc_index(double u) { return (int)((u - sc::big) * 128.0); }
GM64_HD double sc_taylor_sin(double xx, double a, double da) {
  double p = fma_(sc::s5, xx, sc::s4);
  p = fma_(p, xx, sc::s3);
  p = fma_(p, xx, sc::s2);
  p = fma_(p, xx, sc::s1);                   // POLYNOMIAL (xx)
  const double t0 = fma_(p, a, -(0.5 * da));  // POLYNOMIAL (xx) * a - 0.5 * da
  const double t = fma_(t0, xx, da);
  return a + t;
}
GM64_HD double sc_do_cos(double x, double dx) {
  if (x < 0) dx = -dx;
  const double u = sc::big + std::fabs(x);
  x = std::fabs(x) - (u - sc::big) + dx;
  const double xx = x * x;
  const double s = fma_(x * xx, fma_(xx, sc::sn5, sc::sn3), x);
  const double c = xx * fma_(xx, fma_(xx, sc::cs6, sc::cs4), sc::cs2);
  const int k = sc_index(u);
  const double sn = kSinCos128[k][0], ssn = kSinCos128[k][1], cs = kSinCos128[k][2], ccs = kSinCos128[k][3];
  double cor = fma_(-s, ssn, ccs);
  cor = fma_(-cs, c, cor);
  cor = fma_(-sn, s, cor);
  return cs + cor;
}
GM64_HD double sc_do_sin(double x, double dx) {
  const double xold = x;
  if (std::fabs(x) < 0.126) return sc_taylor_sin(x * x, x, dx);
  if (x <= 0) dx = -dx;
  const double u = sc::big + std::fabs(x);
  x = std::fabs(x) - (u - sc::big);
  const double xx = x * x;
  const double s = x + fma_(x * xx, fma_(xx, sc::sn5, sc::sn3), dx);
  const double c = fma_(x, dx, xx * fma_(xx, fma_(xx, sc::cs6, sc::cs4), sc::cs2));
  const int k = sc_index(u);
  const double sn = kSinCos128[k][0], ssn = kSinCos128[k][1], cs = kSinCos128[k][2], ccs = kSinCos128[k][3];
  double cor = fma_(s, ccs, ssn);
  cor = fma_(-sn, c, cor);
  cor = fma_(cs, s, cor);
  return std::copysign(sn + cor, xold);
}
GM64_HD int sc_reduce(double x, double* a, double* da) {
  const double t = fma_(x, sc::hpinv, sc::toint);
  const double xn = t - sc::toint;
  const double y = fma_(-xn, sc::mp2, fma_(-xn, sc::mp1, x));
  const int n = (int)((long long)xn & 3);
  const double t2 = fma_(-xn, sc::pp3, y);
  double db = fma_(-xn, sc::pp3, y - t2);
  const double b = fma_(-xn, sc::pp4, t2);
  db += fma_(-xn, sc::pp4, t2 - b);
  *a = b;
  *da = db;
  return n;
}
GM64_HD double sc_do_sincos(double a, double da, int n) {
  const double r = (n & 1) ? sc_do_cos(a, da) : sc_do_sin(a, da);
  return (n & 2) ? -r : r;
}
GM64_HD uint32_t hi_word(double x) {
  uint64_t b;
  __builtin_memcpy(&b, &x, 8);
  return (uint32_t)(b >> 32) & 0x7fffffffu;
}
GM64_HD double sin(double x) {
  const uint32_t k = hi_word(x);
  if (k < 0x3e500000u) return x;
  if (k < 0x3feb6000u) return sc_do_sin(x, 0.0);
  if (k < 0x400368fdu) return std::copysign(sc_do_cos(sc::hp0 - std::fabs(x), sc::hp1), x);
  if (k < 0x419921FBu) {
    double a, da;
    const int n = sc_reduce(x, &a, &da);
    return sc_do_sincos(a, da, n);
  }
  if (k < 0x7ff00000u) return ::sin(x);
  return x / x;
}
GM64_HD double cos(double x) {
  const uint32_t k = hi_word(x);
  if (k < 0x3e400000u) return 1.0;
  if (k < 0x3feb6000u) return sc_do_cos(x, 0.0);
  if (k < 0x400368fdu) {
    const double y = sc::hp0 - std::fabs(x);
    const double a = y + sc::hp1;
    const double da = (y - a) + sc::hp1;
    return sc_do_sin(a, da);
  }
  if (k < 0x419921FBu) {
    double a, da;
    const int n = sc_reduce(x, &a, &da);
    return sc_do_sincos(a, da, n + 1);
  }
  if (k < 0x7ff00000u) return ::cos(x);
  return x / x;
}

}  // namespace gm64
