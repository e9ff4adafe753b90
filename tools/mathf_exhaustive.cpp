// mathf_exhaustive.cpp — sweep the glibc_mathf.h ports against the live glibc libm.
//
//   g++ -O2 -mfma -ffp-contract=off -fopenmp -I path_planning_pkg_amd/csrc \
//       tools/mathf_exhaustive.cpp -o /tmp/mathf_exhaustive -lm
//   /tmp/mathf_exhaustive [all|fast] [samples2]
//
// "all": every one of the 2^32 float inputs for sinf, cosf, acosf, atanf and
// 2^32 pseudo-random (y, x) pairs for atan2f / hypotf (plus the structured set).
// "fast": the float ranges the planner reaches ([-8, 8] for sin/cos, [-1, 1] for
// acos, all finite pairs with |y|,|x| < 4096 sampled) — a few seconds.
// Prints one line per function: inputs checked, bitwise mismatches (NaN == NaN).
// Exit status 0 iff no mismatch.  Run on a host whose sinf/cosf IFUNC resolves to
// the FMA variant (check: grep -c fma /proc/cpuinfo).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <cmath>
#include <atomic>
#include "glibc_mathf.h"

using namespace gmath;

static bool same(float a, float b) {
  if (std::isnan(a) && std::isnan(b)) return true;
  return fbits(a) == fbits(b);
}

static uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

template <class F, class G>
static uint64_t sweep1(const char* name, uint64_t lo, uint64_t hi, F port, G ref) {
  std::atomic<uint64_t> bad{0};
  uint64_t first = 0;
  bool have = false;
#pragma omp parallel for schedule(dynamic, 1 << 16)
  for (uint64_t u = lo; u < hi; ++u) {
    float x = bitsf((uint32_t)u);
    if (!same(port(x), ref(x))) {
      if (bad.fetch_add(1) == 0) {
#pragma omp critical
        { first = u; have = true; }
      }
    }
  }
  std::printf("%-8s inputs=%llu mismatches=%llu", name, (unsigned long long)(hi - lo),
              (unsigned long long)bad.load());
  if (have) std::printf(" first=0x%08llx", (unsigned long long)first);
  std::printf("\n");
  return bad.load();
}

template <class F, class G>
static uint64_t sweep_range(const char* name, float a, float b, F port, G ref) {
  // all floats in [a, b] (a <= 0 <= b handled as two monotone bit ranges)
  uint64_t bad = 0;
  if (a < 0) bad += sweep1(name, 0x80000000ull, (uint64_t)fbits(a) + 1, port, ref);
  if (b >= 0) bad += sweep1(name, 0, (uint64_t)fbits(b) + 1, port, ref);
  return bad;
}

template <class F, class G>
static uint64_t sweep2(const char* name, uint64_t n, float scale, F port, G ref) {
  std::atomic<uint64_t> bad{0};
#pragma omp parallel for schedule(dynamic, 1 << 14)
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t s = i * 0x632be59bd9b4e019ull + 12345;
    uint64_t r = splitmix(s);
    float y, x;
    if (scale > 0) {
      y = (float)((int64_t)(r & 0xffffffff) - 0x80000000ll) / 2147483648.0f * scale;
      x = (float)((int64_t)(r >> 32) - 0x80000000ll) / 2147483648.0f * scale;
    } else {
      y = bitsf((uint32_t)r);
      x = bitsf((uint32_t)(r >> 32));
    }
    if (!same(port(y, x), ref(y, x))) bad.fetch_add(1);
  }
  std::printf("%-8s pairs=%llu mismatches=%llu (scale %g)\n", name, (unsigned long long)n,
              (unsigned long long)bad.load(), scale);
  return bad.load();
}

int main(int argc, char** argv) {
  const bool all = argc > 1 && std::strcmp(argv[1], "all") == 0;
  const uint64_t n2 = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : (all ? (1ull << 32) : (1ull << 26));
  auto psin = [](float x) { return g_sinf(x); };
  auto rsin = [](float x) { return ::sinf(x); };
  auto pcos = [](float x) { return g_cosf(x); };
  auto rcos = [](float x) { return ::cosf(x); };
  auto pacos = [](float x) { return g_acosf(x); };
  auto racos = [](float x) { return ::acosf(x); };
  auto patan = [](float x) { return g_atanf(x); };
  auto ratan = [](float x) { return ::atanf(x); };
  auto pat2 = [](float y, float x) { return g_atan2f(y, x); };
  auto rat2 = [](float y, float x) { return ::atan2f(y, x); };
  auto phyp = [](float y, float x) { return g_hypotf(y, x); };
  auto rhyp = [](float y, float x) { return ::hypotf(y, x); };
  uint64_t bad = 0;
  if (all) {
    bad += sweep1("sinf", 0, 1ull << 32, psin, rsin);
    bad += sweep1("cosf", 0, 1ull << 32, pcos, rcos);
    bad += sweep1("acosf", 0, 1ull << 32, pacos, racos);
    bad += sweep1("atanf", 0, 1ull << 32, patan, ratan);
  } else {
    bad += sweep_range("sinf", -8.0f, 8.0f, psin, rsin);
    bad += sweep_range("cosf", -8.0f, 8.0f, pcos, rcos);
    bad += sweep_range("acosf", -1.0f, 1.0f, pacos, racos);
    bad += sweep_range("atanf", -64.0f, 64.0f, patan, ratan);
    // large-argument reduction path and specials, sampled
    bad += sweep1("sinf-lg", 0x42f00000ull, 0x42f00000ull + (1u << 22), psin, rsin);
    bad += sweep1("cosf-lg", 0xc7000000ull, 0xc7000000ull + (1u << 22), pcos, rcos);
    bad += sweep1("sinf-sp", 0x7f7ff000ull, 0x80000000ull + 0x10, psin, rsin);
  }
  bad += sweep2("atan2f", n2, 1024.0f, pat2, rat2);
  bad += sweep2("atan2f", n2, 2.0f, pat2, rat2);
  bad += sweep2("atan2f", n2 / 4, 0.0f, pat2, rat2);
  bad += sweep2("hypotf", n2 / 4, 1024.0f, phyp, rhyp);
  bad += sweep2("hypotf", n2 / 16, 0.0f, phyp, rhyp);
  // structured atan2f cases: axes, infinities, signed zeros
  const float sp[] = {0.0f, -0.0f, 1.0f, -1.0f, INFINITY, -INFINITY, NAN, 1e-40f, -1e-40f, 3.0f, -3.0f,
                      1e30f, -1e30f, 1e-30f, -1e-30f};
  uint64_t sbad = 0;
  for (float y : sp)
    for (float x : sp) {
      if (!same(g_atan2f(y, x), ::atan2f(y, x))) ++sbad;
      if (!same(g_hypotf(y, x), ::hypotf(y, x))) ++sbad;
    }
  std::printf("special  pairs=%zu mismatches=%llu\n", sizeof(sp) / sizeof(sp[0]) * sizeof(sp) / sizeof(sp[0]),
              (unsigned long long)sbad);
  bad += sbad;
  std::printf("TOTAL mismatches=%llu\n", (unsigned long long)bad);
  return bad ? 1 : 0;
}
