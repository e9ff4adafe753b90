// libm64_fingerprint.hip — how often the device's f64 sin/cos/atan2/acos/hypot differ from the
// host's glibc (the libm the reference's HybridAStar<double> calls: Dubins.cpp:23-33, 185-263,
// Grid3D.cpp:212-213) on the argument ranges the double planner feeds them.
//
//   hipcc -O3 -ffp-contract=off --offload-arch=gfx950 tools/libm64_fingerprint.hip -o tools/bin/libm64_fingerprint
//   tools/bin/libm64_fingerprint [samples per function, default 2e8] [impl: 0 device libm, 1 gm64 (this repo)]
//
// Inputs come from a counter-based generator (splitmix64 of the sample index), so the device
// and the host draw the same arguments without a transfer.  Prints one JSON line per function:
// samples, mismatches, the ulp-difference histogram and the first mismatching arguments.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include "../path_planning_pkg_amd/csrc/hastar_libm64.h"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      std::exit(2);                                                                    \
    }                                                                                  \
  } while (0)

__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__host__ __device__ inline double unit(uint64_t b) { return (double)(b >> 11) * 0x1.0p-53; }

// argument ranges: fn 0 sin, 1 cos: half in [-pi, pi], half in [-10, 10] (headings and
// heading + arc sums of the Dubins words); 2 atan2(y, x), 4 hypot(x, y): both in [-300, 300]
// (centre and obstacle offsets in metres), a quarter in [-3, 3]; 3 acos: [0, 1] (2 r / dist)
__host__ __device__ inline void args(int fn, uint64_t i, double* a, double* b) {
  const uint64_t r1 = mix64(i * 2 + 0x1234567ull * (uint64_t)(fn + 1)), r2 = mix64(i * 2 + 1 + 0x7654321ull * (uint64_t)(fn + 1));
  const double u = unit(r1), v = unit(r2);
  switch (fn) {
    case 0:
    case 1:
      *a = (i & 1) ? (u * 2.0 - 1.0) * 3.141592653589793 : (u * 2.0 - 1.0) * 10.0;
      *b = 0.0;
      break;
    case 3:
      *a = u;
      *b = 0.0;
      break;
    default: {
      const double s = (i & 3) == 0 ? 3.0 : 300.0;
      *a = (u * 2.0 - 1.0) * s;
      *b = (v * 2.0 - 1.0) * s;
    }
  }
}

template <int IMPL>
__device__ inline double dev_fn(int fn, double a, double b) {
  if (IMPL == 0) {
    switch (fn) {
      case 0: return ::sin(a);
      case 1: return ::cos(a);
      case 2: return ::atan2(a, b);
      case 3: return ::acos(a);
      default: return ::hypot(a, b);
    }
  } else {
    switch (fn) {
      case 0: return gm64::sin(a);
      case 1: return gm64::cos(a);
      case 2: return gm64::atan2(a, b);
      case 3: return gm64::acos(a);
      default: return gm64::hypot(a, b);
    }
  }
}

template <int IMPL>
__global__ void k_eval(int fn, uint64_t base, int n, double* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  double a, b;
  args(fn, base + (uint64_t)t, &a, &b);
  out[t] = dev_fn<IMPL>(fn, a, b);
}

static double host_fn(int fn, double a, double b) {
  switch (fn) {
    case 0: return std::sin(a);
    case 1: return std::cos(a);
    case 2: return std::atan2(a, b);
    case 3: return std::acos(a);
    default: return std::hypot(a, b);
  }
}

static int64_t ord(double d) {  // monotone integer image of a double (ulp distance = difference)
  int64_t i;
  std::memcpy(&i, &d, 8);
  return i < 0 ? (int64_t)0x8000000000000000ull - i : i;
}

int main(int argc, char** argv) {
  const double want = argc > 1 ? std::atof(argv[1]) : 2e8;
  const int impl = argc > 2 ? std::atoi(argv[2]) : 0;
  const int nthreads = argc > 3 ? std::atoi(argv[3]) : 16;
  const uint64_t total = (uint64_t)want;
  const int chunk = 1 << 24;
  double* d_out = nullptr;
  CK(hipMalloc(&d_out, (size_t)chunk * 8));
  std::vector<double> h_out((size_t)chunk);
  const char* names[5] = {"sin", "cos", "atan2", "acos", "hypot"};
  for (int fn = 0; fn < 5; ++fn) {
    uint64_t mism = 0;
    uint64_t hist[5] = {0, 0, 0, 0, 0};  // 1, 2, 3..4, 5..16, more ulps
    std::vector<std::pair<double, double>> ex;
    for (uint64_t base = 0; base < total; base += chunk) {
      const int n = (int)std::min<uint64_t>(chunk, total - base);
      if (impl == 0) k_eval<0><<<(n + 255) / 256, 256>>>(fn, base, n, d_out);
      else k_eval<1><<<(n + 255) / 256, 256>>>(fn, base, n, d_out);
      CK(hipGetLastError());
      CK(hipMemcpy(h_out.data(), d_out, (size_t)n * 8, hipMemcpyDeviceToHost));
      std::vector<uint64_t> tm((size_t)nthreads, 0);
      std::vector<uint64_t> th((size_t)nthreads * 5, 0);
      std::vector<std::vector<std::pair<double, double>>> tex((size_t)nthreads);
      std::vector<std::thread> pool;
      for (int w = 0; w < nthreads; ++w)
        pool.emplace_back([&, w] {
          for (int t = w; t < n; t += nthreads) {
            double a, b;
            args(fn, base + (uint64_t)t, &a, &b);
            const double r = host_fn(fn, a, b);
            if (std::memcmp(&r, &h_out[(size_t)t], 8) != 0) {
              ++tm[(size_t)w];
              const int64_t du = std::llabs(ord(r) - ord(h_out[(size_t)t]));
              const int bin = du <= 1 ? 0 : du == 2 ? 1 : du <= 4 ? 2 : du <= 16 ? 3 : 4;
              ++th[(size_t)w * 5 + bin];
              if (tex[(size_t)w].size() < 4) tex[(size_t)w].push_back({a, b});
            }
          }
        });
      for (auto& p : pool) p.join();
      for (int w = 0; w < nthreads; ++w) {
        mism += tm[(size_t)w];
        for (int q = 0; q < 5; ++q) hist[q] += th[(size_t)w * 5 + q];
        for (auto& e : tex[(size_t)w])
          if (ex.size() < 6) ex.push_back(e);
      }
    }
    std::printf("{\"fn\": \"%s\", \"impl\": \"%s\", \"samples\": %llu, \"mismatches\": %llu, \"rate\": %.3e, "
                "\"ulp_hist\": {\"1\": %llu, \"2\": %llu, \"3-4\": %llu, \"5-16\": %llu, \">16\": %llu}, \"examples\": [",
                names[fn], impl == 0 ? "device libm (ocml)" : "gm64", (unsigned long long)total, (unsigned long long)mism,
                (double)mism / (double)total, (unsigned long long)hist[0], (unsigned long long)hist[1],
                (unsigned long long)hist[2], (unsigned long long)hist[3], (unsigned long long)hist[4]);
    for (size_t e = 0; e < ex.size(); ++e) std::printf("%s[%a, %a]", e ? ", " : "", ex[e].first, ex[e].second);
    std::printf("]}\n");
    std::fflush(stdout);
  }
  CK(hipFree(d_out));
  return 0;
}
