// fetch_calib.hip — calibrates rocprofv3's HBM read counters on gfx950 against known byte
// counts, for the access patterns of the search kernel (profiles/r05_fetch_calib*):
//
//   stream16   every lane reads consecutive 16 B (float4) over 2 GiB: the guide's calibration
//              case (FETCH_SIZE reports half of these bytes on gfx950)
//   scatter4   one 4-B load per distinct 128-B line, lines drawn at random over 16 GiB
//   scatter16  one 16-B load per distinct 128-B line, the same way
//   probe      the inner A*'s probe pattern (hastar_kernels.hip astar_loop_lds): 2048 waves, each
//              a random walk over its own 1024x1024 maps {occ f32, node-map f32, visited bitmap,
//              16-B cell record}; per step the 8 neighbour lanes load occ, the bitmap word,
//              node-map f and the cell record, and lane 0 the centre's cell record (240 B
//              requested per step)
//
//   tools/bin/fetch_calib            runs each pattern once (its own kernel), prints the requested
//                                    bytes and the distinct 128-B lines each touched
// Run it under rocprofv3 --pmc (tools/prof_fetch_calib.sh) to read the counters per kernel.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <string>
#include <unordered_set>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                                   \
    }                                                                                 \
  } while (0)

__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void k_stream16(const v4f* __restrict__ a, size_t n4, float* out) {
  float acc = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const v4f v = a[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.0f) out[0] = acc;  // keeps the loads
}

// line index of load t: a permutation-free random draw (collisions counted on the host)
__host__ __device__ inline uint64_t line_of(uint64_t t, uint64_t n_lines) { return mix64(t) % n_lines; }

__global__ void k_scatter4(const float* __restrict__ a, uint64_t n_lines, uint64_t n, float* out) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t line = line_of(t, n_lines);
  const float v = a[line * 32 + (mix64(t ^ 0xabcdefull) & 31)];
  if (v == 12345.0f) out[0] = v;
}

__global__ void k_scatter16(const v4f* __restrict__ a, uint64_t n_lines, uint64_t n, float* out) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t line = line_of(t, n_lines);
  const v4f v = a[line * 8 + (mix64(t ^ 0xabcdefull) & 7)];
  if (v.x + v.y == 12345.0f) out[0] = v.x;
}

struct Cell {
  uint32_t a, b, c, d;
};

// one wave per "planner": maps of N x N cells at base + w * stride
__global__ __launch_bounds__(64) void k_probe(const char* __restrict__ base, size_t stride, int N, int steps, float* out) {
  const int w = blockIdx.x, lane = threadIdx.x;
  const char* m = base + (size_t)w * stride;
  const size_t NN = (size_t)N * N;
  const float* occ = (const float*)m;
  const float* nmf = (const float*)(m + 4 * NN);
  const uint32_t* vis = (const uint32_t*)(m + 8 * NN);
  const Cell* cells = (const Cell*)(m + 8 * NN + ((NN / 8 + 255) & ~(size_t)255));
  int x = N / 2, y = N / 2;
  const int dx[8] = {-1, -1, -1, 0, 0, 1, 1, 1}, dy[8] = {-1, 0, 1, -1, 1, -1, 0, 1};
  float acc = 0.0f;
  for (int s = 0; s < steps; ++s) {
    const uint64_t r = mix64(((uint64_t)w << 32) | (uint64_t)s);
    if (lane == 0) {
      const Cell c = cells[(size_t)x * N + y];
      acc += (float)c.a;
    }
    if (lane < 8) {
      const int i = x + dx[lane], j = y + dy[lane];
      const size_t cell = (size_t)i * N + j;
      acc += occ[cell] + nmf[cell] + (float)vis[cell >> 5];
      const Cell c = cells[cell];
      acc += (float)c.b;
    }
    // random step (8-connected), kept inside the grid
    const int k = (int)(r & 7);
    x = min(max(x + dx[k], 1), N - 2);
    y = min(max(y + dy[k], 1), N - 2);
  }
  if (acc == 12345.0f) out[0] = acc;
}

int main(int argc, char** argv) {
  const char* only = argc > 1 ? argv[1] : "all";
  float* d_out = nullptr;
  CK(hipMalloc(&d_out, 64));
  auto want = [&](const char* n) { return std::string(only) == "all" || std::string(only) == n; };
  if (want("stream16")) {
    const size_t bytes = (size_t)2 << 30;
    void* a = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMemset(a, 0, bytes));
    CK(hipDeviceSynchronize());
    k_stream16<<<4096, 256>>>((const v4f*)a, bytes / 16, d_out);
    CK(hipDeviceSynchronize());
    std::printf("{\"pattern\": \"stream16\", \"kernel\": \"k_stream16\", \"requested_bytes\": %zu, \"distinct_lines\": %zu}\n",
                bytes, bytes / 128);
    CK(hipFree(a));
  }
  for (int w16 = 0; w16 < 2; ++w16) {
    const char* name = w16 ? "scatter16" : "scatter4";
    if (!want(name)) continue;
    const size_t bytes = (size_t)16 << 30;
    const uint64_t n_lines = bytes / 128, n = (uint64_t)1 << 24;
    void* a = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMemset(a, 0, bytes));
    CK(hipDeviceSynchronize());
    if (w16) k_scatter16<<<(unsigned)(n / 256), 256>>>((const v4f*)a, n_lines, n, d_out);
    else k_scatter4<<<(unsigned)(n / 256), 256>>>((const float*)a, n_lines, n, d_out);
    CK(hipDeviceSynchronize());
    std::unordered_set<uint64_t> lines;
    lines.reserve(n * 2);
    for (uint64_t t = 0; t < n; ++t) lines.insert(line_of(t, n_lines));
    std::printf("{\"pattern\": \"%s\", \"kernel\": \"%s\", \"requested_bytes\": %llu, \"distinct_lines\": %zu}\n", name,
                w16 ? "k_scatter16" : "k_scatter4", (unsigned long long)(n * (w16 ? 16 : 4)), lines.size());
    CK(hipFree(a));
  }
  if (want("probe")) {
    const int N = 1024, W = 2048, steps = 256;
    const size_t NN = (size_t)N * N;
    const size_t stride = ((8 * NN + ((NN / 8 + 255) & ~(size_t)255) + 16 * NN) + 4095) & ~(size_t)4095;
    void* a = nullptr;
    CK(hipMalloc(&a, stride * W));
    CK(hipMemset(a, 0, stride * W));
    CK(hipDeviceSynchronize());
    k_probe<<<W, 64>>>((const char*)a, stride, N, steps, d_out);
    CK(hipDeviceSynchronize());
    // the distinct 128-B lines the walks touched (host replay of the same walks)
    std::unordered_set<uint64_t> lines;
    const int dx[8] = {-1, -1, -1, 0, 0, 1, 1, 1}, dy[8] = {-1, 0, 1, -1, 1, -1, 0, 1};
    const size_t o_nmf = 4 * NN, o_vis = 8 * NN, o_cell = 8 * NN + ((NN / 8 + 255) & ~(size_t)255);
    for (int w = 0; w < W; ++w) {
      const size_t b = (size_t)w * stride;
      int x = N / 2, y = N / 2;
      for (int s = 0; s < steps; ++s) {
        const uint64_t r = mix64(((uint64_t)w << 32) | (uint64_t)s);
        lines.insert((b + o_cell + 16 * ((size_t)x * N + y)) / 128);
        for (int l = 0; l < 8; ++l) {
          const size_t cell = (size_t)(x + dx[l]) * N + (y + dy[l]);
          lines.insert((b + 4 * cell) / 128);
          lines.insert((b + o_nmf + 4 * cell) / 128);
          lines.insert((b + o_vis + 4 * (cell >> 5)) / 128);
          lines.insert((b + o_cell + 16 * cell) / 128);
        }
        const int k = (int)(r & 7);
        x = std::min(std::max(x + dx[k], 1), N - 2);
        y = std::min(std::max(y + dy[k], 1), N - 2);
      }
    }
    std::printf("{\"pattern\": \"probe\", \"kernel\": \"k_probe\", \"requested_bytes\": %llu, \"distinct_lines\": %zu, "
                "\"waves\": %d, \"steps\": %d}\n", (unsigned long long)W * steps * 240ull, lines.size(), W, steps);
    CK(hipFree(a));
  }
  CK(hipFree(d_out));
  return 0;
}
