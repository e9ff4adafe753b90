// hastar_field.hip — the backward grid-distance field to the goal (the "Grid2D heuristic fill"
// of BASELINE.json's north_star), over a block of map rows, so that G ranks can build one
// field together (path_planning_pkg_amd/shard.py:heuristic_field_sharded).
//
// The field is the converged value of the reference's lazy holonomic A* for every cell at once
// (AStar.cpp:118-186 over Grid2D.cpp:22-40's moves: axis moves cost act_cost_axis, diagonal
// ones act_cost_diag, 4 or 8 moves as grid_2d_allow_diag_moves says): d(goal) = 0 and, for
// every other cell v, d(v) = min over the neighbours u that can be expanded (the goal, or
// occupancy < thr) of fl(d(u) + w(u, v)), +inf when no such u exists.  With w > 0 and float
// addition monotone, this system has exactly one solution, so every relaxation order reaches
// the same bits: a float Dijkstra (oracle/field_oracle.c), one GPU, or G ranks exchanging their
// block's edge rows.  That is what lets the rows shard.  The relaxed mode's own field
// (hastar_relaxed.hip: relaxed_heuristic) is a bounded variant of it; a full field computed
// here can be installed in its place (hastar_relaxed_set_field).
//
// Layout: a block of rows [r0, r1) is held in a buffer of (r1 - r0 + 2) rows of N floats:
// local row 0 is the halo row r0 - 1 (the upper neighbour's last row, +inf outside the grid),
// local rows 1 .. R are the block, local row R + 1 is the halo row r1.
//
// Kernel: chaotic relaxation over 32 x 32 tiles.  A workgroup loads its tile and a one-cell
// apron into LDS, relaxes the tile in place until no cell changes (each update is one
// min(d(v), fl(d(u) + w)) from a neighbour's current value, so the tile only moves towards the
// fixed point), writes the changed cells back, and marks the neighbouring tiles active for the
// next pass when a cell on its edge changed.  The host repeats passes until no tile is active.
// It is HBM-bound streaming with a data-dependent pass count.
#include <hip/hip_runtime.h>

#include "hastar_device.h"
#include "hastar_kernels.h"

namespace hastar {

constexpr int FT = 32;           // tile side (cells)
constexpr int FA = FT + 2;       // with the apron
constexpr int FIELD_THREADS = 256;

__global__ __launch_bounds__(256) void k_field_init(float* __restrict__ f, int N, int r0, int rows, int gi, int gj) {
  // rows = R + 2 buffer rows; every cell +inf, the goal 0 when it lies in the block
  const size_t n = (size_t)rows * N;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (size_t)gridDim.x * blockDim.x) {
    const int lr = (int)(k / N), j = (int)(k % N);
    const int gr = r0 - 1 + lr;
    const bool block = lr >= 1 && lr < rows - 1;
    f[k] = (block && gr == gi && j == gj) ? 0.0f : __int_as_float(0x7f800000);
  }
}

// One pass over the active tiles of rows [r0, r1).  act/nxt: one flag per tile (row-major over
// ty x tx tiles); flags: bit 0 any cell changed, bit 1 row r0 changed, bit 2 row r1 - 1 changed;
// *pending counts the tiles activated for the next pass.
__global__ __launch_bounds__(FIELD_THREADS) void k_field_pass(const PlannerDev P, float* __restrict__ f, int r0, int r1,
                                                              const int* __restrict__ act, int* __restrict__ nxt,
                                                              int* __restrict__ flags, int* __restrict__ pending) {
  const int N = P.N, R = r1 - r0;
  const int ntx = (N + FT - 1) / FT, nty = (R + FT - 1) / FT;
  const int t = (int)blockIdx.x;
  if (t >= ntx * nty || act[t] == 0) return;
  const int ty = t / ntx, tx = t % ntx;
  const int lr0 = ty * FT;  // first block row of the tile (0-based within the block)
  const int c0 = tx * FT;
  __shared__ float d[FA][FA];
  __shared__ unsigned char ex[FA][FA];  // 1: the cell can be expanded (goal, or occupancy < thr)
  __shared__ int any, top, bot, edge;
  const int tid = (int)threadIdx.x;
  if (tid == 0) any = top = bot = edge = 0;
  const GAS float* occ = gp(P.occ);
  for (int k = tid; k < FA * FA; k += FIELD_THREADS) {
    const int a = k / FA, b = k % FA;
    const int lr = lr0 + a;  // buffer row (the apron's row a = 0 is buffer row lr0, i.e. block row lr0 - 1)
    const int gr = r0 - 1 + lr, j = c0 - 1 + b;
    float v = __int_as_float(0x7f800000);
    unsigned char e = 0;
    if (lr <= R + 1 && gr >= 0 && gr < N && j >= 0 && j < N) {
      v = f[(size_t)lr * N + j];
      e = (gr == P.goal_cx && j == P.goal_cy) || occ[(size_t)gr * N + j] < P.thr;
    }
    d[a][b] = v;
    ex[a][b] = e;
  }
  __syncthreads();
  const float wa = P.act_cost_axis, wd = P.act_cost_diag;
  const bool diag = P.diag != 0;
  // each thread owns FT * FT / 256 = 4 cells of the tile: (a, b) = (1 + k / FT, 1 + k % FT)
  float orig[FT * FT / FIELD_THREADS];
#pragma unroll
  for (int q = 0; q < FT * FT / FIELD_THREADS; ++q) {
    const int k = tid + q * FIELD_THREADS;
    orig[q] = d[1 + k / FT][1 + k % FT];
  }
  for (;;) {
    int changed = 0;
#pragma unroll
    for (int q = 0; q < FT * FT / FIELD_THREADS; ++q) {
      const int k = tid + q * FIELD_THREADS;
      const int a = 1 + k / FT, b = 1 + k % FT;
      if (lr0 + a > R || c0 + b - 1 >= N) continue;  // outside the block
      float best = d[a][b];
      // the moves of Grid2D.cpp:22-40 (axis moves first), taken backwards: from neighbour u into v
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        if (m >= 4 && !diag) break;
        const int di = m < 4 ? ((m & 1) ? 0 : (m == 0 ? 1 : -1)) : ((m & 1) ? 1 : -1);
        const int dj = m < 4 ? ((m & 1) ? (m == 1 ? 1 : -1) : 0) : ((m & 2) ? 1 : -1);
        if (!ex[a + di][b + dj]) continue;
        const float c = d[a + di][b + dj] + (m < 4 ? wa : wd);
        best = c < best ? c : best;
      }
      if (best < d[a][b]) {
        d[a][b] = best;
        changed = 1;
      }
    }
    if (!__syncthreads_or(changed)) break;
  }
  // write back what changed; note the edges that changed
#pragma unroll
  for (int q = 0; q < FT * FT / FIELD_THREADS; ++q) {
    const int k = tid + q * FIELD_THREADS;
    const int a = 1 + k / FT, b = 1 + k % FT;
    if (lr0 + a > R || c0 + b - 1 >= N) continue;
    const float v = d[a][b];
    if (v < orig[q]) {
      f[(size_t)(lr0 + a) * N + (c0 + b - 1)] = v;
      any = 1;
      if (a == 1 || a == FT || b == 1 || b == FT || lr0 + a == R || c0 + b - 1 == N - 1) edge = 1;
      if (lr0 + a == 1) top = 1;
      if (lr0 + a == R) bot = 1;
    }
  }
  __syncthreads();
  if (tid == 0 && any) {
    atomicOr(flags, 1 | (top ? 2 : 0) | (bot ? 4 : 0));
    // the tile itself is converged for its current apron; its neighbours may improve from
    // its new edge values
    if (edge)
      for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        if (dy == 0 && dx == 0) continue;
        const int y = ty + dy, x = tx + dx;
        if (y < 0 || y >= nty || x < 0 || x >= ntx) continue;
        if (atomicExch(&nxt[y * ntx + x], 1) == 0) atomicAdd(pending, 1);
      }
  }
}

// mark tile rows: all tiles (mode 0), the first tile row (1), the last (2)
__global__ __launch_bounds__(256) void k_field_activate(int* __restrict__ act, int ntx, int nty, int mode,
                                                        int* __restrict__ pending) {
  const int n = ntx * nty;
  for (int k = (int)(blockIdx.x * blockDim.x + threadIdx.x); k < n; k += (int)(gridDim.x * blockDim.x)) {
    const int y = k / ntx;
    const bool on = mode == 0 || (mode == 1 && y == 0) || (mode == 2 && y == nty - 1);
    if (on && atomicExch(&act[k], 1) == 0) atomicAdd(pending, 1);
  }
}

hipError_t launch_field_init(float* f, int N, int r0, int r1, int gi, int gj, hipStream_t st) {
  const size_t n = (size_t)(r1 - r0 + 2) * N;
  const int blocks = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(k_field_init, dim3(blocks), dim3(256), 0, st, f, N, r0, r1 - r0 + 2, gi, gj);
  return hipGetLastError();
}

int field_tiles(int N, int r0, int r1, int* ntx, int* nty) {
  *ntx = (N + FT - 1) / FT;
  *nty = (r1 - r0 + FT - 1) / FT;
  return *ntx * *nty;
}

hipError_t launch_field_activate(int* act, int ntx, int nty, int mode, int* pending, hipStream_t st) {
  const int n = ntx * nty;
  hipLaunchKernelGGL(k_field_activate, dim3((n + 255) / 256 < 1 ? 1 : ((n + 255) / 256 > 1024 ? 1024 : (n + 255) / 256)), dim3(256), 0, st, act, ntx,
                     nty, mode, pending);
  return hipGetLastError();
}

hipError_t launch_field_pass(const PlannerDev& P, float* f, int r0, int r1, const int* act, int* nxt, int* flags,
                             int* pending, hipStream_t st) {
  int ntx, nty;
  const int n = field_tiles(P.N, r0, r1, &ntx, &nty);
  hipLaunchKernelGGL(k_field_pass, dim3(n), dim3(FIELD_THREADS), 0, st, P, f, r0, r1, act, nxt, flags, pending);
  return hipGetLastError();
}

}  // namespace hastar
