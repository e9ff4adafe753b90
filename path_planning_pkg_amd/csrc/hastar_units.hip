// hastar_units.hip — device kernels behind the unit-level drop-in classes
// (include/hastar_units.h; include/path_planning_pkg/{Dubins,VehicleModel}.h):
//
//   Dubins<T>        Dubins.cpp:19-153, 180-563 — shortest CSC length of a batch of start
//                    poses (one thread each) and the sampled shortest path of one pose.
//   VehicleModel<T>  VehicleModel.cpp:63-136 — successors / one simulated action of a batch
//                    of nodes (one thread per node) from the handle's offset tables.
//
// T = float runs the same bit-exact expressions as the search kernel (the glibc float
// ports of glibc_mathf.h; the float Dubins reuses hastar_device.h).  T = double runs the
// ports of glibc 2.35's double sin/cos/atan2/acos (hastar_libm64.h), the functions the host's
// libm dispatches to, so double results are bit-identical to the reference's too.
#include <hip/hip_runtime.h>
#include "hastar_device.h"
#include "hastar_units_dev.h"
#include "hastar_dubins_f64.h"

namespace hastar {

// ------------------------------------------------------------------ math by type ------
template <class T> struct UM;
template <> struct UM<float> {
  __device__ static float sin(float x) { return g_sinf(x); }
  __device__ static float cos(float x) { return g_cosf(x); }
  __device__ static float atan2(float y, float x) { return g_atan2f(y, x); }
  __device__ static float acos(float x) { return g_acosf(x); }
  __device__ static float wrap(float a) { return wrap_pi_f(a); }
  __device__ static int bin(float h, float prec) { return heading_bin(h, prec); }
};
template <> struct UM<double> {
  __device__ static double sin(double x) { return gm64::sin(x); }
  __device__ static double cos(double x) { return gm64::cos(x); }
  __device__ static double atan2(double y, double x) { return gm64::atan2(y, x); }
  __device__ static double acos(double x) { return gm64::acos(x); }
  __device__ static double wrap(double a) { return wrap_pi_d(a); }
  // common.h:31-36 with T = double: round(h / prec) * prec, then (r + pi) / prec truncated
  __device__ static int bin(double h, double prec) {
    const double r = ::round(h / prec) * prec;
    return (int)((r + M_PI) / prec);
  }
};

// Dubins<double> (DubD, dub_shortest_d, dub_sample_d): hastar_dubins_f64.h, shared with the
// double search kernel (hastar_f64.hip).

__global__ void k_dubins_len_f32(float r, const float* __restrict__ s, int n, float gx, float gy, float gh,
                                 float* __restrict__ out, int* __restrict__ word) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int w = 0;
  float prm[4];
  out[i] = dubins_shortest(r, s[3 * i], s[3 * i + 1], s[3 * i + 2], gx, gy, gh, &w, prm);
  word[i] = w;
}
__global__ void k_dubins_len_f64(double r, const double* __restrict__ s, int n, double gx, double gy, double gh,
                                 double* __restrict__ out, int* __restrict__ word) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DubD D;
  D.r = r;
  D.step = D.ang_step = 1;
  out[i] = dub_shortest_d(D, s[3 * i], s[3 * i + 1], s[3 * i + 2], gx, gy, gh);
  word[i] = D.word;
}
// one path (Dubins::get_shortest_path, Dubins.cpp:125-153): float wave-parallel sampling
__global__ __launch_bounds__(64) void k_dubins_path_f32(float r, float step, float sx, float sy, float sh, float gx,
                                                        float gy, float gh, float* xyh, float* curv, int cap,
                                                        int* n_out, float* len_out, int* info) {
  PlannerDev P{};
  P.r_min = r;
  P.step = step;
  P.ang_step = step / r;
  int word = 0;
  float prm[4];
  const float len = dubins_shortest(r, sx, sy, sh, gx, gy, gh, &word, prm);
  const Centres C = dubins_centres(r, sx, sy, sh, gx, gy, gh);
  const int n = dubins_sample(P, C, word, prm, gp(xyh), gp(curv), cap, threadIdx.x);
  if (threadIdx.x == 0) {
    *n_out = n;
    *len_out = len;
    info[0] = fabsf(prm[1]) > (float)M_PI_2;
    info[1] = word;
  }
}
__global__ void k_dubins_path_f64(double r, double step, double sx, double sy, double sh, double gx, double gy,
                                  double gh, double* xyh, double* curv, int cap, int* n_out, double* len_out, int* info) {
  if (threadIdx.x != 0) return;
  DubD D;
  D.r = r;
  D.step = step;
  D.ang_step = step / r;
  const double len = dub_shortest_d(D, sx, sy, sh, gx, gy, gh);
  *n_out = dub_sample_d(D, xyh, curv, cap);
  *len_out = len;
  info[0] = ::fabs(D.prm[1]) > M_PI_2;
  info[1] = D.word;
}

// ------------------------------------------------------------- VehicleModel<T> -------
// VehicleModel::get_neighbors (VehicleModel.cpp:63-105): node i's successors go to
// out[i * maxnb ...]; counts[i] = how many; neglect[i] = the returned flag.
template <class T>
__device__ void vm_successor(const VehicleTablesT<T>& V, const UnitNode3<T>& nd, int a, T vm, UnitNode3<T>* o) {
  const T* off = V.off + 2 * ((size_t)a * (V.bins + 1) + nd.angle_bin);
  o->x = nd.x + off[0];
  o->y = nd.y + off[1];
  o->heading = UM<T>::wrap(nd.heading + V.dth[a]);
  o->g = nd.g + V.cost[a];
  o->vmin_sqr = vm;
  o->curvature_index = a;
  o->angle_bin = UM<T>::bin(o->heading, V.prec);
}
template <class T>
__global__ void k_vehicle_neighbors(VehicleTablesT<T> V, const UnitNode3<T>* __restrict__ nodes, int n, int maxnb,
                                    UnitNode3<T>* __restrict__ out, int* __restrict__ counts, int* __restrict__ neglect) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const UnitNode3<T> nd = nodes[i];
  int lo = nd.curvature_index - V.na;
  lo = lo < 0 ? 0 : lo;
  const int span = 2 * V.na + 1;
  const bool slow = nd.vmin_sqr < (T)1.0;
  int c = 0;
  for (int a = lo; a < lo + span && a < V.nsteer && c < maxnb; ++a) {
    T vm = 0;
    if (!slow) {
      const T lat = nd.vmin_sqr * V.curv_abs[a];
      if (lat > V.a_lat) continue;
      const T al = (T)::sqrt(1.0 - (double)((lat * lat) / V.a_lat2));
      vm = nd.vmin_sqr - 2 * al * V.ts;
    }
    vm_successor(V, nd, a, vm, &out[(size_t)i * maxnb + c]);
    ++c;
  }
  counts[i] = c;
  neglect[i] = slow ? 1 : 0;
}
// VehicleModel::simulate_action (VehicleModel.cpp:108-136)
template <class T>
__global__ void k_vehicle_simulate(VehicleTablesT<T> V, const UnitNode3<T>* __restrict__ nodes, const int* __restrict__ act,
                                   int n, UnitNode3<T>* __restrict__ out, int* __restrict__ ok) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const UnitNode3<T> nd = nodes[i];
  const int a = act[i];
  if (a < 0 || a >= V.nsteer) {
    ok[i] = 0;
    out[i] = nd;
    return;
  }
  T vm = 0;
  if ((double)nd.vmin_sqr > 1.0) {
    const T lat = nd.vmin_sqr * V.curv_abs[a];
    if (lat > V.a_lat) {
      ok[i] = 0;
      out[i] = nd;
      return;
    }
    const T al = (T)::sqrt(1.0 - (double)((lat * lat) / V.a_lat2));
    vm = nd.vmin_sqr - 2 * al * V.ts;
  }
  vm_successor(V, nd, a, vm, &out[i]);
  ok[i] = 1;
}

// ------------------------------------------------------------------ launchers ----------
hipError_t launch_dubins_len_f32(float r, const float* s, int n, float gx, float gy, float gh, float* out, int* word,
                                 hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_dubins_len_f32, dim3((n + 63) / 64), dim3(64), 0, st, r, s, n, gx, gy, gh, out, word);
  return hipGetLastError();
}
hipError_t launch_dubins_len_f64(double r, const double* s, int n, double gx, double gy, double gh, double* out,
                                 int* word, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_dubins_len_f64, dim3((n + 63) / 64), dim3(64), 0, st, r, s, n, gx, gy, gh, out, word);
  return hipGetLastError();
}
hipError_t launch_dubins_path_f32(float r, float step, const float s[3], const float g[3], float* xyh, float* curv,
                                  int cap, int* n_out, float* len_out, int* info, hipStream_t st) {
  hipLaunchKernelGGL(k_dubins_path_f32, dim3(1), dim3(64), 0, st, r, step, s[0], s[1], s[2], g[0], g[1], g[2], xyh, curv,
                     cap, n_out, len_out, info);
  return hipGetLastError();
}
hipError_t launch_dubins_path_f64(double r, double step, const double s[3], const double g[3], double* xyh,
                                  double* curv, int cap, int* n_out, double* len_out, int* info, hipStream_t st) {
  hipLaunchKernelGGL(k_dubins_path_f64, dim3(1), dim3(64), 0, st, r, step, s[0], s[1], s[2], g[0], g[1], g[2], xyh,
                     curv, cap, n_out, len_out, info);
  return hipGetLastError();
}
template <class T>
hipError_t launch_vehicle_neighbors(const VehicleTablesT<T>& V, const UnitNode3<T>* nodes, int n, int maxnb,
                                    UnitNode3<T>* out, int* counts, int* neglect, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_vehicle_neighbors<T>, dim3((n + 63) / 64), dim3(64), 0, st, V, nodes, n, maxnb, out, counts,
                     neglect);
  return hipGetLastError();
}
template <class T>
hipError_t launch_vehicle_simulate(const VehicleTablesT<T>& V, const UnitNode3<T>* nodes, const int* act, int n,
                                   UnitNode3<T>* out, int* ok, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_vehicle_simulate<T>, dim3((n + 63) / 64), dim3(64), 0, st, V, nodes, act, n, out, ok);
  return hipGetLastError();
}
template hipError_t launch_vehicle_neighbors<float>(const VehicleTablesT<float>&, const UnitNode3<float>*, int, int,
                                                    UnitNode3<float>*, int*, int*, hipStream_t);
template hipError_t launch_vehicle_neighbors<double>(const VehicleTablesT<double>&, const UnitNode3<double>*, int, int,
                                                     UnitNode3<double>*, int*, int*, hipStream_t);
template hipError_t launch_vehicle_simulate<float>(const VehicleTablesT<float>&, const UnitNode3<float>*, const int*, int,
                                                   UnitNode3<float>*, int*, hipStream_t);
template hipError_t launch_vehicle_simulate<double>(const VehicleTablesT<double>&, const UnitNode3<double>*, const int*,
                                                    int, UnitNode3<double>*, int*, hipStream_t);

}  // namespace hastar
