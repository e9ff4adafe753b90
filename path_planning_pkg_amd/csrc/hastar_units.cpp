// hastar_units.cpp — host side of include/hastar_units.h: Dubins<T> and VehicleModel<T>
// entry points over the unit kernels (hastar_units.hip).  Each call stages its inputs on
// its own stream, launches, and copies the results back (these are small, synchronous
// calls, like the reference's member functions).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hastar_units.h"
#include "glibc_mathf.h"
#include "hastar_units_dev.h"

using namespace hastar;

namespace {
thread_local std::string u_err;
int ufail(int code, const std::string& m) {
  u_err = m;
  return code;
}
#define UCHK(expr)                                                                                      \
  do {                                                                                                  \
    hipError_t e_ = (expr);                                                                             \
    if (e_ != hipSuccess) return ufail(HASTAR_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

int use_device(int device) {
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0)
    return ufail(HASTAR_EDEVICE, "no HIP device available (this library has no CPU path)");
  if (device < 0 || device >= nd) return ufail(HASTAR_EINVAL, "device ordinal out of range");
  UCHK(hipSetDevice(device));
  return 0;
}

// one device allocation holding a call's staged buffers, freed at scope exit
struct Scratch {
  char* base = nullptr;
  size_t used = 0, cap = 0;
  ~Scratch() {
    if (base) hipFree(base);
  }
  hipError_t init(size_t bytes) {
    cap = bytes + 4096;
    return hipMalloc(reinterpret_cast<void**>(&base), cap);
  }
  template <class T>
  T* take(size_t n) {
    used = (used + 255) & ~(size_t)255;
    T* p = reinterpret_cast<T*>(base + used);
    used += n * sizeof(T);
    return p;
  }
};

template <class T>
int dubins_length(int device, T r, int n, const T* starts, const T goal[3], T* length, int* word, T* centres) {
  if (n < 0 || (n > 0 && (!starts || !goal || !length || !word))) return ufail(HASTAR_EINVAL, "dubins_length: bad argument");
  if (n == 0) return HASTAR_OK;
  if (int rc = use_device(device)) return rc;
  Scratch S;
  UCHK(S.init((size_t)n * (3 * sizeof(T) + sizeof(T) + sizeof(int)) + 1024));
  T* ds = S.take<T>((size_t)n * 3);
  T* dl = S.take<T>((size_t)n);
  int* dw = S.take<int>((size_t)n);
  UCHK(hipMemcpy(ds, starts, (size_t)n * 3 * sizeof(T), hipMemcpyHostToDevice));
  if constexpr (sizeof(T) == 4)
    UCHK(launch_dubins_len_f32(r, ds, n, goal[0], goal[1], goal[2], dl, dw, nullptr));
  else
    UCHK(launch_dubins_len_f64(r, ds, n, goal[0], goal[1], goal[2], dl, dw, nullptr));
  UCHK(hipMemcpy(length, dl, (size_t)n * sizeof(T), hipMemcpyDeviceToHost));
  UCHK(hipMemcpy(word, dw, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
  if (centres) {  // Dubins.cpp:76-87 (the same expressions as the kernels' first step)
    for (int i = 0; i < n; ++i) {
      const T sx = starts[3 * i], sy = starts[3 * i + 1], sh = starts[3 * i + 2];
      T* c = centres + 8 * i;
      T ss, cs, gs, gc;
      if constexpr (sizeof(T) == 4) {
        ss = gmath::g_sinf(sh);
        cs = gmath::g_cosf(sh);
        gs = gmath::g_sinf(goal[2]);
        gc = gmath::g_cosf(goal[2]);
      } else {
        ss = std::sin(sh);
        cs = std::cos(sh);
        gs = std::sin(goal[2]);
        gc = std::cos(goal[2]);
      }
      c[0] = sx + r * ss;
      c[1] = sy - r * cs;
      c[2] = sx - r * ss;
      c[3] = sy + r * cs;
      c[4] = goal[0] + r * gs;
      c[5] = goal[1] - r * gc;
      c[6] = goal[0] - r * gs;
      c[7] = goal[1] + r * gc;
    }
  }
  return HASTAR_OK;
}

template <class T>
int dubins_path(int device, T r, T step, const T s[3], const T g[3], T* xyh, T* curv, int cap, int* n, T* length,
                int* flag, int* word) {
  if (!s || !g || !n || !length || cap < 0 || (cap > 0 && (!xyh || !curv))) return ufail(HASTAR_EINVAL, "dubins_path: bad argument");
  if (int rc = use_device(device)) return rc;
  Scratch S;
  const int dcap = cap > 0 ? cap : 1;
  UCHK(S.init((size_t)dcap * 4 * sizeof(T) + 1024));
  T* dx = S.take<T>((size_t)dcap * 3);
  T* dc = S.take<T>((size_t)dcap);
  int* dn = S.take<int>(1);
  T* dl = S.take<T>(1);
  int* di = S.take<int>(2);
  if constexpr (sizeof(T) == 4)
    UCHK(launch_dubins_path_f32(r, step, s, g, dx, dc, cap, dn, dl, di, nullptr));
  else
    UCHK(launch_dubins_path_f64(r, step, s, g, dx, dc, cap, dn, dl, di, nullptr));
  int info[2];
  UCHK(hipMemcpy(n, dn, sizeof(int), hipMemcpyDeviceToHost));
  UCHK(hipMemcpy(length, dl, sizeof(T), hipMemcpyDeviceToHost));
  UCHK(hipMemcpy(info, di, sizeof(info), hipMemcpyDeviceToHost));
  if (flag) *flag = info[0];
  if (word) *word = info[1];
  if (*n > 0 && *n <= cap) {
    UCHK(hipMemcpy(xyh, dx, (size_t)(*n) * 3 * sizeof(T), hipMemcpyDeviceToHost));
    UCHK(hipMemcpy(curv, dc, (size_t)(*n) * sizeof(T), hipMemcpyDeviceToHost));
  } else if (*n < 0 || *n > cap) {
    if (*n > 0) *n = -*n;
    return ufail(HASTAR_ENOSPC, "dubins_path: buffer too small (*n = -required)");
  }
  return HASTAR_OK;
}
}  // namespace

struct hastar_vehicle_s {
  int device = 0;
  bool dbl = false;
  int nsteer = 0, bins = 0, na = 0;
  double prec = 0;
  void* slab = nullptr;
  VehicleTablesT<float> vf{};
  VehicleTablesT<double> vd{};
  std::vector<double> curv_abs;
};

namespace {
// VehicleModel ctor (VehicleModel.cpp:7-47) on the host, with the reference's own
// expression types: T = float uses the bit-faithful glibc float ports (the search
// kernel's tables are built the same way in hastar_create_f32), T = double the host libm.
template <class T>
int vehicle_create(int device, T ts, T a_lat, T a_dec, T wb, T lr, int bins, int na, int ns, const T* steer, const T* w,
                   hastar_vehicle* out) {
  (void)a_dec;  // stored by the reference, unused by its member functions
  if (!out || ns < 1 || !steer || !w || bins < 1 || na < 0 || !(ts > 0)) return ufail(HASTAR_EINVAL, "vehicle_create: bad argument");
  *out = nullptr;
  if (int rc = use_device(device)) return rc;
  std::vector<T> beta(ns), curv(ns), dth(ns), cost(ns), ca(ns), off((size_t)ns * (bins + 1) * 2, T(0));
  const T prec = (T)(2 * M_PI / bins);
  for (int i = 0; i < ns; ++i) {
    if constexpr (sizeof(T) == 4) {
      beta[i] = gmath::g_atan2f(lr * std::tan(steer[i]), wb);
      curv[i] = gmath::g_cosf(beta[i]) * std::tan(steer[i]) / wb;
    } else {
      beta[i] = std::atan2(lr * std::tan(steer[i]), wb);
      curv[i] = std::cos(beta[i]) * std::tan(steer[i]) / wb;
    }
  }
  for (int i = 0; i < ns; ++i) {
    dth[i] = ts * curv[i];
    cost[i] = ts + w[i] * std::abs(curv[i]);
    ca[i] = std::abs(curv[i]);
    for (int j = 0; j < bins; ++j) {
      const T head = (T)(-M_PI + j * prec);
      const T dt = static_cast<T>(0.001);
      T ox = 0, oy = 0, hh = head;
      const int nup = static_cast<int>(ts / dt);
      for (int k = 0; k < nup; ++k) {
        if constexpr (sizeof(T) == 4) {
          ox += dt * gmath::g_cosf(beta[i] + hh);
          oy += dt * gmath::g_sinf(beta[i] + hh);
        } else {
          ox += dt * std::cos(beta[i] + hh);
          oy += dt * std::sin(beta[i] + hh);
        }
        hh += dt * curv[i];
      }
      off[2 * ((size_t)i * (bins + 1) + j)] = ox;
      off[2 * ((size_t)i * (bins + 1) + j) + 1] = oy;
    }
  }
  hastar_vehicle v = new hastar_vehicle_s();
  v->device = device;
  v->dbl = sizeof(T) == 8;
  v->nsteer = ns;
  v->bins = bins;
  v->na = na;
  v->prec = prec;
  v->curv_abs.assign(ca.begin(), ca.end());
  const size_t bytes = (off.size() + 4 * (size_t)ns) * sizeof(T);
  if (hipMalloc(&v->slab, bytes) != hipSuccess) {
    delete v;
    return ufail(HASTAR_ENOMEM, "vehicle_create: hipMalloc failed");
  }
  T* p = static_cast<T*>(v->slab);
  hipError_t e = hipMemcpy(p, off.data(), off.size() * sizeof(T), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(p + off.size(), dth.data(), ns * sizeof(T), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(p + off.size() + ns, cost.data(), ns * sizeof(T), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(p + off.size() + 2 * ns, ca.data(), ns * sizeof(T), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    hipFree(v->slab);
    delete v;
    return ufail(HASTAR_EDEVICE, std::string("vehicle_create: ") + hipGetErrorString(e));
  }
  VehicleTablesT<T> V{p, p + off.size(), p + off.size() + ns, p + off.size() + 2 * ns, ts, a_lat, a_lat * a_lat, prec,
                      ns, bins, na, 0};
  if constexpr (sizeof(T) == 4) v->vf = V;
  else v->vd = V;
  *out = v;
  return HASTAR_OK;
}

template <class T, class NodeT>
int vehicle_neighbors(hastar_vehicle v, const VehicleTablesT<T>& V, int n, const NodeT* nodes, int maxnb, NodeT* out,
                      int* counts, int* neglect) {
  static_assert(sizeof(NodeT) == sizeof(UnitNode3<T>), "node layout");
  if (!v || n < 0 || maxnb < 0 || (n > 0 && (!nodes || !counts || !neglect || (maxnb > 0 && !out))))
    return ufail(HASTAR_EINVAL, "vehicle_neighbors: bad argument");
  if (n == 0) return HASTAR_OK;
  if (int rc = use_device(v->device)) return rc;
  Scratch S;
  UCHK(S.init((size_t)n * (1 + (size_t)maxnb) * sizeof(NodeT) + (size_t)n * 8 + 2048));
  auto* dn = S.take<UnitNode3<T>>((size_t)n);
  auto* dout = S.take<UnitNode3<T>>((size_t)n * (maxnb > 0 ? maxnb : 1));
  int* dc = S.take<int>((size_t)n);
  int* dg = S.take<int>((size_t)n);
  UCHK(hipMemcpy(dn, nodes, (size_t)n * sizeof(NodeT), hipMemcpyHostToDevice));
  UCHK(launch_vehicle_neighbors<T>(V, dn, n, maxnb, dout, dc, dg, nullptr));
  if (maxnb > 0) UCHK(hipMemcpy(out, dout, (size_t)n * maxnb * sizeof(NodeT), hipMemcpyDeviceToHost));
  UCHK(hipMemcpy(counts, dc, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
  UCHK(hipMemcpy(neglect, dg, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
  return HASTAR_OK;
}

template <class T, class NodeT>
int vehicle_simulate(hastar_vehicle v, const VehicleTablesT<T>& V, int n, const NodeT* nodes, const int* acts, NodeT* out,
                     int* ok) {
  if (!v || n < 0 || (n > 0 && (!nodes || !acts || !out || !ok))) return ufail(HASTAR_EINVAL, "vehicle_simulate: bad argument");
  if (n == 0) return HASTAR_OK;
  if (int rc = use_device(v->device)) return rc;
  Scratch S;
  UCHK(S.init((size_t)n * (2 * sizeof(NodeT) + 8) + 2048));
  auto* dn = S.take<UnitNode3<T>>((size_t)n);
  auto* dout = S.take<UnitNode3<T>>((size_t)n);
  int* da = S.take<int>((size_t)n);
  int* dk = S.take<int>((size_t)n);
  UCHK(hipMemcpy(dn, nodes, (size_t)n * sizeof(NodeT), hipMemcpyHostToDevice));
  UCHK(hipMemcpy(da, acts, (size_t)n * sizeof(int), hipMemcpyHostToDevice));
  UCHK(launch_vehicle_simulate<T>(V, dn, da, n, dout, dk, nullptr));
  UCHK(hipMemcpy(out, dout, (size_t)n * sizeof(NodeT), hipMemcpyDeviceToHost));
  UCHK(hipMemcpy(ok, dk, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
  return HASTAR_OK;
}
}  // namespace

extern "C" {

const char* hastar_units_last_error(void) { return u_err.c_str(); }

int hastar_dubins_length_f32(int device, float r, int n, const float* s, const float g[3], float* len, int* word,
                             float* centres) {
  return dubins_length<float>(device, r, n, s, g, len, word, centres);
}
int hastar_dubins_length_f64(int device, double r, int n, const double* s, const double g[3], double* len, int* word,
                             double* centres) {
  return dubins_length<double>(device, r, n, s, g, len, word, centres);
}
int hastar_dubins_path_f32(int device, float r, float step, const float s[3], const float g[3], float* xyh, float* curv,
                           int cap, int* n, float* len, int* flag, int* word) {
  return dubins_path<float>(device, r, step, s, g, xyh, curv, cap, n, len, flag, word);
}
int hastar_dubins_path_f64(int device, double r, double step, const double s[3], const double g[3], double* xyh,
                           double* curv, int cap, int* n, double* len, int* flag, int* word) {
  return dubins_path<double>(device, r, step, s, g, xyh, curv, cap, n, len, flag, word);
}
int hastar_vehicle_create_f32(int device, float ts, float a_lat, float a_dec, float wb, float lr, int bins, int na,
                              int ns, const float* steer, const float* w, hastar_vehicle* out) {
  return vehicle_create<float>(device, ts, a_lat, a_dec, wb, lr, bins, na, ns, steer, w, out);
}
int hastar_vehicle_create_f64(int device, double ts, double a_lat, double a_dec, double wb, double lr, int bins, int na,
                              int ns, const double* steer, const double* w, hastar_vehicle* out) {
  return vehicle_create<double>(device, ts, a_lat, a_dec, wb, lr, bins, na, ns, steer, w, out);
}
int hastar_vehicle_destroy(hastar_vehicle v) {
  if (!v) return ufail(HASTAR_EINVAL, "null vehicle");
  hipSetDevice(v->device);
  if (v->slab) hipFree(v->slab);
  delete v;
  return HASTAR_OK;
}
int hastar_vehicle_info(hastar_vehicle v, double* precision, int* default_action, int* nsteer) {
  if (!v) return ufail(HASTAR_EINVAL, "null vehicle");
  if (precision) *precision = v->prec;
  if (default_action) *default_action = v->nsteer / 2;  // VehicleModel.cpp:57-60
  if (nsteer) *nsteer = v->nsteer;
  return HASTAR_OK;
}
int hastar_vehicle_abs_curvatures(hastar_vehicle v, void* out) {
  if (!v || !out) return ufail(HASTAR_EINVAL, "bad argument");
  for (int i = 0; i < v->nsteer; ++i) {
    if (v->dbl) static_cast<double*>(out)[i] = v->curv_abs[i];
    else static_cast<float*>(out)[i] = (float)v->curv_abs[i];
  }
  return HASTAR_OK;
}
int hastar_vehicle_neighbors_f32(hastar_vehicle v, int n, const hastar_node3_f32* nodes, int maxnb,
                                 hastar_node3_f32* out, int* counts, int* neglect) {
  if (v && v->dbl) return ufail(HASTAR_EINVAL, "vehicle handle is double");
  return vehicle_neighbors<float>(v, v ? v->vf : VehicleTablesT<float>{}, n, nodes, maxnb, out, counts, neglect);
}
int hastar_vehicle_neighbors_f64(hastar_vehicle v, int n, const hastar_node3_f64* nodes, int maxnb,
                                 hastar_node3_f64* out, int* counts, int* neglect) {
  if (v && !v->dbl) return ufail(HASTAR_EINVAL, "vehicle handle is float");
  return vehicle_neighbors<double>(v, v ? v->vd : VehicleTablesT<double>{}, n, nodes, maxnb, out, counts, neglect);
}
int hastar_vehicle_simulate_f32(hastar_vehicle v, int n, const hastar_node3_f32* nodes, const int* acts,
                                hastar_node3_f32* out, int* ok) {
  if (v && v->dbl) return ufail(HASTAR_EINVAL, "vehicle handle is double");
  return vehicle_simulate<float>(v, v ? v->vf : VehicleTablesT<float>{}, n, nodes, acts, out, ok);
}
int hastar_vehicle_simulate_f64(hastar_vehicle v, int n, const hastar_node3_f64* nodes, const int* acts,
                                hastar_node3_f64* out, int* ok) {
  if (v && !v->dbl) return ufail(HASTAR_EINVAL, "vehicle handle is float");
  return vehicle_simulate<double>(v, v ? v->vd : VehicleTablesT<double>{}, n, nodes, acts, out, ok);
}

}  // extern "C"
