// hastar_units_dev.h — records shared by the unit kernels (hastar_units.hip) and their host
// side (hastar_units.cpp).  UnitNode3<T> has the layout of hastar_node3_f32 / _f64
// (include/hastar_units.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hastar {

template <class T>
struct UnitNode3 {  // Node3D<T> fields the vehicle model reads and writes (Node3D.h:17-24)
  T x, y, heading, g, vmin_sqr;
  int curvature_index, angle_bin;
};

// VehicleModel<T> tables (VehicleModel.cpp:7-47) in device memory
template <class T>
struct VehicleTablesT {
  const T* off;       // nsteer x (bins + 1) x {dx, dy}; row `bins` = (0, 0) (VehicleModel.cpp:145 reads past the end)
  const T* dth;       // nsteer  _offset_heading
  const T* cost;      // nsteer  _actions_cost
  const T* curv_abs;  // nsteer  _abs_curvatures
  T ts, a_lat, a_lat2, prec;
  int nsteer, bins, na, pad;
};

hipError_t launch_dubins_len_f32(float r, const float* s, int n, float gx, float gy, float gh, float* out, int* word,
                                 hipStream_t st);
hipError_t launch_dubins_len_f64(double r, const double* s, int n, double gx, double gy, double gh, double* out,
                                 int* word, hipStream_t st);
hipError_t launch_dubins_path_f32(float r, float step, const float s[3], const float g[3], float* xyh, float* curv,
                                  int cap, int* n_out, float* len_out, int* info, hipStream_t st);
hipError_t launch_dubins_path_f64(double r, double step, const double s[3], const double g[3], double* xyh,
                                  double* curv, int cap, int* n_out, double* len_out, int* info, hipStream_t st);
template <class T>
hipError_t launch_vehicle_neighbors(const VehicleTablesT<T>& V, const UnitNode3<T>* nodes, int n, int maxnb,
                                    UnitNode3<T>* out, int* counts, int* neglect, hipStream_t st);
template <class T>
hipError_t launch_vehicle_simulate(const VehicleTablesT<T>& V, const UnitNode3<T>* nodes, const int* act, int n,
                                   UnitNode3<T>* out, int* ok, hipStream_t st);

}  // namespace hastar
