// hastar_f64_kernels.h — launchers of the double planner's kernels (hastar_f64.hip), called
// by its host runtime (hastar_f64.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include "hastar_f64_layout.h"

namespace hastar {

// VelocityGenerator<double> members (VelocityGenerator.cpp:7-14)
struct VelParams64 {
  double max_velocity, coast_velocity, max_lat_acc, max_lat_acc_sqr, max_long_acc, max_long_dec;
};

hipError_t launch64_search(const Planner64Dev* d_desc, int n, hipStream_t st);
hipError_t launch64_reconstruct(const Planner64Dev* d_desc, int n, hipStream_t st);
hipError_t launch64_init_nodemap(const Planner64Dev* d_desc, int N, hipStream_t st);
hipError_t launch64_decay(double* occ, size_t NN, double fr, double mn, double mx, hipStream_t st);
hipError_t launch64_relocate(int N, double c, double s, double ox, double oy, const double* src, double* dst,
                             int* winner, hipStream_t st);
hipError_t launch64_raster_boxes(double* occ, int* cnt, int N, const int* rp, const double* dl, int nbox, double c,
                                 double s, double mn, double mx, hipStream_t st);
hipError_t launch64_raster_lines(double* occ, int* cnt, int N, int n45, int n2, double res, const double* lp,
                                 const double* seq_len, const double* seq_wid, int stride, int nline, double mn,
                                 double mx, hipStream_t st);
hipError_t launch64_velocity(const VelParams64& vp, int n, const long long* off, const double* xyh, const double* curv,
                             const double* vel_init, const double* vmax_curr, const unsigned char* flags, double* vel,
                             unsigned char* feasible, hipStream_t st);

}  // namespace hastar
