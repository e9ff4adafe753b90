// hastar_libm64.h — the f64 libm of the double planner's device code (hastar_f64.hip,
// hastar_dubins_f64.h): sin, cos, atan2, acos, hypot as the reference's HybridAStar<double> calls
// them (Dubins.cpp:23-33, 185-263, 331-417; Grid3D.cpp:212-213).
//
// These are the device libm's routines.  They agree with the host glibc 2.35 on most arguments,
// not on all (tools/libm64_fingerprint.hip measures how often they differ).
#pragma once
#include <hip/hip_runtime.h>

namespace gm64 {
__host__ __device__ __forceinline__ double sin(double x) { return ::sin(x); }
__host__ __device__ __forceinline__ double cos(double x) { return ::cos(x); }
__host__ __device__ __forceinline__ double atan2(double y, double x) { return ::atan2(y, x); }
__host__ __device__ __forceinline__ double acos(double x) { return ::acos(x); }
__host__ __device__ __forceinline__ double hypot(double x, double y) { return ::hypot(x, y); }
}  // namespace gm64
