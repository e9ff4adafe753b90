"""ctypes mirror of include/hastar.h (the C ABI of the MI355X planner library).

The structs here are plain data: tests and the oracle wrapper reuse them to build
identical parameter blocks for both sides.
"""
import ctypes as C
import math

import numpy as np


class HastarParams(C.Structure):
    """hastar_params (include/hastar.h) == HybridAStar<T> ctor args (HybridAStar.h:33-38)."""

    _fields_ = [
        ("dubins_shot_interval", C.c_int),
        ("dubins_shot_interval_decay", C.c_int),
        ("grid_resolution", C.c_float),
        ("obstacle_threshold", C.c_float),
        ("obstacle_prob_min", C.c_float),
        ("obstacle_prob_max", C.c_float),
        ("obstacle_prob_free", C.c_float),
        ("grid_size", C.c_int),
        ("grid_2d_allow_diag_moves", C.c_int),
        ("step_size", C.c_float),
        ("max_lat_acc", C.c_float),
        ("max_long_dec", C.c_float),
        ("wheelbase", C.c_float),
        ("rear_to_cg", C.c_float),
        ("apf_rep_constant", C.c_float),
        ("apf_active_angle", C.c_float),
        ("num_angle_bins", C.c_int),
        ("num_actions", C.c_int),
        ("num_steering", C.c_int),
        ("steering", C.POINTER(C.c_float)),
        ("curvature_weights", C.POINTER(C.c_float)),
        ("max_pops", C.c_int),
        ("max_astar_nodes", C.c_int),
        ("max_dubins_samples", C.c_int),
    ]


class HastarParamsF64(C.Structure):
    """hastar_params_f64 (include/hastar_f64.h) == HybridAStar<double> ctor args."""

    _fields_ = [(name, C.c_double if t is C.c_float else (C.POINTER(C.c_double) if name in ("steering", "curvature_weights")
                                                           else t))
                for name, t in HastarParams._fields_]


class HastarStats(C.Structure):
    _fields_ = [
        ("pops", C.c_longlong),
        ("successors", C.c_longlong),
        ("astar_pops", C.c_longlong),
        ("astar_searches", C.c_longlong),
        ("shots", C.c_longlong),
        ("closed_size", C.c_longlong),
        ("pop_digest", C.c_ulonglong),
        ("closed_digest", C.c_ulonglong),
        ("via_shot", C.c_int),
        ("status", C.c_int),
        ("parks", C.c_int),
        ("pad", C.c_int),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class HastarRelaxedOpts(C.Structure):
    """hastar_relaxed_opts (include/hastar.h): 0 selects a field's default."""
    _fields_ = [
        ("delta", C.c_float),
        ("h_stop", C.c_float),
        ("max_nodes", C.c_int),
        ("max_rounds", C.c_int),
        ("h_weight", C.c_float),
        ("reuse_heuristic", C.c_int),
        ("h_coarse", C.c_int),
        ("reverse_cost", C.c_float),
        ("gear_cost", C.c_float),
    ]


class PlannerConfig:
    """Python-side planner configuration; owns the float arrays the struct points to."""

    def __init__(self, *, dubins_shot_interval=300, dubins_shot_interval_decay=10, grid_resolution=0.5,
                 obstacle_threshold=0.75, obstacle_prob_min=0.1, obstacle_prob_max=0.95,
                 obstacle_prob_free=0.4, grid_size=60, grid_2d_allow_diag_moves=True, step_size=0.75,
                 max_lat_acc=4.0, max_long_dec=2.0, wheelbase=2.269, rear_to_cg=1.1, apf_rep_constant=1.0,
                 apf_active_angle=None, num_angle_bins=72, num_actions=1, steering=None,
                 curvature_weights=None, max_pops=0, max_astar_nodes=0, max_dubins_samples=0):
        if apf_active_angle is None:
            apf_active_angle = float(np.float32(math.pi / 4))  # static_cast<float>(M_PI/4)
        if steering is None:
            steering = steering_from_degrees([-30.0, -15.0, 0.0, 15.0, 30.0])
        if curvature_weights is None:
            curvature_weights = [0.0] * len(steering)
        if len(curvature_weights) != len(steering):
            raise ValueError("curvature_weights must have one entry per steering angle")
        self.steering = np.ascontiguousarray(steering, dtype=np.float32)
        self.curvature_weights = np.ascontiguousarray(curvature_weights, dtype=np.float32)
        # the same arguments as doubles, unrounded (HybridAStar<double>, include/hastar_f64.h)
        self.steering64 = np.ascontiguousarray(steering, dtype=np.float64)
        self.curvature_weights64 = np.ascontiguousarray(curvature_weights, dtype=np.float64)
        self.values = dict(
            dubins_shot_interval=int(dubins_shot_interval),
            dubins_shot_interval_decay=int(dubins_shot_interval_decay),
            grid_resolution=grid_resolution, obstacle_threshold=obstacle_threshold,
            obstacle_prob_min=obstacle_prob_min, obstacle_prob_max=obstacle_prob_max,
            obstacle_prob_free=obstacle_prob_free, grid_size=int(grid_size),
            grid_2d_allow_diag_moves=int(bool(grid_2d_allow_diag_moves)), step_size=step_size,
            max_lat_acc=max_lat_acc, max_long_dec=max_long_dec, wheelbase=wheelbase, rear_to_cg=rear_to_cg,
            apf_rep_constant=apf_rep_constant, apf_active_angle=apf_active_angle,
            num_angle_bins=int(num_angle_bins), num_actions=int(num_actions),
            max_pops=int(max_pops), max_astar_nodes=int(max_astar_nodes),
            max_dubins_samples=int(max_dubins_samples))

    @property
    def grid_size(self):
        return self.values["grid_size"]

    def struct(self):
        p = HastarParams(**self.values)
        p.num_steering = len(self.steering)
        p.steering = self.steering.ctypes.data_as(C.POINTER(C.c_float))
        p.curvature_weights = self.curvature_weights.ctypes.data_as(C.POINTER(C.c_float))
        return p


    def struct_f64(self):
        """hastar_params_f64 of the same arguments (the Python floats as doubles)."""
        p = HastarParamsF64(**{k: v for k, v in self.values.items()})
        p.num_steering = len(self.steering64)
        p.steering = self.steering64.ctypes.data_as(C.POINTER(C.c_double))
        p.curvature_weights = self.curvature_weights64.ctypes.data_as(C.POINTER(C.c_double))
        return p


def steering_from_degrees(deg):
    """`angle = angle * M_PI/180.0f` on a float (test_hybrid_astar.cpp:36-39)."""
    return [float(np.float32(float(np.float32(d)) * math.pi / 180.0)) for d in deg]


def steering_from_degrees_f64(deg):
    """`angle * deg_to_rad` with T = double (local_planner.cpp:143-146)."""
    return [float(d) * (math.pi / 180.0) for d in deg]


def fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def iptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))
