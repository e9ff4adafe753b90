"""Python mirror of planning::HybridAStar<double> / VelocityGenerator<double> over the MI355X
C ABI (include/hastar_f64.h).

The reference instantiates both classes for double (HybridAStar.cpp:285-286,
VelocityGenerator.cpp:88-89; its ROS node's LocalPlanner<double>, local_planner.cpp:378-500,
uses them).  Same member names as planner.HybridAStar, with float64 arrays.  The search runs
on the GPU in f64; there is no CPU implementation behind these classes.
"""
import ctypes as C

import numpy as np

from .capi import HastarStats, PlannerConfig, dptr, iptr
from .planner import HASTAR_ENOSPC, HastarError, load_library

_bound = False


def _lib():
    global _bound
    L = load_library()
    if not _bound:
        vp, dp, ip = C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int)
        L.hastar64_create.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
        L.hastar64_destroy.argtypes = [vp]
        L.hastar64_update_goal.argtypes = [vp, dp, dp]
        L.hastar64_reset.argtypes = [vp]
        L.hastar64_update_boxes.argtypes = [vp, dp, dp, C.c_int, C.c_double]
        L.hastar64_update_lines.argtypes = [vp, dp, dp, C.c_int, C.c_double]
        L.hastar64_decay.argtypes = [vp]
        L.hastar64_get_obstacles.argtypes = [vp, dp]
        L.hastar64_find_path.argtypes = [vp, C.c_double, dp, dp, dp, C.c_int, ip, dp, ip, C.POINTER(HastarStats)]
        L.hastar64_copy_path.argtypes = [vp, dp, dp, C.c_int, ip]
        L.hastar64_grid_size.argtypes = [vp]
        L.hastar_velocity_profile_batch_f64.argtypes = [C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_longlong), dp, dp,
                                                        dp, dp, C.POINTER(C.c_ubyte), dp, C.POINTER(C.c_ubyte)]
        L.hastar64_debug_memo.argtypes = [vp, dp, C.POINTER(C.c_ubyte)]
        L.hastar64_debug_closed_keys.argtypes = [vp, ip, C.c_int]
        L.hastar64_debug_arena.argtypes = [vp, C.POINTER(C.c_longlong)]
        _bound = True
    return L


def _check(rc):
    if rc < 0:
        raise HastarError(rc, load_library().hastar_last_error().decode(errors="replace"))
    return rc


def _f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a.reshape(shape) if shape is not None else a


class HybridAStar64:
    """GPU planner handle with the member functions of planning::HybridAStar<double>."""

    def __init__(self, cfg: PlannerConfig, device: int = 0):
        self.cfg = cfg
        self._params = cfg.struct_f64()
        self.N = cfg.grid_size
        h = C.c_void_p()
        _check(_lib().hastar64_create(C.byref(self._params), device, C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            _lib().hastar64_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def update_goal(self, goal, start):  # HybridAStar.cpp:55-59
        _check(_lib().hastar64_update_goal(self.h, dptr(_f64(goal)), dptr(_f64(start))))

    def reset(self):  # HybridAStar.cpp:49-52
        _check(_lib().hastar64_reset(self.h))

    def update_obstacles(self, items=None, confidence=None, size=None, kind="boxes"):
        if items is None:
            return self.decay()
        if kind == "boxes":
            return self.update_boxes(items, confidence, size)
        return self.update_lines(items, confidence, size)

    def update_boxes(self, boxes, confidence, apf_added_radius):
        b, c = _f64(boxes, (-1, 4)), _f64(confidence)
        _check(_lib().hastar64_update_boxes(self.h, dptr(b), dptr(c), len(b), float(apf_added_radius)))

    def update_lines(self, lines, confidence, line_width):
        l, c = _f64(lines, (-1, 4)), _f64(confidence)
        _check(_lib().hastar64_update_lines(self.h, dptr(l), dptr(c), len(l), float(line_width)))

    def decay(self):
        _check(_lib().hastar64_decay(self.h))

    def get_obstacles(self):
        out = np.empty((self.N, self.N), np.float64)
        _check(_lib().hastar64_get_obstacles(self.h, dptr(out)))
        return out

    def find_path(self, vel_init, start, cap=4096):  # HybridAStar.cpp:68-88
        L = _lib()
        st = HastarStats()
        ln, ok = C.c_int(0), C.c_int(0)
        cost = C.c_double(0)
        xyh = np.empty((max(cap, 1), 3), np.float64)
        curv = np.empty(max(cap, 1), np.float64)
        rc = L.hastar64_find_path(self.h, float(vel_init), dptr(_f64(start)), dptr(xyh), dptr(curv), cap,
                                  C.byref(ln), C.byref(cost), C.byref(ok), C.byref(st))
        if rc == HASTAR_ENOSPC:
            cap = ln.value
            xyh = np.empty((cap, 3), np.float64)
            curv = np.empty(cap, np.float64)
            rc = L.hastar64_copy_path(self.h, dptr(xyh), dptr(curv), cap, C.byref(ln))
            st.status = 0
        _check(rc)
        n = ln.value
        return dict(cost=cost.value, ok=bool(ok.value), path=xyh[:n].copy(), curvature=curv[:n].copy(),
                    stats=st.as_dict())

    # ---- test hooks
    def memo(self):
        f = np.empty((self.N, self.N), np.float64)
        v = np.empty((self.N, self.N), np.uint8)
        _check(_lib().hastar64_debug_memo(self.h, dptr(f), v.ctypes.data_as(C.POINTER(C.c_ubyte))))
        return f, v

    def closed_keys(self, cap=1 << 20):
        out = np.empty((cap, 3), np.int32)
        n = _check(_lib().hastar64_debug_closed_keys(self.h, iptr(out), cap))
        return out[:min(n, cap)].copy()

    def arena(self):
        out = (C.c_longlong * 4)()
        _check(_lib().hastar64_debug_arena(self.h, out))
        return dict(open3=out[0], open2=out[1], dub=out[2], reruns=out[3])


class HastarVelocityParamsF64(C.Structure):
    """hastar_velocity_params_f64 (include/hastar_f64.h)."""
    _fields_ = [("max_velocity", C.c_double), ("coast_velocity", C.c_double), ("max_lat_acc", C.c_double),
                ("max_long_acc", C.c_double), ("max_long_dec", C.c_double)]


class VelocityGenerator64:
    """Mirror of planning::VelocityGenerator<double> (VelocityGenerator.h:10-28) on the GPU;
    returns (feasible, velocity) like planner.VelocityGenerator."""

    def __init__(self, max_velocity, coast_velocity, max_lat_acc, max_long_acc, max_long_dec, device=0):
        self.params = HastarVelocityParamsF64(max_velocity, coast_velocity, max_lat_acc, max_long_acc, max_long_dec)
        self.device = int(device)

    def generate_velocity_profile(self, vel_init, max_velocity_curr, path, curvature, coast_to_goal,
                                  stop_at_goal=False):
        ok, vel = self.generate_velocity_profiles([vel_init], [max_velocity_curr], [path], [curvature],
                                                  [coast_to_goal], [stop_at_goal])
        return bool(ok[0]), vel[0]

    def generate_velocity_profiles(self, vel_init, max_velocity_curr, paths, curvatures, coast_to_goal,
                                   stop_at_goal=None):
        n = len(paths)
        xyh = [_f64(p, (-1, 3)) for p in paths]
        cv = [_f64(c) for c in curvatures]
        lens = np.array([len(p) for p in xyh], np.int64)
        if any(len(c) != l for c, l in zip(cv, lens)):
            raise ValueError("path and curvature lengths differ")
        off = np.zeros(n + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        X = np.ascontiguousarray(np.concatenate(xyh) if n else np.zeros((0, 3)))
        K = np.ascontiguousarray(np.concatenate(cv) if n else np.zeros(0))
        stop = [False] * n if stop_at_goal is None else stop_at_goal
        flags = np.array([int(bool(c)) | (int(bool(s)) << 1) for c, s in zip(coast_to_goal, stop)], np.uint8)
        vel = np.empty(max(int(off[-1]), 1), np.float64)
        feas = np.zeros(n, np.uint8)
        u8 = C.POINTER(C.c_ubyte)
        _check(_lib().hastar_velocity_profile_batch_f64(
            self.device, C.byref(self.params), n, off.ctypes.data_as(C.POINTER(C.c_longlong)), dptr(X), dptr(K),
            dptr(_f64(vel_init)), dptr(_f64(max_velocity_curr)), flags.ctypes.data_as(u8), dptr(vel),
            feas.ctypes.data_as(u8)))
        return feas.astype(bool), [vel[off[i]:off[i + 1]] for i in range(n)]
