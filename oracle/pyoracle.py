"""ctypes wrapper of oracle/build/libhastar_oracle.so — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as
the checker.  The product (path_planning_pkg_amd) never imports this module.
"""
import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

from path_planning_pkg_amd.capi import HastarStats, dptr, fptr, iptr

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "libhastar_oracle.so"
# the timing build (-DORC_LEAN: no digests / statistics beyond the pop count), for cpu_baseline
LIB_LEAN = HERE / "build" / "libhastar_oracle_lean.so"
_libs = {}


def build(force=False):
    src = (HERE / "hastar_oracle.cpp").stat().st_mtime
    if force or any(not p.exists() or p.stat().st_mtime < src for p in (LIB, LIB_LEAN)):
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib(lean=False):
    """The checker build (default), or the lean timing build (lean=True: its stats carry no
    digests and no counters but pops)."""
    if lean not in _libs:
        path = LIB_LEAN if lean else LIB
        if not path.exists():
            build()
        L = C.CDLL(str(path))
        vp, fp, ip, dp = C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_int), C.POINTER(C.c_double)
        L.orc_create.restype = vp
        L.orc_create.argtypes = [C.c_void_p]
        for name in ("orc_destroy", "orc_reset", "orc_decay"):
            getattr(L, name).argtypes = [vp]
        L.orc_update_goal.argtypes = [vp, fp, fp]
        L.orc_update_boxes.argtypes = [vp, fp, fp, C.c_int, C.c_float]
        L.orc_update_lines.argtypes = [vp, fp, fp, C.c_int, C.c_float]
        L.orc_get_obstacles.argtypes = [vp, fp]
        L.orc_set_obstacles.argtypes = [vp, fp]
        L.orc_heuristic_field.argtypes = [vp, fp]
        L.orc_get_memo.argtypes = [vp, fp, C.POINTER(C.c_ubyte)]
        L.orc_apf_count.argtypes = [vp]
        L.orc_get_apf.argtypes = [vp, fp]
        L.orc_find_path.argtypes = [vp, C.c_float, fp, fp, fp, C.c_int, ip, fp, ip, C.POINTER(HastarStats), dp]
        L.orc_closed_keys.argtypes = [vp, ip, C.c_int]
        L.orc_motion_tables.restype = C.c_float
        L.orc_motion_tables.argtypes = [vp, fp, fp, fp, fp]
        L.orc_min_radius.restype = C.c_float
        L.orc_min_radius.argtypes = [vp]
        L.orc_field.argtypes = [vp, fp, C.c_int, fp]
        L.orc_dubins_len.argtypes = [C.c_float, C.c_float, fp, C.c_int, fp, fp, ip]
        L.orc_dubins_path_d.argtypes = [C.c_double, C.c_double, dp, dp, dp, C.c_int, dp, ip]
        L.orc_dubins_path_f.argtypes = [C.c_float, C.c_float, fp, fp, fp, fp, C.c_int, fp, ip]
        L.orc_vehicle_chain_d.argtypes = [C.c_double, C.c_double, C.c_double, C.c_double, C.c_int, C.c_int,
                                          dp, dp, C.c_int, C.c_double, C.c_int, ip, C.c_int, dp]
        L.orc_libm.argtypes = [C.c_int, fp, fp, fp, C.c_int]
        L.orc_velocity_profile.argtypes = [fp, C.c_float, C.c_float, fp, fp, C.c_int, C.c_int, C.c_int, fp]
        L.orc_set_max_pops.argtypes = [C.c_longlong]
        L.orc_grid2d_goal.argtypes = [vp, fp, fp]
        L.orc_grid2d_start.argtypes = [vp, fp, ip]
        L.orc_astar_cost.restype = C.c_float
        L.orc_astar_cost.argtypes = [vp, C.c_int, C.c_int]
        L.orc_astar_find_path.restype = C.c_float
        L.orc_astar_find_path.argtypes = [vp, fp, fp, C.c_int, fp, C.c_int, ip]
        L.orc_grid3d_neighbors.argtypes = [vp, fp, C.c_int, C.c_int, fp, ip, C.c_int, ip]
        L.orc_check_path.argtypes = [vp, fp, C.c_int]
        L.orc_vehicle_chain_f.argtypes = [C.c_float, C.c_float, C.c_float, C.c_float, C.c_int, C.c_int, fp, fp,
                                          C.c_int, C.c_float, ip, C.c_int, fp]
        L.orc64_create.restype = vp
        L.orc64_create.argtypes = [C.c_void_p]
        for name in ("orc64_destroy", "orc64_reset", "orc64_decay"):
            getattr(L, name).argtypes = [vp]
        L.orc64_update_goal.argtypes = [vp, dp, dp]
        L.orc64_update_boxes.argtypes = [vp, dp, dp, C.c_int, C.c_double]
        L.orc64_update_lines.argtypes = [vp, dp, dp, C.c_int, C.c_double]
        L.orc64_get_obstacles.argtypes = [vp, dp]
        L.orc64_get_memo.argtypes = [vp, dp, C.POINTER(C.c_ubyte)]
        L.orc64_find_path.argtypes = [vp, C.c_double, dp, dp, dp, C.c_int, ip, dp, ip, C.POINTER(HastarStats), dp]
        L.orc64_closed_keys.argtypes = [vp, ip, C.c_int]
        L.orc64_velocity_profile.argtypes = [dp, C.c_double, C.c_double, dp, dp, C.c_int, C.c_int, C.c_int, dp]
        L.orc_run_batch_threads.argtypes = [C.POINTER(C.c_void_p), C.c_int, fp, fp, C.c_int, C.c_int, dp, dp,
                                            C.POINTER(C.c_ulonglong), fp, ip]
        _libs[lean] = L
    return _libs[lean]


def _f32(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if shape is not None:
        a = a.reshape(shape)
    return a


class OraclePlanner:
    """CPU restatement of planning::HybridAStar<float> (same method names)."""

    def __init__(self, cfg, lean=False):
        self.cfg = cfg
        self._params = cfg.struct()
        self.N = cfg.grid_size
        self.lean = lean
        self._L = lib(lean)
        self.h = self._L.orc_create(C.byref(self._params))

    def close(self):
        if self.h:
            self._L.orc_destroy(self.h)
            self.h = None

    __del__ = close

    def update_goal(self, goal, start):
        self._L.orc_update_goal(self.h, fptr(_f32(goal)), fptr(_f32(start)))

    def reset(self):
        self._L.orc_reset(self.h)

    def update_boxes(self, boxes, conf, apf_added_radius):
        b = _f32(boxes, (-1, 4))
        c = _f32(conf)
        self._L.orc_update_boxes(self.h, fptr(b), fptr(c), len(b), apf_added_radius)

    def update_lines(self, lines, conf, width):
        l = _f32(lines, (-1, 4))
        c = _f32(conf)
        self._L.orc_update_lines(self.h, fptr(l), fptr(c), len(l), width)

    def decay(self):
        self._L.orc_decay(self.h)

    def get_obstacles(self):
        out = np.empty((self.N, self.N), np.float32)
        self._L.orc_get_obstacles(self.h, fptr(out))
        return out

    def heuristic_field(self):
        """The backward grid-distance field of the current map (orc_heuristic_field: a float
        Dijkstra from the goal cell), the checker of include/hastar.h's hastar_heuristic_field."""
        out = np.empty((self.N, self.N), np.float32)
        self._L.orc_heuristic_field(self.h, fptr(out))
        return out

    def set_obstacles(self, occ):
        """Test hook: overwrite the log-odds map."""
        a = _f32(occ, (self.N, self.N))
        self._L.orc_set_obstacles(self.h, fptr(a))

    def get_memo(self):
        f = np.empty((self.N, self.N), np.float32)
        v = np.empty((self.N, self.N), np.uint8)
        self._L.orc_get_memo(self.h, fptr(f), v.ctypes.data_as(C.POINTER(C.c_ubyte)))
        return f, v

    def apf(self):
        n = self._L.orc_apf_count(self.h)
        out = np.empty((n, 3), np.float32)
        if n:
            self._L.orc_get_apf(self.h, fptr(out))
        return out

    def find_path(self, vel, start, cap=1 << 16):
        xyh = np.empty((cap, 3), np.float32)
        curv = np.empty(cap, np.float32)
        ln, ok = C.c_int(0), C.c_int(0)
        cost = C.c_float(0)
        st = HastarStats()
        wall = C.c_double(0)
        rc = self._L.orc_find_path(self.h, vel, fptr(_f32(start)), fptr(xyh), fptr(curv), cap, C.byref(ln),
                                 C.byref(cost), C.byref(ok), C.byref(st), C.byref(wall))
        if rc != 0:
            raise RuntimeError(f"oracle find_path rc={rc} len={ln.value}")
        n = ln.value
        return dict(cost=cost.value, ok=bool(ok.value), path=xyh[:n].copy(), curvature=curv[:n].copy(),
                    stats=st.as_dict(), wall_ms=wall.value)

    # ---- the stand-alone AStar<float> on this planner's plain Grid2D (AStar.h)
    def astar_goal_start(self, goal, start):
        """AStar::update_goal_start: re-orient (no relocation), soft-reset the start cell."""
        self._L.orc_grid2d_goal(self.h, fptr(_f32(goal)), fptr(_f32(start)))
        cell = np.zeros(2, np.int32)
        self._L.orc_grid2d_start(self.h, fptr(_f32(start)), iptr(cell))
        return int(cell[0]), int(cell[1])

    def astar_cost(self, i, j):
        return self._L.orc_astar_cost(self.h, int(i), int(j))

    def astar_find_path(self, goal, start, cost_only=False, cap=1 << 14):
        xy = np.zeros((cap, 2), np.float32)
        n = C.c_int(0)
        c = self._L.orc_astar_find_path(self.h, fptr(_f32(goal)), fptr(_f32(start)), int(bool(cost_only)), fptr(xy), cap,
                                      C.byref(n))
        return c, xy[:n.value].copy()

    def grid3d_neighbors(self, node):
        """Grid3D::get_neighbors of node = (x, y, h, g, vmin, ci, bin): (rows n x 7 as
        (x, y, h, g, vmin) floats + (ci, bin) ints, cells n x 2, neglect)."""
        out = np.zeros((64, 7), np.float32)
        cells = np.zeros((64, 2), np.int32)
        ng = C.c_int(0)
        n = self._L.orc_grid3d_neighbors(self.h, fptr(_f32(node[:5])), int(node[5]), int(node[6]), fptr(out), iptr(cells),
                                       64, C.byref(ng))
        return out[:n].copy(), cells[:n].copy(), bool(ng.value)

    def check_path(self, xyh):
        return bool(self._L.orc_check_path(self.h, fptr(_f32(xyh, (-1, 3))), len(xyh)))

    def closed_keys(self, cap=1 << 20):
        out = np.empty((cap, 3), np.int32)
        n = self._L.orc_closed_keys(self.h, iptr(out), cap)
        return out[:min(n, cap)].copy()

    def motion_tables(self):
        ns = len(self.cfg.steering)
        bins = self.cfg.values["num_angle_bins"]
        off = np.empty((ns, bins + 1, 2), np.float32)
        dth = np.empty(ns, np.float32)
        cost = np.empty(ns, np.float32)
        ca = np.empty(ns, np.float32)
        prec = self._L.orc_motion_tables(self.h, fptr(off), fptr(dth), fptr(cost), fptr(ca))
        return dict(offsets=off, dtheta=dth, cost=cost, curv_abs=ca, precision=prec)

    def min_radius(self):
        return self._L.orc_min_radius(self.h)

    def field(self, poses):
        p = _f32(poses, (-1, 3))
        out = np.empty(len(p), np.float32)
        self._L.orc_field(self.h, fptr(p), len(p), fptr(out))
        return out


def dubins_len(r_min, step, starts, goal):
    s = _f32(starts, (-1, 3))
    out = np.empty(len(s), np.float32)
    word = np.empty(len(s), np.int32)
    lib().orc_dubins_len(r_min, step, fptr(s), len(s), fptr(_f32(goal)), fptr(out), iptr(word))
    return out, word


def dubins_path_f(r_min, step, start, goal, cap=1 << 16):
    xyh = np.empty((cap, 3), np.float32)
    curv = np.empty(cap, np.float32)
    length = C.c_float(0)
    flag = C.c_int(0)
    n = lib().orc_dubins_path_f(r_min, step, fptr(_f32(start)), fptr(_f32(goal)), fptr(xyh), fptr(curv), cap,
                                C.byref(length), C.byref(flag))
    return xyh[:n].copy(), curv[:n].copy(), length.value, bool(flag.value)


def dubins_path_d(r_min, step, start, goal, cap=4096):
    dp = C.POINTER(C.c_double)
    out = np.empty((cap, 3), np.float64)
    length = C.c_double(0)
    word = C.c_int(0)
    s = np.ascontiguousarray(start, np.float64)
    g = np.ascontiguousarray(goal, np.float64)
    n = lib().orc_dubins_path_d(r_min, step, s.ctypes.data_as(dp), g.ctypes.data_as(dp), out.ctypes.data_as(dp),
                                cap, C.byref(length), C.byref(word))
    return out[:n].copy(), length.value, word.value


def vehicle_chain_d(ts, a_lat, wheelbase, rear_to_cg, bins, na, steering, weights, vmin0, ci0, actions):
    dp = C.POINTER(C.c_double)
    st = np.ascontiguousarray(steering, np.float64)
    w = np.ascontiguousarray(weights, np.float64)
    acts = np.ascontiguousarray(actions, np.int32)
    out = np.empty((len(acts) + 1, 2), np.float64)
    n = lib().orc_vehicle_chain_d(ts, a_lat, wheelbase, rear_to_cg, bins, na, st.ctypes.data_as(dp),
                                  w.ctypes.data_as(dp), len(st), vmin0, ci0, iptr(acts), len(acts),
                                  out.ctypes.data_as(dp))
    return out[:n].copy()




def set_max_pops(n):
    """Census tools only: stop oracle searches after n pops (0 = unlimited, the reference)."""
    lib().orc_set_max_pops(int(n))


def run_batch_threads(planners, vels, starts, replans, threads):
    """replans x (reset + find_path) of every planner on `threads` C++ threads (one planner
    per thread at a time).  Returns dict(pops, wall_s, plan_s_sum, plans, plan_ms[n, replans],
    digest / cost / ok of each planner's last replan)."""
    n = len(planners)
    hs = (C.c_void_p * n)(*[p.h for p in planners])
    v = _f32(vels)
    s = _f32(starts, (n, 3))
    out = np.zeros(4, np.float64)
    per = np.zeros((n, replans), np.float64)
    dig = np.zeros(n, np.uint64)
    cost = np.zeros(n, np.float32)
    ok = np.zeros(n, np.int32)
    dp = C.POINTER(C.c_double)
    L = planners[0]._L if planners else lib()  # the planners' own build
    L.orc_run_batch_threads(hs, n, fptr(v), fptr(s), int(replans), int(threads), out.ctypes.data_as(dp),
                                per.ctypes.data_as(dp), dig.ctypes.data_as(C.POINTER(C.c_ulonglong)), fptr(cost),
                                iptr(ok))
    return dict(pops=int(out[0]), wall_s=float(out[1]), plan_s_sum=float(out[2]), plans=int(out[3]), plan_ms=per,
                digest=dig, cost=cost, ok=ok.astype(bool))


def vehicle_chain_f(ts, a_lat, wheelbase, rear_to_cg, bins, na, steering, weights, vmin0, actions):
    st = _f32(steering)
    w = _f32(weights)
    acts = np.ascontiguousarray(actions, np.int32)
    out = np.empty((len(acts) + 1, 2), np.float32)
    n = lib().orc_vehicle_chain_f(ts, a_lat, wheelbase, rear_to_cg, bins, na, fptr(st), fptr(w), len(st), vmin0,
                                  iptr(acts), len(acts), fptr(out))
    return out[:n].copy()


def velocity_profile(params, vel_init, max_velocity_curr, xyh, curv, coast_to_goal, stop_at_goal=False):
    """VelocityGenerator<float>::generate_velocity_profile (VelocityGenerator.cpp:19-84).
    params = (max_velocity, coast_velocity, max_lat_acc, max_long_acc, max_long_dec).
    Returns (feasible, velocity) for a goal -> start path."""
    prm = _f32(params)
    xyh = _f32(xyh, (-1, 3))
    curv = _f32(curv)
    assert len(curv) == len(xyh) and len(xyh) > 0
    out = np.empty(len(xyh), np.float32)
    ok = lib().orc_velocity_profile(fptr(prm), vel_init, max_velocity_curr, fptr(xyh), fptr(curv), len(xyh),
                                    int(bool(coast_to_goal)), int(bool(stop_at_goal)), fptr(out))
    return bool(ok), out


def libm(fn, a, b=None):
    """glibc values of the function numbered as in hastar_test_math."""
    a = _f32(a)
    bb = _f32(b) if b is not None else a
    out = np.empty_like(a)
    lib().orc_libm(fn, fptr(a), fptr(bb), fptr(out), len(a))
    return out


def _f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None:
        a = a.reshape(shape)
    return a


class OraclePlanner64:
    """CPU restatement of planning::HybridAStar<double> (same method names, float64 arrays):
    the checker of path_planning_pkg_amd.planner64.HybridAStar64."""

    def __init__(self, cfg):
        self.cfg = cfg
        self._params = cfg.struct_f64()
        self.N = cfg.grid_size
        self.h = lib().orc64_create(C.byref(self._params))

    def close(self):
        if self.h:
            lib().orc64_destroy(self.h)
            self.h = None

    __del__ = close

    def update_goal(self, goal, start):
        lib().orc64_update_goal(self.h, dptr(_f64(goal)), dptr(_f64(start)))

    def reset(self):
        lib().orc64_reset(self.h)

    def update_boxes(self, boxes, conf, apf_added_radius):
        b = _f64(boxes, (-1, 4))
        lib().orc64_update_boxes(self.h, dptr(b), dptr(_f64(conf)), len(b), apf_added_radius)

    def update_lines(self, lines, conf, width):
        l = _f64(lines, (-1, 4))
        lib().orc64_update_lines(self.h, dptr(l), dptr(_f64(conf)), len(l), width)

    def decay(self):
        lib().orc64_decay(self.h)

    def get_obstacles(self):
        out = np.empty((self.N, self.N), np.float64)
        lib().orc64_get_obstacles(self.h, dptr(out))
        return out

    def get_memo(self):
        f = np.empty((self.N, self.N), np.float64)
        v = np.empty((self.N, self.N), np.uint8)
        lib().orc64_get_memo(self.h, dptr(f), v.ctypes.data_as(C.POINTER(C.c_ubyte)))
        return f, v

    def find_path(self, vel, start, cap=1 << 16):
        xyh = np.empty((cap, 3), np.float64)
        curv = np.empty(cap, np.float64)
        ln, ok = C.c_int(0), C.c_int(0)
        cost = C.c_double(0)
        st = HastarStats()
        wall = C.c_double(0)
        rc = lib().orc64_find_path(self.h, vel, dptr(_f64(start)), dptr(xyh), dptr(curv), cap, C.byref(ln),
                                   C.byref(cost), C.byref(ok), C.byref(st), C.byref(wall))
        if rc != 0:
            raise RuntimeError(f"oracle find_path rc={rc} len={ln.value}")
        n = ln.value
        return dict(cost=cost.value, ok=bool(ok.value), path=xyh[:n].copy(), curvature=curv[:n].copy(),
                    stats=st.as_dict(), wall_ms=wall.value)

    def closed_keys(self, cap=1 << 20):
        out = np.empty((cap, 3), np.int32)
        n = lib().orc64_closed_keys(self.h, iptr(out), cap)
        return out[:min(n, cap)].copy()


def velocity_profile64(prm, vel_init, vmax_curr, xyh, curv, coast, stop):
    """VelocityGenerator<double>::generate_velocity_profile (VelocityGenerator.cpp:19-84)."""
    X = _f64(xyh, (-1, 3))
    K = _f64(curv)
    out = np.empty(len(X), np.float64)
    ok = lib().orc64_velocity_profile(dptr(_f64(prm)), vel_init, vmax_curr, dptr(X), dptr(K), len(X), int(coast),
                                      int(stop), dptr(out))
    return bool(ok), out
