"""Python mirror of planning::HybridAStar<float> over the MI355X C ABI (include/hastar.h).

Method names and argument meaning follow the reference class (HybridAStar.h:33-50):
update_goal, reset, update_obstacles (three overloads, dispatched on arguments),
get_obstacles, find_path.  find_path returns the reference's (cost, success) pair plus
the path/curvature lists the reference fills in place, and the search statistics.

There is no CPU implementation behind this class: if libhastar_amd.so or a HIP device is
missing, construction raises.
"""
import ctypes as C
from pathlib import Path

import numpy as np

from .capi import HastarRelaxedOpts, HastarStats, PlannerConfig, fptr, iptr

import os

LIB_PATH = Path(os.environ.get("HASTAR_LIB", Path(__file__).resolve().parent / "lib" / "libhastar_amd.so"))
_lib = None

HASTAR_ENOSPC = -28
HASTAR_EOVERFLOW = -75


class HastarError(RuntimeError):
    def __init__(self, rc, msg):
        super().__init__(f"hastar rc={rc}: {msg}")
        self.rc = rc


def load_library():
    """Load libhastar_amd.so (in-tree build).  Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise FileNotFoundError(f"{LIB_PATH} missing: run __graft_entry__.build() (make -C path_planning_pkg_amd/csrc)")
    # torch (when installed) bundles its own copy of the HIP runtime, under the same soname
    # libamdhip64.so.7.  Loaded first, that copy also serves this library; loaded after
    # /opt/rocm's, it would be a second runtime in the process and find no GPU.  Importing
    # torch only loads its libraries; it does not touch the GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(str(LIB_PATH))
    vp, fp, ip = C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_int)
    L.hastar_create_f32.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
    L.hastar_destroy.argtypes = [vp]
    L.hastar_update_goal.argtypes = [vp, fp, fp]
    L.hastar_reset.argtypes = [vp]
    L.hastar_reset_batch.argtypes = [C.POINTER(C.c_void_p), C.c_int]
    L.hastar_set_cost_hint.argtypes = [vp, C.c_longlong]
    L.hastar_reserve.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_longlong]
    L.hastar_update_boxes.argtypes = [vp, fp, fp, C.c_int, C.c_float]
    L.hastar_update_lines.argtypes = [vp, fp, fp, C.c_int, C.c_float]
    L.hastar_decay.argtypes = [vp]
    L.hastar_find_path.argtypes = [vp, C.c_float, fp, fp, fp, C.c_int, ip, fp, ip, C.POINTER(HastarStats)]
    L.hastar_copy_path.argtypes = [vp, fp, fp, C.c_int, ip]
    L.hastar_find_path_batch.argtypes = [C.POINTER(C.c_void_p), C.c_int, fp, fp, fp, fp, C.c_int, ip, fp, ip,
                                         C.POINTER(HastarStats)]
    L.hastar_find_path_relaxed_batch.argtypes = [C.POINTER(C.c_void_p), C.c_int, fp, fp, fp, fp, C.c_int, ip, fp,
                                                 ip, C.POINTER(HastarStats), C.POINTER(HastarRelaxedOpts)]
    L.hastar_find_path_relaxed_batch_dir.argtypes = [C.POINTER(C.c_void_p), C.c_int, fp, fp, fp, fp, C.c_void_p,
                                                     C.c_int, ip, fp, ip, C.POINTER(HastarStats),
                                                     C.POINTER(HastarRelaxedOpts)]
    L.hastar_test_reeds_shepp.argtypes = [C.c_float, fp, C.c_int, fp, fp, ip, fp, fp]
    L.hastar_get_obstacles.argtypes = [vp, fp]
    L.hastar_grid_size.argtypes = [vp]
    L.hastar_set_row_window.argtypes = [vp, C.c_int, C.c_int]
    L.hastar_export_rows.argtypes = [vp, C.c_int, C.c_int, C.c_void_p]
    L.hastar_import_rows.argtypes = [vp, C.c_int, C.c_int, C.c_void_p]
    L.hastar_heuristic_field.argtypes = [vp, C.c_void_p, ip]
    L.hastar_field_rows.argtypes = [vp, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, ip, ip]
    L.hastar_relaxed_set_field.argtypes = [vp, C.c_void_p]
    L.hastar_last_error.restype = C.c_char_p
    L.hastar_last_search_ms.restype = C.c_float
    L.hastar_test_math.argtypes = [C.c_int, fp, fp, fp, C.c_int]
    L.hastar_test_field.argtypes = [vp, fp, C.c_int, fp]
    L.hastar_test_dubins_len.argtypes = [C.c_float, fp, C.c_int, fp, fp, ip]
    L.hastar_test_dubins_path.argtypes = [vp, fp, fp, fp, C.c_int, ip, fp, ip]
    L.hastar_debug_memo.argtypes = [vp, fp, C.POINTER(C.c_ubyte)]
    L.hastar_debug_apf.argtypes = [vp, fp, C.c_int]
    L.hastar_debug_motion.argtypes = [vp, fp, fp, fp, fp, fp, fp]
    L.hastar_debug_closed_keys.argtypes = [vp, ip, C.c_int]
    L.hastar_debug_cycles.argtypes = [vp, C.POINTER(C.c_ulonglong)]
    L.hastar_debug_astar_modes.argtypes = [vp, C.POINTER(C.c_longlong)]
    L.hastar_debug_timing.argtypes = [vp, C.POINTER(C.c_ulonglong)]
    L.hastar_debug_slots.argtypes = [vp, C.POINTER(C.c_longlong)]
    L.hastar_debug_head_arenas.argtypes = [vp, C.POINTER(C.c_longlong)]
    L.hastar_debug_hw_id.argtypes = [vp, ip]
    L.hastar_debug_split.argtypes = [vp, fp]
    L.hastar_debug_handoffs.argtypes = [vp, C.POINTER(C.c_int)]
    L.hastar_debug_relaxed_pool.argtypes = [vp, C.POINTER(C.c_longlong)]
    L.hastar_debug_pooled_resumes.argtypes = [C.POINTER(C.c_longlong)]
    L.hastar_velocity_profile_batch.argtypes = [C.c_int, C.POINTER(HastarVelocityParams), C.c_int,
                                                C.POINTER(C.c_longlong), fp, fp, fp, fp, C.POINTER(C.c_ubyte), fp,
                                                C.POINTER(C.c_ubyte)]
    L.hastar_grid3d_neighbors.argtypes = [vp, C.c_void_p, C.c_int, C.c_void_p, ip, ip, ip]
    L.hastar_grid3d_check_path.argtypes = [vp, fp, C.c_int, ip]
    L.hastar_grid3d_set_start_node.argtypes = [vp, fp, C.c_void_p, ip]
    L.hastar_create_batch_f32.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    hp = C.POINTER(C.c_void_p)
    L.hastar_update_goal_batch.argtypes = [hp, C.c_int, fp, fp]
    L.hastar_decay_batch.argtypes = [hp, C.c_int]
    L.hastar_update_boxes_batch.argtypes = [hp, C.c_int, fp, fp, ip, C.c_float]
    L.hastar_velocity_profile_last_batch.argtypes = [C.c_int, C.POINTER(HastarVelocityParams), C.c_int, fp, fp,
                                                     C.POINTER(C.c_ubyte), fp, C.POINTER(C.c_ubyte)]
    _lib = L
    return L


def _check(rc):
    if rc < 0:
        raise HastarError(rc, load_library().hastar_last_error().decode(errors="replace"))
    return rc


def _f32(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a.reshape(shape) if shape is not None else a


class HastarVelocityParams(C.Structure):
    """hastar_velocity_params (include/hastar.h)."""
    _fields_ = [("max_velocity", C.c_float), ("coast_velocity", C.c_float), ("max_lat_acc", C.c_float),
                ("max_long_acc", C.c_float), ("max_long_dec", C.c_float)]


class VelocityGenerator:
    """Mirror of planning::VelocityGenerator<float> (VelocityGenerator.h:10-28) on the GPU.

    generate_velocity_profile keeps the reference's arguments (VelocityGenerator.cpp:19-21)
    and returns (feasible, velocity) instead of filling `velocity` in place;
    generate_velocity_profiles runs many paths in one launch (one thread per path)."""

    def __init__(self, max_velocity, coast_velocity, max_lat_acc, max_long_acc, max_long_dec, device=0):
        self.params = HastarVelocityParams(max_velocity, coast_velocity, max_lat_acc, max_long_acc, max_long_dec)
        self.device = int(device)

    def generate_velocity_profile(self, vel_init, max_velocity_curr, path, curvature, coast_to_goal,
                                  stop_at_goal=False):
        ok, vel = self.generate_velocity_profiles([vel_init], [max_velocity_curr], [path], [curvature],
                                                  [coast_to_goal], [stop_at_goal])
        return bool(ok[0]), vel[0]

    def generate_velocity_profiles(self, vel_init, max_velocity_curr, paths, curvatures, coast_to_goal,
                                   stop_at_goal=None):
        n = len(paths)
        xyh = [_f32(p, (-1, 3)) for p in paths]
        cv = [_f32(c) for c in curvatures]
        lens = np.array([len(p) for p in xyh], np.int64)
        if any(len(c) != l for c, l in zip(cv, lens)):
            raise ValueError("path and curvature lengths differ")
        off = np.zeros(n + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        X = np.ascontiguousarray(np.concatenate(xyh) if n else np.zeros((0, 3), np.float32))
        K = np.ascontiguousarray(np.concatenate(cv) if n else np.zeros(0, np.float32))
        v0 = _f32(vel_init)
        vm = _f32(max_velocity_curr)
        stop = [False] * n if stop_at_goal is None else stop_at_goal
        flags = np.array([int(bool(c)) | (int(bool(s)) << 1) for c, s in zip(coast_to_goal, stop)], np.uint8)
        feas, vel = self.profile_packed(off, X, K, v0, vm, flags)
        return feas.astype(bool), [vel[off[i]:off[i + 1]] for i in range(n)]

    def profile_packed(self, off, xyh, curv, vel_init, max_velocity_curr, flags):
        """One hastar_velocity_profile_batch call on packed arrays: off (n+1, int64), xyh
        (points x 3, f32), curv, vel_init, max_velocity_curr (f32), flags (u8: bit 0 coast,
        bit 1 stop).  Returns (feasible u8[n], velocity f32[points])."""
        n = len(off) - 1
        off = np.ascontiguousarray(off, np.int64)
        X, K = _f32(xyh, (-1, 3)), _f32(curv)
        v0, vm = _f32(vel_init), _f32(max_velocity_curr)
        flags = np.ascontiguousarray(flags, np.uint8)
        if len(v0) != n or len(vm) != n or len(flags) != n or len(X) != off[-1] or len(K) != off[-1]:
            raise ValueError("profile_packed: inconsistent array lengths")
        vel = np.empty(int(off[-1]), np.float32)
        feas = np.zeros(n, np.uint8)
        u8 = C.POINTER(C.c_ubyte)
        _check(load_library().hastar_velocity_profile_batch(
            self.device, C.byref(self.params), n, off.ctypes.data_as(C.POINTER(C.c_longlong)), fptr(X), fptr(K),
            fptr(v0), fptr(vm), flags.ctypes.data_as(u8), fptr(vel), feas.ctypes.data_as(u8)))
        return feas, vel


    def profile_last_batch(self, lens, vel_init, max_velocity_curr, flags):
        """Profile the paths of this device's last find_path batch where they already are, in
        HBM (hastar_velocity_profile_last_batch; local_planner.cpp:316-323): lens = the
        batch's returned lengths.  Returns (feasible u8[n], velocity f32[sum(lens)])."""
        n = len(lens)
        v0, vm = _f32(vel_init), _f32(max_velocity_curr)
        flags = np.ascontiguousarray(flags, np.uint8)
        if len(v0) != n or len(vm) != n or len(flags) != n:
            raise ValueError("profile_last_batch: inconsistent array lengths")
        vel = np.empty(max(int(np.sum(lens)), 1), np.float32)
        feas = np.zeros(n, np.uint8)
        u8 = C.POINTER(C.c_ubyte)
        _check(load_library().hastar_velocity_profile_last_batch(
            self.device, C.byref(self.params), n, fptr(v0), fptr(vm), flags.ctypes.data_as(u8), fptr(vel),
            feas.ctypes.data_as(u8)))
        return feas, vel[:int(np.sum(lens))]


class HybridAStar:
    """GPU planner handle with the reference's member functions."""

    def __init__(self, cfg: PlannerConfig, device: int = 0):
        self.cfg = cfg
        self._params = cfg.struct()
        self.N = cfg.grid_size
        h = C.c_void_p()
        _check(load_library().hastar_create_f32(C.byref(self._params), device, C.byref(h)))
        self.h = h

    @classmethod
    def create_batch(cls, cfg: PlannerConfig, n: int, device: int = 0):
        """n planners with the same constructor arguments (hastar_create_batch_f32: one
        allocation for their maps, one shared copy of the motion tables)."""
        params = cfg.struct()
        hs = (C.c_void_p * n)()
        _check(load_library().hastar_create_batch_f32(C.byref(params), n, device, hs))
        out = []
        for i in range(n):
            o = cls.__new__(cls)
            o.cfg, o._params, o.N = cfg, params, cfg.grid_size
            o.h = C.c_void_p(hs[i])
            out.append(o)
        return out

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            load_library().hastar_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # HybridAStar::update_goal (HybridAStar.cpp:55-59)
    def update_goal(self, goal, start):
        _check(load_library().hastar_update_goal(self.h, fptr(_f32(goal)), fptr(_f32(start))))

    # HybridAStar::reset (HybridAStar.cpp:49-52)
    def reset(self):
        _check(load_library().hastar_reset(self.h))

    def set_cost_hint(self, hint):
        """Longest-first key of this planner's next batched search (hastar_set_cost_hint; the
        library sets it to each search's duration; 0 = unknown)."""
        _check(load_library().hastar_set_cost_hint(self.h, int(hint)))

    # the three update_obstacles overloads (HybridAStar.cpp:29-46)
    def update_obstacles(self, items=None, confidence=None, size=None, kind="boxes"):
        if items is None:
            return self.decay()
        if kind == "boxes":
            return self.update_boxes(items, confidence, size)
        return self.update_lines(items, confidence, size)

    def update_boxes(self, boxes, confidence, apf_added_radius):
        b = _f32(boxes, (-1, 4))
        c = _f32(confidence)
        _check(load_library().hastar_update_boxes(self.h, fptr(b), fptr(c), len(b), float(apf_added_radius)))

    def update_lines(self, lines, confidence, line_width):
        l = _f32(lines, (-1, 4))
        c = _f32(confidence)
        _check(load_library().hastar_update_lines(self.h, fptr(l), fptr(c), len(l), float(line_width)))

    def decay(self):
        _check(load_library().hastar_decay(self.h))

    def get_obstacles(self):
        out = np.empty((self.N, self.N), np.float32)
        _check(load_library().hastar_get_obstacles(self.h, fptr(out)))
        return out

    # ---- row-block sharding of the map build (include/hastar.h)
    def set_row_window(self, row0, row1):
        _check(load_library().hastar_set_row_window(self.h, int(row0), int(row1)))

    def export_rows(self, row0, row1, dst_ptr):
        """Copy log-odds rows [row0, row1) into the device buffer at `dst_ptr` (e.g. a
        torch tensor's data_ptr() on this planner's device); synchronous."""
        _check(load_library().hastar_export_rows(self.h, int(row0), int(row1), C.c_void_p(int(dst_ptr))))

    def import_rows(self, row0, row1, src_ptr):
        """Overwrite log-odds rows [row0, row1) from the device buffer at `src_ptr`; synchronous."""
        _check(load_library().hastar_import_rows(self.h, int(row0), int(row1), C.c_void_p(int(src_ptr))))

    # ---- the backward grid-distance field (include/hastar.h: hastar_heuristic_field)
    def heuristic_field(self, dst_ptr):
        """Write the N x N field to the device buffer at `dst_ptr` (row i = x cell); returns the
        relaxation passes it took.  Synchronous."""
        p = C.c_int(0)
        _check(load_library().hastar_heuristic_field(self.h, C.c_void_p(int(dst_ptr)), C.byref(p)))
        return p.value

    def field_rows(self, field_ptr, r0, r1, init, halo_changed=0):
        """Relax rows [r0, r1) of the device buffer at `field_ptr` ((r1 - r0 + 2) x N floats:
        halo row, block, halo row) until stable for its halos; returns (changed mask, passes)."""
        ch, p = C.c_int(0), C.c_int(0)
        _check(load_library().hastar_field_rows(self.h, C.c_void_p(int(field_ptr)), int(r0), int(r1), int(bool(init)),
                                                int(halo_changed), C.byref(ch), C.byref(p)))
        return ch.value, p.value

    def relaxed_set_field(self, src_ptr):
        """Install a whole field (device buffer, N x N) as the relaxed mode's heuristic (used by
        relaxed calls with reuse_heuristic=1, h_coarse=1 until reset / update_goal)."""
        _check(load_library().hastar_relaxed_set_field(self.h, C.c_void_p(int(src_ptr))))

    # HybridAStar::find_path (HybridAStar.cpp:68-88)
    def find_path(self, vel_init, start, cap=4096):
        L = load_library()
        st = HastarStats()
        ln, ok = C.c_int(0), C.c_int(0)
        cost = C.c_float(0)
        xyh = np.empty((max(cap, 1), 3), np.float32)
        curv = np.empty(max(cap, 1), np.float32)
        rc = L.hastar_find_path(self.h, float(vel_init), fptr(_f32(start)), fptr(xyh), fptr(curv), cap, C.byref(ln),
                                C.byref(cost), C.byref(ok), C.byref(st))
        if rc == HASTAR_ENOSPC and st.status == HASTAR_ENOSPC:  # our buffer was short: fetch again
            cap = ln.value
            xyh = np.empty((cap, 3), np.float32)
            curv = np.empty(cap, np.float32)
            rc = L.hastar_copy_path(self.h, fptr(xyh), fptr(curv), cap, C.byref(ln))
            st.status = 0
        if rc != HASTAR_EOVERFLOW:  # an explicit pop budget ended the search: stats["status"]
            _check(rc)
        n = ln.value
        return dict(cost=cost.value, ok=bool(ok.value), path=xyh[:n].copy(), curvature=curv[:n].copy(),
                    stats=st.as_dict())

    # ---- Grid3D<float> members on this planner (include/hastar_units.h) ----
    def grid3d_neighbors(self, node):
        """Grid3D::get_neighbors (Grid3D.cpp:47-74) of node = (x, y, h, g, vmin, ci, bin):
        (rows n x 7 float32 with ci / bin as int bit patterns, cells n x 2, neglect)."""
        inp = np.zeros(7, np.float32)
        inp[:5] = node[:5]
        inp[5:].view(np.int32)[:] = [int(node[5]), int(node[6])]
        out = np.zeros((64, 7), np.float32)
        cells = np.zeros((64, 2), np.int32)
        cnt, ng = C.c_int(0), C.c_int(0)
        _check(load_library().hastar_grid3d_neighbors(self.h, inp.ctypes.data, 64, out.ctypes.data, iptr(cells),
                                                      C.byref(cnt), C.byref(ng)))
        return out[:cnt.value].copy(), cells[:cnt.value].copy(), bool(ng.value)

    def check_path(self, xyh):
        free = C.c_int(0)
        p = _f32(xyh, (-1, 3))
        _check(load_library().hastar_grid3d_check_path(self.h, fptr(p), len(p), C.byref(free)))
        return bool(free.value)

    def set_start_node(self, start):
        """Grid3D::set_start_node: ((x, y, h, g, vmin, ci, bin), cell)."""
        out = np.zeros(7, np.float32)
        cell = np.zeros(2, np.int32)
        _check(load_library().hastar_grid3d_set_start_node(self.h, fptr(_f32(start)), out.ctypes.data, iptr(cell)))
        return out, (int(cell[0]), int(cell[1]))

    def copy_path(self, n):
        """The last search's path again (hastar_copy_path), into buffers of n poses."""
        xyh = np.empty((max(n, 1), 3), np.float32)
        curv = np.empty(max(n, 1), np.float32)
        ln = C.c_int(0)
        _check(load_library().hastar_copy_path(self.h, fptr(xyh), fptr(curv), n, C.byref(ln)))
        return xyh[:ln.value].copy(), curv[:ln.value].copy()

    # ---- debug / unit hooks (include/hastar_test.h)
    def memo(self):
        f = np.empty((self.N, self.N), np.float32)
        v = np.empty((self.N, self.N), np.uint8)
        _check(load_library().hastar_debug_memo(self.h, fptr(f), v.ctypes.data_as(C.POINTER(C.c_ubyte))))
        return f, v

    def apf(self, cap=1 << 16):
        out = np.empty((cap, 3), np.float32)
        n = _check(load_library().hastar_debug_apf(self.h, fptr(out), cap))
        return out[:n].copy()

    def motion_tables(self):
        ns = len(self.cfg.steering)
        bins = self.cfg.values["num_angle_bins"]
        off = np.empty((ns, bins + 1, 2), np.float32)
        dth, cost, ca = (np.empty(ns, np.float32) for _ in range(3))
        prec, rmin = C.c_float(0), C.c_float(0)
        _check(load_library().hastar_debug_motion(self.h, fptr(off), fptr(dth), fptr(cost), fptr(ca), C.byref(prec),
                                                  C.byref(rmin)))
        return dict(offsets=off, dtheta=dth, cost=cost, curv_abs=ca, precision=prec.value, r_min=rmin.value)

    def closed_keys(self, cap=1 << 20):
        out = np.empty((cap, 3), np.int32)
        n = _check(load_library().hastar_debug_closed_keys(self.h, iptr(out), cap))
        return out[:min(n, cap)].copy()

    def cycles(self):
        out = (C.c_ulonglong * 40)()
        _check(load_library().hastar_debug_cycles(self.h, out))
        return list(out)

    def astar_modes(self):
        out = (C.c_longlong * 2)()
        _check(load_library().hastar_debug_astar_modes(self.h, out))
        return {"migrations": out[0], "astar_pops_hbm": out[1]}

    @staticmethod
    def pooled_resumes():
        """Resume arenas carved from idle slot arenas so far (process-wide)."""
        out = C.c_longlong(0)
        _check(load_library().hastar_debug_pooled_resumes(C.byref(out)))
        return out.value

    def slots(self):
        """Search-slot pool of this planner's device (after a find_path)."""
        out = (C.c_longlong * 5)()
        _check(load_library().hastar_debug_slots(self.h, out))
        return {"resident_slots": out[0], "waves_per_cu": out[1], "arenas": out[2], "arena_mib": out[3],
                "head_cus": out[4]}

    def head_arenas(self):
        """The device's head arenas of split launches (after a search parked in one): how many,
        pool arenas carved per head arena (0 = an allocation of their own), their capacity in pops."""
        out = (C.c_longlong * 3)()
        _check(load_library().hastar_debug_head_arenas(self.h, out))
        return {"n": out[0], "pool_k": out[1], "grant": out[2]}

    def split_ms(self):
        """The device's last split launch: ms to head start, head end, bulk start, bulk end."""
        out = np.zeros(4, np.float32)
        _check(load_library().hastar_debug_split(self.h, fptr(out)))
        return [float(v) for v in out]

    def handoffs(self):
        """Searches the device's last split launch handed from batch-kernel slots to latency CUs."""
        out = C.c_int(0)
        _check(load_library().hastar_debug_handoffs(self.h, C.byref(out)))
        return int(out.value)

    def relaxed_pool(self):
        """The device's relaxed-mode arena pool: (arenas, MiB per arena)."""
        out = (C.c_longlong * 2)()
        _check(load_library().hastar_debug_relaxed_pool(self.h, out))
        return int(out[0]), int(out[1])

    def timing(self):
        """(t_start, t_end, slot) of the last search; times in 10 ns ticks."""
        out = (C.c_ulonglong * 3)()
        _check(load_library().hastar_debug_timing(self.h, out))
        return out[0], out[1], int(out[2])

    def hw_id(self):
        """(XCC, CU, SE, SH, SIMD) of the wavefront that ran the last search (HW_REG_XCC_ID /
        HW_REG_HW_ID: wave 3:0, SIMD 5:4, pipe 7:6, CU 11:8, SH 12, SE 15:13)."""
        v = C.c_int(0)
        _check(load_library().hastar_debug_hw_id(self.h, C.byref(v)))
        x = v.value
        return (x >> 16) & 0xF, (x >> 8) & 0xF, (x >> 13) & 0x7, (x >> 12) & 1, (x >> 4) & 3

    def field(self, poses):
        p = _f32(poses, (-1, 3))
        out = np.empty(len(p), np.float32)
        _check(load_library().hastar_test_field(self.h, fptr(p), len(p), fptr(out)))
        return out

    def dubins_path(self, start, cap=1 << 15):
        xyh = np.empty((cap, 3), np.float32)
        curv = np.empty(cap, np.float32)
        n, flag = C.c_int(0), C.c_int(0)
        length = C.c_float(0)
        _check(load_library().hastar_test_dubins_path(self.h, fptr(_f32(start)), fptr(xyh), fptr(curv), cap,
                                                      C.byref(n), C.byref(length), C.byref(flag)))
        k = n.value
        return xyh[:max(k, 0)].copy(), curv[:max(k, 0)].copy(), length.value, bool(flag.value)


class BatchResult:
    """Array view of one hastar_find_path_batch call (no per-planner Python objects).

    stats["status"][i] is planner i's own outcome: 0, HASTAR_EOVERFLOW (search ended by
    HASTAR_MAX_POPS_HARD or by device memory) or HASTAR_ENOSPC (its path did not fit `cap`:
    lens[i] is the length needed; result(i) fetches it with hastar_copy_path)."""

    def __init__(self, cost, ok, lens, xyh, curv, stats, kernel_ms, planners=None):
        self.cost, self.ok, self.lens, self.xyh, self.curv = cost, ok, lens, xyh, curv
        self.stats = stats            # numpy structured array with the hastar_stats fields
        self.kernel_ms = kernel_ms
        self.planners = planners

    def __len__(self):
        return len(self.cost)

    def result(self, i):
        k = int(self.lens[i])
        st = {name: self.stats[name][i].item() for name in self.stats.dtype.names}
        if st["status"] == HASTAR_ENOSPC and self.planners is not None and k > self.xyh.shape[1]:
            path, curv = self.planners[i].copy_path(k)
            st["status"] = 0
            return dict(cost=float(self.cost[i]), ok=bool(self.ok[i]), path=path, curvature=curv, stats=st)
        return dict(cost=float(self.cost[i]), ok=bool(self.ok[i]), path=self.xyh[i, :k].copy(),
                    curvature=self.curv[i, :k].copy(), stats=st)


class BatchBuffers:
    """Reusable host-side arguments/outputs of hastar_find_path_batch for a fixed list of
    planners (a replan loop calls the batch every tick: no per-call allocation, no page
    faults on fresh output arrays)."""

    def __init__(self, planners, cap=4096):
        n = len(planners)
        self.n, self.cap = n, cap
        self.hs = (C.c_void_p * n)(*[p.h.value for p in planners])
        # zero-filled here, so that their pages are mapped once at set-up, not at a first call's
        # path copies (np.empty maps nothing until the first write)
        self.xyh = np.zeros((n, cap, 3), np.float32)
        self.xyh.fill(0.0)
        self.curv = np.zeros((n, cap), np.float32)
        self.curv.fill(0.0)
        self.ln = np.zeros(n, np.int32)
        self.ok = np.zeros(n, np.int32)
        self.cost = np.zeros(n, np.float32)
        self.stats = (HastarStats * n)()
        self.st = np.ctypeslib.as_array(self.stats)


def reserve(planners, path_points=0):
    """hastar_reserve: size the device pool (search arenas, batch tables, packed-path buffers of
    `path_points` points) for a batched find_path of these planners, ahead of its first call."""
    n = len(planners)
    hs = (C.c_void_p * n)(*[p.h.value for p in planners])
    _check(load_library().hastar_reserve(hs, n, int(path_points)))


def reset_batch(planners_or_buffers):
    """reset() of every planner in one C call (hastar_reset_batch)."""
    b = planners_or_buffers
    if isinstance(b, BatchBuffers):
        hs, n = b.hs, b.n
    else:
        n = len(b)
        hs = (C.c_void_p * n)(*[p.h.value for p in b])
    _check(load_library().hastar_reset_batch(hs, n))


def _handles(planners_or_buffers):
    b = planners_or_buffers
    if isinstance(b, BatchBuffers):
        return b.hs, b.n
    return (C.c_void_p * len(b))(*[p.h.value for p in b]), len(b)


def update_goal_batch(planners, goals, starts):
    """update_goal of every planner in one call (hastar_update_goal_batch)."""
    hs, n = _handles(planners)
    _check(load_library().hastar_update_goal_batch(hs, n, fptr(_f32(goals, (n, 3))), fptr(_f32(starts, (n, 3)))))


def decay_batch(planners):
    """update_obstacles() of every planner in one launch (hastar_decay_batch)."""
    hs, n = _handles(planners)
    _check(load_library().hastar_decay_batch(hs, n))


def update_boxes_batch(planners, boxes_list, conf_list, apf_added_radius):
    """update_obstacles(boxes, confidence, r) of every planner (hastar_update_boxes_batch):
    boxes_list[i] is planner i's (k_i x 4) boxes, conf_list[i] its k_i confidences."""
    hs, n = _handles(planners)
    counts = np.array([len(b) for b in boxes_list], np.int32)
    B = _f32(np.concatenate([_f32(b, (-1, 4)) for b in boxes_list]) if n else np.zeros((0, 4)), (-1, 4))
    Cf = _f32(np.concatenate([_f32(c) for c in conf_list]) if n else np.zeros(0))
    if len(B) != counts.sum() or len(Cf) != counts.sum():
        raise ValueError("update_boxes_batch: box and confidence counts differ")
    _check(load_library().hastar_update_boxes_batch(hs, n, fptr(B), fptr(Cf), iptr(counts), float(apf_added_radius)))


def find_path_batch_arrays(planners, vels, starts, cap=4096, buffers=None):
    """hastar_find_path_batch with array outputs (BatchResult).  With `buffers` (a
    BatchBuffers of the same planners) the outputs are written into its arrays, which the
    returned BatchResult then views (valid until the next call with those buffers)."""
    L = load_library()
    b = buffers if buffers is not None else BatchBuffers(planners, cap)
    assert b.n == len(planners)
    v = _f32(vels)
    s = _f32(starts, (b.n, 3))
    rc = L.hastar_find_path_batch(b.hs, b.n, fptr(v), fptr(s), fptr(b.xyh), fptr(b.curv), b.cap, iptr(b.ln),
                                  fptr(b.cost), iptr(b.ok), b.stats)
    if rc not in (HASTAR_EOVERFLOW, HASTAR_ENOSPC):  # per-planner outcomes are in stats["status"]
        _check(rc)
    return BatchResult(b.cost, b.ok, b.ln, b.xyh, b.curv, b.st, float(L.hastar_last_search_ms()), planners)


def find_path_batch(planners, vels, starts, cap=4096, relaxed=None):
    """hastar_find_path_batch: one launch, one wavefront per planner.  relaxed: None for the
    exact mode, else a dict of hastar_relaxed_opts fields (may be empty) for the non-parity
    frontier-parallel mode (hastar_find_path_relaxed_batch, one workgroup per planner)."""
    L = load_library()
    n = len(planners)
    hs = (C.c_void_p * n)(*[p.h.value for p in planners])
    v = _f32(vels)
    s = _f32(starts, (n, 3))
    xyh = np.empty((n, cap, 3), np.float32)
    curv = np.empty((n, cap), np.float32)
    ln = np.zeros(n, np.int32)
    ok = np.zeros(n, np.int32)
    cost = np.zeros(n, np.float32)
    stats = (HastarStats * n)()
    if relaxed is None:
        rc = L.hastar_find_path_batch(hs, n, fptr(v), fptr(s), fptr(xyh), fptr(curv), cap, iptr(ln), fptr(cost),
                                      iptr(ok), stats)
    else:
        opts = HastarRelaxedOpts(**relaxed)
        dirs = np.zeros((n, cap), np.int8)
        rc = L.hastar_find_path_relaxed_batch_dir(hs, n, fptr(v), fptr(s), fptr(xyh), fptr(curv),
                                                  dirs.ctypes.data_as(C.c_void_p), cap, iptr(ln), fptr(cost),
                                                  iptr(ok), stats, C.byref(opts))
    if rc not in (HASTAR_EOVERFLOW, HASTAR_ENOSPC):  # per-planner outcomes are in stats[i]["status"]
        _check(rc)
    ms = float(L.hastar_last_search_ms())
    out = []
    for i in range(n):
        k = int(ln[i])
        st = stats[i].as_dict()
        if st["status"] == HASTAR_ENOSPC and k > cap:  # the path did not fit `cap`: fetch it
            path, cv = planners[i].copy_path(k)
            st["status"] = 0
        else:
            path, cv = xyh[i, :k].copy(), curv[i, :k].copy()
        out.append(dict(cost=float(cost[i]), ok=bool(ok[i]), path=path, curvature=cv, stats=st))
        if relaxed is not None and k <= cap:  # each pose's direction of travel (+1 / -1)
            out[-1]["direction"] = dirs[i, :k].copy()
    return out, ms


def gpu_math(fn, a, b=None):
    """Evaluate one libm port on the GPU (hastar_test_math)."""
    a = _f32(a)
    bb = _f32(b) if b is not None else a
    out = np.empty_like(a)
    _check(load_library().hastar_test_math(fn, fptr(a), fptr(bb), fptr(out), len(a)))
    return out


def gpu_reeds_shepp(r_min, starts, goal):
    """The relaxed mode's Reeds-Shepp code on the GPU (hastar_test_reeds_shepp): per start pose
    the shortest length (m), word, 5 segment lengths (radius units) and the grouped-lane lengths
    (groups of 4 and 16 lanes)."""
    s = _f32(starts, (-1, 3))
    n = len(s)
    ln = np.empty(n, np.float32)
    word = np.empty(n, np.int32)
    seg = np.empty((n, 5), np.float32)
    grp = np.empty((n, 2), np.float32)
    _check(load_library().hastar_test_reeds_shepp(float(r_min), fptr(s), n, fptr(_f32(goal)), fptr(ln), iptr(word),
                                                  fptr(seg), fptr(grp)))
    return ln, word, seg, grp


def gpu_dubins_len(r_min, starts, goal):
    s = _f32(starts, (-1, 3))
    out = np.empty(len(s), np.float32)
    word = np.empty(len(s), np.int32)
    _check(load_library().hastar_test_dubins_len(float(r_min), fptr(s), len(s), fptr(_f32(goal)), fptr(out),
                                                 iptr(word)))
    return out, word
