"""The reference's ROS node, src/local_planner.cpp, compiled UNCHANGED against the drop-in planner
headers (include/path_planning_pkg/HybridAStar.h, VelocityGenerator.h) and linked against
libhastar_amd.so — the boundary north_star names ("local_planner.cpp can link it unchanged").

local_planner.cpp compiles both LocalPlanner specializations (local_planner.h:98-135): the
float one (its main, :504-512) and the double one, whose members construct and call
HybridAStar<double> and VelocityGenerator<double> (:158-166, :378-500).  ROS is absent from the
image; tests/cxx/stubs/ stands in for ros/, tf/, std_msgs/, nav_msgs/, geometry_msgs/,
perception_pkg/ and path_planning_pkg/Waypoint.h.  The reference's lib/PedestrianHandler.cpp
(not on the planner path) is compiled from /root/reference over the drop-in value types.

CPU: the node and the test driver build (oracle/ref.mk, when /root/reference is present; the
build is the check), and the double drop-ins compile on their own.
GPU: the prebuilt driver (oracle/_ref/local_planner_driver, which runs the node's own callbacks
and run() loop on a scripted scenario) publishes the trajectory the oracle predicts for the same
call sequence, bit for bit for LocalPlanner<float> and LocalPlanner<double> (the double
planner's device libm is a port of glibc's).
"""
import math
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "path_planning_pkg_amd" / "lib"
REF = Path("/root/reference")
DRIVER = ROOT / "oracle" / "_ref" / "local_planner_driver"


def test_reference_local_planner_compiles_and_links(tmp_path):
    if not (REF / "src" / "local_planner.cpp").exists():
        pytest.skip("reference tree not present (GPU box)")
    if not (LIB / "libhastar_amd.so").exists():
        pytest.skip("library not built")
    r = subprocess.run(["make", "-s", "-f", str(ROOT / "oracle" / "ref.mk"), f"OUT={tmp_path}"], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    node = tmp_path / "local_planner_node"
    assert node.exists() and (tmp_path / "local_planner_driver").exists()
    syms = subprocess.run(["nm", "-C", str(node)], capture_output=True, text=True, check=True).stdout
    # both specializations are in the binary, and the double one calls the f64 entry points
    assert "LocalPlanner<double>::update_trajectory()" in syms and "LocalPlanner<float>::update_trajectory()" in syms
    for sym in ("hastar64_create", "hastar64_find_path", "hastar_velocity_profile_batch_f64", "hastar_create_f32",
                "hastar_find_path", "hastar_velocity_profile_batch"):
        assert f" U {sym}" in syms, sym


DOUBLE_MAIN = r"""
#include <cstdio>
#include "HybridAStar.h"
#include "VelocityGenerator.h"
int main() {
  std::vector<double> st{-0.5, 0.0, 0.5}, w{0.0, 0.0, 0.0};
  try {
    planning::HybridAStar<double> p(300, 10, 0.5, 0.75, 0.1, 0.95, 0.4, 60, true, 0.75, 4.0, 2.0, 2.269, 1.1, 1.0,
                                    0.785, 72, 1, st, w);
    planning::VelocityGenerator<double> vg(6.0, 1.5, 4.0, 1.5, 2.0);
    std::vector<planning::Vector3D<double>> path;
    std::vector<double> curv, vel;
    auto r = p.find_path(2.0, planning::Vector3D<double>(18.0, 18.0, 0.0), path, curv);
    if (r.second) vg.generate_velocity_profile(2.0, 6.0, path, curv, vel, false, false);
  } catch (const std::exception& e) {
    std::printf("%s\n", e.what());
  }
  return 0;
}
"""


def test_double_dropins_compile_and_link(tmp_path):
    if not (LIB / "libhastar_amd.so").exists():
        pytest.skip("library not built")
    src = tmp_path / "d.cpp"
    src.write_text(DOUBLE_MAIN)
    cmd = ["g++", "-O2", "-std=c++17", f"-I{ROOT / 'include' / 'path_planning_pkg'}", str(src), f"-L{LIB}",
           "-lhastar_amd", f"-Wl,-rpath,{LIB}", "-o", str(tmp_path / "d")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


# ------------------------------------------------------------------ the node, replayed on the oracle
def _parse(out, dt):
    lines = out.strip().splitlines()
    res, i = {}, 0
    while i < len(lines):
        _, turn, n = lines[i].split()
        n = int(n)
        bits = [int(v, 16) for v in lines[i + 1:i + 1 + n]]
        res[int(turn)] = np.array(bits, np.uint32 if dt == np.float32 else np.uint64).view(dt)
        i += 1 + n
    return res


def _node_on_oracle(T):
    """The call sequence local_planner.cpp makes for tests/cxx/local_planner_driver.cpp's scenario,
    with the reference's T arithmetic, on the oracle's HybridAStar<T> / VelocityGenerator<T>."""
    from oracle import pyoracle
    from path_planning_pkg_amd.capi import PlannerConfig
    t = T
    deg = t(math.pi / 180.0)                                   # T deg_to_rad = M_PI/180.0 (:143)
    steer = [t(t(d) * deg) for d in (-30.0, -15.0, 0.0, 15.0, 30.0)]
    apf_ang = t(t(45.0) * deg)                                 # apf_active_angle *= deg_to_rad (:144)
    cfg = PlannerConfig(grid_size=60, grid_resolution=0.5, obstacle_threshold=0.75, obstacle_prob_min=0.1,
                        obstacle_prob_max=0.95, obstacle_prob_free=0.4, step_size=0.75, max_lat_acc=4.0,
                        max_long_dec=2.0, wheelbase=2.269, rear_to_cg=1.1, apf_rep_constant=1.0,
                        apf_active_angle=float(apf_ang), num_angle_bins=72, num_actions=1,
                        dubins_shot_interval=300, dubins_shot_interval_decay=10, steering=[float(s) for s in steer],
                        curvature_weights=[float(t(v)) for v in (0.0, 0.1, 0.0, 0.1, 0.0)])
    if T == np.float32:
        P = pyoracle.OraclePlanner(cfg)
        prof = lambda *a: pyoracle.velocity_profile(*a)  # noqa: E731
        vmax_curr = float(np.finfo(np.float32).max)
    else:
        P = pyoracle.OraclePlanner64(cfg)
        prof = lambda *a: pyoracle.velocity_profile64(*a)  # noqa: E731
        vmax_curr = float(np.finfo(np.float64).max)
    vel_prm = (6.0, 1.5, 4.0, 1.5, 2.0)                        # max_velocity, coast, lat, long_acc, long_dec
    vw2 = t(t(1.2) / t(2))                                    # _vehicle_width_2 = vehicle_width/2
    pose = [float(t(18.0)), float(-t(-18.0)), 0.0]            # {pose._y, -pose._x, yaw} (:180-183)
    velocity = float(t(math.hypot(2.0, 0.0)))
    P.update_goal([0.0, 0.0, 0.0], [0.0, 0.0, 0.0])           # (:166)

    def objects(dx):
        boxes, conf = [], []
        for cx, cy, L in ((18.0, 22.8, 3.4), (14.25, 28.5, 3.0), (18.0, 34.8, 3.4)):
            l, w = np.float32(L), np.float32(L - 0.5)
            dim = t(t(max(l, w)) + vw2)                       # std::max(length, width) + _vehicle_width_2
            boxes.append([float(t(cx + dx)), float(t(cy)), float(dim), float(dim)])
            conf.append(float(t(t(0.5) + t(np.float32(0.8) / np.float32(2)))))
        P.update_boxes(boxes, conf, float(t(2.5)))

    lane_vals = np.array([21.9, 4.5, 21.9, 31.5, 10.5, 4.5, 10.5, 40.5, 9.0, 42.0, 39.0, 42.0], T).reshape(-1, 4)

    def lanes():
        P.update_lines(lane_vals.astype(np.float64), [float(t(0.55))] * 3, float(vw2))
        P.decay()

    path_prev = np.array([pose], np.float64)
    curv_prev = np.zeros(1)
    out = {}
    for turn in (1, 2):
        if turn == 1:
            P.update_goal([26.0, 36.0, 0.0], pose)            # callback_waypoint (:204-205)
            P.reset()
        objects(0.0 if turn == 1 else 0.5)
        lanes()
        r = P.find_path(velocity, pose)
        if r["ok"]:
            path, curv = r["path"], r["curvature"]
            _, vel = prof(vel_prm, velocity, vmax_curr, path, curv, False, False)
            path_prev, curv_prev = path, curv
        else:
            path, curv = path_prev, curv_prev
            _, vel = prof(vel_prm, velocity, vmax_curr, path, curv, False, False)
        rev = np.asarray(path)[::-1]
        out[turn] = np.concatenate([rev[:, 0], rev[:, 1], rev[:, 2], np.asarray(vel)]).astype(T)
        out[f"ok{turn}"] = r["ok"]
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["float", "double"])
def test_local_planner_node_publishes_the_oracle_trajectory(mode):
    if not DRIVER.exists():
        pytest.fail(f"{DRIVER} missing: build it in the container (__graft_entry__.build(), oracle/ref.mk)")
    T = np.float32 if mode == "float" else np.float64
    r = subprocess.run([str(DRIVER), mode], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    got = _parse(r.stdout, T)
    want = _node_on_oracle(T)
    assert want["ok1"] and want["ok2"]
    for turn in (1, 2):
        g, w = got[turn], want[turn]
        assert g.shape == w.shape, (turn, g.shape, w.shape)
        # bit for bit in both instantiations (round 5: the double planner's device libm is a port
        # of glibc's, csrc/hastar_libm64.h)
        bits = np.uint32 if T == np.float32 else np.uint64
        assert np.array_equal(g.view(bits), w.view(bits)), turn
