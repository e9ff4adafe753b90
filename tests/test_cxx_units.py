"""The unit-level drop-in classes (include/path_planning_pkg/{AStar,Dubins,VehicleModel,
Node2D,Node3D,common,Obstacle}.h over include/hastar_units.h).

CPU: tests/cxx/units_main.cpp compiles and links against the headers and libhastar_amd.so,
and so do the reference's own manual harnesses (utils/astar/test_astar.cpp,
utils/vehicle_dubins/test_vehicle_dubins.cpp, utils/hybrid_astar/test_hybrid_astar.cpp,
compiled from /root/reference where it exists: the drop-in claim).
GPU: the harness scenarios run through the classes and match
  * the reference's golden vectors: utils/dubins_paths.py:6 (73-pose RSL path),
    utils/vehicle_mode.py:12 (33 positions), compared at their printed %g precision;
  * the costs test_astar printed in the survey container (31.4706, 20.935,
    25.5208, 31.4706) at %g;
  * the oracle bit for bit (float Dubins, float and double vehicle chains, every AStar cost,
    path point and map cell), and the double Dubins path, length and word bit for bit too
    (the device runs ports of glibc's double libm, csrc/hastar_libm64.h).
"""
import json
import math
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

from tests.scenarios import GOLDEN

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "path_planning_pkg_amd" / "lib"
REF = Path("/root/reference")


def _compile(src, exe, extra=()):
    cmd = ["g++", "-O2", "-std=c++17", "-ffp-contract=off", f"-I{ROOT / 'include' / 'path_planning_pkg'}", *extra,
           str(src), f"-L{LIB}", "-lhastar_amd", f"-Wl,-rpath,{LIB}", "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def test_units_program_compiles(tmp_path):
    if not (LIB / "libhastar_amd.so").exists():
        pytest.skip("library not built")
    assert _compile(ROOT / "tests" / "cxx" / "units_main.cpp", tmp_path / "units").exists()


@pytest.mark.parametrize("harness", ["astar/test_astar.cpp", "vehicle_dubins/test_vehicle_dubins.cpp",
                                     "hybrid_astar/test_hybrid_astar.cpp"])
def test_reference_harness_compiles_against_dropins(tmp_path, harness):
    """The reference's own harness sources, unchanged, build against the drop-in headers
    (-DSTORE_GRID_AS_REFERENCE as its CMakeLists.txt:128 sets it)."""
    src = REF / "utils" / harness
    if not src.exists():
        pytest.skip("reference tree not present (GPU box)")
    if not (LIB / "libhastar_amd.so").exists():
        pytest.skip("library not built")
    assert _compile(src, tmp_path / Path(harness).stem, ("-DSTORE_GRID_AS_REFERENCE",)).exists()


def _g6(v):
    return float("%g" % v)


def _h2f(h):
    return np.array([int(x, 16) for x in h], np.uint32).view(np.float32)


def _parse(out):
    lines = out.strip().splitlines()
    sec, i = {}, 0
    while i < len(lines):
        head = lines[i].split()
        tag = head[0]
        if tag in ("D", "F", "VD", "VF", "AP", "AM"):
            n = int(head[3]) if tag in ("D", "F") else int(head[1])
            sec[tag] = (head, [ln.split() for ln in lines[i + 1:i + 1 + n]])
            i += 1 + n
        elif tag in ("NB", "SIM"):
            n = int(head[1])
            sec[tag] = (head, [ln.split() for ln in lines[i + 1:i + 1 + n]])
            i += 1 + n
        else:
            sec[tag] = (head, [])
            i += 1
    return sec


@pytest.mark.gpu
def test_units_match_golden_and_oracle(tmp_path, oracle_lib):
    exe = _compile(ROOT / "tests" / "cxx" / "units_main.cpp", tmp_path / "units")
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, check=True).stdout
    S = _parse(out)

    # Dubins<double>: the reference's golden RSL path (utils/dubins_paths.py:6)
    g = json.loads((GOLDEN / "dubins_rsl.json").read_text())
    head, rows = S["D"]
    assert head[1] == "RSL"
    path_d = np.array([[float(v) for v in r] for r in rows])
    assert [[_g6(v) for v in r] for r in path_d.tolist()] == g["path"]
    rmin = float(head[6])
    assert "%g" % rmin == "4.08106"
    ref_d, len_d, word_d = oracle_lib.dubins_path_d(rmin, 0.5, [0.0, 0.0, 0.0], [20.0, -20.0, math.pi / 2])
    assert word_d == 1 and path_d.shape == ref_d.shape
    assert np.array_equal(path_d.view(np.uint64), ref_d.view(np.uint64))
    assert float(head[2]) == len_d and float(head[4]) == len_d

    # Dubins<float>: bit-exact with the oracle
    head, rows = S["F"]
    rmin_f = _h2f([head[5]])[0]
    got = _h2f([v for r in rows for v in r]).reshape(-1, 4)
    assert len(got) == int(head[3])
    xf, cf, Lf, flag_f = oracle_lib.dubins_path_f(float(rmin_f), 0.5, [0.0, 0.0, 0.0], [20.0, -20.0, float(np.float32(math.pi / 2))])
    assert np.array_equal(got[:, :3].view(np.uint32), xf.view(np.uint32))
    assert np.array_equal(got[:, 3].view(np.uint32), cf.view(np.uint32))
    assert np.array_equal(_h2f([head[2]]).view(np.uint32), np.float32([Lf]).view(np.uint32))
    assert bool(int(head[4])) == flag_f

    # VehicleModel<double>: golden positions (utils/vehicle_mode.py:12) and the oracle, exactly
    gv = json.loads((GOLDEN / "vehicle_chain.json").read_text())
    head, rows = S["VD"]
    pos_d = np.array([[float(v) for v in r] for r in rows])
    assert [[_g6(v) for v in r] for r in pos_d.tolist()] == gv["positions"]
    st = [d * math.pi / 180.0 for d in gv["steering_deg"]]
    ref_v = oracle_lib.vehicle_chain_d(0.5, 4.0, 2.269, 1.1, 72, 1, st, [0.0] * 7, 16.0, 3, gv["actions"])
    assert np.array_equal(pos_d, ref_v)

    # VehicleModel<float>: the oracle's float chain, bit for bit
    head, rows = S["VF"]
    pos_f = _h2f([v for r in rows for v in r]).reshape(-1, 2)
    st_f = [float(np.float32(d * math.pi / 180.0)) for d in gv["steering_deg"]]
    ref_f = oracle_lib.vehicle_chain_f(0.5, 4.0, 2.269, 1.1, 72, 1, st_f, [0.0] * 7, 16.0, gv["actions"])
    assert np.array_equal(pos_f.view(np.uint32), ref_f.view(np.uint32))
    head, rows = S["NB"]
    assert int(head[2]) == 0  # the chain's node 5 still moves fast: accelerations apply
    # get_neighbors == simulate_action over the same action window, feasible ones, in order
    assert rows == S["SIM"][1] and 1 <= len(rows) <= 3

    # AStar<float>: the survey's printed costs and the oracle's search, bit for bit
    from path_planning_pkg_amd.capi import PlannerConfig
    cfg = PlannerConfig(grid_size=60)
    o = oracle_lib.OraclePlanner(cfg)
    goal, start = [25.5, 36.0], [18.0, 18.0]
    ci, cj = o.astar_goal_start(goal, start)
    lines = np.array([[21.9, 4.5, 21.9, 31.5], [20.4, 33.0, 38.4, 33.0], [10.5, 4.5, 10.5, 40.5],
                      [9.0, 42.0, 39.0, 42.0]], np.float32)
    boxes = np.array([[18.0, 22.8, 4.0, 3.4], [14.25, 28.5, 3.0, 5.8], [18.0, 34.8, 4.0, 3.4]], np.float32)
    for _ in range(5):
        o.decay()
        o.update_lines(lines, [0.6] * 4, 1.0)
        o.update_boxes(boxes, [0.75] * 3, 0.0)
    costs_o = [o.astar_cost(ci, cj), o.astar_cost(33, 36), o.astar_cost(ci + 6, cj + 10)]
    c4, pts = o.astar_find_path(goal, start)
    costs_o.append(c4)
    head, _ = S["A"]
    costs_g = _h2f(head[1:5])
    assert (int(head[5]), int(head[6])) == (ci, cj)
    assert np.array_equal(costs_g.view(np.uint32), np.float32(costs_o).view(np.uint32))
    assert ["%g" % c for c in costs_g] == ["31.4706", "20.935", "25.5208", "31.4706"]
    head, rows = S["AP"]
    path_a = _h2f([v for r in rows for v in r]).reshape(-1, 2)
    assert len(path_a) == len(pts) + 1
    assert np.array_equal(path_a[0], np.float32(goal)) and np.array_equal(path_a[1:].view(np.uint32), pts.view(np.uint32))
    head, rows = S["AM"]
    grid = _h2f([v for r in rows for v in r]).reshape(60, 60)
    assert np.array_equal(grid.view(np.uint32), o.get_obstacles().view(np.uint32))


@pytest.mark.gpu
def test_grid3d_members_match_oracle(oracle_lib):
    """Grid3D<float>::get_neighbors / check_path / set_start_node on a planner handle (the
    device entry points behind include/path_planning_pkg/Grid3D.h) vs the oracle's
    restatement, on the reference harness map: every successor's pose, cost (APF included),
    speed, action, bin and cell bit for bit, over a breadth-first sweep of 200 nodes."""
    from path_planning_pkg_amd import planner as gpu
    from tests.scenarios import drive, harness
    cfg, proto, _ = harness()
    g, o = gpu.HybridAStar(cfg), oracle_lib.OraclePlanner(cfg)
    drive(g, proto)
    drive(o, proto)
    node, cell = g.set_start_node(proto["start"])
    node = [float(v) for v in node[:5]] + [int(v) for v in node[5:].view(np.int32)]
    node[4] = 4.0  # a moving start (v = 2 m/s): the acceleration branch of VehicleModel.cpp:80-92
    frontier, seen = [node], 0
    while frontier and seen < 200:
        nd = frontier.pop(0)
        rg, cg, ng = g.grid3d_neighbors(nd)
        ro, co, no = o.grid3d_neighbors(nd)
        assert ng == no and len(rg) == len(ro), (nd, len(rg), len(ro))
        assert np.array_equal(rg.view(np.uint32), ro.view(np.uint32)) and np.array_equal(cg, co)
        for r in rg:
            frontier.append([float(v) for v in r[:5]] + [int(v) for v in r[5:].view(np.int32)])
        seen += 1
    rng = np.random.default_rng(5)
    for _ in range(50):
        p = np.stack([rng.uniform(0, 30, 20), rng.uniform(0, 30, 20), rng.uniform(-3, 3, 20)], 1).astype(np.float32)
        assert g.check_path(p) == o.check_path(p)
