"""Randomised planner configurations against the oracle (round 6): the exact mode (float on
both kernels, and HybridAStar<double>) must stay bit-identical (success, cost bits, statistics, pop and closed digests, path and curvature) for
parameter combinations the fixed cases do not reach: grid size and resolution, heading bins,
steering sets of 3 / 5 / 7 angles with random curvature weights, num_actions 1-3, 4- or
8-connected holonomic grids, step size, vehicle geometry and limits, shot interval and decay,
APF constant, box and line obstacles, start speed and headings.

The planners of one seed run in ONE batch on each kernel (HASTAR_WIDE=0: the batch kernel,
HASTAR_WIDE=1: the latency kernel), and the oracle replays the same call sequence on host
threads.  Grids stay small (48-160 cells a side) and the obstacles keep clear of the endpoints,
so the oracle's floods stay short.
"""
import math
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from tests.scenarios import drive
from tests.test_gpu_parity import compare_results

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    from path_planning_pkg_amd import planner
    planner.load_library()
    return planner


def random_case(rng):
    from path_planning_pkg_amd.capi import PlannerConfig, steering_from_degrees
    N = int(rng.integers(48, 161))
    res = float(rng.choice([0.25, 0.5, 0.5, 1.0]))
    W = N * res
    S = int(rng.choice([3, 5, 5, 7]))
    amax = float(rng.uniform(15.0, 35.0))
    steer = steering_from_degrees([float(np.float32(v)) for v in np.linspace(-amax, amax, S)])
    weights = [float(np.float32(w)) for w in rng.uniform(0.0, 1.0, S)]
    weights[S // 2] = 0.0
    cfg = PlannerConfig(
        grid_size=N, grid_resolution=res, num_angle_bins=int(rng.choice([36, 60, 72])),
        num_actions=int(rng.integers(1, (S - 1) // 2 + 1)), steering=steer, curvature_weights=weights,
        grid_2d_allow_diag_moves=bool(rng.random() < 0.8), step_size=float(np.float32(rng.uniform(0.5, 1.5))),
        wheelbase=float(np.float32(rng.uniform(2.0, 3.5))), rear_to_cg=float(np.float32(rng.uniform(0.6, 1.6))),
        max_lat_acc=float(np.float32(rng.uniform(2.0, 6.0))), max_long_dec=float(np.float32(rng.uniform(1.0, 3.0))),
        dubins_shot_interval=int(rng.choice([50, 150, 300])), dubins_shot_interval_decay=int(rng.choice([0, 5, 10])),
        apf_rep_constant=float(np.float32(rng.uniform(0.5, 2.0))))
    # the goal anywhere; the start 5 m .. 0.7 x the grid's reach behind it (update_goal aligns the
    # grid with the start -> goal direction, goal cell (0.8 N, N / 2))
    gx, gy = rng.uniform(-50, 50, 2)
    d = rng.uniform(5.0, max(6.0, 0.7 * 0.8 * W))
    a = rng.uniform(-math.pi, math.pi)
    sx, sy = gx - d * math.cos(a), gy - d * math.sin(a)
    goal = [float(np.float32(gx)), float(np.float32(gy)), float(np.float32(rng.uniform(-3.1, 3.1)))]
    start = [float(np.float32(sx)), float(np.float32(sy)), float(np.float32(a + rng.uniform(-1.2, 1.2)))]

    def clear(x, y, r):
        return math.hypot(x - gx, y - gy) > r and math.hypot(x - sx, y - sy) > r

    boxes = []
    for _ in range(int(rng.integers(0, 25))):
        t = rng.uniform(0, 1)
        x = sx + t * (gx - sx) + rng.normal(0, 0.25 * d)
        y = sy + t * (gy - sy) + rng.normal(0, 0.25 * d)
        w, h = rng.uniform(0.5, 4.0, 2)
        if clear(x, y, 4.0 + max(w, h)):
            boxes.append([x, y, w, h])
    lines = []
    for _ in range(int(rng.integers(0, 4))):
        x0, y0 = sx + rng.uniform(-0.5, 1.5) * (gx - sx), sy + rng.uniform(-0.5, 1.5) * (gy - sy)
        ang, ln = rng.uniform(-math.pi, math.pi), rng.uniform(2.0, 10.0)
        x1, y1 = x0 + ln * math.cos(ang), y0 + ln * math.sin(ang)
        if all(clear(x0 + u * (x1 - x0), y0 + u * (y1 - y0), 5.0) for u in np.linspace(0, 1, 9)):
            lines.append([x0, y0, x1, y1])
    proto = dict(goal=goal, start=start, vel=float(np.float32(rng.uniform(0.0, 5.0))), cycles=int(rng.integers(1, 6)),
                 lines=np.array(lines, np.float32).reshape(-1, 4), line_conf=float(rng.uniform(0.55, 0.9)),
                 line_width=float(rng.uniform(0.5, 1.5)), boxes=np.array(boxes, np.float32).reshape(-1, 4),
                 box_conf=float(rng.uniform(0.6, 0.95)), apf_r=float(rng.uniform(0.0, 4.0)))
    return cfg, proto


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6])
def test_random_configurations_both_kernels(gpu, oracle_lib, monkeypatch, seed):
    rng = np.random.default_rng(1000 + seed)
    cases = [random_case(rng) for _ in range(16)]

    def oracle(i):
        cfg, proto = cases[i]
        o = oracle_lib.OraclePlanner(cfg)
        drive(o, proto)
        r = o.find_path(proto["vel"], proto["start"])
        o.close()
        return r

    with ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
        ref = list(ex.map(oracle, range(len(cases))))
    for wide in ("0", "1"):
        monkeypatch.setenv("HASTAR_WIDE", wide)
        gs = []
        for cfg, proto in cases:
            g = gpu.HybridAStar(cfg)
            drive(g, proto)
            gs.append(g)
        res, _ = gpu.find_path_batch(gs, [p["vel"] for _, p in cases], [p["start"] for _, p in cases], cap=16384)
        for i, (r, ro) in enumerate(zip(res, ref)):
            cfg = cases[i][0].values
            compare_results(r, ro, f"seed {seed} case {i} wide={wide} (N={cfg['grid_size']}, res={cfg['grid_resolution']}, "
                                   f"bins={cfg['num_angle_bins']}, actions={cfg['num_actions']})")
        for g in gs:
            g.close()
    print(f"seed {seed}: {sum(r['ok'] for r in ref)}/{len(ref)} found, pops {[r['stats']['pops'] for r in ref]}")


@pytest.mark.parametrize("seed", [1, 2])
def test_random_configurations_double(seed):
    """HybridAStar<double> (include/hastar_f64.h) on the same random configurations: bit equality
    with the oracle's double instantiation (cost, statistics, digests, closed set, path,
    curvature and the memo after the search; tests/test_gpu_f64.py::_compare)."""
    from oracle.pyoracle import OraclePlanner64
    from path_planning_pkg_amd.planner64 import HybridAStar64
    from tests.test_gpu_f64 import _compare, _proto64
    rng = np.random.default_rng(1000 + seed)
    for i in range(16):
        cfg, proto = random_case(rng)
        proto = _proto64(proto)
        g, o = HybridAStar64(cfg), OraclePlanner64(cfg)
        drive(g, proto)
        drive(o, proto)
        _compare(g.find_path(proto["vel"], proto["start"]), o.find_path(proto["vel"], proto["start"]), g, o,
                 f"double seed {seed} case {i}")
