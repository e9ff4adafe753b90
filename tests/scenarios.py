"""Scenario builders shared by tests, smoke() and bench.py (synthetic inputs of SURVEY.md §8d).

The harness scenario restates utils/hybrid_astar/test_hybrid_astar.cpp:13-98; the synthetic
generator restates SURVEY.md §8d (W = N*res, goal (0,0,0), start (-0.6W, 0, 0), K boxes with
sides U(1,6) m, centres x in [-0.8W, 0.2W], y in [-0.5W, 0.5W], rejected within 8 m of the
endpoints) with numpy's PCG64 instead of std::mt19937 (the inputs are then fixed by the seed and
recorded in each fixture, so both sides see identical floats).
"""
import json
import math
from pathlib import Path

import numpy as np

from path_planning_pkg_amd.capi import PlannerConfig, steering_from_degrees

GOLDEN = Path(__file__).resolve().parent / "golden"


def f32(v):
    return float(np.float32(v))


def harness():
    """test_hybrid_astar.cpp scenario: returns (cfg, protocol dict)."""
    g = json.loads((GOLDEN / "harness_60.json").read_text())
    cfg = PlannerConfig(grid_size=60, steering=steering_from_degrees(g["params"]["steering_deg"]))
    proto = dict(goal=[26.0, 36.0, 0.0], start=[18.0, 18.0, f32(math.pi / 2)], vel=2.0, cycles=5,
                 lines=np.array(g["lines"], np.float32), line_conf=0.6, line_width=1.25,
                 boxes=np.array(g["boxes"], np.float32), box_conf=0.75, apf_r=2.5)
    return cfg, proto, g


def synthetic(N, bins, K, seed, res=0.5, clear=8.0):
    """SURVEY.md §8d synthetic case (harness vehicle parameters)."""
    W = N * res
    rng = np.random.default_rng(seed)
    boxes = []
    start = np.array([-0.6 * W, 0.0])
    goal = np.array([0.0, 0.0])
    while len(boxes) < K:
        sx, sy = rng.uniform(1.0, 6.0, 2)
        cx = rng.uniform(-0.8 * W, 0.2 * W)
        cy = rng.uniform(-0.5 * W, 0.5 * W)
        r = math.hypot(sx, sy) / 2
        if math.hypot(cx - start[0], cy - start[1]) < clear + r or math.hypot(cx - goal[0], cy - goal[1]) < clear + r:
            continue
        boxes.append([cx, cy, sx, sy])
    cfg = PlannerConfig(grid_size=N, num_angle_bins=bins, steering=steering_from_degrees([-30, -15, 0, 15, 30]))
    proto = dict(goal=[0.0, 0.0, 0.0], start=[float(-0.6 * W), 0.0, 0.0], vel=2.0, cycles=5,
                 lines=np.zeros((0, 4), np.float32), line_conf=0.6, line_width=1.25,
                 boxes=np.array(boxes, np.float32), box_conf=0.75, apf_r=2.5)
    return cfg, proto


def drive(planner, proto):
    """The fixture protocol: update_goal, 5 x {decay, lines, boxes}, reset."""
    planner.update_goal(proto["goal"], proto["start"])
    for _ in range(proto["cycles"]):
        planner.decay()
        if len(proto["lines"]):
            planner.update_lines(proto["lines"], [proto["line_conf"]] * len(proto["lines"]), proto["line_width"])
        if len(proto["boxes"]):
            planner.update_boxes(proto["boxes"], [proto["box_conf"]] * len(proto["boxes"]), proto["apf_r"])
    planner.reset()
