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


def _synthetic_boxes_loop(W, K, rng, clear):
    """The generator's definition, one candidate at a time (kept as the test's reference for
    the vectorised draw below)."""
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
    return boxes


def _synthetic_boxes(W, K, rng, clear):
    """Vectorised draw of the same candidates: every candidate consumes 4 doubles of the
    stream in the order (sx, sy, cx, cy) and numpy's uniform(a, b) is a + (b - a) * u, so
    drawing blocks of candidates and keeping the first K accepted gives the loop's boxes."""
    out = []
    while len(out) < K:
        u = rng.random((2 * K + 16, 4))
        sx = 1.0 + (6.0 - 1.0) * u[:, 0]
        sy = 1.0 + (6.0 - 1.0) * u[:, 1]
        cx = -0.8 * W + (0.2 * W - -0.8 * W) * u[:, 2]
        cy = -0.5 * W + (0.5 * W - -0.5 * W) * u[:, 3]
        r = np.hypot(sx, sy) / 2
        ok = ~((np.hypot(cx - (-0.6 * W), cy - 0.0) < clear + r) | (np.hypot(cx - 0.0, cy - 0.0) < clear + r))
        for k in np.nonzero(ok)[0]:
            out.append([cx[k], cy[k], sx[k], sy[k]])
            if len(out) == K:
                break
    return out


def synthetic(N, bins, K, seed, res=0.5, clear=8.0):
    """SURVEY.md §8d synthetic case (harness vehicle parameters)."""
    W = N * res
    rng = np.random.default_rng(seed)
    boxes = _synthetic_boxes(W, K, rng, clear)
    cfg = PlannerConfig(grid_size=N, num_angle_bins=bins, steering=steering_from_degrees([-30, -15, 0, 15, 30]))
    proto = dict(goal=[0.0, 0.0, 0.0], start=[float(-0.6 * W), 0.0, 0.0], vel=2.0, cycles=5,
                 lines=np.zeros((0, 4), np.float32), line_conf=0.6, line_width=1.25,
                 boxes=np.array(boxes, np.float32), box_conf=0.75, apf_r=2.5)
    return cfg, proto


class MT19937:
    """std::mt19937 with its default (init_genrand) seeding, as libstdc++ defines it."""

    def __init__(self, seed):
        mt = [seed & 0xffffffff]
        for i in range(1, 624):
            mt.append((1812433253 * (mt[i - 1] ^ (mt[i - 1] >> 30)) + i) & 0xffffffff)
        self.mt, self.i = mt, 624

    def __call__(self):
        mt = self.mt
        if self.i >= 624:
            for k in range(624):
                y = (mt[k] & 0x80000000) | (mt[(k + 1) % 624] & 0x7fffffff)
                mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ (0x9908b0df if y & 1 else 0)
            self.i = 0
        y = mt[self.i]
        self.i += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9d2c5680
        y ^= (y << 15) & 0xefc60000
        return (y ^ (y >> 18)) & 0xffffffff


def _uniform_f32(rng, a, b):
    """std::uniform_real_distribution<float>(a, b)(rng) of libstdc++: generate_canonical<float,
    24> takes one 32-bit draw, u / 2^32 in float (clamped below 1), then canonical * (b - a) + a."""
    c = np.float32(rng()) / np.float32(4294967296.0)
    if c >= np.float32(1):
        c = np.nextafter(np.float32(1), np.float32(0))
    return np.float32(c * np.float32(b - a)) + a


def _uniform_f32_vec(u, a, b):
    """_uniform_f32 over an array of raw 32-bit draws (float32 arithmetic, op by op)."""
    c = u.astype(np.float32) / np.float32(4294967296.0)
    c = np.where(c >= np.float32(1), np.nextafter(np.float32(1), np.float32(0)), c).astype(np.float32)
    return (c * np.float32(b - a)).astype(np.float32) + np.float32(a)


def synthetic_ref_boxes(N, K, seed, res=0.5, clear=8.0):
    """The box list of synthetic_ref, vectorised: numpy's RandomState(seed) is std::mt19937
    with init_genrand seeding, and randint(0, 2^32) returns its raw 32-bit draws in order
    (tests/test_oracle_golden.py checks it against the scalar MT19937 above)."""
    f = np.float32
    W = f(N) * f(res)
    ax, bx = f(-0.8 * float(W)), f(0.2 * float(W))
    ay, by = f(-0.5 * float(W)), f(0.5 * float(W))
    stx = f(-0.6 * float(W))
    rs = np.random.RandomState(seed & 0xffffffff)
    out = np.zeros((0, 4), np.float32)
    while len(out) < K:
        u = rs.randint(0, 2 ** 32, size=(2 * K + 16, 4), dtype=np.uint64)
        cx, cy = _uniform_f32_vec(u[:, 0], ax, bx), _uniform_f32_vec(u[:, 1], ay, by)
        sx, sy = _uniform_f32_vec(u[:, 2], f(1), f(6)), _uniform_f32_vec(u[:, 3], f(1), f(6))
        keep = ~((np.hypot((cx - stx).astype(np.float32), cy) < f(clear)) | (np.hypot(cx, cy) < f(clear)))
        out = np.concatenate([out, np.stack([cx, cy, sx, sy], 1)[keep]])
    return out[:K].astype(np.float32), float(stx)


def synthetic_ref_boxes_scalar(N, K, seed, res=0.5, clear=8.0):
    """The same boxes one draw at a time with the MT19937 class (the definition)."""
    f = np.float32
    W = f(N) * f(res)
    ax, bx = f(-0.8 * float(W)), f(0.2 * float(W))
    ay, by = f(-0.5 * float(W)), f(0.5 * float(W))
    stx = f(-0.6 * float(W))
    rng = MT19937(seed)
    boxes = []
    while len(boxes) < K:
        cx, cy = _uniform_f32(rng, ax, bx), _uniform_f32(rng, ay, by)
        sx, sy = _uniform_f32(rng, f(1), f(6)), _uniform_f32(rng, f(1), f(6))
        if f(np.hypot(f(cx - stx), cy)) < f(clear) or f(np.hypot(cx, cy)) < f(clear):
            continue
        boxes.append([cx, cy, sx, sy])
    return np.array(boxes, np.float32).reshape(-1, 4), float(stx)


def _mt19937_words(seeds, n_words):
    """The first n_words raw 32-bit outputs of std::mt19937(seed) for every seed at once
    (uint32, shape (len(seeds), n_words)): init_genrand seeding and the twist as libstdc++
    defines them, vectorised over the seeds.  The twist's in-place recurrence splits into four
    block steps: words 0..226 read old words only, 227..453 read the new words 0..226,
    454..622 the new words 227..395, and word 623 the new words 0 and 396."""
    s = np.asarray(seeds, np.uint64) & np.uint64(0xffffffff)
    S = len(s)
    mt = np.empty((624, S), np.uint64)
    mt[0] = s
    for i in range(1, 624):
        p = mt[i - 1]
        mt[i] = (np.uint64(1812433253) * (p ^ (p >> np.uint64(30))) + np.uint64(i)) & np.uint64(0xffffffff)
    mt = mt.astype(np.uint32)
    up, lo, ma = np.uint32(0x80000000), np.uint32(0x7fffffff), np.uint32(0x9908b0df)

    def f(a, b):  # y = upper bit of a | lower bits of b; (y >> 1) ^ (y & 1 ? MATRIX_A : 0)
        y = (a & up) | (b & lo)
        return (y >> np.uint32(1)) ^ np.where((y & np.uint32(1)) != 0, ma, np.uint32(0))

    out = np.empty((S, n_words), np.uint32)
    got = 0
    while got < n_words:
        old = mt
        new = np.empty_like(old)
        new[0:227] = old[397:624] ^ f(old[0:227], old[1:228])
        new[227:454] = new[0:227] ^ f(old[227:454], old[228:455])
        new[454:623] = new[227:396] ^ f(old[454:623], old[455:624])
        new[623] = new[396] ^ f(old[623], new[0])
        mt = new
        y = mt.copy()
        y ^= y >> np.uint32(11)
        y ^= (y << np.uint32(7)) & np.uint32(0x9d2c5680)
        y ^= (y << np.uint32(15)) & np.uint32(0xefc60000)
        y ^= y >> np.uint32(18)
        take = min(624, n_words - got)
        out[:, got:got + take] = y[:take].T
        got += take
    return out


def _ref_candidates(N, K, seeds, res=0.5, clear=8.0):
    """The first 2K + 16 box candidates of synthetic_ref_boxes for every seed at once, with the
    same float32 arithmetic: (cx, cy, sx, sy, sel, stx); sel marks the first K accepted ones.
    Rows whose candidates hold fewer than K accepted ones have sel.sum() < K."""
    f = np.float32
    W = f(N) * f(res)
    ax, bx = f(-0.8 * float(W)), f(0.2 * float(W))
    ay, by = f(-0.5 * float(W)), f(0.5 * float(W))
    stx = f(-0.6 * float(W))
    M = 2 * K + 16
    u = _mt19937_words(seeds, 4 * M).reshape(len(seeds), M, 4).astype(np.uint64)
    cx, cy = _uniform_f32_vec(u[..., 0], ax, bx), _uniform_f32_vec(u[..., 1], ay, by)
    sx, sy = _uniform_f32_vec(u[..., 2], f(1), f(6)), _uniform_f32_vec(u[..., 3], f(1), f(6))
    keep = ~((np.hypot((cx - stx).astype(np.float32), cy) < f(clear)) | (np.hypot(cx, cy) < f(clear)))
    sel = keep & (np.cumsum(keep, axis=1) <= K)
    return cx, cy, sx, sy, sel, float(stx)


def synthetic_ref_boxes_many(N, K, seeds, res=0.5, clear=8.0):
    """synthetic_ref_boxes for many seeds at once: boxes float32 (len(seeds), K, 4) and stx.  A
    seed whose first 2K + 16 candidates hold fewer than K accepted ones (a near-impossible draw)
    falls back to the per-seed generator."""
    cx, cy, sx, sy, sel, stx = _ref_candidates(N, K, seeds, res, clear)
    out = np.empty((len(seeds), K, 4), np.float32)
    full = sel.sum(axis=1) == K
    r, c = np.nonzero(sel[full])
    out[full] = np.stack([a[full][r, c] for a in (cx, cy, sx, sy)], 1).reshape(-1, K, 4)
    for i in np.nonzero(~full)[0]:
        out[i] = synthetic_ref_boxes(N, K, int(seeds[i]), res, clear)[0]
    return out, stx


def route_score(boxes, start, goal):
    """The library's cold-order key (hastar_capi.cpp:route_score) for many box sets at once:
    boxes (Q, K, 4) {x, y, dx, dy} in the world frame, start/goal (2,) or (Q, 2): sum over a
    row's boxes of (1 + t) / (1 + d)^3, d = distance between the axis-aligned box and the start-goal
    segment (0 when the segment crosses it)."""
    b = np.asarray(boxes, np.float64)
    s = np.broadcast_to(np.asarray(start, np.float64), (b.shape[0], 2))[:, None, :]
    g = np.broadcast_to(np.asarray(goal, np.float64), (b.shape[0], 2))[:, None, :]
    x0, y0 = b[..., 0] - b[..., 2] / 2, b[..., 1] - b[..., 3] / 2
    x1, y1 = b[..., 0] + b[..., 2] / 2, b[..., 1] + b[..., 3] / 2
    ax, ay, dx, dy = s[..., 0], s[..., 1], g[..., 0] - s[..., 0], g[..., 1] - s[..., 1]
    # slab test: does the segment cross the box?
    t0, t1 = np.zeros_like(x0), np.ones_like(x0)
    hit = np.ones(x0.shape, bool)
    for o, d, lo, hi in ((ax, dx, x0, x1), (ay, dy, y0, y1)):
        flat = np.abs(d) < 1e-12
        with np.errstate(divide="ignore", invalid="ignore"):
            ta, tb = (lo - o) / np.where(flat, 1.0, d), (hi - o) / np.where(flat, 1.0, d)
        lo_t, hi_t = np.minimum(ta, tb), np.maximum(ta, tb)
        t0 = np.where(flat, t0, np.maximum(t0, lo_t))
        t1 = np.where(flat, t1, np.minimum(t1, hi_t))
        hit &= np.where(flat, (o >= lo) & (o <= hi), True)
    hit &= t0 <= t1

    def pt_box(px, py):
        return np.hypot(np.maximum(np.maximum(x0 - px, px - x1), 0), np.maximum(np.maximum(y0 - py, py - y1), 0))

    def pt_seg(px, py):
        L2 = dx * dx + dy * dy
        t = np.clip(np.where(L2 > 0, ((px - ax) * dx + (py - ay) * dy) / np.where(L2 > 0, L2, 1.0), 0.0), 0, 1)
        return np.hypot(ax + t * dx - px, ay + t * dy - py)

    m = np.minimum(pt_box(ax, ay), pt_box(ax + dx, ay + dy))
    for px, py in ((x0, y0), (x1, y0), (x0, y1), (x1, y1)):
        m = np.minimum(m, pt_seg(px, py))
    d = np.where(hit, 0.0, m)
    cx, cy = b[..., 0], b[..., 1]
    L2 = dx * dx + dy * dy
    t = np.clip(np.where(L2 > 0, ((cx - ax) * dx + (cy - ay) * dy) / np.where(L2 > 0, L2, 1.0), 0.0), 0, 1)
    return ((1.0 + t) / (1.0 + d) ** 3).sum(axis=-1)


def predicted_cost(N, K, query_ids, res=0.5, apf_r=2.5, chunk=8192):
    """A cheap predictor of a synthetic_ref query's search cost (query q = seed q + 1): the
    library's cold-order key, route_score of its boxes (start (stx, 0), goal (0, 0)).  Boxes on or
    near the straight route make the search work around them.  Over the 23,552 bench queries
    and their measured GPU search times (round 3), ordering by it gives a simulated
    longest-first step of 3.24 s against 3.74 s for the nearest-box clearance used before and
    2.86 s for perfect foreknowledge.  Larger = costlier."""
    ids = np.asarray(query_ids, np.int64)
    out = np.empty(len(ids), np.float64)
    for a in range(0, len(ids), chunk):
        seeds = ids[a:a + chunk] + 1
        boxes, stx = synthetic_ref_boxes_many(N, K, seeds, res)
        out[a:a + chunk] = route_score(boxes, [stx, 0.0], [0.0, 0.0])
    return out


def synthetic_ref(N, bins, K, seed, res=0.5, clear=8.0):
    """SURVEY.md §8d's synthetic case drawn the way the survey's reference runs drew it:
    std::mt19937(seed) and std::uniform_real_distribution<float>; per candidate box the centre
    (x in [-0.8W, 0.2W], y in [-0.5W, 0.5W]) then the sides U(1, 6) m; a box whose centre lies
    within 8 m of the start or the goal is redrawn.  With these draws the oracle reproduces the
    pop counts the survey measured on the compiled reference (cfg3 seed 1: 3,297 pops; seed 3:
    7,107 pops, 21,170 successors, 20,234 inner A* pops), which
    pins it at full size (tools/mt19937_synth.cpp is the same generator in C++).  bench.py's
    workloads use this generator (seed = query id + 1)."""
    boxes, stx = synthetic_ref_boxes(N, K, seed, res, clear)
    cfg = PlannerConfig(grid_size=N, num_angle_bins=bins, steering=steering_from_degrees([-30, -15, 0, 15, 30]))
    proto = dict(goal=[0.0, 0.0, 0.0], start=[stx, 0.0, 0.0], vel=2.0, cycles=5,
                 lines=np.zeros((0, 4), np.float32), line_conf=0.6, line_width=1.25,
                 boxes=boxes, box_conf=0.75, apf_r=2.5)
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


def drive_batch(gpu, planners, protos):
    """drive() of many GPU planners through the batched map-update entry points
    (hastar_update_goal_batch / hastar_decay_batch / hastar_update_boxes_batch): the same
    call sequence per planner, bit for bit, in a handful of launches.  Lines (absent from the
    synthetic workloads) go through the per-planner call."""
    gpu.update_goal_batch(planners, [p["goal"] for p in protos], [p["start"] for p in protos])
    cycles = protos[0]["cycles"]
    assert all(p["cycles"] == cycles for p in protos)
    apf_r = protos[0]["apf_r"]
    assert all(p["apf_r"] == apf_r for p in protos)
    for _ in range(cycles):
        gpu.decay_batch(planners)
        for pl, p in zip(planners, protos):
            if len(p["lines"]):
                pl.update_lines(p["lines"], [p["line_conf"]] * len(p["lines"]), p["line_width"])
        gpu.update_boxes_batch(planners, [p["boxes"] for p in protos],
                               [np.full(len(p["boxes"]), p["box_conf"], np.float32) for p in protos], apf_r)
    gpu.reset_batch(planners)


def replan_pairs(N, bins, K, n_pairs, seed, res=0.5, clear=8.0):
    """n_pairs start/goal pairs on an N x N grid.  Each goal is uniform in
    +-0.15 W with a uniform heading; the start lies U(0.3, 0.6) W behind it along that
    heading (same heading).  K boxes per pair (sides U(1, 6) m, centres uniform over the
    square spanned by the pair, rejected within `clear` m of start/goal) with per-box
    velocities U(-2, 2) m/s per axis.  Returns [(cfg, proto, box_vel)]."""
    W = N * res
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_pairs):
        g = rng.uniform(-0.15 * W, 0.15 * W, 2)
        th = float(rng.uniform(-math.pi, math.pi))
        d = float(rng.uniform(0.3, 0.6)) * W
        s = g - d * np.array([math.cos(th), math.sin(th)])
        lo, hi = np.minimum(s, g) - 0.2 * W, np.maximum(s, g) + 0.2 * W
        boxes = []
        while len(boxes) < K:
            sx, sy = rng.uniform(1.0, 6.0, 2)
            cx, cy = rng.uniform(lo, hi)
            r = math.hypot(sx, sy) / 2
            if math.hypot(cx - s[0], cy - s[1]) < clear + r or math.hypot(cx - g[0], cy - g[1]) < clear + r:
                continue
            boxes.append([cx, cy, sx, sy])
        vel = rng.uniform(-2.0, 2.0, (K, 2)).astype(np.float32)
        cfg = PlannerConfig(grid_size=N, num_angle_bins=bins, steering=steering_from_degrees([-30, -15, 0, 15, 30]))
        proto = dict(goal=[f32(g[0]), f32(g[1]), f32(th)], start=[f32(s[0]), f32(s[1]), f32(th)], vel=2.0, cycles=5,
                     lines=np.zeros((0, 4), np.float32), line_conf=0.6, line_width=1.25,
                     boxes=np.array(boxes, np.float32), box_conf=0.75, apf_r=2.5)
        out.append((cfg, proto, vel))
    return out


def replan_tick_inputs(proto, box_vel, tick, dt=0.05):
    """Inputs of replan tick `tick` (0-based) of a cfg5 pair: the start pose advanced by
    vel * dt per tick along its heading, and the boxes moved by box_vel * dt per tick.
    Both are computed from tick 0 in float64 and rounded once, so every caller sees the
    same float32 values."""
    sx, sy, sh = proto["start"]
    step = proto["vel"] * dt * tick
    start = [f32(sx + step * math.cos(sh)), f32(sy + step * math.sin(sh)), f32(sh)]
    boxes = proto["boxes"].astype(np.float64)
    boxes[:, :2] += box_vel.astype(np.float64) * (dt * tick)
    return start, boxes.astype(np.float32)


def replan_tick(planner, proto, box_vel, tick):
    """One tick of the L3 loop after its find_path (local_planner.cpp:241, 288): free-space
    decay, then the moved boxes.  No reset: memo and stale node-map values carry over."""
    _, boxes = replan_tick_inputs(proto, box_vel, tick + 1)
    planner.decay()
    planner.update_boxes(boxes, [proto["box_conf"]] * len(boxes), proto["apf_r"])

