"""GPU (libhastar_amd.so on gfx950) vs the CPU oracle: bit-exact parity.

Parity bar (north_star + SURVEY.md §8): identical closed-set membership, identical
goal-reached decision, path cost within 1e-4 relative.  We test a stricter bar: every
float the planner produces (obstacle map, APF list, memo, path, curvature, cost) is
bit-identical, and the ordered pop digest (cell, bin, g of every pop) plus the closed-set
digest are identical, i.e. the GPU replays the reference's exact search trajectory.
"""
import math

import numpy as np
import pytest

from tests.parity_util import assert_bits_equal, bits  # noqa: F401 (re-exported)
from tests.scenarios import drive, harness, synthetic, synthetic_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    from path_planning_pkg_amd import planner
    planner.load_library()
    return planner


def both(cfg, gpu, oracle_lib):
    return gpu.HybridAStar(cfg), oracle_lib.OraclePlanner(cfg)


def compare_results(rg, ro, what):
    assert rg["ok"] == ro["ok"], f"{what}: success {rg['ok']} vs {ro['ok']}"
    assert_bits_equal(np.float32(rg["cost"]), np.float32(ro["cost"]), f"{what} cost")
    sg, so = rg["stats"], ro["stats"]
    assert sg["status"] == 0, f"{what}: device status {sg['status']}"
    for k in ("pops", "successors", "astar_pops", "astar_searches", "shots", "closed_size", "pop_digest",
              "closed_digest", "via_shot"):
        assert sg[k] == so[k], f"{what}: stats[{k}] {sg[k]} vs {so[k]}"
    assert_bits_equal(rg["path"], ro["path"], f"{what} path")
    assert_bits_equal(rg["curvature"], ro["curvature"], f"{what} curvature")


# ------------------------------------------------------------------ building blocks --
def test_libm_ports_on_gpu(gpu, oracle_lib):
    rng = np.random.default_rng(7)
    n = 1 << 20
    x = rng.uniform(-8, 8, n).astype(np.float32)
    x[:16] = [0, -0.0, 1e-40, 1e-7, 3.1415927, -3.1415927, 1.5707964, 120.0, -200.5, 1e6, 7.8539818e-01, 2.0,
              0.5, -0.5, 4.0, 1e30]
    y = rng.uniform(-8, 8, n).astype(np.float32)
    u = rng.uniform(-1, 1, n).astype(np.float32)
    u[:6] = [1.0, -1.0, 0.5, -0.5, 0.0, 2.9e-8]
    for fn, a, b in ((0, x, None), (1, x, None), (2, y, x), (3, u, None), (4, y, x), (5, x * 2.0, None), (7, x, None)):
        assert_bits_equal(gpu.gpu_math(fn, a, b), oracle_lib.libm(fn, a, b), f"libm fn {fn}")
    prec = np.full(n, np.float32(2 * math.pi / 72), np.float32)
    h = rng.uniform(-3.1416, 3.1416, n).astype(np.float32)
    h[:4] = [np.float32(math.pi), np.float32(-math.pi), 0.0, np.float32(3.1415925)]
    assert_bits_equal(gpu.gpu_math(6, h, prec), oracle_lib.libm(6, h, prec), "heading index")


def test_motion_tables(gpu, oracle_lib):
    cfg, _, _ = harness()
    g, o = both(cfg, gpu, oracle_lib)
    tg, to = g.motion_tables(), o.motion_tables()
    for k in ("offsets", "dtheta", "cost", "curv_abs"):
        assert_bits_equal(tg[k], to[k], k)
    assert_bits_equal(np.float32(tg["precision"]), np.float32(to["precision"]), "precision")
    assert_bits_equal(np.float32(tg["r_min"]), np.float32(o.min_radius()), "r_min")


def test_map_upkeep_harness(gpu, oracle_lib):
    cfg, proto, _ = harness()
    g, o = both(cfg, gpu, oracle_lib)
    for p in (g, o):
        p.update_goal(proto["goal"], proto["start"])
    assert_bits_equal(g.get_obstacles(), o.get_obstacles(), "map after update_goal")
    for cyc in range(proto["cycles"]):
        for p in (g, o):
            p.decay()
        assert_bits_equal(g.get_obstacles(), o.get_obstacles(), f"map after decay {cyc}")
        for p in (g, o):
            p.update_lines(proto["lines"], [proto["line_conf"]] * 4, proto["line_width"])
        assert_bits_equal(g.get_obstacles(), o.get_obstacles(), f"map after lines {cyc}")
        for p in (g, o):
            p.update_boxes(proto["boxes"], [proto["box_conf"]] * 3, proto["apf_r"])
        assert_bits_equal(g.get_obstacles(), o.get_obstacles(), f"map after boxes {cyc}")
    assert_bits_equal(g.apf(), o.apf(), "APF list")
    # a goal change relocates the map (rotate + scatter, Grid3D.cpp:169-203)
    for p in (g, o):
        p.update_goal([30.0, 30.0, 0.7], [10.0, 14.0, 0.0])
    assert_bits_equal(g.get_obstacles(), o.get_obstacles(), "map after relocation")


def test_map_raster_overlapping_boxes(gpu, oracle_lib):
    """Many overlapping boxes with per-box confidences, at a rotated goal frame: the
    layered parallel raster must apply overlapping boxes in the reference's order, with
    the per-update clamp (Grid2D.cpp:99-139) saturating at both bounds."""
    from path_planning_pkg_amd.capi import PlannerConfig
    rng = np.random.default_rng(11)
    cfg = PlannerConfig(grid_size=200, num_angle_bins=36)
    g, o = both(cfg, gpu, oracle_lib)
    for p in (g, o):
        p.update_goal([5.0, 3.0, 0.4], [-30.0, -20.0, 0.0])
    for cyc in range(4):
        k = 150
        boxes = np.stack([rng.uniform(-40, 10, k), rng.uniform(-30, 20, k), rng.uniform(0.5, 9, k),
                          rng.uniform(0.5, 9, k)], 1).astype(np.float32)
        conf = rng.uniform(0.05, 0.97, k).astype(np.float32)
        for p in (g, o):
            p.decay()
            p.update_boxes(boxes, conf, 1.5)
        assert_bits_equal(g.get_obstacles(), o.get_obstacles(), f"map after overlapping boxes {cyc}")
    assert_bits_equal(g.apf(), o.apf(), "APF list")


def test_apf_field_and_dubins_units(gpu, oracle_lib):
    cfg, proto, _ = harness()
    g, o = both(cfg, gpu, oracle_lib)
    for p in (g, o):
        drive(p, proto)
    rng = np.random.default_rng(3)
    apf = o.apf()
    poses = []
    for ox, oy, r in apf:
        for _ in range(200):
            a, d = rng.uniform(0, 2 * math.pi), rng.uniform(0, 1.2 * r)
            poses.append([ox + d * math.cos(a), oy + d * math.sin(a), rng.uniform(-math.pi, math.pi)])
    poses = np.array(poses, np.float32)
    assert_bits_equal(g.field(poses), o.field(poses), "APF field")
    rmin = o.min_radius()
    starts = np.stack([rng.uniform(0, 30, 4000), rng.uniform(0, 30, 4000), rng.uniform(-math.pi, math.pi, 4000)],
                      1).astype(np.float32)
    goal = [24.0, 15.0, 0.3]
    lg, wg = gpu.gpu_dubins_len(rmin, starts, goal)
    lo, wo = oracle_lib.dubins_len(rmin, 0.75, starts, goal)
    assert_bits_equal(lg, lo, "Dubins length")
    assert (wg == wo).all()
    # the handle's goal pose in the grid frame: (n45*res, n2*res, wrap_pi(goal.h - grid_heading))
    gh = oracle_lib.libm(2, np.float32([36.0 - 18.0]), np.float32([26.0 - 18.0]))[0]
    goal_grid = [48 * 0.5, 30 * 0.5, float(oracle_lib.libm(5, np.float32([np.float32(0.0) - gh]))[0])]
    for s in starts[:40]:
        xg, cg, Lg, fg = g.dubins_path(s)
        xo, co, Lo, fo = oracle_lib.dubins_path_f(rmin, 0.75, s, goal_grid)
        assert_bits_equal(np.float32(Lg), np.float32(Lo), "shot length")
        assert fg == fo
        assert_bits_equal(xg, xo, "shot samples")
        assert_bits_equal(cg, co, "shot curvature")


# ----------------------------------------------------------------------- full path --
def test_harness_search_parity_and_golden(gpu, oracle_lib):
    cfg, proto, gold = harness()
    g, o = both(cfg, gpu, oracle_lib)
    for p in (g, o):
        drive(p, proto)
    rg = g.find_path(proto["vel"], proto["start"])
    ro = o.find_path(proto["vel"], proto["start"])
    compare_results(rg, ro, "harness")
    assert [[float("%g" % v) for v in row] for row in rg["path"][::-1]] == gold["path_start_to_goal"]
    fg, vg = g.memo()
    fo, vo = o.get_memo()
    assert_bits_equal(fg, fo, "memo f")
    assert (vg == vo).all()
    assert (g.closed_keys() == o.closed_keys()).all()


@pytest.mark.parametrize("N,bins,K,seed", [(256, 36, 10, s) for s in (1, 2, 3, 4)] + [(512, 72, 50, 1), (512, 72, 50, 2)]
                         + [(256, 36, 40, s) for s in (1, 2, 4)] + [(256, 72, 60, s) for s in (1, 2, 4, 5)])
def test_synthetic_parity(gpu, oracle_lib, N, bins, K, seed):
    cfg, proto = synthetic(N, bins, K, seed)
    g, o = both(cfg, gpu, oracle_lib)
    for p in (g, o):
        drive(p, proto)
    assert_bits_equal(g.get_obstacles(), o.get_obstacles(), "map")
    rg = g.find_path(proto["vel"], proto["start"])
    ro = o.find_path(proto["vel"], proto["start"])
    compare_results(rg, ro, f"N{N} K{K} seed{seed}")
    fg, vg = g.memo()
    fo, vo = o.get_memo()
    assert_bits_equal(fg, fo, "memo f")
    assert (vg == vo).all()


def test_replans_without_reset(gpu, oracle_lib):
    """L3 semantics (local_planner.cpp:204-205,241,316): memo and stale node-map f carry over."""
    cfg, proto = synthetic(256, 36, 10, 5)
    g, o = both(cfg, gpu, oracle_lib)
    for p in (g, o):
        drive(p, proto)
    rng = np.random.default_rng(11)
    boxes = proto["boxes"].copy()
    start = list(proto["start"])
    for tick in range(6):
        r = [p.find_path(2.0, start) for p in (g, o)]
        compare_results(r[0], r[1], f"tick {tick}")
        boxes[:, :2] += rng.uniform(-0.2, 0.2, (len(boxes), 2)).astype(np.float32)
        start[0] += 1.5
        for p in (g, o):
            p.decay()
            p.update_boxes(boxes, [0.75] * len(boxes), 2.5)


def test_replan_loop_batched(gpu, oracle_lib):
    """cfg5 semantics at test size: several start/goal pairs replanned
    together each tick (one batched launch), with decay + moved boxes between ticks and
    no reset (local_planner.cpp:241,288,316).  Every pair, every tick, bit-exact."""
    from tests.scenarios import replan_pairs, replan_tick, replan_tick_inputs
    pairs = replan_pairs(256, 36, 12, 6, seed=21)
    gs, os_ = [], []
    for cfg, proto, _ in pairs:
        g, o = both(cfg, gpu, oracle_lib)
        drive(g, proto)
        drive(o, proto)
        gs.append(g)
        os_.append(o)
    bufs = gpu.BatchBuffers(gs, cap=4096)
    for tick in range(4):
        starts = [replan_tick_inputs(proto, v, tick)[0] for _, proto, v in pairs]
        br = gpu.find_path_batch_arrays(gs, [proto["vel"] for _, proto, _ in pairs], starts, buffers=bufs)
        for i, (o, (_, proto, v)) in enumerate(zip(os_, pairs)):
            compare_results(br.result(i), o.find_path(proto["vel"], starts[i]), f"tick {tick} pair {i}")
            replan_tick(gs[i], proto, v, tick)
            replan_tick(o, proto, v, tick)


def test_reset_batch_equals_reset(gpu, oracle_lib):
    """hastar_reset_batch (one kernel clearing every visited bitmap) == reset() per planner:
    a warm memo is dropped, the stale node-map f values stay (AStar.cpp:56-60)."""
    cases = [synthetic(256, 36, 10, s) for s in (12, 13, 14)]
    gs, os_ = [], []
    for cfg, proto in cases:
        g, o = both(cfg, gpu, oracle_lib)
        drive(g, proto)
        drive(o, proto)
        gs.append(g)
        os_.append(o)
    vels = [c[1]["vel"] for c in cases]
    starts = [c[1]["start"] for c in cases]
    gpu.find_path_batch(gs, vels, starts)
    for (cfg, proto), o in zip(cases, os_):
        o.find_path(proto["vel"], proto["start"])
        o.reset()
    gpu.reset_batch(gs)
    res, _ = gpu.find_path_batch(gs, vels, starts)
    for i, ((cfg, proto), o) in enumerate(zip(cases, os_)):
        compare_results(res[i], o.find_path(proto["vel"], proto["start"]), f"after reset_batch {i}")
        fg, vg = gs[i].memo()
        fo, vo = o.get_memo()
        assert_bits_equal(fg, fo, "memo f")
        assert (vg == vo).all()


@pytest.mark.parametrize("wide", ["1", "0"], ids=["latency_kernel", "batch_kernel"])
def test_batch_with_fewer_slots(gpu, oracle_lib, monkeypatch, wide):
    """Fewer slots than planners (3 latency workgroups, or 3 waves of one batch-kernel
    workgroup whose 5 other waves take no work): the persistent queue hands every planner to
    a slot, and every result is still the oracle's."""
    monkeypatch.setenv("HASTAR_WIDE", wide)
    monkeypatch.setenv("HASTAR_SLOTS", "3")
    cases = [synthetic(128, 36, 6, s) for s in (31, 32, 33, 34, 35, 36, 37)]
    gs, os_ = [], []
    for cfg, proto in cases:
        g, o = both(cfg, gpu, oracle_lib)
        drive(g, proto)
        drive(o, proto)
        gs.append(g)
        os_.append(o)
    res, _ = gpu.find_path_batch(gs, [c[1]["vel"] for c in cases], [c[1]["start"] for c in cases])
    for i, ((cfg, proto), o) in enumerate(zip(cases, os_)):
        compare_results(res[i], o.find_path(proto["vel"], proto["start"]), f"3-slot batch {i}")


@pytest.mark.parametrize("wide", ["1", "0"], ids=["latency_kernel", "batch_kernel"])
def test_small_inner_arena_bounds_both_kernels_alike(gpu, oracle_lib, monkeypatch, wide):
    """max_astar_nodes below the LDS pool (1024 / 2048 nodes): the LDS tree migrates before the
    pool could outgrow the arena's HBM tree, so a search either ends like the oracle's or, when
    an inner search needs more nodes than the arena holds, with HASTAR_EOVERFLOW on both kernels
    alike (the latency kernel copied up to 2048 nodes into a 601-node open2)."""
    monkeypatch.setenv("HASTAR_WIDE", wide)
    from path_planning_pkg_amd.capi import PlannerConfig
    outs = []
    for cap in (600, 1500):
        cfg, proto = synthetic_ref(1024, 72, 200, 1)
        cfg = PlannerConfig(**{**cfg.values, "max_astar_nodes": cap}, steering=cfg.steering)
        g, o = both(cfg, gpu, oracle_lib)
        drive(g, proto)
        drive(o, proto)
        r = g.find_path(proto["vel"], proto["start"])
        outs.append(r["stats"]["status"])
        if r["stats"]["status"] == 0:
            compare_results(r, o.find_path(proto["vel"], proto["start"]), f"max_astar_nodes={cap}")
        else:
            assert r["stats"]["status"] == -75 and not r["ok"]
    # seed 1's inner searches need more than 600 nodes but not more than 1500 (tools/astar_shape_stats.py)
    assert outs == [-75, 0], outs


def test_reserve_then_batch(gpu, oracle_lib):
    """hastar_reserve sizes the device pool ahead of a batch (and rejects bad arguments); the
    batch that follows still returns the oracle's results."""
    cases = [synthetic(128, 36, 6, s) for s in (41, 42, 43)]
    gs, os_ = [], []
    for cfg, proto in cases:
        g, o = both(cfg, gpu, oracle_lib)
        drive(g, proto)
        drive(o, proto)
        gs.append(g)
        os_.append(o)
    with pytest.raises(gpu.HastarError):
        gpu.reserve(gs, path_points=-1)
    gpu.reserve(gs, path_points=4096)
    res, _ = gpu.find_path_batch(gs, [c[1]["vel"] for c in cases], [c[1]["start"] for c in cases])
    for i, ((cfg, proto), o) in enumerate(zip(cases, os_)):
        compare_results(res[i], o.find_path(proto["vel"], proto["start"]), f"reserved batch {i}")


@pytest.mark.parametrize("wide", ["1", "0"], ids=["latency_kernel", "batch_kernel"])
def test_batch_equals_single(gpu, oracle_lib, monkeypatch, wide):
    monkeypatch.setenv("HASTAR_WIDE", wide)
    cases = [synthetic(256, 36, 10, s) for s in (6, 7, 8)] + [harness()[:2]]
    planners, oracles = [], []
    for cfg, proto in cases:
        g, o = both(cfg, gpu, oracle_lib)
        drive(g, proto)
        drive(o, proto)
        planners.append(g)
        oracles.append(o)
    res, ms = gpu.find_path_batch(planners, [c[1]["vel"] for c in cases], [c[1]["start"] for c in cases])
    assert ms > 0
    for i, (cfg, proto) in enumerate(cases):
        compare_results(res[i], oracles[i].find_path(proto["vel"], proto["start"]), f"batch {i}")


def test_edge_cases(gpu, oracle_lib):
    # start outside the grid -> cell (0, 0) with pose (0, 0, 0) (Grid3D.cpp:153-159)
    cfg, proto = synthetic(128, 36, 4, 9)
    g, o = both(cfg, gpu, oracle_lib)
    for p in (g, o):
        drive(p, proto)
    far = [-500.0, 300.0, 1.0]
    compare_results(g.find_path(1.0, far), o.find_path(1.0, far), "start outside")
    # goal cell fully walled in: search fails on both (small grid, bounded flood)
    cfg, proto = synthetic(48, 36, 0, 1)
    proto["boxes"] = np.array([[0.0, 0.0, 4.0, 4.0]], np.float32)
    proto["start"] = [-14.0, 0.0, 0.0]
    g, o = both(cfg, gpu, oracle_lib)
    for p in (g, o):
        drive(p, proto)
    rg, ro = g.find_path(2.0, proto["start"]), o.find_path(2.0, proto["start"])
    compare_results(rg, ro, "blocked goal")
    assert not rg["ok"]
    # lines only, no boxes, num_actions = 2, 4-connected holonomic A*
    from path_planning_pkg_amd.capi import PlannerConfig, steering_from_degrees
    cfg = PlannerConfig(grid_size=80, num_angle_bins=72, num_actions=2, grid_2d_allow_diag_moves=False,
                        steering=steering_from_degrees([-30, -20, -10, 0, 10, 20, 30]),
                        curvature_weights=[0.5, 0.2, 0.1, 0.0, 0.1, 0.2, 0.5])
    proto = dict(goal=[5.0, 3.0, -0.4], start=[-20.0, -6.0, 0.3], vel=3.0, cycles=3,
                 lines=np.array([[-10, -10, -10, 2], [-2, 0, 3, 12]], np.float32), line_conf=0.7, line_width=1.0,
                 boxes=np.zeros((0, 4), np.float32), box_conf=0.75, apf_r=2.5)
    g, o = both(cfg, gpu, oracle_lib)
    for p in (g, o):
        drive(p, proto)
    assert_bits_equal(g.get_obstacles(), o.get_obstacles(), "lines-only map")
    compare_results(g.find_path(3.0, proto["start"]), o.find_path(3.0, proto["start"]), "lines only")


def test_small_output_buffer(gpu):
    from path_planning_pkg_amd import planner
    cfg, proto, _ = harness()
    g = gpu.HybridAStar(cfg)
    drive(g, proto)
    r = g.find_path(proto["vel"], proto["start"], cap=5)   # wrapper retries after HASTAR_ENOSPC
    assert r["ok"] and len(r["path"]) == 43
    assert planner.HASTAR_ENOSPC == -28


@pytest.mark.parametrize("N,world", [(254, 3), (256, 4)])
def test_row_sharded_map_build(gpu, oracle_lib, N, world):
    """cfg4's map build: `world` planners on this GPU stand in for the ranks.
    Each builds only its row block (hastar_set_row_window), exports it into one buffer laid out
    as all_gather_into_tensor would, and imports the whole map back.  The window must confine
    decay and both rasters to its rows (N = 254, world = 3: blocks start off a 16-B boundary),
    and the gathered map and the search on it must equal the oracle's single-core build."""
    import torch
    from path_planning_pkg_amd.shard import row_blocks
    cfg, proto = synthetic(N, 36, 10, 7)
    proto["lines"] = np.array([[-60.0, -20.0, -20.0, 10.0], [-90.0, 30.0, -40.0, -30.0]], np.float32)
    o = oracle_lib.OraclePlanner(cfg)
    drive(o, proto)
    ref = o.get_obstacles()
    blocks, R = row_blocks(N, world)
    buf = torch.zeros(world * R * N, dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    shards = [gpu.HybridAStar(cfg) for _ in range(world)]
    for r, (p, (r0, r1)) in enumerate(zip(shards, blocks)):
        p.update_goal(proto["goal"], proto["start"])
        p.set_row_window(r0, r1)
        for _ in range(proto["cycles"]):
            p.decay()
            p.update_lines(proto["lines"], [proto["line_conf"]] * len(proto["lines"]), proto["line_width"])
            p.update_boxes(proto["boxes"], [proto["box_conf"]] * len(proto["boxes"]), proto["apf_r"])
        p.set_row_window(0, N)
        m = p.get_obstacles()
        assert_bits_equal(m[r0:r1], ref[r0:r1], f"rank {r} block")
        assert not m[:r0].any() and not m[r1:].any(), f"rank {r} wrote outside its rows"
        p.export_rows(r0, r1, buf.data_ptr() + r * R * N * 4)
    for p in shards:
        p.import_rows(0, N, buf.data_ptr())
        p.reset()
        assert_bits_equal(p.get_obstacles(), ref, "gathered map")
    compare_results(shards[-1].find_path(proto["vel"], proto["start"]), o.find_path(proto["vel"], proto["start"]),
                    f"search on the gathered map N{N} x{world}")
    with pytest.raises(gpu.HastarError):
        shards[0].set_row_window(5, N + 1)
