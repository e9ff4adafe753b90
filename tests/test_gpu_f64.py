"""HybridAStar<double> / VelocityGenerator<double> on the GPU (include/hastar_f64.h) against the
oracle's double instantiation (oracle/hastar_oracle.cpp, Planner<double>).

The reference instantiates both classes for double (HybridAStar.cpp:285-286,
VelocityGenerator.cpp:88-89) and its LocalPlanner<double> calls them (local_planner.cpp:378-500).
The device's sin, cos, atan2, acos and hypot are ports of the host glibc 2.35's own routines
(csrc/hastar_libm64.h: the FMA variants __sin_fma / __cos_fma / __ieee754_atan2_fma /
__ieee754_acos_fma and e_hypot.c; 0 mismatches in 2e8 device samples each,
tools/libm64_fingerprint.hip, and tests/test_libm64_ports.py on the host).  They are bit-exact
for every finite argument except sin/cos of |x| >= 2^27 * pi/2 (~1.05e8), where glibc's
__branred reduction is not ported; the planner's angles are wrapped to [-pi, pi].  So the bar
here is bit equality: success, cost bits, pop count and digest, the closed set, path and
curvature bits, and the memo after the search.  Parity is unpinned at the reference: the reference holds no
double fixture for the planner (its double golden vectors, utils/dubins_paths.py:6 and
utils/vehicle_mode.py:12, pin the Dubins / VehicleModel units, tests/test_cxx_units.py); the
oracle's float instantiation of the same template is pinned by the reference's golden path.
"""
import numpy as np
import pytest

from tests.scenarios import drive, harness, replan_pairs, replan_tick, replan_tick_inputs, synthetic_ref

pytestmark = pytest.mark.gpu

# bench queries of the double cfg3 sample: 0-2 (the survey's seeds 1-3) and every 1000th up to
# 18000 (the bench draws query q with seed q + 1)
CFG3_QUERIES = [0, 1, 2] + [1000 * k for k in range(1, 19)]


def _pair(cfg):
    from oracle.pyoracle import OraclePlanner64
    from path_planning_pkg_amd.planner64 import HybridAStar64
    return HybridAStar64(cfg), OraclePlanner64(cfg)


def _proto64(proto):
    out = dict(proto)
    for k in ("boxes", "lines"):
        out[k] = np.asarray(proto[k], np.float64)
    return out


def _bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


def _compare(rg, ro, g, o, label=""):
    """Bit equality of one double search: success, cost bits, statistics and digests, the closed
    set, path and curvature bits, and the memo (node-map f bits and visited flags) after it."""
    assert rg["ok"] == ro["ok"], label
    sg, so = rg["stats"], ro["stats"]
    for k in ("pops", "successors", "astar_pops", "astar_searches", "shots", "closed_size", "pop_digest",
              "closed_digest", "via_shot"):
        assert sg[k] == so[k], (label, k, sg[k], so[k])
    assert np.array_equal(g.closed_keys(), o.closed_keys()), label
    assert np.float64(rg["cost"]).view(np.uint64) == np.float64(ro["cost"]).view(np.uint64), (label, rg["cost"], ro["cost"])
    if ro["ok"]:
        assert np.array_equal(_bits(rg["path"]), _bits(ro["path"])), label
        assert np.array_equal(_bits(rg["curvature"]), _bits(ro["curvature"])), label
    fg, vg = g.memo()
    fo, vo = o.get_memo()
    assert np.array_equal(vg, vo), label
    assert np.array_equal(_bits(fg), _bits(fo)), label


def test_f64_harness_matches_oracle():
    cfg, proto, _ = harness()
    proto = _proto64(proto)
    g, o = _pair(cfg)
    drive(g, proto)
    drive(o, proto)
    assert np.array_equal(g.get_obstacles(), o.get_obstacles())  # map upkeep: no libm on the device
    rg, ro = g.find_path(proto["vel"], proto["start"]), o.find_path(proto["vel"], proto["start"])
    assert ro["ok"]
    _compare(rg, ro, g, o, "harness")
    # a replan without reset: the memo and the stale node-map values carry over
    rg2, ro2 = g.find_path(proto["vel"], proto["start"]), o.find_path(proto["vel"], proto["start"])
    _compare(rg2, ro2, g, o, "harness replan")


@pytest.mark.parametrize("N,bins,K,seed", [(256, 36, 10, 1), (256, 36, 10, 3), (256, 36, 40, 7), (512, 72, 50, 1)])
def test_f64_synthetic_matches_oracle(N, bins, K, seed):
    cfg, proto = synthetic_ref(N, bins, K, seed)
    proto = _proto64(proto)
    g, o = _pair(cfg)
    drive(g, proto)
    drive(o, proto)
    assert np.array_equal(g.get_obstacles(), o.get_obstacles())
    _compare(g.find_path(proto["vel"], proto["start"]), o.find_path(proto["vel"], proto["start"]), g, o, f"N={N} seed={seed}")


@pytest.mark.parametrize("q", CFG3_QUERIES)
def test_f64_cfg3_queries_match_oracle(q):
    """cfg3 size (1024x1024x72, K = 200), a stratified sample of 21 bench queries: the double
    search is a search of its own (other pop counts than the float one) and must equal the
    oracle's double one bit for bit."""
    cfg, proto = synthetic_ref(1024, 72, 200, q + 1)
    proto = _proto64(proto)
    g, o = _pair(cfg)
    drive(g, proto)
    drive(o, proto)
    _compare(g.find_path(proto["vel"], proto["start"]), o.find_path(proto["vel"], proto["start"]), g, o, f"cfg3 query {q}")


def test_f64_cfg5_pair_three_ticks():
    """cfg5 at its own size, bench pair 0 (seed 1000), 3 ticks of the replan loop without reset
    (local_planner.cpp:204-205, 241, 316; the double node calls HybridAStar<double>): moving boxes,
    decay, the memo and stale node-map values carried over, each tick bit-equal to the oracle."""
    cfg, proto, v = replan_pairs(1024, 72, 200, 1, seed=1000)[0]
    proto = _proto64(proto)
    g, o = _pair(cfg)
    drive(g, proto)
    drive(o, proto)
    for tick in range(3):
        start = [float(x) for x in replan_tick_inputs(proto, v, tick)[0]]
        _compare(g.find_path(proto["vel"], start), o.find_path(proto["vel"], start), g, o, f"cfg5 tick {tick}")
        _, boxes = replan_tick_inputs(proto, v, tick + 1)
        for p in (g, o):
            p.decay()
            p.update_boxes(np.asarray(boxes, np.float64), [proto["box_conf"]] * len(boxes), proto["apf_r"])
        assert np.array_equal(g.get_obstacles(), o.get_obstacles())


def test_f64_arena_growth_reruns_give_the_same_result():
    """Tiny arenas: the search stops, the memo is restored and it re-runs in 4x arenas until it
    fits (no limit, HybridAStar.cpp:107): the result equals the oracle's and a default run's."""
    from path_planning_pkg_amd.capi import PlannerConfig
    cfg, proto = synthetic_ref(256, 36, 10, 3)
    proto = _proto64(proto)
    small = PlannerConfig(**{**cfg.values, "max_pops": 16, "max_astar_nodes": 8, "max_dubins_samples": 4},
                          steering=cfg.steering64, curvature_weights=cfg.curvature_weights64)
    from oracle.pyoracle import OraclePlanner64
    from path_planning_pkg_amd.planner64 import HybridAStar64
    g, o = HybridAStar64(small), OraclePlanner64(small)
    drive(g, proto)
    drive(o, proto)
    rg, ro = g.find_path(proto["vel"], proto["start"]), o.find_path(proto["vel"], proto["start"])
    assert g.arena()["reruns"] >= 3, g.arena()
    _compare(rg, ro, g, o, "arena growth")


def test_f64_edge_cases():
    """Lines-only 4-connected map with 7 actions, a path longer than the caller's cap, a start
    outside the grid (the (0, 0) default node, Grid3D.cpp:150-159), a walled-in goal (no path:
    the search empties its open set)."""
    from path_planning_pkg_amd.capi import PlannerConfig, steering_from_degrees_f64
    cfg = PlannerConfig(grid_size=40, grid_2d_allow_diag_moves=False, num_actions=3, num_angle_bins=36,
                        steering=steering_from_degrees_f64([-30, -20, -10, 0, 10, 20, 30]))
    lines = np.array([[-6.0, -4.0, -6.0, 4.0], [-10.0, 2.0, -8.0, 8.0]])
    g, o = _pair(cfg)
    for p in (g, o):
        p.update_goal([0.0, 0.0, 0.3], [-12.0, 1.0, 0.0])
        for _ in range(3):
            p.decay()
            p.update_lines(lines, [0.7, 0.7], 1.0)
        p.reset()
    assert np.array_equal(g.get_obstacles(), o.get_obstacles())
    _compare(g.find_path(1.5, [-12.0, 1.0, 0.1], cap=4), o.find_path(1.5, [-12.0, 1.0, 0.1]), g, o, "short cap")
    _compare(g.find_path(0.5, [500.0, -300.0, 0.0]), o.find_path(0.5, [500.0, -300.0, 0.0]), g, o, "start outside")
    box = np.array([[0.0, 0.0, 4.0, 4.0]])
    for p in (g, o):
        for _ in range(6):
            p.update_boxes(box, [0.95], 1.0)
    assert np.array_equal(g.get_obstacles(), o.get_obstacles())
    rg, ro = g.find_path(1.5, [-12.0, 1.0, 0.1]), o.find_path(1.5, [-12.0, 1.0, 0.1])
    assert not ro["ok"]
    _compare(rg, ro, g, o, "walled-in goal")


def test_f64_velocity_generator_matches_oracle():
    from oracle.pyoracle import velocity_profile64
    from path_planning_pkg_amd.planner64 import VelocityGenerator64
    rng = np.random.default_rng(11)
    prm = (10.0, 3.0, 2.5, 1.5, 3.0)
    vg = VelocityGenerator64(*prm)
    paths, curvs, v0, vm, coast, stop = [], [], [], [], [], []
    for i in range(200):
        n = int(rng.integers(1, 300))
        xy = np.cumsum(rng.normal(0, 0.5, (n, 2)), axis=0)
        paths.append(np.concatenate([xy, rng.uniform(-3, 3, (n, 1))], 1))
        curvs.append(np.where(rng.random(n) < 0.3, 0.0, rng.uniform(0, 0.3, n)))
        v0.append(float(rng.uniform(0, 8)))
        vm.append(float(rng.uniform(2, 12)))
        coast.append(bool(i % 3 == 0))
        stop.append(bool(i % 2 == 0))
    ok, vel = vg.generate_velocity_profiles(v0, vm, paths, curvs, coast, stop)
    for i in range(200):
        ok_o, v_o = velocity_profile64(prm, v0[i], vm[i], paths[i], curvs[i], coast[i], stop[i])
        assert ok[i] == ok_o
        # bit for bit (the device hypot is glibc's), NaN where 1 - lat²/a² < 0 as in the reference
        assert np.array_equal(np.asarray(vel[i], np.float64).view(np.uint64), np.asarray(v_o, np.float64).view(np.uint64)), i
