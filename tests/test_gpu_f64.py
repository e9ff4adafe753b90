"""HybridAStar<double> / VelocityGenerator<double> on the GPU (include/hastar_f64.h) against the
oracle's double instantiation (oracle/hastar_oracle.cpp, Planner<double>).

The reference instantiates both classes for double (HybridAStar.cpp:285-286,
VelocityGenerator.cpp:88-89) and its LocalPlanner<double> calls them (local_planner.cpp:378-500).
Bar (BASELINE.json north_star): the same goal-reached decision, identical closed-set membership,
final cost within 1e-4 relative.  The device's f64 sin/cos/atan2/acos/hypot are within an ulp or
two of glibc's, so the comparison is by tolerance; the tests also require the same pop count and
report how many results are bit-identical.  Parity is unpinned at the reference: the reference
holds no double fixture for the planner (its double golden vectors, utils/dubins_paths.py:6 and
utils/vehicle_mode.py:12, pin the Dubins / VehicleModel units, tests/test_cxx_units.py); the
oracle's float instantiation of the same template is pinned by the reference's golden path.
"""
import numpy as np
import pytest

from tests.scenarios import drive, harness, synthetic_ref

pytestmark = pytest.mark.gpu

REL = 1e-4  # north_star's cost tolerance


def _pair(cfg):
    from oracle.pyoracle import OraclePlanner64
    from path_planning_pkg_amd.planner64 import HybridAStar64
    return HybridAStar64(cfg), OraclePlanner64(cfg)


def _proto64(proto):
    out = dict(proto)
    for k in ("boxes", "lines"):
        out[k] = np.asarray(proto[k], np.float64)
    return out


def _compare(rg, ro, g, o, exact_counter):
    assert rg["ok"] == ro["ok"]
    sg, so = rg["stats"], ro["stats"]
    assert sg["pops"] == so["pops"] and sg["closed_size"] == so["closed_size"], (sg, so)
    assert np.array_equal(g.closed_keys(), o.closed_keys())
    if ro["ok"]:
        assert abs(rg["cost"] - ro["cost"]) <= REL * abs(ro["cost"]), (rg["cost"], ro["cost"])
        assert rg["path"].shape == ro["path"].shape
        assert np.allclose(rg["path"], ro["path"], rtol=1e-9, atol=1e-9)
        assert np.allclose(rg["curvature"], ro["curvature"], rtol=1e-12, atol=0)
    same = (rg["cost"] == ro["cost"] and sg["pop_digest"] == so["pop_digest"] and np.array_equal(rg["path"], ro["path"]))
    exact_counter.append(bool(same))


def test_f64_harness_matches_oracle():
    cfg, proto, _ = harness()
    proto = _proto64(proto)
    g, o = _pair(cfg)
    drive(g, proto)
    drive(o, proto)
    assert np.array_equal(g.get_obstacles(), o.get_obstacles())  # map upkeep: no libm on the device
    exact = []
    rg, ro = g.find_path(proto["vel"], proto["start"]), o.find_path(proto["vel"], proto["start"])
    assert ro["ok"]
    _compare(rg, ro, g, o, exact)
    fg, vg = g.memo()
    fo, vo = o.get_memo()
    assert np.array_equal(vg, vo)
    assert np.allclose(fg, fo, rtol=1e-12, atol=1e-12)
    # a replan without reset: the memo and the stale node-map values carry over
    rg2, ro2 = g.find_path(proto["vel"], proto["start"]), o.find_path(proto["vel"], proto["start"])
    _compare(rg2, ro2, g, o, exact)
    print("bit-identical:", exact)


@pytest.mark.parametrize("N,bins,K,seed", [(256, 36, 10, 1), (256, 36, 10, 3), (256, 36, 40, 7), (512, 72, 50, 1)])
def test_f64_synthetic_matches_oracle(N, bins, K, seed):
    cfg, proto = synthetic_ref(N, bins, K, seed)
    proto = _proto64(proto)
    g, o = _pair(cfg)
    drive(g, proto)
    drive(o, proto)
    assert np.array_equal(g.get_obstacles(), o.get_obstacles())
    exact = []
    _compare(g.find_path(proto["vel"], proto["start"]), o.find_path(proto["vel"], proto["start"]), g, o, exact)
    print(f"N={N} seed={seed} bit-identical:", exact)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_f64_cfg3_queries_match_oracle(seed):
    """cfg3 size (1024x1024x72, K = 200; bench queries 0-2): the double search is a search of its
    own (other pop counts than the float one) and must still equal the oracle's double one."""
    cfg, proto = synthetic_ref(1024, 72, 200, seed)
    proto = _proto64(proto)
    g, o = _pair(cfg)
    drive(g, proto)
    drive(o, proto)
    exact = []
    _compare(g.find_path(proto["vel"], proto["start"]), o.find_path(proto["vel"], proto["start"]), g, o, exact)
    print(f"cfg3 seed {seed} bit-identical:", exact)


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
    _compare(rg, ro, g, o, [])


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
    exact = []
    _compare(g.find_path(1.5, [-12.0, 1.0, 0.1], cap=4), o.find_path(1.5, [-12.0, 1.0, 0.1]), g, o, exact)
    _compare(g.find_path(0.5, [500.0, -300.0, 0.0]), o.find_path(0.5, [500.0, -300.0, 0.0]), g, o, exact)
    box = np.array([[0.0, 0.0, 4.0, 4.0]])
    for p in (g, o):
        for _ in range(6):
            p.update_boxes(box, [0.95], 1.0)
    assert np.array_equal(g.get_obstacles(), o.get_obstacles())
    rg, ro = g.find_path(1.5, [-12.0, 1.0, 0.1]), o.find_path(1.5, [-12.0, 1.0, 0.1])
    assert not ro["ok"]
    _compare(rg, ro, g, o, exact)
    print("bit-identical:", exact)


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
        assert np.allclose(vel[i], v_o, rtol=1e-12, atol=1e-12, equal_nan=True), i  # NaN where 1 - lat²/a² < 0, as in the reference
