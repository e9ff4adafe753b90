"""The CPU oracle against the reference's own known-answer vectors.

These pin the oracle: utils/hybrid_astar/plot.py:47-51, utils/dubins_paths.py:6 and
utils/vehicle_mode.py:12 were printed by the reference with ostream's default %g; we
compare at that precision, element by element.  At full cfg3 size the oracle is pinned by the
pop / successor / inner-A* counts the survey measured on the compiled reference for its
std::mt19937 inputs (tests/golden/survey_reference_counts.json).
"""
import json
import math

import numpy as np

from tests.scenarios import GOLDEN, drive, harness


def g6(v):
    return float("%g" % v)


def test_harness_path_matches_plot_py(oracle_lib):
    cfg, proto, gold = harness()
    o = oracle_lib.OraclePlanner(cfg)
    drive(o, proto)
    r = o.find_path(proto["vel"], proto["start"])
    assert r["ok"]
    assert "%g" % r["cost"] == "33.0305"
    mine = [[g6(v) for v in row] for row in r["path"][::-1]]   # harness prints path.rbegin()..rend()
    assert mine == gold["path_start_to_goal"]
    assert len(r["curvature"]) == len(r["path"])


def test_dubins_rsl_matches_dubins_paths_py(oracle_lib):
    g = json.loads((GOLDEN / "dubins_rsl.json").read_text())
    ms = 30.0 * math.pi / 180.0
    beta = math.atan2(1.1 * math.tan(ms), 2.269)
    rmin = 2.269 / (math.tan(ms) * math.cos(beta))
    path, length, word = oracle_lib.dubins_path_d(rmin, 0.5, [0.0, 0.0, 0.0], [20.0, -20.0, math.pi / 2])
    assert word == 1  # RSL
    assert "%g" % rmin == "4.08106"
    assert [[g6(v) for v in row] for row in path.tolist()] == g["path"]


def test_vehicle_chain_matches_vehicle_mode_py(oracle_lib):
    g = json.loads((GOLDEN / "vehicle_chain.json").read_text())
    st = [d * math.pi / 180.0 for d in g["steering_deg"]]
    pos = oracle_lib.vehicle_chain_d(0.5, 4.0, 2.269, 1.1, 72, 1, st, [0.0] * 7, 16.0, 3, g["actions"])
    assert [[g6(v) for v in row] for row in pos.tolist()] == g["positions"]


def test_equal_f_insert_is_dropped(oracle_lib):
    """utils/node3D/test_node3D.cpp:29-65 semantics: the reference comparator drops equal-f
    inserts; reproduced indirectly — the harness closed set is smaller than its pops."""
    cfg, proto, _ = harness()
    o = oracle_lib.OraclePlanner(cfg)
    drive(o, proto)
    r = o.find_path(proto["vel"], proto["start"])
    st = r["stats"]
    assert st["closed_size"] <= st["pops"]
    keys = o.closed_keys()
    assert len(keys) == st["closed_size"]
    assert len({tuple(k) for k in keys.tolist()}) == len(keys)


def test_oracle_matches_survey_reference_counts(oracle_lib):
    """The oracle against counts the survey measured on the compiled reference at 256² to 2048²,
    including full cfg3 size (tests/golden/survey_reference_counts.json): the same std::mt19937
    inputs (tests/scenarios.py:synthetic_ref) give the same pops, successors and inner A* pops."""
    from tests.scenarios import synthetic_ref
    g = json.loads((GOLDEN / "survey_reference_counts.json").read_text())
    for case in g["cases"]:
        cfg, proto = synthetic_ref(case["grid"], case["angle_bins"], case["obstacles"], case["seed"])
        o = oracle_lib.OraclePlanner(cfg)
        drive(o, proto)
        r = o.find_path(proto["vel"], proto["start"])
        o.close()
        assert r["ok"]
        for k in ("pops", "successors", "astar_pops"):
            if k in case:
                assert r["stats"][k] == case[k], f"{case}: {k} {r['stats'][k]} vs reference {case[k]}"


def test_reference_generator_definitions_agree(tmp_path):
    """synthetic_ref's vectorised draw == the scalar std::mt19937 restatement == the C++
    generator compiled with libstdc++ (tools/mt19937_synth.cpp, variant 3), bit for bit."""
    import subprocess
    from pathlib import Path
    from tests.scenarios import synthetic_ref_boxes, synthetic_ref_boxes_scalar
    root = Path(__file__).resolve().parents[1]
    exe = tmp_path / "mt19937_synth"
    subprocess.run(["g++", "-O2", "-std=c++17", str(root / "tools" / "mt19937_synth.cpp"), "-o", str(exe)], check=True)
    for seed in (1, 3, 10227):
        a, _ = synthetic_ref_boxes(1024, 200, seed)
        b, _ = synthetic_ref_boxes_scalar(1024, 200, seed)
        c = np.array(json.loads(subprocess.run([str(exe), "1024", "200", str(seed), "3"], capture_output=True,
                                               text=True, check=True).stdout), np.float32).reshape(-1, 4)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
        assert np.array_equal(a.view(np.uint32), c.view(np.uint32))
