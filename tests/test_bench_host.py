"""Host-side logic of bench.py (no GPU): workload defaults and the step-balance summary.

bench.py's cfg3 default arena size (196,608 pops) must cover the batch's longest search
(query 2395: 172,207 pops in the oracle census, profiles/census_cfg3_mt19937_r02.csv), or that
search would park and resume after the rest of the batch; cfg4 fills the HBM with 7680
planners (its step is bound by one 597k-pop search).
"""
import csv
from pathlib import Path

import bench

ROOT = Path(__file__).resolve().parents[1]


def test_workload_defaults():
    a = bench.parse_args([])
    assert a.workload == "cfg3" and a.grid == 1024 and a.batch == 23552 and a.max_pops == 196608
    c4 = bench.parse_args(["--workload", "cfg4"])
    assert c4.grid == 2048 and c4.max_pops == 0
    assert bench.parse_args(["--max-pops", "0"]).max_pops == 0  # the library's default arena


def test_cfg3_arena_covers_the_longest_search():
    with open(ROOT / "profiles" / "census_cfg3_mt19937_r02.csv") as f:
        pops = [int(r["pops"]) for r in csv.DictReader(f)]
    assert len(pops) == 23552
    assert max(pops) < bench.parse_args([]).max_pops


class _Planner:
    def __init__(self, t0, t1, slot):
        self._t = (t0, t1, slot)

    def timing(self):
        return self._t


def test_step_balance():
    # two slots; slot 0 runs a 3-ms search and a 1-ms one, slot 1 one 2-ms search (10 ns ticks)
    ps = [_Planner(0, 300000, 0), _Planner(300000, 400000, 0), _Planner(50000, 250000, 1)]
    b = bench.step_balance(ps)
    assert b["slots_used"] == 2
    assert abs(b["span_ms"] - 4.0) < 1e-9
    assert abs(b["slot_busy_mean_ms"] - 3.0) < 1e-9
    assert abs(b["busy_frac"] - 0.75) < 1e-9
    assert abs(b["longest_search_under_load_ms"] - 3.0) < 1e-9 and b["longest_search_start_ms"] == 0.0


def test_parity_sample_compares_every_field():
    """bench.parity_sample (the bench's bit-exact check of a stratified sample of its own batch):
    results equal to the oracle's pass, a one-bit difference in a path or a digest fails."""
    import numpy as np
    import bench
    from oracle.pyoracle import OraclePlanner
    from tests.scenarios import drive, synthetic_ref
    cfgs = [synthetic_ref(256, 36, 20, s) for s in (1, 2, 3)]
    ref = {}
    for i, (cfg, proto) in enumerate(cfgs):
        o = OraclePlanner(cfg)
        drive(o, proto)
        o.reset()
        ref[i] = o.find_path(proto["vel"], proto["start"])
        o.close()
    r = bench.parity_sample(cfgs, ref, [0, 1, 2])
    assert r["bit_exact"] and r["queries"] == 3 and r["path_poses_checked"] > 0, r
    bent = dict(ref)
    p = ref[1]["path"].copy()
    p.view(np.uint32)[0, 0] ^= 1
    bent[1] = dict(ref[1], path=p)
    r = bench.parity_sample(cfgs, bent, [10, 11, 12])
    assert not r["bit_exact"] and r["mismatched_queries"] == [11], r
    st = dict(ref[2]["stats"], closed_digest=ref[2]["stats"]["closed_digest"] ^ 1)
    bent = dict(ref)
    bent[2] = dict(ref[2], stats=st)
    assert bench.parity_sample(cfgs, bent, [0, 1, 2])["mismatched_queries"] == [2]


def test_parity_sample_replays_every_replan_for_the_last_step():
    """With the last timed step given, the oracle replays reset + find_path `replans` times (the
    node map's f values persist across reset, HybridAStar.cpp:49-52) and compares its last replan
    with it; a one-bit difference in the last step's path fails that check alone."""
    import numpy as np
    import bench
    from oracle.pyoracle import OraclePlanner
    from tests.scenarios import drive, synthetic_ref
    cfgs = [synthetic_ref(256, 36, 20, s) for s in (1, 3)]
    first, fourth = {}, {}
    for i, (cfg, proto) in enumerate(cfgs):
        o = OraclePlanner(cfg)
        drive(o, proto)
        for k in range(4):
            o.reset()
            r = o.find_path(proto["vel"], proto["start"])
            if k == 0:
                first[i] = r
        fourth[i] = r
        o.close()
    r = bench.parity_sample(cfgs, first, [0, 1], fourth, 4)
    assert r["bit_exact"] and r["last_timed_step"]["bit_exact"] and r["last_timed_step"]["replans_replayed"] == 4, r
    p = fourth[1]["path"].copy()
    p.view(np.uint32)[0, 0] ^= 1
    bent = dict(fourth)
    bent[1] = dict(fourth[1], path=p)
    r = bench.parity_sample(cfgs, first, [7, 8], bent, 4)
    assert r["mismatched_queries"] == [] and not r["bit_exact"], r
    assert r["last_timed_step"]["mismatched_queries"] == [8], r


def test_parity_all_checks_every_query():
    """bench.parity_all (--parity-all): every query's cold-step statistics, digests (compared
    modulo 2^64, whatever the integer width they arrive in), success, cost bits and the digest of
    its path and curvature bits."""
    import numpy as np
    import bench
    from oracle.pyoracle import OraclePlanner
    from tests.scenarios import drive, synthetic_ref
    cfgs = [synthetic_ref(256, 36, 20, s) for s in (1, 2)]
    keys = ("pops", "successors", "astar_pops", "astar_searches", "shots", "closed_size", "pop_digest",
            "closed_digest", "via_shot")
    st = np.zeros(2, dtype=[(k, "i8") for k in keys])
    cost, ok = np.zeros(2, np.float32), np.zeros(2, np.int32)
    paths = []
    for i, (cfg, proto) in enumerate(cfgs):
        o = OraclePlanner(cfg)
        drive(o, proto)
        o.reset()
        r = o.find_path(proto["vel"], proto["start"])
        o.close()
        for k in keys:
            st[k][i] = np.uint64(r["stats"][k]).astype(np.int64)
        cost[i], ok[i] = r["cost"], r["ok"]
        paths.append(bench.path_digest(r))
    res = bench.parity_all(cfgs, st, cost, ok, paths, [5, 6])
    assert res["bit_exact"] and res["path_poses_checked"] > 0
    st["closed_digest"][1] ^= 1
    r = bench.parity_all(cfgs, st, cost, ok, paths, [5, 6])
    assert r["mismatched_queries"] == [6] and r["n_mismatched"] == 1
    st["closed_digest"][1] ^= 1
    paths[0] = bench.path_digest(dict(path=np.zeros((1, 3), np.float32), curvature=np.zeros(1, np.float32)))
    r = bench.parity_all(cfgs, st, cost, ok, paths, [5, 6])
    assert r["mismatched_queries"] == [5] and r["n_mismatched"] == 1
