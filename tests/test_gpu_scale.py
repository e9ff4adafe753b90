"""GPU vs oracle at the BASELINE.json configurations' own sizes, and the arena park/resume path.

BASELINE.json configs[2..4]: cfg3 1024x1024x72 with K = 200 boxes, cfg4
2048x2048x72 (plus its row-sharded map build), cfg5 the 1024^2 replan loop without reset.
The cfg3 query ids are bench.py's (seed = id + 1, the std::mt19937 generator
tests/scenarios.py:synthetic_ref); the long ones come from the oracle's pop census
(profiles/census_cfg3_mt19937_r02.csv, tools/pop_census.py): cfg3 query 2395 (172,207 pops).
cfg4 query 1830 (650,107 pops, profiles/census_cfg4_mt19937_r02.csv) outgrows the default
262,144-pop arena and must finish through a park + resume, as the reference (no limit,
HybridAStar.cpp:107) does.

The bar is the one of test_gpu_parity.py: bit-identical pops, successors, A* pops, shots,
ordered pop digest, closed-set digest, path, curvature and cost.
"""
import os

import numpy as np
import pytest

from tests.scenarios import drive, replan_pairs, replan_tick, replan_tick_inputs, synthetic
from tests.test_gpu_parity import assert_bits_equal, compare_results

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    from path_planning_pkg_amd import planner
    planner.load_library()
    return planner


def _pair(gpu, oracle_lib, cfg, proto):
    g, o = gpu.HybridAStar(cfg), oracle_lib.OraclePlanner(cfg)
    drive(g, proto)
    drive(o, proto)
    return g, o


# ----------------------------------------------------------------- park / resume ------
@pytest.mark.parametrize("N,bins,K,seed", [(256, 36, 40, 1), (256, 36, 40, 2), (256, 36, 40, 4), (512, 72, 50, 1)])
def test_park_resume_tiny_arena(gpu, oracle_lib, N, bins, K, seed):
    """An initial arena of 64 pops: the search parks at every 4x boundary (64, 256, 1024,
    ...) and resumes in a larger arena; the result must be the oracle's, bit for bit."""
    cfg, proto = synthetic(N, bins, K, seed)
    cfg.values["max_pops"] = 64
    g, o = _pair(gpu, oracle_lib, cfg, proto)
    rg = g.find_path(proto["vel"], proto["start"])
    ro = o.find_path(proto["vel"], proto["start"])
    compare_results(rg, ro, f"tiny arena N{N} seed{seed}")
    assert rg["stats"]["parks"] >= 1, "the 64-pop arena should have been outgrown"
    fg, vg = g.memo()
    fo, vo = o.get_memo()
    assert_bits_equal(fg, fo, "memo f")
    assert (vg == vo).all()


def test_park_resume_with_fewer_slots(gpu, oracle_lib, monkeypatch):
    """Two slots, seven planners with 64-pop arenas: every wave parks its search and stops
    taking work, the host re-queues the planners no wave took, moves the parked ones into
    larger arenas and resumes them — until all are done.  Every result is the oracle's."""
    monkeypatch.setenv("HASTAR_SLOTS", "2")
    cases = [synthetic(128, 36, 6, s) for s in (31, 32, 33, 34, 35, 36, 37)]
    gs, os_ = [], []
    for cfg, proto in cases:
        cfg.values["max_pops"] = 64
        g, o = _pair(gpu, oracle_lib, cfg, proto)
        gs.append(g)
        os_.append(o)
    res, _ = gpu.find_path_batch(gs, [c[1]["vel"] for c in cases], [c[1]["start"] for c in cases])
    for i, ((cfg, proto), o) in enumerate(zip(cases, os_)):
        compare_results(res[i], o.find_path(proto["vel"], proto["start"]), f"2 slots, planner {i}")
    assert sum(r["stats"]["parks"] for r in res) > 0


@pytest.mark.parametrize("slots", [None, "2"])
def test_resume_arenas_carved_from_the_pool(gpu, oracle_lib, monkeypatch, slots):
    """Resume arenas taken from idle slot arenas of the pool (what happens when a resume
    arena cannot be allocated; HASTAR_RESUME_POOL=1 makes it the first choice).  The parked
    searches must still end with the oracle's results, and the lent pool arenas must come
    back as fresh ones: a second batch on the same pool is checked too.  With 2 slots the
    host also re-queues planners no wave took, beside resume arenas lent from the pool."""
    monkeypatch.setenv("HASTAR_RESUME_POOL", "1")
    if slots:
        monkeypatch.setenv("HASTAR_SLOTS", slots)
    cases = [synthetic(128, 36, 6, s) for s in (41, 42, 43, 44, 45)]
    gs, os_ = [], []
    for cfg, proto in cases:
        cfg.values["max_pops"] = 64
        g, o = _pair(gpu, oracle_lib, cfg, proto)
        gs.append(g)
        os_.append(o)
    before = gpu.HybridAStar.pooled_resumes()
    for rep in range(2):
        for g in gs:
            g.reset()
        for o in os_:
            o.reset()
        res, _ = gpu.find_path_batch(gs, [c[1]["vel"] for c in cases], [c[1]["start"] for c in cases])
        for i, ((cfg, proto), o) in enumerate(zip(cases, os_)):
            compare_results(res[i], o.find_path(proto["vel"], proto["start"]), f"pooled resume, rep {rep}, planner {i}")
        assert sum(r["stats"]["parks"] for r in res) > 0
    assert gpu.HybridAStar.pooled_resumes() > before, "no resume arena was carved from the pool"


def test_statuses_reported_per_planner(gpu, oracle_lib, monkeypatch):
    """One batch, two outcomes: planner 0 exceeds an explicit pop budget
    (HASTAR_MAX_POPS_HARD -> HASTAR_EOVERFLOW, a failed search), planner 1 finishes with a
    path longer than the caller's cap (HASTAR_ENOSPC: its length is reported and the path is
    fetched with hastar_copy_path).  Neither hides the other."""
    monkeypatch.setenv("HASTAR_MAX_POPS_HARD", "400")
    (cfg_a, pa), (cfg_b, pb) = synthetic(256, 36, 40, 1), synthetic(256, 36, 10, 1)  # 2947 and 307 pops
    ga, oa = _pair(gpu, oracle_lib, cfg_a, pa)
    gb, ob = _pair(gpu, oracle_lib, cfg_b, pb)
    br = gpu.find_path_batch_arrays([ga, gb], [pa["vel"], pb["vel"]], [pa["start"], pb["start"]], cap=8)
    assert int(br.stats["status"][0]) == gpu.HASTAR_EOVERFLOW and not br.ok[0]
    assert int(br.stats["pops"][0]) == 400
    assert int(br.stats["status"][1]) == gpu.HASTAR_ENOSPC and br.ok[1] and br.lens[1] > 8
    oracle_lib.set_max_pops(400)
    try:
        ro_a = oa.find_path(pa["vel"], pa["start"])
    finally:
        oracle_lib.set_max_pops(0)
    assert not ro_a["ok"] and ro_a["stats"]["pops"] == 400
    assert br.stats["pop_digest"][0] == ro_a["stats"]["pop_digest"]
    compare_results(br.result(1), ob.find_path(pb["vel"], pb["start"]), "short cap planner")


# ------------------------------------------------------------------ cfg3 (1024^2) ------
# Both search kernels run the same search code: the latency kernel (one search per CU, outer
# open tree and a 2048-node holonomic pool in LDS; batches up to the CU count) and the batch
# kernel (8 searches per CU).  HASTAR_WIDE forces one or the other for the same batch.
KERNELS = [pytest.param("1", id="latency_kernel"), pytest.param("0", id="batch_kernel")]


@pytest.mark.parametrize("wide", KERNELS)
def test_cfg3_parity_batch(gpu, oracle_lib, monkeypatch, wide):
    """BASELINE configs[2]: 1024x1024x72, K = 200, bench query ids 0, 1, 2 and the longest
    query of the bench batch (2395, 172,207 pops: its open set outgrows the latency kernel's
    LDS tree, which moves to HBM mid-search), searched in one batched launch, plus round 1's
    longest PCG64 query (10226, 177,407 pops)."""
    monkeypatch.setenv("HASTAR_WIDE", wide)
    from tests.scenarios import synthetic_ref
    qs = [0, 1, 2, 2395, "pcg64:10226"]
    cases = [synthetic_ref(1024, 72, 200, seed=q + 1) if isinstance(q, int) else
             synthetic(1024, 72, 200, seed=int(q.split(":")[1]) + 1) for q in qs]
    gs, os_ = [], []
    for cfg, proto in cases:
        g, o = _pair(gpu, oracle_lib, cfg, proto)
        gs.append(g)
        os_.append(o)
    res, _ = gpu.find_path_batch(gs, [c[1]["vel"] for c in cases], [c[1]["start"] for c in cases], cap=8192)
    for q, r, o, (cfg, proto), g in zip(qs, res, os_, cases, gs):
        ro = o.find_path(proto["vel"], proto["start"])
        compare_results(r, ro, f"cfg3 query {q}")
        fg, vg = g.memo()
        fo, vo = o.get_memo()
        assert_bits_equal(fg, fo, f"cfg3 query {q} memo f")
        assert (vg == vo).all()
    assert max(r["stats"]["pops"] for r in res) > 100000  # the long query is in the batch


@pytest.mark.parametrize("mode", ["1", "2"])
def test_split_launch_head_and_bulk(gpu, oracle_lib, monkeypatch, mode):
    """A batch split over both kernels at once (HASTAR_SPLIT, as large batches run): the head of
    the queue on the latency CUs, the rest on the batch kernel beside them, one work counter
    (mode 2: the head on single-wave head workgroups of the batch kernel itself).  Every
    planner's result is the oracle's, and both the head and the bulk took work."""
    monkeypatch.setenv("HASTAR_WIDE", "0")
    monkeypatch.setenv("HASTAR_SPLIT", "1")
    monkeypatch.setenv("HASTAR_SPLIT_MODE", mode)
    cases = [synthetic(256, 36, 10 + (s % 4) * 10, s) for s in range(1, 25)] + [synthetic(512, 72, 50, 1)]
    gs, os_ = [], []
    for cfg, proto in cases:
        g, o = _pair(gpu, oracle_lib, cfg, proto)
        gs.append(g)
        os_.append(o)
    res, _ = gpu.find_path_batch(gs, [c[1]["vel"] for c in cases], [c[1]["start"] for c in cases], cap=8192)
    for i, ((cfg, proto), o) in enumerate(zip(cases, os_)):
        compare_results(res[i], o.find_path(proto["vel"], proto["start"]), f"split launch planner {i}")
    slots = {int(g.timing()[2]) for g in gs}
    sl = gs[0].slots()
    head, n_arenas = sl["head_cus"], sl["arenas"]
    on_head = [s < head or s >= n_arenas for s in slots]  # head arenas have slot ids n_arenas + b
    assert any(on_head) and not all(on_head), (slots, head)


def test_split_launch_head_arenas(gpu, oracle_lib, monkeypatch):
    """Head arenas: searches that parked in a split launch (64-pop arenas) make the next split
    launches give the latency CUs arenas sized for them, so the head's searches run through
    without parking.  Every result is the oracle's in all three calls, and after a launch
    without the split (pool arenas back in their plain layout) too."""
    monkeypatch.setenv("HASTAR_WIDE", "0")
    monkeypatch.setenv("HASTAR_SPLIT", "1")
    cases = [synthetic(256, 36, 10 + (s % 4) * 10, s) for s in range(1, 25)] + [synthetic(512, 72, 50, 1)]
    gs, os_ = [], []
    for cfg, proto in cases:
        cfg.values["max_pops"] = 64
        g, o = _pair(gpu, oracle_lib, cfg, proto)
        gs.append(g)
        os_.append(o)
    vels, starts = [c[1]["vel"] for c in cases], [c[1]["start"] for c in cases]
    parks = []
    for rep in range(4):
        if rep == 3:
            monkeypatch.setenv("HASTAR_SPLIT", "0")
        for g, o in zip(gs, os_):
            g.reset()
            o.reset()
        res, _ = gpu.find_path_batch(gs, vels, starts, cap=8192)
        for i, ((cfg, proto), o) in enumerate(zip(cases, os_)):
            compare_results(res[i], o.find_path(proto["vel"], proto["start"]), f"head arenas, call {rep}, planner {i}")
        ha = gs[0].head_arenas()
        head_parks = [r["stats"]["parks"] for g, r in zip(gs, res) if int(g.timing()[2]) >= gs[0].slots()["arenas"]]
        parks.append((sum(r["stats"]["parks"] for r in res), ha, head_parks))
    assert parks[0][0] > 0 and parks[0][1]["n"] == 0, parks       # first call: plain arenas, searches park
    assert parks[1][1]["n"] > 0 and parks[1][1]["grant"] > 64, parks  # then head arenas, sized for them
    assert parks[1][2] and not any(parks[1][2]), parks                # the head's searches did not park
    assert parks[3][1]["n"] == 0, parks                               # released by the unsplit launch


@pytest.mark.parametrize("max_pops", [0, 256])
def test_split_launch_handoff(gpu, oracle_lib, monkeypatch, max_pops):
    """Handoff (HandoffBoard): with HASTAR_HANDOFF_POPS=64 every batch-kernel
    search past 64 pops is offered to the latency CUs, which claim offers as they come free; the
    claimed searches park at their next 64-pop check, are copied into the latency wave's arena and
    continue there in resume mode.  Every result is the oracle's, bit for bit, searches were
    handed over, and a second call on the same pool (planners with history: HASTAR_HANDOFF_WARM
    keeps handoffs on) agrees too.  max_pops = 256: capacity parks (and their host resumes) on
    top of the handoffs (offers at 64, 128 and 192 pops come before the first park)."""
    monkeypatch.setenv("HASTAR_WIDE", "0")
    monkeypatch.setenv("HASTAR_SPLIT", "1")
    monkeypatch.setenv("HASTAR_HANDOFF_POPS", "64")
    monkeypatch.setenv("HASTAR_HANDOFF_WARM", "1")  # the second call has history: handoffs stay on
    cases = [synthetic(256, 36, 10 + (s % 4) * 10, s) for s in range(1, 49)] + [synthetic(512, 72, 50, 1)]
    gs, os_ = [], []
    for cfg, proto in cases:
        if max_pops:
            cfg.values["max_pops"] = max_pops
        g, o = _pair(gpu, oracle_lib, cfg, proto)
        gs.append(g)
        os_.append(o)
    vels, starts = [c[1]["vel"] for c in cases], [c[1]["start"] for c in cases]
    handed = []
    for rep in range(2):
        for g, o in zip(gs, os_):
            g.reset()
            o.reset()
        res, _ = gpu.find_path_batch(gs, vels, starts, cap=8192)
        for i, ((cfg, proto), o) in enumerate(zip(cases, os_)):
            compare_results(res[i], o.find_path(proto["vel"], proto["start"]), f"handoff, call {rep}, planner {i}")
        handed.append(gs[0].handoffs())
    assert max(handed) > 0, handed


@pytest.mark.parametrize("wide", KERNELS)
def test_cfg3_survey_reference_cases(gpu, oracle_lib, monkeypatch, wide):
    """The survey's own cases, 256² to 2048² including cfg3 seeds 1 and 3 (std::mt19937 inputs,
    tests/scenarios.py:synthetic_ref): GPU == oracle bit for bit, and both equal the counts the
    survey measured on the compiled reference (tests/golden/survey_reference_counts.json)."""
    monkeypatch.setenv("HASTAR_WIDE", wide)
    import json
    from tests.scenarios import GOLDEN, synthetic_ref
    g = json.loads((GOLDEN / "survey_reference_counts.json").read_text())
    cases = [synthetic_ref(c["grid"], c["angle_bins"], c["obstacles"], c["seed"]) for c in g["cases"]]
    gs, os_ = [], []
    for cfg, proto in cases:
        gp, op = _pair(gpu, oracle_lib, cfg, proto)
        gs.append(gp)
        os_.append(op)
    res, _ = gpu.find_path_batch(gs, [c[1]["vel"] for c in cases], [c[1]["start"] for c in cases], cap=8192)
    for ref, r, o, (cfg, proto) in zip(g["cases"], res, os_, cases):
        compare_results(r, o.find_path(proto["vel"], proto["start"]), f"survey case {ref}")
        for k in ("pops", "successors", "astar_pops"):
            if k in ref:
                assert r["stats"][k] == ref[k], f"{ref}: {k} {r['stats'][k]} vs reference {ref[k]}"


# ------------------------------------------------------------------ cfg4 (2048^2) ------
@pytest.mark.parametrize("q", [0, 3, 1830])
def test_cfg4_parity(gpu, oracle_lib, q):
    """BASELINE configs[3] at its own size: 2048x2048x72, K = 200, bench query ids (std::mt19937
    inputs).  Query 1830 is the longest of the bench batch (650,107 pops,
    profiles/census_cfg4_mt19937_r02.csv): it parks at the default arena's 262,144 and resumes,
    and must end with the oracle's success, cost and path (round 1 cut such queries off)."""
    from tests.scenarios import synthetic_ref
    cfg, proto = synthetic_ref(2048, 72, 200, seed=q + 1)
    g, o = _pair(gpu, oracle_lib, cfg, proto)
    assert_bits_equal(g.get_obstacles(), o.get_obstacles(), f"cfg4 query {q} map")
    rg = g.find_path(proto["vel"], proto["start"], cap=16384)
    ro = o.find_path(proto["vel"], proto["start"])
    compare_results(rg, ro, f"cfg4 query {q}")
    if ro["stats"]["pops"] > 262144:
        assert rg["stats"]["parks"] >= 1


def test_cfg4_row_sharded_map_build(gpu, oracle_lib):
    """cfg4's sharded map build at its own size: 2048^2 over 4 stand-in ranks."""
    from tests import test_gpu_parity as tp  # (a module import: pytest must not collect it here)
    tp.test_row_sharded_map_build(gpu, oracle_lib, 2048, 4)


# ------------------------------------------------------------------ cfg5 (replans) -----
def test_cfg5_replan_loop_parity(gpu, oracle_lib):
    """BASELINE configs[4] at its own size: 1024x1024x72 maps, K = 200 moving boxes, ALL 64 bench
    pairs (ids 0..63, bench.py run_cfg5), 4 batched ticks WITHOUT reset (local_planner.cpp:
    204-205, 241, 316): memo and stale node-map values carry over between ticks.  The oracle's
    replays run on host threads (each pair's calls stay in order)."""
    from concurrent.futures import ThreadPoolExecutor
    pairs = []
    for q in range(64):
        pairs += replan_pairs(1024, 72, 200, 1, seed=1000 + q)
    gs, os_ = [], []
    for cfg, proto, _ in pairs:
        g, o = _pair(gpu, oracle_lib, cfg, proto)
        gs.append(g)
        os_.append(o)
    bufs = gpu.BatchBuffers(gs, cap=8192)
    for tick in range(4):
        starts = [replan_tick_inputs(proto, v, tick)[0] for _, proto, v in pairs]
        br = gpu.find_path_batch_arrays(gs, [proto["vel"] for _, proto, _ in pairs], starts, buffers=bufs)

        def oracle_tick(i):
            _, proto, v = pairs[i]
            r = os_[i].find_path(proto["vel"], starts[i])
            replan_tick(os_[i], proto, v, tick)
            return r
        with ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
            ores = list(ex.map(oracle_tick, range(len(pairs))))
        for i, (_, proto, v) in enumerate(pairs):
            compare_results(br.result(i), ores[i], f"cfg5 tick {tick} pair {i}")
            replan_tick(gs[i], proto, v, tick)


# ------------------------------------------------- device-resident velocity profile ----
def test_velocity_profile_of_last_batch(gpu, oracle_lib):
    """hastar_velocity_profile_last_batch profiles the batch's paths where they are (HBM);
    it must equal the host-buffer entry point and the oracle, bit for bit."""
    cases = [synthetic(256, 36, 10, s) for s in (1, 2, 3, 4, 5)]
    gs = []
    for cfg, proto in cases:
        g = gpu.HybridAStar(cfg)
        drive(g, proto)
        gs.append(g)
    br = gpu.find_path_batch_arrays(gs, [c[1]["vel"] for c in cases], [c[1]["start"] for c in cases], cap=4096)
    lens = br.lens.astype(np.int64).copy()
    prm = (10.0, 3.0, 2.5, 1.5, 3.0)
    vg = gpu.VelocityGenerator(*prm)
    v0 = np.full(len(gs), 2.0, np.float32)
    vm = np.full(len(gs), 10.0, np.float32)
    flags = np.array([2, 0, 1, 3, 2], np.uint8)
    feas, vel = vg.profile_last_batch(lens, v0, vm, flags)
    off = np.zeros(len(gs) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    for i in range(len(gs)):
        a, b = off[i], off[i + 1]
        ok_o, vo = oracle_lib.velocity_profile(prm, 2.0, 10.0, br.xyh[i, :lens[i]], br.curv[i, :lens[i]],
                                               bool(flags[i] & 1), bool(flags[i] & 2))
        assert bool(feas[i]) == ok_o
        assert_bits_equal(vel[a:b], vo, f"velocity of path {i}")


def test_velocity_last_batch_after_all_failed(gpu):
    """A batch whose searches all fail returns no path: profiling it must report every planner
    infeasible and must not read the previous batch's path offsets."""
    cases = [synthetic(256, 36, 10, s) for s in (1, 2)]
    gs = []
    for cfg, proto in cases:
        g = gpu.HybridAStar(cfg)
        drive(g, proto)
        gs.append(g)
    br = gpu.find_path_batch_arrays(gs, [2.0, 2.0], [c[1]["start"] for c in cases], cap=4096)
    assert br.ok.all() and (br.lens > 0).all()  # a previous batch with paths packed in HBM
    blocked = []
    for _ in range(3):  # goal cell walled in (test_edge_cases): every search fails
        cfg, proto = synthetic(48, 36, 0, 1)
        proto["boxes"] = np.array([[0.0, 0.0, 4.0, 4.0]], np.float32)
        proto["start"] = [-14.0, 0.0, 0.0]
        g = gpu.HybridAStar(cfg)
        drive(g, proto)
        blocked.append(g)
    bb = gpu.find_path_batch_arrays(blocked, [2.0] * 3, [[-14.0, 0.0, 0.0]] * 3, cap=4096)
    assert not bb.ok.any() and (bb.lens == 0).all()
    vg = gpu.VelocityGenerator(10.0, 3.0, 2.5, 1.5, 3.0)
    feas, vel = vg.profile_last_batch(bb.lens.astype(np.int64), np.full(3, 2.0, np.float32),
                                      np.full(3, 10.0, np.float32), np.full(3, 2, np.uint8))
    assert (feas == 0).all() and len(vel) == 0


def test_velocity_last_batch_with_short_caller_buffer(gpu, oracle_lib):
    """A planner whose path exceeds the caller's `cap` (ENOSPC, fetched with copy_path) is still
    packed on the device at its full length, so the device-resident velocities of the planners
    after it line up with the returned lengths."""
    from tests.scenarios import harness
    cases = [synthetic(256, 36, 10, 1), harness()[:2], harness()[:2]]  # paths of 103, 43 and 43 poses
    gs = []
    for cfg, proto in cases:
        g = gpu.HybridAStar(cfg)
        drive(g, proto)
        gs.append(g)
    vels, starts = [c[1]["vel"] for c in cases], [c[1]["start"] for c in cases]
    full = gpu.find_path_batch(gs, vels, starts, cap=4096)[0]
    lens = np.array([len(r["path"]) for r in full], np.int64)
    cap = int(lens[0]) - 1  # planner 0's path does not fit; the others do
    assert (lens[1:] <= cap).all(), lens
    res, _ = gpu.find_path_batch(gs, vels, starts, cap=cap)
    # (find_path_batch fetched the long path with copy_path and cleared its ENOSPC status)
    assert res[0]["stats"]["status"] == 0 and len(res[0]["path"]) == lens[0]
    prm = (10.0, 3.0, 2.5, 1.5, 3.0)
    v0 = np.asarray(vels, np.float32)
    feas, vel = gpu.VelocityGenerator(*prm).profile_last_batch(lens, v0, np.full(3, 10.0, np.float32),
                                                              np.full(3, 2, np.uint8))
    off = np.concatenate([[0], np.cumsum(lens)])
    for i in range(3):
        ok_o, vo = oracle_lib.velocity_profile(prm, float(v0[i]), 10.0, res[i]["path"], res[i]["curvature"], False,
                                               True)
        assert bool(feas[i]) == ok_o
        assert_bits_equal(vel[off[i]:off[i + 1]], vo, f"velocity of path {i}")


# ---------------------------------------------------------- map relocation ------------
@pytest.mark.parametrize("N", [61, 1024, 2048, 4095])
def test_relocation_of_random_maps(gpu, oracle_lib, N):
    """Grid3D::relocate_obstacles (Grid3D.cpp:169-203) on maps of distinct random values, so every
    destination's winning source (the largest row-major source index that rounds there) is
    visible: single update_goal calls and batched ones (one planner named twice: relocated twice,
    in order) at headings and offsets that rotate by up to 180 degrees and move the goal by up to a
    third of the grid, against the oracle's own loop.  The GPU inverts the rotation per
    destination cell (k_relocate_invert_batch); N = 61 and 4095 are not multiples of the kernel's
    tile, N = 4095 also puts a 4-byte cell index near 2^24 where float rounding of i * N + j
    would go wrong."""
    import torch
    from path_planning_pkg_amd.capi import PlannerConfig
    rng = np.random.default_rng(N)
    cfg = PlannerConfig(grid_size=N, num_angle_bins=36)
    span = N * float(cfg.values["grid_resolution"]) / 3.0
    nb = 1 if N >= 2048 else 3
    gs = [gpu.HybridAStar(cfg) for _ in range(nb)]
    os_ = [oracle_lib.OraclePlanner(cfg) for _ in range(nb)]
    for g, o in zip(gs, os_):
        m = rng.uniform(-5.0, 5.0, (N, N)).astype(np.float32)
        t = torch.from_numpy(m).to("cuda:0")
        g.import_rows(0, N, t.data_ptr())
        o.set_obstacles(m)
        assert_bits_equal(g.get_obstacles(), o.get_obstacles(), "map set")

    def draw(k):
        goals = np.concatenate([rng.uniform(-span, span, (k, 2)), rng.uniform(-3.1, 3.1, (k, 1))], 1).astype(np.float32)
        starts = np.concatenate([rng.uniform(-span, span, (k, 2)), np.zeros((k, 1))], 1).astype(np.float32)
        return goals, starts
    for step in range(3):  # single calls
        goals, starts = draw(nb)
        for g, o, g0, s0 in zip(gs, os_, goals, starts):
            g.update_goal(g0, s0)
            o.update_goal(g0, s0)
            assert_bits_equal(g.get_obstacles(), o.get_obstacles(), f"N={N} single relocation {step}")
    for step in range(2):  # batched: planner 0 twice
        idx = [0] + list(range(nb)) if nb > 1 else [0, 0]
        goals, starts = draw(len(idx))
        gpu.update_goal_batch([gs[i] for i in idx], goals, starts)
        for i, g0, s0 in zip(idx, goals, starts):
            os_[i].update_goal(g0, s0)
        for i in range(nb):
            assert_bits_equal(gs[i].get_obstacles(), os_[i].get_obstacles(), f"N={N} batched relocation {step} map {i}")


# ---------------------------------------------------------- batched map updates --------
def test_batched_map_updates_equal_single_calls(gpu, oracle_lib):
    """hastar_update_goal_batch / hastar_decay_batch / hastar_update_boxes_batch over planners
    of different grid sizes, goal frames, row windows and overlapping boxes with per-box
    confidences: every map and APF list equals the oracle's per-instance updates (Grid2D.cpp:
    99-208, Grid3D.cpp:22-44, 102-203), and a search on a batch-built map equals the oracle's."""
    from path_planning_pkg_amd.capi import PlannerConfig
    rng = np.random.default_rng(23)
    sizes = [128, 200, 256, 97, 256, 180]
    cfgs = [PlannerConfig(grid_size=N, num_angle_bins=36) for N in sizes]
    gs = [gpu.HybridAStar(c) for c in cfgs]
    os_ = [oracle_lib.OraclePlanner(c) for c in cfgs]
    goals = rng.uniform(-5, 5, (len(gs), 3)).astype(np.float32)
    starts = np.concatenate([rng.uniform(-40, -20, (len(gs), 2)), np.zeros((len(gs), 1))], 1).astype(np.float32)
    gs[4].set_row_window(37, 201)  # a row window applies to decay and boxes alike
    gpu.update_goal_batch(gs, goals, starts)
    for o, g0, s0 in zip(os_, goals, starts):
        o.update_goal(g0, s0)
    for cyc in range(4):
        bl, cl = [], []
        for i in range(len(gs)):
            k = int(rng.integers(0, 90))
            b = np.stack([rng.uniform(-40, 10, k), rng.uniform(-30, 20, k), rng.uniform(0.5, 9, k),
                          rng.uniform(0.5, 9, k)], 1).astype(np.float32)
            bl.append(b)
            cl.append(rng.uniform(0.05, 0.97, k).astype(np.float32))
        gpu.decay_batch(gs)
        gpu.update_boxes_batch(gs, bl, cl, 1.5)
        for o, b, c in zip(os_, bl, cl):
            o.decay()
            o.update_boxes(b, c, 1.5)
        for i, (g, o) in enumerate(zip(gs, os_)):
            m, ref = g.get_obstacles(), o.get_obstacles()
            if i == 4:
                assert_bits_equal(m[37:201], ref[37:201], f"windowed map {i} cycle {cyc}")
            else:
                assert_bits_equal(m, ref, f"map {i} cycle {cyc}")
            assert_bits_equal(g.apf(), o.apf(), f"APF list {i} cycle {cyc}")
    # a second goal change relocates every map in one batched call
    goals2 = rng.uniform(-5, 5, (len(gs), 3)).astype(np.float32)
    gpu.update_goal_batch(gs, goals2, starts)
    for i, (o, g0, s0) in enumerate(zip(os_, goals2, starts)):
        o.update_goal(g0, s0)
        if i != 4:
            assert_bits_equal(gs[i].get_obstacles(), o.get_obstacles(), f"relocated map {i}")
    # the synthetic workload built with drive_batch searches like the oracle
    from tests.scenarios import drive_batch
    cases = [synthetic(256, 36, 40, s) for s in (1, 2, 4)]
    gb = [gpu.HybridAStar(c) for c, _ in cases]
    drive_batch(gpu, gb, [p for _, p in cases])
    for g, (cfg, proto) in zip(gb, cases):
        o = oracle_lib.OraclePlanner(cfg)
        drive(o, proto)
        assert_bits_equal(g.get_obstacles(), o.get_obstacles(), "drive_batch map")
        compare_results(g.find_path(proto["vel"], proto["start"]), o.find_path(proto["vel"], proto["start"]),
                        "search on a drive_batch map")


def test_batch_created_planners_equal_single(gpu, oracle_lib):
    """hastar_create_batch_f32: planners sharing one allocation and one copy of the motion
    tables plan exactly like the oracle (and so like singly created ones), and destroying
    some of them leaves the others intact."""
    from tests.scenarios import drive_batch
    cases = [synthetic(256, 36, 40, s) for s in (1, 2, 4, 5)]
    gs = gpu.HybridAStar.create_batch(cases[0][0], len(cases))
    drive_batch(gpu, gs, [p for _, p in cases])
    gs[1].close()
    for i in (0, 2, 3):
        cfg, proto = cases[i]
        o = oracle_lib.OraclePlanner(cfg)
        drive(o, proto)
        assert_bits_equal(gs[i].get_obstacles(), o.get_obstacles(), f"batch-created map {i}")
        compare_results(gs[i].find_path(proto["vel"], proto["start"]), o.find_path(proto["vel"], proto["start"]),
                        f"batch-created planner {i}")
