"""The backward grid-distance field on the GPU (include/hastar.h: hastar_heuristic_field,
hastar_field_rows, hastar_relaxed_set_field; csrc/hastar_field.hip) against the oracle's float
Dijkstra (orc_heuristic_field, pinned by tests/test_field.py), bit for bit:

  * one GPU, whole grid: synthetic cfg2 / cfg3 maps, 4- and 8-connected moves;
  * the row-sharded protocol with 2, 3 and 5 stand-in ranks on the one GPU
    (shard.py:heuristic_field_standins, the same exchange as heuristic_field_sharded);
  * a field installed as the relaxed mode's heuristic is used as is (no rebuild) and the
    relaxed search on it returns valid paths.
The reference has no such precompute, so this is parity with the field's own definition
("parity unpinned" against the reference; tests/test_field.py).
"""
import math

import numpy as np
import pytest

from tests.scenarios import drive, synthetic_ref
from tests.test_gpu_relaxed import check_valid

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


def _gpu_field(g):
    import torch
    N = g.N
    out = torch.empty(N * N, dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    passes = g.heuristic_field(out.data_ptr())
    return out.cpu().numpy().reshape(N, N), passes


@pytest.mark.parametrize("N,bins,K,seed,diag", [(256, 36, 20, 1, True), (512, 72, 50, 2, True),
                                                (1024, 72, 200, 1, True), (512, 72, 50, 3, False)])
def test_field_matches_oracle(gpu, oracle_lib, N, bins, K, seed, diag):
    cfg, proto = synthetic_ref(N, bins, K, seed)
    if not diag:
        cfg.values["grid_2d_allow_diag_moves"] = 0
    g, o = _pair(gpu, oracle_lib, cfg, proto)
    f, passes = _gpu_field(g)
    ref = o.heuristic_field()
    o.close()
    assert np.isfinite(ref).sum() > N * N // 2
    bad = np.flatnonzero(f.view(np.uint32) != ref.view(np.uint32))
    assert bad.size == 0, f"{bad.size} cells differ, first {np.unravel_index(bad[0], f.shape)}: " \
                          f"{f.flat[bad[0]]} vs {ref.flat[bad[0]]}"
    print(f"N={N} diag={diag}: {passes} passes")
    g.close()


@pytest.mark.parametrize("world", [2, 3, 5])
def test_field_standin_ranks(gpu, oracle_lib, world):
    import torch
    from path_planning_pkg_amd import shard
    cfg, proto = synthetic_ref(512, 72, 50, 4)
    g, o = _pair(gpu, oracle_lib, cfg, proto)
    ref = o.heuristic_field()
    o.close()
    full, rounds, passes = shard.heuristic_field_standins(g, world, torch.device("cuda:0"))
    f = full.cpu().numpy().reshape(g.N, g.N)
    assert np.array_equal(f.view(np.uint32), ref.view(np.uint32))
    assert rounds >= 2
    print(f"{world} stand-in ranks: {rounds} exchange rounds, {passes} passes")
    g.close()


@pytest.mark.parametrize("N,world,diag", [(60, 7, True), (97, 4, False), (128, 3, True)])
def test_field_standins_small_blocks(gpu, oracle_lib, N, world, diag):
    """Grids that are not a multiple of the 32-cell tile, blocks of a few rows (60 rows over 7
    stand-ins: 9-row blocks, the last one 6), the goal row (0.8 N) near a block edge, 4- and
    8-connected: still the oracle's field bit for bit."""
    import torch
    from path_planning_pkg_amd import shard
    from path_planning_pkg_amd.capi import PlannerConfig
    cfg = PlannerConfig(grid_size=N, grid_resolution=0.5, num_angle_bins=36, grid_2d_allow_diag_moves=diag)
    rng = np.random.default_rng(N)
    W = N * 0.5
    boxes = np.stack([rng.uniform(-0.8 * W, 0.2 * W, 40), rng.uniform(-0.5 * W, 0.5 * W, 40),
                      rng.uniform(0.5, 2.5, 40), rng.uniform(0.5, 2.5, 40)], 1).astype(np.float32)
    boxes = boxes[np.hypot(boxes[:, 0], boxes[:, 1]) > 4.0]
    proto = dict(goal=[0.0, 0.0, 0.0], start=[-0.6 * W, 0.0, 0.0], vel=1.0, cycles=3,
                 lines=np.zeros((0, 4), np.float32), line_conf=0.6, line_width=1.0, boxes=boxes, box_conf=0.8,
                 apf_r=1.0)
    g, o = _pair(gpu, oracle_lib, cfg, proto)
    ref = o.heuristic_field()
    o.close()
    one, _ = _gpu_field(g)
    full, rounds, _ = shard.heuristic_field_standins(g, world, torch.device("cuda:0"))
    f = full.cpu().numpy().reshape(N, N)
    assert np.array_equal(one.view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(f.view(np.uint32), ref.view(np.uint32)), f"{world} stand-ins, {rounds} rounds"
    g.close()


def test_field_rows_validation(gpu):
    import torch
    cfg, proto = synthetic_ref(256, 36, 20, 1)
    g = gpu.HybridAStar(cfg)
    buf = torch.empty(258 * 256, dtype=torch.float32, device="cuda:0")
    with pytest.raises(gpu.HastarError):  # before update_goal
        g.field_rows(buf.data_ptr(), 0, 256, 1)
    drive(g, proto)
    for r0, r1 in ((0, 0), (-1, 10), (10, 257), (20, 10)):
        with pytest.raises(gpu.HastarError):
            g.field_rows(buf.data_ptr(), r0, r1, 1)
    with pytest.raises(gpu.HastarError):
        g.field_rows(0, 0, 256, 1)
    g.close()


def test_relaxed_mode_on_an_installed_field(gpu, oracle_lib):
    """The whole field installed as the relaxed heuristic (reuse_heuristic=1, h_coarse=1): the
    relaxed call does not build its own (cycles()[2] == 0) and its paths are valid."""
    import torch
    cases = [synthetic_ref(1024, 72, 200, s) for s in (1, 2)]
    for cfg, proto in cases:
        g, o = _pair(gpu, oracle_lib, cfg, proto)
        N, res = cfg.values["grid_size"], cfg.values["grid_resolution"]
        buf = torch.empty(N * N, dtype=torch.float32, device="cuda:0")
        torch.cuda.synchronize()
        g.heuristic_field(buf.data_ptr())
        g.relaxed_set_field(buf.data_ptr())
        (r,), _ = gpu.find_path_batch([g], [proto["vel"]], [proto["start"]], cap=16384,
                                      relaxed=dict(reuse_heuristic=1, h_coarse=1))
        assert g.cycles()[2] == 0, "the installed field was rebuilt"
        assert r["stats"]["status"] == 0
        ro = o.find_path(proto["vel"], proto["start"])
        o.close()
        if ro["ok"]:
            p = cfg.values["obstacle_threshold"]
            thr = np.float32(math.log(p / (1.0 - p)))
            ex_gap = float(np.hypot(np.diff(ro["path"][:, 0]), np.diff(ro["path"][:, 1])).max())
            max_step = max(1.05 * ex_gap, 3.0 * cfg.values["step_size"]) + 1e-3
            check_valid(r, g.get_obstacles(), thr, proto, N, res, max_step, "installed field")
            assert r["cost"] <= 1.5 * ro["cost"]
        g.close()
