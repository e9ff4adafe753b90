"""The backward grid-distance field (include/hastar.h: hastar_heuristic_field / hastar_field_rows;
csrc/hastar_field.hip) on the host: its checker and its row-sharded exchange protocol.

The reference has no such precompute (its holonomic heuristic is lazy, AStar.cpp:100-186), so
nothing in it pins the field ("parity unpinned" against the reference).  What pins the checker
(oracle/hastar_oracle.cpp: orc_heuristic_field, a float Dijkstra) is the field's definition:
field(goal) = 0 and field(v) = min over expandable neighbours u of fl(field(u) + move cost),
checked here cell by cell, and a from-scratch Jacobi relaxation in numpy reaching the same bits.
The sharded protocol (shard.py:heuristic_field_sharded) runs over two gloo ranks with that
numpy relaxation standing in for the GPU kernel (test infrastructure only), and must give the
checker's field bit for bit.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
MOVES = [(1, 0), (0, 1), (-1, 0), (0, -1), (-1, -1), (1, 1), (-1, 1), (1, -1)]


def field_params(cfg):
    """thr and the move costs as the planner computes them (float32, Grid2D.cpp:22-40)."""
    v = cfg.values
    p = np.float64(np.float32(v["obstacle_threshold"]))
    thr = np.float32(np.log(p / (1.0 - p)))
    res = np.float32(v["grid_resolution"])
    return thr, res, np.float32(res * np.sqrt(np.float32(2.0))), bool(v["grid_2d_allow_diag_moves"])


def expandable(occ, thr, goal):
    ex = occ < thr
    ex[goal] = True
    return ex


def relax_block(d, ex, wa, wd, diag):
    """Jacobi relaxation of d (rows 1 .. R of a (R + 2) x N array; rows 0 and R + 1 are fixed
    halos) to its fixed point, float32 throughout.  Returns the number of sweeps."""
    R = d.shape[0] - 2
    inf = np.float32(np.inf)
    sweeps = 0
    while True:
        sweeps += 1
        best = d[1:R + 1].copy()
        for k, (di, dj) in enumerate(MOVES[:8 if diag else 4]):
            w = wa if k < 4 else wd
            # neighbour u = v + (di, dj): shift the padded array
            src = np.full_like(d, inf)
            e = np.zeros_like(ex)
            rs = slice(max(0, di), d.shape[0] + min(0, di))
            rd = slice(max(0, -di), d.shape[0] + min(0, -di))
            cs = slice(max(0, dj), d.shape[1] + min(0, dj))
            cd = slice(max(0, -dj), d.shape[1] + min(0, -dj))
            src[rd, cd] = d[rs, cs]
            e[rd, cd] = ex[rs, cs]
            cand = np.where(e[1:R + 1], src[1:R + 1] + np.float32(w), inf).astype(np.float32)
            best = np.minimum(best, cand)
        if np.array_equal(best, d[1:R + 1]):
            return sweeps
        d[1:R + 1] = best


def numpy_field(occ, thr, goal, wa, wd, diag):
    N = occ.shape[0]
    d = np.full((N + 2, N), np.inf, np.float32)
    d[goal[0] + 1, goal[1]] = 0.0
    ex = np.zeros((N + 2, N), bool)
    ex[1:N + 1] = expandable(occ, thr, goal)
    relax_block(d, ex, wa, wd, diag)
    return d[1:N + 1]


def _random_oracle_case(seed, N=48, diag=True):
    from oracle.pyoracle import OraclePlanner
    from tests.scenarios import drive
    from path_planning_pkg_amd.capi import PlannerConfig
    rng = np.random.default_rng(seed)
    cfg = PlannerConfig(grid_size=N, grid_resolution=0.5, num_angle_bins=36, grid_2d_allow_diag_moves=diag)
    W = N * 0.5
    boxes = np.stack([rng.uniform(-0.8 * W, 0.2 * W, 30), rng.uniform(-0.5 * W, 0.5 * W, 30),
                      rng.uniform(0.5, 3.0, 30), rng.uniform(0.5, 3.0, 30)], 1).astype(np.float32)
    boxes = boxes[np.hypot(boxes[:, 0], boxes[:, 1]) > 5.0]  # keep the goal free
    proto = dict(goal=[0.0, 0.0, 0.0], start=[-0.6 * W, 0.0, 0.0], vel=1.0, cycles=3,
                 lines=np.zeros((0, 4), np.float32), line_conf=0.6, line_width=1.0, boxes=boxes, box_conf=0.8,
                 apf_r=1.0)
    o = OraclePlanner(cfg)
    drive(o, proto)
    return cfg, o


@pytest.mark.parametrize("seed,diag", [(1, True), (2, True), (3, False)])
def test_oracle_field_is_the_fixed_point(oracle_lib, seed, diag):
    cfg, o = _random_oracle_case(seed, diag=diag)
    N = cfg.values["grid_size"]
    occ, f = o.get_obstacles(), o.heuristic_field()
    o.close()
    thr, wa, wd, dg = field_params(cfg)
    goal = (int(round(N * 0.8)), int(round(N * 0.5)))
    assert f[goal] == 0.0
    ex = expandable(occ, thr, goal)
    assert (occ >= thr).sum() > 0, "the case needs obstacles"
    # the equations, cell by cell
    for i in range(N):
        for j in range(N):
            if (i, j) == goal:
                continue
            best = np.float32(np.inf)
            for k, (di, dj) in enumerate(MOVES[:8 if dg else 4]):
                u = (i + di, j + dj)
                if 0 <= u[0] < N and 0 <= u[1] < N and ex[u]:
                    best = min(best, np.float32(f[u] + (wa if k < 4 else wd)))
            assert f[i, j] == best, (i, j, f[i, j], best)
    # an independent relaxation order reaches the same bits
    assert np.array_equal(numpy_field(occ, thr, goal, wa, wd, dg), f)
    assert np.isfinite(f).sum() > N * N // 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _MapOnly:
    def __init__(self, N):
        self.N = N


def _numpy_relax(occ, thr, goal, wa, wd, diag):
    """shard.heuristic_field_sharded's `relax` callback with numpy in place of the GPU kernel."""
    N = occ.shape[0]

    def relax(buf, r0, r1, init, halo_changed):
        R = r1 - r0
        d = buf[:(R + 2) * N].numpy().reshape(R + 2, N)
        if init:
            d[:] = np.inf
            if r0 <= goal[0] < r1:
                d[goal[0] - r0 + 1, goal[1]] = 0.0
        ex = np.zeros((R + 2, N), bool)
        lo = r0 - 1
        full = expandable(occ, thr, goal)
        for lr in range(R + 2):
            g = lo + lr
            if 0 <= g < N:
                ex[lr] = full[g]
        before = d.copy()
        sweeps = relax_block(d, ex, wa, wd, diag)
        mask = 0
        if not np.array_equal(before, d):
            mask |= 1
        if not np.array_equal(before[1], d[1]):
            mask |= 2
        if not np.array_equal(before[R], d[R]):
            mask |= 4
        return mask, sweeps
    return relax


def _field_rank_main(rank, world, port, q, occ, thr, goal, wa, wd, diag):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from path_planning_pkg_amd import shard
    full, rounds, _ = shard.heuristic_field_sharded(_MapOnly(occ.shape[0]), rank, world, "cpu",
                                                     relax=_numpy_relax(occ, thr, goal, wa, wd, diag))
    q.put((rank, full.numpy().copy(), rounds))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_field_protocol_gloo(oracle_lib, world):
    import torch.multiprocessing as mp
    cfg, o = _random_oracle_case(4)
    N = cfg.values["grid_size"]
    occ, ref = o.get_obstacles(), o.heuristic_field()
    o.close()
    thr, wa, wd, dg = field_params(cfg)
    goal = (int(round(N * 0.8)), int(round(N * 0.5)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_field_rank_main, args=(r, world, port, q, occ, thr, goal, wa, wd, dg))
             for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=150) for _ in range(world)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert np.isfinite(ref).sum() > N * N // 2
    for rank, full, rounds in out:
        assert np.array_equal(full.reshape(N, N), ref), rank
        assert rounds >= 2  # the goal's block reached the others through the exchange


def test_halo_updates_follow_the_edge_masks():
    import torch
    from path_planning_pkg_amd import shard
    N = 4
    blocks, _ = shard.row_blocks(10, 3)
    e = torch.zeros(3, 2 * N + 1)
    e[0, N:2 * N] = 7.0
    e[0, 2 * N] = 4   # rank 0's last row changed
    e[2, :N] = 9.0
    e[2, 2 * N] = 2   # rank 2's first row changed
    up, dn, bits = shard._halo_updates(e, 1, blocks, N)
    assert bits == 3 and float(up[0]) == 7.0 and float(dn[0]) == 9.0
    e[0, 2 * N] = 1   # an interior change only
    up, dn, bits = shard._halo_updates(e, 1, blocks, N)
    assert up is None and bits == 2
