"""bench.py — Hybrid A* node expansions/sec on the 1024x1024x72 grid (BASELINE.json configs[2]).

Workload (one "step"): a batch of B independent planners (SURVEY.md §8d synthetic
generator: N = 1024, 72 angle bins, K = 200 box obstacles, seed = query id; the reference's
only motion mode: forward Dubins), each already set up in HBM (update_goal, 5 x {decay,
boxes}); the step resets the holonomic memo of every planner (HybridAStar::reset) and runs
ONE batched find_path launch — one wavefront per planner.
value = total pops of all planners on all ranks / wall time of the K timed steps (max over
ranks).  One rank per GPU (torch.distributed over RCCL for the barrier/reductions only):
planners are sharded across ranks with no data-path collective -> weak scaling.

Extra fields: plan latency of a single query (median of single-planner searches),
roofline of the search kernel (algorithmic bytes of SURVEY.md §8d per launch / kernel time
from HIP events on the launch stream), and the CPU oracle timed on the host (rank 0).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algorithmic_bytes(st, K):
    """B = 40 P + 44 S + 208 A + 12 K per plan, summed over the batch
    (st: the stats structured array of one batched call)."""
    return float(40 * st["pops"].astype(np.float64).sum() + 44 * st["successors"].astype(np.float64).sum()
                 + 208 * st["astar_pops"].astype(np.float64).sum() + 12.0 * K * len(st))


def shard_query_ids(rank, world, batch):
    """Queries of one rank: weak scaling, B per GPU, disjoint across ranks, no exchange."""
    assert 0 <= rank < world
    return [rank * batch + i for i in range(batch)]


def reduce_over_ranks(dist, elapsed, pops, device):
    """(max elapsed, total pops) over ranks; identity without a process group."""
    if dist is None:
        return elapsed, float(pops)
    import torch
    t = torch.tensor([elapsed, float(pops)], dtype=torch.float64, device=device)
    tmax, tsum = t[:1].clone(), t[1:].clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
    return float(tmax[0]), float(tsum[0])


def build_planners(gpu, cfgs, device):
    from tests.scenarios import drive
    planners = []
    for cfg, proto in cfgs:
        p = gpu.HybridAStar(cfg, device=device)
        drive(p, proto)
        planners.append(p)
    return planners


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("HASTAR_BENCH_BATCH", "23552")),
                    help="planners (queries) per GPU")
    ap.add_argument("--grid", type=int, default=None, help="default 1024 (cfg3, cfg5) or 2048 (cfg4)")
    ap.add_argument("--bins", type=int, default=72)
    ap.add_argument("--obstacles", type=int, default=200)
    ap.add_argument("--max-pops", type=int, default=0, help="0 = library default (262144)")
    ap.add_argument("--max-astar-nodes", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU-oracle baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--latency-queries", type=int, default=3)
    ap.add_argument("--workload", choices=("cfg3", "cfg4", "cfg5"), default="cfg3",
                    help="cfg3: batch of independent queries (default, the headline line); "
                         "cfg4: 2048^2 queries with the map build row-sharded over the ranks + RCCL all-gather "
                         "(BASELINE.json configs[3]); cfg5: 20 Hz replan loop of start/goal pairs (configs[4])")
    ap.add_argument("--map-queries", type=int, default=16, help="cfg4: maps built both locally and row-sharded")
    ap.add_argument("--pairs", type=int, default=64, help="cfg5: start/goal pairs per GPU")
    args = ap.parse_args()
    if args.grid is None:
        args.grid = 2048 if args.workload == "cfg4" else 1024
    if args.workload == "cfg4" and "--batch" not in sys.argv and "HASTAR_BENCH_BATCH" not in os.environ:
        args.batch = 6144  # 2048^2 maps: 32 MiB per planner; the arena pool takes the rest of the HBM

    # search arenas may take 95% of the HBM left after the planners' maps (library default 80%)
    os.environ.setdefault("HASTAR_ARENA_FRAC", "0.95")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist_mod
        dist = dist_mod
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")
    device = local_rank

    from path_planning_pkg_amd import planner as gpu
    from path_planning_pkg_amd.capi import PlannerConfig
    from tests.scenarios import synthetic

    if args.workload == "cfg5":
        return run_cfg5(args, gpu, dist, torch, rank, world, device)
    B = args.batch
    map_build = map_build_phase(args, gpu, dist, torch, rank, world, device) if args.workload == "cfg4" else None

    def cfg_for(q):
        cfg, proto = synthetic(args.grid, args.bins, args.obstacles, seed=q + 1)
        cfg.values["max_pops"] = args.max_pops
        cfg.values["max_astar_nodes"] = args.max_astar_nodes
        return cfg, proto

    qids = shard_query_ids(rank, world, B)
    cfgs = [cfg_for(q) for q in qids]
    t_setup = time.perf_counter()
    planners = build_planners(gpu, cfgs, device)
    t_setup = time.perf_counter() - t_setup
    vels = [c[1]["vel"] for c in cfgs]
    starts = [c[1]["start"] for c in cfgs]

    # host-side batch arguments and output arrays are allocated once and reused every step
    bufs = gpu.BatchBuffers(planners, cap=8192)

    def step():
        gpu.reset_batch(bufs)  # HybridAStar::reset() of every planner
        br = gpu.find_path_batch_arrays(planners, vels, starts, buffers=bufs)
        return br, br.kernel_ms

    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    pops = 0
    kernel_ms = []
    alg_bytes = []
    statuses = set()
    oks = 0
    last = None
    for _ in range(args.steps):
        res, kms = step()
        kernel_ms.append(kms)
        st = res.stats
        pops += int(st["pops"].sum())
        alg_bytes.append(algorithmic_bytes(st, args.obstacles))
        statuses |= set(int(v) for v in np.unique(st["status"]))
        oks += int(res.ok.sum())
        last = res
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    elapsed, pops_all = reduce_over_ranks(dist, elapsed, pops, f"cuda:{device}")

    out = None
    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = pops_all / elapsed
        avg_kernel_ms = float(np.mean(kernel_ms))
        achieved = float(np.mean(alg_bytes)) / (avg_kernel_ms * 1e-3) / 1e9
        # single-query plan latency (the second half of the metric)
        lat = []
        for p, c in list(zip(planners, cfgs))[: args.latency_queries]:
            p.reset()
            r, kms = gpu.find_path_batch([p], [c[1]["vel"]], [c[1]["start"]], cap=8192)
            lat.append(kms)
        vel_prof = velocity_profile_phase(gpu, last, device, [c[1]["vel"] for c in cfgs])
        traffic = None
        pmc = ROOT / "profiles" / "pmc_search_summary.json"
        if pmc.exists():
            try:
                pm = json.loads(pmc.read_text())
                if pm.get("batch") == B and pm.get("grid") == args.grid:
                    traffic = pm.get("hbm_bytes_per_launch")
            except (ValueError, OSError):
                traffic = None
        out = {
            "metric": "Hybrid A* node expansions/sec + plan latency, 1024x1024x72 grid",
            "value": value,
            "unit": "expansions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (SURVEY.md §8d generator; seeds = query ids)",
            "config": {"workload": f"{args.workload}: {args.grid}x{args.grid}x{args.bins} grid, {args.obstacles} box "
                                   f"obstacles, batch of {B} independent queries per GPU, forward Dubins"
                                   + (", map build row-sharded over the ranks + RCCL all-gather (map_build)"
                                      if map_build else ""),
                       "grid": args.grid, "angle_bins": args.bins, "obstacles": args.obstacles,
                       "queries_per_gpu": B, "global_batch": B * world, "parallelism": f"query-sharded x{world}"},
            "plan_latency_ms": float(np.median(lat)) if lat else None,
            "pops_per_step": pops_all / args.steps,
            "success_rate": oks / (B * args.steps),
            "search_status": sorted(statuses),
            "setup_s_per_gpu": t_setup,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                         "kernel": "hastar_search_kernel", "kernel_ms": avg_kernel_ms,
                         "alg_bytes_per_launch": float(np.mean(alg_bytes))},
        }
        if map_build:
            out["map_build"] = map_build
        out["velocity_profile"] = vel_prof
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cfgs, last, args.cpu_seconds, args.warmup + args.steps)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    if out is not None:
        print(json.dumps(out))


# VelocityGenerator parameters for the post-search stage (synthetic; the reference's
# ROS parameters are not part of the benchmark config): max, coast, lateral, accel, decel.
VEL_PARAMS = (10.0, 3.0, 2.5, 1.5, 3.0)


def velocity_profile_phase(gpu, last, device, vels):
    """VelocityGenerator<float> over every successful path of the last timed step
    (SURVEY §8(f) rank 3): one packed hastar_velocity_profile_batch call, timed after a
    warm-up call.  Host buffers in and out, so the time is PCIe-inclusive."""
    idx = np.nonzero(last.ok & (last.lens > 0))[0]
    if len(idx) == 0:
        return None
    lens = last.lens[idx].astype(np.int64)
    off = np.zeros(len(idx) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    X = np.concatenate([last.xyh[i, :last.lens[i]] for i in idx]).reshape(-1, 3)
    K = np.concatenate([last.curv[i, :last.lens[i]] for i in idx])
    v0 = np.asarray([vels[i] for i in idx], np.float32)
    vm = np.full(len(idx), VEL_PARAMS[0], np.float32)
    flags = np.full(len(idx), 2, np.uint8)  # stop_at_goal
    vg = gpu.VelocityGenerator(*VEL_PARAMS, device=device)
    vg.profile_packed(off, X, K, v0, vm, flags)
    t0 = time.perf_counter()
    feas, vel = vg.profile_packed(off, X, K, v0, vm, flags)
    ms = (time.perf_counter() - t0) * 1e3
    # the oracle (1 thread) over the same paths: CPU time and bit parity
    from oracle import pyoracle
    cpu_s, same = 0.0, True
    for j in range(len(idx)):
        a, b = int(off[j]), int(off[j + 1])
        t1 = time.perf_counter()
        ok_o, vo = pyoracle.velocity_profile(VEL_PARAMS, float(v0[j]), float(vm[j]), X[a:b], K[a:b], False, True)
        cpu_s += time.perf_counter() - t1
        vg_ = vel[a:b]
        nan = np.isnan(vo) & np.isnan(vg_)  # NaN payloads are not part of the contract
        same = same and ok_o == bool(feas[j]) and bool((nan | (vo.view(np.uint32) == vg_.view(np.uint32))).all())
    return {"paths": int(len(idx)), "points": int(off[-1]), "ms_pcie_inclusive": ms,
            "paths_per_s": len(idx) / (ms * 1e-3), "feasible_rate": float(feas.mean()),
            "cpu_oracle_ms": cpu_s * 1e3, "cpu_oracle_cores": 1, "parity_with_oracle": bool(same),
            "params": dict(zip(("max_velocity", "coast_velocity", "max_lat_acc", "max_long_acc", "max_long_dec"),
                               VEL_PARAMS))}


def map_build_phase(args, gpu, dist, torch, rank, world, device):
    """cfg4 (BASELINE.json configs[3]): the map build of `map_queries` queries
    (the same query ids on every rank), timed two ways on the same planners: (a) local — each
    rank builds the whole map (tests/scenarios.py::drive); (b) row-sharded — each rank builds
    N/world rows, then one RCCL all-gather per map and an import
    (path_planning_pkg_amd/shard.py).  Times are per map, max over ranks; `parity` says whether
    every sharded map equals the local build bit for bit on every rank."""
    from path_planning_pkg_amd.shard import drive_sharded
    from tests.scenarios import drive, synthetic
    M = args.map_queries
    cases = [synthetic(args.grid, args.bins, args.obstacles, seed=q + 1) for q in range(M)]
    loc = [gpu.HybridAStar(c, device=device) for c, _ in cases]
    shd = [gpu.HybridAStar(c, device=device) for c, _ in cases]

    def timed(fn):
        if dist:
            dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(device)
        el = time.perf_counter() - t0
        el, _ = reduce_over_ranks(dist, el, 0, f"cuda:{device}")
        return el / M * 1e3

    def local():
        for p, (_, proto) in zip(loc, cases):
            drive(p, proto)

    def sharded():
        for p, (_, proto) in zip(shd, cases):
            drive_sharded(p, proto, rank, world, device)

    t_loc = timed(local)
    t_shd = timed(sharded)
    same = all(np.array_equal(a.get_obstacles().view(np.uint32), b.get_obstacles().view(np.uint32))
               for a, b in zip(loc, shd))
    if dist:
        flag = torch.tensor([0 if same else 1], device=f"cuda:{device}")
        dist.all_reduce(flag)
        same = int(flag[0]) == 0
    for p in loc + shd:
        p.close()
    N = args.grid
    return {"maps": M, "grid": N, "ranks": world, "local_ms_per_map": t_loc, "sharded_ms_per_map": t_shd,
            "allgather_bytes_per_map": N * N * 4, "parity": bool(same),
            "protocol": "update_goal + 5 x {decay, 200 boxes} per map (tests/scenarios.py::drive)"}


def run_cfg5(args, gpu, dist, torch, rank, world, device):
    """BASELINE.json configs[4] / SURVEY.md §8d cfg5: the local planner's replan loop for
    `pairs` start/goal pairs per GPU (pair ids rank*pairs ...; weak scaling, no exchange).
    One step = one 20 Hz tick of every pair: a batched find_path WITHOUT reset (memo and
    stale node-map values carry over, local_planner.cpp:316), then free-space decay and the
    boxes moved by their velocity (local_planner.cpp:241,288).  value = pops / tick wall
    (max over ranks); the tick wall includes the map upkeep."""
    from tests.scenarios import drive, replan_pairs, replan_tick, replan_tick_inputs
    P = args.pairs
    pairs = []
    for q in shard_query_ids(rank, world, P):  # one generator draw per pair id
        pairs += replan_pairs(args.grid, args.bins, args.obstacles, 1, seed=1000 + q)
    t_setup = time.perf_counter()
    planners = []
    for cfg, proto, _ in pairs:
        cfg.values["max_pops"] = args.max_pops
        cfg.values["max_astar_nodes"] = args.max_astar_nodes
        p = gpu.HybridAStar(cfg, device=device)
        drive(p, proto)
        planners.append(p)
    t_setup = time.perf_counter() - t_setup
    bufs = gpu.BatchBuffers(planners, cap=8192)
    vels = [proto["vel"] for _, proto, _ in pairs]
    tick = [0]

    def step():
        t = tick[0]
        starts = [replan_tick_inputs(proto, v, t)[0] for _, proto, v in pairs]
        br = gpu.find_path_batch_arrays(planners, vels, starts, buffers=bufs)
        st = br.stats.copy()
        for p, (_, proto, v) in zip(planners, pairs):
            replan_tick(p, proto, v, t)
        tick[0] += 1
        return st, br.kernel_ms, int(br.ok.sum())

    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    pops, kms, oks, alg = 0, [], 0, []
    for _ in range(args.steps):
        st, k, ok = step()
        pops += int(st["pops"].sum())
        kms.append(k)
        oks += ok
        alg.append(algorithmic_bytes(st, args.obstacles))
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    elapsed, pops_all = reduce_over_ranks(dist, elapsed, pops, f"cuda:{device}")
    out = None
    if rank == 0:
        avg_k = float(np.mean(kms))
        achieved = float(np.mean(alg)) / (avg_k * 1e-3) / 1e9
        out = {
            "metric": "Hybrid A* node expansions/sec + plan latency, 1024x1024x72 grid",
            "value": pops_all / elapsed, "unit": "expansions/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (SURVEY.md §8d cfg5 generator; pair ids seed the boxes, goals and box velocities)",
            "config": {"workload": f"cfg5: {args.grid}x{args.grid}x{args.bins} grid, {args.obstacles} moving boxes, "
                                   f"{P} start/goal pairs per GPU replanned every 50 ms tick without reset",
                       "grid": args.grid, "angle_bins": args.bins, "obstacles": args.obstacles, "pairs_per_gpu": P,
                       "global_batch": P * world, "parallelism": f"pair-sharded x{world}"},
            "replan_latency_ms": avg_k, "tick_ms": elapsed / args.steps * 1e3,
            "tick_budget_ms": 50.0, "success_rate": oks / (P * args.steps), "setup_s_per_gpu": t_setup,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS, "traffic": None, "kernel": "hastar_search_kernel",
                         "kernel_ms": avg_k, "alg_bytes_per_launch": float(np.mean(alg))},
        }
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_cfg5(pairs, args.cpu_seconds, args.warmup + args.steps)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    if out is not None:
        print(json.dumps(out))


def cpu_baseline_cfg5(pairs, budget_s, ticks):
    """The oracle replaying the same pairs' replan loops (1 thread, find_path timed only)."""
    from oracle.pyoracle import OraclePlanner
    from tests.scenarios import drive, replan_tick, replan_tick_inputs
    pops, wall, n = 0, 0.0, 0
    for cfg, proto, v in pairs:
        o = OraclePlanner(cfg)
        drive(o, proto)
        for t in range(ticks):
            r = o.find_path(proto["vel"], replan_tick_inputs(proto, v, t)[0])
            pops += r["stats"]["pops"]
            wall += r["wall_ms"] * 1e-3
            replan_tick(o, proto, v, t)
        o.close()
        n += 1
        if wall >= budget_s:
            break
    return {"value": pops / wall if wall > 0 else None, "unit": "expansions/s", "cores": 1, "kind": "port",
            "sample": f"first {n} pairs x {ticks} ticks (same call sequence as the GPU run), find_path only, "
                      f"1 thread (oracle/hastar_oracle.cpp)"}


def cpu_baseline(cfgs, gpu_results, budget_s, replans):
    """The oracle (CPU restatement, 'port') on the host: single thread, find_path only,
    as the reference harness times it (test_hybrid_astar.cpp:123-126).  Each sampled query
    replays the GPU planner's exact call sequence — the map drive, then `replans` x
    (reset + find_path), warm-up and timed steps alike (the node map's f values persist
    across reset, HybridAStar.cpp:49-52, so later replans differ from the first) — and
    every replan is timed.  The last replan is compared with the GPU's last timed step."""
    from oracle.pyoracle import OraclePlanner
    from tests.scenarios import drive
    pops = 0
    wall = 0.0
    n = 0
    plans = 0
    parity = True
    for i, (cfg, proto) in enumerate(cfgs):
        o = OraclePlanner(cfg)
        drive(o, proto)
        for _ in range(replans):
            o.reset()
            r = o.find_path(proto["vel"], proto["start"])
            pops += r["stats"]["pops"]
            wall += r["wall_ms"] * 1e-3
            plans += 1
        n += 1
        g = gpu_results.result(i)
        parity &= (r["stats"]["pop_digest"] == g["stats"]["pop_digest"] and r["ok"] == g["ok"]
                   and np.float32(r["cost"]).tobytes() == np.float32(g["cost"]).tobytes())
        o.close()
        if wall >= budget_s:
            break
    return {"value": pops / wall if wall > 0 else None, "unit": "expansions/s", "cores": 1, "kind": "port",
            "sample": f"first {n} queries of the GPU batch x {replans} replans each (same call sequence as the GPU "
                      f"run), find_path only, 1 thread (oracle/hastar_oracle.cpp)",
            "mean_plan_ms": wall / plans * 1e3 if plans else None, "parity_with_gpu": bool(parity)}


if __name__ == "__main__":
    main()
