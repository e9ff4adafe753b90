"""bench.py — Hybrid A* node expansions/sec on the 1024x1024x72 grid (BASELINE.json configs[2]).

Workload (one "step"): a batch of B independent planners per GPU (SURVEY.md §8d synthetic
generator with its std::mt19937 draws, tests/scenarios.py:synthetic_ref: N = 1024, 72 angle bins,
K = 200 box obstacles, seed = query id + 1; the
reference's only motion mode: forward Dubins), each already set up in HBM (update_goal,
5 x {decay, boxes} through the batched map-update ABI); the step resets the holonomic memo
of every planner (HybridAStar::reset) and runs ONE batched find_path — one wavefront per
planner (plus resume launches for searches that outgrow their arena, if any).
value = total pops of all planners on all ranks / wall time of the K timed steps (max over
ranks).  One rank per GPU (torch.distributed; RCCL for the barrier / reductions only):
planners are sharded across ranks with no data-path collective -> weak scaling.

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment starts
torch.distributed.run with N ranks as a child process (before anything touches a GPU) and
exits with its status.

Extra fields: the first (cold: no longest-first history) step's throughput, plan latency of
single queries on the GPU and on one CPU core for the SAME queries, the search kernel's
roofline (SURVEY.md §8d algorithmic bytes / kernel time from HIP events on its stream), and
the CPU oracle timed on `cores` host threads, one private planner per thread (rank 0).
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "Hybrid A* node expansions/sec + plan latency, 1024x1024x72 grid"


_T0 = time.perf_counter()


def progress(msg):
    """One progress line on stderr (a long run under a profiler keeps showing signs of life)."""
    print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def algorithmic_bytes(st, K):
    """B = 40 P + 44 S + 208 A + 12 K per plan, summed over the batch
    (st: the stats structured array of one batched call)."""
    return float(40 * st["pops"].astype(np.float64).sum() + 44 * st["successors"].astype(np.float64).sum()
                 + 208 * st["astar_pops"].astype(np.float64).sum() + 12.0 * K * len(st))


def step_balance(planners):
    """What bounds the last timed step: the resident slots' busy time (the bulk of the
    batch) or the longest search (its straggler).  From every search's start/end stamps
    (s_memrealtime, 10 ns ticks) and the slot that ran it."""
    t = np.array([p.timing() for p in planners], dtype=np.float64)
    dur = (t[:, 1] - t[:, 0]) * 1e-5  # ms
    span = (t[:, 1].max() - t[:, 0].min()) * 1e-5
    slots = len(set(int(s) for s in t[:, 2]))
    li = int(np.argmax(dur))
    return {"span_ms": float(span), "slots_used": slots, "slot_busy_mean_ms": float(dur.sum() / slots),
            "busy_frac": float(dur.sum() / (slots * span)), "longest_search_under_load_ms": float(dur[li]),
            "longest_search_start_ms": float((t[li, 0] - t[:, 0].min()) * 1e-5)}


def cold_tail(t, pops, qids, k=6):
    """The k searches of a step that ended last: query, pops, start and end (ms from the step's
    first start), and the slot that ended it (>= the pool's arena count: a head arena)."""
    if t is None:
        return None
    t0 = t[:, 0].min()
    idx = np.argsort(-t[:, 1], kind="stable")[:k]
    return [{"query": int(qids[i]), "pops": int(pops[i]), "start_ms": float((t[i, 0] - t0) * 1e-5),
             "end_ms": float((t[i, 1] - t0) * 1e-5), "slot": int(t[i, 2])} for i in idx]


def step_diag(planners, res):
    """One step's schedule: span of the searches, the split launch's event times, and the start
    offset / duration (ms) of the searches on the latency CUs (arenas 0 .. head_cus - 1) and of
    the step's longest search."""
    t = np.array([p.timing() for p in planners], dtype=np.float64)
    t0 = t[:, 0].min()
    dur = (t[:, 1] - t[:, 0]) * 1e-5
    head_cus = int(planners[0].slots()["head_cus"])
    head = np.nonzero(t[:, 2] < head_cus)[0]
    first = head[np.argsort(t[head, 0])][:16]
    li = int(np.argmax(dur))
    st = res.stats
    # where each search ran: (XCC, SE, SH, CU) of its wavefront; a CU pair (CU, CU ^ 1) shares
    # an instruction cache, so the partner CU's searches (other kernel or not) are counted
    hw = [p.hw_id() for p in planners]
    cu_key = [(x, se, sh, cu) for x, cu, se, sh, _ in hw]
    from collections import Counter
    on_cu = Counter(cu_key)

    def row(i):  # start offset ms, duration ms, arena, planner index, pops, inner A* pops, XCC, SE, SH, CU,
        x, se, sh, cu = cu_key[i]  # searches on the instruction-cache partner CU in this step, shader MHz
        cyc = planners[i].cycles()  # [38], [39]: s_memtime at the search's start and end (0 if parked)
        mhz = (cyc[39] - cyc[38]) / ((t[i, 1] - t[i, 0]) * 1e-8) / 1e6 if (cyc[39] > cyc[38] and int(st["parks"][i]) == 0
                                                                       and t[i, 1] > t[i, 0]) else None
        return [round(float((t[i, 0] - t0) * 1e-5), 1), round(float(dur[i]), 1), int(t[i, 2]), int(i),
                int(st["pops"][i]), int(st["astar_pops"][i]), x, se, sh, cu, on_cu[(x, se, sh, cu ^ 1)],
                round(mhz, 1) if mhz else None]
    return {"kernel_ms": float(res.kernel_ms), "span_ms": float((t[:, 1].max() - t0) * 1e-5),
            "split_ms": planners[0].split_ms(), "head": [row(i) for i in first], "longest": row(li)}


def shard_query_ids(rank, world, batch, pred=None):
    """Queries of one rank: weak scaling, B per GPU, disjoint across ranks, no exchange.  The
    global queries 0 .. world * B - 1 are dealt by predicted cost (`pred`, one value per global
    query, larger = costlier; every rank computes the same values from the inputs alone): sorted
    costliest first, then dealt in snake order (0, 1, .., W-1, W-1, .., 0, ...), so every rank
    gets the same number of queries and a like share of the predicted-long ones, and no rank's
    block collects the tail.  Each rank's ids come back in ascending id order: the batch's own
    order carries no prediction (a batch with no history is ordered by the library's cold key,
    hastar_capi.cpp:cold_key, the same score).  pred None: contiguous blocks."""
    assert 0 <= rank < world
    if pred is None:
        return [rank * batch + i for i in range(batch)]
    pred = np.asarray(pred, np.float64)
    assert len(pred) == world * batch
    order = np.argsort(-pred, kind="stable")
    pos = np.arange(world * batch)
    rnd, k = pos // world, pos % world
    owner = np.where(rnd % 2 == 0, k, world - 1 - k)
    return sorted(int(q) for q in order[owner == rank])


def shard_global_ids(rank, world, total):
    """A fixed global set of `total` ids dealt round-robin over the ranks (strong scaling)."""
    assert 0 <= rank < world
    return list(range(rank, total, world))


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


def cpu_threads():
    """Host threads of the CPU baseline: HASTAR_CPU_THREADS, else OMP_NUM_THREADS (the GPU
    box sets it to this job's CPU share), else the visible cores."""
    for k in ("HASTAR_CPU_THREADS", "OMP_NUM_THREADS"):
        v = os.environ.get(k)
        if v and v.isdigit() and int(v) > 0:
            return int(v)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def launch_ranks(args):
    """Start `args.gpus` ranks under torch.distributed.run (a child process; this process has
    not touched a GPU) and return its exit status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve())] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); > 1 without WORLD_SIZE spawns them")
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 3; cfg5: 20 ticks, SURVEY.md §8(d)'s 20 ticks at 20 Hz)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("HASTAR_BENCH_BATCH", "23552")),
                    help="planners (queries) per GPU")
    ap.add_argument("--grid", type=int, default=None, help="default 1024 (cfg3, cfg5) or 2048 (cfg4)")
    ap.add_argument("--bins", type=int, default=72)
    ap.add_argument("--obstacles", type=int, default=200)
    ap.add_argument("--max-pops", type=int, default=None,
                    help="initial arena of a search in pops (0 = the library's 262144; default: 196608 for cfg3 "
                         "so that ~1984 arenas of 46 MiB fit next to the planners' maps, 0 otherwise)")
    ap.add_argument("--max-astar-nodes", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU-oracle baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-all", action="store_true",
                    help="check EVERY query's cold step against the oracle (success, cost bits, statistics, "
                         "pop/closed digests; about a minute of 16 host threads at cfg3)")
    ap.add_argument("--step-diag", action="store_true",
                    help="per-step schedule diagnostics in the JSON line (reads every search's timing per step)")
    ap.add_argument("--latency-queries", type=int, default=3)
    ap.add_argument("--workload", choices=("cfg3", "cfg4", "cfg5"), default="cfg3",
                    help="cfg3: batch of independent queries (default, the headline line); "
                         "cfg4: 2048^2 queries with the map build row-sharded over the ranks + RCCL all-gather "
                         "(BASELINE.json configs[3]); cfg5: 20 Hz replan loop of start/goal pairs (configs[4])")
    ap.add_argument("--map-queries", type=int, default=16, help="cfg4: maps built both locally and row-sharded")
    ap.add_argument("--pairs", type=int, default=64, help="cfg5: start/goal pairs in total, dealt over the ranks")
    ap.add_argument("--generator", choices=("mt19937", "pcg64"), default="mt19937",
                    help="cfg3/cfg4 inputs: SURVEY.md §8d's std::mt19937 draws (the survey's reference runs) or "
                         "round 1's numpy PCG64 draws")
    ap.add_argument("--relaxed-delta", type=float, default=0.25, help="relaxed mode: frontier width (m)")
    ap.add_argument("--relaxed-weight", type=float, default=1.35, help="relaxed mode: heuristic weight (the library default)")
    ap.add_argument("--no-relaxed", action="store_true", help="cfg5: skip the relaxed-mode comparison")
    ap.add_argument("--relaxed-batch-nodes", type=int, default=1 << 16,
                    help="relaxed batch: node capacity per search (hastar_relaxed_opts.max_nodes)")
    ap.add_argument("--relaxed-reverse-cost", type=float, default=1.5,
                    help="relaxed batch leg: also run it with the reversing model at this reverse cost (0: skip)")
    ap.add_argument("--relaxed-gear-cost", type=float, default=1.0, help="... and this gear-change cost (m)")
    ap.add_argument("--relaxed-batch", type=int, default=4096,
                    help="cfg3/cfg4: queries of the batch also planned in one relaxed call (query rate)")
    ap.add_argument("--dump-timings", default=None,
                    help="write every search's start/end/slot of the last timed step and of the cold-order "
                         "step (npz) to this path")
    ap.add_argument("--no-deal", action="store_true",
                    help="cfg3/cfg4: contiguous query blocks per rank instead of the predicted-cost deal")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL; gloo for rehearsals)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU work: exercises the launcher, sharding and reductions only (CPU rehearsal)")
    args = ap.parse_args(argv)
    if args.grid is None:
        args.grid = 2048 if args.workload == "cfg4" else 1024
    if args.max_pops is None:
        # cfg3: 8 search wavefronts per CU need ~2048 arenas; at 196608 pops (the batch's longest
        # search needs 172207) they take 46 MiB each and 1984 fit beside 23552 planners' maps.
        # A search that outgrows its arena parks and resumes in a 4x one, so this is no limit.
        args.max_pops = 196608 if args.workload == "cfg3" else 0
    if args.workload == "cfg4" and "--batch" not in sys.argv and "HASTAR_BENCH_BATCH" not in os.environ:
        # 2048^2 maps: 32 MiB per planner.  The step is bound by the batch's longest search (597k
        # pops), so planners are worth more than arenas: 7680 planners leave ~360 arenas of 107 MiB,
        # which finish the rest of the batch in ~65 % of the step (profiles/r02w_cfg4_*).
        args.batch = 7680
    if args.steps is None:
        # cfg5 times SURVEY.md §8(d)'s 20 ticks at 20 Hz (local_planner.cpp:204-205, 241, 316)
        args.steps = 20 if args.workload == "cfg5" else 3
    return args


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
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
        if args.backend == "nccl":
            torch.cuda.set_device(local_rank)
        # rank 0 checks parity on the host after the timed region while the others wait at the
        # closing barrier: a generous timeout
        import datetime
        dist.init_process_group(args.backend, timeout=datetime.timedelta(minutes=30))
    # HASTAR_BENCH_DEVICE: put every rank on one device (a multi-rank rehearsal on a one-GPU box,
    # with --backend gloo); by default rank r uses GPU LOCAL_RANK
    device = int(os.environ.get("HASTAR_BENCH_DEVICE", local_rank))
    red_dev = f"cuda:{device}" if args.backend == "nccl" and not args.dry_run else "cpu"
    if args.dry_run:
        return run_dry(args, dist, rank, world, red_dev)

    from path_planning_pkg_amd import planner as gpu

    if args.workload == "cfg5":
        return run_cfg5(args, gpu, dist, torch, rank, world, device)
    B = args.batch
    map_build = map_build_phase(args, gpu, dist, torch, rank, world, device) if args.workload == "cfg4" else None
    # every rank derives the same predicted costs of all world * B queries from their inputs
    # (no exchange); the deal balances predicted cost and orders each rank's batch by it
    t_pred = time.perf_counter()
    pred = None
    if args.generator == "mt19937" and not args.no_deal:
        from tests.scenarios import predicted_cost
        pred = predicted_cost(args.grid, args.obstacles, np.arange(world * B))
    t_pred = time.perf_counter() - t_pred
    qids = shard_query_ids(rank, world, B, pred)
    t_gen = time.perf_counter()
    cfgs = [query_case(args, q) for q in qids]
    t_gen = time.perf_counter() - t_gen
    t_setup = time.perf_counter()
    planners, setup_split = build_planners(gpu, cfgs, device)
    t_setup = time.perf_counter() - t_setup
    progress(f"{B} planners set up")
    vels = [c[1]["vel"] for c in cfgs]
    starts = [c[1]["start"] for c in cfgs]

    # host-side batch arguments and output arrays are allocated once and reused every step
    bufs = gpu.BatchBuffers(planners, cap=8192)
    # the device pool (search arenas, batch tables, packed-path buffers) is reserved once at
    # setup, as a serving process reserves its memory at start-up; the cold first step then
    # measures the missing longest-first history alone
    t_res = time.perf_counter()
    gpu.reserve(planners, path_points=1024 * len(planners))
    torch.cuda.synchronize(device)
    setup_split["reserve_s"] = time.perf_counter() - t_res

    def step():
        gpu.reset_batch(bufs)  # HybridAStar::reset() of every planner
        return gpu.find_path_batch_arrays(planners, vels, starts, buffers=bufs)

    # the first step is cold: the longest-first queue has no history yet
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    r0 = step()
    cold_s = time.perf_counter() - t0
    cold_handoffs = planners[0].handoffs()
    # what bounded the cold step: its last-ending searches (start, end, slot, pops), host-side
    cold_t = np.array([p.timing() for p in planners], dtype=np.float64) if rank == 0 else None
    progress("cold first step done")
    # the first step's outcome of a stratified sample (every 64th query and the 8 with the most
    # pops), paths included, for the bit-exact check against the oracle after the timed region
    # (host-side bookkeeping of the bench, outside the step's time)
    strat = sorted(set(range(0, B, 64)) | set(np.argsort(-r0.stats["pops"], kind="stable")[:8].tolist()))
    cold_sample = {i: r0.result(i) for i in strat} if (rank == 0 and not args.no_cpu_baseline) else None
    cold_all = None
    if rank == 0 and args.parity_all:  # every query's outcome, paths as digests of their bits
        cold_all = (r0.stats.copy(), r0.cost.copy(), r0.ok.copy(),
                    [path_digest(r0.result(i)) for i in range(B)])
    cold_pops = int(r0.stats["pops"].sum())
    r0_pops = r0.stats["pops"].copy()
    cold_s, cold_pops_all = reduce_over_ranks(dist, cold_s, cold_pops, f"cuda:{device}")
    for _ in range(max(args.warmup - 1, 0)):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    pops = 0
    kernel_ms, alg_bytes = [], []
    statuses = set()
    oks, parks = 0, 0
    last = None
    diag = []
    for _ in range(args.steps):
        res = step()
        kernel_ms.append(res.kernel_ms)
        if args.step_diag:  # per-step schedule diagnostics (inside the timed region: off by default)
            diag.append(step_diag(planners, res))
        st = res.stats
        pops += int(st["pops"].sum())
        alg_bytes.append(algorithmic_bytes(st, args.obstacles))
        statuses |= set(int(v) for v in np.unique(st["status"]))
        oks += int(res.ok.sum())
        parks += int(st["parks"].sum())
        last = res
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    elapsed, pops_all = reduce_over_ranks(dist, elapsed, pops, f"cuda:{device}")

    out = None
    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        avg_kernel_ms = float(np.mean(kernel_ms))
        achieved = float(np.mean(alg_bytes)) / (avg_kernel_ms * 1e-3) / 1e9
        balance = step_balance(planners)  # before any other find_path overwrites the timings
        balance["pool"] = planners[0].slots()
        balance["split_launch_ms"] = dict(zip(("head_start", "head_end", "bulk_start", "bulk_end"),
                                              planners[0].split_ms()))
        # searches the last step's split launch moved from batch slots to free latency CUs
        balance["handoffs"] = planners[0].handoffs()
        pool = balance["pool"]  # the library splits a batch over 4x the CU count (hastar_capi.cpp batch_shape)
        split_launch = (os.environ.get("HASTAR_SPLIT", "1") != "0" and pool["head_cus"] > 0
                        and B > 4 * (pool["resident_slots"] // max(pool["waves_per_cu"], 1)))
        timings = {"qids": np.asarray(qids), "pops": last.stats["pops"].copy(),
                   "astar_pops": last.stats["astar_pops"].copy(),
                   "warm": np.array([p.timing() for p in planners], dtype=np.float64)}
        progress("timed steps done")
        # the last timed replan of the same stratified sample, paths included, for the oracle's
        # replay of the whole call sequence (the node map's f values persist across reset, so a
        # later replan is not the first one again)
        last_sample = {i: last.result(i) for i in cold_sample} if cold_sample is not None else None
        vel_prof = velocity_profile_phase(gpu, last, device, vels)  # before any other find_path
        # the outcome arrays of the last timed step outlive the later steps on the same buffers
        # (paths are not kept: only the velocity phase above reads them)
        last = gpu.BatchResult(last.cost.copy(), last.ok.copy(), last.lens.copy(), None, None,
                               last.stats.copy(), last.kernel_ms)
        # a batch of fresh queries on a warm device: no longest-first history (every cost hint
        # cleared), arenas already allocated — the library orders the queue by its cold key
        for p in planners:
            p.set_cost_hint(0)
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        rc = step()
        cold_order_s = time.perf_counter() - t0
        if args.dump_timings:
            timings["cold_order"] = np.array([p.timing() for p in planners], dtype=np.float64)
            np.savez(args.dump_timings, **timings)
        cold_order = {"value": float(rc.stats["pops"].sum()) / cold_order_s, "ms": cold_order_s * 1e3,
                      "note": "a step with every planner's cost hint cleared (no longest-first history) on an "
                              "initialised device: the library orders the queue by its cold key"}
        # latency queries: the survey's first seeds (query ids 0, 1, ..) where this rank has them
        pos = {q: i for i, q in enumerate(qids)}
        lat_ids = [pos[q] for q in range(args.latency_queries) if q in pos]
        lat_ids += [i for i in range(B) if i not in lat_ids][:max(0, min(args.latency_queries, B) - len(lat_ids))]
        lat = []
        for i in lat_ids:  # single-query plan latency (the second half of the metric)
            planners[i].reset()
            _, kms = gpu.find_path_batch([planners[i]], [vels[i]], [starts[i]], cap=8192)
            lat.append(kms)
        # the batch's longest search alone (its latency bounds the step)
        li = int(np.argmax(last.stats["pops"]))
        longest = {"query": qids[li], "pops": int(last.stats["pops"][li])}
        planners[li].reset()
        _, longest["gpu_ms_alone"] = gpu.find_path_batch([planners[li]], [vels[li]], [starts[li]], cap=8192)
        progress("latency queries done")
        relaxed = relaxed_latency_phase(gpu, planners, vels, starts, last, lat_ids + [li], qids, args,
                                        lat + [longest["gpu_ms_alone"]], B / (ms_per_step * 1e-3))
        traffic = None
        pmc = ROOT / "profiles" / "pmc_search_summary.json"
        if pmc.exists():
            try:
                pm = json.loads(pmc.read_text())
                # only for the kernel it was measured on (sources hash), else traffic = null
                from path_planning_pkg_amd.buildinfo import search_kernel_hash
                if (pm.get("batch") == B and pm.get("grid") == args.grid
                        and pm.get("kernel_src_sha") == search_kernel_hash()):
                    traffic = pm.get("hbm_bytes_per_launch")
            except (ValueError, OSError):
                traffic = None
        out = {
            "metric": METRIC,
            "value": pops_all / elapsed,
            "unit": "expansions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic (SURVEY.md §8d generator, std::mt19937 draws as in the survey's reference runs; "
                     "seeds = query ids + 1)") if args.generator == "mt19937" else
                    "synthetic (SURVEY.md §8d geometry, numpy PCG64 draws; seeds = query ids + 1)",
            "config": {"workload": f"{args.workload}: {args.grid}x{args.grid}x{args.bins} grid, {args.obstacles} box "
                                   f"obstacles, batch of {B} independent queries per GPU, forward Dubins"
                                   + (", map build row-sharded over the ranks + RCCL all-gather (map_build)"
                                      if map_build else ""),
                       "grid": args.grid, "angle_bins": args.bins, "obstacles": args.obstacles,
                       "queries_per_gpu": B, "global_batch": B * world, "parallelism": f"query-sharded x{world}"},
            "kernel_only_value": pops_all / elapsed * ms_per_step / avg_kernel_ms,
            "kernel_ms_per_step": [float(k) for k in kernel_ms],
            **({"step_diag": diag} if diag else {}),
            "cold_first_step": {"value": cold_pops_all / cold_s, "ms": cold_s * 1e3, "handoffs": cold_handoffs,
                                "last_to_end": cold_tail(cold_t, r0_pops, qids),
                                "note": "first launch of the batch: no longest-first history (the library orders the "
                                        "queue by its cold key: boxes near the start-goal route, hastar.h "
                                        "hastar_set_cost_hint); the device pool was reserved at setup "
                                        "(hastar_reserve, setup_split_s.reserve_s)"},
            "cold_order_step": cold_order,
            "plan_latency_ms": {"gpu_median": float(np.median(lat)) if lat else None, "queries": [qids[i] for i in lat_ids],
                                "gpu": lat},
            "longest_query": longest,
            "step_balance": balance,
            "pops_per_step": pops_all / args.steps,
            "success_rate": oks / (B * args.steps),
            "search_status": sorted(statuses),
            "parks_per_step": parks / args.steps,
            "setup_s_per_gpu": t_setup + setup_split["reserve_s"],
            "setup_split_s": dict(setup_split, inputs_generated_s=t_gen, cost_prediction_s=t_pred),
            "query_deal": "predicted-cost snake deal over the ranks (tests/scenarios.py:predicted_cost = the library's "
                          "cold key), ids ascending within a rank" if pred is not None
                          else "contiguous blocks",
            "roofline": {"bound": "latency", "roof": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                         "kernel": ("hastar_search_kernel + hastar_search_wide_kernel (split launch: the batch "
                                    "kernel beside the latency kernel on the queue's head)" if split_launch
                                    else "hastar_search_kernel"),
                         "kernel_ms": avg_kernel_ms,
                         "alg_bytes_per_launch": float(np.mean(alg_bytes)),
                         "note": "kernel_ms: HIP events from the fork to the join of the launch; achieved = "
                                 "SURVEY §8(d) algorithmic bytes of the whole batch / kernel_ms.  traffic: HBM bytes "
                                 "per launch from a PMC pass (FETCH_SIZE/WRITE_SIZE, profiles/pmc_search_summary.json) "
                                 "of the same batch with HASTAR_SPLIT=0 (the batch kernel alone: counter collection "
                                 "serialises the split launch's two kernels), null unless its kernel-source hash "
                                 "matches this build.  Dependent per-wave round trips bound the search, not HBM "
                                 "bandwidth (SQ/TCC counters in profiles/, DESIGN.md §4.1)"},
        }
        if map_build:
            out["map_build"] = map_build
        out["velocity_profile"] = vel_prof
        out["relaxed_mode"] = relaxed
        if not args.no_cpu_baseline:
            # the CPU sample runs the rank's queries in query-id order (a representative sample,
            # not the predicted-costliest head of the GPU batch), latency queries first
            sample = lat_ids + [i for i in np.argsort(qids, kind="stable") if i not in lat_ids]
            progress("parity sample")
            out["parity_sample"] = parity_sample(cfgs, cold_sample, [qids[i] for i in sorted(cold_sample)],
                                                 last_sample, args.warmup + args.steps)
            if cold_all is not None:
                progress("parity of every query")
                out["parity_all"] = parity_all(cfgs, *cold_all, qids)
            if world == 1:  # the CPU baseline is an N = 1 figure (rank 0 of a one-GPU run)
                progress("cpu baseline")
                cb = cpu_baseline(cfgs, last, args.cpu_seconds, args.warmup + args.steps, lat_ids, sample)
                out["cpu_baseline"] = cb
                out["plan_latency_ms"]["cpu_same_queries_median"] = cb.pop("latency_same_queries_ms", None)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    if out is not None:
        print(json.dumps(out))


def query_case(args, q):
    from tests.scenarios import synthetic, synthetic_ref
    gen = synthetic_ref if args.generator == "mt19937" else synthetic
    cfg, proto = gen(args.grid, args.bins, args.obstacles, seed=q + 1)
    cfg.values["max_pops"] = args.max_pops
    cfg.values["max_astar_nodes"] = args.max_astar_nodes
    return cfg, proto


def build_planners(gpu, cfgs, device):
    """Create the planners and run the fixture protocol on all of them through the batched
    map-update ABI (tests/scenarios.py::drive_batch)."""
    import torch
    from tests.scenarios import drive_batch
    t0 = time.perf_counter()
    # every query of the workload has the same planner parameters: one batched create
    planners = gpu.HybridAStar.create_batch(cfgs[0][0], len(cfgs), device=device)
    t1 = time.perf_counter()
    drive_batch(gpu, planners, [proto for _, proto in cfgs])
    torch.cuda.synchronize(device)
    t2 = time.perf_counter()
    return planners, {"create_s": t1 - t0, "map_updates_s": t2 - t1}


def run_dry(args, dist, rank, world, red_dev):
    """--dry-run: the launcher / sharding / reduction path without GPU work (each 'query'
    counts one pop), so a CPU box can rehearse `bench.py --gpus N`."""
    ids = shard_global_ids(rank, world, args.pairs) if args.workload == "cfg5" else shard_query_ids(rank, world, args.batch)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    elapsed, pops_all = reduce_over_ranks(dist, time.perf_counter() - t0, len(ids), red_dev)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": pops_all / elapsed, "unit": "expansions/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3,
                          "higher_is_better": True, "scaling": "strong" if args.workload == "cfg5" else "weak",
                          "vs_baseline": None, "dtype": "f32", "data": "dry run (no GPU work)",
                          "config": {"workload": args.workload, "units_total": int(pops_all),
                                     "parallelism": f"x{world}"}}))
    if dist:
        dist.barrier()
        dist.destroy_process_group()


# VelocityGenerator parameters for the post-search stage (synthetic; the reference's
# ROS parameters are not part of the benchmark config): max, coast, lateral, accel, decel.
VEL_PARAMS = (10.0, 3.0, 2.5, 1.5, 3.0)


def velocity_profile_phase(gpu, last, device, vels):
    """VelocityGenerator<float> over every path of the last timed step,
    two ways: (a) device-resident — hastar_velocity_profile_last_batch profiles the paths where
    the batch packed them in HBM (local_planner.cpp:316-323 profiles the search's own output),
    velocities back to the host; (b) host buffers in and out (PCIe-inclusive, paths uploaded).
    (b) is compared with the oracle bit for bit, (a) with (b).  Must run before any other
    find_path call on the device (it would replace the last batch)."""
    idx = np.nonzero(last.ok & (last.lens > 0))[0]
    if len(idx) == 0:
        return None
    n_all = len(last.lens)
    vg = gpu.VelocityGenerator(*VEL_PARAMS, device=device)
    v0a = np.asarray(vels, np.float32)
    vma = np.full(n_all, VEL_PARAMS[0], np.float32)
    fla = np.full(n_all, 2, np.uint8)
    lens_all = last.lens.astype(np.int64).copy()
    vg.profile_last_batch(lens_all, v0a, vma, fla)
    ms_dev = float("inf")  # best of 3 (host-side page faults on the output arrays vary)
    for _ in range(3):
        t0 = time.perf_counter()
        feas_a, vel_a = vg.profile_last_batch(lens_all, v0a, vma, fla)
        ms_dev = min(ms_dev, (time.perf_counter() - t0) * 1e3)
    lens = last.lens[idx].astype(np.int64)
    off = np.zeros(len(idx) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    X = np.concatenate([last.xyh[i, :last.lens[i]] for i in idx]).reshape(-1, 3)
    K = np.concatenate([last.curv[i, :last.lens[i]] for i in idx])
    v0 = np.asarray([vels[i] for i in idx], np.float32)
    vm = np.full(len(idx), VEL_PARAMS[0], np.float32)
    flags = np.full(len(idx), 2, np.uint8)  # stop_at_goal
    vg.profile_packed(off, X, K, v0, vm, flags)
    ms = float("inf")
    for _ in range(3):
        t0 = time.perf_counter()
        feas, vel = vg.profile_packed(off, X, K, v0, vm, flags)
        ms = min(ms, (time.perf_counter() - t0) * 1e3)
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
    # (a) vs (b): the device-resident profile of every successful path, bit for bit
    off_all = np.zeros(n_all + 1, np.int64)
    np.cumsum(lens_all, out=off_all[1:])
    same_dev = bool(all(bool(feas_a[i]) == bool(feas[j]) and np.array_equal(
        vel_a[off_all[i]:off_all[i + 1]].view(np.uint32), vel[off[j]:off[j + 1]].view(np.uint32))
        for j, i in enumerate(idx)))
    return {"paths": int(len(idx)), "points": int(off[-1]), "ms_device_resident": ms_dev,
            "device_resident_equals_host_path": same_dev, "ms_pcie_inclusive": ms,
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
    field = field_phase(shd[0], dist, torch, rank, world, device)
    for p in loc + shd:
        p.close()
    N = args.grid
    return {"maps": M, "grid": N, "ranks": world, "local_ms_per_map": t_loc, "sharded_ms_per_map": t_shd,
            "allgather_bytes_per_map": N * N * 4, "parity": bool(same),
            "protocol": "update_goal + 5 x {decay, 200 boxes} per map (tests/scenarios.py::drive)",
            "heuristic_field": field}


def field_phase(p, dist, torch, rank, world, device, standins=4):
    """cfg4's heuristic precompute (BASELINE.json configs[3]; include/hastar.h:
    hastar_heuristic_field): the backward grid-distance field of the first map, (a) whole on every
    rank, (b) row-sharded over the job's ranks with edge-row all-gathers
    (shard.py:heuristic_field_sharded), and on one rank (c) with `standins` stand-in ranks on
    the one GPU.  Times are max over ranks; `parity`: (b) and (c) equal (a) bit for bit."""
    from path_planning_pkg_amd.shard import heuristic_field_sharded, heuristic_field_standins
    N = p.N
    dev = f"cuda:{device}"
    out = torch.empty(N * N, dtype=torch.float32, device=dev)
    torch.cuda.synchronize(device)
    p.heuristic_field(out.data_ptr())  # warm-up

    def timed(fn):
        if dist:
            dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize(device)
        el, _ = reduce_over_ranks(dist, time.perf_counter() - t0, 0, dev)
        return el * 1e3, r

    t_one, passes = timed(lambda: p.heuristic_field(out.data_ptr()))
    t_shd, (full, rounds, spasses) = timed(lambda: heuristic_field_sharded(p, rank, world, dev))
    same = bool(torch.equal(full.view(torch.int32), out.view(torch.int32)))
    res = {"grid": N, "one_gpu_ms": t_one, "passes": passes, "finite_cells": int(torch.isfinite(out).sum()),
           "ranks": world, "sharded_ms": t_shd, "exchange_rounds": rounds, "sharded_passes": spasses}
    if world == 1:
        t_st, (sfull, srounds, _) = timed(lambda: heuristic_field_standins(p, standins, torch.device(dev)))
        same = same and bool(torch.equal(sfull.view(torch.int32), out.view(torch.int32)))
        res.update(standin_ranks=standins, standin_ms=t_st, standin_rounds=srounds)
    if dist:
        flag = torch.tensor([0 if same else 1], device=dev)
        dist.all_reduce(flag)
        same = int(flag[0]) == 0
    res["parity"] = same
    res["note"] = ("backward 8-connected grid distance to the goal over the free cells (csrc/hastar_field.hip); "
                   "sharded: row blocks + edge-row all-gathers until no block edge changes; bit-equal by construction "
                   "(the field's equations have one solution) and by this check")
    return res


def relaxed_latency_phase(gpu, planners, vels, starts, last, ids, qids, args, exact_ms, exact_qps):
    """The RELAXED mode (hastar_find_path_relaxed_batch, SURVEY.md §8(f) rank 4: non-parity,
    frontier-parallel with a backward-Dijkstra heuristic) on the latency queries and the longest
    query, one query per call, beside the exact mode's result for the same inputs (the last timed
    step).  Not part of `value`: a different algorithm, reported separately."""
    opts = dict(delta=args.relaxed_delta, h_weight=args.relaxed_weight)
    ms, ratios, ok, exp = [], [], 0, []
    for i in ids:
        r, kms = gpu.find_path_batch([planners[i]], [vels[i]], [starts[i]], cap=8192, relaxed=opts)
        r = r[0]
        ms.append(kms)
        ok += int(r["ok"])
        exp.append(int(r["stats"]["pops"]))
        if r["ok"] and last.ok[i]:
            ratios.append(float(r["cost"]) / float(last.cost[i]))
    # the batch's first queries in one relaxed call (one workgroup per planner, every CU busy),
    # against the exact mode's query rate of the timed steps
    nb = min(args.relaxed_batch, len(planners))
    batch = None
    if nb > 0:
        # node capacity 64 k per search (these queries expand < 5 k nodes; the library's default
        # 256 k sizes an arena at 34 MiB, and beside the exact pool the HBM then holds only a
        # quarter as many arenas as CUs)
        bopts = dict(opts, max_nodes=args.relaxed_batch_nodes)
        t0 = time.perf_counter()
        rb, bms = gpu.find_path_batch(planners[:nb], vels[:nb], starts[:nb], cap=8192, relaxed=bopts)
        wall = time.perf_counter() - t0
        groups, arena_mib = planners[0].relaxed_pool()
        br = [float(r["cost"]) / float(last.cost[i]) for i, r in enumerate(rb) if r["ok"] and last.ok[i]]
        batch = {"queries": nb, "kernel_ms": bms, "wall_ms": wall * 1e3, "queries_per_s": nb / (bms * 1e-3),
                 "exact_queries_per_s": exact_qps, "ok": sum(int(r["ok"]) for r in rb),
                 "exact_ok": int(sum(int(last.ok[i]) for i in range(nb))),
                 "status": sorted({int(r["stats"]["status"]) for r in rb}),
                 "cost_ratio_vs_exact_mean": float(np.mean(br)) if br else None,
                 "cost_ratio_vs_exact_max": float(np.max(br)) if br else None,
                 "workgroups": groups, "arena_mib": arena_mib, "max_nodes": args.relaxed_batch_nodes}
        if args.relaxed_reverse_cost > 0:
            # BASELINE.json configs[2] names "Reeds-Shepp reversals enabled": the same batch with the
            # relaxed mode's reversing model (the reference itself drives forward only)
            ropts = dict(bopts, reverse_cost=args.relaxed_reverse_cost, gear_cost=args.relaxed_gear_cost)
            rr, rms = gpu.find_path_batch(planners[:nb], vels[:nb], starts[:nb], cap=8192, relaxed=ropts)
            rrat = [float(r["cost"]) / float(last.cost[i]) for i, r in enumerate(rr) if r["ok"] and last.ok[i]]
            rev_poses = sum(int((r["direction"] < 0).sum()) for r in rr if r["ok"] and "direction" in r)
            all_poses = sum(len(r["path"]) for r in rr if r["ok"])
            batch["reversing"] = {
                "reverse_cost": args.relaxed_reverse_cost, "gear_cost": args.relaxed_gear_cost, "kernel_ms": rms,
                "queries_per_s": nb / (rms * 1e-3), "ok": sum(int(r["ok"]) for r in rr),
                "status": sorted({int(r["stats"]["status"]) for r in rr}),
                "cost_ratio_vs_exact_mean": float(np.mean(rrat)) if rrat else None,
                "cost_ratio_vs_exact_max": float(np.max(rrat)) if rrat else None,
                "paths_with_reverse": sum(int((r["direction"] < 0).any()) for r in rr if r["ok"] and "direction" in r),
                "reverse_pose_fraction": rev_poses / max(all_poses, 1),
                "note": "reverse arcs (action cost x reverse_cost), Reeds-Shepp heuristic and shots "
                        "(csrc/hastar_rs.h); costs relative to the exact forward-only result"}
    return {"batch": batch, "queries": [qids[i] for i in ids], "gpu_ms": ms, "gpu_median_ms": float(np.median(ms)) if ms else None,
            "exact_gpu_ms_same_queries": exact_ms, "ok": ok, "exact_ok": int(sum(int(last.ok[i]) for i in ids)),
            "cost_ratio_vs_exact": ratios, "expansions": exp, "opts": opts,
            "note": "non-parity mode: valid paths (tests/test_gpu_relaxed.py), cost relative to the exact "
                    "(reference-identical) result of the same query"}



def run_cfg5(args, gpu, dist, torch, rank, world, device):
    """BASELINE.json configs[4] / SURVEY.md §8d cfg5: the local planner's replan loop for
    `pairs` start/goal pairs IN TOTAL, dealt round-robin over the ranks (strong scaling, no
    exchange; pair id q uses seed 1000 + q).  One step = one 20 Hz tick of every pair: a
    batched find_path WITHOUT reset (memo and stale node-map values carry over,
    local_planner.cpp:316), then free-space decay and the boxes moved by their velocity
    (local_planner.cpp:241,288).  value = pops / tick wall (max over ranks); the tick wall
    includes the map upkeep."""
    from tests.scenarios import drive_batch, replan_pairs, replan_tick_inputs
    ids = shard_global_ids(rank, world, args.pairs)
    pairs = []
    for q in ids:  # one generator draw per pair id
        pairs += replan_pairs(args.grid, args.bins, args.obstacles, 1, seed=1000 + q)
    t_setup = time.perf_counter()
    planners = []
    for cfg, proto, _ in pairs:
        cfg.values["max_pops"] = args.max_pops
        cfg.values["max_astar_nodes"] = args.max_astar_nodes
        planners.append(gpu.HybridAStar(cfg, device=device))
    drive_batch(gpu, planners, [proto for _, proto, _ in pairs])
    bufs = gpu.BatchBuffers(planners, cap=8192)
    gpu.reserve(planners, path_points=1024 * len(planners))  # the device pool, once at setup
    t_setup = time.perf_counter() - t_setup
    vels = [proto["vel"] for _, proto, _ in pairs]
    conf = [np.full(len(proto["boxes"]), proto["box_conf"], np.float32) for _, proto, _ in pairs]
    apf_r = pairs[0][1]["apf_r"] if pairs else 2.5
    tick = [0]

    # the replan loop never resets: the relaxed mode keeps each pair's heuristic field across
    # ticks, as the exact mode keeps its A* memo
    relaxed_opts = dict(delta=args.relaxed_delta, h_weight=args.relaxed_weight, reuse_heuristic=1)
    rx = {"kernel_ms": [], "wall_ms": [], "upkeep_ms": [], "ok": 0, "ratios": []}
    slowest = []
    # every (pair, tick) outcome of the exact loop, warm-up ticks included, for the parity
    # readout against the oracle's replay of the same loop (cpu_baseline_cfg5)
    gpu_ticks = [[] for _ in pairs]

    def step(timed):
        """One tick; returns (stats, kernel ms, successes, seconds of the exact tick).  When
        timed, the relaxed mode also plans the tick's queries on the same maps (between the
        exact find_path and the upkeep; its time is not part of the exact tick)."""
        t = tick[0]
        t0 = time.perf_counter()
        starts = [replan_tick_inputs(proto, v, t)[0] for _, proto, v in pairs]
        br = gpu.find_path_batch_arrays(planners, vels, starts, buffers=bufs)
        st = br.stats.copy()
        t_exact = time.perf_counter() - t0
        for i in range(len(planners)):
            gpu_ticks[i].append(tick_key(br.result(i)))
        if timed:  # the tick's slowest search (it bounds the tick): its pops and inner A* pops
            tm = np.array([p.timing() for p in planners], dtype=np.float64)
            j = int(np.argmax(tm[:, 1] - tm[:, 0]))
            slowest.append({"pair": int(ids[j]), "ms": float((tm[j, 1] - tm[j, 0]) * 1e-5), "pops": int(st["pops"][j]),
                            "astar_pops": int(st["astar_pops"][j])})
        if timed and not args.no_relaxed and planners:
            t1 = time.perf_counter()
            rel, rms = gpu.find_path_batch(planners, vels, starts, cap=8192, relaxed=relaxed_opts)
            rx["wall_ms"].append((time.perf_counter() - t1) * 1e3)
            rx["kernel_ms"].append(rms)
            rx["ok"] += sum(int(r["ok"]) for r in rel)
            rx["ratios"] += [float(r["cost"]) / float(br.cost[i]) for i, r in enumerate(rel) if r["ok"] and br.ok[i]]
        # the tick's map upkeep (local_planner.cpp:241,288), batched: decay + moved boxes
        t2 = time.perf_counter()
        gpu.decay_batch(bufs)
        gpu.update_boxes_batch(bufs, [replan_tick_inputs(proto, v, t + 1)[1] for _, proto, v in pairs], conf, apf_r)
        torch.cuda.synchronize(device)
        up = time.perf_counter() - t2
        if timed:
            rx["upkeep_ms"].append(up * 1e3)
        tick[0] += 1
        return st, br.kernel_ms, int(br.ok.sum()), t_exact + up

    for _ in range(args.warmup):
        step(False)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(device)
    pops, kms, oks, alg = 0, [], 0, []
    elapsed = 0.0
    for _ in range(args.steps):
        st, k, ok, secs = step(True)
        elapsed += secs
        pops += int(st["pops"].sum())
        kms.append(k)
        oks += ok
        alg.append(algorithmic_bytes(st, args.obstacles))
    torch.cuda.synchronize(device)
    elapsed, pops_all = reduce_over_ranks(dist, elapsed, pops, f"cuda:{device}")
    out = None
    if rank == 0:
        avg_k = float(np.mean(kms))
        achieved = float(np.mean(alg)) / (avg_k * 1e-3) / 1e9
        out = {
            "metric": METRIC,
            "value": pops_all / elapsed, "unit": "expansions/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (SURVEY.md §8d cfg5 generator; pair ids seed the boxes, goals and box velocities)",
            "config": {"workload": f"cfg5: {args.grid}x{args.grid}x{args.bins} grid, {args.obstacles} moving boxes, "
                                   f"{args.pairs} start/goal pairs in total replanned every 50 ms tick without reset",
                       "grid": args.grid, "angle_bins": args.bins, "obstacles": args.obstacles,
                       "pairs_total": args.pairs, "pairs_rank0": len(ids), "global_batch": args.pairs,
                       "parallelism": f"pair-sharded x{world}"},
            "replan_latency_ms": avg_k, "tick_ms": elapsed / args.steps * 1e3, "slowest_search_per_tick": slowest,
            "tick_budget_ms": 50.0, "tick_over_budget_x": elapsed / args.steps * 1e3 / 50.0,
            "success_rate": oks / max(len(ids) * args.steps, 1), "setup_s_per_gpu": t_setup,
            "roofline": {"bound": "latency", "roof": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS, "traffic": None,
                         "kernel": "hastar_search_wide_kernel (the latency kernel: one search per CU)",
                         "kernel_ms": avg_k, "alg_bytes_per_launch": float(np.mean(alg))},
        }
        if rx["kernel_ms"]:
            out["relaxed_mode"] = {
                "tick_search_ms": float(np.mean(rx["kernel_ms"])), "tick_find_wall_ms": float(np.mean(rx["wall_ms"])),
                "tick_ms": float(np.mean(rx["wall_ms"]) + np.mean(rx["upkeep_ms"])),
                "tick_over_budget_x": float(np.mean(rx["wall_ms"]) + np.mean(rx["upkeep_ms"])) / 50.0,
                "success_rate": rx["ok"] / max(len(ids) * args.steps, 1),
                "cost_ratio_vs_exact_mean": float(np.mean(rx["ratios"])) if rx["ratios"] else None,
                "cost_ratio_vs_exact_max": float(np.max(rx["ratios"])) if rx["ratios"] else None,
                "opts": relaxed_opts,
                "note": "non-parity mode (hastar_find_path_relaxed_batch) on the same ticks' maps and starts as the "
                        "exact loop (rank 0); tick_ms = its find_path wall + the same batched upkeep"}
        if not args.no_cpu_baseline:
            out["cpu_baseline"], replay = cpu_baseline_cfg5(pairs, args.cpu_seconds, args.warmup + args.steps, args.warmup)
            out["parity_sample"] = cfg5_parity(gpu_ticks, replay, ids)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    if out is not None:
        print(json.dumps(out))


def tick_key(r):
    """What parity compares for one (pair, tick) search: success, cost bits, pops, pop and closed
    digests, and a hash of the path and curvature bits."""
    h = hashlib.blake2b(np.ascontiguousarray(r["path"], np.float32).tobytes(), digest_size=8)
    h.update(np.ascontiguousarray(r["curvature"], np.float32).tobytes())
    st = r["stats"]
    return (bool(r["ok"]), np.float32(r["cost"]).tobytes().hex(), int(st["pops"]), int(st["pop_digest"]),
            int(st["closed_digest"]), h.hexdigest())


def cfg5_parity(gpu_ticks, replay, ids):
    """Every (pair, tick) of the GPU loop against the oracle's replay of the same loop (the
    pairs cpu_baseline_cfg5 replayed: all of them unless its budget ran out first)."""
    bad, checked, pops = [], 0, 0
    for i, ticks in replay.items():
        for t, (g, o) in enumerate(zip(gpu_ticks[i], ticks)):
            checked += 1
            pops += o[2]
            if g != o:
                bad.append([int(ids[i]), t])
    return {"pairs": len(replay), "ticks_per_pair": len(gpu_ticks[0]) if gpu_ticks else 0, "searches": checked,
            "bit_exact": not bad and checked == sum(len(t) for t in gpu_ticks), "mismatched_pair_ticks": bad[:16],
            "pops_checked": int(pops),
            "note": "every pair x every tick (warm-up included) of the exact replan loop, without reset, against the "
                    "oracle's replay of the same call sequence: success, cost bits, pops, pop/closed digests, "
                    "path+curvature bits (hash)"}


def cpu_baseline_cfg5(pairs, budget_s, ticks, warm=0):
    """The oracle replaying the same pairs' replan loops on `cpu_threads()` host threads, one
    private planner per thread (find_path timed only; ctypes calls release the GIL).  Pairs are
    taken in order, one thread per pair, in rounds of T pairs until every pair is replayed (the
    parity readout needs them all) or the rounds' parallel wall time reaches 4x the budget.
    value = pops / parallel find_path wall.  A tick's pairs are independent, so with a core per
    pair the CPU's tick takes as long as its slowest pair (tick_ms_one_core_per_pair: the mean
    over the timed ticks, the first `warm` ticks being the GPU run's warm-up; every tick's
    maximum in tick_max_ms).  Also returns {pair index: [tick_key per tick]} of the replayed pairs."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle.pyoracle import OraclePlanner
    from tests.scenarios import drive, replan_tick, replan_tick_inputs
    T = cpu_threads()

    def run_pair(pv, lean):
        cfg, proto, v = pv
        o = OraclePlanner(cfg, lean=lean)
        drive(o, proto)
        ms, pops, keys = [], 0, []
        for t in range(ticks):
            r = o.find_path(proto["vel"], replan_tick_inputs(proto, v, t)[0])
            pops += r["stats"]["pops"]
            ms.append(r["wall_ms"])
            keys.append(None if lean else tick_key(r))
            replan_tick(o, proto, v, t)
        o.close()
        return pops, ms, keys

    pops, wall, n = 0, 0.0, 0
    tick_max = np.zeros(ticks)
    per_tick = [[] for _ in range(ticks)]  # every replayed pair's find_path ms, per tick
    replay = {}
    with ThreadPoolExecutor(T) as ex:
        while n < len(pairs) and wall < 4 * budget_s:
            # timed: the lean build (the checker's digests compiled out); then the checker build
            # replays the same pairs untimed for the parity keys
            rnd = list(ex.map(lambda pv: run_pair(pv, True), pairs[n:n + T]))
            keys_rnd = list(ex.map(lambda pv: run_pair(pv, False)[2], pairs[n:n + T]))
            # the round's find_path time on T cores: its slowest pair's summed find_path time
            wall += max(sum(ms) for _, ms, _ in rnd) * 1e-3
            for j, (p, ms, _) in enumerate(rnd):
                pops += p
                tick_max = np.maximum(tick_max, ms)
                for t in range(ticks):
                    per_tick[t].append(ms[t])
                replay[n + j] = keys_rnd[j]
            n += len(rnd)

    def makespan(ms, cores):  # longest-processing-time-first list schedule of one tick's pairs
        load = [0.0] * cores
        for x in sorted(ms, reverse=True):
            load[load.index(min(load))] += x
        return max(load)
    return ({"value": pops / wall if wall > 0 else None, "unit": "expansions/s", "cores": T, "kind": "port",
             "build": "lean (oracle/build/libhastar_oracle_lean.so: -O3 -DORC_LEAN, digests and counters compiled out)",
             "sample": f"first {n} pairs of rank 0 x {ticks} ticks (same call sequence as the GPU run), find_path "
                       f"only, {T} threads with one private planner each (oracle/hastar_oracle.cpp -DORC_LEAN, -O3)",
             # the timed ticks (as the GPU's tick_ms; ticks before `warm` are its warm-up)
             "tick_ms_one_core_per_pair": float(tick_max[warm:].mean()) if n else None,
             "tick_max_ms": [float(x) for x in tick_max] if n else None,
             "tick_ms_one_core_per_pair_all_ticks": float(tick_max.mean()) if n else None,
             # the same ticks on this box's T host threads: each tick's replayed pairs list-scheduled
             # longest first over T cores (a tick of 64 pairs on 16 threads takes at least 4 pairs' time)
             f"tick_ms_{T}_threads": float(np.mean([makespan(m, T) for m in per_tick[warm:]])) if n else None}, replay)


def parity_sample(cfgs, gpu, qids, gpu_last=None, replans=1):
    """Bit-exact check at the bench's own size, outside the timed region: a stratified sample of
    the batch (`gpu`: planner index -> result of the first, cold step; every 64th query plus the 8
    longest) against the oracle on the same maps, on the host's threads.  The oracle replays the
    GPU planner's whole call sequence, `replans` x (reset + find_path); its first replan is compared
    with `gpu` and its last with `gpu_last` (the last timed step): success, cost bits, the search
    statistics and digests, path and curvature bits."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle.pyoracle import OraclePlanner
    from tests.scenarios import drive
    idx = sorted(gpu)
    replans = replans if gpu_last is not None else 1

    def run(i):
        o = OraclePlanner(cfgs[i][0])
        drive(o, cfgs[i][1])
        out = []
        for k in range(replans):
            o.reset()
            r = o.find_path(cfgs[i][1]["vel"], cfgs[i][1]["start"])
            if k == 0 or k == replans - 1:
                out.append(r)
        o.close()
        return out

    t0 = time.perf_counter()
    with ThreadPoolExecutor(cpu_threads()) as ex:
        res = list(ex.map(run, idx))
    keys = ("pops", "successors", "astar_pops", "astar_searches", "shots", "closed_size", "pop_digest",
            "closed_digest", "via_shot")

    def same(g, o):
        return (g["ok"] == o["ok"] and np.float32(g["cost"]).tobytes() == np.float32(o["cost"]).tobytes()
                and all(g["stats"][k] == o["stats"][k] for k in keys)
                and g["path"].tobytes() == o["path"].tobytes() and g["curvature"].tobytes() == o["curvature"].tobytes())

    bad, bad_last = [], []
    for i, q, o in zip(idx, qids, res):
        if not same(gpu[i], o[0]):
            bad.append(int(q))
        if gpu_last is not None and not same(gpu_last[i], o[-1]):
            bad_last.append(int(q))
    out = {"queries": len(idx), "bit_exact": not bad and not bad_last, "mismatched_queries": bad[:16],
           "pops_checked": int(sum(int(gpu[i]["stats"]["pops"]) for i in idx)),
           "path_poses_checked": int(sum(len(gpu[i]["path"]) for i in idx)), "oracle_s": time.perf_counter() - t0,
           "note": "first (cold) step of every 64th query and the 8 longest, against the oracle's reset + "
                   "find_path: success, cost, statistics, pop/closed digests, path and curvature bits"}
    if gpu_last is not None:
        out["last_timed_step"] = {
            "replans_replayed": replans, "bit_exact": not bad_last, "mismatched_queries": bad_last[:16],
            "pops_checked": int(sum(int(gpu_last[i]["stats"]["pops"]) for i in idx)),
            "path_poses_checked": int(sum(len(gpu_last[i]["path"]) for i in idx)),
            "note": "the same queries' last timed replan against the oracle's replay of every replan before it "
                    "(reset + find_path each; warm-up and timed steps): the same fields"}
    return out


def path_digest(r):
    """A digest of a result's path and curvature bits (parity_all compares these)."""
    import hashlib
    h = hashlib.blake2b(digest_size=16)
    h.update(np.ascontiguousarray(r["path"], np.float32).tobytes())
    h.update(np.ascontiguousarray(r["curvature"], np.float32).tobytes())
    return h.digest()


def parity_all(cfgs, stats, cost, ok, paths, qids):
    """Every query of the batch (`--parity-all`): the first (cold) step's outcome against the
    oracle's reset + find_path on the same maps, on the host's threads: success, cost bits,
    every statistic and digest, and the path and curvature bits (as 128-bit digests)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle.pyoracle import OraclePlanner
    from tests.scenarios import drive
    keys = ("pops", "successors", "astar_pops", "astar_searches", "shots", "closed_size", "pop_digest",
            "closed_digest", "via_shot")

    def run(i):
        o = OraclePlanner(cfgs[i][0])
        drive(o, cfgs[i][1])
        o.reset()
        r = o.find_path(cfgs[i][1]["vel"], cfgs[i][1]["start"])
        o.close()
        same = (bool(ok[i]) == bool(r["ok"]) and np.float32(cost[i]).tobytes() == np.float32(r["cost"]).tobytes()
                and all((int(stats[k][i]) - int(r["stats"][k])) % (1 << 64) == 0 for k in keys)
                and paths[i] == path_digest(r))
        return same, int(r["stats"]["pops"]), len(r["path"])

    t0 = time.perf_counter()
    with ThreadPoolExecutor(cpu_threads()) as ex:
        res = list(ex.map(run, range(len(cfgs))))
    bad = [int(qids[i]) for i, (same, _, _) in enumerate(res) if not same]
    return {"queries": len(cfgs), "bit_exact": not bad, "mismatched_queries": bad[:16], "n_mismatched": len(bad),
            "pops_checked": int(sum(p for _, p, _ in res)), "path_poses_checked": int(sum(k for _, _, k in res)),
            "oracle_s": time.perf_counter() - t0,
            "note": "every query's first (cold) step against the oracle's reset + find_path: success, cost bits, "
                    "statistics, pop/closed digests, path and curvature bits (digests)"}


def cpu_baseline(cfgs, gpu_results, budget_s, replans, lat_ids, sample=None):
    """The oracle (CPU restatement, 'port') on `cpu_threads()` host threads, one private
    planner per thread at a time (BASELINE.md "Plan for the CPU baseline"), find_path timed
    only, as the reference harness times it (test_hybrid_astar.cpp:123-126).  Each sampled
    query replays the GPU planner's exact call sequence — the map drive, then `replans` x
    (reset + find_path), warm-up and timed steps alike (the node map's f values persist across
    reset, HybridAStar.cpp:49-52, so later replans differ from the first).  Queries are taken
    in `sample` order (planner indices; default the batch's order), in chunks of 16 per thread,
    until the chunks' parallel wall time reaches the budget.  value = pops / parallel wall (chunk tails included).  Each query's
    last replan is compared with the GPU's last timed step (success, cost bits).  The timed build is
    the oracle's lean one (-DORC_LEAN: the checker's digests and counters compiled out, the same
    search); parity_sample checks digests and paths with the checker build."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle.pyoracle import OraclePlanner, run_batch_threads
    from tests.scenarios import drive
    T = cpu_threads()
    chunk = 16 * T
    pops, wall, plans, plan_s = 0, 0.0, 0, 0.0
    n, parity, lat = 0, True, []
    sample = list(range(len(cfgs))) if sample is None else list(sample)

    def make(c):
        o = OraclePlanner(c[0], lean=True)
        drive(o, c[1])
        return o

    with ThreadPoolExecutor(T) as ex:
        while n < len(sample) and wall < budget_s:
            idx = sample[n:n + chunk]
            sub = [cfgs[i] for i in idx]
            ors = list(ex.map(make, sub))
            r = run_batch_threads(ors, [c[1]["vel"] for c in sub], [c[1]["start"] for c in sub], replans, T)
            pops += r["pops"]
            wall += r["wall_s"]
            plans += r["plans"]
            plan_s += r["plan_s_sum"]
            for j in range(len(sub)):
                i = idx[j]
                parity &= (bool(r["ok"][j]) == bool(gpu_results.ok[i])
                           and np.float32(r["cost"][j]).tobytes() == np.float32(gpu_results.cost[i]).tobytes())
                if idx[j] in lat_ids:
                    lat.append(float(np.median(r["plan_ms"][j])))
            for o in ors:
                o.close()
            n += len(sub)
    return {"value": pops / wall if wall > 0 else None, "unit": "expansions/s", "cores": T, "kind": "port",
            "build": "lean (oracle/build/libhastar_oracle_lean.so: -O3 -DORC_LEAN, digests and counters compiled out)",
            "sample": f"first {n} queries of the GPU batch x {replans} replans each (same call sequence as the GPU "
                      f"run), find_path only, {T} threads with one private planner each (oracle/hastar_oracle.cpp "
                      f"-DORC_LEAN, -O3)",
            "per_core_value": pops / plan_s if plan_s > 0 else None,
            "mean_plan_ms": plan_s / plans * 1e3 if plans else None, "parity_with_gpu": bool(parity),
            "latency_same_queries_ms": float(np.median(lat)) if lat else None}


if __name__ == "__main__":
    main()
