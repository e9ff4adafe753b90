"""Throughput vs batch size of the search kernel (cfg3 planners, one wavefront each).

  python tools/batch_scaling.py --batches 64 256 1024 2048
Builds max(batches) planners once (seeds 1..B), then for each B runs one batched search
(after reset) and prints kernel ms, pops, A* pops, overflow count and pops/s.
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from path_planning_pkg_amd import planner as gpu  # noqa: E402
from tests.scenarios import drive, synthetic  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batches", type=int, nargs="+", default=[64, 256, 1024])
ap.add_argument("--grid", type=int, default=1024)
ap.add_argument("--obstacles", type=int, default=200)
ap.add_argument("--max-pops", type=int, default=0)
ap.add_argument("--max-astar-nodes", type=int, default=0)
ap.add_argument("--repeat", type=int, default=1, help="runs per batch (later runs use the longest-first order)")
ap.add_argument("--prio", type=int, nargs="*", default=None, help="HASTAR_PRIO_N values to sweep")
ap.add_argument("--slots", type=int, nargs="*", default=None, help="HASTAR_SLOTS values to sweep")
ap.add_argument("--iso", type=int, nargs="*", default=None, help="HASTAR_ISO values to sweep (head isolation)")
args = ap.parse_args()
import os


def timing_summary(planners, res):
    """Per-planner start/end times (s_memrealtime, 10 ns) -> span, straggler and balance."""
    import numpy as np
    t = np.array([p.timing() for p in planners], dtype=np.float64)
    t0 = t[:, 0].min()
    dur = (t[:, 1] - t[:, 0]) * 1e-5          # ms
    end = (t[:, 1] - t0) * 1e-5
    i = int(np.argmax(dur))
    work = np.array([r["stats"]["pops"] + r["stats"]["astar_pops"] for r in res], np.float64)
    slots = t[:, 2].astype(int)
    busy = np.bincount(slots, weights=dur)
    return {"span_ms": float(end.max()), "max_dur_ms": float(dur.max()), "max_dur_seed": i + 1,
            "max_dur_start_ms": float((t[i, 0] - t0) * 1e-5), "max_dur_work": float(work[i]),
            "mean_slot_busy_ms": float(busy[busy > 0].mean()), "n_slots": int((busy > 0).sum()),
            "ns_per_work": float(dur.sum() * 1e6 / work.sum())}
Bmax = max(args.batches)
t = time.time()
ps, cf = [], []
for q in range(Bmax):
    cfg, proto = synthetic(args.grid, 72, args.obstacles, q + 1)
    cfg.values["max_pops"] = args.max_pops
    cfg.values["max_astar_nodes"] = args.max_astar_nodes
    p = gpu.HybridAStar(cfg)
    drive(p, proto)
    ps.append(p)
    cf.append(proto)
print(json.dumps({"setup_s": time.time() - t, "planners": Bmax}), flush=True)
for B in args.batches:
  for prio, slots, iso in [(p_, s_, i_) for p_ in (args.prio or [None]) for s_ in (args.slots or [None])
                           for i_ in (args.iso or [None])]:
   if iso is not None:
       os.environ["HASTAR_ISO"] = str(iso)
   if prio is not None:
       os.environ["HASTAR_PRIO_N"] = str(prio)
   if slots is not None:
       os.environ["HASTAR_SLOTS"] = str(slots)
   for rep in range(args.repeat):
        for p in ps[:B]:
            p.reset()
        t0 = time.time()
        res, kms = gpu.find_path_batch(ps[:B], [c["vel"] for c in cf[:B]], [c["start"] for c in cf[:B]], cap=8192)
        wall = time.time() - t0
        pops = sum(r["stats"]["pops"] for r in res)
        apops = sum(r["stats"]["astar_pops"] for r in res)
        bad = [i + 1 for i, r in enumerate(res) if r["stats"]["status"] != 0]
        modes = [p.astar_modes() for p in ps[:B]]
        hbm = sum(m["astar_pops_hbm"] for m in modes)
        migr = sum(m["migrations"] for m in modes)
        print(json.dumps({"batch": B, "prio": prio, "slots": slots, "iso": iso, "rep": rep, "kernel_ms": kms, "wall_ms": wall * 1e3, "pops": pops, "astar_pops": apops,
                          "pops_per_s": pops / (kms * 1e-3), "astar_pops_hbm": hbm, "astar_migrations": migr,
                          "astar_searches": sum(r["stats"]["astar_searches"] for r in res), "overflow_seeds": bad[:20], "n_overflow": len(bad),
                          "max_work": max(r["stats"]["pops"] + r["stats"]["astar_pops"] for r in res),
                          **timing_summary(ps[:B], res),
                          "pool": ps[0].slots(),
                          "mean_work": (pops + apops) / B}),
              flush=True)
