"""Slot utilisation of one batched find_path (the bench's cfg3 batch): how much of the kernel's
time the resident slots are busy, from each search's s_memrealtime start/end (10 ns ticks).

    python tools/tail_analysis.py [--batch 23552] [--steps 2]
Prints the kernel time, sum of search durations / slots (the ideal time with no tail), the
busy fraction, and the number of busy slots over time (deciles of the kernel)."""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from path_planning_pkg_amd import planner as gpu  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=23552)
ap.add_argument("--steps", type=int, default=2)
ap.add_argument("--clock", action="store_true", help="stamps build: shader clock of the searches under load")
ap.add_argument("--dump", default=None, help="save every step's per-query {duration ms, slot} to this .npz")
a = ap.parse_args()
args = bench.parse_args(["--batch", str(a.batch)])
if args.grid is None:
    args.grid = 1024
cfgs = [bench.query_case(args, q) for q in range(a.batch)]
planners, _ = bench.build_planners(gpu, cfgs, 0)
vels = [c[1]["vel"] for c in cfgs]
starts = [c[1]["start"] for c in cfgs]
bufs = gpu.BatchBuffers(planners, cap=8192)
dumps = {}
for step in range(a.steps):
    gpu.reset_batch(bufs)
    r = gpu.find_path_batch_arrays(planners, vels, starts, buffers=bufs)
    t = np.array([p.timing() for p in planners], dtype=np.float64)
    t0, t1 = t[:, 0].min(), t[:, 1].max()
    dur = (t[:, 1] - t[:, 0]) * 1e-5  # ms
    dumps[f"dur{step}"] = dur
    dumps[f"slot{step}"] = t[:, 2]
    dumps[f"start{step}"] = (t[:, 0] - t[:, 0].min()) * 1e-5
    slots = len(set(int(s) for s in t[:, 2]))
    span = (t1 - t0) * 1e-5
    grid = np.linspace(t0, t1, 11)
    busy = [int(((t[:, 0] <= g) & (t[:, 1] > g)).sum()) for g in grid[:-1]]
    clock = None
    if a.clock:  # stamps build: s_memtime (shader clock) cycles of the search loop / its realtime span
        li = int(np.argmax(dur))
        cyc = np.array([planners[i].cycles()[6] for i in range(len(planners))], dtype=np.float64)
        mhz = cyc / np.maximum(dur * 1e3, 1e-9)  # cycles per us
        long_ix = np.argsort(-dur)[:16]
        cl = planners[li].cycles()
        pops = float(r.stats["pops"][li])
        names = {0: "pop", 1: "expand", 2: "bookkeeping(incl A*)", 3: "astar", 4: "shot", 7: "astar_hbm",
                 13: "find3", 14: "insert3", 16: "succ_gen", 17: "apf", 18: "dubins", 19: "insert_walk",
                 20: "insert_link", 21: "probe_wait"}
        longest_phases = {n: round(cl[i] / max(pops, 1)) for i, n in names.items()}
        longest_phases.update(loop_per_pop=round(cl[6] / max(pops, 1)), fills_per_pop=cl[22] / max(pops, 1),
                              cycles_per_fill=cl[26] / max(cl[22], 1))
        clock = {"longest_phases_per_pop": longest_phases,
                 "longest_mhz": float(mhz[li]), "top16_mhz_mean": float(mhz[long_ix].mean()),
                 "median_mhz_over_searches_gt_1ms": float(np.median(mhz[dur > 1.0]))}
    print(json.dumps({"clock": clock, "step": step, "kernel_ms": r.kernel_ms, "span_ms": span, "slots_used": slots,
                      "sum_dur_ms": float(dur.sum()), "ideal_ms": float(dur.sum() / slots),
                      "busy_frac": float(dur.sum() / (slots * span)), "longest_ms": float(dur.max()),
                      "busy_slots_by_decile": busy}), flush=True)
if a.dump:
    np.savez(a.dump, **dumps)
