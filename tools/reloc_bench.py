"""Batched map relocation throughput (hastar_update_goal_batch, Grid3D.cpp:169-203) on the GPU:
B planners of N^2 maps, R calls with fresh goals each; prints one JSON line with the wall time
per call and the rate on the algorithmic 8 N^2 bytes per map (read + write).  Run it under
`rocprofv3 --kernel-trace --stats` for the kernels' own durations.

  python tools/reloc_bench.py [--n 2048] [--grid 1024] [--reps 5]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from path_planning_pkg_amd import planner as gpu  # noqa: E402
from path_planning_pkg_amd.capi import PlannerConfig  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=2048)
ap.add_argument("--grid", type=int, default=1024)
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
import torch  # noqa: E402

cfg = PlannerConfig(grid_size=args.grid, num_angle_bins=72)
ps = gpu.HybridAStar.create_batch(cfg, args.n)
rng = np.random.default_rng(5)
walls = []
for r in range(args.reps + 1):
    goals = np.concatenate([rng.uniform(-20, 20, (args.n, 2)), rng.uniform(-3, 3, (args.n, 1))], 1).astype(np.float32)
    starts = np.concatenate([rng.uniform(-60, -30, (args.n, 2)), np.zeros((args.n, 1))], 1).astype(np.float32)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gpu.update_goal_batch(ps, goals, starts)
    torch.cuda.synchronize()
    if r:  # the first call loads the kernels
        walls.append(time.perf_counter() - t0)
bytes_alg = 8.0 * args.grid * args.grid * args.n
w = float(np.median(walls))
print(json.dumps({"maps": args.n, "grid": args.grid, "reps": args.reps, "wall_ms_median": w * 1e3,
                  "wall_ms_all": [x * 1e3 for x in walls], "alg_bytes_per_call": bytes_alg,
                  "alg_TBps_wall": bytes_alg / w / 1e12}))
