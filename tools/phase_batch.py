"""Phase breakdown of the search kernel under load (diagnostic build with -DHASTAR_STAMPS).

  make -C path_planning_pkg_amd/csrc EXTRA=-DHASTAR_STAMPS OUTDIR=$PWD/path_planning_pkg_amd/lib_stamps
  HASTAR_LIB=path_planning_pkg_amd/lib_stamps/libhastar_amd.so python tools/phase_batch.py --batch 1 4096

For each batch size: one batched find_path over planners seeded 1..B (bench workload), then
s_memtime cycles summed over planners per phase, normalised per outer pop / inner A* pop.
Comparing B = 1 with a chip-filling B shows which phases slow down under contention.
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from path_planning_pkg_amd import planner as gpu  # noqa: E402
from tests.scenarios import drive, synthetic  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=1024)
ap.add_argument("--bins", type=int, default=72)
ap.add_argument("--obstacles", type=int, default=200)
ap.add_argument("--batch", type=int, nargs="+", default=[1, 2048])
args = ap.parse_args()

names = {0: "pop", 1: "expand", 2: "bookkeeping(incl A*)", 3: "astar", 4: "shot", 5: "reconstruct", 6: "loop",
         7: "astar_hbm", 8: "a_pop_probe", 9: "a_find", 10: "a_insert", 11: "a_unlink_hit", 12: "a_memoise",
         13: "find3", 14: "insert3", 15: "unlink3"}
Bmax = max(args.batch)
planners, protos = [], []
for q in range(Bmax):
    cfg, proto = synthetic(args.grid, args.bins, args.obstacles, seed=q + 1)
    p = gpu.HybridAStar(cfg)
    drive(p, proto)
    planners.append(p)
    protos.append(proto)
for B in args.batch:
    ps = planners[:B]
    for p in ps:
        p.reset()
    res = gpu.find_path_batch_arrays(ps, [pr["vel"] for pr in protos[:B]], [pr["start"] for pr in protos[:B]],
                                     cap=8192)
    st = res.stats
    cyc = np.array([p.cycles() for p in ps], dtype=np.float64).sum(axis=0)
    pops = float(st["pops"].sum())
    apops = float(st["astar_pops"].sum())
    out = dict(batch=B, kernel_ms=res.kernel_ms, pops=pops, astar_pops=apops, succ=float(st["successors"].sum()),
               astar_searches=float(st["astar_searches"].sum()), loop_cycles_per_pop=cyc[6] / pops,
               per_pop={names[i]: round(cyc[i] / pops) for i in (0, 1, 2, 3, 4, 5, 13, 14, 15)},
               per_apop={names[i]: round(cyc[i] / apops) for i in (3, 7, 8, 9, 10, 11, 12)},
               share={names[i]: round(cyc[i] / cyc[6], 4) for i in (0, 1, 2, 3, 4, 13, 14, 15)})
    print(json.dumps(out), flush=True)
