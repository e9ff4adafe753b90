"""Two search dispatches for SQ counter passes: one planner alone (seed 1), then a batch.

  rocprofv3 --pmc <SQ counters> --output-format csv -d DIR -o sq -- python3 tools/sq_probe.py --batch 2048
"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from path_planning_pkg_amd import planner as gpu  # noqa: E402
from tests.scenarios import drive, synthetic  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=2048)
ap.add_argument("--grid", type=int, default=1024)
ap.add_argument("--max-pops", type=int, default=131072)
a = ap.parse_args()
ps, cf = [], []
for q in range(a.batch):
    cfg, proto = synthetic(a.grid, 72, 200, q + 1)
    cfg.values["max_pops"] = a.max_pops
    p = gpu.HybridAStar(cfg)
    drive(p, proto)
    ps.append(p)
    cf.append(proto)
r1, k1 = gpu.find_path_batch(ps[:1], [cf[0]["vel"]], [cf[0]["start"]])
for p in ps:
    p.reset()
rb, kb = gpu.find_path_batch(ps, [c["vel"] for c in cf], [c["start"] for c in cf])
print({"single_ms": k1, "single_pops": r1[0]["stats"]["pops"], "single_apops": r1[0]["stats"]["astar_pops"],
       "batch_ms": kb, "batch_pops": sum(r["stats"]["pops"] for r in rb),
       "batch_apops": sum(r["stats"]["astar_pops"] for r in rb)})
