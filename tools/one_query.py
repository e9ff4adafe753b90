"""One cfg3 query (the survey generator, seed = query id + 1) planned R times on the GPU, for
profilers (rocprofv3 PC sampling / counters of a single search on the latency kernel).

  python tools/one_query.py [--seed 3] [--reps 3] [--batch-kernel]
"""
import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from path_planning_pkg_amd import planner as gpu  # noqa: E402
from tests.scenarios import drive, synthetic_ref  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seed", type=int, default=3)
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
cfg, proto = synthetic_ref(1024, 72, 200, args.seed)
p = gpu.HybridAStar(cfg)
drive(p, proto)
for r in range(args.reps):
    p.reset()
    t0 = time.perf_counter()
    res, ms = gpu.find_path_batch([p], [proto["vel"]], [proto["start"]])
    print(f"rep {r}: {res[0]['stats']['pops']} pops, {res[0]['stats']['astar_pops']} inner pops, kernel {ms:.1f} ms, "
          f"wall {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
