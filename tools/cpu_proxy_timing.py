"""The cpu_baseline proxy, stated: the oracle restatement's find_path wall time on
the survey's cfg1/cfg3 seeds, best of R fresh instances, single thread, in this container, beside
the compiled reference's timings that BASELINE.md records for the same inputs (61 / 115 ms at
1024^2 seeds 1 / 3; 0.95 ms at 256^2 seed 1).

  python tools/cpu_proxy_timing.py [--reps 7]     -> one JSON line per case
"""
import argparse
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from oracle.pyoracle import OraclePlanner  # noqa: E402  (test infrastructure: the checker / CPU baseline)
from tests.scenarios import drive, synthetic_ref  # noqa: E402

REF = {(1024, 1): 61.0, (1024, 3): 115.0, (256, 1): 0.95, (512, 1): 9.2, (512, 2): 20.4}
ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=7)
args = ap.parse_args()
for (N, bins, K, seed) in [(256, 36, 10, 1), (512, 72, 50, 1), (512, 72, 50, 2), (1024, 72, 200, 1), (1024, 72, 200, 3)]:
    cfg, proto = synthetic_ref(N, bins, K, seed)
    walls, pops = [], None
    for _ in range(args.reps):
        o = OraclePlanner(cfg)
        drive(o, proto)
        r = o.find_path(proto["vel"], proto["start"])
        walls.append(r["wall_ms"])
        pops = r["stats"]["pops"]
        del o
    print(json.dumps(dict(grid=N, bins=bins, K=K, seed=seed, pops=pops, oracle_best_ms=round(min(walls), 3),
                          oracle_median_ms=round(sorted(walls)[len(walls) // 2], 3), reps=args.reps,
                          reference_ms=REF.get((N, seed)), host_cpus=os.cpu_count())), flush=True)
