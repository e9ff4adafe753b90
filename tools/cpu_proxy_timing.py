"""The cpu_baseline proxy, stated: the oracle restatement's find_path wall time on
the survey's cfg1/cfg3 seeds, best of R fresh instances, single thread, in this container — the
checker build and the lean timing build (-DORC_LEAN, bench.py's cpu_baseline) interleaved rep by
rep, so both see the same host load — beside the compiled reference's timings that BASELINE.md
records for the same inputs (taken in the survey's session; the reference itself is unbuildable
under this build's rules: it needs a Boost stand-in header).

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
    walls = {False: [], True: []}
    res = {}
    for _ in range(args.reps):
        for lean in (False, True):
            o = OraclePlanner(cfg, lean=lean)
            drive(o, proto)
            r = o.find_path(proto["vel"], proto["start"])
            walls[lean].append(r["wall_ms"])
            res[lean] = (r["stats"]["pops"], float(r["cost"]), bool(r["ok"]))
            o.close()
    assert res[False] == res[True], res  # the lean build plans the same search
    best = {k: min(v) for k, v in walls.items()}
    ref = REF.get((N, seed))
    print(json.dumps(dict(grid=N, bins=bins, K=K, seed=seed, pops=res[False][0], oracle_best_ms=round(best[False], 3),
                          oracle_median_ms=round(sorted(walls[False])[len(walls[False]) // 2], 3),
                          lean_best_ms=round(best[True], 3),
                          lean_median_ms=round(sorted(walls[True])[len(walls[True]) // 2], 3),
                          lean_vs_full=round(best[True] / best[False], 3), reps=args.reps, reference_ms=ref,
                          lean_vs_reference=round(best[True] / ref, 3) if ref else None, host_cpus=os.cpu_count())),
          flush=True)
