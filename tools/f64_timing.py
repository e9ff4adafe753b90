"""Wall time of single find_path calls, HybridAStar<float> against HybridAStar<double> on the GPU
and the oracle's float/double instantiations on one host core, for a few cfg3-size queries
(tests/scenarios.py:synthetic_ref, the bench's generator; seed = query id + 1).

    python tools/f64_timing.py [--seeds 1 2 3] [--grid 1024]
One JSON line per query: pops, GPU ms (float, double; the second of two reset + find_path calls),
CPU ms (float, double), whether the double result equals the oracle's (pops, closed set, cost
within 1e-4)."""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tests.scenarios import drive, synthetic_ref  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seeds", type=int, nargs="+", default=[1, 2, 3])
ap.add_argument("--grid", type=int, default=1024)
a = ap.parse_args()

from oracle.pyoracle import OraclePlanner, OraclePlanner64  # noqa: E402
from path_planning_pkg_amd.planner import HybridAStar  # noqa: E402
from path_planning_pkg_amd.planner64 import HybridAStar64  # noqa: E402


def timed(p, proto):
    p.reset()
    p.find_path(proto["vel"], proto["start"])  # first call: allocation, code objects
    p.reset()
    t0 = time.perf_counter()
    r = p.find_path(proto["vel"], proto["start"])
    return r, (time.perf_counter() - t0) * 1e3


for s in a.seeds:
    cfg, proto = synthetic_ref(a.grid, 72, 200, s)
    p64 = dict(proto)
    for k in ("boxes", "lines"):
        p64[k] = np.asarray(proto[k], np.float64)
    out = {"query": s - 1}
    for name, cls, pr in (("gpu_f32", HybridAStar, proto), ("gpu_f64", HybridAStar64, p64),
                          ("cpu_f32", OraclePlanner, proto), ("cpu_f64", OraclePlanner64, p64)):
        p = cls(cfg)
        drive(p, pr)
        r, ms = timed(p, pr)
        out[name + "_ms"] = round(ms, 2)
        out[name + "_pops"] = int(r["stats"]["pops"])
        out[name + "_cost"] = float(r["cost"])
        if name == "gpu_f64":
            g64 = p
        if name == "cpu_f64":
            out["f64_same_closed_set"] = bool(np.array_equal(g64.closed_keys(), p.closed_keys()))
            p.close()
        elif name == "cpu_f32":
            p.close()
    out["f64_cost_rel_diff"] = abs(out["gpu_f64_cost"] - out["cpu_f64_cost"]) / max(abs(out["cpu_f64_cost"]), 1e-30)
    print(json.dumps(out), flush=True)
