"""Time the backward grid-distance field (include/hastar.h: hastar_heuristic_field) on one GPU and
with G stand-in ranks (shard.py:heuristic_field_standins) on cfg3 / cfg4 maps; one JSON line per
case.  tools/field_bench.py [--grids 1024 2048] [--ranks 4]"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", type=int, nargs="+", default=[1024, 2048])
    ap.add_argument("--ranks", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    from path_planning_pkg_amd import planner, shard
    from tests.scenarios import drive, synthetic_ref
    planner.load_library()
    dev = torch.device("cuda:0")
    for N in a.grids:
        cfg, proto = synthetic_ref(N, 72, 200 if N <= 1024 else 800, 1)
        g = planner.HybridAStar(cfg)
        drive(g, proto)
        out = torch.empty(N * N, dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        g.heuristic_field(out.data_ptr())  # warm-up
        ts, passes = [], 0
        for _ in range(a.reps):
            t0 = time.perf_counter()
            passes = g.heuristic_field(out.data_ptr())
            ts.append((time.perf_counter() - t0) * 1e3)
        one = out.cpu().numpy()
        ts2, rounds = [], 0
        for _ in range(a.reps):
            t0 = time.perf_counter()
            full, rounds, p2 = shard.heuristic_field_standins(g, a.ranks, dev)
            ts2.append((time.perf_counter() - t0) * 1e3)
        same = bool(np.array_equal(full.cpu().numpy().view(np.uint32), one.view(np.uint32)))
        print(json.dumps({"grid": N, "one_gpu_ms": min(ts), "passes": passes, "finite_cells": int(np.isfinite(one).sum()),
                          "standin_ranks": a.ranks, "standin_ms": min(ts2), "rounds": rounds, "standin_passes": p2,
                          "standin_equals_one_gpu": same}), flush=True)
        g.close()


if __name__ == "__main__":
    main()
